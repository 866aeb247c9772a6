"""Per-shape timing of the plain / residual-form GEMM launches the round-4
vendor path used to take (round 4's plain_gemm_vendor_probe rows + the fp32
residual forms), micro-batch (B=128) and whole-batch (B=256) row counts of the
C2 step: this library's kernel with its default tile / split choice ("own"),
the same with the split off ("own_dp"), and torch's bf16 matmul ("vendor":
hipBLASLt through torch, calibration only -- the product never calls it; for
the residual forms it is the plain bf16 product, without the fp32 residual
read / fp32 store of the own launch). One process, interleaved rounds, median
per-launch time (us). One JSON line per shape."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
MODES = {"own": {"MAECLIP_GEMM_SK": ""}, "own_dp": {"MAECLIP_GEMM_SK": "0"}, "vendor": None}


def shapes(B):
    E, D = B * 50, B * 197
    # name, M, N, K, b_layout, residual form
    return [("enc qkv fwd", E, 2304, 768, 0, False), ("enc fc1 dgrad", E, 768, 3072, 1, False),
            ("enc qkv dgrad", E, 768, 2304, 1, False), ("enc proj dgrad", E, 768, 768, 1, False),
            ("dec qkv fwd", D, 1536, 512, 0, False), ("dec fc1 dgrad", D, 512, 2048, 1, False),
            ("dec qkv dgrad", D, 512, 1536, 1, False), ("dec proj dgrad", D, 512, 512, 1, False),
            ("dec pred dgrad", D, 512, 768, 1, False),
            ("enc proj fwd+res", E, 768, 768, 0, True), ("enc fc2 fwd+res", E, 768, 3072, 0, True),
            ("text out fwd+res", B * 25, 768, 768, 0, True), ("text lin2 fwd+res", B * 25, 768, 3072, 0, True),
            ("text qkv fwd", B * 25, 2304, 768, 0, False)]


def time_one(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def setenv(mode):
    for k, v in (MODES[mode] or {}).items():
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)


only = set(sys.argv[1:])
for B in (128, 256):
    for name, M, N, Kd, lb, res in shapes(B):
        if only and name not in only:
            continue
        g = torch.Generator().manual_seed(M + N + Kd)
        A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        Bm = ((torch.randn(N, Kd, generator=g) if lb == 0 else torch.randn(Kd, N, generator=g)) * 0.5
              ).to(torch.bfloat16).to(dev)
        bias = torch.randn(N, generator=g).to(dev) if (res or lb == 0) else None
        R = torch.randn(M, N, generator=g).to(dev) if res else None
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if res else torch.bfloat16)
        Cv = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Bt = Bm.t() if lb == 0 else Bm
        epi = K.EPI_RESID if res else K.EPI_NONE
        own = lambda: K.gemm(A, Bm, C, M, N, Kd, A.stride(0), Bm.stride(0), N, 0, lb, epilogue=epi, bias=bias,
                             resid=R, ldr=N if res else 0)
        vendor = lambda: torch.matmul(A, Bt, out=Cv)
        t = {m: [] for m in MODES}
        outs = {}
        for m in MODES:
            setenv(m)
            fn = vendor if MODES[m] is None else own
            fn()
            fn()
            torch.cuda.synchronize()
            outs[m] = (Cv if MODES[m] is None else C).float().clone()
        for r in range(5):
            for m in MODES:
                setenv(m)
                t[m].append(time_one(vendor if MODES[m] is None else own))
        med = {m: statistics.median(v) for m, v in t.items()}
        ref = outs["vendor"] + (R if res else 0) + (bias if bias is not None else 0)
        dev_own = ((outs["own"] - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps(dict(B=B, name=name, M=M, N=N, K=Kd, own_us=round(med["own"], 1),
                              own_dp_us=round(med["own_dp"], 1), vendor_us=round(med["vendor"], 1),
                              own_vs_vendor=round(med["vendor"] / med["own"], 3), max_rel_diff=dev_own)), flush=True)
