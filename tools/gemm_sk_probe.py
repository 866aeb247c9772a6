"""Stream-K A/B on the production fwd / input-gradient GEMM shapes (with their
epilogues), micro-batch (B = 128) and whole-batch (B = 256) row counts:
MAECLIP_GEMM_SK=0 (data-parallel) vs 1 (auto plan), interleaved rounds in one
process; median per-launch time. One JSON line per shape. The stream-K path
it measured (commit a8fe7cd) was reverted after this A/B
(profiles/r04/gemm_stream_k_ab_r4h.jsonl); on later builds both legs run the
data-parallel kernel."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def shapes(B):
    E, D = B * 50, B * 197
    return [  # name, M, N, K, b_layout, epi
        ("enc qkv fwd", E, 2304, 768, 0, K.EPI_NONE), ("enc proj fwd+res", E, 768, 768, 0, K.EPI_RESID),
        ("enc fc1 fwd gelu'", E, 3072, 768, 0, K.EPI_GELU_D), ("enc fc2 fwd+res", E, 768, 3072, 0, K.EPI_RESID),
        ("enc fc2 dgrad*gelu'", E, 3072, 768, 1, K.EPI_MUL_AUX), ("enc fc1 dgrad", E, 768, 3072, 1, K.EPI_NONE),
        ("enc qkv dgrad", E, 768, 2304, 1, K.EPI_NONE), ("enc proj dgrad", E, 768, 768, 1, K.EPI_NONE),
        ("dec qkv fwd", D, 1536, 512, 0, K.EPI_NONE), ("dec fc1 fwd gelu'", D, 2048, 512, 0, K.EPI_GELU_D),
        ("dec fc2 fwd+res", D, 512, 2048, 0, K.EPI_RESID), ("dec fc2 dgrad*gelu'", D, 2048, 512, 1, K.EPI_MUL_AUX),
        ("dec fc1 dgrad", D, 512, 2048, 1, K.EPI_NONE), ("dec qkv dgrad", D, 512, 1536, 1, K.EPI_NONE),
    ]


def make(M, N, Kd, lb, epi):
    A = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
    Bm = (torch.randn(N, Kd, device=dev) * 0.5).to(torch.bfloat16) if lb == 0 else \
        (torch.randn(Kd, N, device=dev) * 0.5).to(torch.bfloat16)
    kw = {}
    out = torch.bfloat16
    if epi == K.EPI_RESID:
        kw = dict(resid=torch.randn(M, N, device=dev), ldr=N)
        out = torch.float32
    elif epi == K.EPI_GELU_D:
        kw = dict(aux_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16), ldaux=N, bias=torch.randn(N, device=dev))
    elif epi == K.EPI_MUL_AUX:
        kw = dict(aux=torch.rand(M, N, device=dev).to(torch.bfloat16), ldaux=N)
    C = torch.empty(M, N, device=dev, dtype=out)
    return lambda: K.gemm(A, Bm, C, M, N, Kd, A.stride(0), Bm.stride(0), N, 0, lb, epilogue=epi, **kw)


def time_one(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for B in (128, 256):
    for name, M, N, Kd, lb, epi in shapes(B):
        fn = make(M, N, Kd, lb, epi)
        t = {"0": [], "1": []}
        for mode in ("0", "1"):
            os.environ["MAECLIP_GEMM_SK"] = mode
            fn(); fn()
        torch.cuda.synchronize()
        for r in range(5):
            for mode in ("0", "1"):
                os.environ["MAECLIP_GEMM_SK"] = mode
                t[mode].append(time_one(fn))
        d0, d1 = statistics.median(t["0"]), statistics.median(t["1"])
        fl = 2.0 * M * N * Kd
        print(json.dumps(dict(B=B, name=name, M=M, N=N, K=Kd, dp_us=round(d0, 1), sk_us=round(d1, 1),
                              speedup=round(d0 / d1, 3), sk_tflops=round(fl / d1 / 1e6, 1))), flush=True)
