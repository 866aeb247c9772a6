"""Stream-K diagnosis on the micro-batch shapes that leave the 256 CUs idle
(75-tile encoder launches, the decoder's N = 512 dgrads): per-launch time with
MAECLIP_GEMM_SK = 0 (data-parallel) / 1 (forced) / auto, for the library
MAECLIP_LIB points at (diagnostic builds: -DSKX_NO_REDUCE, -DSKX_NO_PUBLISH,
-DGEMM4_STAMPS). With a GEMM4_STAMPS build and STAMPS=1 it also prints, per
job slot, the median cycles of: DMA wait, K loop, fix-up + epilogue.
python tools/sk_diag.py [label]"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mae_clip_amd import kernels as K, _lib

dev = torch.device("cuda")
label = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(_lib.LIB_PATH)
lib = _lib.load()
SHAPES = [  # name, M, N, K, b_layout, epilogue
    ("enc fc2 fwd+res", 6400, 768, 3072, 0, K.EPI_RESID),
    ("enc fc1 dgrad", 6400, 768, 3072, 1, K.EPI_NONE),
    ("enc qkv dgrad", 6400, 768, 2304, 1, K.EPI_NONE),
    ("enc proj fwd+res", 6400, 768, 768, 0, K.EPI_RESID),
    ("dec fc1 dgrad", 25216, 512, 2048, 1, K.EPI_NONE),
    ("dec qkv dgrad", 25216, 512, 1536, 1, K.EPI_NONE),
    ("text lin2 fwd+res", 3200, 768, 3072, 0, K.EPI_RESID),
    ("enc qkv fwd", 6400, 2304, 768, 0, K.EPI_NONE),
    ("enc fc1 dgrad B256", 12800, 768, 3072, 1, K.EPI_NONE),
    ("enc fc2 fwd+res B256", 12800, 768, 3072, 0, K.EPI_RESID),
]
only = os.environ.get("ONLY")


def make(M, N, Kd, lb, epi):
    g = torch.Generator().manual_seed(M + N + Kd)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    Bm = ((torch.randn(N, Kd, generator=g) if lb == 0 else torch.randn(Kd, N, generator=g)) * 0.5
          ).to(torch.bfloat16).to(dev)
    res = epi == K.EPI_RESID
    R = torch.randn(M, N, generator=g).to(dev) if res else None
    bias = torch.randn(N, generator=g).to(dev) if lb == 0 else None
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if res else torch.bfloat16)
    return C, lambda: K.gemm(A, Bm, C, M, N, Kd, A.stride(0), Bm.stride(0), N, 0, lb, epilogue=epi, bias=bias,
                             resid=R, ldr=N if res else 0)


def time_one(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


MODES = {"dp": {"MAECLIP_GEMM_SK": "0"}, "auto": {}, "dp256": {"MAECLIP_GEMM_SK": "0", "MAECLIP_GEMM_BM": "256"},
         "dp192": {"MAECLIP_GEMM_SK": "0", "MAECLIP_GEMM_BM": "192"},
         "dp128": {"MAECLIP_GEMM_SK": "0", "MAECLIP_GEMM_BM": "128"}}
for d in (0, 2, 4, 6, 8):
    MODES[f"split2_192_d{d}"] = {"MAECLIP_GEMM_SPLIT": "2", "MAECLIP_GEMM_BM": "192", "MAECLIP_GEMM_SPLIT_D": str(d)}
if os.environ.get("SKMODES"):
    MODES = {k: v for k, v in MODES.items() if k in os.environ["SKMODES"].split(",")}


def setmode(v):
    for k in ("MAECLIP_GEMM_SK", "MAECLIP_GEMM_BM", "MAECLIP_GEMM_SPLIT", "MAECLIP_GEMM_SPLIT_D", "MAECLIP_GEMM_BM128"):
        os.environ.pop(k, None)
    if isinstance(v, str):
        v = {"MAECLIP_GEMM_SK": v}
    os.environ.update(v)


for name, M, N, Kd, lb, epi in SHAPES:
    if only and name not in only.split(","):
        continue
    C, fn = make(M, N, Kd, lb, epi)
    outs, t = {}, {m: [] for m in MODES}
    for m, v in MODES.items():
        setmode(v)
        fn()
        fn()
        torch.cuda.synchronize()
        outs[m] = C.float().clone()
    for _ in range(5):
        for m, v in MODES.items():
            setmode(v)
            t[m].append(time_one(fn))
    med = {m: round(statistics.median(x), 1) for m, x in t.items()}
    ref = outs[next(iter(MODES))]
    diff = max(((outs[m] - ref).abs().max() / ref.abs().max()).item() for m in MODES)
    rec = dict(lib=label, name=name, M=M, N=N, K=Kd, us=med, max_rel_diff_vs_dp=diff)
    if os.environ.get("STAMPS") and hasattr(lib, "maeclip_debug_gemm4_stamps"):
        f = lib.maeclip_debug_gemm4_stamps
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        NS = 256 * 8 * 2 * 4
        setmode("1")
        torch.cuda.synchronize()
        assert f(None, -1) == 0       # zero the stamp buffer
        fn()
        torch.cuda.synchronize()
        buf = np.zeros(NS, dtype=np.uint64)
        assert f(buf.ctypes.data, NS) == 0
        s = buf.reshape(256, 8, 2, 4).astype(np.int64)
        t0 = s[:, :, :, 0][s[:, :, :, 0] > 0].min()
        ph = []
        for j in range(8):
            v = s[:, j, 0, :]
            v = v[v[:, 0] > 0]
            if len(v) == 0:
                continue
            ph.append(dict(job=j, blocks=int(len(v)), start=int(np.median(v[:, 0] - t0)),
                           wait=int(np.median(v[:, 1] - v[:, 0])), kloop=int(np.median(v[:, 2] - v[:, 1])),
                           fix_epi=int(np.median(v[:, 3] - v[:, 2])), fix_epi_p90=int(np.percentile(v[:, 3] - v[:, 2], 90)),
                           end_max=int((v[:, 3] - t0).max())))
        rec["stamps_sk"] = ph
    print(json.dumps(rec), flush=True)
