"""Plain bf16 GEMM shapes of the C2 step (micro-batch and whole-batch row counts):
this library's v4 kernel (MAECLIP_GEMM_LIB=0) vs the vendor library (=2), one
process, interleaved rounds, median per-launch time. One JSON line per shape."""
import json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def shapes(B):
    E, D = B * 50, B * 197
    return [("enc qkv fwd", E, 2304, 768, 0), ("enc fc1 dgrad", E, 768, 3072, 1), ("enc qkv dgrad", E, 768, 2304, 1),
            ("enc proj dgrad", E, 768, 768, 1), ("dec qkv fwd", D, 1536, 512, 0), ("dec fc1 dgrad", D, 512, 2048, 1),
            ("dec qkv dgrad", D, 512, 1536, 1), ("dec proj dgrad", D, 512, 512, 1), ("dec pred dgrad", D, 512, 768, 1)]


def time_one(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for B in (128, 256):
    for name, M, N, Kd, lb in shapes(B):
        A = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
        Bm = ((torch.randn(N, Kd, device=dev) if lb == 0 else torch.randn(Kd, N, device=dev)) * 0.5).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: K.gemm(A, Bm, C, M, N, Kd, A.stride(0), Bm.stride(0), N, 0, lb)
        t = {"0": [], "2": []}
        for mode in ("0", "2"):
            os.environ["MAECLIP_GEMM_LIB"] = mode
            fn(); fn()
        torch.cuda.synchronize()
        for r in range(5):
            for mode in ("0", "2"):
                os.environ["MAECLIP_GEMM_LIB"] = mode
                t[mode].append(time_one(fn))
        a, b = statistics.median(t["0"]), statistics.median(t["2"])
        print(json.dumps(dict(B=B, name=name, M=M, N=N, K=Kd, own_us=round(a, 1), vendor_us=round(b, 1),
                              vendor_speedup=round(a / b, 3))), flush=True)
