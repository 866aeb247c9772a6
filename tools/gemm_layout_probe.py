"""Why is the KC x KC (forward) GEMM slower than KC x RC (dgrad) at equal
shapes (profiles/r04/gemm_sq_vs_hipblaslt.jsonl: sq4096 1056 vs 1184 TF/s)?
Times the same product with B stored [N][K] (KC) and [K][N] (RC), with and
without a padded leading dimension (power-of-two row strides alias in the
caches), plain epilogue, bf16 out. usage: python tools/gemm_layout_probe.py"""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def time_fn(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


for (M, N, Kd) in [(4096, 4096, 4096), (8192, 8192, 8192), (12800, 3072, 768), (12800, 768, 3072),
                   (50432, 2048, 512), (50432, 512, 2048)]:
    res = {"M": M, "N": N, "K": Kd}
    for pad in (0, 64):
        A = (torch.randn(M, Kd + pad, device=dev) * 0.5).to(torch.bfloat16)
        Bk = (torch.randn(N, Kd + pad, device=dev) * 0.5).to(torch.bfloat16)     # KC: [N][K]
        Br = (torch.randn(Kd, N + pad, device=dev) * 0.5).to(torch.bfloat16)     # RC: [K][N]
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * Kd
        t = time_fn(lambda: K.gemm(A, Bk, C, M, N, Kd, A.stride(0), Bk.stride(0), N, 0, 0))
        res[f"KC_KC_pad{pad}"] = round(fl / t / 1e12, 1)
        t = time_fn(lambda: K.gemm(A, Br, C, M, N, Kd, A.stride(0), Br.stride(0), N, 0, 1))
        res[f"KC_RC_pad{pad}"] = round(fl / t / 1e12, 1)
        del A, Bk, Br, C
    print(json.dumps(res), flush=True)
