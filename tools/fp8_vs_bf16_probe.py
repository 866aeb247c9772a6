"""C4 encoder GEMM shapes (ViT-L/14@336, B = 128 micro-batched to 64: M = 9280
token rows; whole batch 18560) on the fp8 kernel vs the bf16 kernel with the
same epilogue: per-launch median time (us) and the fp8 / bf16 speed ratio.
The fp8 operands are quantised once outside the timing (the step's separate
quantisation passes are not in these numbers). One JSON line per shape."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def shapes(M):
    # name, N, K, epilogue, A fmt (fwd: e4m3 activations, dgrad: e5m2 gradients)
    return [("qkv fwd", M, 3072, 1024, K.EPI_NONE, K.FP8_E4M3), ("proj fwd+res", M, 1024, 1024, K.EPI_RESID, K.FP8_E4M3),
            ("fc1 fwd gelu'", M, 4096, 1024, K.EPI_GELU_D, K.FP8_E4M3),
            ("fc2 fwd+res", M, 1024, 4096, K.EPI_RESID, K.FP8_E4M3),
            ("fc2 dgrad*gelu'", M, 4096, 1024, K.EPI_MUL_AUX, K.FP8_E5M2),
            ("fc1 dgrad", M, 1024, 4096, K.EPI_NONE, K.FP8_E5M2), ("qkv dgrad", M, 1024, 3072, K.EPI_NONE, K.FP8_E5M2),
            ("proj dgrad", M, 1024, 1024, K.EPI_NONE, K.FP8_E5M2)]


def time_fn(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) * 1e3 for s, e in ts)


for M in (9280, 18560):
    for name, M_, N, Kd, epi, fmt in shapes(M):
        g = torch.Generator(device=dev).manual_seed(N + Kd)
        a = torch.randn(M_, Kd, generator=g, device=dev)
        w = torch.randn(N, Kd, generator=g, device=dev) * 0.05
        ab, wb = a.to(torch.bfloat16), w.to(torch.bfloat16)
        aq, wq = K.quant_rows_fp8(ab, fmt), K.quant_rows_fp8(wb, K.FP8_E4M3)
        out = torch.float32 if epi == K.EPI_RESID else torch.bfloat16
        C = torch.empty(M_, N, device=dev, dtype=out)
        kw = {}
        if epi == K.EPI_RESID:
            kw = dict(resid=torch.randn(M_, N, generator=g, device=dev))
        elif epi == K.EPI_GELU_D:
            kw = dict(aux_out=torch.empty(M_, N, device=dev, dtype=torch.bfloat16), bias=torch.randn(N, device=dev))
        elif epi == K.EPI_MUL_AUX:
            kw = dict(aux=torch.rand(M_, N, generator=g, device=dev).to(torch.bfloat16))
        f8 = lambda: K.gemm_fp8(aq, wq, C, epilogue=epi, **kw)
        kwb = dict(kw)
        if "resid" in kwb:
            kwb["ldr"] = N
        if "aux_out" in kwb or "aux" in kwb:
            kwb["ldaux"] = N
        bf = lambda: K.gemm(ab, wb, C, M_, N, Kd, Kd, Kd, N, K.KC, K.KC, epilogue=epi, **kwb)
        t8, tb = [], []
        for _ in range(3):
            t8.append(time_fn(f8))
            tb.append(time_fn(bf))
        t8, tb = statistics.median(t8), statistics.median(tb)
        fl = 2.0 * M_ * N * Kd
        print(json.dumps(dict(M=M_, name=name, N=N, K=Kd, fp8_us=round(t8, 1), bf16_us=round(tb, 1),
                              fp8_speedup=round(tb / t8, 3), fp8_tflops=round(fl / t8 / 1e6, 1),
                              bf16_tflops=round(fl / tb / 1e6, 1))), flush=True)
