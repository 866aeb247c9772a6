"""Where the epilogue-heavy GEMMs spend their time: the same launch (shape,
layouts, tile plan) with the epilogue switched -- no epilogue (bf16 C only),
GELU without / with the second bf16 output, GELU + GELU' output (the step's
fc1 forward), and the fc2 dgrad with / without the GELU' multiply. The
difference between rows is the epilogue's own cost (VALU math, second store
stream, aux read). One JSON line per (shape, epilogue): median us per launch,
algorithmic bytes and the rate they imply."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


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


def run(tag, M, N, Kd, variants):
    g = torch.Generator(device=dev).manual_seed(M + N + Kd)
    a = (torch.randn(M, Kd, generator=g, device=dev)).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g, device=dev) * 0.05).to(torch.bfloat16)   # [N, K]
    wt = w.t().contiguous()                                                           # [K, N]
    bias = torch.randn(N, device=dev) * 0.1
    aux = torch.rand(M, N, generator=g, device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    aux_out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for name, epi, kw, bl in variants:
        kws = {}
        nbytes = (M * Kd + N * Kd) * 2 + M * N * 2
        if "bias" in kw:
            kws["bias"] = bias
        if "aux_out" in kw:
            kws.update(aux_out=aux_out, ldaux=N)
            nbytes += M * N * 2
        if "aux" in kw:
            kws.update(aux=aux, ldaux=N)
            nbytes += M * N * 2
        B = w if bl == K.KC else wt
        ldb = Kd if bl == K.KC else N
        fn = lambda: K.gemm(a, B, C, M, N, Kd, Kd, ldb, N, K.KC, bl, epilogue=epi, **kws)
        t = statistics.median(time_fn(fn) for _ in range(3))
        print(json.dumps(dict(shape=tag, M=M, N=N, K=Kd, epilogue=name, us=round(t, 1), alg_MB=round(nbytes / 1e6, 1),
                              TBps=round(nbytes / t / 1e6, 2), TFs=round(2.0 * M * N * Kd / t / 1e6, 1))), flush=True)


FWD = [("none", K.EPI_NONE, (), K.KC), ("none+bias", K.EPI_NONE, ("bias",), K.KC),
       ("gelu", K.EPI_GELU, ("bias",), K.KC), ("gelu+pre_out", K.EPI_GELU, ("bias", "aux_out"), K.KC),
       ("gelu+gelu'_out", K.EPI_GELU_D, ("bias", "aux_out"), K.KC)]
DGRAD = [("none", K.EPI_NONE, (), K.RC), ("mul_aux", K.EPI_MUL_AUX, ("aux",), K.RC)]

for M in (25216, 50432):
    run("dec fc1 fwd", M, 2048, 512, FWD)
    run("dec fc2 dgrad", M, 2048, 512, DGRAD)
for M in (6400, 12800):
    run("enc fc1 fwd", M, 3072, 768, FWD)
    run("enc fc2 dgrad", M, 3072, 768, DGRAD)
