"""Contention scan of the persistent v4 GEMM: the same launch with the grid
capped at 256 / 128 / 64 workgroups (MAECLIP_GEMM_GRID). Per-CU tile time =
launch time / rounds; if it stays flat as the grid shrinks the kernel is bound
per CU (issue / MFMA / LDS), if it drops the full-chip launch is bound by a
shared resource (HBM / fabric / L2). Production epilogues of the C2 step."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
D, E = 256 * 197, 256 * 50


def t_us(f, reps=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def mk(r, c):
    return (torch.randn(r, c, device=dev) * 0.5).to(torch.bfloat16)


cases = []
x, w = mk(D, 512), mk(2048, 512)
aux_out = torch.empty(D, 2048, device=dev, dtype=torch.bfloat16)
bias = torch.randn(2048, device=dev)
cases.append(("dec fc1 fwd gelu_d", D, 2048, 512, lambda: K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU_D, aux_out=aux_out)))
cases.append(("dec fc1 fwd none", D, 2048, 512, lambda: K.linear_fwd(x, w)))
dy, w2 = mk(D, 512), mk(512, 2048)
aux = torch.rand(D, 2048, device=dev).to(torch.bfloat16)
cases.append(("dec fc2 dgrad mulaux", D, 2048, 512, lambda: K.linear_dgrad(dy, w2, epilogue=K.EPI_MUL_AUX, aux=aux)))
a2, w3 = mk(D, 2048), mk(512, 2048)
res, b3 = torch.randn(D, 512, device=dev), torch.randn(512, device=dev)
cases.append(("dec fc2 fwd resid", D, 512, 2048, lambda: K.linear_fwd(a2, w3, b3, out_dtype=torch.float32,
                                                                         epilogue=K.EPI_RESID, resid=res)))
xe, we = mk(E, 768), mk(3072, 768)
cases.append(("enc fc1 fwd none", E, 3072, 768, lambda: K.linear_fwd(xe, we)))
for name, M, N, Kd, f in cases:
    tiles = (M + 255) // 256 * ((N + 255) // 256)
    out = dict(name=name, tiles=tiles)
    for g in (256, 128, 64):
        os.environ["MAECLIP_GEMM_GRID"] = str(g)
        os.environ["MAECLIP_GEMM_BM"] = "256"
        us = t_us(f)
        rounds = (tiles + g - 1) // g
        out[f"g{g}_us"] = round(us, 1)
        out[f"g{g}_us_per_round"] = round(us / rounds, 2)
    os.environ.pop("MAECLIP_GEMM_GRID")
    os.environ.pop("MAECLIP_GEMM_BM")
    print(json.dumps(out), flush=True)
