"""Per-phase cycle split of the v4 GEMM from a GEMM4_STAMPS build:
MAECLIP_LIB=mae_clip_amd/libmaeclip_stamps.so MAECLIP_GEMM_VARIANT=8 python tools/stamp_run.py"""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mae_clip_amd import kernels as K, _lib
dev = torch.device("cuda")
D, E = 256 * 197, 256 * 50
lib = _lib.load()
fn = lib.maeclip_debug_gemm4_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
NS = 256 * 8 * 2 * 4


def read():
    buf = np.zeros(NS, dtype=np.uint64)
    assert fn(buf.ctypes.data, NS) == 0
    return buf.reshape(256, 8, 2, 4).astype(np.int64)


cases = [("dec fc2 dgrad none", D, 2048, 512, K.EPI_NONE), ("dec fc2 dgrad mulaux", D, 2048, 512, K.EPI_MUL_AUX),
         ("dec fc1 fwd gelu_d", D, 2048, 512, ("fwd", K.EPI_GELU_D)), ("dec fc2 fwd resid", D, 512, 2048, ("fwd", K.EPI_RESID)),
         ("enc fc1 fwd none", E, 3072, 768, ("fwd", K.EPI_NONE))]
for name, M, N, Kd, epi in cases:
    if isinstance(epi, tuple):
        x = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) * 0.5).to(torch.bfloat16)
        e = epi[1]
        if e == K.EPI_GELU_D:
            bias, aux_out = torch.randn(N, device=dev), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            f = lambda: K.linear_fwd(x, w, bias, epilogue=e, aux_out=aux_out)
        elif e == K.EPI_RESID:
            bias, res = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
            f = lambda: K.linear_fwd(x, w, bias, out_dtype=torch.float32, epilogue=e, resid=res)
        else:
            f = lambda: K.linear_fwd(x, w)
    else:
        dy = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(Kd, N, device=dev) * 0.5).to(torch.bfloat16)
        aux = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == K.EPI_MUL_AUX else None
        f = lambda: K.linear_dgrad(dy, w, epilogue=epi, aux=aux)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s = read()
    t0 = s[:, :, :, 0][s[:, :, :, 0] > 0].min()
    tiles = (M + 255) // 256 * ((N + 255) // 256)
    per = (tiles + 255) // 256
    print(f"===== {name}: {tiles} tiles, <= {per} per block")
    for ti in range(min(per, 8)):
        for w in range(2):
            v = s[:, ti, w, :]
            ok = v[:, 0] > 0
            v = v[ok]
            if len(v) == 0:
                continue
            wait, main, epi_ = v[:, 1] - v[:, 0], v[:, 2] - v[:, 1], v[:, 3] - v[:, 2]
            start = v[:, 0] - t0
            print(f"tile{ti} grp{w}: start p10/50/90 {np.percentile(start,10):8.0f} {np.median(start):8.0f} {np.percentile(start,90):8.0f} | "
                  f"wait {np.median(wait):7.0f} main {np.median(main):7.0f} (p90 {np.percentile(main,90):7.0f}) epi {np.median(epi_):7.0f} (n={len(v)})")
