"""Run one GEMM shape repeatedly (for rocprofv3 --pmc / --kernel-trace).

usage: python tools/gemm_one.py M N K a_layout b_layout [epilogue] [reps]
  layouts: 0 = KC (row-major, K contiguous), 1 = RC (K-major rows)
  epilogue: 0 none, 1 gelu, 2 resid(f32 out), 4 gelu+gelu' aux_out, 5 mul-aux
The operands are random bf16 (random data: DVFS, MI355X_MICROARCH.md).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

argv = [int(x) for x in sys.argv[1:]]
M, N, Kd, la, lb = argv[:5] if len(argv) >= 5 else (12800, 3072, 768, 0, 0)
epi = argv[5] if len(argv) > 5 else 0
reps = argv[6] if len(argv) > 6 else 20
dev = torch.device("cuda")
A = (torch.randn((M, Kd) if la == 0 else (Kd, M), device=dev) * 0.5).to(torch.bfloat16)
B = (torch.randn((N, Kd) if lb == 0 else (Kd, N), device=dev) * 0.5).to(torch.bfloat16)
out_dtype = torch.float32 if epi == K.EPI_RESID else torch.bfloat16
C = torch.empty(M, N, device=dev, dtype=out_dtype)
kw = {}
if epi == K.EPI_RESID:
    kw = dict(resid=torch.randn(M, N, device=dev), ldr=N)
elif epi in (K.EPI_GELU, K.EPI_GELU_D):
    kw = dict(aux_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16), ldaux=N,
              bias=torch.randn(N, device=dev))
elif epi in (K.EPI_MUL_AUX, K.EPI_DGELU):
    kw = dict(aux=torch.rand(M, N, device=dev).to(torch.bfloat16), ldaux=N)
for _ in range(reps):
    K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, la, lb, epilogue=epi, **kw)
torch.cuda.synchronize()
