"""Run one GEMM shape repeatedly (for rocprofv3 --pmc)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K
M, N, Kd, la, lb = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (12800, 3072, 768, 0, 0)))
dev = torch.device("cuda")
A = (torch.randn((M, Kd) if la == 0 else (Kd, M), device=dev) * 0.5).to(torch.bfloat16)
B = (torch.randn((N, Kd) if lb == 0 else (Kd, N), device=dev) * 0.5).to(torch.bfloat16)
C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(20):
    K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, la, lb)
torch.cuda.synchronize()
