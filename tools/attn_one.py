"""Run one attention shape repeatedly (for rocprofv3 --pmc / --kernel-trace).
usage: python tools/attn_one.py B n H hd [bwd=1] [reps=20]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K
B, n, H, hd = (int(x) for x in sys.argv[1:5])
bwd = int(sys.argv[5]) if len(sys.argv) > 5 else 1
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda")
qkv = (torch.randn(B * n, 3 * H * hd, device=dev) * 0.5).to(torch.bfloat16)
o, lse = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
do = (torch.randn(B * n, H * hd, device=dev) * 0.5).to(torch.bfloat16)
for _ in range(reps):
    if bwd:
        K.attn_bwd(qkv, o, do, lse, B, n, H, hd, hd ** -0.5)
    else:
        K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
torch.cuda.synchronize()
