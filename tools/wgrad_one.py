"""The C2 step's decoder weight-gradient launch alone: one maeclip_wgrad_grouped
call over the 8 layers x (fc2, fc1, proj, qkv) problems at M = 256 * 197 tokens,
in the backward's order (the bench key wgrad_grouped M50432 x32 N512 K2048).
usage: python tools/wgrad_one.py [reps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda")
M, D, F = 256 * 197, 512, 2048
g = torch.Generator(device=dev).manual_seed(0)


def mk(r, c):
    return (torch.randn(r, c, device=dev, generator=g) * 0.5).to(torch.bfloat16)


items = []
for _ in range(8):
    for n, k in ((D, F), (F, D), (D, D), (3 * D, D)):   # fc2, fc1, proj, qkv
        items.append((mk(M, n), mk(M, k), torch.empty(n, k, device=dev)))
for _ in range(reps):
    K.wgrad_grouped(items)
torch.cuda.synchronize()
print("ok", len(items), "problems,", reps, "launches")
