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
ts = []
for _ in range(reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    K.wgrad_grouped(items)
    e.record()
    ts.append((s, e))
torch.cuda.synchronize()
us = sorted(s.elapsed_time(e) * 1e3 for s, e in ts)[len(ts) // 2]
flops = sum(2.0 * M * it[0].shape[1] * it[1].shape[1] for it in items)
print("ok", len(items), "problems,", reps, "launches, median", round(us, 1), "us,", round(flops / us / 1e6, 1), "TF/s")
