"""Per-phase cycle split of the attention forward from an ATTN_STAMPS build:
MAECLIP_LIB=mae_clip_amd/libmaeclip_stamps.so python tools/attn_fwd_stamps.py B n H hd
stamps: 0 start, 1 K/V images in LDS (after the barrier), 2 first query tile done, 3 exit"""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mae_clip_amd import kernels as K, _lib
B, n, H, hd = (int(x) for x in sys.argv[1:5])
lib = _lib.load()
fn = lib.maeclip_debug_attn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
NS = 4096 * 8 * 8
qkv = (torch.randn(B * n, 3 * H * hd, device="cuda") * 0.5).to(torch.bfloat16)
for _ in range(3):
    K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
torch.cuda.synchronize()
buf = np.zeros(NS, dtype=np.uint64)
assert fn(buf.ctypes.data, NS) == 0
s = buf.reshape(4096, 8, 8).astype(np.int64)[: min(4096, B * H)]
nw = int((s[0, :, 0] > 0).sum())
s = s[:, :nw]
life = s[:, :, 3].max(1) - s[:, :, 0].min(1)
print(f"{len(s)} workgroups x {nw} waves; WG lifetime median {np.median(life):.0f}")
for nm, (x, y) in (("load K/V", (0, 1)), ("first tile", (1, 2)), ("rest", (2, 3))):
    d = s[:, :, y] - s[:, :, x]
    print(f"  {nm:11s} per wave p10/50/90 {np.percentile(d,10):7.0f} {np.median(d):7.0f} {np.percentile(d,90):7.0f}")
print("  exit by wave (median, from start):", np.median(s[:, :, 3] - s[:, :, 0].min(1)[:, None], axis=0).astype(int).tolist())
