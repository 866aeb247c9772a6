"""Per-phase cycle split of the attention backward from an ATTN_STAMPS build:
MAECLIP_LIB=mae_clip_amd/libmaeclip_stamps.so python tools/attn_stamps.py B n H hd"""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mae_clip_amd import kernels as K, _lib
B, n, H, hd = (int(x) for x in sys.argv[1:5])
dev = torch.device("cuda")
lib = _lib.load()
fn = lib.maeclip_debug_attn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
NS = 4096 * 8 * 8
qkv = (torch.randn(B * n, 3 * H * hd, device=dev) * 0.5).to(torch.bfloat16)
o, lse = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
do = (torch.randn(B * n, H * hd, device=dev) * 0.5).to(torch.bfloat16)
for colsum in (False, True):
    for _ in range(3):
        K.attn_bwd(qkv, o, do, lse, B, n, H, hd, hd ** -0.5, want_colsum=colsum)
    torch.cuda.synchronize()
    buf = np.zeros(NS, dtype=np.uint64)
    assert fn(buf.ctypes.data, NS) == 0
    s = buf.reshape(4096, 8, 8).astype(np.int64)[: B * H]
    nw = int((s[0, :, 0] > 0).sum())
    s = s[:, :nw]
    t0 = s[:, :, 0].min()
    wg_start = s[:, :, 0].min(1) - t0
    wg_end = s[:, :, 5].max(1) - t0 if colsum else s[:, :, 4].max(1) - t0
    print(f"== colsum {colsum}: {B*H} workgroups x {nw} waves; span {wg_end.max()} cycles; "
          f"WG lifetime median {np.median(wg_end - wg_start):.0f}")
    names = ["prologue", "phase1", "ph1->ph2", "phase2", "colsum"]
    for k in range(5 if colsum else 4):
        d = s[:, :, k + 1] - s[:, :, k]
        print(f"  {names[k]:9s} per wave p10/50/90 {np.percentile(d,10):7.0f} {np.median(d):7.0f} {np.percentile(d,90):7.0f}"
              f"   wave-max median {np.median(d.max(1)):7.0f}")
    if (s[:, :, 6] > 0).all():
        for nm, (x, y) in (("pro:loads+zero", (0, 6)), ("pro:lds+shfl", (6, 7)), ("pro:barrier", (7, 1))):
            d = s[:, :, y] - s[:, :, x]
            print(f"  {nm:15s} per wave p10/50/90 {np.percentile(d,10):7.0f} {np.median(d):7.0f} {np.percentile(d,90):7.0f}")
    per_wave_p1 = np.median(s[:, :, 2] - s[:, :, 1], axis=0)
    print("  phase1 median by wave:", per_wave_p1.astype(int).tolist())
    starts = np.sort(wg_start)
    print("  WG start gaps: first 8", starts[:8].tolist(), " concurrency ~",
          f"{np.median(wg_end - wg_start) * len(starts) / max(1, wg_end.max()) :.1f} WGs in flight")
