"""Time the fused soft-target CLIP loss (maeclip_clip_loss, CLIP.py:34-43,
forward + gradient rows in one call) at the batch sizes of BASELINE.json:
N = 256 (C1/C2, one GPU), N = 1024 (C4 global batch, 128 gradient rows per
rank) and N = 2048 (C3 global batch, the 256 gradient rows of rank r).
HIP events on the launching stream, 50 calls after 5 warm-ups; also checks
each rank's gradient rows against the full-gradient call. One JSON line per case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
cases = [(256, None, "C1/C2 N=256 full"), (1024, (0, 128), "C4 N=1024 rows 0..127"),
         (1024, (896, 128), "C4 N=1024 rows 896..1023"), (2048, (0, 256), "C3 N=2048 rows 0..255 (rank 0)"),
         (2048, (1792, 256), "C3 N=2048 rows 1792..2047 (rank 7)"), (2048, None, "N=2048 all rows")]
g = torch.Generator(device="cpu").manual_seed(0)
for N, rows, name in cases:
    I = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g), (256,)).to(dev)
    T = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g), (256,)).to(dev)
    for _ in range(5):
        K.clip_loss(I, T, 1.0, want_grad=True, grad_rows=rows)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    s.record()
    for _ in range(reps):
        K.clip_loss(I, T, 1.0, want_grad=True, grad_rows=rows)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    rec = dict(case=name, N=N, grad_rows=rows, us_per_call=round(us, 2),
               gflops=round((6 + 8) * N * N * 256 / 1e9, 3))
    if rows is not None:
        lf, dIf, dTf = K.clip_loss(I, T, 1.0)
        lr, dIr, dTr = K.clip_loss(I, T, 1.0, grad_rows=rows)
        r0, nr = rows
        rec["rows_match_full"] = bool(torch.equal(dIr, dIf[r0:r0 + nr]) and torch.equal(dTr, dTf[r0:r0 + nr])
                                      and torch.equal(lr, lf))
    print(json.dumps(rec), flush=True)
