"""LayerNorm kernels alone at the micro-batch shapes of the C2 step (decoder
25216 x 512, encoder 6400 x 768) and at the whole batch: time per launch and
the HBM rate of the bytes each moves (forward: x f32 read, y bf16 written;
backward: dy bf16, x f32, residual gradient f32 read, dx f32 + bf16 copy
written). Separates the kernels' own rate from the in-step contention."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def time_fn(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


for name, M, D in (("dec mb", 128 * 197, 512), ("enc mb", 128 * 50, 768), ("dec", 256 * 197, 512),
                   ("enc", 256 * 50, 768)):
    x = torch.randn(M, D, device=dev)
    g = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    tf = time_fn(lambda: K.ln_fwd(x, g, b, 1e-6, out_dtype=torch.bfloat16, y_out=y, mean_out=mean, rstd_out=rstd))
    # every row written, and right (bf16 rounding of the torch fp32 reference)
    ref = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-6)
    err = ((y.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
    assert err < 1e-2, (name, err)
    assert torch.allclose(mean, x.mean(1), atol=1e-5) and torch.allclose(rstd, torch.rsqrt(x.var(1, unbiased=False) + 1e-6), rtol=1e-4)
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, D, device=dev)
    tb = time_fn(lambda: K.ln_bwd(dy, x, mean, rstd, g, dres=dres, want_bf16=True, want_colsum=True))
    fb = M * D * (4 + 2) + M * 8
    bb = M * D * (2 + 4 + 4 + 4 + 2)
    print(json.dumps(dict(name=name, M=M, D=D, fwd_us=round(tf * 1e6, 1), fwd_TBps=round(fb / tf / 1e12, 2),
                          bwd_us=round(tb * 1e6, 1), bwd_TBps=round(bb / tb / 1e12, 2))), flush=True)
