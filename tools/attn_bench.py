"""Attention fwd/bwd kernel time at the production shapes of the C2 step
(ViT-B/16 MAE+CLIP, B=256) vs torch SDPA (for reference only), plus a
numerics check of the bwd against fp32 torch autograd on a small batch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
SHAPES = [("enc", 256, 50, 12, 64), ("dec", 256, 197, 16, 32), ("text", 256, 25, 12, 64),
          ("C1 enc", 256, 197, 12, 64), ("C4 enc", 128, 145, 16, 64), ("C4 dec", 128, 577, 16, 32)]


def time_fn(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def ref(qkv, B, n, H, hd):
    x = qkv.float().view(B, n, 3, H, hd).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(x[0], x[1], x[2]).permute(0, 2, 1, 3).reshape(B * n, H * hd)


for name, B, n, H, hd in SHAPES:
    D = H * hd
    qkv = (torch.randn(B * n, 3 * D, device=dev)).to(torch.bfloat16)
    dout = (torch.randn(B * n, D, device=dev) * 0.1).to(torch.bfloat16)
    scale = hd ** -0.5
    o, lse = K.attn_fwd(qkv, B, n, H, hd, scale)
    tf = time_fn(lambda: K.attn_fwd(qkv, B, n, H, hd, scale))
    tb = time_fn(lambda: K.attn_bwd(qkv, o, dout, lse, B, n, H, hd, scale))
    fl = 4.0 * B * H * n * n * hd
    # numerics on 4 samples
    b4 = 4
    q4 = qkv[: b4 * n].float().requires_grad_(True)
    r = ref(q4, b4, n, H, hd)
    r.backward(dout[: b4 * n].float())
    dq, _ = K.attn_bwd(qkv, o, dout, lse, B, n, H, hd, scale)
    err_o = ((o[: b4 * n].float() - r).abs().max() / r.abs().max()).item()
    err_d = ((dq[: b4 * n].float() - q4.grad).abs().max() / q4.grad.abs().max()).item()
    print(json.dumps(dict(name=name, B=B, n=n, H=H, hd=hd, fwd_us=round(tf * 1e6, 1), bwd_us=round(tb * 1e6, 1),
                          fwd_tflops=round(fl / tf / 1e12, 1), bwd_tflops=round(2.5 * fl / tb / 1e12, 1),
                          rel_err_o=err_o, rel_err_dqkv=err_d)), flush=True)
