"""Micro-batch stream overlap probe: a transformer stack's forward chain
(LN -> qkv -> attention -> proj+res -> LN -> fc1+GELU' -> fc2+res) on the whole
batch on one stream, against the same chain on two half-batches issued
alternately on two streams (their kernels fill each other's partial last
rounds and launch gaps). Prints ms per stack for both and the ratio.
usage: python tools/mb_overlap.py [dec|enc] [splits]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")
which = sys.argv[1] if len(sys.argv) > 1 else "dec"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 2
B, n, D, H, depth = (256, 197, 512, 16, 8) if which == "dec" else (256, 50, 768, 12, 12)
hd = D // H
bf = torch.bfloat16
g = torch.Generator(device="cpu").manual_seed(0)
W = dict(qkv=(torch.randn(3 * D, D, generator=g) * 0.02).to(dev, bf), proj=(torch.randn(D, D, generator=g) * 0.02).to(dev, bf),
         fc1=(torch.randn(4 * D, D, generator=g) * 0.02).to(dev, bf), fc2=(torch.randn(D, 4 * D, generator=g) * 0.02).to(dev, bf))
bq = torch.zeros(3 * D, device=dev)
bp = torch.zeros(D, device=dev)
b1 = torch.zeros(4 * D, device=dev)
b2 = torch.zeros(D, device=dev)
lw = torch.ones(D, device=dev)
lb = torch.zeros(D, device=dev)


def block(x, Bs):
    M = Bs * n
    h1 = K.ln_fwd(x, lw, lb, 1e-6, out_dtype=bf)[0]
    qkv = K.linear_fwd(h1, W["qkv"], bias=bq)
    o, _ = K.attn_fwd(qkv, Bs, n, H, hd, hd ** -0.5)
    x1 = K.linear_fwd(o, W["proj"], bias=bp, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=x)
    h2 = K.ln_fwd(x1, lw, lb, 1e-6, out_dtype=bf)[0]
    dg = torch.empty((M, 4 * D), device=dev, dtype=bf)
    a = K.linear_fwd(h2, W["fc1"], bias=b1, epilogue=K.EPI_GELU_D, aux_out=dg)
    return K.linear_fwd(a, W["fc2"], bias=b2, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=x1)


x0 = torch.randn(B * n, D, device=dev, generator=None) * 0.5
streams = [torch.cuda.Stream() for _ in range(S)]


def run_one():
    x = x0
    for _ in range(depth):
        x = block(x, B)
    return x


def run_split():
    main = torch.cuda.current_stream()
    Bs = B // S
    xs = [x0[i * Bs * n:(i + 1) * Bs * n] for i in range(S)]
    for s in streams:
        s.wait_stream(main)
    for _ in range(depth):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                xs[i] = block(xs[i], Bs)
    for s in streams:
        main.wait_stream(s)
    return xs


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g_ = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_):
        fn()
    for _ in range(3):
        g_.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g_.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t1 = timed(run_one)
t2 = timed(run_split)
y1 = run_one()
y2 = torch.cat(run_split())
torch.cuda.synchronize()
print(f"{which} stack fwd (depth {depth}, B {B}): one stream {t1:.3f} ms, {S} half-batches on {S} streams {t2:.3f} ms, "
      f"ratio {t2 / t1:.3f}, bitwise equal {torch.equal(y1, y2)}")
