"""LayerNorm forward / backward kernel time at the C2 step's shapes (decoder
50432 x 512, encoder 12800 x 768) and the bytes each moves."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K

dev = torch.device("cuda")


def time_fn(fn, reps=30):
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


for name, M, D in (("dec", 256 * 197, 512), ("enc", 256 * 50, 768), ("dec mb", 128 * 197, 512), ("enc mb", 128 * 50, 768)):
    x = torch.randn(M, D, device=dev)
    res = torch.randn(M, D, device=dev)
    g = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    y, mean, rstd, yb, xs = K.ln_fwd(x, g, b, 1e-6, out_dtype=torch.bfloat16, res=res, xsum=True)
    tf = time_fn(lambda: K.ln_fwd(x, g, b, 1e-6, out_dtype=torch.bfloat16, res=res, xsum=True))
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, D, device=dev)
    tb = time_fn(lambda: K.ln_bwd(dy, xs, mean, rstd, g, dres=dres, want_bf16=True, want_colsum=True))
    bb = M * D * (2 + 4 + 4 + 4 + 2)
    print(json.dumps(dict(name=name, M=M, D=D, fwd_us=round(tf * 1e6, 1), bwd_us=round(tb * 1e6, 1),
                          bwd_TBps=round(bb / tb / 1e12, 2))), flush=True)
