"""Hash the attention backward outputs at the diagonal kernel's shapes (fixed
seeds, 5 repeats each): run once per library build (MAECLIP_LIB=...) and compare
the printed hashes -- equal hashes = bitwise-identical results across builds and
repeats. usage: python tools/attn_bitcmp.py"""
import hashlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mae_clip_amd import kernels as K
dev = torch.device("cuda")
out = {}
for (B, n, H, hd) in [(256, 197, 16, 32), (64, 197, 12, 64), (32, 50, 12, 64), (16, 33, 16, 32), (8, 256, 16, 32)]:
    g = torch.Generator(device="cpu").manual_seed(1234 + n)
    qkv = torch.randn(B * n, 3 * H * hd, generator=g).to(dev).to(torch.bfloat16)
    do = (torch.randn(B * n, H * hd, generator=g) * 0.5).to(dev).to(torch.bfloat16)
    o, lse = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
    hs = set()
    for _ in range(5):
        dq, part = K.attn_bwd(qkv, o, do, lse, B, n, H, hd, hd ** -0.5)
        torch.cuda.synchronize()
        hs.add(hashlib.sha256(dq.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16])
    out[f"{B}x{n}x{H}x{hd}"] = sorted(hs)
print(json.dumps(out))
