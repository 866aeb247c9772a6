import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import build_pair, make_batch
from mae_clip_amd import kernels as K

def d(name, a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    print(f"{name:28s} maxabs={(a-b).abs().max().item():.3e} scale={b.abs().max().item():.3e}")

prod, ref = build_pair("fp32", mask_ratio=0.0)
prod.eval(); ref.eval()
b = make_batch(8, 32)
ids = b["input_ids"]; am = b["attention_mask"]
tm = prod.text_encoder.model; rm = ref.text_encoder.model
B, T, D, H = 8, 25, 768, 12
with torch.no_grad():
    x = rm.embeddings(ids)
    xg = x.float().cuda().view(B * T, D)
    lyr = tm.transformer.layer[0]; rl = rm.transformer.layer[0]
    wqkv, bqkv, wout, w1, w2 = tm._weights(torch.float32)[0]
    qkv = K.linear_fwd(xg, wqkv, bqkv)
    at = rl.attention
    rq, rk, rv = at.q_lin(x), at.k_lin(x), at.v_lin(x)
    d("qkv", qkv.view(B, T, -1), torch.cat([rq, rk, rv], -1))
    amf = am.float().cuda()
    o, _ = K.attn_fwd(qkv, B, T, H, 64, 64 ** -0.5, key_mask=amf, want_lse=False)
    sh = lambda t: t.view(B, T, H, 64).transpose(1, 2)
    s = (sh(rq) @ sh(rk).transpose(-1, -2)) * 64 ** -0.5
    ro = (s.softmax(-1) @ sh(rv)).transpose(1, 2).reshape(B, T, D)
    d("attn o", o.view(B, T, D), ro)
    o2, _ = K.attn_fwd(qkv, B, T, H, 64, 64 ** -0.5, key_mask=None, want_lse=False)
    d("attn o (no mask)", o2.view(B, T, D), ro)
    sa = K.linear_fwd(o, wout, lyr.attention.out_lin.bias, out_dtype=torch.float32)
    d("out_lin", sa.view(B, T, D), at.out_lin(ro))
    a = K.ln_fwd(sa, lyr.sa_layer_norm.weight, lyr.sa_layer_norm.bias, 1e-12, res=xg, want_stats=False)[0]
    ra = rl.sa_layer_norm(at.out_lin(ro) + x)
    d("sa_ln", a.view(B, T, D), ra)
    pre = torch.empty((B * T, 3072), device="cuda")
    f1 = K.linear_fwd(a, w1, lyr.ffn.lin1.bias, epilogue=K.EPI_GELU, aux_out=pre)
    d("lin1 pre", pre.view(B, T, -1), rl.ffn.lin1(ra))
    d("gelu", f1.view(B, T, -1), torch.nn.functional.gelu(rl.ffn.lin1(ra)))
    f2 = K.linear_fwd(f1, w2, lyr.ffn.lin2.bias, out_dtype=torch.float32)
    d("lin2", f2.view(B, T, D), rl.ffn(ra))
    h = K.ln_fwd(f2, lyr.output_layer_norm.weight, lyr.output_layer_norm.bias, 1e-12, res=a, want_stats=False)[0]
    d("out_ln", h.view(B, T, D), rl(x, am))
