"""Stage-by-stage product (GPU, fp32 parity mode) vs oracle (CPU fp64) diffs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import build_pair, make_batch
from mae_clip_amd import functions as Fn, kernels as K
from mae_clip_amd.modules import compute_dtype

def d(name, a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    print(f"{name:28s} maxabs={(a-b).abs().max().item():.3e} scale={b.abs().max().item():.3e}")

for mr in (0.0,):
    prod, ref = build_pair("fp32", mask_ratio=mr)
    prod.eval(); ref.eval()
    b = make_batch(8, 32)
    bd = {k: v.cuda() for k, v in b.items()}
    rb = dict(b, image=b["image"].double())
    dt = torch.float32
    cache = prod._weight_cache()
    vit = prod.image_encoder.model
    rvit = ref.image_encoder.model
    with torch.no_grad():
        # text
        tp = prod.text_encoder(bd["input_ids"], bd["attention_mask"])
        tr = ref.text_encoder(rb["input_ids"], rb["attention_mask"])
        d("text cls", tp, tr)
        x = ref.text_encoder.model.embeddings(rb["input_ids"])
        e = K.embed_fwd(bd["input_ids"], prod.text_encoder.model.embeddings.word_embeddings.weight,
                        prod.text_encoder.model.embeddings.position_embeddings.weight)
        emb = prod.text_encoder.model.embeddings
        h = K.ln_fwd(e, emb.LayerNorm.weight, emb.LayerNorm.bias, 1e-12, want_stats=False)[0]
        d("text emb+LN", h.view(8, 25, -1), x)
        # image tokens
        tok = vit.forward_tokens(bd["image"], dt, cache)
        rtok = rvit.forward_tokens(rb["image"])
        d("vit tokens", tok, rtok)
        t0 = rvit.tokens(rb["image"])
        from mae_clip_amd.functions import PatchSpec, PatchTokensFn
        pe = vit.patch_embed
        spec = PatchSpec(B=8, L=4, keep=4, p=16, kpad=768, dtype=dt, w_T=pe.proj.weight.view(192, 768))
        x0 = PatchTokensFn.apply(bd["image"], None, None, spec, pe.proj.weight, pe.proj.bias, vit.cls_token, vit.pos_embed)
        d("patch tokens", x0, t0)
        # one block
        from mae_clip_amd.modules import run_stack
        y1 = run_stack(vit.blocks[:1], x0, vit.num_heads, dt, cache)
        d("block0", y1, rvit.blocks[0](t0))
        blk = rvit.blocks[0]
        a = blk.attn(blk.norm1(t0))
        # attention only
        h1 = K.ln_fwd(x0.view(-1, 192), vit.blocks[0].norm1.weight, vit.blocks[0].norm1.bias, 1e-6)[0]
        d("ln1", h1.view(8, 5, 192), blk.norm1(t0))
        qkv = K.linear_fwd(h1, vit.blocks[0].attn.qkv.weight, vit.blocks[0].attn.qkv.bias)
        d("qkv", qkv.view(8, 5, -1), blk.attn.qkv(blk.norm1(t0)))
        o, lse = K.attn_fwd(qkv, 8, 5, 3, 64, 64 ** -0.5)
        q, k, v = blk.attn.qkv(blk.norm1(t0)).reshape(8, 5, 3, 3, 64).permute(2, 0, 3, 1, 4)
        ro = ((q @ k.transpose(-1, -2)) * 64 ** -0.5).softmax(-1) @ v
        d("attn o", o.view(8, 5, 192), ro.transpose(1, 2).reshape(8, 5, 192))
        feat = Fn.EncoderHeadFn.apply(tok, dt, vit.fc_norm.weight, vit.fc_norm.bias, None, None)
        d("feat", feat, rvit.pool(rtok))
        ie = prod.image_projection(feat); rie = ref.image_projection(rvit.pool(rtok))
        d("img emb", ie, rie)
        te = prod.text_projection(tp); rte = ref.text_projection(tr)
        d("txt emb", te, rte)
