"""Generate the golden vectors that pin the oracle (tests/golden/*.npz).

Run in the build container (the only place /root/reference exists):
    python tools/gen_golden.py

Sources of truth, all executed here, in float64 on the CPU:
  * the reference's own CLIP.py / modules.py (/root/reference), imported with
    a `timm` stub (timm 0.9.12 is not installed; SURVEY.md §8c recipe) whose
    create_model() returns an avg-pool ViT built from HF ViTMAE layers
    (mask_ratio 0, identity noise, no final norm, fc_norm) -- the timm
    VisionTransformer(num_classes=0, global_pool="avg") arithmetic;
  * HF transformers ViTMAE (random_masking, patchify, decoder, loss) and
    DistilBERT -- the reference's own dependencies (transformers 5.15 here,
    4.36.2 pinned by requirements.txt:207; the arithmetic used is unchanged).
Only inputs/outputs/weights are written; no reference source is copied.
Weights are small test-size models (ViT 64-d x 2 layers, 16x16 images, 8x8
patches; DistilBERT 64-d x 2 layers, vocab 320; projection_dim 32).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
from torch import nn

import transformers  # noqa: F401  (must precede the timm stub)
from transformers import DistilBertConfig, ViTMAEConfig, ViTMAEForPreTraining, ViTMAEModel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import maskrng  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")
torch.set_default_dtype(torch.float64)

VIT = dict(image_size=16, patch_size=8, num_channels=3, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
           intermediate_size=256, hidden_act="gelu", layer_norm_eps=1e-6, qkv_bias=True,
           hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
TEXT = dict(vocab_size=320, dim=64, n_layers=2, n_heads=2, hidden_dim=256, max_position_embeddings=32)
PROJ_DIM = 32


class HFAvgViT(nn.Module):
    """timm.create_model(name, pretrained, num_classes=0, global_pool="avg") stand-in."""

    def __init__(self, vit_cfg=None):
        super().__init__()
        vit_cfg = vit_cfg or VIT
        self.vit = ViTMAEModel(ViTMAEConfig(mask_ratio=0.0, **vit_cfg))
        with torch.no_grad():
            self.vit.embeddings.initialize_weights()
        self.fc_norm = nn.LayerNorm(vit_cfg["hidden_size"], eps=1e-6)

    def forward(self, x):
        B = x.shape[0]
        L = self.vit.embeddings.patch_embeddings.num_patches
        noise = torch.arange(L, dtype=x.dtype).expand(B, L)  # identity order
        h, _, _ = self.vit.embeddings(x, noise=noise)
        for layer in self.vit.layers:
            h = layer(h)
        return self.fc_norm(h[:, 1:].mean(dim=1))


# what the stub builds next (gen_train_curve switches these to the C0 sizes)
STUB = {"vit": None, "text": TEXT}


def import_reference():
    stub = types.ModuleType("timm")
    stub.create_model = lambda name, pretrained=False, num_classes=0, global_pool="avg": HFAvgViT(STUB["vit"])
    sys.modules["timm"] = stub
    sys.path.insert(0, REF)
    import config as RCFG  # the reference's config.py
    RCFG.projection_dim = PROJ_DIM       # bound at def time by modules.py:59-60
    import modules as RM
    import CLIP as RC
    RM.DistilBertConfig = lambda: DistilBertConfig(**STUB["text"])
    RM.TextEncoder.__init__.__defaults__ = ("distilbert-base-uncased", False, False)
    RM.ImageEncoder.__init__.__defaults__ = ("vit_pico", False, True)
    return RCFG, RM, RC


def round32(module):
    """Make every weight exactly fp32-representable so the fixtures can store fp32."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            if t.is_floating_point():
                t.copy_(t.float().double())
    return module


def _arr(v):
    a = v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
    return a.astype(np.float32) if a.dtype == np.float64 else a


def npz(name, keep64=(), **arrs):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: (np.asarray(v, dtype=np.float64) if k in keep64 else _arr(v))
                                 for k, v in arrs.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


def sd_arrays(prefix, module):
    return {f"{prefix}{k}": v for k, v in module.state_dict().items()}


def grad_arrays(prefix, module):
    return {f"{prefix}{k}": p.grad for k, p in module.named_parameters() if p.grad is not None}


def make_batch(B, S, T=25, seed=0, pad=False):
    g = torch.Generator().manual_seed(seed)
    px = torch.randint(0, 256, (B, 3, S, S), generator=g).double() / 255.0
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    img = (px - mean) / std
    g1 = torch.Generator().manual_seed(seed + 1)
    ids = torch.randint(5, 300, (B, T), generator=g1)
    am = torch.ones(B, T, dtype=torch.int64)
    if pad:
        lens = torch.randint(5, T + 1, (B,), generator=g1)
        for b in range(B):
            am[b, lens[b]:] = 0
            ids[b, lens[b]:] = 0
    return img, ids, am


class _Ident(nn.Module):
    def forward(self, x=None, input_ids=None, attention_mask=None):
        return x if x is not None else input_ids


def gen_clip_loss(RC):
    """CLIP.py:34-43 on given embeddings (encoders/projections replaced by identity)."""
    m = RC.CLIPModel(temperature=1.0, image_embedding=64, text_embedding=64)
    m.image_encoder = _Ident()
    m.text_encoder = _Ident()
    m.image_projection = nn.Identity()
    m.text_projection = nn.Identity()
    out = {}
    for N in (8, 64, 256):
        g = torch.Generator().manual_seed(100 + N)
        I = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g), (256,)).float().double()
        T = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g), (256,)).float().double()
        I.requires_grad_(True)
        T.requires_grad_(True)
        loss = m({"image": I, "input_ids": T, "attention_mask": None})
        loss.backward()
        out.update({f"loss_{N}": loss, f"dI_{N}": I.grad, f"dT_{N}": T.grad})
        if N < 256:  # N=256 inputs are regenerated from the seed by the test
            out.update({f"I_{N}": I, f"T_{N}": T})
    # temperature != 1 (multiplies inside the target softmax, CLIP.py:37-39)
    m.temperature = 0.5
    I = torch.from_numpy(_arr(out["I_8"])).double().requires_grad_(True)
    T = torch.from_numpy(_arr(out["T_8"])).double().requires_grad_(True)
    loss = m({"image": I, "input_ids": T, "attention_mask": None})
    loss.backward()
    out.update({"loss_8_t05": loss, "dI_8_t05": I.grad, "dT_8_t05": T.grad})
    npz("clip_loss.npz", **out)


def gen_projection_head(RM):
    torch.manual_seed(1)
    head = round32(RM.ProjectionHead(embedding_dim=64))
    head.eval()
    x = torch.randn(8, 64).float().double().requires_grad_(True)
    y = head(x)
    w = torch.randn_like(y).float().double()
    (y * w).sum().backward()
    npz("projection_head.npz", x=x, y=y, w=w, dx=x.grad, **sd_arrays("sd.", head), **grad_arrays("g.", head))


def gen_masking():
    model = ViTMAEModel(ViTMAEConfig(image_size=224, patch_size=16, hidden_size=64, num_hidden_layers=1,
                                     num_attention_heads=2, intermediate_size=64, mask_ratio=0.75))
    B, L = 32, 196
    noise = torch.from_numpy(maskrng.noise(2, 3, 0, B, L)).double()
    seq = torch.arange(L, dtype=torch.float64).view(1, L, 1).expand(B, L, 1).contiguous()
    unmasked, mask, ids_restore = model.embeddings.random_masking(seq, noise=noise)
    npz("masking.npz", noise=noise.float(), keys24=maskrng.keys24(2, 3, 0, B, L), ids_keep=unmasked[..., 0].long(),
        mask=mask, ids_restore=ids_restore)


def gen_patchify():
    out = {}
    for S, p in ((32, 16), (28, 14), (16, 8)):
        cfg = ViTMAEConfig(image_size=S, patch_size=p, hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                           intermediate_size=32, decoder_hidden_size=32, decoder_num_hidden_layers=1,
                           decoder_num_attention_heads=2, decoder_intermediate_size=32)
        m = ViTMAEForPreTraining(cfg)
        g = torch.Generator().manual_seed(S)
        img = torch.randn(2, 3, S, S, generator=g)
        pt = m.patchify(img)
        out[f"img_{S}"] = img
        out[f"patches_{S}"] = pt
        out[f"unpatch_{S}"] = m.unpatchify(pt)
    npz("patchify.npz", **out)


def gen_mae():
    out = {}
    for norm_pix in (False, True):
        torch.manual_seed(3)
        cfg = ViTMAEConfig(mask_ratio=0.75, norm_pix_loss=norm_pix, decoder_hidden_size=64,
                           decoder_num_hidden_layers=2, decoder_num_attention_heads=2, decoder_intermediate_size=256,
                           **VIT)
        m = ViTMAEForPreTraining(cfg)
        with torch.no_grad():  # HF 5.x leaves the fixed sin-cos tables zero on direct construction
            m.vit.embeddings.initialize_weights()
            m.decoder.initialize_weights(m.vit.embeddings.patch_embeddings.num_patches)
        m = round32(m)
        img, _, _ = make_batch(8, 16, seed=5)
        img = img.float().double()
        L = m.vit.embeddings.patch_embeddings.num_patches
        noise = torch.from_numpy(maskrng.noise(2, 0, 0, 8, L)).double()
        o = m(pixel_values=img, noise=noise)
        o.loss.backward()
        tag = "np" if norm_pix else "raw"
        out.update({f"{tag}.loss": o.loss, f"{tag}.logits": o.logits, f"{tag}.mask": o.mask,
                    f"{tag}.ids_restore": o.ids_restore})
        if not norm_pix:  # same seed -> same weights for both variants
            out.update(sd_arrays("sd.", m))
        out.update(grad_arrays(f"{tag}.g.", m))
        out["img"] = img
        out["noise"] = noise
    npz("mae.npz", **out)


def gen_clip_model(RM, RC):
    out = {}
    for pad in (False, True):
        torch.manual_seed(4)
        m = round32(RC.CLIPModel(temperature=1.0, image_embedding=64, text_embedding=64))
        m.eval()  # dropout off (ProjectionHead p=0.1, DistilBERT p=0.1)
        img, ids, am = make_batch(8, 16, seed=7, pad=pad)
        img = img.float().double()
        loss = m({"image": img, "input_ids": ids, "attention_mask": am})
        loss.backward()
        tag = "pad" if pad else "full"
        out.update({f"{tag}.loss": loss, f"{tag}.img": img, f"{tag}.ids": ids, f"{tag}.am": am})
        if not pad:
            out.update(sd_arrays("sd.", m))
        out.update(grad_arrays(f"{tag}.g.", m))
        # the text tower alone (frozen; forward only)
        with torch.no_grad():
            out[f"{tag}.text_cls"] = m.text_encoder(input_ids=ids, attention_mask=am)
    npz("clip_model.npz", **out)


C0_VIT = dict(image_size=32, patch_size=16, num_channels=3, hidden_size=192, num_hidden_layers=12,
              num_attention_heads=3, intermediate_size=768, hidden_act="gelu", layer_norm_eps=1e-6, qkv_bias=True,
              hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
C0_TEXT = dict(n_layers=2)   # DistilBertConfig defaults otherwise: 768-d, 12 heads, vocab 30522
CURVE_STEPS = 20


def product_c0_state(seed=0):
    """The product's own C0 initial weights (mask 0: the reference's CLIP path),
    built on the CPU in fp32 exactly as tests/helpers.build_pair does, so the
    GPU test can rebuild them from the seed instead of shipping 30 MB."""
    from tests.helpers import C0, product_config
    from mae_clip_amd.CLIP import CLIPModel
    kw = dict(C0, mask_ratio=0.0)
    kw.pop("batch_size")
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float32)
    try:
        torch.manual_seed(seed)
        with product_config(precision="fp32", **kw):
            prod = CLIPModel()
    finally:
        torch.set_default_dtype(old)
    return {k: v.detach().clone() for k, v in prod.state_dict().items()}


def timm_to_hf(sd, layers):
    """product (timm names, fused qkv) -> the stub's HF ViTMAE names."""
    out = {}
    src, dst = "image_encoder.model.", "image_encoder.model.vit."
    for k, v in sd.items():
        if not k.startswith(src):
            out[k] = v
    out[dst + "embeddings.cls_token"] = sd[src + "cls_token"]
    out[dst + "embeddings.position_embeddings"] = sd[src + "pos_embed"]
    out[dst + "embeddings.patch_embeddings.projection.weight"] = sd[src + "patch_embed.proj.weight"]
    out[dst + "embeddings.patch_embeddings.projection.bias"] = sd[src + "patch_embed.proj.bias"]
    out[src + "fc_norm.weight"] = sd[src + "fc_norm.weight"]
    out[src + "fc_norm.bias"] = sd[src + "fc_norm.bias"]
    names = {"norm1": "layernorm_before", "norm2": "layernorm_after", "attn.proj": "attention.o_proj",
             "mlp.fc1": "mlp.fc1", "mlp.fc2": "mlp.fc2"}
    for i in range(layers):
        b, h = f"{src}blocks.{i}.", f"{dst}layers.{i}."
        for a, c in names.items():
            for kind in ("weight", "bias"):
                out[f"{h}{c}.{kind}"] = sd[f"{b}{a}.{kind}"]
        for kind in ("weight", "bias"):
            q, k_, v_ = sd[f"{b}attn.qkv.{kind}"].chunk(3, 0)
            out[f"{h}attention.q_proj.{kind}"] = q
            out[f"{h}attention.k_proj.{kind}"] = k_
            out[f"{h}attention.v_proj.{kind}"] = v_
    return out


def gen_train_curve(RC):
    """the reference's own training loop semantics
    (main.py:54-66: model(batch), zero_grad, backward, AdamW step; AdamW(lr 1e-3,
    wd 1e-3) over model.parameters() as main.py:101-103, constant LR because the
    scheduler is never stepped, main.py:60-61,107) run for 20 steps on the
    reference CLIPModel (CLIP.py / modules.py, ViT-Tiny/16 @32 stub + 2-layer
    DistilBERT = C0, mask 0) from the product's C0 initial weights, eval mode
    (dropout off: the product draws its own dropout masks), batch k =
    tests.helpers.make_batch(8, 32, seed=300 + k). Stores the 20 losses and
    per-tensor sums of the initial weights (the test's seed check)."""
    from tests.helpers import make_batch as h_make_batch
    STUB["vit"], STUB["text"] = C0_VIT, C0_TEXT
    sd0 = product_c0_state(0)
    ref = RC.CLIPModel(temperature=1.0, image_embedding=192, text_embedding=768)
    STUB["vit"], STUB["text"] = None, TEXT
    ref.image_projection = type(ref.image_projection)(embedding_dim=192, projection_dim=256, dropout=0.1)
    ref.text_projection = type(ref.text_projection)(embedding_dim=768, projection_dim=256, dropout=0.1)
    hf = {k: v.double() for k, v in timm_to_hf(sd0, 12).items()}
    missing, unexpected = ref.load_state_dict(hf, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith("image_encoder.model.vit.layernorm.") for k in missing), missing
    ref.double().eval()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-3)
    losses = []
    for k in range(CURVE_STEPS):
        b = h_make_batch(8, 32, seed=300 + k)
        batch = {"image": b["image"].double(), "input_ids": b["input_ids"], "attention_mask": b["attention_mask"]}
        loss = ref(batch)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
        print(f"step {k}: loss {loss.item():.10f}")
    sums = {f"sum.{k}": v.double().sum().item() for k, v in sd0.items() if v.is_floating_point()}
    npz("train_curve.npz", keep64=("losses",) + tuple(sums), losses=losses, **sums)


def main():
    RCFG, RM, RC = import_reference()
    if sys.argv[1:] == ["train_curve"]:
        gen_train_curve(RC)
        return
    gen_clip_loss(RC)
    gen_projection_head(RM)
    gen_masking()
    gen_patchify()
    gen_mae()
    gen_clip_model(RM, RC)
    gen_train_curve(RC)


if __name__ == "__main__":
    main()
