"""Shared test helpers: config switching and product<->oracle model pairs."""
import contextlib

import torch

C0 = dict(model_name="vit_tiny_patch16_224", size=32, image_embedding=192, text_layers=2, mask_ratio=0.75,
          decoder_embed_dim=128, decoder_depth=2, decoder_num_heads=4, batch_size=8)


@contextlib.contextmanager
def product_config(**kw):
    from mae_clip_amd import config as CFG
    old = {k: getattr(CFG, k) for k in kw}
    for k, v in kw.items():
        setattr(CFG, k, v)
    try:
        yield CFG
    finally:
        for k, v in old.items():
            setattr(CFG, k, v)


def oracle_config(**kw):
    from oracle.ref_model import OracleConfig
    return OracleConfig(model_name=kw.get("model_name", "vit_tiny_patch16_224"), img_size=kw.get("size", 32),
                        text_layers=kw.get("text_layers", 2), mask_ratio=kw.get("mask_ratio", 0.75),
                        decoder_dim=kw.get("decoder_embed_dim", 128), decoder_depth=kw.get("decoder_depth", 2),
                        decoder_heads=kw.get("decoder_num_heads", 4), norm_pix_loss=kw.get("norm_pix_loss", False),
                        vit_depth=kw.get("vit_depth"))


def make_batch(B, S, T=25, seed=0, pad=False, device="cpu"):
    """Synthetic inputs of SURVEY.md §8d: uint8 pixels ImageNet-normalised (dataset.py:49),
    input_ids randint(5,300) (CLIP.py:56-57), attention_mask ones (or ragged)."""
    g = torch.Generator().manual_seed(seed)
    px = torch.randint(0, 256, (B, 3, S, S), generator=g).float() / 255.0
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
    return {"image": img.to(device), "input_ids": ids.to(device), "attention_mask": am.to(device)}


def build_pair(precision="fp32", seed=0, **overrides):
    """(product CLIPModel on cuda, oracle CLIPModel on cpu fp64) with identical weights."""
    from mae_clip_amd.CLIP import CLIPModel
    from oracle.ref_model import CLIPModel as RefCLIP
    kw = dict(C0)
    kw.update(overrides)
    vit_depth = kw.pop("vit_depth", None)
    torch.manual_seed(seed)
    with product_config(precision=precision, **{k: v for k, v in kw.items() if k != "batch_size"}):
        prod = CLIPModel()
        if vit_depth is not None:
            prod.image_encoder.model.blocks = prod.image_encoder.model.blocks[:vit_depth]
    ref = RefCLIP(oracle_config(vit_depth=vit_depth, **kw))
    sd = {k: v.detach().clone() for k, v in prod.state_dict().items()}
    missing, unexpected = ref.load_state_dict(sd, strict=True), None
    return prod.cuda(), ref.double()


def record_parity(name, **vals):
    """Append one measured deviation record (JSON line) to $MAECLIP_PARITY_OUT
    when set (tools/gpu_r3.sh points it into gpurun_out/; the merged records
    are committed as profiles/<round>/parity.json). Always printed as well."""
    import json
    import os
    rec = dict(test=name, **{k: (float(v) if isinstance(v, (int, float)) else v) for k, v in vals.items()})
    print("PARITY", json.dumps(rec))
    path = os.environ.get("MAECLIP_PARITY_OUT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def train_curve(device, precision="bf16", B=4, steps=5):
    """The reference's train loop (main.py:54-66: forward, zero_grad, backward,
    AdamW(lr 1e-3, wd 1e-3) step, main.py:101-103) for `steps` steps at the
    metric's model shapes (ViT-B/16 @224, mask .75, 8x512 decoder, 6-layer
    text) in TRAIN mode: the product at `precision` with its fused AdamW vs the
    fp64 CPU oracle with torch.optim.AdamW, identical initial weights, batches
    and MAE masks (both advance the mask step every training forward). Dropout
    is set to 0 on both sides (the two RNG streams cannot match)."""
    from mae_clip_amd.optim import AdamW
    kw = dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, text_layers=6, mask_ratio=0.75,
              decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16, dropout=0.0, text_dropout=0.0,
              text_attention_dropout=0.0)
    prod, ref = build_pair(precision, **kw)
    for m in ref.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    prod.train()
    ref.train()
    opt_p = AdamW([p for p in prod.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    opt_r = torch.optim.AdamW([p for p in ref.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    rows = []
    for k in range(steps):
        b = make_batch(B, 224, seed=40 + k)
        lp = prod({kk: v.to(device) for kk, v in b.items()})
        opt_p.zero_grad()
        lp.backward()
        opt_p.step()
        lr = ref(dict(b, image=b["image"].double()))
        opt_r.zero_grad()
        lr.backward()
        opt_r.step()
        lpv, lrv = lp.item(), lr.item()
        rows.append({"step": k, "product": lpv, "oracle": lrv, "rel": abs(lpv - lrv) / max(1.0, abs(lrv))})
    return {"precision": precision, "steps": steps, "batch": B, "worst_rel": max(r["rel"] for r in rows),
            "last_rel": rows[-1]["rel"], "curve": rows,
            "config": "C2 model shapes, train mode (dropout 0 both sides), AdamW lr 1e-3 wd 1e-3 (main.py:54-66, "
                      ":101-103) vs the fp64 CPU oracle + torch.optim.AdamW"}
