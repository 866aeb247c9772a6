"""Pin the CPU oracle (oracle/ref_model.py) against golden vectors produced by the
reference itself (tools/gen_golden.py: the reference's CLIP.py/modules.py with a
timm stub + HF ViTMAE / DistilBERT). CPU only, float64."""
import os

import numpy as np
import pytest
import torch

from oracle import maskrng
from oracle import ref_model as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name))


def t(a):
    return torch.from_numpy(np.asarray(a)).double() if np.asarray(a).dtype.kind == "f" else torch.from_numpy(np.asarray(a))


def close(a, b, rtol=2e-5, atol=1e-9):
    a = a.detach().double()
    b = torch.as_tensor(b).double()
    scale = b.abs().max().item() + atol
    err = (a - b).abs().max().item()
    assert err <= rtol * scale + atol, (err, scale)


# ---------------------------------------------------------------- CLIP loss
@pytest.mark.parametrize("N", [8, 64, 256])
def test_clip_loss_vs_reference(N):
    z = load("clip_loss.npz")
    if N < 256:
        I, T = t(z[f"I_{N}"]), t(z[f"T_{N}"])
    else:
        g = torch.Generator().manual_seed(100 + N)
        I = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g, dtype=torch.float64), (256,)).float().double()
        T = torch.nn.functional.layer_norm(torch.randn(N, 256, generator=g, dtype=torch.float64), (256,)).float().double()
    I.requires_grad_(True)
    T.requires_grad_(True)
    loss = R.clip_loss(I, T, 1.0)
    loss.backward()
    assert abs(loss.item() - float(z[f"loss_{N}"])) < 1e-5
    close(I.grad, t(z[f"dI_{N}"]))
    close(T.grad, t(z[f"dT_{N}"]))


def test_clip_loss_temperature():
    z = load("clip_loss.npz")
    I, T = t(z["I_8"]).requires_grad_(True), t(z["T_8"]).requires_grad_(True)
    loss = R.clip_loss(I, T, 0.5)
    loss.backward()
    assert abs(loss.item() - float(z["loss_8_t05"])) < 1e-5
    close(I.grad, t(z["dI_8_t05"]))


def test_clip_loss_closed_form_backward():
    """SURVEY.md Appendix B closed form == autograd (what the HIP kernel implements)."""
    z = load("clip_loss.npz")
    I, T = t(z["I_64"]), t(z["T_64"])
    N = I.shape[0]
    tau = 0.7
    L = T @ I.T / tau
    S = (I @ I.T + T @ T.T) / 2 * tau
    Y = S.softmax(-1)
    Pr, Pc = L.softmax(-1), L.softmax(0)
    G = -(L.log_softmax(-1) + L.log_softmax(0)) / (2 * N)
    dS = Y * (G - (G * Y).sum(1, keepdim=True))
    D = (dS + dS.T) * tau / 2
    dL = (Pr - 2 * Y + Pc * Y.sum(0, keepdim=True)) / (2 * N)
    dI = D @ I + dL.T @ T / tau
    dT = D @ T + dL @ I / tau
    I2, T2 = I.clone().requires_grad_(True), T.clone().requires_grad_(True)
    R.clip_loss(I2, T2, tau).backward()
    close(dI, I2.grad, rtol=1e-10)
    close(dT, T2.grad, rtol=1e-10)
    assert abs((Y * G).sum().item() - R.clip_loss(I, T, tau).item()) < 1e-12


# ---------------------------------------------------------- ProjectionHead
def test_projection_head_vs_reference():
    z = load("projection_head.npz")
    head = R.ProjectionHead(64, 32).double()
    head.load_state_dict({k[3:]: t(z[k]) for k in z.files if k.startswith("sd.")})
    head.eval()
    x = t(z["x"]).requires_grad_(True)
    y = head(x)
    close(y, t(z["y"]), rtol=1e-6)
    (y * t(z["w"])).sum().backward()
    close(x.grad, t(z["dx"]), rtol=1e-5)
    for n, p in head.named_parameters():
        close(p.grad, t(z["g." + n]), rtol=1e-5)


# ----------------------------------------------------------------- masking
def test_mask_noise_and_ids_vs_hf_random_masking():
    z = load("masking.npz")
    B, L = z["noise"].shape
    assert np.array_equal(maskrng.keys24(2, 3, 0, B, L), z["keys24"])
    noise = maskrng.noise(2, 3, 0, B, L)
    assert np.array_equal(noise, z["noise"])
    keep = int(L * (1 - 0.75))
    ids_s, ids_r, mask = R.random_masking_ids(torch.from_numpy(noise), keep)
    assert torch.equal(ids_s[:, :keep], torch.from_numpy(z["ids_keep"]))
    assert torch.equal(ids_r, torch.from_numpy(z["ids_restore"]))
    assert torch.equal(mask.double(), t(z["mask"]))


def test_masking_tie_break_is_stable():
    # equal keys -> lower patch index first
    noise = torch.tensor([[0.5, 0.25, 0.5, 0.25, 0.0, 0.5]])
    ids_s, ids_r, mask = R.random_masking_ids(noise, 3)
    assert ids_s.tolist() == [[4, 1, 3, 0, 2, 5]]
    assert torch.equal(torch.argsort(ids_s, 1), ids_r)


# ----------------------------------------------------------------- patchify
@pytest.mark.parametrize("S,p", [(32, 16), (28, 14), (16, 8)])
def test_patchify_vs_hf(S, p):
    z = load("patchify.npz")
    img = t(z[f"img_{S}"])
    pt = R.patchify(img, p)
    assert torch.equal(pt.float(), t(z[f"patches_{S}"]).float())
    back = R.unpatchify(pt, p, 3, S // p, S // p)
    assert torch.equal(back, img)


# --------------------------------------------------------------------- MAE
def _hf_layer_map(src, dst):
    """HF ViTMAE (transformers 5.x) layer names -> timm-style names."""
    return {
        f"{src}.layernorm_before.weight": f"{dst}.norm1.weight", f"{src}.layernorm_before.bias": f"{dst}.norm1.bias",
        f"{src}.layernorm_after.weight": f"{dst}.norm2.weight", f"{src}.layernorm_after.bias": f"{dst}.norm2.bias",
        f"{src}.attention.o_proj.weight": f"{dst}.attn.proj.weight",
        f"{src}.attention.o_proj.bias": f"{dst}.attn.proj.bias",
        f"{src}.mlp.fc1.weight": f"{dst}.mlp.fc1.weight", f"{src}.mlp.fc1.bias": f"{dst}.mlp.fc1.bias",
        f"{src}.mlp.fc2.weight": f"{dst}.mlp.fc2.weight", f"{src}.mlp.fc2.bias": f"{dst}.mlp.fc2.bias",
    }


def map_hf(arr, hf_prefix, layers, dst_prefix, dec_layers=0, dec_hf="decoder", dec_dst="mae_decoder",
           enc_dst="image_encoder.model"):
    """Build an oracle-named dict from HF-named arrays (with q|k|v fused)."""
    out = {}
    e = f"{hf_prefix}vit." if hf_prefix is not None else ""
    simple = {
        f"{e}embeddings.cls_token": f"{enc_dst}.cls_token",
        f"{e}embeddings.position_embeddings": f"{enc_dst}.pos_embed",
        f"{e}embeddings.patch_embeddings.projection.weight": f"{enc_dst}.patch_embed.proj.weight",
        f"{e}embeddings.patch_embeddings.projection.bias": f"{enc_dst}.patch_embed.proj.bias",
    }
    for i in range(layers):
        simple.update(_hf_layer_map(f"{e}layers.{i}", f"{enc_dst}.blocks.{i}"))
    if dec_layers:
        d = f"{hf_prefix}{dec_hf}." if hf_prefix is not None else ""
        simple.update({
            f"{e}layernorm.weight": f"{dec_dst}.mae_norm.weight", f"{e}layernorm.bias": f"{dec_dst}.mae_norm.bias",
            f"{d}mask_token": f"{dec_dst}.mask_token", f"{d}decoder_pos_embed": f"{dec_dst}.decoder_pos_embed",
            f"{d}decoder_embed.weight": f"{dec_dst}.decoder_embed.weight",
            f"{d}decoder_embed.bias": f"{dec_dst}.decoder_embed.bias",
            f"{d}decoder_norm.weight": f"{dec_dst}.decoder_norm.weight",
            f"{d}decoder_norm.bias": f"{dec_dst}.decoder_norm.bias",
            f"{d}decoder_pred.weight": f"{dec_dst}.decoder_pred.weight",
            f"{d}decoder_pred.bias": f"{dec_dst}.decoder_pred.bias",
        })
        for i in range(dec_layers):
            simple.update(_hf_layer_map(f"{d}decoder_layers.{i}", f"{dec_dst}.decoder_layers.{i}"))
    for k, v in simple.items():
        key = dst_prefix + k
        if key in arr:
            out[v] = t(arr[key])
    # fused qkv
    groups = [(f"{e}layers.{i}", f"{enc_dst}.blocks.{i}") for i in range(layers)]
    if dec_layers:
        groups += [(f"{d}decoder_layers.{i}", f"{dec_dst}.decoder_layers.{i}") for i in range(dec_layers)]
    for src, dst in groups:
        for kind in ("weight", "bias"):
            parts = [dst_prefix + f"{src}.attention.{n}_proj.{kind}" for n in ("q", "k", "v")]
            if all(p in arr for p in parts):
                out[f"{dst}.attn.qkv.{kind}"] = torch.cat([t(arr[p]) for p in parts], 0)
    return out


@pytest.mark.parametrize("tag", ["raw", "np"])
def test_mae_pretraining_vs_hf(tag):
    z = load("mae.npz")
    cfg = R.OracleConfig(model_name="vit_pico_patch8_16", img_size=16, mask_ratio=0.75, norm_pix_loss=(tag == "np"),
                         decoder_dim=64, decoder_depth=2, decoder_heads=2)
    vit = R.VisionTransformer(cfg.model_name, 16).double()
    dec = R.MAEDecoder(64, 4, 8, 64, 2, 2).double()
    holder = torch.nn.Module()
    holder.image_encoder = torch.nn.Module()
    holder.image_encoder.model = vit
    holder.mae_decoder = dec
    sd = map_hf(z, "", 2, "sd.", dec_layers=2)
    # decoder_pos_embed is a fixed buffer: our sin-cos builder must reproduce HF's
    close(dec.decoder_pos_embed, sd["mae_decoder.decoder_pos_embed"], rtol=1e-6)
    missing = holder.load_state_dict(sd, strict=False)
    assert not [k for k in missing.missing_keys if "fc_norm" not in k], missing
    img = t(z["img"])
    noise = torch.from_numpy(z["noise"]).float()
    ids_s, ids_r, mask = R.random_masking_ids(noise, 1)
    assert torch.equal(ids_r, torch.from_numpy(z[f"{tag}.ids_restore"]))
    assert torch.equal(mask.double(), t(z[f"{tag}.mask"]))
    tokens = vit.forward_tokens(img, ids_s[:, :1])
    pred = dec(tokens, ids_r)
    close(pred, t(z[f"{tag}.logits"]), rtol=1e-5)
    loss = R.mae_loss(pred, img, mask.double(), 8, norm_pix_loss=(tag == "np"))
    assert abs(loss.item() - float(z[f"{tag}.loss"])) < 1e-5 * max(1, abs(float(z[f"{tag}.loss"])))
    loss.backward()
    g = map_hf(z, "", 2, f"{tag}.g.", dec_layers=2)
    named = dict(holder.named_parameters())
    checked = 0
    for k, ref in g.items():
        if k in named and named[k].grad is not None:
            close(named[k].grad, ref, rtol=1e-4)
            checked += 1
    assert checked >= 30


# ------------------------------------------------------------- CLIPModel
@pytest.mark.parametrize("tag", ["full", "pad"])
def test_clip_model_vs_reference(tag):
    z = load("clip_model.npz")
    cfg = R.OracleConfig(model_name="vit_pico_patch8_16", img_size=16, text_layers=2, text_dim=64, text_heads=2,
                         text_hidden=256, vocab_size=320, max_position=32, projection_dim=32, mask_ratio=0.0)
    m = R.CLIPModel(cfg).double()
    sd = map_hf(z, "sd.image_encoder.model.", 2, "")
    sd = {k: v for k, v in sd.items()}
    sd["image_encoder.model.fc_norm.weight"] = t(z["sd.image_encoder.model.fc_norm.weight"])
    sd["image_encoder.model.fc_norm.bias"] = t(z["sd.image_encoder.model.fc_norm.bias"])
    for k in z.files:
        if k.startswith("sd.") and not k.startswith("sd.image_encoder"):
            sd[k[3:]] = t(z[k])
    res = m.load_state_dict(sd, strict=False)
    assert not res.missing_keys, res.missing_keys
    m.eval()
    batch = {"image": t(z[f"{tag}.img"]), "input_ids": torch.from_numpy(z[f"{tag}.ids"]),
             "attention_mask": torch.from_numpy(z[f"{tag}.am"])}
    with torch.no_grad():
        cls = m.text_encoder(batch["input_ids"], batch["attention_mask"])
    close(cls, t(z[f"{tag}.text_cls"]), rtol=1e-5)
    loss = m(batch)
    assert abs(loss.item() - float(z[f"{tag}.loss"])) < 1e-6 * max(1, abs(float(z[f"{tag}.loss"])))
    loss.backward()
    g = map_hf(z, f"{tag}.g.image_encoder.model.", 2, "")
    g.update({k[len(tag) + 3:]: t(z[k]) for k in z.files
              if k.startswith(f"{tag}.g.") and not k.startswith(f"{tag}.g.image_encoder.model.vit")})
    named = dict(m.named_parameters())
    checked = 0
    for k, ref in g.items():
        if k in named and named[k].grad is not None:
            close(named[k].grad, ref, rtol=1e-4)
            checked += 1
    assert checked >= 25, checked


def test_resize_oracle_properties():
    """The OpenCV INTER_LINEAR restatement (oracle/input_ref.py; opencv is
    absent: parity unpinned) on cases with a known answer: constant images stay
    constant at any scale, equal size copies, exact 2x downscale is the rounded
    2x2 mean, and a 2x upscale of a horizontal ramp is monotone."""
    import numpy as np
    from oracle.input_ref import resize_u8_linear_ref
    c = np.full((37, 53, 3), 201, np.uint8)
    for s in (7, 32, 224):
        assert np.all(resize_u8_linear_ref(c, s) == 201)
    im = np.random.default_rng(0).integers(0, 256, (16, 16, 3), dtype=np.uint8)
    assert np.array_equal(resize_u8_linear_ref(im, 16), im)
    d = resize_u8_linear_ref(im, 8).astype(int)
    i = im.astype(int)
    assert np.array_equal(d, (i[0::2, 0::2] + i[0::2, 1::2] + i[1::2, 0::2] + i[1::2, 1::2] + 2) >> 2)
    ramp = np.tile(np.arange(0, 256, 16, dtype=np.uint8)[None, :, None], (16, 1, 3))
    up = resize_u8_linear_ref(ramp, 32).astype(int)
    assert np.all(np.diff(up[0, :, 0]) >= 0) and up[0, 0, 0] == 0 and up[0, -1, 0] == 240
