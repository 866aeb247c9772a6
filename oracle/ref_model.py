"""CPU restatement of the reference's CLIP(+MAE) hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle. Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import it; the product package mae_clip_amd
never does (it has no CPU fallback).

Pinned against golden vectors generated from the reference itself
(tools/gen_golden.py -> tests/golden/*.npz): the reference's CLIP.py /
modules.py imported with a timm stub, plus HF transformers ViTMAE / DistilBERT
(the reference's own dependencies). See tests/test_oracle_golden.py.

Semantics restated (file:line into /root/reference unless marked HF/...):
  * CLIPModel.forward / loss            CLIP.py:23-43, cross_entropy CLIP.py:46-52
  * ProjectionHead                      modules.py:55-76
  * ImageEncoder = timm 0.9.12 VisionTransformer(num_classes=0, global_pool="avg")
                                        modules.py:17-19 (timm not vendored)
  * TextEncoder = DistilBERT, CLS row   modules.py:34-51, HF/models/distilbert
  * MAE head (absent from the reference, specified by BASELINE.json) =
    HF ViTMAE random_masking / decoder / patchify / loss
                                        HF/models/vit_mae/modeling_vit_mae.py:297-327,455-580,706-745,852-859
Plain torch ops in float64 or float32 on the CPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
from torch import nn
import torch.nn.functional as F

from . import maskrng

VIT_SPECS = {
    # name: (embed_dim, depth, heads, patch, default img)
    "vit_pico_patch8_16": (64, 2, 2, 8, 16),   # test-only size used by the golden fixtures
    "vit_tiny_patch16_224": (192, 12, 3, 16, 224),
    "vit_small_patch16_224": (384, 12, 6, 16, 224),
    "vit_base_patch16_224": (768, 12, 12, 16, 224),
    "vit_large_patch16_224": (1024, 24, 16, 16, 224),
    "vit_large_patch14_336": (1024, 24, 16, 14, 336),
}


@dataclass
class OracleConfig:
    model_name: str = "vit_tiny_patch16_224"
    img_size: int = 32
    vit_depth: int | None = None          # override (tests)
    text_layers: int = 2
    text_dim: int = 768
    text_heads: int = 12
    text_hidden: int = 3072
    vocab_size: int = 30522
    max_position: int = 512
    projection_dim: int = 256
    temperature: float = 1.0
    mask_ratio: float = 0.75
    mae_weight: float = 1.0
    norm_pix_loss: bool = False
    decoder_dim: int = 128
    decoder_depth: int = 2
    decoder_heads: int = 4
    decoder_mlp_ratio: float = 4.0
    mask_seed: int = 2
    extra: dict = field(default_factory=dict)


# ----------------------------------------------------------------- CLIP loss
def cross_entropy(preds, targets, reduction="none"):
    """CLIP.py:46-52."""
    loss = (-targets * F.log_softmax(preds, dim=-1)).sum(1)
    if reduction == "none":
        return loss
    return loss.mean()


def clip_loss(image_embeddings, text_embeddings, temperature=1.0):
    """CLIP.py:34-43 (soft targets, gradient flows through the targets)."""
    logits = (text_embeddings @ image_embeddings.T) / temperature
    images_similarity = image_embeddings @ image_embeddings.T
    texts_similarity = text_embeddings @ text_embeddings.T
    targets = F.softmax((images_similarity + texts_similarity) / 2 * temperature, dim=-1)
    texts_loss = cross_entropy(logits, targets, reduction="none")
    images_loss = cross_entropy(logits.T, targets.T, reduction="none")
    loss = (images_loss + texts_loss) / 2.0
    return loss.mean()


# ----------------------------------------------------------- ProjectionHead
class ProjectionHead(nn.Module):
    """modules.py:55-76: Linear -> GELU -> Linear -> Dropout -> +projected -> LayerNorm."""

    def __init__(self, embedding_dim, projection_dim=256, dropout=0.1):
        super().__init__()
        self.projection = nn.Linear(embedding_dim, projection_dim)
        self.gelu = nn.GELU()
        self.fc = nn.Linear(projection_dim, projection_dim)
        self.dropout = nn.Dropout(dropout)
        self.layer_norm = nn.LayerNorm(projection_dim)

    def forward(self, x):
        projected = self.projection(x)
        x = self.gelu(projected)
        x = self.fc(x)
        x = self.dropout(x)
        x = x + projected
        return self.layer_norm(x)


# ------------------------------------------------------------------- ViT
class Attention(nn.Module):
    """timm 0.9.12 Attention: fused qkv (bias), SDPA, proj."""

    def __init__(self, dim, heads):
        super().__init__()
        self.num_heads = heads
        self.head_dim = dim // heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, key_mask=None):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        attn = (q @ k.transpose(-2, -1)) * self.scale
        if key_mask is not None:
            attn = attn.masked_fill(key_mask.view(B, 1, 1, N) == 0, float("-inf"))
        attn = attn.softmax(dim=-1)
        x = (attn @ v).transpose(1, 2).reshape(B, N, C)
        return self.proj(x)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class Block(nn.Module):
    """timm Block (pre-LN, eps 1e-6, no LayerScale / drop-path by default).
    Also the HF ViTMAELayer structure (layernorm_before/after) of the decoder."""

    def __init__(self, dim, heads, mlp_ratio=4.0, eps=1e-6):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=eps)
        self.attn = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=eps)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        x = x + self.mlp(self.norm2(x))
        return x


class PatchEmbed(nn.Module):
    def __init__(self, img_size, patch, in_chans, dim):
        super().__init__()
        self.patch_size = patch
        self.grid = img_size // patch
        self.num_patches = self.grid * self.grid
        self.proj = nn.Conv2d(in_chans, dim, kernel_size=patch, stride=patch)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class VisionTransformer(nn.Module):
    """timm VisionTransformer(num_classes=0, global_pool="avg"): fc_norm after the
    mean over non-prefix tokens, final norm = Identity (use_fc_norm)."""

    def __init__(self, model_name, img_size, depth=None):
        super().__init__()
        D, dep, H, p, _ = VIT_SPECS[model_name]
        depth = dep if depth is None else depth
        self.embed_dim = D
        self.num_heads = H
        self.patch_embed = PatchEmbed(img_size, p, 3, D)
        L = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.pos_embed = nn.Parameter(torch.randn(1, L + 1, D) * 0.02)
        self.blocks = nn.ModuleList([Block(D, H) for _ in range(depth)])
        self.fc_norm = nn.LayerNorm(D, eps=1e-6)

    def tokens(self, x, ids_keep=None):
        """PatchEmbed + _pos_embed on all patches (ids_keep None) or FLIP-style on the
        visible ones."""
        t = self.patch_embed(x) + self.pos_embed[:, 1:, :]
        if ids_keep is not None:
            t = torch.gather(t, 1, ids_keep.unsqueeze(-1).expand(-1, -1, t.shape[-1]))
        cls = (self.cls_token + self.pos_embed[:, :1, :]).expand(t.shape[0], -1, -1)
        return torch.cat([cls, t], dim=1)

    def forward_tokens(self, x, ids_keep=None):
        t = self.tokens(x, ids_keep)
        for blk in self.blocks:
            t = blk(t)
        return t

    def pool(self, t):
        return self.fc_norm(t[:, 1:].mean(dim=1))

    def forward(self, x):
        return self.pool(self.forward_tokens(x))


# --------------------------------------------------------------- MAE pieces
def patchify(imgs, p):
    """HF/.../modeling_vit_mae.py:706-745: [B,C,h*p,w*p] -> [B, h*w, p*p*C] (ky,kx,c)."""
    B, C, Hh, Ww = imgs.shape
    h, w = Hh // p, Ww // p
    x = imgs.reshape(B, C, h, p, w, p).permute(0, 2, 4, 3, 5, 1)
    return x.reshape(B, h * w, p * p * C)


def unpatchify(x, p, C, h, w):
    """HF/.../modeling_vit_mae.py:747-795."""
    B = x.shape[0]
    x = x.reshape(B, h, w, p, p, C).permute(0, 5, 1, 3, 2, 4)
    return x.reshape(B, C, h * p, w * p)


def random_masking_ids(noise, len_keep):
    """HF/.../modeling_vit_mae.py:297-327 with a stable argsort."""
    ids_shuffle = torch.argsort(noise, dim=1, stable=True)
    ids_restore = torch.argsort(ids_shuffle, dim=1, stable=True)
    B, L = noise.shape
    mask = torch.ones(B, L, dtype=torch.float32)
    mask[:, :len_keep] = 0
    mask = torch.gather(mask, 1, ids_restore)
    return ids_shuffle, ids_restore, mask


def build_2d_sincos(grid, dim):
    """HF build_2d_sinusoidal_position_embedding(cls_token=True) + the h/w half
    rotation of ViTMAEDecoder.initialize_weights (HF/.../modeling_vit_mae.py:521-534)."""
    pos_dim = dim // 4
    omega = torch.arange(pos_dim, dtype=torch.float64) / pos_dim
    omega = 1.0 / 10000.0 ** omega
    gh, gw = torch.meshgrid(torch.arange(grid, dtype=torch.float64), torch.arange(grid, dtype=torch.float64),
                            indexing="ij")
    eh = gh.flatten().outer(omega)
    ew = gw.flatten().outer(omega)
    pe = torch.cat([eh.sin(), eh.cos(), ew.sin(), ew.cos()], dim=1)
    pe = torch.cat([torch.zeros(1, dim, dtype=torch.float64), pe], dim=0)
    half = dim // 2
    pe = torch.cat([pe[..., half:], pe[..., :half]], dim=-1)
    return pe.to(torch.float32)


class MAEDecoder(nn.Module):
    """mae_norm (App. A.2) + HF ViTMAEDecoder (modeling_vit_mae.py:455-580)."""

    def __init__(self, enc_dim, num_patches, patch, dim=512, depth=8, heads=16, mlp_ratio=4.0, in_chans=3):
        super().__init__()
        self.mae_norm = nn.LayerNorm(enc_dim, eps=1e-6)
        self.decoder_embed = nn.Linear(enc_dim, dim)
        self.mask_token = nn.Parameter(torch.randn(1, 1, dim) * 0.02)
        grid = int(round(num_patches ** 0.5))
        self.register_buffer("decoder_pos_embed", build_2d_sincos(grid, dim).unsqueeze(0), persistent=True)
        self.decoder_layers = nn.ModuleList([Block(dim, heads, mlp_ratio) for _ in range(depth)])
        self.decoder_norm = nn.LayerNorm(dim, eps=1e-6)
        self.decoder_pred = nn.Linear(dim, patch * patch * in_chans)

    def forward(self, latent, ids_restore):
        x = self.decoder_embed(self.mae_norm(latent))
        B, L = ids_restore.shape
        mask_tokens = self.mask_token.repeat(B, L + 1 - x.shape[1], 1)
        x_ = torch.cat([x[:, 1:, :], mask_tokens], dim=1)
        x_ = torch.gather(x_, 1, ids_restore.unsqueeze(-1).repeat(1, 1, x.shape[2]))
        x = torch.cat([x[:, :1, :], x_], dim=1)
        x = x + self.decoder_pos_embed
        for blk in self.decoder_layers:
            x = blk(x)
        x = self.decoder_norm(x)
        return self.decoder_pred(x)[:, 1:, :]


def mae_loss(pred, imgs, mask, p, norm_pix_loss=False):
    """HF/.../modeling_vit_mae.py:852-859."""
    target = patchify(imgs, p)
    if norm_pix_loss:
        mean = target.mean(dim=-1, keepdim=True)
        var = target.var(dim=-1, keepdim=True)
        target = (target - mean) / (var + 1.0e-6) ** 0.5
    loss = ((pred - target) ** 2).mean(dim=-1)
    return (loss * mask).sum() / mask.sum()


# ------------------------------------------------------------- DistilBERT
class DistilBertEmbeddings(nn.Module):
    def __init__(self, vocab, dim, max_pos):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab, dim)
        self.position_embeddings = nn.Embedding(max_pos, dim)
        self.LayerNorm = nn.LayerNorm(dim, eps=1e-12)
        self.dropout = nn.Dropout(0.1)   # HF DistilBertConfig dropout (identity in eval mode)

    def forward(self, ids):
        pos = torch.arange(ids.shape[1])
        return self.dropout(self.LayerNorm(self.word_embeddings(ids) + self.position_embeddings(pos)[None]))


class DistilBertAttention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.n_heads = heads
        self.q_lin = nn.Linear(dim, dim)
        self.k_lin = nn.Linear(dim, dim)
        self.v_lin = nn.Linear(dim, dim)
        self.out_lin = nn.Linear(dim, dim)
        self.dropout = nn.Dropout(0.1)   # attention_dropout (identity in eval mode)

    def forward(self, x, mask):
        B, T, D = x.shape
        hd = D // self.n_heads
        sh = lambda t: t.view(B, T, self.n_heads, hd).transpose(1, 2)
        q, k, v = sh(self.q_lin(x)), sh(self.k_lin(x)), sh(self.v_lin(x))
        s = (q @ k.transpose(-1, -2)) * hd ** -0.5
        s = s.masked_fill(mask.view(B, 1, 1, T) == 0, torch.finfo(s.dtype).min)
        o = (self.dropout(s.softmax(-1)) @ v).transpose(1, 2).reshape(B, T, D)
        return self.out_lin(o)


class DistilBertFFN(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.lin1 = nn.Linear(dim, hidden)
        self.lin2 = nn.Linear(hidden, dim)
        self.dropout = nn.Dropout(0.1)   # HF dropout (identity in eval mode)

    def forward(self, x):
        return self.dropout(self.lin2(F.gelu(self.lin1(x))))


class DistilBertLayer(nn.Module):
    """HF/.../modeling_distilbert.py:227-284 (post-LN, eps 1e-12)."""

    def __init__(self, dim, heads, hidden):
        super().__init__()
        self.attention = DistilBertAttention(dim, heads)
        self.sa_layer_norm = nn.LayerNorm(dim, eps=1e-12)
        self.ffn = DistilBertFFN(dim, hidden)
        self.output_layer_norm = nn.LayerNorm(dim, eps=1e-12)

    def forward(self, x, mask):
        a = self.sa_layer_norm(self.attention(x, mask) + x)
        return self.output_layer_norm(self.ffn(a) + a)


class DistilBertTransformer(nn.Module):
    def __init__(self, n_layers, dim, heads, hidden):
        super().__init__()
        self.layer = nn.ModuleList([DistilBertLayer(dim, heads, hidden) for _ in range(n_layers)])


class DistilBertModel(nn.Module):
    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.embeddings = DistilBertEmbeddings(cfg.vocab_size, cfg.text_dim, cfg.max_position)
        self.transformer = DistilBertTransformer(cfg.text_layers, cfg.text_dim, cfg.text_heads, cfg.text_hidden)

    def forward(self, input_ids, attention_mask):
        x = self.embeddings(input_ids)
        for layer in self.transformer.layer:
            x = layer(x, attention_mask)
        return x


# ------------------------------------------------------------- CLIPModel
class ImageEncoder(nn.Module):
    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.model = VisionTransformer(cfg.model_name, cfg.img_size, cfg.vit_depth)


class TextEncoder(nn.Module):
    """modules.py:34-51 (frozen; CLS row, target_token_idx = 0)."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.model = DistilBertModel(cfg)
        for p in self.model.parameters():
            p.requires_grad = False
        self.target_token_idx = 0

    def forward(self, input_ids, attention_mask):
        return self.model(input_ids, attention_mask)[:, self.target_token_idx, :]


class CLIPModel(nn.Module):
    """CLIP.py:9-43 plus the MAE head of BASELINE.json."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.cfg = cfg
        self.image_encoder = ImageEncoder(cfg)
        self.text_encoder = TextEncoder(cfg)
        D = self.image_encoder.model.embed_dim
        self.image_projection = ProjectionHead(D, cfg.projection_dim)
        self.text_projection = ProjectionHead(cfg.text_dim, cfg.projection_dim)
        self.temperature = cfg.temperature
        pe = self.image_encoder.model.patch_embed
        if cfg.mask_ratio > 0:
            self.mae_decoder = MAEDecoder(D, pe.num_patches, pe.patch_size, cfg.decoder_dim, cfg.decoder_depth,
                                          cfg.decoder_heads, cfg.decoder_mlp_ratio)
        else:
            self.mae_decoder = None
        self.step = 0
        self.last_losses = {}

    def mask_for_batch(self, B, step, sample_offset=0):
        L = self.image_encoder.model.patch_embed.num_patches
        keep = int(L * (1 - self.cfg.mask_ratio))
        noise = maskrng.noise(self.cfg.mask_seed, step, sample_offset, B, L)
        ids_shuffle, ids_restore, mask = random_masking_ids(torch.from_numpy(noise), keep)
        return ids_shuffle, ids_restore, mask, keep

    def forward(self, batch, step=None, sample_offset=0):
        vit = self.image_encoder.model
        img = batch["image"]
        B = img.shape[0]
        if self.mae_decoder is not None:
            step = self.step if step is None else step
            ids_shuffle, ids_restore, mask, keep = self.mask_for_batch(B, step, sample_offset)
            tokens = vit.forward_tokens(img, ids_shuffle[:, :keep])
        else:
            tokens = vit.forward_tokens(img)
        image_features = vit.pool(tokens)
        text_features = self.text_encoder(batch["input_ids"], batch["attention_mask"])
        image_embeddings = self.image_projection(image_features)
        text_embeddings = self.text_projection(text_features)
        loss = clip_loss(image_embeddings, text_embeddings, self.temperature)
        self.last_losses = {"clip": loss.detach()}
        if self.mae_decoder is not None:
            pred = self.mae_decoder(tokens, ids_restore)
            ml = mae_loss(pred, img, mask, vit.patch_embed.patch_size, self.cfg.norm_pix_loss)
            self.last_losses["mae"] = ml.detach()
            loss = loss + self.cfg.mae_weight * ml
        if self.training:
            self.step += 1
        return loss
