"""Drop-in nn.Modules for the reference's modules.py (modules.py:8-76), backed by
libmaeclip kernels through mae_clip_amd.functions.

Same class names, constructor argument order, submodule/attribute names and
state_dict keys as the reference + timm 0.9.12 / HF DistilBERT:
  ImageEncoder.model  : VisionTransformer (timm names: patch_embed.proj,
                        cls_token, pos_embed, blocks.i.{norm1,attn.qkv,attn.proj,
                        norm2,mlp.fc1,mlp.fc2}, fc_norm)
  TextEncoder.model   : DistilBertModel (HF names: embeddings.*,
                        transformer.layer.i.{attention.{q,k,v,out}_lin,
                        sa_layer_norm, ffn.lin1, ffn.lin2, output_layer_norm})
  ProjectionHead      : projection, gelu, fc, dropout, layer_norm
Defaults are read from config at construction time (the reference binds them at
def time, modules.py:14,59-60) so tests can switch configs.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import config as CFG
from . import functions as Fn
from . import kernels as K

VIT_SPECS = {
    # name: (embed_dim, depth, heads, patch, default img)
    "vit_pico_patch8_16": (64, 2, 2, 8, 16),   # test-only size used by the golden fixtures
    "vit_tiny_patch16_224": (192, 12, 3, 16, 224),
    "vit_small_patch16_224": (384, 12, 6, 16, 224),
    "vit_base_patch16_224": (768, 12, 12, 16, 224),
    "vit_large_patch16_224": (1024, 24, 16, 16, 224),
    "vit_large_patch14_336": (1024, 24, 16, 14, 336),
}


def compute_dtype(precision=None) -> torch.dtype:
    precision = precision or CFG.precision
    if precision in ("bf16", "fp8"):     # fp8: bf16 activations, fp8 transformer-stack GEMM operands
        return torch.bfloat16
    if precision == "fp32":
        return torch.float32
    raise ValueError(f"precision must be 'bf16', 'fp8' or 'fp32', got {precision!r}")


def _require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"mae_clip_amd: {what} must be on a ROCm device (no CPU fallback); "
                           "move the model and batch to 'cuda'")


def as_model_image(img, size):
    """Validate an image batch: fp32 NCHW [B,3,S,S] (other float dtypes are
    cast) or uint8 HWC pixels [B,S,S,3] (kept as they are: the kernels read
    the pixels and apply A.Normalize themselves). Returns a contiguous tensor."""
    if K.is_u8_image(img):
        if img.shape[1] != size or img.shape[2] != size:
            raise ValueError(f"uint8 pixel batch must be [B,{size},{size},3], got {tuple(img.shape)}")
        return img.contiguous()
    if img.dim() != 4 or img.shape[1] != 3 or img.shape[2] != size or img.shape[3] != size:
        raise ValueError(f"image batch must be [B,3,{size},{size}] (fp32) or [B,{size},{size},3] (uint8), "
                         f"got {tuple(img.shape)}")
    img = img if img.dtype == torch.float32 else img.float()
    return img.contiguous()


def _trunc_normal_(t, std=0.02):
    nn.init.trunc_normal_(t, std=std, a=-2 * std, b=2 * std)


# parameter -> its bf16 shadow (a view into a WeightCache buffer), kept as an
# attribute of the parameter. The fused AdamW (optim.py) writes the shadow in
# the same pass as the update, so a shadow stays equal to bf16(p) without a
# cast launch; any other in-place change of p (load_state_dict, torch ops,
# another optimizer) bumps p._version and the next refresh() casts again.
def shadow_of(p):
    return getattr(p, "_mc_bf16_shadow", None)


def _set_shadow(p, view):
    p._mc_bf16_shadow = view


class WeightCache:
    """bf16 shadows of the GEMM weights: one multi-tensor cast launch when a
    master weight changed outside the fused AdamW (which keeps the shadows
    current itself, shadow_of); fp32 master weights stay the nn.Parameters.

    fp8=True (precision "fp8", C4): the transformer stacks' GEMM weights are
    also quantised once per forward from their fp32 masters (get_fp8): W with
    one e4m3 scale per output channel (forward GEMM B operand) and W^T with one
    per input channel (dgrad GEMM B operand)."""

    def __init__(self, fp8=False):
        self.entries = []    # (param, shape2d)
        self.views = {}
        self.key = None
        self.vers = None
        self.plan = None
        self.buf = None
        self.fp8 = fp8
        self.f8 = {}
        self.f8_params = []   # fp32 masters quantised by refresh() in fp8 mode
        self.f8_plan = None
        self.f8_key = None

    def register(self, p: torch.Tensor, shape2d):
        self.entries.append((p, tuple(shape2d)))

    def register_fp8(self, p: torch.Tensor):
        """p [N, K]: an fp8 stack GEMM weight (used in fp8 mode only)."""
        self.f8_params.append(p)

    def refresh(self, dtype):
        if self.fp8 and dtype == torch.bfloat16 and self.f8_params:
            # all fp8 weight operands of the step: one batched quantisation
            key = tuple(p.data_ptr() for p in self.f8_params)
            if key != self.f8_key:
                self.f8_plan = K.Fp8WeightPlan([p.detach() for p in self.f8_params], self.f8_params[0].device)
                self.f8 = {id(p): ops for p, ops in zip(self.f8_params, self.f8_plan.ops)}
                self.f8_key = key
            self.f8_plan.run()
        if dtype == torch.float32 or not self.entries:
            return
        key = tuple(p.data_ptr() for p, _ in self.entries)
        vers = tuple(p._version for p, _ in self.entries)
        if key == self.key and vers == self.vers and all(shadow_of(p) is self.views[id(p)] for p, _ in self.entries):
            return   # every shadow is bf16(p): cast at the last refresh or written by the fused AdamW
        for p, _ in self.entries:   # (another cache's shadows may have been the ones AdamW kept current)
            if id(p) in self.views:
                _set_shadow(p, self.views[id(p)])
        if key != self.key:
            dev = self.entries[0][0].device
            total = sum(p.numel() for p, _ in self.entries)
            self.buf = torch.empty(total, device=dev, dtype=torch.bfloat16)
            ents, off = [], 0
            self.views = {}
            for p, shp in self.entries:
                v = self.buf[off:off + p.numel()].view(shp)
                self.views[id(p)] = v
                ents.append((p.data_ptr(), None, None, None, v.data_ptr(), p.numel()))
                off += p.numel()
            self.plan = K.MultiTensorPlan(ents, dev)
            self.key = key
            for p, _ in self.entries:
                _set_shadow(p, self.views[id(p)])
        K.cast_multi(self.plan)
        self.vers = vers

    def get(self, p: torch.Tensor, dtype, shape2d=None):
        if dtype == torch.float32:
            return p if shape2d is None else p.view(shape2d)
        return self.views[id(p)]

    def get_fp8(self, p: torch.Tensor):
        """(W, W^T) fp8 operands of GEMM weight p [N, K] for this step: the
        ones refresh() quantised (registered weights), else quantised now."""
        if self.f8_plan is not None and id(p) in self.f8:
            return self.f8[id(p)]
        w = p.detach()
        wq = K.quant_rows_fp8(w, K.FP8_E4M3)
        wt = K.quant_cols_fp8(w)
        return wq, wt


# ------------------------------------------------------------------ ViT
class Attention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.num_heads = heads
        self.head_dim = dim // heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    """timm Block / HF ViTMAELayer: pre-LN (eps 1e-6) attention + MLP. Its compute
    lives in functions.TransformerStackFn (one launch sequence per stack)."""

    def __init__(self, dim, heads, mlp_ratio=4.0, eps=1e-6):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=eps)
        self.attn = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=eps)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def stack_params(self):
        return [self.norm1.weight, self.norm1.bias, self.attn.qkv.weight, self.attn.qkv.bias,
                self.attn.proj.weight, self.attn.proj.bias, self.norm2.weight, self.norm2.bias,
                self.mlp.fc1.weight, self.mlp.fc1.bias, self.mlp.fc2.weight, self.mlp.fc2.bias]

    def gemm_weights(self):
        return [self.attn.qkv.weight, self.attn.proj.weight, self.mlp.fc1.weight, self.mlp.fc2.weight]

    def init_weights(self):
        for lin in (self.attn.qkv, self.attn.proj, self.mlp.fc1, self.mlp.fc2):
            _trunc_normal_(lin.weight)
            nn.init.zeros_(lin.bias)


def chunk_bounds(n, chunk):
    """[c0, c1) block ranges of a stack in forward order. chunk: None (one
    Function), an int (equal chunks), or a tuple of chunk sizes in forward
    order whose last entry repeats (e.g. (2, 4, 6): blocks 0-1, 2-5, 6-11 --
    the backward runs the top chunk first, so the bottom chunk, whose
    all-reduce cannot overlap any later backward work, is the small one)."""
    if not chunk:
        return [(0, n)]
    sizes = [chunk] if isinstance(chunk, int) else [int(c) for c in chunk]
    if any(c <= 0 for c in sizes):
        raise ValueError(f"chunk sizes must be positive: {chunk}")
    out, c0, i = [], 0, 0
    while c0 < n:
        c1 = min(n, c0 + sizes[min(i, len(sizes) - 1)])
        out.append((c0, c1))
        c0, i = c1, i + 1
    return out


def run_stack(blocks, x, heads, dtype, cache: WeightCache, chunk=None, fp8=True):
    """The blocks as one TransformerStackFn, or as consecutive Functions of
    `chunk` blocks: autograd accumulates a Function's parameter gradients when
    its backward returns, so under data parallelism a chunked encoder hands its
    upper blocks' gradients to the bucketed all-reduce while the backward of the
    lower blocks is still running (the all-reduce of the last stack in the
    backward is otherwise fully exposed). fp8=False keeps a stack on bf16 GEMMs
    when the cache is in fp8 mode."""
    B, n, D = x.shape
    for c0, c1 in chunk_bounds(len(blocks), chunk):
        part = blocks[c0:c1]
        wT = [tuple(cache.get(w, dtype) for w in blk.gemm_weights()) for blk in part]
        w8 = ([tuple(cache.get_fp8(w) for w in blk.gemm_weights()) for blk in part]
              if fp8 and getattr(cache, "fp8", False) and dtype == torch.bfloat16 else None)
        spec = Fn.StackSpec(B=B, n=n, D=D, H=heads, eps=part[0].norm1.eps, dtype=dtype, wT=wT,
                            side=bool(CFG.side_stream), grouped_wgrad=bool(CFG.wgrad_grouped), w8=w8)
        params = [p for blk in part for p in blk.stack_params()]
        x = Fn.TransformerStackFn.apply(x, spec, *params)
    return x


class PatchEmbed(nn.Module):
    def __init__(self, img_size, patch, in_chans, dim):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch
        self.grid = img_size // patch
        self.num_patches = self.grid * self.grid
        self.proj = nn.Conv2d(in_chans, dim, kernel_size=patch, stride=patch)


class VisionTransformer(nn.Module):
    """timm VisionTransformer(num_classes=0, global_pool="avg") parameter layout
    (fc_norm used, final norm Identity)."""

    def __init__(self, model_name, img_size=None, depth=None):
        super().__init__()
        if model_name not in VIT_SPECS:
            raise ValueError(f"unsupported image model {model_name!r}; supported: {sorted(VIT_SPECS)}")
        D, dep, H, p, default_img = VIT_SPECS[model_name]
        img_size = img_size or default_img
        self.embed_dim = D
        self.num_heads = H
        self.patch_embed = PatchEmbed(img_size, p, 3, D)
        L = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.pos_embed = nn.Parameter(torch.zeros(1, L + 1, D))
        self.blocks = nn.ModuleList([Block(D, H) for _ in range(depth or dep)])
        self.fc_norm = nn.LayerNorm(D, eps=1e-6)
        self.num_features = D
        self.precision = CFG.precision
        _trunc_normal_(self.pos_embed)
        nn.init.normal_(self.cls_token, std=1e-6)
        for blk in self.blocks:
            blk.init_weights()

    def register_weights(self, cache: WeightCache):
        D = self.embed_dim
        w = self.patch_embed.proj.weight
        cache.register(w, (D, w[0].numel()))
        for blk in self.blocks:
            for p in blk.gemm_weights():
                cache.register(p, p.shape)
                cache.register_fp8(p)

    def forward_tokens(self, img, dtype, cache, ids_shuffle=None, ids_restore=None, keep=None, world=1):
        """img: the reference's fp32 NCHW batch [B,3,S,S] (dataset.py:34), or the
        decoded uint8 RGB pixels [B,S,S,3] (HWC), normalised inside the patch
        gather (A.Normalize of dataset.py:49 fused; no fp32 image in HBM)."""
        _require_device(img, "image batch")
        img = as_model_image(img, self.patch_embed.img_size)
        pe = self.patch_embed
        B = img.shape[0]
        L = pe.num_patches
        keep = L if keep is None else keep
        w = pe.proj.weight
        kreal = w[0].numel()
        epc = 8 if dtype == torch.bfloat16 else 4
        w_T, kpad = cache.get(w, dtype, (self.embed_dim, kreal)), kreal
        if kreal % epc or (dtype == torch.bfloat16 and kreal % 64):
            # p*p*3 = 588 at patch 14: the patch rows are gathered with zero
            # columns up to a multiple of 64 (16-B rows, the v4 GEMM's K step)
            # and the weight shadow is padded to match (dW is sliced back)
            kpad = (kreal + 63) // 64 * 64
            buf = getattr(self, "_w_pad", None)
            if buf is None or buf.shape != (self.embed_dim, kpad) or buf.dtype != dtype or buf.device != w.device:
                buf = torch.zeros((self.embed_dim, kpad), device=w.device, dtype=dtype)
                self._w_pad = buf
            buf[:, :kreal].copy_(w_T)
            w_T = buf
        spec = Fn.PatchSpec(B=B, L=L, keep=keep, p=pe.patch_size, kpad=kpad, dtype=dtype, w_T=w_T)
        x = Fn.PatchTokensFn.apply(img, ids_shuffle, ids_restore, spec, w, pe.proj.bias, self.cls_token,
                                   self.pos_embed)
        # under data parallelism (world = size of the model's process group) the
        # stack is cut into chunks so upper blocks' gradients reach the all-reduce early
        chunk = (CFG.dp_encoder_chunk or None) if world > 1 else None
        return run_stack(self.blocks, x, self.num_heads, dtype, cache, chunk=chunk)

    def forward(self, img):
        """timm semantics: pooled + fc_norm features [B, D] (no masking)."""
        dtype = compute_dtype(self.precision)
        cache = getattr(self, "_cache", None)
        if cache is None:
            cache = WeightCache(fp8=self.precision == "fp8")
            self.register_weights(cache)
            self._cache = cache
        cache.refresh(dtype)
        x = self.forward_tokens(img, dtype, cache)
        return Fn.EncoderHeadFn.apply(x, dtype, self.fc_norm.weight, self.fc_norm.bias, None, None)


class ImageEncoder(nn.Module):
    """modules.py:8-31: encode images to a fixed size vector (timm ViT, avg pool)."""

    def __init__(self, model_name=None, pretrained=None, trainable=None, img_size=None, depth=None):
        super().__init__()
        model_name = model_name or CFG.model_name
        pretrained = CFG.pretrained if pretrained is None else pretrained
        trainable = CFG.trainable if trainable is None else trainable
        if pretrained:
            raise RuntimeError("pretrained hub weights are unavailable offline; load a state_dict instead")
        self.model = VisionTransformer(model_name, img_size or CFG.size, depth)
        for p in self.model.parameters():
            p.requires_grad = trainable

    def forward(self, x):
        return self.model(x)


# ------------------------------------------------------------ DistilBERT
class DistilBertEmbeddings(nn.Module):
    def __init__(self, vocab, dim, max_pos):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab, dim)
        self.position_embeddings = nn.Embedding(max_pos, dim)
        self.LayerNorm = nn.LayerNorm(dim, eps=1e-12)


class DistilBertSelfAttention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.n_heads = heads
        self.q_lin = nn.Linear(dim, dim)
        self.k_lin = nn.Linear(dim, dim)
        self.v_lin = nn.Linear(dim, dim)
        self.out_lin = nn.Linear(dim, dim)


class FFN(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.lin1 = nn.Linear(dim, hidden)
        self.lin2 = nn.Linear(hidden, dim)


class TransformerBlock(nn.Module):
    def __init__(self, dim, heads, hidden):
        super().__init__()
        self.attention = DistilBertSelfAttention(dim, heads)
        self.sa_layer_norm = nn.LayerNorm(dim, eps=1e-12)
        self.ffn = FFN(dim, hidden)
        self.output_layer_norm = nn.LayerNorm(dim, eps=1e-12)


class Transformer(nn.Module):
    def __init__(self, n_layers, dim, heads, hidden):
        super().__init__()
        self.n_layers = n_layers
        self.layer = nn.ModuleList([TransformerBlock(dim, heads, hidden) for _ in range(n_layers)])


class DistilBertModel(nn.Module):
    """HF DistilBertModel parameter layout; forward-only (the reference freezes it,
    modules.py:35,42-43). Dropout (p=0.1 embeddings/attention/FFN) follows
    self.training like HF."""

    def __init__(self, n_layers=None, dim=768, heads=None, hidden=None, vocab=None, max_pos=None, dropout=None,
                 attention_dropout=None):
        super().__init__()
        self.n_layers = n_layers or CFG.text_layers
        self.dim = dim
        self.n_heads = heads or CFG.text_heads
        self.hidden = hidden or CFG.text_hidden
        self.dropout_p = CFG.text_dropout if dropout is None else dropout
        self.attn_dropout_p = CFG.text_attention_dropout if attention_dropout is None else attention_dropout
        self.embeddings = DistilBertEmbeddings(vocab or CFG.text_vocab_size, dim, max_pos or CFG.text_max_position)
        self.transformer = Transformer(self.n_layers, dim, self.n_heads, self.hidden)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
                if isinstance(m, nn.Linear):
                    nn.init.zeros_(m.bias)
        self.precision = CFG.precision
        self._wc_key = None
        self._wc = None

    def _weights(self, dtype):
        """Per-layer fused q|k|v weight/bias and GEMM weights in `dtype` (frozen:
        rebuilt only when a parameter changes, e.g. load_state_dict)."""
        key = (dtype, tuple((p.data_ptr(), p._version) for p in self.parameters()))
        if key != self._wc_key:
            layers = []
            for lyr in self.transformer.layer:
                at = lyr.attention
                wqkv = torch.cat([at.q_lin.weight, at.k_lin.weight, at.v_lin.weight], 0).to(dtype).contiguous()
                bqkv = torch.cat([at.q_lin.bias, at.k_lin.bias, at.v_lin.bias], 0).float().contiguous()
                layers.append((wqkv, bqkv, at.out_lin.weight.to(dtype).contiguous(),
                               lyr.ffn.lin1.weight.to(dtype).contiguous(), lyr.ffn.lin2.weight.to(dtype).contiguous()))
            self._wc = layers
            self._wc_key = key
        return self._wc

    @torch.no_grad()
    def forward(self, input_ids, attention_mask, dtype=None, seed=0, step_ptr=None):
        """Returns last_hidden_state [B, T, dim] (f32)."""
        _require_device(input_ids, "input_ids")
        dtype = dtype or compute_dtype(self.precision)
        B, T = input_ids.shape
        D, H = self.dim, self.n_heads
        hd = D // H
        train = self.training
        pdrop = self.dropout_p if train else 0.0
        padrop = self.attn_dropout_p if train else 0.0
        bf = dtype == torch.bfloat16
        ids = input_ids.to(torch.int64).contiguous()
        emb = self.embeddings
        if attention_mask.dtype == torch.int64 and attention_mask.is_contiguous() \
                and attention_mask.device == input_ids.device:
            # the tokenizer's int64 mask -> the f32 key mask inside the embedding launch
            x, am = K.embed_fwd(ids, emb.word_embeddings.weight, emb.position_embeddings.weight, mask=attention_mask)
        else:
            am = attention_mask.to(device=input_ids.device, dtype=torch.float32).contiguous()
            x = K.embed_fwd(ids, emb.word_embeddings.weight, emb.position_embeddings.weight)
        h, _, _, hT, _ = K.ln_fwd(x, emb.LayerNorm.weight, emb.LayerNorm.bias, 1e-12, out_dtype=torch.float32,
                                  out_dropout=pdrop, seed_out=seed * 131 + 1, want_stats=False, y2=bf,
                                  step_ptr=step_ptr)
        hT = hT if bf else h
        for li, (lyr, (wqkv, bqkv, wout, w1, w2)) in enumerate(zip(self.transformer.layer, self._weights(dtype))):
            qkv = K.linear_fwd(hT, wqkv, bqkv)
            o, _ = K.attn_fwd(qkv, B, T, H, hd, hd ** -0.5, key_mask=am, dropout_p=padrop,
                              seed=seed * 131 + 7 * li + 2, want_lse=False, step_ptr=step_ptr)
            sa = K.linear_fwd(o, wout, lyr.attention.out_lin.bias, out_dtype=torch.float32)
            a, _, _, aT, _ = K.ln_fwd(sa, lyr.sa_layer_norm.weight, lyr.sa_layer_norm.bias, 1e-12,
                                      out_dtype=torch.float32, res=h, want_stats=False, y2=bf)
            aT = aT if bf else a
            f1 = K.linear_fwd(aT, w1, lyr.ffn.lin1.bias, epilogue=K.EPI_GELU)   # frozen tower: no aux
            f2 = K.linear_fwd(f1, w2, lyr.ffn.lin2.bias, out_dtype=torch.float32)
            h, _, _, hT, _ = K.ln_fwd(f2, lyr.output_layer_norm.weight, lyr.output_layer_norm.bias, 1e-12,
                                      out_dtype=torch.float32, res=a, in_dropout=pdrop, seed_in=seed * 131 + 7 * li + 3,
                                      want_stats=False, y2=bf, step_ptr=step_ptr)
            hT = hT if bf else h
        return h.view(B, T, D)


class TextEncoder(nn.Module):
    """modules.py:34-51: DistilBERT, frozen by default, CLS-token embedding."""

    def __init__(self, model_name=None, pretrained=False, trainable=False, n_layers=None):
        super().__init__()
        self.model_name = model_name or CFG.text_encoder_model
        if pretrained:
            raise RuntimeError("DistilBertModel.from_pretrained needs the network; construct with "
                               "pretrained=False and load a state_dict")
        if trainable:
            raise NotImplementedError("the text tower is forward-only (the reference freezes it, modules.py:35)")
        self.model = DistilBertModel(n_layers=n_layers)
        for p in self.model.parameters():
            p.requires_grad = trainable
        self.target_token_idx = 0

    def forward(self, input_ids, attention_mask, seed=0, dtype=None, step_ptr=None):
        last_hidden_state = self.model(input_ids=input_ids, attention_mask=attention_mask, seed=seed, dtype=dtype,
                                       step_ptr=step_ptr)
        return last_hidden_state[:, self.target_token_idx, :]


# -------------------------------------------------------- ProjectionHead
class ProjectionHead(nn.Module):
    """modules.py:55-76 (computed in fp32 by one fused launch sequence)."""

    def __init__(self, embedding_dim, projection_dim=None, dropout=None):
        super().__init__()
        projection_dim = projection_dim or CFG.projection_dim
        dropout = CFG.dropout if dropout is None else dropout
        self.projection = nn.Linear(embedding_dim, projection_dim)
        self.gelu = nn.GELU()
        self.fc = nn.Linear(projection_dim, projection_dim)
        self.dropout = nn.Dropout(dropout)
        self.layer_norm = nn.LayerNorm(projection_dim)

    def forward(self, x, seed=0, step_ptr=None, bwd_step_ptr=None):
        """step_ptr: device step counter keying the dropout mask; bwd_step_ptr:
        where that step's value will be when the backward runs (CLIPModel's
        snapshot slot; None: the backward keeps a copy of it)."""
        _require_device(x, "projection input")
        p = self.dropout.p if self.training else 0.0
        spec = Fn.ProjSpec(p_drop=p, seed=seed, step_ptr=step_ptr, bwd_step_ptr=bwd_step_ptr)
        return Fn.ProjectionHeadFn.apply(x, spec, self.projection.weight, self.projection.bias, self.fc.weight,
                                         self.fc.bias, self.layer_norm.weight, self.layer_norm.bias)


# ----------------------------------------------------------- MAE decoder
def build_2d_sincos(grid, dim):
    """HF build_2d_sinusoidal_position_embedding(cls_token=True) + the h/w half
    rotation of ViTMAEDecoder.initialize_weights (modeling_vit_mae.py:521-534)."""
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
    """MAE reconstruction head: mae_norm + HF ViTMAEDecoder
    (decoder_embed, mask_token, fixed sin-cos decoder_pos_embed, decoder_layers,
    decoder_norm, decoder_pred)."""

    def __init__(self, enc_dim, num_patches, patch, dim=None, depth=None, heads=None, mlp_ratio=None, in_chans=3):
        super().__init__()
        dim = dim or CFG.decoder_embed_dim
        depth = depth or CFG.decoder_depth
        heads = heads or CFG.decoder_num_heads
        mlp_ratio = mlp_ratio or CFG.decoder_mlp_ratio
        self.num_heads = heads
        self.patch_size = patch
        self.mae_norm = nn.LayerNorm(enc_dim, eps=1e-6)
        self.decoder_embed = nn.Linear(enc_dim, dim)
        self.mask_token = nn.Parameter(torch.zeros(1, 1, dim))
        grid = int(round(num_patches ** 0.5))
        self.register_buffer("decoder_pos_embed", build_2d_sincos(grid, dim).unsqueeze(0), persistent=True)
        self.decoder_layers = nn.ModuleList([Block(dim, heads, mlp_ratio) for _ in range(depth)])
        self.decoder_norm = nn.LayerNorm(dim, eps=1e-6)
        self.decoder_pred = nn.Linear(dim, patch * patch * in_chans)
        nn.init.normal_(self.mask_token, std=0.02)
        # HF ViTMAEPreTrainedModel._init_weights: every Linear trunc-normal(0.02), zero bias
        for blk in self.decoder_layers:
            blk.init_weights()
        _trunc_normal_(self.decoder_embed.weight)
        nn.init.zeros_(self.decoder_embed.bias)
        _trunc_normal_(self.decoder_pred.weight)
        nn.init.zeros_(self.decoder_pred.bias)
        self._pred_pad = None

    def padded_pred(self, w_T):
        """decoder_pred weight shadow / bias copied into buffers whose output rows
        are rounded up to a multiple of 64 (pad rows / entries stay zero)."""
        P, Dd = w_T.shape
        npad = (P + 63) // 64 * 64
        pad = self._pred_pad
        if pad is None or pad[0].shape != (npad, Dd) or pad[0].dtype != w_T.dtype or pad[0].device != w_T.device:
            pad = (torch.zeros((npad, Dd), device=w_T.device, dtype=w_T.dtype),
                   torch.zeros((npad,), device=w_T.device, dtype=torch.float32))
            self._pred_pad = pad
        pad[0][:P].copy_(w_T)
        pad[1][:P].copy_(self.decoder_pred.bias.detach())
        return pad

    def register_weights(self, cache: WeightCache):
        cache.register(self.decoder_embed.weight, self.decoder_embed.weight.shape)
        for blk in self.decoder_layers:
            for p in blk.gemm_weights():
                cache.register(p, p.shape)
                if CFG.fp8_decoder:
                    cache.register_fp8(p)
        cache.register(self.decoder_pred.weight, self.decoder_pred.weight.shape)
