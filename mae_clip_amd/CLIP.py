"""Drop-in for the reference's CLIP.py (CLIP.py:9-52): CLIPModel + cross_entropy.

CLIPModel.forward(batch) -> 0-d loss, exactly the reference contract used by
main.py:56-59 (model(batch); loss.backward(); optimizer.step()) and
main.py:76 (no_grad eval). With config.mask_ratio > 0 the MAE head of
BASELINE.json is added: the encoder runs once on the
visible patches (FLIP-style), the CLIP image feature is the mean over visible
patch tokens -> fc_norm, the decoder reconstructs the masked patches and
loss = clip + mae_weight * mae. With mask_ratio == 0 the path is the
reference's CLIP path exactly.

Data parallel (one process per GPU): if torch.distributed is initialised and
`model.process_group` is set (mae_clip_amd.distributed.DataParallel does it),
the projection embeddings are all-gathered so the contrastive loss uses the
global batch, and the MAE term's gradient is scaled by 1/world so that a SUM
all-reduce of parameter gradients yields the exact global-batch gradient.
"""
from __future__ import annotations

import torch
from torch import nn
import torch.nn.functional as F

from . import config as CFG
from . import functions as Fn
from . import kernels as K
from .modules import (ImageEncoder, TextEncoder, ProjectionHead, MAEDecoder, WeightCache, compute_dtype,
                      run_stack, _require_device, as_model_image)


class CLIPModel(nn.Module):
    def __init__(self, temperature=None, image_embedding=None, text_embedding=None):
        super().__init__()
        temperature = CFG.temperature if temperature is None else temperature
        image_embedding = image_embedding or CFG.image_embedding
        text_embedding = text_embedding or CFG.text_embedding
        self.image_encoder = ImageEncoder()
        self.text_encoder = TextEncoder()
        if self.image_encoder.model.embed_dim != image_embedding:
            raise ValueError(f"image_embedding={image_embedding} but {CFG.model_name} has "
                             f"{self.image_encoder.model.embed_dim} features")
        self.image_projection = ProjectionHead(embedding_dim=image_embedding)
        self.text_projection = ProjectionHead(embedding_dim=text_embedding)
        self.temperature = temperature
        self.mask_ratio = CFG.mask_ratio
        self.mae_weight = CFG.mae_weight
        self.norm_pix_loss = CFG.norm_pix_loss
        self.precision = CFG.precision
        self.mask_seed = CFG.mask_seed
        self.dropout_seed = CFG.dropout_seed
        vit = self.image_encoder.model
        if self.mask_ratio > 0:
            self.mae_decoder = MAEDecoder(vit.embed_dim, vit.patch_embed.num_patches, vit.patch_embed.patch_size)
        else:
            self.mae_decoder = None
        self.step = 0
        # device-resident step: keys the MAE mask noise and every dropout mask, and
        # is advanced by a kernel at the end of each training forward, so a
        # captured HIP graph of the step (mae_clip_amd.graph) draws fresh masks
        # on every replay. Not persistent: state_dict keys stay the reference's.
        self.register_buffer("step_counter", torch.zeros(1, dtype=torch.int64), persistent=False)
        # step_snaps[s % 8]: the step_counter value training forward s ran with,
        # written by the kernel that advances the counter; that forward's
        # backward re-draws its dropout masks from it (up to 8 forwards in flight)
        self.register_buffer("step_snaps", torch.zeros(8, dtype=torch.int64), persistent=False)
        self.last_losses = {}
        self.process_group = None
        self.grad_arena = None     # set by distributed.DataParallel (flat all-reduce buffer)
        self._cache = None

    # ------------------------------------------------------------------
    def _weight_cache(self):
        if self._cache is None:
            c = WeightCache(fp8=self.precision == "fp8")
            self.image_encoder.model.register_weights(c)
            if self.mae_decoder is not None:
                self.mae_decoder.register_weights(c)
            self._cache = c
        return self._cache

    def _world(self):
        pg = self.process_group
        if pg is None or not torch.distributed.is_initialized():
            return 1, 0
        return torch.distributed.get_world_size(pg), torch.distributed.get_rank(pg)

    def masking(self, B, sample_offset, device):
        """HF random_masking ids of the current device step (step_counter)."""
        vit = self.image_encoder.model
        L = vit.patch_embed.num_patches
        keep = int(L * (1 - self.mask_ratio))
        ids_shuffle, ids_restore, mask, _ = K.mask_ids(B, L, keep, self.mask_seed, 0, sample_offset, device,
                                                       step_ptr=self.step_counter)
        return ids_shuffle, ids_restore, mask, keep

    def forward(self, batch):
        """batch["image"]: the reference's fp32 NCHW normalised images
        (dataset.py:44-58, :34), or the decoded uint8 RGB HWC pixels
        [B, S, S, 3] -- then A.Normalize and the permute run inside the patch
        gather and the MAE target read (data.py)."""
        img = batch["image"]
        _require_device(img, "image batch")
        dtype = compute_dtype(self.precision)
        vit = self.image_encoder.model
        B = img.shape[0]
        world, rank = self._world()
        Fn.set_grad_arena(self.grad_arena if torch.is_grad_enabled() else None)
        sc = self.step_counter
        _require_device(sc, "CLIPModel.step_counter (call .to(device))")
        # step-independent seed base; the kernels add step_counter * MAECLIP_STEP_MULT
        seed = (self.dropout_seed * 1000003 + rank) & 0x7FFFFFFFFFFFFFFF
        # the frozen text tower (no autograd, own bf16 weights) is independent of
        # the image path: it runs on the side stream, overlapped with the image
        # encoder, and is issued first so it also overlaps the weight-shadow cast
        use_side = bool(CFG.side_stream)
        main = torch.cuda.current_stream(img.device)
        if use_side:
            side = Fn.side_stream(img.device)
            side.wait_stream(main)
            with torch.cuda.stream(side), K.gemm_split_scope(bool(CFG.text_gemm_split)):
                text_features = self.text_encoder(batch["input_ids"], batch["attention_mask"], seed=seed + 17,
                                                  dtype=dtype, step_ptr=sc)
        cache = self._weight_cache()
        cache.refresh(dtype)
        mae = self.mae_decoder is not None
        if mae:
            ids_shuffle, ids_restore, mask, keep = self.masking(B, rank * B, img.device)
            tokens = vit.forward_tokens(img, dtype, cache, ids_shuffle, ids_restore, keep, world=world)
            dec = self.mae_decoder
            feat, latent = Fn.EncoderHeadFn.apply(tokens, dtype, vit.fc_norm.weight, vit.fc_norm.bias,
                                                  dec.mae_norm.weight, dec.mae_norm.bias)
        else:
            tokens = vit.forward_tokens(img, dtype, cache, world=world)
            feat = Fn.EncoderHeadFn.apply(tokens, dtype, vit.fc_norm.weight, vit.fc_norm.bias, None, None)
        if use_side:
            main.wait_stream(side)
            text_features.record_stream(main)
        else:
            text_features = self.text_encoder(batch["input_ids"], batch["attention_mask"], seed=seed + 17,
                                              dtype=dtype, step_ptr=sc)
        snap = self.step_snaps[self.step % 8:self.step % 8 + 1] if self.training else None
        image_embeddings = self.image_projection(feat, seed=seed + 29, step_ptr=sc, bwd_step_ptr=snap)
        text_embeddings = self.text_projection(text_features, seed=seed + 31, step_ptr=sc, bwd_step_ptr=snap)
        clip = clip_loss(image_embeddings, text_embeddings, self.temperature,
                         group=self.process_group if world > 1 else None)
        loss = clip
        self.last_losses = {"clip": clip.detach()}
        if mae:
            L = vit.patch_embed.num_patches
            dspec = Fn.DecSpec(B=B, L=L, keep=keep, dtype=dtype, w_T=cache.get(dec.decoder_embed.weight, dtype))
            xd = Fn.DecoderEmbedFn.apply(latent, ids_shuffle, ids_restore, dspec, dec.decoder_embed.weight,
                                         dec.decoder_embed.bias, dec.mask_token, dec.decoder_pos_embed)
            # fp8 mode: the decoder stack on fp8 GEMMs too unless CFG.fp8_decoder is
            # off (A/B in DESIGN.md Round 6: +1.9 %, its K = 512 GEMMs stay
            # epilogue-bound)
            xd = run_stack(dec.decoder_layers, xd, dec.num_heads, dtype, cache,
                           chunk=(CFG.dp_decoder_chunk or None) if world > 1 else None, fp8=CFG.fp8_decoder)
            wp_T, bp_pad = cache.get(dec.decoder_pred.weight, dtype), None
            P = wp_T.shape[0]
            if dtype == torch.bfloat16 and P % 64:
                # p*p*C = 588 at patch 14: pad decoder_pred's output rows to a
                # multiple of 64 (16-B rows for every GEMM of the head); zero
                # weight rows / bias entries, pred's pad columns are never read
                wp_T, bp_pad = dec.padded_pred(wp_T)
            hspec = Fn.MaeHeadSpec(p=vit.patch_embed.patch_size, norm_pix=self.norm_pix_loss,
                                   mask_count=float(B * (L - keep)), loss_scale=1.0 / world, dtype=dtype,
                                   w_T=wp_T, b_pad=bp_pad)
            ml = Fn.MaeHeadLossFn.apply(xd, as_model_image(img, vit.patch_embed.img_size), mask, hspec,
                                        dec.decoder_norm.weight, dec.decoder_norm.bias, dec.decoder_pred.weight,
                                        dec.decoder_pred.bias)
            self.last_losses["mae"] = ml.detach()
            loss = Fn.CombineLossFn.apply(clip, ml, self.mae_weight)
            self.last_mask = (ids_shuffle, ids_restore, mask)
        if self.training:
            K.counter_add_snap(sc, snap, 1)
            self.step += 1
        return loss


def clip_loss(image_embeddings, text_embeddings, temperature=1.0, group=None):
    """CLIP.py:34-43 on the fused fp32 kernel (group: data-parallel gather)."""
    if torch.is_grad_enabled() and (image_embeddings.requires_grad or text_embeddings.requires_grad):
        return Fn.ClipLossFn.apply(image_embeddings, text_embeddings, temperature, group)
    I, T = image_embeddings.contiguous(), text_embeddings.contiguous()
    if group is not None:
        from .distributed import all_gather_rows
        I, T = all_gather_rows(I, group), all_gather_rows(T, group)
    loss, _, _ = K.clip_loss(I, T, temperature, want_grad=False)
    return loss


def cross_entropy(preds, targets, reduction="none"):
    """CLIP.py:46-52, kept for API compatibility (not used on the fused path)."""
    log_softmax = nn.LogSoftmax(dim=-1)
    loss = (-targets * log_softmax(preds)).sum(1)
    if reduction == "none":
        return loss
    elif reduction == "mean":
        return loss.mean()
