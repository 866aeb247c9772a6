"""Embedding search of the reference's inference.py on libmaeclip kernels
(SURVEY.md §8f row 4).

inference.py:13-27 (get_image_embeddings) runs the image tower + projection
over the validation loader; inference.py:29-47 (find_matches) embeds one
tokenised query, L2-normalises both sides (F.normalize), forms
text_n @ image_n.T and keeps every 5th of the top n*5 matches. The same calls
are made here, with the normalisation, the fp32 similarity GEMM and the top-k
selection on the device (maeclip_l2_normalize / maeclip_gemm /
maeclip_topk_rows). Tokenisation (DistilBertTokenizer.from_pretrained) and the
matplotlib display stay with the caller: there is no tokenizer download here.
"""
from __future__ import annotations

import torch

from . import kernels as K
from .kernels import _dev, _call, _stream


def l2_normalize(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """F.normalize(x, p=2, dim=-1) for fp32 [M, P] (inference.py:40-41)."""
    _dev(x)
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("l2_normalize: fp32 [M, P] with unit column stride expected")
    y = torch.empty(x.shape, device=x.device, dtype=torch.float32)
    _call("maeclip_l2_normalize", x.data_ptr(), y.data_ptr(), x.shape[0], x.shape[1], x.stride(0), y.stride(0), eps,
          _stream())
    return y


def topk_rows(s: torch.Tensor, k: int):
    """torch.topk(s, k, dim=-1) for fp32 [Q, N]: values descending, ties -> lower index."""
    _dev(s)
    if s.dtype != torch.float32 or s.dim() != 2 or s.stride(1) != 1:
        raise ValueError("topk_rows: fp32 [Q, N] with unit column stride expected")
    Q, N = s.shape
    vals = torch.empty((Q, k), device=s.device, dtype=torch.float32)
    idx = torch.empty((Q, k), device=s.device, dtype=torch.int64)
    _call("maeclip_topk_rows", s.data_ptr(), Q, N, s.stride(0), int(k), vals.data_ptr(), idx.data_ptr(), _stream())
    return vals, idx


def similarity(text_embeddings: torch.Tensor, image_embeddings: torch.Tensor) -> torch.Tensor:
    """normalize(text) @ normalize(image).T (inference.py:40-42), fp32 [Q, N]."""
    tn = l2_normalize(text_embeddings.float().contiguous())
    im = l2_normalize(image_embeddings.float().contiguous())
    Q, P = tn.shape
    N = im.shape[0]
    # the GEMM writes 4-column groups: a gallery of any size is padded with zero
    # rows to a multiple of 4 and the padded similarity columns are cut off
    # (a view with row stride Npad: topk_rows honours it)
    Npad = (N + 3) // 4 * 4
    if Npad != N:
        im = torch.cat([im, im.new_zeros((Npad - N, P))])
    out = torch.empty((Q, Npad), device=tn.device, dtype=torch.float32)
    K.gemm(tn, im, out, Q, Npad, P, tn.stride(0), im.stride(0), Npad, K.KC, K.KC)
    return out[:, :N]


@torch.no_grad()
def get_image_embeddings(model, image_batches):
    """inference.py:13-27 minus the loader: image tower + projection over an
    iterable of device image batches ([B, 3, S, S] fp32) in eval mode."""
    model.eval()
    out = [model.image_projection(model.image_encoder(b)) for b in image_batches]
    return torch.cat(out)


@torch.no_grad()
def find_matches(model, image_embeddings, input_ids, attention_mask, n=9):
    """inference.py:29-45: indices of the n matches of one tokenised query
    (torch.topk(..., n * 5) then every 5th, as the reference does)."""
    model.eval()
    text_features = model.text_encoder(input_ids=input_ids, attention_mask=attention_mask)
    text_embeddings = model.text_projection(text_features)
    sim = similarity(text_embeddings, image_embeddings)
    _, indices = topk_rows(sim[:1], n * 5)
    return indices[0, ::5]
