"""C-ABI boundary checks that need no GPU: the library loads, exports exactly
what include/maeclip.h declares, validates arguments and reports errors
through maeclip_last_error (the torch RuntimeError convention main.py relies on)."""
import ctypes
import os
import re

import pytest
import torch

from mae_clip_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "maeclip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(maeclip_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_abi():
    lib = L.load()
    assert lib.maeclip_abi_version() == L.ABI_VERSION


def test_every_declared_symbol_is_exported_and_bound():
    lib = L.load()
    decl = header_functions()
    assert len(decl) >= 30
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in include/maeclip.h but not exported"
        assert name in L.EXPORTED_SYMBOLS, f"{name} not bound in mae_clip_amd/_lib.py"


def test_struct_layouts_match_header_sizes():
    # field counts of the ctypes mirrors vs the header structs
    src = open(os.path.join(ROOT, "include", "maeclip.h")).read()
    for cname, pyname in [("maeclip_gemm_args", "GemmArgs"), ("maeclip_attn_args", "AttnArgs"),
                          ("maeclip_ln_fwd_args", "LnFwdArgs"), ("maeclip_ln_bwd_args", "LnBwdArgs"),
                          ("maeclip_mask_args", "MaskArgs"), ("maeclip_clip_args", "ClipArgs"),
                          ("maeclip_mae_loss_args", "MaeLossArgs"), ("maeclip_unshuffle_args", "UnshuffleArgs"),
                          ("maeclip_tokens_args", "TokensArgs"), ("maeclip_patch_args", "PatchArgs"),
                          ("maeclip_mt_entry", "MtEntry"), ("maeclip_colsum_entry", "ColsumEntry")]:
        body = re.search(r"typedef struct \{([^{}]*)\}\s*" + cname + ";", src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        body = re.sub(r"//[^\n]*", "", body)
        n = sum(len([v for v in decl.split(";")[0].split(",")]) for decl in body.split(";") if decl.strip())
        assert n == len(getattr(L, pyname)._fields_), (cname, n, len(getattr(L, pyname)._fields_))


def test_argument_validation_and_error_string():
    lib = L.load()
    a = L.GemmArgs(M=4, N=4, K=8, lda=8, ldb=8, ldc=4, batch=1, dtype=7, out_dtype=0)
    rc = lib.maeclip_gemm(ctypes.byref(a), None)
    assert rc < 0
    assert b"bad dtype" in lib.maeclip_last_error()
    rc = lib.maeclip_colsum_reduce(None, 0, 0, None, 0, 1.0, None, None)
    assert rc < 0 and b"colsum_reduce" in lib.maeclip_last_error()
    m = L.MaskArgs(B=1, L=2000, len_keep=1)
    assert lib.maeclip_mask_ids(ctypes.byref(m), None) < 0   # L > 1024 rejected before launch


def test_splitk_plan():
    lib = L.load()
    assert lib.maeclip_gemm_splitk(2048, 512, 50432) > 1
    assert lib.maeclip_gemm_splitk(12800, 3072, 768) == 1


def test_no_cpu_fallback():
    """The product raises on CPU tensors instead of silently computing elsewhere."""
    from mae_clip_amd import kernels as K
    x = torch.randn(4, 8)
    with pytest.raises(L.MaeClipNativeError):
        K.linear_fwd(x, torch.randn(4, 8))
    from tests.helpers import product_config, C0, make_batch
    from mae_clip_amd.CLIP import CLIPModel
    kw = {k: v for k, v in C0.items() if k != "batch_size"}
    with product_config(precision="fp32", **kw):
        m = CLIPModel()
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(make_batch(2, 32))


def test_api_surface_matches_reference():
    """modules.py / CLIP.py names and state_dict keys (reference + timm/HF layouts)."""
    from mae_clip_amd import modules, CLIP
    from tests.helpers import product_config, C0
    for name in ("ImageEncoder", "TextEncoder", "ProjectionHead"):
        assert hasattr(modules, name)
    assert hasattr(CLIP, "CLIPModel") and hasattr(CLIP, "cross_entropy")
    kw = {k: v for k, v in C0.items() if k != "batch_size"}
    with product_config(**kw):
        m = CLIP.CLIPModel()
    for attr in ("image_encoder", "text_encoder", "image_projection", "text_projection", "temperature"):
        assert hasattr(m, attr)
    keys = set(m.state_dict())
    for k in ("image_encoder.model.patch_embed.proj.weight", "image_encoder.model.blocks.0.attn.qkv.weight",
              "image_encoder.model.fc_norm.weight", "text_encoder.model.embeddings.word_embeddings.weight",
              "text_encoder.model.transformer.layer.0.attention.q_lin.weight",
              "text_encoder.model.transformer.layer.1.output_layer_norm.bias",
              "image_projection.projection.weight", "image_projection.fc.bias", "image_projection.layer_norm.weight",
              "text_projection.projection.weight"):
        assert k in keys, k
    # the text tower is frozen (modules.py:35,42-43)
    assert not any(p.requires_grad for p in m.text_encoder.parameters())
    assert m.text_encoder.target_token_idx == 0
    head = modules.ProjectionHead(embedding_dim=192)
    assert [n for n, _ in head.named_children()] == ["projection", "gelu", "fc", "dropout", "layer_norm"]


def test_cross_entropy_matches_reference_formula():
    from mae_clip_amd.CLIP import cross_entropy
    from oracle.ref_model import cross_entropy as ref_ce
    p, t = torch.randn(5, 7), torch.softmax(torch.randn(5, 7), -1)
    assert torch.allclose(cross_entropy(p, t), ref_ce(p, t))
    assert torch.allclose(cross_entropy(p, t, "mean"), ref_ce(p, t, "mean"))
