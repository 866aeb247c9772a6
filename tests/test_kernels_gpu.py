"""Kernel-level numerics: each HIP kernel vs a plain PyTorch fp32/fp64 reference
of the same op (same seeded inputs). Runs on the GPU box only."""
import math

import pytest
import torch

from mae_clip_amd import kernels as K

pytestmark = pytest.mark.gpu


def _rand(shape, dtype, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dtype).to(dev)


def _ref_mm(A, B):
    return (A.double() @ B.double())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("lay", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("mnk", [(256, 256, 128), (200, 136, 72), (16, 8, 64), (384, 640, 1024), (264, 520, 64), (520, 264, 192),
                                 (640, 520, 256)])
def test_gemm_layouts(dev, dtype, lay, mnk):
    M, N, Kd = mnk
    a_lay, b_lay = lay
    A = _rand((M, Kd) if a_lay == 0 else (Kd, M), dtype, dev, seed=1)
    B = _rand((N, Kd) if b_lay == 0 else (Kd, N), dtype, dev, seed=2)
    C = torch.empty((M, N), device=dev, dtype=torch.float32)
    K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, a_lay, b_lay, alpha=0.5)
    Am = A if a_lay == 0 else A.t()
    Bm = B.t() if b_lay == 0 else B
    ref = 0.5 * _ref_mm(Am, Bm)
    err = (C.double() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err / scale < (2e-6 if dtype == torch.float32 else 2e-5) * math.sqrt(Kd), (err, scale)


@pytest.mark.parametrize("b_lay", [0, 1])
@pytest.mark.parametrize("mnk", [(12800, 768, 768), (1000, 520, 192), (50000, 512, 256), (192, 256, 64), (193, 264, 128),
                                 (12800, 3072, 768), (6400, 768, 3072), (300, 264, 64)])
@pytest.mark.parametrize("bm", ["192", "128"])
def test_gemm_bm192(dev, b_lay, mnk, bm, opts):
    """192- and 128-row tiles of the v4 kernel (forced): ragged M / N, one tile, several persistent tiles per
    block (M = 50000: 261 x 2 tiles on 256 CUs at 192 rows), one K-tile, KC x KC and KC x RC."""
    opts(GEMM_BM=int(bm))
    M, N, Kd = mnk
    A = _rand((M, Kd), torch.bfloat16, dev, seed=1)
    B = _rand((N, Kd) if b_lay == 0 else (Kd, N), torch.bfloat16, dev, seed=2)
    for out in (torch.float32, torch.bfloat16):
        C = torch.empty((M, N), device=dev, dtype=out)
        K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, 0, b_lay, alpha=0.5)
        ref = 0.5 * _ref_mm(A, B.t() if b_lay == 0 else B)
        err = (C.double() - ref).abs().max().item()
        scale = ref.abs().max().item() + 1e-6
        assert err / scale < (2e-5 * math.sqrt(Kd) if out == torch.float32 else 1e-2), (out, err, scale)


def _ncu(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _plan_workspace(dev, M, N, Kd, b_lay):
    """scratch bytes maeclip_gemm asks for this plain bf16 launch under the
    current options (> 0: a split plan was chosen)"""
    import ctypes
    from mae_clip_amd import _lib as L
    a = L.GemmArgs(A=16, B=16, C=16, M=M, N=N, K=Kd, lda=Kd, ldb=Kd if b_lay == 0 else N, ldc=N, batch=1,
                   dtype=L.BF16, out_dtype=L.F32, a_layout=0, b_layout=b_lay, alpha=1.0, splitk=1)
    return int(L.lib().maeclip_gemm_workspace(ctypes.byref(a)))


def _sk_counters_zero():
    """every per-stream GEMM scratch: the stream-K arrival counters (its first
    16 KiB) are back to zero after the launches completed"""
    torch.cuda.synchronize()
    for t in K._SCRATCH.values():
        assert int(t[:4096].view(torch.int32).abs().sum().item()) == 0


@pytest.mark.parametrize("b_lay", [0, 1])
@pytest.mark.parametrize("mnk", [(6400, 768, 3072), (6400, 2304, 768), (25216, 512, 2048), (50432, 512, 1536),
                                 (1000, 520, 192), (300, 264, 640), (12800, 768, 768)])
@pytest.mark.parametrize("mode", ["auto", "split2_192", "split2_192_lead0", "split2_192_lead9"])
def test_gemm_stream_k(dev, b_lay, mnk, mode, opts):
    """Split plain launches (every tile's K range cut into S slices, the
    slices summed in the same launch by the block that arrives last, gemm4.hip
    sk_fixup): forced on 192-row tiles ("split2_192", slice 0's lead per
    other slice 4 K-tiles by default, 0 = equal slices, 9) or the cost model's
    own choice ("auto"). Shapes: the micro-batch's encoder dgrads
    (75 tiles for 256 CUs), the decoder's N = 512 dgrads (198 tiles: 396
    units of S = 2 = two rounds of the grid), small ragged launches (slices of
    one or two K-tiles, partial edge tiles).
    vs fp64; bitwise equal on repeat (the summation order is fixed whichever
    block arrives last); counters left zero."""
    if mode.startswith("split"):
        opts(GEMM_SPLIT=int(mode[5]))
        opts(GEMM_BM=192)
    else:
        opts(GEMM_SK=1)   # the cost model (off by default)
    if "_lead" in mode:
        opts(GEMM_SPLIT_D=int(mode.split("_lead")[1]))
    M, N, Kd = mnk
    if mode.startswith("split"):
        # the forced split is taken wherever it fits (tiles <= 256, 2 slices
        # per tile <= 2 rounds of the grid, >= 2 K-tiles per slice), else the
        # best data-parallel plan: the workspace query says which
        T = -(-M // 192) * -(-N // 256)
        fits = T <= 256 and 2 * T <= 2 * _ncu(dev) and Kd // 64 >= 4
        assert (_plan_workspace(dev, M, N, Kd, b_lay) > 0) == fits, (mnk, T)
    A = _rand((M, Kd), torch.bfloat16, dev, seed=11)
    B = _rand((N, Kd) if b_lay == 0 else (Kd, N), torch.bfloat16, dev, scale=0.5, seed=12)
    ref = _ref_mm(A, B.t() if b_lay == 0 else B)
    scale = ref.abs().max().item()
    for out in (torch.float32, torch.bfloat16):
        C = torch.empty((M, N), device=dev, dtype=out)
        K.gemm(A, B, C, M, N, Kd, A.stride(0), B.stride(0), N, 0, b_lay)
        err = (C.double() - ref).abs().max().item()
        assert err / scale < (2e-5 * math.sqrt(Kd) if out == torch.float32 else 1e-2), (out, err, scale)
        C2 = torch.empty_like(C)
        for _ in range(2):
            K.gemm(A, B, C2, M, N, Kd, A.stride(0), B.stride(0), N, 0, b_lay)
            assert torch.equal(C, C2)
    _sk_counters_zero()


@pytest.mark.parametrize("mode", ["split2_192", "split2_192_lead0", "bm128"])
def test_gemm_stream_k_epilogues(dev, mode, opts):
    """Every fused epilogue behind the split fix-up (the last block runs it
    on the summed tile): bias + GELU / GELU' (aux_out), fp32 residual, column
    sums, dGELU, mul-aux + residual; M = 3000 x N = 768 (36 / 48 tiles, every
    tile cut) at K = 1024."""
    if mode == "bm128":   # the 128-row tile's epilogues (no split)
        opts(GEMM_BM=128)
    else:
        opts(GEMM_SPLIT=int(mode[5]))
        opts(GEMM_BM=192)
    if "_lead" in mode:
        opts(GEMM_SPLIT_D=int(mode.split("_lead")[1]))
    M, N, Kd = 3000, 768, 1024
    if mode != "bm128":   # 16 x 3 tiles: every tile is cut
        assert _plan_workspace(dev, M, N, Kd, 0) > 0
    x = _rand((M, Kd), torch.bfloat16, dev, seed=13)
    w = _rand((N, Kd), torch.bfloat16, dev, scale=0.03, seed=14)
    bias = _rand((N,), torch.float32, dev, seed=15)
    resid = _rand((M, N), torch.float32, dev, seed=16)
    ref = _ref_mm(x, w.t()) + bias.double()
    tol = 4e-2
    pre = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    y = K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU, aux_out=pre)
    assert (pre.double() - ref).abs().max().item() < tol
    assert (y.double() - torch.nn.functional.gelu(ref)).abs().max().item() < tol
    y2 = K.linear_fwd(x, w, bias, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=resid)
    assert (y2.double() - (ref + resid.double())).abs().max().item() < 1e-3
    part = torch.empty((K.gemm_colsum_rows(M), N), device=dev, dtype=torch.float32)
    y3 = K.linear_fwd(x, w, bias, out_dtype=torch.float32, colsum=part)
    assert (K.colsum_reduce(part).double() - y3.double().sum(0)).abs().max().item() < 1e-2
    d = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    y4 = K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU_D, aux_out=d)
    r64 = ref.clone().requires_grad_(True)
    gref = torch.autograd.grad(torch.nn.functional.gelu(r64).sum(), r64)[0]
    assert (y4.double() - torch.nn.functional.gelu(ref)).abs().max().item() < tol
    assert (d.double() - gref).abs().max().item() < tol
    dy = _rand((M, N), torch.bfloat16, dev, seed=17)
    aux = _rand((M, Kd), torch.bfloat16, dev, seed=18)
    dx = K.linear_dgrad(dy, w, epilogue=K.EPI_DGELU, aux=aux, out_dtype=torch.float32)
    a64 = aux.double().requires_grad_(True)
    g = torch.autograd.grad(torch.nn.functional.gelu(a64).sum(), a64)[0]
    ref_dx = _ref_mm(dy, w) * g
    assert (dx.double() - ref_dx).abs().max().item() < 1e-3 * max(1.0, ref_dx.abs().max().item())
    rd = _rand((M, Kd), torch.float32, dev, seed=19)
    dx5 = K.linear_dgrad(dy, w, epilogue=K.EPI_MUL_AUX, aux=aux, out_dtype=torch.float32, resid=rd)
    ref5 = _ref_mm(dy, w) * aux.double() + rd.double()
    assert (dx5.double() - ref5).abs().max().item() < 1e-3 * max(1.0, ref5.abs().max().item())
    _sk_counters_zero()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M", [300, 700])   # fp32: 32x32-tile small kernel / 128x128 MFMA kernel
@pytest.mark.parametrize("bm", ["auto", "192"])
def test_gemm_epilogues(dev, dtype, M, bm, opts):
    """bm = "192": every epilogue on 192-row tiles (forced; colsum launches keep
    256)."""
    if bm != "auto":
        if dtype == torch.float32:
            pytest.skip("192-row tiles: bf16 operands")
        opts(GEMM_BM=192)
    N, Kd = 384, 256
    x = _rand((M, Kd), dtype, dev, seed=3)
    w = _rand((N, Kd), dtype, dev, scale=0.05, seed=4)
    bias = _rand((N,), torch.float32, dev, seed=5)
    resid = _rand((M, N), torch.float32, dev, seed=6)
    ref = _ref_mm(x, w.t()) + bias.double()
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    # bias + gelu (pre stored to aux_out)
    pre = torch.empty((M, N), device=dev, dtype=dtype)
    y = K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU, aux_out=pre)
    assert (pre.double() - ref).abs().max().item() < tol * 4
    assert (y.double() - torch.nn.functional.gelu(ref)).abs().max().item() < tol * 4
    # residual
    y2 = K.linear_fwd(x, w, bias, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=resid)
    assert (y2.double() - (ref + resid.double())).abs().max().item() < tol * 4
    # colsum partial
    part = torch.empty((K.gemm_colsum_rows(M), N), device=dev, dtype=torch.float32)
    y3 = K.linear_fwd(x, w, bias, out_dtype=torch.float32, colsum=part)
    cs = K.colsum_reduce(part)
    assert (cs.double() - y3.double().sum(0)).abs().max().item() < 1e-3
    # dgelu: dx = (dy @ w) * gelu'(aux)
    dy = _rand((M, N), dtype, dev, seed=7)
    aux = _rand((M, Kd), dtype, dev, seed=8)
    dx = K.linear_dgrad(dy, w, epilogue=K.EPI_DGELU, aux=aux, out_dtype=torch.float32)
    a64 = aux.double().requires_grad_(True)
    g = torch.autograd.grad(torch.nn.functional.gelu(a64).sum(), a64)[0]
    ref_dx = _ref_mm(dy, w) * g
    assert (dx.double() - ref_dx).abs().max().item() < tol * 4
    # GELU' epilogue (aux_out <- gelu'(pre)) and mul-aux: the MLP's fused pair
    d = torch.empty((M, N), device=dev, dtype=dtype)
    y4 = K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU_D, aux_out=d)
    r64 = ref.clone().requires_grad_(True)
    gref = torch.autograd.grad(torch.nn.functional.gelu(r64).sum(), r64)[0]
    assert (y4.double() - torch.nn.functional.gelu(ref)).abs().max().item() < tol * 4
    assert (d.double() - gref).abs().max().item() < tol * 4
    y5 = K.linear_fwd(x, w, bias, epilogue=K.EPI_GELU)   # no aux_out: gelu only
    assert (y5.double() - torch.nn.functional.gelu(ref)).abs().max().item() < tol * 4
    dx5 = K.linear_dgrad(dy, w, epilogue=K.EPI_MUL_AUX, aux=aux, out_dtype=torch.float32, resid=resid[:, :Kd].contiguous())
    ref5 = _ref_mm(dy, w) * aux.double() + resid[:, :Kd].double()
    assert (dx5.double() - ref5).abs().max().item() < tol * 4 * max(1.0, ref5.abs().max().item() / 4)
    # wgrad
    dW = K.linear_wgrad(dy, x)
    assert (dW.double() - _ref_mm(dy.t(), x)).abs().max().item() / _ref_mm(dy.t(), x).abs().max().item() < 1e-4


def _attn_ref(qkv, B, n, H, hd, scale, key_mask=None):
    q, k, v = qkv.double().view(B, n, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    if key_mask is not None:
        s = s.masked_fill(key_mask.view(B, 1, 1, n) == 0, float("-inf"))
    p = s.softmax(-1)
    return (p @ v).transpose(1, 2).reshape(B * n, H * hd)


@pytest.mark.parametrize("mode", ["four", "two", "two3", "diag", "bw16", "rows"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 50, 3, 64), (2, 197, 2, 64), (2, 37, 4, 32), (3, 5, 2, 32), (1, 130, 2, 64),
                                   (1, 197, 2, 32), (1, 256, 2, 64), (2, 224, 2, 32), (1, 577, 2, 32),
                                   (2, 145, 2, 64), (2, 256, 2, 32)])
def test_attention_fwd_bwd(dev, dtype, shape, mode, opts):
    """fp32 parity mode holds two [n][hd] f32 images at a time in the
    backward, so the C1 encoder (n = 197, hd = 64) runs in fp32 as well. bf16
    backward variants: four LDS images ("four"), two images with K/V (phase 1)
    and Q/dO (phase 2) tiles from HBM ("two", picked when it fits more
    workgroups per CU; "two3": its 3-workgroups-per-CU register budget at
    hd = 32), one-pass diagonal schedule with dQ accumulated in LDS ("diag": bf16, n <= 256 at
    hd = 32, n <= 224 at hd = 64; the default there). fp32 beyond its LDS images (n = 577, the C4
    decoder) streams 64-row blocks through LDS ("rows"; forced here at every
    shape, picked by itself at n = 577 in "four"); "bw16": the two-image
    layout with up to 16 waves (bf16, more than 8 16-row tiles; the default at
    hd = 32 beyond the diagonal kernel, forced here at hd 64 too)."""
    B, n, H, hd = shape
    if dtype == torch.float32 and mode not in ("four", "rows"):
        pytest.skip("fp32 parity mode: MFMA kernel (two images) or the rows path")
    if dtype == torch.bfloat16 and mode == "rows":
        pytest.skip("rows path: fp32 parity mode only")
    opts(ATTN_ROWS=1 if mode == "rows" else 0)
    if mode == "diag" and (dtype == torch.float32 or n > (256 if hd == 32 else 224)):
        pytest.skip("diagonal backward: bf16, n <= 256 at hd 32, n <= 224 at hd 64")
    opts(ATTN_DIAG=1 if mode == "diag" else 0)
    if mode == "bw16" and (dtype == torch.float32 or n <= 128):
        pytest.skip("16-wave backward: bf16 with more than 8 16-row tiles")
    opts(ATTN_BW16=1 if mode == "bw16" else 0)
    opts(ATTN_TWO={"two": 1, "two3": 3}.get(mode, 0))
    scale = hd ** -0.5
    qkv = _rand((B * n, 3 * H * hd), dtype, dev, seed=11)
    o, lse = K.attn_fwd(qkv, B, n, H, hd, scale)
    ref = _attn_ref(qkv, B, n, H, hd, scale)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert (o.double() - ref).abs().max().item() < tol
    # backward vs autograd fp64
    dout = _rand((B * n, H * hd), dtype, dev, seed=12)
    dqkv, part = K.attn_bwd(qkv, o, dout, lse, B, n, H, hd, scale)
    x64 = qkv.double().detach().requires_grad_(True)
    r = _attn_ref(x64, B, n, H, hd, scale)
    (r * dout.double()).sum().backward()
    g = x64.grad
    gs = g.abs().max().item()
    tolb = 1e-4 if dtype == torch.float32 else 3e-2
    assert (dqkv.double() - g).abs().max().item() / gs < tolb
    cs = part.sum(0)
    gsum = g.view(B * n, 3, H * hd).sum(0)
    assert (cs.double() - gsum.view(-1)).abs().max().item() / (gs * n) < tolb
    # the identities the bias partials use: sum over keys of dK is zero (softmax
    # is invariant to a per-query constant), sum over keys of dV = sum of dO
    assert gsum[1].abs().max().item() < 1e-9 * gs * n
    assert (cs.view(3, -1)[1] == 0).all()
    assert (cs.view(3, -1)[2].double() - dout.double().sum(0)).abs().max().item() < 1e-4 * max(1.0, n ** 0.5)


def test_attention_key_mask(dev):
    B, n, H, hd = 3, 25, 4, 64
    qkv = _rand((B * n, 3 * H * hd), torch.bfloat16, dev, seed=13)
    km = torch.ones((B, n), device=dev)
    km[1, 10:] = 0
    km[2, 3:] = 0
    o, _ = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5, key_mask=km)
    ref = _attn_ref(qkv, B, n, H, hd, hd ** -0.5, key_mask=km)
    assert (o.double() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("rows", [False, True])
def test_attention_key_mask_f32(dev, rows, opts):
    """fp32 parity mode with DistilBERT's key-padding mask, MFMA kernel and the
    long-sequence rows path; the backward of the rows path honours the mask too."""
    opts(ATTN_ROWS=1 if rows else 0)
    B, n, H, hd = 3, 70, 2, 64
    qkv = _rand((B * n, 3 * H * hd), torch.float32, dev, seed=14)
    km = torch.ones((B, n), device=dev)
    km[1, 10:] = 0
    km[2, 65:] = 0
    o, lse = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5, key_mask=km)
    ref = _attn_ref(qkv, B, n, H, hd, hd ** -0.5, key_mask=km)
    assert (o.double() - ref).abs().max().item() < 2e-5
    if rows:
        dout = _rand((B * n, H * hd), torch.float32, dev, seed=15)
        dqkv, _ = K.attn_bwd(qkv, o, dout, lse, B, n, H, hd, hd ** -0.5, key_mask=km)
        x64 = qkv.double().detach().requires_grad_(True)
        (_attn_ref(x64, B, n, H, hd, hd ** -0.5, key_mask=km) * dout.double()).sum().backward()
        assert (dqkv.double() - x64.grad).abs().max().item() / x64.grad.abs().max().item() < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm(dev, dtype):
    M, D = 333, 768
    x = _rand((M, D), torch.float32, dev, seed=21) * 3 + 1
    res = _rand((M, D), torch.float32, dev, seed=22)
    g = _rand((D,), torch.float32, dev, seed=23)
    b = _rand((D,), torch.float32, dev, seed=24)
    y, mean, rstd, yb, xs = K.ln_fwd(x, g, b, 1e-6, out_dtype=dtype, res=res, y2=True, xsum=True)
    xr = (x + res).double()
    ref = torch.nn.functional.layer_norm(xr, (D,), g.double(), b.double(), 1e-6)
    rel = 1e-6 if dtype == torch.float32 else 2 ** -8  # bf16 output rounding
    assert ((y.double() - ref).abs() - rel * ref.abs()).max().item() < 1e-4
    assert (xs.double() - xr).abs().max().item() < 1e-5
    dy = _rand((M, D), torch.float32, dev, seed=25)
    dres = _rand((M, D), torch.float32, dev, seed=26)
    dx, dxb, pg, pb, pc = K.ln_bwd(dy, xs, mean, rstd, g, dres=dres, want_bf16=True, want_colsum=True)
    x64 = xr.clone().requires_grad_(True)
    g64 = g.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    out = torch.nn.functional.layer_norm(x64, (D,), g64, b64, 1e-6)
    (out * dy.double()).sum().backward()
    assert (dx.double() - (x64.grad + dres.double())).abs().max().item() < 1e-3
    assert (K.colsum_reduce(pg).double() - g64.grad).abs().max().item() < 1e-2
    assert (K.colsum_reduce(pb).double() - b64.grad).abs().max().item() < 1e-2
    assert (K.colsum_reduce(pc).double() - dx.double().sum(0)).abs().max().item() < 1e-2


def _clip_ref64(I, T, tau):
    """CLIP.py:34-43 + cross_entropy (CLIP.py:46-52) in fp64 autograd."""
    I64 = I.detach().double().cpu().requires_grad_(True)
    T64 = T.detach().double().cpu().requires_grad_(True)
    logits = T64 @ I64.T / tau
    tgt = torch.softmax((I64 @ I64.T + T64 @ T64.T) / 2 * tau, -1)
    lt = (-tgt * torch.log_softmax(logits, -1)).sum(1)
    li = (-tgt.T * torch.log_softmax(logits.T, -1)).sum(1)
    ref = ((li + lt) / 2).mean()
    ref.backward()
    return ref.item(), I64.grad, T64.grad


@pytest.mark.parametrize("N", [1, 3, 5, 7, 8, 64, 100, 256, 1024, 2048, 2500, 4100])
@pytest.mark.parametrize("tau", [1.0, 0.5])
def test_clip_loss_kernel_vs_torch(dev, N, tau):
    """Fused CLIP loss (no N x N in HBM) vs fp64 autograd of the reference
    formula, any N (the reference DataLoader keeps the last partial batch,
    main.py:42-47), LayerNorm'd 256-d embeddings as the projection heads emit."""
    I = torch.nn.functional.layer_norm(_rand((N, 256), torch.float32, dev, seed=31 + N), (256,))
    T = torch.nn.functional.layer_norm(_rand((N, 256), torch.float32, dev, seed=32 + N), (256,))
    loss, dI, dT = K.clip_loss(I, T, tau)
    ref, gI, gT = _clip_ref64(I, T, tau)
    assert abs(loss.item() - ref) < 1e-5 * max(1.0, abs(ref)), (loss.item(), ref)
    sc = max(gI.abs().max().item(), gT.abs().max().item(), 1e-30)   # N = 1: loss and gradient are exactly 0
    assert (dI.double().cpu() - gI).abs().max().item() <= 1e-4 * sc
    assert (dT.double().cpu() - gT).abs().max().item() <= 1e-4 * sc
    # deterministic: fixed-order partials, bit-identical on a second call
    loss2, dI2, dT2 = K.clip_loss(I, T, tau)
    assert torch.equal(loss, loss2) and torch.equal(dI, dI2) and torch.equal(dT, dT2)


@pytest.mark.parametrize("N,rows", [(2048, (256, 256)), (1024, (896, 128)), (100, (37, 50)), (256, (0, 256)),
                                    (2500, (2100, 400)), (4100, (0, 2048)), (4100, (4000, 100))])
def test_clip_loss_gradient_rows(dev, N, rows):
    """Data-parallel form: every rank evaluates the loss of the gathered batch
    and asks for the gradient of its own row slice only -- equal to that slice
    of the full gradient, loss identical; no-grad path and per-row losses."""
    I = torch.nn.functional.layer_norm(_rand((N, 256), torch.float32, dev, seed=7), (256,))
    T = torch.nn.functional.layer_norm(_rand((N, 256), torch.float32, dev, seed=8), (256,))
    lf, dIf, dTf = K.clip_loss(I, T, 1.0)
    ls, dIs, dTs = K.clip_loss(I, T, 1.0, grad_rows=rows)
    r0, nr = rows
    assert torch.equal(lf, ls)
    assert torch.allclose(dIs, dIf[r0:r0 + nr], rtol=0, atol=1e-6 * dIf.abs().max().item())
    assert torch.allclose(dTs, dTf[r0:r0 + nr], rtol=0, atol=1e-6 * dTf.abs().max().item())
    ln, _, _, rl = K.clip_loss(I, T, 1.0, want_grad=False, row_loss=True)
    assert torch.equal(ln, lf)
    assert abs(rl.double().sum().item() - lf.item()) < 1e-5 * max(1.0, abs(lf.item()))


def test_clip_loss_p128_and_strided(dev):
    """projection_dim 128 and row-strided inputs (views into a wider buffer)."""
    N = 40
    big = torch.nn.functional.layer_norm(_rand((N, 256), torch.float32, dev, seed=9), (256,))
    I, T = big[:, :128], big[:, 128:]
    loss, dI, dT = K.clip_loss(I, T, 1.0)
    ref, gI, gT = _clip_ref64(I, T, 1.0)
    assert abs(loss.item() - ref) < 1e-5 * max(1.0, abs(ref))
    sc = max(gI.abs().max().item(), gT.abs().max().item())
    assert (dI.double().cpu() - gI).abs().max().item() < 1e-4 * sc


def test_mask_ids_golden_fixture(dev):
    """maeclip_mask_ids on the GPU vs tests/golden/masking.npz (HF ViTMAE
    random_masking run on the same counter-based noise: B=32, L=196, keep 49,
    seed 2, step 3): noise bits, ids_keep, ids_restore and mask bit-exact."""
    import numpy as np
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "masking.npz"))
    B, L_ = z["noise"].shape
    keep = z["ids_keep"].shape[1]
    ids_s, ids_r, mask, noise = K.mask_ids(B, L_, keep, seed=2, step=3, sample_offset=0, device=dev, want_noise=True)
    assert np.array_equal(noise.cpu().numpy().view(np.uint32), z["noise"].view(np.uint32))
    assert np.array_equal(ids_s[:, :keep].cpu().long().numpy(), z["ids_keep"])
    assert np.array_equal(ids_r.cpu().long().numpy(), z["ids_restore"])
    assert np.array_equal(mask.cpu().numpy(), z["mask"])


def test_mask_ids_with_tied_keys(dev):
    """A mask step whose 24-bit keys tie inside a sample (step 20 of seed 2 at
    B=32, L=196; P(tie) ~ 1.1e-3 per sample): the GPU ids equal the
    oracle's stable argsort (lower patch index first) bit for bit."""
    import numpy as np
    from oracle import maskrng
    from oracle.ref_model import random_masking_ids
    B, L_, keep, step = 32, 196, 49, 20
    k = maskrng.keys24(2, step, 0, B, L_)
    assert any(len(np.unique(r)) < r.size for r in k)
    ids_s, ids_r, mask, _ = K.mask_ids(B, L_, keep, seed=2, step=step, sample_offset=0, device=dev)
    r_s, r_r, r_m = random_masking_ids(torch.from_numpy(maskrng.noise(2, step, 0, B, L_)), keep)
    assert torch.equal(ids_s.cpu().long(), r_s)
    assert torch.equal(ids_r.cpu().long(), r_r)
    assert torch.equal(mask.cpu(), r_m.float())


def test_dropout_statistics(dev):
    """nn.Dropout semantics of the library's counter-based masks (ProjectionHead
    p=0.1, modules.py:66,73; DistilBERT hidden/attention dropout p=0.1):
    drop rate within 5 sigma of p, kept values scaled by 1/(1-p), masks
    deterministic for a seed and fresh for every device step."""
    p = 0.1
    M, D = 4096, 256
    x = torch.ones((M, D), device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    y1 = K.dropout(x, p, seed=5, step_ptr=step)
    y1b = K.dropout(x, p, seed=5, step_ptr=step)
    K.counter_add(step, 1)
    y2 = K.dropout(x, p, seed=5, step_ptr=step)
    n = M * D
    sig = (p * (1 - p) / n) ** 0.5
    for y in (y1, y2):
        frac = (y == 0).float().mean().item()
        assert abs(frac - p) < 5 * sig, frac
        kept = y[y != 0]
        assert torch.allclose(kept, torch.full_like(kept, 1 / (1 - p)))
    assert torch.equal(y1, y1b)
    assert not torch.equal(y1, y2)
    # LayerNorm input dropout (ProjectionHead: dropout(fc(.)) + residual, fused in the LN launch)
    gamma, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    _, _, _, _, xs = K.ln_fwd(x, gamma, beta, 1e-5, out_dtype=torch.float32, res=torch.zeros_like(x),
                              in_dropout=p, seed_in=9, xsum=True, step_ptr=step)
    frac = (xs == 0).float().mean().item()
    assert abs(frac - p) < 5 * sig, frac
    # attention-probability dropout (DistilBERT attention.dropout): q = k = 0 gives
    # uniform p_k = 1/n, V rows one-hot, so O[q, k] = mask(q, k) / (n (1 - p))
    B, n, H, hd = 64, 25, 1, 32
    qkv = torch.zeros((B * n, 3 * H * hd), device=dev)
    qkv.view(B, n, 3 * hd)[:, :, 2 * hd:2 * hd + n] = torch.eye(n, device=dev)
    o, _ = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5, dropout_p=p, seed=3, want_lse=False, step_ptr=step)
    oo = o.view(B, n, hd)[:, :, :n]
    nz = oo[oo != 0]
    assert torch.allclose(nz, torch.full_like(nz, 1 / (n * (1 - p))), rtol=1e-5)
    frac = (oo == 0).float().mean().item()
    sig2 = (p * (1 - p) / oo.numel()) ** 0.5
    assert abs(frac - p) < 5 * sig2, frac


def test_mask_ids_is_stable_argsort(dev):
    B, L_, keep = 16, 196, 49
    ids_s, ids_r, mask, noise = K.mask_ids(B, L_, keep, seed=2, step=5, sample_offset=0, device=dev, want_noise=True)
    ref_s = torch.argsort(noise.cpu(), dim=1, stable=True)
    assert torch.equal(ids_s.cpu().long(), ref_s)
    assert torch.equal(ids_r.cpu().long(), torch.argsort(ref_s, dim=1))
    m = torch.ones(B, L_)
    m[:, :keep] = 0
    assert torch.equal(mask.cpu(), torch.gather(m, 1, ids_r.cpu().long()))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_wgrad_splitk(dev, dtype):
    M, N, Kd = 20000, 256, 136   # long token dim -> split-K (deterministic slab reduce)
    dy = _rand((M, N), dtype, dev, seed=41)
    x = _rand((M, Kd), dtype, dev, seed=42)
    from mae_clip_amd import _lib
    assert _lib.lib().maeclip_gemm_splitk(N, Kd, M) > 1
    dW = K.linear_wgrad(dy, x)
    ref = _ref_mm(dy.t(), x)
    assert (dW.double() - ref).abs().max().item() / ref.abs().max().item() < 1e-5
    dW2 = K.linear_wgrad(dy, x)
    assert torch.equal(dW, dW2)  # deterministic


@pytest.mark.parametrize("mnk", [(12800, 768, 768), (4096, 512, 2048), (3200, 2304, 768)])
def test_wgrad_splitk_v4(dev, mnk):
    """Production wgrad shapes (bf16, token dim % 64 == 0, >= 256x256 output):
    the v4 kernel's split-K slabs + deterministic splitk_reduce."""
    M, N, Kd = mnk
    from mae_clip_amd import _lib
    assert _lib.lib().maeclip_gemm_splitk(N, Kd, M) > 1
    dy = _rand((M, N), torch.bfloat16, dev, seed=44)
    x = _rand((M, Kd), torch.bfloat16, dev, seed=45)
    dW = K.linear_wgrad(dy, x)
    ref = _ref_mm(dy.t(), x)
    assert (dW.double() - ref).abs().max().item() / ref.abs().max().item() < 1e-5
    dW2 = K.linear_wgrad(dy, x)
    assert torch.equal(dW, dW2)


@pytest.mark.parametrize("case", ["encoder4", "decoder2x4", "few_tiles_splitk", "strided", "fp32_fallback",
                                  "whole_plus_streamk", "uniform_slices"])
def test_wgrad_grouped(dev, case, opts):
    """maeclip_wgrad_grouped: the 4 weight gradients of transformer blocks
    (qkv, proj, fc1, fc2) in one launch vs fp64 torch; stream-K remainder
    (fewer tiles than CUs; whole tiles + a remainder dealt out by K-tiles, with
    edge tiles in both parts), uniform split-K slices (MAECLIP_WG_SK=0, and too
    little K for stream-K), strided dy (a column slice), beta accumulation, the
    per-problem fallback for fp32 -- bit-identical across repeated runs."""
    from mae_clip_amd import _lib
    dt = torch.float32 if case == "fp32_fallback" else torch.bfloat16
    if case in ("encoder4", "strided", "fp32_fallback"):
        M, shapes = 3200, [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    elif case in ("decoder2x4", "uniform_slices"):
        M, shapes = 6400, [(1536, 512), (512, 512), (2048, 512), (512, 2048)] * 2
        if case == "uniform_slices":
            opts(WG_SK=0)
    elif case == "whole_plus_streamk":
        # 144 + 108 + 132 = 384 tiles: 256 whole, 128 (2600-row edge tiles among
        # them) over the grid by K-tiles
        M, shapes = 2048, [(3072, 3072), (3072, 2056), (2600, 3072)]
    else:
        M, shapes = 4096, [(512, 256), (256, 512)]   # 4 tiles -> split-K slices
    items, refs = [], []
    for i, (N, Kd) in enumerate(shapes):
        if case == "strided":
            dy = _rand((M, N + 64), dt, dev, seed=60 + i)[:, 32:32 + N]
        else:
            dy = _rand((M, N), dt, dev, seed=60 + i)
        x = _rand((M, Kd), dt, dev, seed=80 + i)
        out = torch.empty((N, Kd), device=dev, dtype=torch.float32)
        items.append((dy, x, out))
        refs.append(_ref_mm(dy.t(), x))
    if case == "few_tiles_splitk":
        probs = (_lib.WgradProblem * 2)()
        for q, (dy, x, out) in zip(probs, items):
            q.dy, q.x, q.dw, q.N, q.K, q.ldy, q.ldx = dy.data_ptr(), x.data_ptr(), out.data_ptr(), dy.shape[1], \
                x.shape[1], dy.stride(0), x.stride(0)
        assert _lib.lib().maeclip_wgrad_grouped_workspace(probs, 2, M, 1) > 0
    K.wgrad_grouped(items)
    for (dy, x, out), ref in zip(items, refs):
        assert (out.double() - ref).abs().max().item() / ref.abs().max().item() < 1e-5
    first = [o.clone() for _, _, o in items]
    K.wgrad_grouped(items)
    for (_, _, out), f in zip(items, first):
        assert torch.equal(out, f)
    K.wgrad_grouped(items, beta=1.0)      # dW += dy^T x
    for (dy, x, out), ref in zip(items, refs):
        assert (out.double() - 2 * ref).abs().max().item() / ref.abs().max().item() < 1e-5


def test_colsum_two_pass(dev):
    part = _rand((1000, 768), torch.float32, dev, seed=43)
    out = K.colsum_reduce(part)
    assert (out.double() - part.double().sum(0)).abs().max().item() < 1e-3


@pytest.mark.parametrize("P", [7, 4096, 4097, 50176, 200003])
def test_vector_sum_two_level(dev, P):
    """N == 1 (the MAE loss's per-patch rows): grid-wide pass 1 + one-block
    pass 2, fixed order (bitwise reproducible), accumulate and scale."""
    x = _rand((P, 1), torch.float32, dev, seed=44)
    out = K.colsum_reduce(x, scale=0.5)
    ref = x.double().sum().item() * 0.5
    assert abs(out.item() - ref) < 1e-5 * max(1.0, x.double().abs().sum().item())
    assert torch.equal(out, K.colsum_reduce(x, scale=0.5))
    acc = torch.full((1,), 3.0, device=dev)
    K.colsum_reduce(x, out=acc, accumulate=True, scale=0.5)
    assert abs(acc.item() - (3.0 + ref)) < 1e-5 * max(1.0, x.double().abs().sum().item())


@pytest.mark.parametrize("shape", [(4, 224, 224), (3, 32, 30), (2, 336, 336), (1, 7, 5)])
def test_image_normalize_u8_bit_exact(dev, shape):
    """Device input pipeline (dataset.py:49, 34): uint8 HWC -> normalised fp32
    NCHW, bit-exact vs the numpy restatement of albumentations' normalize()."""
    import numpy as np
    from mae_clip_amd.data import normalize_u8
    from oracle.input_ref import normalize_u8_ref
    g = torch.Generator().manual_seed(sum(shape))
    imgs = torch.randint(0, 256, shape + (3,), generator=g, dtype=torch.uint8)
    imgs[0, 0, 0] = torch.tensor([0, 255, 128], dtype=torch.uint8)
    out = normalize_u8(imgs.to(dev)).cpu().numpy()
    ref = normalize_u8_ref(imgs.numpy())
    assert out.shape == ref.shape and out.dtype == np.float32
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("QNk", [(1, 6000, 45), (3, 1000, 7), (2, 300, 300), (1, 1001, 45), (2, 9, 9), (1, 7, 3)])
def test_retrieval_normalize_similarity_topk(dev, QNk):
    """inference.py:40-45 on the device: F.normalize, text_n @ image_n.T, topk
    (values within fp32 rounding of the fp64 reference; indices equal to the
    reference order, value descending / index ascending, with planted ties)."""
    from mae_clip_amd.retrieval import l2_normalize, similarity, topk_rows
    Q, N, k = QNk
    t = _rand((Q, 256), torch.float32, dev, seed=91)
    im = _rand((N, 256), torch.float32, dev, seed=92)
    im[min(5, N - 1)] = im[3 % N]   # exact duplicate candidates -> tied scores
    im[N // 2] = 0.0                # zero row: F.normalize's eps clamp
    n = l2_normalize(im)
    ref_n = torch.nn.functional.normalize(im.double(), p=2, dim=-1)
    assert (n.double() - ref_n).abs().max().item() < 1e-6
    s = similarity(t, im)
    ref_s = torch.nn.functional.normalize(t.double(), dim=-1) @ ref_n.T
    assert (s.double() - ref_s).abs().max().item() < 1e-5
    vals, idx = topk_rows(s, k)
    sc = s.double().cpu()
    for q in range(Q):
        order = sorted(range(N), key=lambda i: (-sc[q, i].item(), i))[:k]
        assert idx[q].tolist() == order
        assert torch.equal(vals[q].cpu(), s[q].cpu()[idx[q].cpu()])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", [(4, 224, 16, False), (3, 224, 16, True), (2, 336, 14, False), (2, 32, 8, True)])
def test_mae_loss_kernels_vs_torch(dev, dtype, cfg):
    """HF ViTMAE forward_loss (modeling_vit_mae.py:852-859) over patchify
    (:706-745) on the fused kernels: per-patch loss rows and the gradient of
    the scaled mean, incl. norm_pix and the padded pred rows of patch 14
    (P = 588 in a 640-wide row; dpred pad columns must come back zero)."""
    from oracle.ref_model import patchify
    B, S, p, norm_pix = cfg
    L_ = (S // p) ** 2
    P = 3 * p * p
    ldp = (P + 63) // 64 * 64
    keep = L_ // 4
    img = _rand((B, 3, S, S), torch.float32, dev, seed=51)
    pred_full = _rand((B * (L_ + 1), ldp), dtype, dev, seed=52)
    _, _, mask, _ = K.mask_ids(B, L_, keep, seed=2, step=7, sample_offset=0, device=dev)
    row = K.mae_loss_fwd(pred_full, img, mask, p, norm_pix)
    tgt = patchify(img.double().cpu(), p)
    if norm_pix:
        mean = tgt.mean(-1, keepdim=True)
        var = tgt.var(-1, keepdim=True)
        tgt = (tgt - mean) / (var + 1e-6) ** 0.5
    pr = pred_full.double().cpu().view(B, L_ + 1, ldp)[:, 1:, :P].clone().requires_grad_(True)
    ref_row = ((pr - tgt) ** 2).mean(-1) * mask.double().cpu()
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    assert (row.double().cpu().view(B, L_) - ref_row).abs().max().item() < tol * ref_row.abs().max().item() + 1e-6
    mc = float(mask.sum().item())
    gl = torch.tensor(0.7, device=dev)
    dpred, cs = K.mae_loss_bwd(pred_full, img, mask, p, norm_pix, gl, mc, loss_scale=0.5)
    (ref_row.sum() / mc * 0.5 * 0.7).backward()
    d = dpred.double().cpu().view(B, L_ + 1, ldp)
    gs = pr.grad.abs().max().item()
    tolg = 1e-5 if dtype == torch.float32 else 1e-2
    assert (d[:, 1:, :P] - pr.grad).abs().max().item() < tolg * gs
    assert torch.count_nonzero(d[:, 0]) == 0 and torch.count_nonzero(d[:, :, P:]) == 0
    # bias-gradient partials are summed from the fp32 values (before dpred's rounding)
    assert (cs.double().cpu().sum(0) - pr.grad.sum((0, 1))).abs().max().item() < tolg * gs * L_


@pytest.mark.parametrize("B", [16, 300])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tokens_and_unshuffle_bwd_vs_torch(dev, dtype, B):
    """timm _pos_embed / PatchEmbed backward on the visible tokens and the HF
    decoder unshuffle backward (modeling_vit_mae.py:548-566): gathered rows
    exact, position / mask-token / bias partial sums vs fp64 (B = 300: more
    samples than one 256-sample ballot chunk of tokens_bwd_pos, ragged tail)."""
    L_, keep, D, Dd = 196, 49, 768, 512
    ids_s, ids_r, mask, _ = K.mask_ids(B, L_, keep, seed=2, step=1, sample_offset=0, device=dev)
    dx = _rand((B, keep + 1, D), torch.float32, dev, seed=61)
    dy, dpos, dcls = K.tokens_bwd(dx, ids_r, B, L_, keep, dtype)
    assert torch.equal(dy.float().view(B, keep, D).cpu(), dx[:, 1:].to(dtype).float().cpu())
    ref = torch.zeros(L_ + 1, D, dtype=torch.float64)
    x64 = dx.double().cpu()
    ref[0] = x64[:, 0].sum(0)
    s = ids_s.cpu().long()
    for b in range(B):
        ref[1 + s[b, :keep]] += x64[b, 1:]
    assert (dpos.double().cpu() - ref).abs().max().item() < 1e-4
    assert torch.equal(dcls, dpos[0])
    dout = _rand((B, L_ + 1, Dd), torch.float32, dev, seed=62)
    dy2, dmask, cs = K.unshuffle_bwd(dout, ids_r, B, L_, keep, dtype)
    o64 = dout.double().cpu()
    r = ids_r.cpu().long()
    ref_dy = torch.zeros(B, keep + 1, Dd, dtype=torch.float64)
    ref_dy[:, 0] = o64[:, 0]
    ref_dm = torch.zeros(Dd, dtype=torch.float64)
    for b in range(B):
        kept = r[b] < keep
        ref_dy[b, 1 + r[b][kept]] = o64[b, 1:][kept]
        ref_dm += o64[b, 1:][~kept].sum(0)
    assert torch.equal(dy2.float().view(B, keep + 1, Dd).cpu(), ref_dy.float().to(dtype).float())
    assert (dmask.double().cpu().sum(0) - ref_dm).abs().max().item() < 1e-3
    assert (cs.double().cpu().sum(0) - ref_dy.sum((0, 1))).abs().max().item() < 1e-3


@pytest.mark.parametrize("B", [129, 300])
@pytest.mark.parametrize("D", [64, 192, 384, 1024])
def test_tokens_bwd_pos_narrow_rows(dev, D, B):
    """pos_embed / cls_token gradients when D/4 is not a multiple of 64: the
    lanes past the last column still cast their sample's ballot vote (a lane
    is both a column chunk and a sample of the restore-index ballot), so no
    sample is dropped from dpos for ViT-Tiny / ViT-S widths."""
    L_, keep = 196, 49
    ids_s, ids_r, _, _ = K.mask_ids(B, L_, keep, seed=3, step=2, sample_offset=0, device=dev)
    dx = _rand((B, keep + 1, D), torch.float32, dev, seed=63)
    _, dpos, dcls = K.tokens_bwd(dx, ids_r, B, L_, keep, torch.bfloat16)
    x64 = dx.double().cpu()
    ref = torch.zeros(L_ + 1, D, dtype=torch.float64)
    ref[0] = x64[:, 0].sum(0)
    s = ids_s.cpu().long()
    for b in range(B):
        ref[1 + s[b, :keep]] += x64[b, 1:]
    assert (dpos.double().cpu() - ref).abs().max().item() < 1e-4
    assert torch.equal(dcls, dpos[0])



def test_image_preprocess_resize_bit_exact(dev):
    """maeclip_image_preprocess_u8 (A.Resize INTER_LINEAR + A.Normalize +
    permute, dataset.py:44-58 / :34) vs the numpy restatement of OpenCV's
    fixed-point uint8 resize (oracle/input_ref.py): bit-exact fp32 output for
    up- and down-scales, non-square and odd sizes, the equal-size copy, the exact
    2x INTER_AREA case and a row-strided (cropped) source."""
    import numpy as np
    from mae_clip_amd.data import preprocess_images
    from oracle.input_ref import preprocess_ref
    rng = np.random.default_rng(5)
    S = 224
    shapes = [(375, 500), (224, 224), (448, 448), (100, 37), (1, 1), (225, 223), (640, 427)]
    ims = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    big = torch.from_numpy(rng.integers(0, 256, (300, 400, 3), dtype=np.uint8)).to(dev)
    crop = big[10:260, 20:330]                      # row stride 1200 B, not 3 * 310
    dev_ims = [torch.from_numpy(im).to(dev) for im in ims] + [crop]
    out = preprocess_images(dev_ims, S).cpu().numpy()
    ref = preprocess_ref(ims + [crop.cpu().numpy()], S)
    assert out.shape == (len(dev_ims), 3, S, S)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("shape", [(64, 50, 12, 64), (8, 197, 16, 32), (4, 197, 12, 64), (16, 25, 12, 64),
                                   # production grids of the kernels that order their waves with
                                   # per-wave LDS flags (many co-resident workgroups per CU):
                                   (256, 197, 16, 32),    # C2 decoder: diagonal backward, 4096 workgroups
                                   (128, 197, 16, 32),    # C2 decoder micro-batch
                                   (256, 197, 12, 64),    # C1 encoder: hd-64 diagonal backward at n = 197
                                   (128, 577, 16, 32)])   # C4 decoder: 16-wave forward and backward
def test_attention_deterministic(dev, shape):
    """fwd and bwd are bitwise reproducible (no atomics; fixed reduction order),
    also at the full production grids where the diagonal backward's waves
    drift apart by up to a round between their flag waits."""
    B, n, H, hd = shape
    qkv = _rand((B * n, 3 * H * hd), torch.bfloat16, dev, seed=31)
    dout = _rand((B * n, H * hd), torch.bfloat16, dev, seed=32)
    runs = []
    for _ in range(3):
        o, lse = K.attn_fwd(qkv, B, n, H, hd, hd ** -0.5)
        dq, part = K.attn_bwd(qkv, o, dout, lse, B, n, H, hd, hd ** -0.5)
        runs.append((o.clone(), lse.clone(), dq.clone(), part.clone()))
    for r in runs[1:]:
        for x, y in zip(r, runs[0]):
            assert torch.equal(x, y)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(6, 224, 16, 49), (3, 336, 14, 144), (4, 32, 8, 4), (2, 224, 16, 196)])
def test_uint8_pixels_fused_into_gather_and_mae_targets(dev, dtype, geo):
    """A.Normalize + permute (dataset.py:49, :34) folded
    into the patch gather and the MAE target read. Reading the uint8 HWC pixels
    directly must give the SAME bits as normalize_u8 (the materialised fp32
    NCHW image, itself bit-exact vs the numpy restatement) + the fp32 kernels:
    gathered rows, per-patch losses (norm_pix off / on) and dpred."""
    from mae_clip_amd.data import normalize_u8
    B, S, p, keep = geo
    L_ = (S // p) ** 2
    g = torch.Generator().manual_seed(71)
    px = torch.randint(0, 256, (B, S, S, 3), generator=g, dtype=torch.uint8).to(dev)
    img = normalize_u8(px)
    ids_s, _, mask, _ = K.mask_ids(B, L_, keep, seed=2, step=5, sample_offset=0, device=dev)
    kpad = (3 * p * p + 63) // 64 * 64
    a = K.patch_gather(px, ids_s, keep, p, kpad, dtype)
    b = K.patch_gather(img, ids_s, keep, p, kpad, dtype)
    assert torch.equal(a, b)
    P = 3 * p * p
    ldp = (P + 63) // 64 * 64
    pred = _rand((B * (L_ + 1), ldp), dtype, dev, seed=72)
    gl = torch.tensor(0.3, device=dev)
    if keep == L_:
        return   # mask ratio 0 (C1): no MAE targets
    for norm_pix in (False, True):
        assert torch.equal(K.mae_loss_fwd(pred, px, mask, p, norm_pix), K.mae_loss_fwd(pred, img, mask, p, norm_pix))
        d1, c1 = K.mae_loss_bwd(pred, px, mask, p, norm_pix, gl, float(mask.sum().item()))
        d2, c2 = K.mae_loss_bwd(pred, img, mask, p, norm_pix, gl, float(mask.sum().item()))
        assert torch.equal(d1, d2) and torch.equal(c1, c2)


@pytest.mark.parametrize("n", [1, 3, 5, 7, 1023, 4097, 65539])
@pytest.mark.parametrize("direction", ["f32_bf16", "bf16_f32"])
def test_cast_flat_odd_sizes(dev, n, direction):
    """maeclip_cast_flat (the bf16 gradient all-reduce's bucket casts) at odd
    sizes and vector tails, at an odd 16-B-aligned start offset inside a
    buffer (a bucket slice of the GradArena): RNE f32 -> bf16 like torch,
    exact bf16 -> f32, scale applied, nothing written past n."""
    torch.manual_seed(n)
    base = torch.randn(n + 8, device=dev) * 3.0
    if direction == "f32_bf16":
        src = base[4:4 + n]
        dst_buf = torch.full((n + 8,), 7.0, device=dev, dtype=torch.bfloat16)
        dst = dst_buf[4:4 + n]
        K.cast_flat(src, dst, scale=0.5)
        ref = (src * 0.5).to(torch.bfloat16)
    else:
        src = base.to(torch.bfloat16)[4:4 + n]
        dst_buf = torch.full((n + 8,), 7.0, device=dev)
        dst = dst_buf[4:4 + n]
        K.cast_flat(src, dst, scale=2.0)
        ref = src.float() * 2.0
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)
    assert (dst_buf[:4] == 7.0).all() and (dst_buf[4 + n:] == 7.0).all()


def test_small_step_kernels(dev):
    """ABI v6 step helpers that replace torch kernels inside the captured step:
    the counter snapshot, the loss combination and the scaling of stored
    gradients by a device grad_output; the embedding launch's mask convert."""
    c = torch.tensor([41], device=dev, dtype=torch.int64)
    snap = torch.zeros(3, device=dev, dtype=torch.int64)
    K.counter_add_snap(c, snap[1:2], 1)
    assert c.item() == 42 and snap.tolist() == [0, 41, 0]
    a = torch.tensor(1.25, device=dev)
    b = torch.tensor(-3.5, device=dev)
    assert K.scalar_axpy(a, b, 0.5).item() == 1.25 - 1.75
    s = torch.tensor([0.75], device=dev)
    for n0, n1 in [(65536, 65536), (5, 0), (1023, 4097), (0, 3)]:
        x = torch.randn(n0, device=dev)
        y = torch.randn(n1, device=dev)
        ox, oy = K.scale_by_scalar(s, 2.0, x if n0 else None, y if n1 else None,
                                   out_x=None, out_y=None) if n0 and n1 else (None, None)
        if n0 and n1:
            assert torch.equal(ox, x * 1.5) and torch.equal(oy, y * 1.5)
        # in place
        x2, y2 = x.clone(), y.clone()
        K.scale_by_scalar(s, 1.0, x2 if n0 else None, y2 if n1 else None, x2 if n0 else None, y2 if n1 else None)
        assert torch.equal(x2, x * 0.75) and torch.equal(y2, y * 0.75)
    one = torch.empty((), device=dev)
    out, _ = K.scale_by_scalar(s, 4.0, out_x=one)
    assert out.item() == 3.0
    ids = torch.randint(0, 100, (3, 7), device=dev)
    word = torch.randn(100, 64, device=dev)
    pos = torch.randn(7, 64, device=dev)
    m = torch.randint(0, 2, (3, 7), device=dev)
    e, mf = K.embed_fwd(ids, word, pos, mask=m)
    assert torch.equal(mf, m.float())
    assert torch.equal(e, (word[ids] + pos[None]).reshape(21, 64))


def test_combined_loss_backward_matches_torch(dev):
    """CombineLossFn / ClipLossFn backward (device-scalar scaling kernels) ==
    torch autograd of clip + w * mae with a non-unit grad_output."""
    from mae_clip_amd import functions as Fn
    clip = torch.tensor(2.0, device=dev, requires_grad=True)
    mae = torch.tensor(0.5, device=dev, requires_grad=True)
    loss = Fn.CombineLossFn.apply(clip, mae, 0.3)
    assert abs(loss.item() - 2.15) < 1e-6
    loss.backward(torch.tensor(2.0, device=dev))
    assert clip.grad.item() == 2.0 and abs(mae.grad.item() - 0.6) < 1e-7
    I = torch.nn.functional.layer_norm(torch.randn(16, 256, device=dev), (256,)).requires_grad_()
    T = torch.nn.functional.layer_norm(torch.randn(16, 256, device=dev), (256,)).requires_grad_()
    l = Fn.ClipLossFn.apply(I, T, 1.0, None)
    l.backward(torch.tensor(3.0, device=dev))
    _, dI, dT = K.clip_loss(I.detach(), T.detach(), 1.0)
    assert torch.allclose(I.grad, 3.0 * dI, rtol=1e-6, atol=1e-9)
    assert torch.allclose(T.grad, 3.0 * dT, rtol=1e-6, atol=1e-9)


