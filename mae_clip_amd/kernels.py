"""Thin torch-tensor wrappers over the libmaeclip C-ABI (include/maeclip.h).

Every function launches on torch's current HIP stream, validates shapes on the
host and raises MaeClipNativeError on any failure. Nothing here computes on the
CPU: tensors must live on a ROCm device.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L

KC, RC = 0, 1
EPI_NONE, EPI_GELU, EPI_RESID, EPI_DGELU, EPI_GELU_D, EPI_MUL_AUX = 0, 1, 2, 3, 4, 5

# Optional instrumentation: LAUNCH_HOOK(key, flops, nbytes, launch_fn) wraps every
# GEMM launch and every grouped weight-gradient launch (bench.py brackets them
# with HIP events / timestamps on the current stream).
LAUNCH_HOOK = None


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return L.BF16
    if t.dtype == torch.float32:
        return L.F32
    raise TypeError(f"unsupported dtype {t.dtype}")


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.MaeClipNativeError("mae_clip_amd kernels need ROCm device tensors (no CPU fallback)")


def _call(name, *args):
    lib = L.lib()
    rc = getattr(lib, name)(*args)
    L.check(rc, name)


# ------------------------------------------------------------------ GEMM
_SCRATCH = {}
_SCRATCH_RETIRED = []
_STREAM_ALIAS = {}   # capture stream -> the stream its graph is replayed on


def alias_stream(capture_stream, replay_stream):
    """While a graph is captured on `capture_stream` (torch.cuda.graph's own
    stream), its GEMMs use the scratch of `replay_stream`, the stream the graph
    is later replayed on: eager launches and replays are ordered on it, so they
    can share one buffer, and the capture allocates (and zero-fills inside the
    graph) nothing. `replay_stream=None` removes the alias."""
    if replay_stream is None:
        _STREAM_ALIAS.pop(capture_stream, None)
    else:
        _STREAM_ALIAS[capture_stream] = replay_stream


def set_option(name: str, value) -> int:
    """Set one plan option of the library (include/maeclip.h maeclip_set_option;
    None / -1 = the built-in default); returns the previous value (-1: default).
    The library snapshots the MAECLIP_<name> environment once; later changes of
    the environment are not seen, this is the way to switch a plan at run time."""
    key = L.OPTIONS.index(name)
    return int(L.lib().maeclip_set_option(key, -1 if value is None else int(value)))


def get_option(name: str) -> int:
    return int(L.lib().maeclip_get_option(L.OPTIONS.index(name)))


class options:
    """Scope of plan options: `with K.options(GEMM_BM=192, GEMM_SPLIT=2): ...`
    sets them for the launches issued inside and restores the previous values."""

    def __init__(self, **kw):
        self.kw, self.prev = kw, {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.prev[k] = set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_option(k, v)
        return False


def gemm_split_scope(enabled=True):
    """Launches issued inside the scope may take maeclip_gemm's split plan
    (option GEMM_SK = 1); restores the previous setting on exit."""
    return options(GEMM_SK=1) if enabled else options()


def _stream_scratch(device, nbytes):
    """Per-(device, stream) scratch kept for the process (maeclip_gemm's
    stream-K counters and partial tiles): launches on one stream run in order
    and share it; a concurrently running stream gets its own. Allocated zeroed
    (the stream-K arrival counters at its start must be zero; every completed
    launch leaves them zero). A buffer outgrown by a larger request is kept
    alive, never freed: a captured HIP graph may still address it."""
    s = torch.cuda.current_stream(device).cuda_stream
    key = (device.index, _STREAM_ALIAS.get(s, s))
    t = _SCRATCH.get(key)
    if t is None or t.numel() * 4 < nbytes:
        if torch.cuda.is_current_stream_capturing():
            # a buffer made here would come from the graph's private pool with
            # its zero-fill baked into every replay: the eager steps before a
            # capture (graph.CapturedStep) size the replay stream's scratch
            raise L.MaeClipNativeError(
                f"GEMM scratch of {nbytes} B first requested inside a graph capture; run the step eagerly first")
        if t is not None:
            _SCRATCH_RETIRED.append(t)
        t = torch.zeros((nbytes + 3) // 4, device=device, dtype=torch.float32)
        _SCRATCH[key] = t
    return t


def gemm(A, B, Cout, M, N, K, lda, ldb, ldc, a_layout=KC, b_layout=KC, epilogue=EPI_NONE, alpha=1.0, beta=0.0,
         bias=None, aux=None, aux_out=None, ldaux=0, resid=None, ldr=0, colsum=None, batch=1,
         strides=(0, 0, 0), splitk=1, workspace=None, q8=None):
    _dev(A, B, Cout, bias, aux, aux_out, resid, colsum, workspace)
    if A.dtype != B.dtype:
        raise TypeError("gemm: A and B dtypes differ")
    a = L.GemmArgs(A=A.data_ptr(), B=B.data_ptr(), C=Cout.data_ptr(), M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=ldc,
                   batch=batch, strideA=strides[0], strideB=strides[1], strideC=strides[2],
                   dtype=_dt(A), out_dtype=_dt(Cout), a_layout=a_layout, b_layout=b_layout, epilogue=epilogue,
                   alpha=alpha, beta=beta, bias=_ptr(bias), aux=_ptr(aux), aux_out=_ptr(aux_out), ldaux=ldaux,
                   resid=_ptr(resid), ldr=ldr, colsum_partial=_ptr(colsum), splitk=splitk,
                   workspace=_ptr(workspace))
    _set_q8(a, q8)
    if workspace is None and splitk <= 1:
        nb = int(L.lib().maeclip_gemm_workspace(C.byref(a)))
        if nb > 0:
            workspace = (torch.empty((nb // 4,), device=A.device, dtype=torch.float32) if A.dtype == torch.float32
                         else _stream_scratch(A.device, nb))
            a.workspace = workspace.data_ptr()
    if LAUNCH_HOOK is None:
        _call("maeclip_gemm", C.byref(a), _stream())
    else:
        ea, ec = A.element_size(), Cout.element_size()
        # algorithmic HBM bytes of the launch: operands once, C written once
        # (read too when beta != 0), aux read / aux_out written, fp32 residual read
        nbytes = (M * K + N * K) * ea * batch + M * N * ec * batch * (2 if beta != 0.0 else 1)
        if aux is not None:
            nbytes += M * N * aux.element_size() * batch
        if aux_out is not None:
            nbytes += M * N * aux_out.element_size() * batch
        if resid is not None:
            nbytes += M * N * 4 * batch
        key = (f"M{M} N{N} K{K} {'KR'[a_layout]}{'KR'[b_layout]} epi{epilogue} "
               f"{'bf16' if A.dtype == torch.bfloat16 else 'f32'}>{'bf16' if Cout.dtype == torch.bfloat16 else 'f32'}")
        LAUNCH_HOOK(key, 2.0 * M * N * K * batch, nbytes, lambda: _call("maeclip_gemm", C.byref(a), _stream()))


# ------------------------------------------------------------------ fp8
FP8_E4M3, FP8_E5M2 = 2, 3     # MAECLIP_FP8_* (OCP e4m3fn / e5m2)


class Fp8Rows:
    """An fp8 GEMM operand: q uint8 [rows, cols] (OCP bytes) + per-row
    dequantisation scales s f32 [rows] (x ~= s[r] * q[r, :])."""
    __slots__ = ("q", "s", "fmt")

    def __init__(self, q, s, fmt):
        self.q, self.s, self.fmt = q, s, fmt

    @property
    def shape(self):
        return self.q.shape


class Fp8Blocks:
    """An fp8-blocks GEMM operand (include/maeclip.h "fp8 blocks", the MX
    layout of the block-scaled MFMA): q uint8 [rows, cols] (OCP bytes) + e8m0
    exponents e uint8, one per 32 consecutive columns of a row, in the GEMM's
    read layout (x ~= 2^(e - 127) q). Producers that own only part of a row
    (a GEMM epilogue tile, an attention head) write it without a whole-row
    amax; the block-scaled MFMA applies the scales itself."""
    __slots__ = ("q", "e", "fmt")

    def __init__(self, q, e, fmt):
        self.q, self.e, self.fmt = q, e, fmt

    @property
    def shape(self):
        return self.q.shape


def fp8b_scale_bytes(rows: int, cols: int) -> int:
    return int(L.lib().maeclip_fp8b_scale_bytes(rows, cols))


def new_fp8_blocks(rows, cols, fmt, device):
    """An empty Fp8Blocks for a producer to fill (a GEMM's q8 output, ...)."""
    return Fp8Blocks(torch.empty((rows, cols), device=device, dtype=torch.uint8),
                     torch.empty((fp8b_scale_bytes(rows, cols),), device=device, dtype=torch.uint8), fmt)


def quant_blocks_fp8(x, fmt=FP8_E4M3, out=None):
    """fp8-blocks quantisation of x [rows, cols] (bf16 / f32, cols % 128 == 0):
    per 32-column block e = the smallest power of two keeping |x| / 2^(e-127)
    <= FMT_MAX, q = rne(x 2^(127-e))."""
    _dev(x)
    rows, cols = x.shape
    if out is None:
        out = new_fp8_blocks(rows, cols, fmt, x.device)
    _call("maeclip_quant_blocks_fp8", x.data_ptr(), _dt(x), rows, cols, x.stride(0), out.q.data_ptr(),
          out.q.stride(0), out.e.data_ptr(), fmt, _stream())
    return out


def _set_q8(a, q8):
    """maeclip_gemm_args' optional fp8-blocks copy of a bf16 output"""
    if q8 is not None:
        a.q8, a.ldq8, a.q8_scale, a.q8_fmt = q8.q.data_ptr(), q8.q.stride(0), q8.e.data_ptr(), q8.fmt


def new_fp8_rows(rows, cols, fmt, device):
    """An empty Fp8Rows to be filled by a producer kernel (ln_fwd / ln_bwd q8=)."""
    return Fp8Rows(torch.empty((rows, cols), device=device, dtype=torch.uint8),
                   torch.empty((rows,), device=device, dtype=torch.float32), fmt)


def quant_rows_fp8(x, fmt=FP8_E4M3, out=None):
    """Row-wise fp8 quantisation of x [rows, cols] (bf16 / f32): one pass,
    s = amax(row) / FMT_MAX."""
    _dev(x)
    rows, cols = x.shape
    if out is None:
        out = Fp8Rows(torch.empty((rows, cols), device=x.device, dtype=torch.uint8),
                      torch.empty((rows,), device=x.device, dtype=torch.float32), fmt)
    _call("maeclip_quant_rows_fp8", x.data_ptr(), _dt(x), rows, cols, x.stride(0), out.q.data_ptr(), out.q.stride(0),
          out.s.data_ptr(), fmt, _stream())
    return out


def quant_cols_fp8(w, out=None):
    """W^T quantised (e4m3) from the fp32 master W [rows, cols]: q [cols, rows],
    one scale per column of W (= per row of W^T)."""
    _dev(w)
    rows, cols = w.shape
    if w.dtype != torch.float32 or w.stride(1) != 1:
        raise TypeError("quant_cols_fp8: fp32 row-major W")
    if out is None:
        ldq = (rows + 15) // 16 * 16
        out = Fp8Rows(torch.empty((cols, ldq), device=w.device, dtype=torch.uint8)[:, :rows],
                      torch.empty((cols,), device=w.device, dtype=torch.float32), FP8_E4M3)
    nb = int(L.lib().maeclip_quant_cols_fp8_workspace(rows, cols))
    ws = torch.empty((nb // 4,), device=w.device, dtype=torch.float32)
    _call("maeclip_quant_cols_fp8", w.data_ptr(), rows, cols, w.stride(0), out.q.data_ptr(), out.q.stride(0),
          out.s.data_ptr(), ws.data_ptr(), nb, _stream())
    return out


class Fp8WeightPlan:
    """fp8 operands of a set of fp32 GEMM weights W [N, K], refreshed for all of
    them in one maeclip_quant_weights_fp8 call (two launches, W read twice): W
    per output channel (forward B operand) and W^T per input channel (dgrad B
    operand). Weights with K > 4096 (beyond the batched call's row registers)
    take the per-weight quant_rows_fp8 / quant_cols_fp8 launches instead."""

    WQ_MAX_COLS = 4096

    def __init__(self, weights, device):
        self.ops = []
        batched, self.single = [], []
        for w in weights:
            N, Kd = w.shape
            ldqt = (N + 15) // 16 * 16
            wq = Fp8Rows(torch.empty((N, Kd), device=device, dtype=torch.uint8),
                         torch.empty((N,), device=device, dtype=torch.float32), FP8_E4M3)
            wt = Fp8Rows(torch.empty((Kd, ldqt), device=device, dtype=torch.uint8)[:, :N],
                         torch.empty((Kd,), device=device, dtype=torch.float32), FP8_E4M3)
            self.ops.append((wq, wt))
            (batched if Kd <= self.WQ_MAX_COLS else self.single).append((w, wq, wt))
        n = len(batched)
        self.n = n
        if n:
            self.host = (L.Fp8wEntry * n)()
            for i, (w, wq, wt) in enumerate(batched):
                e = self.host[i]
                e.w, e.q, e.sq = w.data_ptr(), wq.q.data_ptr(), wq.s.data_ptr()
                e.qt, e.sqt = wt.q.data_ptr(), wt.s.data_ptr()
                e.rows, e.cols, e.ld, e.ldqt = w.shape[0], w.shape[1], w.stride(0), wt.q.stride(0)
            nb = int(L.lib().maeclip_quant_weights_fp8_prepare(self.host, n))
            self.ws_bytes = max(nb, 4)
            self.ws = torch.empty((self.ws_bytes // 4,), device=device, dtype=torch.float32)
            self.dev = torch.frombuffer(bytearray(bytes(self.host)), dtype=torch.uint8).to(device)

    def run(self):
        if self.n:
            _call("maeclip_quant_weights_fp8", self.dev.data_ptr(), self.host, self.n, self.ws.data_ptr(),
                  self.ws_bytes, _stream())
        for w, wq, wt in self.single:
            quant_rows_fp8(w, FP8_E4M3, out=wq)
            quant_cols_fp8(w, out=wt)


def gemm_fp8(A, B: Fp8Rows, Cout, epilogue=EPI_NONE, alpha=1.0, bias=None, aux=None, aux_out=None,
             resid=None, colsum=None, q8=None):
    """Cout[M, N] = epilogue(alpha * s_B[n] * sum_k s_A qA[m, k] qB[n, k]) on the
    block-scaled fp8 MFMA (A e4m3 or e5m2, B e4m3; KC x KC, K % 128 == 0). A is
    an Fp8Rows (per-row s_A, applied in the epilogue) or an Fp8Blocks (e8m0
    per 32 K, applied by the MFMA; maeclip_gemm_fp8_blocks); q8: an Fp8Blocks
    the epilogue fills with the bf16 output's fp8 copy."""
    blocks = isinstance(A, Fp8Blocks)
    M, K = A.q.shape
    N = B.q.shape[0]
    if B.q.shape[1] != K or B.fmt != FP8_E4M3:
        raise ValueError("gemm_fp8: B must be e4m3 [N, K] with A's K")
    _dev(A.q, B.q, Cout, bias, aux, aux_out, resid, colsum)
    a = L.GemmArgs(A=A.q.data_ptr(), B=B.q.data_ptr(), C=Cout.data_ptr(), M=M, N=N, K=K, lda=A.q.stride(0),
                   ldb=B.q.stride(0), ldc=Cout.stride(0), batch=1, strideA=0, strideB=0, strideC=0,
                   dtype=A.fmt, out_dtype=_dt(Cout), a_layout=KC, b_layout=KC, epilogue=epilogue,
                   alpha=alpha, beta=0.0, bias=_ptr(bias), aux=_ptr(aux), aux_out=_ptr(aux_out),
                   ldaux=(aux.stride(0) if aux is not None else aux_out.stride(0) if aux_out is not None else 0),
                   resid=_ptr(resid), ldr=(resid.stride(0) if resid is not None else 0),
                   colsum_partial=_ptr(colsum), splitk=1, workspace=None)
    _set_q8(a, q8)
    if blocks:
        launch = lambda: _call("maeclip_gemm_fp8_blocks", C.byref(a), A.e.data_ptr(), B.s.data_ptr(), _stream())
    else:
        nb = int(L.lib().maeclip_gemm_workspace(C.byref(a)))
        if nb > 0:   # the split plan's counters + partial tiles (per stream)
            a.workspace = _stream_scratch(A.q.device, nb).data_ptr()
        launch = lambda: _call("maeclip_gemm_fp8", C.byref(a), A.s.data_ptr(), B.s.data_ptr(), _stream())
    if LAUNCH_HOOK is None:
        launch()
        return Cout
    ec = Cout.element_size()
    nbytes = M * K + N * K + M * N * ec
    for t in (aux, aux_out):
        if t is not None:
            nbytes += M * N * t.element_size()
    if resid is not None:
        nbytes += M * N * 4
    if q8 is not None:
        nbytes += M * N + fp8b_scale_bytes(M, N)
    key = (f"M{M} N{N} K{K} KK epi{epilogue} fp8{'e5' if A.fmt == FP8_E5M2 else 'e4'}{'b' if blocks else ''}"
           f">{'bf16' if ec == 2 else 'f32'}")
    LAUNCH_HOOK(key, 2.0 * M * N * K, nbytes, launch)
    return Cout


def linear_fp8(xq, wq: Fp8Rows, bias=None, out_dtype=torch.bfloat16, epilogue=EPI_NONE, resid=None,
               aux_out=None, aux=None, colsum=None, q8=None, out=None):
    """y[M, N] = x[M, K] w[N, K]^T on fp8 operands (forward: w = W [N_out, K_in];
    dgrad: x = dY, w = W^T [K_in, N_out]); xq Fp8Rows or Fp8Blocks."""
    y = out if out is not None else torch.empty((xq.q.shape[0], wq.q.shape[0]), device=xq.q.device, dtype=out_dtype)
    return gemm_fp8(xq, wq, y, epilogue=epilogue, bias=bias, resid=resid, aux_out=aux_out, aux=aux, colsum=colsum,
                    q8=q8)


def gemm_colsum_rows(M: int) -> int:
    return int(L.lib().maeclip_gemm_colsum_rows(M))


def linear_fwd(x, w, bias=None, out_dtype=None, epilogue=EPI_NONE, resid=None, aux_out=None, colsum=None, out=None,
               q8=None):
    """y[M,N] = x[M,K] w[N,K]^T (+bias) with epilogue (nn.Linear forward);
    out: an [M, N] row-major destination (e.g. a row slice of a larger buffer)."""
    M, K = x.shape
    N = w.shape[0]
    out_dtype = out_dtype or x.dtype
    y = out if out is not None else torch.empty((M, N), device=x.device, dtype=out_dtype)
    gemm(x, w, y, M, N, K, x.stride(0), w.stride(0), y.stride(0), KC, KC, epilogue=epilogue, bias=bias, resid=resid,
         ldr=(resid.stride(0) if resid is not None else 0), aux_out=aux_out,
         ldaux=(aux_out.stride(0) if aux_out is not None else 0), colsum=colsum, q8=q8)
    return y


def linear_dgrad(dy, w, out_dtype=None, epilogue=EPI_NONE, aux=None, resid=None, colsum=None, out=None, q8=None):
    """dx[M,K] = dy[M,N] w[N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    out = out if out is not None else torch.empty((M, K), device=dy.device, dtype=out_dtype or dy.dtype)
    gemm(dy, w, out, M, K, N, dy.stride(0), w.stride(0), out.stride(0), KC, RC, epilogue=epilogue, aux=aux,
         ldaux=(aux.stride(0) if aux is not None else 0), resid=resid,
         ldr=(resid.stride(0) if resid is not None else 0), colsum=colsum, q8=q8)
    return out


def linear_wgrad(dy, x, out=None, beta=0.0, bias_grad_out=None):
    """dW[N,K] = dy[M,N]^T x[M,K]  (fp32), split-K over the token dimension."""
    M, N = dy.shape
    K = x.shape[1]
    out = out if out is not None else torch.empty((N, K), device=dy.device, dtype=torch.float32)
    S = int(L.lib().maeclip_gemm_splitk(N, K, M)) if out.stride(0) == K else 1
    ws = torch.empty((S * N * K,), device=dy.device, dtype=torch.float32) if S > 1 else None
    gemm(dy, x, out, N, K, M, dy.stride(0), x.stride(0), out.stride(0), RC, RC, beta=beta, splitk=S, workspace=ws)
    return out


def wgrad_grouped(items, beta=0.0):
    """dW_p = dy_p^T x_p for a list of (dy [M, N_p], x [M, K_p], out [N_p, K_p] f32)
    sharing the token count M, in one maeclip_wgrad_grouped call (one persistent
    launch per 48 problems on the bf16 path)."""
    if not items:
        return
    M = items[0][0].shape[0]
    n = len(items)
    probs = (L.WgradProblem * n)()
    for i, (dy, x, out) in enumerate(items):
        _dev(dy, x, out)
        if dy.shape[0] != M or x.shape[0] != M or dy.dtype != x.dtype or out.dtype != torch.float32:
            raise ValueError("wgrad_grouped: problems must share the token count and dtype (fp32 dW)")
        if out.shape != (dy.shape[1], x.shape[1]) or out.stride(0) != x.shape[1] or dy.stride(1) != 1 \
                or x.stride(1) != 1:
            raise ValueError("wgrad_grouped: dW must be dense [N, K]; dy/x row-major")
        q = probs[i]
        q.dy, q.x, q.dw = dy.data_ptr(), x.data_ptr(), out.data_ptr()
        q.N, q.K, q.ldy, q.ldx = dy.shape[1], x.shape[1], dy.stride(0), x.stride(0)
    dt = _dt(items[0][0])
    lib = L.lib()
    nb = int(lib.maeclip_wgrad_grouped_workspace(probs, n, M, dt))
    ws = torch.empty((max(nb, 4) // 4,), device=items[0][0].device, dtype=torch.float32) if nb > 0 else None
    launch = lambda: _call("maeclip_wgrad_grouped", probs, n, M, dt, beta, _ptr(ws), nb, _stream())
    if LAUNCH_HOOK is None:
        launch()
        return
    es = items[0][0].element_size()
    flops = sum(2.0 * M * dy.shape[1] * x.shape[1] for dy, x, _ in items)
    # algorithmic bytes: dy and x once each, dW written (read too when beta != 0)
    nbytes = sum(M * (dy.shape[1] + x.shape[1]) * es + dy.shape[1] * x.shape[1] * 4 * (2 if beta else 1)
                 for dy, x, _ in items)
    key = f"wgrad_grouped M{M} x{n} N{items[0][0].shape[1]} K{items[0][1].shape[1]} {'bf16' if dt == L.BF16 else 'f32'}>f32"
    LAUNCH_HOOK(key, flops, nbytes, launch)


# ------------------------------------------------------------- reductions
def colsum_reduce(partial, out=None, accumulate=False, scale=1.0):
    _dev(partial)
    P, N = partial.shape
    out = out if out is not None else torch.empty((N,), device=partial.device, dtype=torch.float32)
    ns = int(L.lib().maeclip_colsum_scratch(P, N))
    scratch = torch.empty((ns,), device=partial.device, dtype=torch.float32) if ns > 0 else None
    _call("maeclip_colsum_reduce", partial.data_ptr(), P, N, out.data_ptr(), int(accumulate), scale, _ptr(scratch),
          _stream())
    return out


def rows_colsum(x, out_bf16=None, q8=None):
    """partial column sums [G, D] of x [M, D] (f32/bf16); optional bf16 copy
    and (with it) its fp8 rows q8 (Fp8Rows, == quant_rows_fp8(out_bf16))."""
    _dev(x, out_bf16)
    M, D = x.shape
    G = int(L.lib().maeclip_rows_colsum_partial_rows(M))
    part = torch.empty((G, D), device=x.device, dtype=torch.float32)
    if q8 is not None:
        _call("maeclip_rows_colsum_q8", x.data_ptr(), _dt(x), M, D, x.stride(0), _ptr(out_bf16), part.data_ptr(),
              q8.q.data_ptr(), q8.q.stride(0), q8.s.data_ptr(), q8.fmt, _stream())
        return part
    _call("maeclip_rows_colsum", x.data_ptr(), _dt(x), M, D, x.stride(0), _ptr(out_bf16), part.data_ptr(), _stream())
    return part


def pool_fwd(x):
    B, n, D = x.shape
    out = torch.empty((B, D), device=x.device, dtype=torch.float32)
    _call("maeclip_pool_fwd", x.data_ptr(), B, n, D, out.data_ptr(), _stream())
    return out


def pool_bwd(dout, n, dx=None, accumulate=False):
    B, D = dout.shape
    dx = dx if dx is not None else torch.empty((B, n, D), device=dout.device, dtype=torch.float32)
    _call("maeclip_pool_bwd", dout.data_ptr(), B, n, D, dx.data_ptr(), int(accumulate), _stream())
    return dx


def dropout(x, p, seed, out=None, step_ptr=None):
    M, D = x.shape
    out = out if out is not None else torch.empty_like(x)
    _call("maeclip_dropout", x.data_ptr(), out.data_ptr(), M, D, x.stride(0), float(p), int(seed), _ptr(step_ptr),
          _stream())
    return out


def embed_fwd(ids, word, pos, mask=None):
    """word + position embedding rows [B*T, D] (f32). mask (optional, int64
    [B, T] attention_mask): also returns it as the f32 key mask [B, T],
    converted in the same launch."""
    _dev(ids, word, pos)
    B, T = ids.shape
    V, D = word.shape
    out = torch.empty((B * T, D), device=word.device, dtype=torch.float32)
    mo = None
    if mask is not None:
        _dev(mask)
        if mask.dtype != torch.int64 or mask.shape != (B, T) or not mask.is_contiguous():
            raise ValueError("embed_fwd: mask must be a dense int64 [B, T] tensor")
        mo = torch.empty((B, T), device=word.device, dtype=torch.float32)
    _call("maeclip_embed_fwd", ids.data_ptr(), word.data_ptr(), pos.data_ptr(), B, T, D, V, out.data_ptr(),
          _ptr(mask), _ptr(mo), _stream())
    return out if mask is None else (out, mo)


# -------------------------------------------------------------- LayerNorm
def ln_fwd(x, gamma, beta, eps, out_dtype=None, res=None, in_dropout=0.0, out_dropout=0.0, seed_in=0, seed_out=0,
           want_stats=True, y2=False, xsum=False, step_ptr=None, q8=None, y_out=None, mean_out=None, rstd_out=None):
    """Returns (y, mean, rstd, y2_bf16, xsum). q8 (Fp8Rows, optional): also
    filled with the fp8 row quantisation of y (== quant_rows_fp8(y, q8.fmt)).
    y_out / mean_out / rstd_out: dense destinations (row slices of larger buffers)."""
    _dev(x, gamma, beta, res)
    M, D = x.shape
    dev = x.device
    y = y_out if y_out is not None else torch.empty((M, D), device=dev, dtype=out_dtype or x.dtype)
    if y.stride(0) != D:
        raise ValueError("ln_fwd: y must be dense [M, D] rows")
    mean = (mean_out if mean_out is not None else torch.empty((M,), device=dev, dtype=torch.float32)) \
        if want_stats else None
    rstd = (rstd_out if rstd_out is not None else torch.empty((M,), device=dev, dtype=torch.float32)) \
        if want_stats else None
    yb = torch.empty((M, D), device=dev, dtype=torch.bfloat16) if y2 else None
    xs = torch.empty((M, D), device=dev, dtype=torch.float32) if xsum else None
    a = L.LnFwdArgs(x=x.data_ptr(), x_dtype=_dt(x), res=_ptr(res), ldres=(res.stride(0) if res is not None else 0),
                    in_dropout_p=in_dropout, gamma=gamma.data_ptr(), beta=beta.data_ptr(), y=y.data_ptr(),
                    y_dtype=_dt(y), y2=_ptr(yb), ldy2=D, xsum_out=_ptr(xs), ldxs=D, mean=_ptr(mean), rstd=_ptr(rstd),
                    out_dropout_p=out_dropout, seed_in=int(seed_in), seed_out=int(seed_out), step_ptr=_ptr(step_ptr),
                    M=M, D=D, ldx=x.stride(0), ldy=D, eps=eps)
    if q8 is not None:
        a.q8, a.ldq8, a.q8_scale, a.q8_fmt = q8.q.data_ptr(), q8.q.stride(0), q8.s.data_ptr(), q8.fmt
    _call("maeclip_ln_fwd", C.byref(a), _stream())
    return y, mean, rstd, yb, xs


def ln_bwd_partial_rows(M: int, D: int) -> int:
    return int(L.lib().maeclip_ln_bwd_partial_rows(M, D))


def ln_bwd(dy, x, mean, rstd, gamma, dres=None, want_bf16=False, want_param_grads=True, want_colsum=False,
           dres_pool=None, pool_n=0, q8=None, dx_out=None, dxb_out=None, pg_out=None, pb_out=None, pc_out=None):
    """Returns (dx f32, dx_bf16, dgamma_partial, dbeta_partial, dx_colsum_partial).
    q8 (Fp8Rows, with want_bf16): also filled with quant_rows_fp8(dx_bf16, q8.fmt).
    dres_pool [M / pool_n, D]: residual gradient = the avg-pool backward of it
    (1/(pool_n-1) on every non-cls row), fused instead of a dres tensor."""
    _dev(dy, x, mean, rstd, gamma, dres, dres_pool)
    M, D = x.shape
    dev = x.device
    G = ln_bwd_partial_rows(M, D)
    e = lambda o, shape, dt: o if o is not None else torch.empty(shape, device=dev, dtype=dt)
    dx = e(dx_out, (M, D), torch.float32)
    dxb = e(dxb_out, (M, D), torch.bfloat16) if want_bf16 else None
    pg = e(pg_out, (G, D), torch.float32) if want_param_grads else None
    pb = e(pb_out, (G, D), torch.float32) if want_param_grads else None
    pc = e(pc_out, (G, D), torch.float32) if want_colsum else None
    for t, rows in ((dx, M), (dxb, M), (pg, G), (pb, G), (pc, G)):
        if t is not None and (t.stride(0) != D or t.shape[0] != rows):
            raise ValueError("ln_bwd: outputs must be dense rows of the expected count")
    a = L.LnBwdArgs(dy=dy.data_ptr(), dy_dtype=_dt(dy), x=x.data_ptr(), x_dtype=_dt(x), mean=mean.data_ptr(),
                    rstd=rstd.data_ptr(), gamma=gamma.data_ptr(), dres=_ptr(dres), dx=dx.data_ptr(), dx_bf=_ptr(dxb),
                    lddx_bf=D, dgamma_partial=_ptr(pg), dbeta_partial=_ptr(pb), dx_colsum_partial=_ptr(pc),
                    M=M, D=D, ldx=x.stride(0), lddy=dy.stride(0), lddx=D, dres_pool=_ptr(dres_pool),
                    pool_n=int(pool_n))
    if q8 is not None:
        a.q8, a.ldq8, a.q8_scale, a.q8_fmt = q8.q.data_ptr(), q8.q.stride(0), q8.s.data_ptr(), q8.fmt
    _call("maeclip_ln_bwd", C.byref(a), _stream())
    return dx, dxb, pg, pb, pc


# -------------------------------------------------------------- attention
def attn_fwd(qkv, B, n, H, hd, scale, key_mask=None, dropout_p=0.0, seed=0, want_lse=True, step_ptr=None,
             o_out=None, lse_out=None, q8=None):
    """(o, lse); q8 (Fp8Blocks [B*n, H*hd], optional): also filled with the fp8
    blocks of o as stored (the proj GEMM's operand in fp8 mode)."""
    _dev(qkv, key_mask)
    D = H * hd
    o = o_out if o_out is not None else torch.empty((B * n, D), device=qkv.device, dtype=qkv.dtype)
    if o.stride(0) != D:
        raise ValueError("attn_fwd: o must be dense [B*n, D] rows")
    lse = (lse_out if lse_out is not None else torch.empty((B, H, n), device=qkv.device, dtype=torch.float32)) \
        if want_lse else None
    a = L.AttnArgs(qkv=qkv.data_ptr(), o=o.data_ptr(), lse=_ptr(lse), dout=None, dqkv=None, key_mask=_ptr(key_mask),
                   colsum_partial=None, ld_qkv=qkv.stride(0), ld_o=D, ld_dqkv=0, B=B, n=n, H=H, head_dim=hd,
                   dtype=_dt(qkv), scale=scale, dropout_p=dropout_p, seed=int(seed), step_ptr=_ptr(step_ptr))
    _set_q8(a, q8)
    _call("maeclip_attn_fwd", C.byref(a), _stream())
    return o, lse


def attn_bwd(qkv, o, dout, lse, B, n, H, hd, scale, want_colsum=True, key_mask=None, dqkv_out=None, part_out=None,
             q8=None):
    """(dqkv, bias-gradient partials); q8 (Fp8Blocks [B*n, 3*H*hd], optional):
    the fp8 blocks of dqkv as stored (the qkv dgrad GEMM's operand)."""
    _dev(qkv, o, dout, lse, key_mask)
    D = H * hd
    dqkv = dqkv_out if dqkv_out is not None else torch.empty((B * n, 3 * D), device=qkv.device, dtype=qkv.dtype)
    if dqkv.stride(0) != 3 * D:
        raise ValueError("attn_bwd: dqkv must be dense [B*n, 3D] rows")
    part = (part_out if part_out is not None else torch.empty((B, 3 * D), device=qkv.device, dtype=torch.float32)) \
        if want_colsum else None
    a = L.AttnArgs(qkv=qkv.data_ptr(), o=o.data_ptr(), lse=lse.data_ptr(), dout=dout.data_ptr(), dqkv=dqkv.data_ptr(),
                   key_mask=_ptr(key_mask), colsum_partial=_ptr(part), ld_qkv=qkv.stride(0), ld_o=o.stride(0),
                   ld_dqkv=3 * D, B=B, n=n, H=H, head_dim=hd, dtype=_dt(qkv), scale=scale, dropout_p=0.0, seed=0)
    _set_q8(a, q8)
    _call("maeclip_attn_bwd", C.byref(a), _stream())
    return dqkv, part


# --------------------------------------------------------------------- MAE
def mask_ids(B, L_, len_keep, seed, step, sample_offset, device, want_noise=False, step_ptr=None):
    """HF random_masking ids for mask step `step` (+ *step_ptr when given)."""
    ids_shuffle = torch.empty((B, L_), device=device, dtype=torch.int32)
    ids_restore = torch.empty((B, L_), device=device, dtype=torch.int32)
    mask = torch.empty((B, L_), device=device, dtype=torch.float32)
    noise = torch.empty((B, L_), device=device, dtype=torch.float32) if want_noise else None
    a = L.MaskArgs(ids_shuffle=ids_shuffle.data_ptr(), ids_restore=ids_restore.data_ptr(), mask=mask.data_ptr(),
                   noise=_ptr(noise), B=B, L=L_, len_keep=len_keep, seed=int(seed), step=int(step),
                   sample_offset=int(sample_offset), step_ptr=_ptr(step_ptr))
    _call("maeclip_mask_ids", C.byref(a), _stream())
    return ids_shuffle, ids_restore, mask, noise


# albumentations A.Normalize defaults of the reference's transforms (dataset.py:49)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def is_u8_image(img):
    """uint8 [B, S, S, 3] decoded RGB pixels (HWC), normalised inside the kernels."""
    return img.dtype == torch.uint8 and img.dim() == 4 and img.shape[-1] == 3


def image_geometry(img):
    """(B, C, S) of an fp32 NCHW batch or a uint8 HWC pixel batch."""
    if is_u8_image(img):
        return img.shape[0], 3, img.shape[1]
    return img.shape[0], img.shape[1], img.shape[2]


def _u8_fields(img):
    """img_u8 / Normalize constants of the ABI structs (img: NCHW fp32 -> unset)."""
    if not is_u8_image(img):
        return dict(img=img.data_ptr())
    return dict(img=None, img_u8=img.data_ptr(), u8_mean=(C.c_float * 3)(*IMAGENET_MEAN),
                u8_std=(C.c_float * 3)(*IMAGENET_STD), u8_max_pixel=255.0)


def patch_gather(img, ids_shuffle, keep, p, kpad, dtype):
    """Visible-patch rows for the patch-embed GEMM from an fp32 NCHW image or
    from uint8 HWC pixels (A.Normalize + permute fused, dataset.py:49, :34)."""
    _dev(img, ids_shuffle)
    B, Cc, S = image_geometry(img)
    out = torch.empty((B * keep, kpad), device=img.device, dtype=dtype)
    a = L.PatchArgs(ids_shuffle=_ptr(ids_shuffle), out=out.data_ptr(), ld_out=kpad, B=B, C=Cc, S=S,
                    p=p, keep=keep, dtype=_dt(out), **_u8_fields(img))
    _call("maeclip_patch_gather", C.byref(a), _stream())
    return out


def tokens_fwd(y, ids_shuffle, pos, cls, B, L_, keep):
    D = pos.shape[-1]
    x = torch.empty((B, keep + 1, D), device=y.device, dtype=torch.float32)
    a = L.TokensArgs(y=y.data_ptr(), ldy=y.stride(0), ids_shuffle=_ptr(ids_shuffle), ids_restore=None,
                     pos=pos.data_ptr(), cls=cls.data_ptr(), x=x.data_ptr(), dx=None, dy=None, dpos=None, dcls=None,
                     B=B, L=L_, keep=keep, D=D, dtype=_dt(y))
    _call("maeclip_tokens_fwd", C.byref(a), _stream())
    return x


def tokens_bwd(dx, ids_restore, B, L_, keep, dy_dtype, dpos=None, dcls=None):
    D = dx.shape[-1]
    dy = torch.empty((B * keep, D), device=dx.device, dtype=dy_dtype)
    if dpos is None:
        dpos = torch.empty((L_ + 1, D), device=dx.device, dtype=torch.float32)
    if dcls is None:
        dcls = torch.empty((D,), device=dx.device, dtype=torch.float32)
    if dpos.shape != (L_ + 1, D) or dcls.shape != (D,) or not (dpos.is_contiguous() and dcls.is_contiguous()):
        raise ValueError("tokens_bwd: dpos [L+1, D] / dcls [D] must be dense")
    a = L.TokensArgs(y=None, ldy=D, ids_shuffle=None, ids_restore=_ptr(ids_restore), pos=None, cls=None, x=None,
                     dx=dx.data_ptr(), dy=dy.data_ptr(), dpos=dpos.data_ptr(), dcls=dcls.data_ptr(),
                     B=B, L=L_, keep=keep, D=D, dtype=_dt(dy))
    _call("maeclip_tokens_bwd", C.byref(a), _stream())
    return dy, dpos, dcls


def unshuffle_fwd(y, ids_restore, mask_token, pos, B, L_, keep):
    D = pos.shape[-1]
    out = torch.empty((B, L_ + 1, D), device=y.device, dtype=torch.float32)
    a = L.UnshuffleArgs(y=y.data_ptr(), ldy=y.stride(0), ids_shuffle=None, ids_restore=ids_restore.data_ptr(),
                        mask_token=mask_token.data_ptr(), pos=pos.data_ptr(), out=out.data_ptr(), dout=None, dy=None,
                        dmask_partial=None, colsum_partial=None, B=B, L=L_, keep=keep, D=D, dtype=L.F32)
    _call("maeclip_unshuffle_fwd", C.byref(a), _stream())
    return out


def unshuffle_bwd(dout, ids_restore, B, L_, keep, dy_dtype):
    D = dout.shape[-1]
    dy = torch.empty((B * (keep + 1), D), device=dout.device, dtype=dy_dtype)
    G = int(L.lib().maeclip_unshuffle_bwd_partial_rows(B))
    dmask = torch.empty((G, D), device=dout.device, dtype=torch.float32)
    cs = torch.empty((G, D), device=dout.device, dtype=torch.float32)
    a = L.UnshuffleArgs(y=None, ldy=D, ids_shuffle=None, ids_restore=ids_restore.data_ptr(), mask_token=None,
                        pos=None, out=None, dout=dout.data_ptr(), dy=dy.data_ptr(), dmask_partial=dmask.data_ptr(),
                        colsum_partial=cs.data_ptr(), B=B, L=L_, keep=keep, D=D, dtype=_dt(dy))
    _call("maeclip_unshuffle_bwd", C.byref(a), _stream())
    return dy, dmask, cs


def mae_loss_fwd(pred, img, mask, p, norm_pix):
    B, Cc, S = image_geometry(img)
    L_ = mask.shape[1]
    row = torch.empty((B * L_,), device=img.device, dtype=torch.float32)
    a = L.MaeLossArgs(pred=pred.data_ptr(), ldp=pred.stride(0), mask=mask.data_ptr(),
                      row_loss=row.data_ptr(), dpred=None, lddp=0, grad_out=None, colsum_partial=None,
                      loss_scale=1.0, mask_count=1.0, B=B, C=Cc, S=S, p=p, L=L_, norm_pix=int(norm_pix),
                      dtype=_dt(pred), **_u8_fields(img))
    _call("maeclip_mae_loss_fwd", C.byref(a), _stream())
    return row


def mae_loss_bwd(pred, img, mask, p, norm_pix, grad_out, mask_count, loss_scale=1.0):
    B, Cc, S = image_geometry(img)
    L_ = mask.shape[1]
    P = Cc * p * p
    # padded pred rows (decoder_pred N rounded up for the GEMM): the kernel
    # zeroes dpred's pad columns (they meet the zero rows of the padded weight)
    dpred = torch.empty_like(pred)
    G = int(L.lib().maeclip_mae_loss_bwd_partial_rows(B, L_))
    cs = torch.empty((G, P), device=img.device, dtype=torch.float32)
    a = L.MaeLossArgs(pred=pred.data_ptr(), ldp=pred.stride(0), mask=mask.data_ptr(),
                      row_loss=None, dpred=dpred.data_ptr(), lddp=dpred.stride(0), grad_out=_ptr(grad_out),
                      colsum_partial=cs.data_ptr(), loss_scale=loss_scale, mask_count=float(mask_count),
                      B=B, C=Cc, S=S, p=p, L=L_, norm_pix=int(norm_pix), dtype=_dt(pred), **_u8_fields(img))
    _call("maeclip_mae_loss_bwd", C.byref(a), _stream())
    return dpred, cs


# --------------------------------------------------------------- CLIP loss
def clip_loss(I, T, temperature, want_grad=True, grad_rows=None, row_loss=False):
    """Fused soft-target CLIP loss (CLIP.py:34-43). grad_rows = (row0, count):
    gradients only for that slice of the rows (data parallel: the local rows
    of the gathered batch); default all rows. Returns (loss, dI, dT[, rl])."""
    _dev(I, T)
    N, P = I.shape
    r0, nr = (0, N) if grad_rows is None else grad_rows
    if not (0 <= r0 and nr >= 1 and r0 + nr <= N):
        raise ValueError(f"clip_loss: gradient rows {grad_rows} out of range for N={N}")
    ws_bytes = int(L.lib().maeclip_clip_loss_workspace(N, P, nr if want_grad else 0))
    ws = torch.empty((ws_bytes // 4,), device=I.device, dtype=torch.float32)
    loss = torch.empty((), device=I.device, dtype=torch.float32)
    dI = torch.empty((nr, P), device=I.device, dtype=torch.float32) if want_grad else None
    dT = torch.empty((nr, P), device=I.device, dtype=torch.float32) if want_grad else None
    rl = torch.empty((N,), device=I.device, dtype=torch.float32) if row_loss else None
    a = L.ClipArgs(I=I.data_ptr(), T=T.data_ptr(), ld_I=I.stride(0), ld_T=T.stride(0), N=N, P=P,
                   temperature=float(temperature), loss=loss.data_ptr(), row_loss_out=_ptr(rl), dI=_ptr(dI),
                   dT=_ptr(dT), ld_dI=P, ld_dT=P, grad_row0=r0, grad_rows=nr, workspace=ws.data_ptr(),
                   ws_bytes=ws_bytes)
    _call("maeclip_clip_loss", C.byref(a), _stream())
    if row_loss:
        return loss, dI, dT, rl
    return loss, dI, dT


# ------------------------------------------------------------ multi-tensor
def counter_add_snap(counter, snap, delta=1):
    """snap[0] = counter[0]; counter[0] += delta (stream-ordered, one launch)."""
    _dev(counter, snap)
    _call("maeclip_counter_add_snap", counter.data_ptr(), int(delta), snap.data_ptr(), _stream())


def scalar_axpy(a, b, w):
    """a + w * b on device f32 scalars (no host sync)."""
    _dev(a, b)
    out = torch.empty((), device=a.device, dtype=torch.float32)
    _call("maeclip_scalar_axpy", a.data_ptr(), b.data_ptr(), float(w), out.data_ptr(), _stream())
    return out


def copy_words(src, dst):
    """dst <- src, bit for bit, for small contiguous device tensors of equal byte
    size (4-byte words through maeclip_copy_f32: one launch of ours instead of
    a runtime blit kernel)"""
    _dev(src, dst)
    nb = src.numel() * src.element_size()
    if nb != dst.numel() * dst.element_size() or nb % 4 or not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("copy_words: contiguous tensors of one byte size, a multiple of 4")
    _call("maeclip_copy_f32", src.data_ptr(), dst.data_ptr(), nb // 4, _stream())
    return dst


class HostScalars:
    """n f32 values in pinned, device-mapped host memory (maeclip_host_mapped_alloc):
    a kernel writes them on the stream (publish), the host reads them after
    synchronising that stream (values) -- no device-to-host copy launch."""

    def __init__(self, n=1, slots=1):
        self.n, self.slots = int(n), int(slots)
        h, d = C.c_void_p(), C.c_void_p()
        _call("maeclip_host_mapped_alloc", 4 * self.n * self.slots, C.byref(h), C.byref(d))
        self.host, self.dev = h.value, d.value
        self._view = (C.c_float * (self.n * self.slots)).from_address(self.host)

    def publish(self, src, counter=None):
        """copy the first n values of device f32 tensor `src` here (stream-ordered);
        with `counter` (device int64) into slot counter & 1 of a 2-slot buffer
        (HostScalars(n, slots=2))"""
        _dev(src)
        if src.dtype != torch.float32 or src.numel() < self.n or not src.is_contiguous():
            raise TypeError("HostScalars.publish: contiguous f32 device tensor with >= n values")
        if counter is None:
            _call("maeclip_copy_f32", src.data_ptr(), self.dev, self.n, _stream())
        else:
            if self.slots != 2 or counter.dtype != torch.int64:
                raise TypeError("HostScalars.publish: slot publishing needs slots=2 and an int64 counter")
            _call("maeclip_copy_f32_slot", src.data_ptr(), self.dev, self.n, counter.data_ptr(), _stream())

    def values(self, slot=0):
        return [float(v) for v in self._view[slot * self.n:(slot + 1) * self.n]]

    def __del__(self):
        try:
            if getattr(self, "host", None):
                L.lib().maeclip_host_mapped_free(self.host)
                self.host = None
        except Exception:
            pass


def scale_by_scalar(s, w=1.0, x=None, y=None, out_x=None, out_y=None):
    """(w * s[0]) * x and (w * s[0]) * y in one launch (s: device f32 scalar;
    x None: the constant 1, then out_x must be given). Returns (out_x, out_y)."""
    _dev(s)
    def prep(src, dst):
        if src is None and dst is None:
            return None, None, 0
        if src is not None:
            _dev(src)
            if src.dtype != torch.float32 or not src.is_contiguous():
                raise ValueError("scale_by_scalar: dense f32 tensors")
            if dst is None:
                dst = torch.empty_like(src)
        return src, dst, dst.numel()
    x, out_x, nx = prep(x, out_x)
    y, out_y, ny = prep(y, out_y)
    _call("maeclip_scale_by_scalar2", _ptr(x), _ptr(out_x), nx, _ptr(y), _ptr(out_y), ny, s.data_ptr(), float(w),
          _stream())
    return out_x, out_y


def counter_add(counter, delta=1):
    """counter (device int64[1]) += delta, stream-ordered (graph-capturable)."""
    _dev(counter)
    _call("maeclip_counter_add", counter.data_ptr(), int(delta), _stream())


def _capturing() -> bool:
    return torch.cuda.is_current_stream_capturing()


class PinnedStager:
    """Host -> device staging of small descriptor arrays through a ring of pinned
    buffers; a buffer is reused only after the async copy that read it is done.

    Under HIP-graph capture the descriptors of a stage are constants of the
    graph (every pointer in them is fixed for its life), so they are uploaded
    ONCE, at capture time, on an uncaptured upload stream into a device buffer
    kept in `captured` for the graph's life: the graph holds no memcpy node
    and a replay copies nothing."""

    def __init__(self, slots=4):
        self.bufs = [None] * slots
        self.events = [None] * slots
        self.k = 0
        self.captured = []
        self.upload = {}

    def _upload_stream(self, device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        s = self.upload.get(idx)
        if s is None:
            s = self.upload[idx] = torch.cuda.Stream(device=idx)
        return s

    def stage(self, host_struct_array, device):
        nbytes = C.sizeof(host_struct_array)
        if _capturing():
            pin = torch.empty(max(nbytes, 16), dtype=torch.uint8).pin_memory()
            pin[:nbytes].numpy()[:] = memoryview(host_struct_array).cast("B")
            up = self._upload_stream(device)
            # allocated and filled on the upload stream: outside the capture (and
            # its private pool), finished before the captured kernels can run
            with torch.cuda.stream(up):
                dev = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
                _call("maeclip_memcpy_h2d", dev.data_ptr(), pin.data_ptr(), nbytes, up.cuda_stream)
            up.synchronize()
            self.captured.append((pin, dev))
            return dev
        k = self.k
        self.k = (k + 1) % len(self.bufs)
        if self.events[k] is not None:
            self.events[k].synchronize()
        buf = self.bufs[k]
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 4096), dtype=torch.uint8).pin_memory()
            self.bufs[k] = buf
        buf[:nbytes].numpy()[:] = memoryview(host_struct_array).cast("B")
        dev = buf[:nbytes].to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        return dev


_STAGER = PinnedStager()


class ReduceBatch:
    """Collects column reductions and runs them as ONE maeclip_colsum_multi launch."""

    def __init__(self):
        self.items = []

    def add(self, partial, scale=1.0, out=None):
        P, N = partial.shape
        if out is None:
            out = torch.empty((N,), device=partial.device, dtype=torch.float32)
        elif out.numel() != N or not out.is_contiguous():
            raise ValueError("ReduceBatch.add: out must be a dense [N] tensor")
        self.items.append((partial, out, scale))
        return out

    def flush(self):
        if not self.items:
            return
        n = len(self.items)
        host = (L.ColsumEntry * n)()
        start = 0
        for i, (part, out, scale) in enumerate(self.items):
            h = host[i]
            h.partial, h.out = part.data_ptr(), out.data_ptr()
            h.P, h.N = part.shape
            h.scale, h.accumulate, h.block_start = scale, 0, start
            start += (part.shape[1] + 63) // 64
        dev = _STAGER.stage(host, self.items[0][0].device)
        _call("maeclip_colsum_multi", dev.data_ptr(), host, n, _stream())
        self.items = []


class MultiTensorPlan:
    """Host + device entry arrays for one multi-tensor launch."""

    def __init__(self, entries, device):
        chunk = int(L.lib().maeclip_mt_chunk())
        n = len(entries)
        self.host = (L.MtEntry * n)()
        start = 0
        for i, e in enumerate(entries):
            h = self.host[i]
            h.p0, h.p1, h.p2, h.p3, h.p4 = e[:5]
            h.n = e[5]
            h.chunk_start = start
            start += (e[5] + chunk - 1) // chunk
        raw = bytes(self.host)
        self.dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.n = n


def cast_flat(src, dst, scale=1.0):
    """dst = scale * src elementwise (f32 <-> bf16, same numel, dense)."""
    _dev(src, dst)
    if src.numel() != dst.numel() or not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("cast_flat: dense tensors of equal size")
    _call("maeclip_cast_flat", src.data_ptr(), _dt(src), dst.data_ptr(), _dt(dst), src.numel(), float(scale),
          _stream())
    return dst


def cast_multi(plan: MultiTensorPlan):
    _call("maeclip_cast_multi", plan.dev.data_ptr(), plan.host, plan.n, _stream())


def adamw_multi(plan: MultiTensorPlan, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, step_ptr=None):
    """step: host step count t (>= 1), or step_ptr: device int64 holding t."""
    bc1 = 1.0 - beta1 ** max(step, 1)
    bc2 = 1.0 - beta2 ** max(step, 1)
    hp = L.AdamwHparams(lr=lr, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay, step_size=lr / bc1,
                        bc2_sqrt=bc2 ** 0.5, grad_scale=grad_scale, step_ptr=_ptr(step_ptr))
    _call("maeclip_adamw_multi", plan.dev.data_ptr(), plan.host, plan.n, C.byref(hp), _stream())
