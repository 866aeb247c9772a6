"""torch.autograd.Functions of the hot path, each a fixed sequence of
libmaeclip kernel launches (no torch compute kernels inside).

Granularity follows the fusion boundaries, not nn.Module boundaries: a whole
pre-LN transformer stack is ONE Function, so the residual-stream gradient, its
bf16 copy and the bias-gradient column partials flow from block to block
inside the backward without extra passes over HBM.

Reference ops replaced (file:line):
  TransformerStackFn  timm Block x depth (modules.py:17-19 -> timm 0.9.12) and
                      HF ViTMAELayer x decoder_depth (modeling_vit_mae.py:455-580)
  PatchTokensFn       timm PatchEmbed + _pos_embed (+ MAE visible-patch gather)
  EncoderHeadFn       timm global_pool="avg" + fc_norm; MAE mae_norm
  DecoderEmbedFn      HF decoder_embed + mask-token unshuffle + pos (:536-566)
  MaeHeadLossFn       HF decoder_norm + decoder_pred + loss (:568-578, :852-859)
  ProjectionHeadFn    modules.py:69-76 (always fp32)
  ClipLossFn          CLIP.py:34-43
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import kernels as K


def _reduce(part, out=None):
    return K.colsum_reduce(part, out=out)


# --------------------------------------------------------- gradient arena
# Data parallel (mae_clip_amd.distributed.DataParallel) keeps every trainable
# gradient in ONE flat fp32 buffer; the backward of each Function below writes
# a parameter's gradient straight into that parameter's slot, autograd adopts
# the slot as p.grad, and the bucketed all-reduce runs on slices of the flat
# buffer -- no flatten / unflatten copies. Without an arena (single GPU) every
# gradient is a fresh tensor as before.
_ARENA = [None]


def set_grad_arena(arena):
    """Called at the start of every forward: slots are handed out again from here."""
    _ARENA[0] = arena
    if arena is not None:
        arena.begin_forward()


def _arena():
    return _ARENA[0]


def gout(arena, p, shape=None):
    """Output buffer for p's gradient: its arena slot (a fresh view object, so
    autograd's AccumulateGrad adopts it without a copy) when p.grad is None and
    the slot has not been handed out since the forward, else a new tensor
    (gradient accumulation / a second use of p: autograd adds it)."""
    if arena is not None:
        v = arena.slot(p)
        if v is not None:
            return v if shape is None else v.view(shape)
    return torch.empty(shape if shape is not None else p.shape, device=p.device, dtype=torch.float32)


# ------------------------------------------------------------ side stream
_SIDE = {}


def side_stream(device) -> torch.cuda.Stream:
    """One extra HIP stream per device for work that is independent of the
    current stream's chain (weight gradients, the frozen text tower)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = _SIDE[idx] = torch.cuda.Stream(device=idx)
    return s


class WgradQueue:
    """Weight-gradient GEMMs of a transformer stack's backward.

    grouped (default): every dW = dy^T x of the stack is queued and join()
    computes them all in ONE maeclip_wgrad_grouped call on the current stream
    -- one persistent launch whose tiles (4 x layers problems) fill the 256 CUs
    without the fp32 split-K slab round trip that a single 768x3072 or
    512x2048 dW needs to occupy the chip (its inputs stay alive until then).
    Otherwise each dW runs as it becomes ready, on the side stream beside the
    dgrad -> LN -> attention chain (side=True) or inline. Inputs used on the
    side stream get record_stream() so the caching allocator does not hand
    their memory to the current stream while the side stream may still read
    it; join() makes the current stream wait for every queued dW.
    """

    def __init__(self, device, enabled=True, grouped=True):
        self.main = torch.cuda.current_stream(device)
        self.side = side_stream(device) if (enabled and not grouped) else None
        self.grouped = grouped
        self.items = []

    def wgrad(self, dy, x, out=None):
        if self.grouped:
            if out is None:
                out = torch.empty((dy.shape[1], x.shape[1]), device=dy.device, dtype=torch.float32)
            if self.items and self.items[0][0].shape[0] != dy.shape[0]:
                self.flush()
            self.items.append((dy, x, out))
            return out
        if self.side is None:
            return K.linear_wgrad(dy, x, out=out)
        M, N = dy.shape
        if out is None:
            out = torch.empty((N, x.shape[1]), device=dy.device, dtype=torch.float32)
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            K.linear_wgrad(dy, x, out=out)
        dy.record_stream(self.side)
        x.record_stream(self.side)
        out.record_stream(self.side)
        return out

    def flush(self):
        if self.items:
            K.wgrad_grouped(self.items)
            self.items = []

    def join(self):
        self.flush()
        if self.side is not None:
            self.main.wait_stream(self.side)


# ---------------------------------------------------------------- stacks
@dataclass
class StackSpec:
    B: int
    n: int
    D: int
    H: int
    eps: float
    dtype: torch.dtype              # compute dtype of GEMM operands / activations
    wT: list                        # per block: (qkv, proj, fc1, fc2) weights in `dtype`
    side: bool = True               # weight gradients on the side stream (when not grouped)
    grouped_wgrad: bool = True      # one grouped launch for all weight gradients of the stack
    w8: list = None                 # fp8 mode: per block ((W, W^T) fp8 operands) x (qkv, proj, fc1, fc2)


def _quant8(x, fmt, colsum):
    """fp8 operand of x made by a separate pass (its producer wrote none):
    fp8 blocks, or per-row scales for a launch with column sums (those run on
    the 256-row tile, which has no room for the block scales' LDS images)"""
    return K.quant_rows_fp8(x, fmt) if colsum is not None else K.quant_blocks_fp8(x, fmt)


def _fwd(x, w, w8, xq=None, q8=None, **kw):
    """Forward GEMM of a stack: bf16 / fp32 (w), or fp8 (w8 = (W, W^T)): x in
    e4m3 (xq: already quantised by its producer -- per token by a LayerNorm,
    fp8 blocks by a GEMM epilogue; else a pass here) times W (per output
    channel); q8: an Fp8Blocks the epilogue fills with the output's fp8 copy."""
    if w8 is None:
        return K.linear_fwd(x, w, q8=q8, **kw)
    kw.setdefault("out_dtype", x.dtype)
    xq = xq if xq is not None else _quant8(x, K.FP8_E4M3, kw.get("colsum"))
    return K.linear_fp8(xq, w8[0], q8=q8, **kw)


def _gfmt():
    """fp8 format of the gradient operands (config.fp8_grad_format)"""
    from . import config as CFG
    return K.FP8_E5M2 if getattr(CFG, "fp8_grad_format", "e4m3") == "e5m2" else K.FP8_E4M3


def _dgrad(dy, w, w8, dyq=None, q8=None, **kw):
    """dgrad GEMM dX = dY W: fp8 mode takes dY in config.fp8_grad_format
    (dyq: already quantised by its producer) times W^T (per input channel)."""
    if w8 is None:
        return K.linear_dgrad(dy, w, q8=q8, **kw)
    kw.setdefault("out_dtype", dy.dtype)
    dyq = dyq if dyq is not None else _quant8(dy, _gfmt(), kw.get("colsum"))
    return K.linear_fp8(dyq, w8[1], q8=q8, **kw)


def _b8(f8, M, D, fmt, dev):
    """Fp8Blocks for a GEMM epilogue to fill when its consumer GEMM runs in fp8."""
    return K.new_fp8_blocks(M, D, fmt, dev) if f8 is not None else None


def _attn_q8(f8, M, D, fmt, dev, bwd):
    """Fp8Blocks for the attention to fill (config.fp8_attn_q8), else None (the
    consumer GEMM's operand is then made by a standalone pass)"""
    from . import config as CFG
    return _b8(f8, M, D, fmt, dev) if CFG.fp8_attn_q8[1 if bwd else 0] else None


def _q8(f8, M, D, fmt, dev):
    """Fp8Rows for a LayerNorm to fill when its consumer GEMM runs in fp8."""
    return K.new_fp8_rows(M, D, fmt, dev) if f8 is not None else None


PER_BLOCK = 12  # n1w n1b qkvw qkvb projw projb n2w n2b fc1w fc1b fc2w fc2b


_MB_STREAMS = {}


def mb_stream(device, i):
    """Extra HIP stream i (>= 1) per device for micro-batch i of a stack."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, i)
    s = _MB_STREAMS.get(key)
    if s is None:
        s = _MB_STREAMS[key] = torch.cuda.Stream(device=idx)
    return s


class MicroBatches:
    """The stack's samples cut into S equal micro-batches, each issued on its
    own stream (micro-batch 0 on the current one). A kernel of one
    micro-batch fills the CUs the other's kernel leaves idle in its partial
    last round of tiles and around its launch, so the two chains overlap;
    every kernel still sees whole samples (attention) and whole 64-row groups
    (GEMM column-sum partials), so each micro-batch computes exactly the rows
    the whole-batch launch would (tools/mb_overlap.py: bitwise equal).
    Outputs are row slices of whole-batch buffers, so the grouped weight
    gradients and the column reductions run once on the whole batch."""

    def __init__(self, B, n, S, device):
        self.S = S
        self.Bs = B // S
        self.rows = [(i * self.Bs * n, (i + 1) * self.Bs * n) for i in range(S)]
        self.main = torch.cuda.current_stream(device)
        self.streams = [self.main] + [mb_stream(device, i) for i in range(1, S)]
        # stagger (A/B, MAECLIP_MB_STAGGER=k): micro-batch i > 0 starts a block only
        # after micro-batch i - 1 has issued k launches of it, so that different
        # kernels of the block (GEMM epilogues vs attention / LayerNorm) coincide
        self.stagger = int(os.environ.get("MAECLIP_MB_STAGGER", "0") or 0)
        self._ticks = 0
        self._gate = None

    def tick(self):
        """after each launch of a block: records the stagger gate on the
        micro-batch's stream after its k-th launch"""
        if self.stagger <= 0:
            return
        self._ticks += 1
        if self._ticks == self.stagger:
            self._gate = torch.cuda.Event()
            self._gate.record()

    def fork(self):
        for st in self.streams[1:]:
            st.wait_stream(self.main)

    def join(self):
        for st in self.streams[1:]:
            self.main.wait_stream(st)

    def each(self):
        """(index, row slice, batch slice) under each micro-batch's stream."""
        for i, st in enumerate(self.streams):
            r0, r1 = self.rows[i]
            _MB_ACTIVE[0] = i
            if self._gate is not None:
                st.wait_event(self._gate)
            self._ticks, self._gate = 0, None
            try:
                with torch.cuda.stream(st):
                    yield i, slice(r0, r1), slice(i * self.Bs, (i + 1) * self.Bs)
            finally:
                _MB_ACTIVE[0] = None


_MB_ACTIVE = [None]


def microbatch_active():
    """Index of the micro-batch whose launches are being issued (None outside
    MicroBatches.each): its kernels run concurrently with the other chain's
    (bench.py's launch timer then reports them as overlapped)."""
    return _MB_ACTIVE[0]


def microbatch_count(spec) -> int:
    """Micro-batches for a stack: CFG.stack_microbatches on the bf16 and fp8
    paths (the fp32 parity mode runs one), when every micro-batch keeps whole
    64-row groups of the GEMM column-sum partials (and of the fp8 blocks'
    scale layout)."""
    from . import config as CFG
    import os
    S = int(getattr(CFG, "stack_microbatches", 1) or 1)
    # A/B scans only: MAECLIP_MB_D<width> overrides the count for stacks of that width
    S = int(os.environ.get(f"MAECLIP_MB_D{spec.D}", S))
    if S <= 1 or spec.dtype != torch.bfloat16 or spec.B % S:
        return 1
    return S if (spec.B // S * spec.n) % 64 == 0 else 1


class TransformerStackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, spec: StackSpec, *params):
        B, n, D, H = spec.B, spec.n, spec.D, spec.H
        hd = D // H
        scale = hd ** -0.5
        T = spec.dtype
        M = B * n
        xi = x.reshape(M, D)
        dev = x.device
        S = microbatch_count(spec)
        if S > 1:
            return TransformerStackFn._forward_mb(ctx, xi, spec, params, S)
        saved = []
        for i, (wqkv, wproj, w1, w2) in enumerate(spec.wT):
            p = params[i * PER_BLOCK:(i + 1) * PER_BLOCK]
            n1w, n1b, _, bqkv, _, bproj, n2w, n2b, _, b1, _, b2 = p
            f8 = spec.w8[i] if spec.w8 is not None else (None,) * 4
            q1 = _q8(f8[0], M, D, K.FP8_E4M3, dev)
            h1, m1, r1, _, _ = K.ln_fwd(xi, n1w, n1b, spec.eps, out_dtype=T, q8=q1)
            qkv = _fwd(h1, wqkv, f8[0], xq=q1, bias=bqkv)
            del q1
            o8 = _attn_q8(f8[1], M, D, K.FP8_E4M3, dev, False)   # the proj GEMM's fp8 operand
            o, lse = K.attn_fwd(qkv, B, n, H, hd, scale, q8=o8)
            x1 = _fwd(o, wproj, f8[1], xq=o8, bias=bproj, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=xi)
            del o8
            q2 = _q8(f8[2], M, D, K.FP8_E4M3, dev)
            h2, m2, r2, _, _ = K.ln_fwd(x1, n2w, n2b, spec.eps, out_dtype=T, q8=q2)
            # fc1 epilogue: a = gelu(h), dgelu = gelu'(h) saved for the backward
            # (+ a's fp8 blocks for fc2 in fp8 mode)
            dgelu = torch.empty((M, w1.shape[0]), device=dev, dtype=T)
            a8 = _b8(f8[3], M, w1.shape[0], K.FP8_E4M3, dev)
            a = _fwd(h2, w1, f8[2], xq=q2, q8=a8, bias=b1, epilogue=K.EPI_GELU_D, aux_out=dgelu)
            del q2
            x2 = _fwd(a, w2, f8[3], xq=a8, bias=b2, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=x1)
            del a8
            saved.append([xi, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dgelu, a])
            xi = x2
        ctx.saved = saved
        ctx.spec = spec
        ctx.params = params
        ctx.arena = _arena()
        ctx.S = 1
        return xi.view(B, n, D)

    @staticmethod
    def _forward_mb(ctx, xi, spec, params, S):
        B, n, D, H = spec.B, spec.n, spec.D, spec.H
        hd = D // H
        scale = hd ** -0.5
        T = spec.dtype
        M = B * n
        dev = xi.device
        mb = MicroBatches(B, n, S, dev)
        e = lambda shape, dt=T: torch.empty(shape, device=dev, dtype=dt)
        saved = []
        # whole-batch buffers allocated on the current stream before the fork;
        # each micro-batch writes its rows on its own stream
        for wqkv, wproj, w1, w2 in spec.wT:
            F = w1.shape[0]
            saved.append([None, e((M, D)), e((M,), torch.float32), e((M,), torch.float32), e((M, 3 * D)),
                          e((M, D)), e((B, H, n), torch.float32), e((M, D), torch.float32), e((M, D)),
                          e((M,), torch.float32), e((M,), torch.float32), e((M, F)), e((M, F))])
        outs = [e((M, D), torch.float32) for _ in spec.wT]
        mb.fork()
        xin = [xi[slice(r0, r1)] for r0, r1 in mb.rows]
        # block by block, each micro-batch's launches on its stream in turn (the
        # captured graph then holds S interleaved chains the replay overlaps)
        Ms = M // S
        for i, (wqkv, wproj, w1, w2) in enumerate(spec.wT):
            p = params[i * PER_BLOCK:(i + 1) * PER_BLOCK]
            n1w, n1b, _, bqkv, _, bproj, n2w, n2b, _, b1, _, b2 = p
            _, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dgelu, a = saved[i]
            f8 = spec.w8[i] if spec.w8 is not None else (None,) * 4
            for mi, rs, bs in mb.each():
                xr = xin[mi]
                # fp8 mode: each micro-batch's fp8 operands (LayerNorm rows, fc1's blocks)
                q1 = _q8(f8[0], Ms, D, K.FP8_E4M3, dev)
                K.ln_fwd(xr, n1w, n1b, spec.eps, out_dtype=T, y_out=h1[rs], mean_out=m1[rs], rstd_out=r1[rs], q8=q1)
                mb.tick()
                _fwd(h1[rs], wqkv, f8[0], xq=q1, bias=bqkv, out=qkv[rs])
                mb.tick()
                o8 = _attn_q8(f8[1], Ms, D, K.FP8_E4M3, dev, False)
                K.attn_fwd(qkv[rs], mb.Bs, n, H, hd, scale, o_out=o[rs], lse_out=lse[bs], q8=o8)
                mb.tick()
                _fwd(o[rs], wproj, f8[1], xq=o8, bias=bproj, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=xr,
                     out=x1[rs])
                mb.tick()
                q2 = _q8(f8[2], Ms, D, K.FP8_E4M3, dev)
                K.ln_fwd(x1[rs], n2w, n2b, spec.eps, out_dtype=T, y_out=h2[rs], mean_out=m2[rs], rstd_out=r2[rs], q8=q2)
                mb.tick()
                a8 = _b8(f8[3], Ms, w1.shape[0], K.FP8_E4M3, dev)
                _fwd(h2[rs], w1, f8[2], xq=q2, q8=a8, bias=b1, epilogue=K.EPI_GELU_D, aux_out=dgelu[rs], out=a[rs])
                mb.tick()
                _fwd(a[rs], w2, f8[3], xq=a8, bias=b2, out_dtype=torch.float32, epilogue=K.EPI_RESID, resid=x1[rs],
                     out=outs[i][rs])
                xin[mi] = outs[i][rs]
        mb.join()
        for i in range(len(spec.wT)):
            saved[i][0] = xi if i == 0 else outs[i - 1]
        ctx.saved = saved
        ctx.spec = spec
        ctx.params = params
        ctx.arena = _arena()
        ctx.S = S
        return outs[-1].view(B, n, D)

    @staticmethod
    def backward(ctx, gy):
        if ctx.S > 1:
            return TransformerStackFn._backward_mb(ctx, gy)
        spec = ctx.spec
        B, n, D, H = spec.B, spec.n, spec.D, spec.H
        hd = D // H
        scale = hd ** -0.5
        T = spec.dtype
        bf = T == torch.bfloat16
        M = B * n
        params = ctx.params
        grads = [None] * len(params)
        rb = K.ReduceBatch()
        wq = WgradQueue(gy.device, spec.side, spec.grouped_wgrad)
        g = gy.reshape(M, D)
        if not g.is_contiguous():
            g = g.contiguous()
        gT = torch.empty((M, D), device=g.device, dtype=torch.bfloat16) if bf else None
        # fp8 copy of gT for the top fc2 dgrad: made with gT here (fp8 mode), then
        # by the LayerNorm backward that produces each next gT
        gq = _q8(spec.w8[-1][3], M, D, _gfmt(), g.device) if (bf and spec.w8 is not None) else None
        cpart = K.rows_colsum(g, out_bf16=gT, q8=gq)
        if not bf:
            gT = g
        for i in reversed(range(len(spec.wT))):
            wqkv, wproj, w1, w2 = spec.wT[i]
            f8 = spec.w8[i] if spec.w8 is not None else (None,) * 4
            p = params[i * PER_BLOCK:(i + 1) * PER_BLOCK]
            n1w, n2w = p[0], p[6]
            xi, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dgelu, a = ctx.saved[i]
            gi = [None] * PER_BLOCK
            ar = ctx.arena
            # mlp.fc2 (+ GELU backward fused into the dgrad epilogue: dA = (dy W2) * gelu'(h))
            gi[11] = rb.add(cpart, out=gout(ar, p[11]))
            dA_part = torch.empty((K.gemm_colsum_rows(M), w1.shape[0]), device=g.device, dtype=torch.float32)
            dA8 = _b8(f8[2], M, w1.shape[0], _gfmt(), g.device)   # fc1's dgrad operand (fp8 mode)
            dA = _dgrad(gT, w2, f8[3], dyq=gq, q8=dA8, epilogue=K.EPI_MUL_AUX, aux=dgelu, colsum=dA_part)
            gq = None
            gi[10] = wq.wgrad(gT, a, out=gout(ar, p[10]))
            del a, dgelu
            # mlp.fc1
            gi[9] = rb.add(dA_part, out=gout(ar, p[9]))
            dh2 = _dgrad(dA, w1, f8[2], dyq=dA8)
            del dA8
            gi[8] = wq.wgrad(dA, h2, out=gout(ar, p[8]))
            del dA
            # norm2 (+ residual gradient)
            q1 = _q8(f8[1], M, D, _gfmt(), g.device) if bf else None
            dx1, dx1T, pg, pb, pc = K.ln_bwd(dh2, x1, m2, r2, n2w, dres=g, want_bf16=bf, want_colsum=True, q8=q1)
            gi[6], gi[7] = rb.add(pg, out=gout(ar, p[6])), rb.add(pb, out=gout(ar, p[7]))
            if not bf:
                dx1T = dx1
            # attn.proj
            gi[5] = rb.add(pc, out=gout(ar, p[5]))
            dO = _dgrad(dx1T, wproj, f8[1], dyq=q1)
            del q1
            gi[4] = wq.wgrad(dx1T, o, out=gout(ar, p[4]))
            # attention
            dq8 = _attn_q8(f8[0], M, 3 * D, _gfmt(), g.device, True)   # the qkv dgrad's fp8 operand
            dqkv, qpart = K.attn_bwd(qkv, o, dO, lse, B, n, H, hd, scale, q8=dq8)
            del dO
            gi[3] = rb.add(qpart, out=gout(ar, p[3]))
            dh1 = _dgrad(dqkv, wqkv, f8[0], dyq=dq8)
            del dq8
            gi[2] = wq.wgrad(dqkv, h1, out=gout(ar, p[2]))
            del dqkv
            # norm1 (+ residual gradient)
            # the next (lower) block's fc2 dgrad reads dxT: quantised here when it is fp8
            f8n = (spec.w8[i - 1][3] if spec.w8 is not None and i > 0 else None)
            gq = _q8(f8n, M, D, _gfmt(), g.device) if bf else None
            dx, dxT, pg, pb, pc = K.ln_bwd(dh1, xi, m1, r1, n1w, dres=dx1, want_bf16=bf, want_colsum=True, q8=gq)
            gi[0], gi[1] = rb.add(pg, out=gout(ar, p[0])), rb.add(pb, out=gout(ar, p[1]))
            ctx.saved[i] = None
            g, gT, cpart = dx, (dxT if bf else dx), pc
            for j in range(PER_BLOCK):
                grads[i * PER_BLOCK + j] = gi[j].view(p[j].shape)
            del gi
        rb.flush()
        wq.join()
        ctx.saved = None
        return (g.view(B, n, D), None, *grads)

    @staticmethod
    def _backward_mb(ctx, gy):
        spec = ctx.spec
        S = ctx.S
        B, n, D, H = spec.B, spec.n, spec.D, spec.H
        hd = D // H
        scale = hd ** -0.5
        T = spec.dtype
        M = B * n
        dev = gy.device
        params = ctx.params
        grads = [None] * len(params)
        rb = K.ReduceBatch()
        wq = WgradQueue(dev, spec.side, spec.grouped_wgrad)
        mb = MicroBatches(B, n, S, dev)
        e = lambda shape, dt=T: torch.empty(shape, device=dev, dtype=dt)
        f32 = torch.float32
        Ms = M // S
        G = K.ln_bwd_partial_rows(Ms, D)       # LayerNorm partial rows per micro-batch
        GC = K.gemm_colsum_rows(M)              # GEMM column-sum partial rows (64-row groups)
        g = gy.reshape(M, D)
        if not g.is_contiguous():
            g = g.contiguous()
        gT = e((M, D))
        gq0 = _q8(spec.w8[-1][3], M, D, _gfmt(), dev) if spec.w8 is not None else None   # top fp8 operand
        cpart = K.rows_colsum(g, out_bf16=gT, q8=gq0)
        # whole-batch gradient buffers of every block, written per micro-batch
        bufs = []
        for wqkv, wproj, w1, w2 in spec.wT:
            F = w1.shape[0]
            bufs.append(dict(dA=e((M, F)), dA_part=e((GC, F), f32), dh2=e((M, D)), dx1=e((M, D), f32),
                             dx1T=e((M, D)), pg2=e((S * G, D), f32), pb2=e((S * G, D), f32),
                             pc2=e((S * G, D), f32), dO=e((M, D)), dqkv=e((M, 3 * D)), qpart=e((B, 3 * D), f32),
                             dh1=e((M, D)), dx=e((M, D), f32), dxT=e((M, D)), pg1=e((S * G, D), f32),
                             pb1=e((S * G, D), f32), pc1=e((S * G, D), f32)))
        mb.fork()
        # per micro-batch: (f32 residual gradient, its bf16 copy, the copy's fp8
        # rows from the LayerNorm backward that made it -- fp8 mode)
        gin = [(g[slice(r0, r1)], gT[slice(r0, r1)],
                None if gq0 is None else K.Fp8Rows(gq0.q[r0:r1], gq0.s[r0:r1], gq0.fmt)) for r0, r1 in mb.rows]
        for i in reversed(range(len(spec.wT))):
            wqkv, wproj, w1, w2 = spec.wT[i]
            n1w, n2w = params[i * PER_BLOCK], params[i * PER_BLOCK + 6]
            xi, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dgelu, a = ctx.saved[i]
            b = bufs[i]
            f8 = spec.w8[i] if spec.w8 is not None else (None,) * 4
            f8n = spec.w8[i - 1][3] if spec.w8 is not None and i > 0 else None
            for mi, rs, bs in mb.each():
                gs, gTs, gq = gin[mi]
                ps = slice(mi * G, (mi + 1) * G)
                cs = slice(rs.start // 64, rs.stop // 64)
                dA8 = _b8(f8[2], Ms, w1.shape[0], _gfmt(), dev)
                _dgrad(gTs, w2, f8[3], dyq=gq, q8=dA8, epilogue=K.EPI_MUL_AUX, aux=dgelu[rs],
                       colsum=b["dA_part"][cs], out=b["dA"][rs])
                mb.tick()
                _dgrad(b["dA"][rs], w1, f8[2], dyq=dA8, out=b["dh2"][rs])
                mb.tick()
                q1 = _q8(f8[1], Ms, D, _gfmt(), dev)
                K.ln_bwd(b["dh2"][rs], x1[rs], m2[rs], r2[rs], n2w, dres=gs, want_bf16=True, want_colsum=True,
                         dx_out=b["dx1"][rs], dxb_out=b["dx1T"][rs], pg_out=b["pg2"][ps], pb_out=b["pb2"][ps],
                         pc_out=b["pc2"][ps], q8=q1)
                mb.tick()
                _dgrad(b["dx1T"][rs], wproj, f8[1], dyq=q1, out=b["dO"][rs])
                mb.tick()
                dq8 = _attn_q8(f8[0], Ms, 3 * D, _gfmt(), dev, True)
                K.attn_bwd(qkv[rs], o[rs], b["dO"][rs], lse[bs], mb.Bs, n, H, hd, scale,
                           dqkv_out=b["dqkv"][rs], part_out=b["qpart"][bs], q8=dq8)
                mb.tick()
                _dgrad(b["dqkv"][rs], wqkv, f8[0], dyq=dq8, out=b["dh1"][rs])
                mb.tick()
                gq = _q8(f8n, Ms, D, _gfmt(), dev)
                K.ln_bwd(b["dh1"][rs], xi[rs], m1[rs], r1[rs], n1w, dres=b["dx1"][rs], want_bf16=True,
                         want_colsum=True, dx_out=b["dx"][rs], dxb_out=b["dxT"][rs], pg_out=b["pg1"][ps],
                         pb_out=b["pb1"][ps], pc_out=b["pc1"][ps], q8=gq)
                gin[mi] = (b["dx"][rs], b["dxT"][rs], gq)
        mb.join()
        ar = ctx.arena
        for i in reversed(range(len(spec.wT))):
            p = params[i * PER_BLOCK:(i + 1) * PER_BLOCK]
            xi, h1, m1, r1, qkv, o, lse, x1, h2, m2, r2, dgelu, a = ctx.saved[i]
            b = bufs[i]
            gi = [None] * PER_BLOCK
            gi[11] = rb.add(cpart, out=gout(ar, p[11]))
            gi[10] = wq.wgrad(gT, a, out=gout(ar, p[10]))
            gi[9] = rb.add(b["dA_part"], out=gout(ar, p[9]))
            gi[8] = wq.wgrad(b["dA"], h2, out=gout(ar, p[8]))
            gi[6], gi[7] = rb.add(b["pg2"], out=gout(ar, p[6])), rb.add(b["pb2"], out=gout(ar, p[7]))
            gi[5] = rb.add(b["pc2"], out=gout(ar, p[5]))
            gi[4] = wq.wgrad(b["dx1T"], o, out=gout(ar, p[4]))
            gi[3] = rb.add(b["qpart"], out=gout(ar, p[3]))
            gi[2] = wq.wgrad(b["dqkv"], h1, out=gout(ar, p[2]))
            gi[0], gi[1] = rb.add(b["pg1"], out=gout(ar, p[0])), rb.add(b["pb1"], out=gout(ar, p[1]))
            gT, cpart = b["dxT"], b["pc1"]
            for j in range(PER_BLOCK):
                grads[i * PER_BLOCK + j] = gi[j].view(p[j].shape)
        rb.flush()
        wq.join()
        g = bufs[0]["dx"]
        ctx.saved = None
        return (g.view(B, n, D), None, *grads)


# ------------------------------------------------------------ patch embed
@dataclass
class PatchSpec:
    B: int
    L: int
    keep: int
    p: int
    kpad: int
    dtype: torch.dtype
    w_T: torch.Tensor        # [D, kpad] patch-embed weight in `dtype`


class PatchTokensFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, ids_shuffle, ids_restore, spec: PatchSpec, w, b, cls, pos):
        Xp = K.patch_gather(img, ids_shuffle, spec.keep, spec.p, spec.kpad, spec.dtype)
        Y = K.linear_fwd(Xp, spec.w_T, b, out_dtype=torch.float32)
        x = K.tokens_fwd(Y, ids_shuffle, pos.view(-1, pos.shape[-1]), cls.view(-1), spec.B, spec.L, spec.keep)
        ctx.save = (Xp, ids_restore)
        ctx.spec = spec
        ctx.wshape = w.shape
        ctx.params = (w, b, cls, pos)
        ctx.arena = _arena()
        return x

    @staticmethod
    def backward(ctx, gx):
        spec = ctx.spec
        Xp, ids_restore = ctx.save
        gx = gx.contiguous()
        w, b, cls, pos = ctx.params
        ar = ctx.arena
        D = pos.shape[-1]
        dY, dpos, dcls = K.tokens_bwd(gx, ids_restore, spec.B, spec.L, spec.keep, spec.dtype,
                                      dpos=gout(ar, pos, (spec.L + 1, D)), dcls=gout(ar, cls, (D,)))
        Kreal = ctx.wshape[1] * ctx.wshape[2] * ctx.wshape[3]
        dWo = gout(ar, w, (ctx.wshape[0], Kreal))
        if Kreal != spec.kpad:
            dWo.copy_(K.linear_wgrad(dY, Xp)[:, :Kreal])
        else:
            K.linear_wgrad(dY, Xp, out=dWo)
        db = _reduce(K.rows_colsum(dY), out=gout(ar, b))
        return None, None, None, None, dWo.view(ctx.wshape), db, dcls.view(1, 1, D), dpos.view(1, -1, D)


# ------------------------------------------------------- encoder outputs
class EncoderHeadFn(torch.autograd.Function):
    """features = fc_norm(mean_{t>=1} x[:, t]) ; latent = mae_norm(x) (optional)."""

    @staticmethod
    def forward(ctx, x, latent_dtype, fcn_w, fcn_b, mn_w, mn_b):
        B, n, D = x.shape
        pooled = K.pool_fwd(x)
        feat, fm, fr, _, _ = K.ln_fwd(pooled, fcn_w, fcn_b, 1e-6, out_dtype=torch.float32)
        ctx.mae = mn_w is not None
        latent = None
        if ctx.mae:
            latent, lm, lr, _, _ = K.ln_fwd(x.view(B * n, D), mn_w, mn_b, 1e-6, out_dtype=latent_dtype)
            ctx.lstats = (lm, lr)
        ctx.save = (x, pooled, fm, fr)
        ctx.w = (fcn_w, mn_w)
        ctx.b = (fcn_b, mn_b)
        ctx.arena = _arena()
        if latent is None:
            return feat
        return feat, latent

    @staticmethod
    def backward(ctx, gfeat, glatent=None):
        x, pooled, fm, fr = ctx.save
        fcn_w, mn_w = ctx.w
        B, n, D = x.shape
        dpooled, _, pg, pb, _ = K.ln_bwd(gfeat.contiguous(), pooled, fm, fr, fcn_w)
        fcn_b, mn_b = ctx.b
        ar = ctx.arena
        g_fw, g_fb = _reduce(pg, out=gout(ar, fcn_w)), _reduce(pb, out=gout(ar, fcn_b))
        g_mw = g_mb = None
        if ctx.mae and glatent is not None:
            # the avg-pool backward rides in the mae_norm LN backward as its
            # residual gradient (no [B, n, D] pool-gradient tensor in HBM)
            lm, lr = ctx.lstats
            dx2, _, pg2, pb2, _ = K.ln_bwd(glatent.contiguous(), x.view(B * n, D), lm, lr, mn_w,
                                           dres_pool=dpooled, pool_n=n)
            dx = dx2.view(B, n, D)
            g_mw, g_mb = _reduce(pg2, out=gout(ar, mn_w)), _reduce(pb2, out=gout(ar, mn_b))
        else:
            dx = K.pool_bwd(dpooled, n)
        return dx, None, g_fw, g_fb, g_mw, g_mb


# ------------------------------------------------------------ MAE decoder
@dataclass
class DecSpec:
    B: int
    L: int
    keep: int
    dtype: torch.dtype
    w_T: torch.Tensor        # decoder_embed weight in dtype


class DecoderEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, latent, ids_shuffle, ids_restore, spec: DecSpec, w, b, mask_token, pos):
        y = K.linear_fwd(latent, spec.w_T, b, out_dtype=torch.float32)
        xd = K.unshuffle_fwd(y, ids_restore, mask_token.view(-1), pos.view(-1, pos.shape[-1]), spec.B, spec.L,
                             spec.keep)
        ctx.save = (latent, ids_restore)
        ctx.spec = spec
        ctx.params = (w, b, mask_token)
        ctx.arena = _arena()
        return xd

    @staticmethod
    def backward(ctx, gxd):
        spec = ctx.spec
        latent, ids_restore = ctx.save
        dy, dmask_part, cs = K.unshuffle_bwd(gxd.contiguous(), ids_restore, spec.B, spec.L, spec.keep, spec.dtype)
        w, b, mask_token = ctx.params
        ar = ctx.arena
        dlatent = K.linear_dgrad(dy, spec.w_T)
        dW = K.linear_wgrad(dy, latent, out=gout(ar, w))
        db = _reduce(cs, out=gout(ar, b))
        dmask = _reduce(dmask_part, out=gout(ar, mask_token, (mask_token.shape[-1],)))
        return dlatent, None, None, None, dW, db, dmask.view(1, 1, -1), None


@dataclass
class MaeHeadSpec:
    p: int
    norm_pix: bool
    mask_count: float
    loss_scale: float
    dtype: torch.dtype
    w_T: torch.Tensor        # decoder_pred weight in dtype, [Npad, Dd] (zero rows past p*p*C)
    b_pad: torch.Tensor = None   # decoder_pred bias padded to Npad (None: no padding)


class MaeHeadLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xd, img, mask, spec: MaeHeadSpec, dn_w, dn_b, wp, bp):
        B, n, Dd = xd.shape
        x2 = xd.view(B * n, Dd)
        h, m, r, _, _ = K.ln_fwd(x2, dn_w, dn_b, 1e-6, out_dtype=spec.dtype)
        pred = K.linear_fwd(h, spec.w_T, bp if spec.b_pad is None else spec.b_pad)
        row = K.mae_loss_fwd(pred, img, mask, spec.p, spec.norm_pix)
        loss = K.colsum_reduce(row.view(-1, 1), scale=1.0 / spec.mask_count).view(())
        ctx.save = (x2, h, m, r, pred, img, mask)
        ctx.spec = spec
        ctx.dn_w = dn_w
        ctx.shape = xd.shape
        ctx.P = wp.shape[0]
        ctx.params = (dn_w, dn_b, wp, bp)
        ctx.arena = _arena()
        return loss

    @staticmethod
    def backward(ctx, gl):
        spec = ctx.spec
        x2, h, m, r, pred, img, mask = ctx.save
        dpred, cs = K.mae_loss_bwd(pred, img, mask, spec.p, spec.norm_pix, gl.contiguous(), spec.mask_count,
                                   spec.loss_scale)
        dn_w, dn_b, wp, bp = ctx.params
        ar = ctx.arena
        dh = K.linear_dgrad(dpred, spec.w_T)
        dWp = gout(ar, wp)
        if dpred.shape[1] != ctx.P:      # padded pred rows (patch 14): slice back
            dWp.copy_(K.linear_wgrad(dpred, h)[:ctx.P])
            dbp = _reduce(cs[:, :ctx.P].contiguous() if cs.shape[1] != ctx.P else cs, out=gout(ar, bp))
        else:
            K.linear_wgrad(dpred, h, out=dWp)
            dbp = _reduce(cs, out=gout(ar, bp))
        dx, _, pg, pb, _ = K.ln_bwd(dh, x2, m, r, ctx.dn_w)
        return (dx.view(ctx.shape), None, None, None, _reduce(pg, out=gout(ar, dn_w)), _reduce(pb, out=gout(ar, dn_b)),
                dWp, dbp)


# --------------------------------------------------------- projection head
@dataclass
class ProjSpec:
    p_drop: float
    seed: int
    step_ptr: torch.Tensor = None   # device step counter (dropout mask of the current step)
    bwd_step_ptr: torch.Tensor = None   # the same step's value as the backward will find it (snapshot slot)


class ProjectionHeadFn(torch.autograd.Function):
    """modules.py:69-76 in fp32: z = dropout(fc(gelu(proj(x)))) + proj(x); LN(z)."""

    @staticmethod
    def forward(ctx, x, spec: ProjSpec, wp, bp, wf, bf, lw, lb):
        x = x.contiguous() if x.stride(-1) != 1 else x
        Bn, P = x.shape[0], wp.shape[0]
        pre = torch.empty((Bn, P), device=x.device, dtype=torch.float32)
        g = K.linear_fwd(x, wp, bp, epilogue=K.EPI_GELU, aux_out=pre)
        f = K.linear_fwd(g, wf, bf)
        out, m, r, _, z = K.ln_fwd(f, lw, lb, 1e-5, out_dtype=torch.float32, res=pre, in_dropout=spec.p_drop,
                                   seed_in=spec.seed, xsum=True, step_ptr=spec.step_ptr)
        ctx.save = (x, pre, g, z, m, r)
        ctx.w = (wp, wf, lw)
        ctx.params = (wp, bp, wf, bf, lw, lb)
        ctx.arena = _arena()
        ctx.spec = spec
        # the step counter advances at the end of the forward: the backward
        # re-draws this forward's dropout mask from a snapshot of the step
        ctx.step_snap = None
        if spec.step_ptr is not None and spec.p_drop > 0:
            ctx.step_snap = spec.bwd_step_ptr if spec.bwd_step_ptr is not None else spec.step_ptr.clone()
        return out

    @staticmethod
    def backward(ctx, gout_):
        x, pre, g, z, m, r = ctx.save
        wp, wf, lw = ctx.w
        spec = ctx.spec
        wp_, bp_, wf_, bf_, lw_, lb_ = ctx.params
        ar = ctx.arena
        dz, _, pg, pb, _ = K.ln_bwd(gout_.contiguous(), z, m, r, lw)
        df = K.dropout(dz, spec.p_drop, spec.seed, step_ptr=ctx.step_snap) if spec.p_drop > 0 else dz
        dwf = K.linear_wgrad(df, g, out=gout(ar, wf_))
        dbf = _reduce(K.rows_colsum(df), out=gout(ar, bf_))
        dpre = K.linear_dgrad(df, wf, out_dtype=torch.float32, epilogue=K.EPI_DGELU, aux=pre, resid=dz)
        dwp = K.linear_wgrad(dpre, x, out=gout(ar, wp_))
        dbp = _reduce(K.rows_colsum(dpre), out=gout(ar, bp_))
        dx = K.linear_dgrad(dpre, wp, out_dtype=torch.float32)
        return dx, None, dwp, dbp, dwf, dbf, _reduce(pg, out=gout(ar, lw_)), _reduce(pb, out=gout(ar, lb_))


# ------------------------------------------------------------- CLIP loss
class ClipLossFn(torch.autograd.Function):
    """CLIP.py:34-43 on the fused fp32 kernel (the gradients come out of the
    same call; the backward only scales them by grad_output).

    group (data parallel, world > 1): the local [B, P] embeddings of every rank
    are all-gathered in rank order (the global contrastive denominator, SURVEY
    §8e), every rank evaluates the loss of the gathered batch and asks the
    kernel for the gradient of its own B rows only -- so a SUM all-reduce of
    the parameter gradients is the exact global-batch gradient."""

    @staticmethod
    def forward(ctx, I, T, temperature, group=None):
        I = I.contiguous()
        T = T.contiguous()
        rows = None
        if group is not None:
            from .distributed import all_gather_rows, world_rank, check_equal_rows
            world, rank = world_rank(group)
            if world > 1:
                B = I.shape[0]
                check_equal_rows(B, group, I.device)
                I = all_gather_rows(I, group)
                T = all_gather_rows(T, group)
                rows = (rank * B, B)
        loss, dI, dT = K.clip_loss(I, T, temperature, want_grad=True, grad_rows=rows)
        ctx.grads = (dI, dT)
        return loss

    @staticmethod
    def backward(ctx, gl):
        dI, dT = ctx.grads
        ctx.grads = None
        # scaled in place by the device grad_output: one launch, no host sync
        K.scale_by_scalar(gl.reshape(1).contiguous(), 1.0, dI, dT, dI, dT)
        return dI, dT, None, None


class CombineLossFn(torch.autograd.Function):
    """loss = clip + w * mae on device scalars (one launch; backward: grad_output
    to the CLIP term as is, w * grad_output to the MAE term in one launch)."""

    @staticmethod
    def forward(ctx, clip, mae, w):
        ctx.w = float(w)
        return K.scalar_axpy(clip, mae, w)

    @staticmethod
    def backward(ctx, gl):
        g = gl.reshape(1).contiguous()
        gm, _ = K.scale_by_scalar(g, ctx.w, out_x=torch.empty((), device=g.device, dtype=torch.float32))
        return gl, gm, None
