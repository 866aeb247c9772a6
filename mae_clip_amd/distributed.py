"""Data parallelism over the GPUs of one node: one process per GPU,
torch.distributed with backend "nccl" (= RCCL over xGMI on ROCm).

The reference has no distributed code; this is the single
parallel strategy of the build:
  * forward : all_gather of the fp32 projection embeddings [B_local, 256] so the
              soft-target contrastive loss (CLIP.py:34-43) sees the global batch;
              every rank evaluates the full N x N loss redundantly;
  * backward: the gather's backward keeps the local row slice (exact: the loss
              is identical on every rank), the MAE term is scaled by 1/world in
              its kernel, and a SUM all-reduce of parameter gradients (bucketed,
              launched from per-parameter hooks while the backward is still
              running) gives the exact global-batch gradient.
Tested with the gloo backend on CPU (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world_rank(group=None):
    return dist.get_world_size(group), dist.get_rank(group)


def _staged(group, t):
    """gloo moves host memory: collectives on device tensors go through a CPU copy."""
    return dist.get_backend(group) == "gloo" and t.is_cuda


def all_gather_rows(x, group=None):
    """[B, ...] on every rank -> [world*B, ...] in rank order (no autograd)."""
    world = dist.get_world_size(group)
    x = x.detach().contiguous()
    if _staged(group, x):
        parts = [torch.empty_like(x, device="cpu") for _ in range(world)]
        dist.all_gather(parts, x.cpu(), group=group)
        return torch.cat(parts).to(x.device)
    out = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


_CTRL = {}


def control_group(group=None, create=False):
    """A gloo group over the same ranks as `group`, for host-side control
    messages (batch-size checks): a collective on it moves CPU memory only, so
    it never synchronises the host with the GPU stream. None for a group that
    is already gloo, and for one whose control group was never created.

    dist.new_group must be entered by EVERY rank of the default group, so the
    group is only ever created eagerly (create=True), by DataParallel.__init__
    over the whole world, where every rank constructs one; a subgroup gets
    none (check_equal_rows then all-reduces on the group itself)."""
    key = group if group is not None else dist.group.WORLD
    if dist.get_backend(group) == "gloo":
        return None
    if key not in _CTRL and create:
        _CTRL[key] = dist.new_group(ranks=dist.get_process_group_ranks(key), backend="gloo")
    return _CTRL.get(key)


def check_equal_rows(n, group=None, device=None):
    """Raise if the ranks hold different local batch sizes.

    all_gather_into_tensor and the gradient row slice (rank * B, B) of the
    sharded CLIP loss both assume every rank has the same B; a ragged last
    batch (the reference's DataLoader keeps it, main.py:42-47) would otherwise
    hang or fail inside RCCL. One MAX all-reduce of (B, -B) per eager step, on
    the host over the gloo control group (no device sync: the host keeps
    running ahead of the GPU); skipped under graph capture (a captured step has
    fixed shapes on every rank by construction)."""
    if device is not None and device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        return
    t = torch.tensor([n, -n], dtype=torch.int64)
    ctrl = control_group(group)
    if ctrl is None and dist.get_backend(group) != "gloo" and device is not None:
        t = t.to(device)   # no control group (a subgroup): the device group itself
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl if ctrl is not None else group)
    hi, lo = int(t[0]), -int(t[1])
    if hi != lo:
        raise RuntimeError(f"data parallel: ranks hold different local batch sizes ({lo}..{hi}); "
                           "use drop_last=True or pad the last batch so every rank has the same B")


def _cast(src, dst):
    """dtype conversion of a bucket: the libmaeclip kernel on the device; on
    the CPU (the gloo tests drive DataParallel with the oracle's CPU modules)
    a host copy."""
    if src.is_cuda:
        from . import kernels as K
        K.cast_flat(src, dst)
    else:
        dst.copy_(src)


class GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.rank, ctx.n = dist.get_rank(group), x.shape[0]
        return all_gather_rows(x, group)

    @staticmethod
    def backward(ctx, g):
        return g.narrow(0, ctx.rank * ctx.n, ctx.n), None


def gather_rows(x, group=None):
    """all_gather along dim 0 with a backward that returns the local slice."""
    return GatherRowsFn.apply(x, group)


class GradArena:
    """All trainable gradients in one flat fp32 buffer, laid out in reverse
    registration order (~ the order the backward produces them), so that every
    all-reduce bucket is one contiguous slice. slot(p) hands a Function's
    backward a fresh view of p's range to write the gradient into."""

    def __init__(self, params, device):
        self.params = list(params)
        self.offsets = {}
        off = 0
        for p in self.params:
            self.offsets[id(p)] = (off, p.numel(), tuple(p.shape))
            # slots start on 16-B boundaries (the flat cast / reduction kernels
            # take vector accesses); the padding stays zero and sums to zero
            off += (p.numel() + 3) // 4 * 4
        self.flat = torch.zeros(off, device=device, dtype=torch.float32)

        # parameters whose slot has been handed out since the last forward
        # (begin_forward): a parameter that reaches several backward Functions
        # (tied weights, two forwards sharing one backward) gets its slot only
        # once -- autograd sums the incoming gradients before AccumulateGrad,
        # and two aliases of one buffer would sum to 2*g2 instead of g1+g2
        self.handed = set()

    def begin_forward(self):
        self.handed.clear()

    def view(self, p):
        off, n, shape = self.offsets[id(p)]
        return self.flat[off:off + n].view(shape)

    def slot(self, p):
        e = self.offsets.get(id(p))
        if e is None or p.grad is not None or p.dtype != torch.float32 or id(p) in self.handed:
            return None
        self.handed.add(id(p))
        return self.view(p)

    def owns(self, p):
        g = p.grad
        return g is not None and g.data_ptr() == self.flat.data_ptr() + 4 * self.offsets[id(p)][0]


class DataParallel:
    """Gradient synchroniser for a model replicated on every rank.

    The gradients live in a GradArena: the product's autograd Functions write
    each parameter's gradient directly into its slot (autograd adopts the slot
    as p.grad), so a bucket is all-reduced in place on a slice of the flat
    buffer -- no flatten / unflatten copies. Gradients produced elsewhere (the
    CPU oracle modules of the gloo tests, gradient accumulation) are copied
    into their slots first and back afterwards.

    bucket_mb: gradient bytes per all-reduce. xGMI is point-to-point (7 links x
    ~153 GB/s per MI355X), so a ring all-reduce is per-link bound; 64 MB buckets
    keep RCCL at full link rate while letting the first buckets start while the
    backward of the earlier layers is still running.
    """

    def __init__(self, model, group=None, bucket_mb=64.0, broadcast=True, grad_dtype=torch.float32, tail_mb=32.0):
        """grad_dtype=torch.bfloat16 (opt-in): each bucket is cast to bf16, SUM-
        all-reduced in bf16 (half the xGMI bytes: 225 instead of 449 MB per step
        at ViT-B MAE+CLIP) and cast back into the fp32 arena; the sum carries
        bf16 rounding (tests/test_distributed_cpu.py bounds the deviation)."""
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("DataParallel: grad_dtype must be torch.float32 or torch.bfloat16")
        self.model = model
        self.group = group
        self.grad_dtype = grad_dtype
        self.world = dist.get_world_size(group)
        model.process_group = group if group is not None else dist.group.WORLD
        if group is None or group == dist.group.WORLD:
            control_group(group, create=True)   # collective over the world: every rank constructs a DataParallel
        self.params = [p for p in model.parameters() if p.requires_grad]
        if broadcast:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    if _staged(group, t):
                        h = t.detach().cpu()
                        dist.broadcast(h, src=0, group=group)
                        t.copy_(h)
                    else:
                        dist.broadcast(t, src=0, group=group)
        order = list(reversed(self.params))
        self.arena = GradArena(order, self.params[0].device)
        if hasattr(model, "grad_arena"):
            model.grad_arena = self.arena
        # buckets = contiguous arena ranges in reverse registration order, cut
        # from the END of the arena: the last bucket holds the gradients the
        # backward produces last (the bottom encoder chunk and the patch
        # embedding), whose all-reduce no later backward work can hide, so it
        # is capped at tail_mb; the others at bucket_mb
        cap = int(bucket_mb * 2 ** 20)
        tcap = int(min(tail_mb, bucket_mb) * 2 ** 20)
        rev, cur, size = [], [], 0
        for p in reversed(order):
            nb = p.numel() * 4
            if cur and size + nb > (tcap if not rev else cap):
                rev.append(cur[::-1])
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            rev.append(cur[::-1])
        self.buckets = rev[::-1]
        self.ranges = []
        for b in self.buckets:
            o0 = self.arena.offsets[id(b[0])][0]
            o1 = self.arena.offsets[id(b[-1])][0] + b[-1].numel()
            self.ranges.append((o0, o1))
        self._bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        # bf16 reduction buffers (one per bucket, allocated once)
        self._low = ([torch.empty(o1 - o0, device=self.arena.flat.device, dtype=torch.bfloat16)
                      for o0, o1 in self.ranges] if grad_dtype == torch.bfloat16 else None)
        self._pending = [0] * len(self.buckets)
        self._works = []
        self._copied = [[] for _ in self.buckets]
        self.overlap = True
        self.adopted = 0      # gradients that arrived already in their arena slot (last step)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _on_grad(self, p):
        if not self.overlap:
            return
        i = self._bucket_of[id(p)]
        self._pending[i] += 1
        if self._pending[i] == len(self.buckets[i]):
            self._launch(i)

    def _launch(self, i):
        copied = []
        for p in self.buckets[i]:
            if p.grad is None:
                self.arena.view(p).zero_()
                p.grad = self.arena.view(p)
            elif self.arena.owns(p):
                self.adopted += 1
            else:
                self.arena.view(p).copy_(p.grad)
                copied.append(p)
        self._copied[i] = copied
        o0, o1 = self.ranges[i]
        buf = self.arena.flat[o0:o1]
        if self._low is not None:
            _cast(buf, self._low[i])
            buf = self._low[i]
        if _staged(self.group, buf):
            host = buf.cpu()
            w = dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._works.append((i, w, host))
        else:
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._works.append((i, w, None))

    def sync_gradients(self):
        """Finish (or, with overlap off, perform) the SUM all-reduce of all grads."""
        launched = {i for i, _, _ in self._works}
        for i in range(len(self.buckets)):
            if i not in launched:
                self._launch(i)
        for i, w, host in self._works:
            w.wait()
            o0, o1 = self.ranges[i]
            if host is not None:
                (self._low[i] if self._low is not None else self.arena.flat[o0:o1]).copy_(host)
            if self._low is not None:
                _cast(self._low[i], self.arena.flat[o0:o1])
            for p in self._copied[i]:
                p.grad.copy_(self.arena.view(p))
        self._works = []
        self._copied = [[] for _ in self.buckets]
        self._pending = [0] * len(self.buckets)

    def reset_stats(self):
        self.adopted = 0
