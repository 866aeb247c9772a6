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


class DataParallel:
    """Gradient synchroniser for a model replicated on every rank.

    bucket_mb: gradient bytes per all-reduce. xGMI is point-to-point (7 links x
    ~153 GB/s per MI355X), so a ring all-reduce is per-link bound; 64 MB buckets
    keep RCCL at full link rate while letting the first buckets start while the
    backward of the earlier layers is still running.
    """

    def __init__(self, model, group=None, bucket_mb=64.0, broadcast=True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        model.process_group = group if group is not None else dist.group.WORLD
        self.params = [p for p in model.parameters() if p.requires_grad]
        if broadcast:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t, src=0, group=group)
        # buckets in reverse registration order (~ the order grads become ready)
        cap = int(bucket_mb * 2 ** 20)
        self.buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            nb = p.numel() * p.element_size()
            if cur and size + nb > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self._pending = [0] * len(self.buckets)
        self._works = []
        self._flats = [None] * len(self.buckets)
        self.overlap = True
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _on_grad(self, p):
        if not self.overlap:
            return
        i = self._bucket_of[id(p)]
        self._pending[i] += 1
        if self._pending[i] == len(self.buckets[i]):
            self._launch(i)

    def _launch(self, i):
        grads = [p.grad for p in self.buckets[i]]
        flat = torch._utils._flatten_dense_tensors(grads)
        self._flats[i] = flat
        self._works.append((i, dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)))

    def sync_gradients(self):
        """Finish (or, with overlap off, perform) the SUM all-reduce of all grads."""
        launched = {i for i, _ in self._works}
        for i in range(len(self.buckets)):
            if i not in launched:
                if any(p.grad is None for p in self.buckets[i]):
                    for p in self.buckets[i]:
                        if p.grad is None:
                            p.grad = torch.zeros_like(p)
                self._launch(i)
        for i, w in self._works:
            w.wait()
            grads = [p.grad for p in self.buckets[i]]
            # one multi-tensor copy per bucket (not one launch per parameter)
            torch._foreach_copy_(grads, torch._utils._unflatten_dense_tensors(self._flats[i], grads))
        self._works = []
        self._flats = [None] * len(self.buckets)
        self._pending = [0] * len(self.buckets)
