"""Fused multi-tensor AdamW on the libmaeclip kernel.

Same update as torch.optim.AdamW (main.py:101-103: lr 1e-3, weight_decay 1e-3,
betas (0.9, 0.999), eps 1e-8), one kernel launch for all parameters. It
optionally refreshes a model's bf16 weight shadows in the same pass.
"""
from __future__ import annotations

import torch

from . import kernels as K
from . import _lib as L


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._pinned = [None, None]
        self._events = [None, None]
        self._flip = 0

    def _plan(self, entries, device):
        """Entry array staged through alternating pinned buffers (async H2D)."""
        chunk = int(L.lib().maeclip_mt_chunk())
        n = len(entries)
        host = (L.MtEntry * n)()
        start = 0
        for i, e in enumerate(entries):
            h = host[i]
            h.p0, h.p1, h.p2, h.p3, h.p4 = e[:5]
            h.n = e[5]
            h.chunk_start = start
            start += (e[5] + chunk - 1) // chunk
        nbytes = C_sizeof(host)
        k = self._flip
        self._flip ^= 1
        if self._events[k] is not None:
            self._events[k].synchronize()  # the H2D copy that last read this buffer is done
        buf = self._pinned[k]
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
            self._pinned[k] = buf
        buf[:nbytes].numpy()[:] = memoryview(host).cast("B")
        dev = buf[:nbytes].to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._events[k] = ev
        plan = K.MultiTensorPlan.__new__(K.MultiTensorPlan)
        plan.host, plan.dev, plan.n = host, dev, n
        return plan

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            entries = []
            device = None
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda:
                    raise RuntimeError("mae_clip_amd.optim.AdamW needs ROCm device parameters")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                entries.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                None, p.numel(), st["step"]))
                device = p.device
            if not entries:
                continue
            # all parameters of a group share the step count after the first step
            steps = {e[6] for e in entries}
            b1, b2 = group["betas"]
            for s in sorted(steps):
                sub = [e[:6] for e in entries if e[6] == s]
                plan = self._plan(sub, device)
                K.adamw_multi(plan, group["lr"], b1, b2, group["eps"], group["weight_decay"], s)
        return loss


def C_sizeof(obj):
    import ctypes
    return ctypes.sizeof(obj)
