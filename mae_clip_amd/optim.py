"""Fused multi-tensor AdamW on the libmaeclip kernel.

Same update as torch.optim.AdamW (main.py:101-103: lr 1e-3, weight_decay 1e-3,
betas (0.9, 0.999), eps 1e-8), one kernel launch for all parameters.

The step count t lives on the device as well (`_step_dev`, advanced by a
kernel before the update and read by it for the bias corrections), so the
optimizer step can be captured into a HIP graph together with the forward and
backward (mae_clip_amd.graph.CapturedStep). The per-parameter host
state["step"] is kept equal to it (state_dict / load_state_dict compatible
with torch.optim.AdamW).
"""
from __future__ import annotations

import torch

from . import kernels as K
from . import _lib as L
from .modules import shadow_of


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._stager = K.PinnedStager(slots=2)
        self._step_dev = None     # device int64[1]: step count t of the uniform-step path
        self._dev_mirror = 0      # host copy of the value *_step_dev will hold when the stream gets there

    def _plan(self, entries, device):
        """Entry array staged through the pinned stager (async H2D, capturable)."""
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
        plan = K.MultiTensorPlan.__new__(K.MultiTensorPlan)
        plan.host, plan.dev, plan.n = host, self._stager.stage(host, device), n
        return plan

    def _device_step(self, t, device):
        """Advance the device step counter to t (normally +1) on the stream."""
        if self._step_dev is None or self._step_dev.device != device:
            self._step_dev = torch.zeros(1, dtype=torch.int64, device=device)
            self._dev_mirror = 0
        K.counter_add(self._step_dev, t - self._dev_mirror)
        self._dev_mirror = t
        return self._step_dev

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
                K._dev(p)   # ROCm device parameters only (raises otherwise)
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] = int(st["step"]) + 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                # the bf16 GEMM shadow of p (if any) is written in the same pass
                sh = shadow_of(p)
                sh = sh.data_ptr() if sh is not None and sh.numel() == p.numel() else None
                entries.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                sh, p.numel(), st["step"]))
                device = p.device
            if not entries:
                continue
            b1, b2 = group["betas"]
            steps = sorted({e[6] for e in entries})
            if len(steps) == 1:
                # every parameter at the same t (the training loop's case): t on the device
                t = steps[0]
                plan = self._plan([e[:6] for e in entries], device)
                K.adamw_multi(plan, group["lr"], b1, b2, group["eps"], group["weight_decay"], t,
                              step_ptr=self._device_step(t, device))
            else:
                for s in steps:
                    plan = self._plan([e[:6] for e in entries if e[6] == s], device)
                    K.adamw_multi(plan, group["lr"], b1, b2, group["eps"], group["weight_decay"], s)
        return loss

    def _advance_host_steps(self, delta):
        """Host bookkeeping for graph replays / capture (no kernel launched)."""
        for st in self.state.values():
            if "step" in st:
                st["step"] = int(st["step"]) + delta
        self._dev_mirror += delta
