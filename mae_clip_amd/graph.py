"""Whole-training-step HIP graph: forward + backward + AdamW captured once and
replayed (DESIGN.md §5 "Host").

main.py's loop (main.py:54-66) issues ~600 kernel launches per step through
Python; at ViT-B/16 shapes the host falls behind the GPU in the backward and
at every step boundary. CapturedStep runs the first step eagerly (it also
creates the optimizer state, the bf16 weight shadows and the multi-tensor
descriptor arrays), captures the second one into a torch.cuda.CUDAGraph (the
side stream of the text tower / weight gradients joins the capture through its
events) and replays that graph for every later step: one launch per step.

Everything that changes from step to step is device-resident, so a replay is
a faithful training step: the MAE mask noise and every dropout mask are keyed
by CLIPModel.step_counter, AdamW's bias corrections by AdamW._step_dev, and
both counters are advanced by kernels inside the graph. Batch tensors are
copied into static input buffers before each replay.

Usage (drop-in around the reference's train_epoch body):
    runner = CapturedStep(model, optimizer)
    for batch in loader:
        loss = runner.step(batch)      # model(batch); loss.backward(); optimizer.step()

Data parallel (CapturedStep(..., dp=DataParallel(model))): the step becomes
model(batch); backward; dp.sync_gradients(); optimizer.step(), and the RCCL
collectives (the embedding all-gather of the forward, the bucketed gradient
all-reduces launched from the backward's hooks) are captured with it: every
rank replays the same collective sequence, so the N>1 step is one graph launch
per rank as at N=1. The gloo backend (host-staged copies) cannot be captured:
CapturedStep then stays eager.
"""
from __future__ import annotations

import torch

from . import kernels as K


class CapturedStep:
    def __init__(self, model, optimizer, enabled: bool = True, eager_steps: int = 1, dp=None):
        self.model = model
        self.opt = optimizer
        self.dp = dp
        if dp is not None and torch.distributed.get_backend(dp.group) != "nccl":
            enabled = False
        self.enabled = enabled
        self.eager_steps = max(1, eager_steps)
        self.graph = None
        self.static = None
        self.loss = None
        self.calls = 0
        self.captures = 0
        self.hp_key = None
        self.graph_grads = None
        self.state_key = None
        self._host = None   # kernels.HostScalars: the loss, published inside the step (loss_value)
        self._last = None
        self._done = []     # (end-of-step event, model.step) of the last two steps queued

    def _state_key(self):
        """What a replay bakes in besides the batch: every parameter's storage
        and version (load_state_dict, in-place edits, another optimizer bump
        p._version) and the optimizer state buffers (optimizer.load_state_dict
        replaces them). The captured forward reads bf16 weight shadows that only
        the fused AdamW keeps current, and the frozen text tower's cached bf16
        weights, so a change here means the graph would replay stale weights.
        Writes through p.data are invisible to _version: call invalidate()."""
        params = tuple((p.data_ptr(), p._version) for p in self.model.parameters())
        st = tuple(t.data_ptr() for s in self.opt.state.values() for t in s.values() if torch.is_tensor(t))
        return params, st

    def invalidate(self):
        """Drop the captured graph: the next step runs eagerly (re-casting the
        weight shadows from the fp32 masters) and the one after re-captures."""
        self.graph = None
        self.calls = 0

    def _hparams(self):
        """Optimizer hyper-parameters baked into the captured AdamW launch."""
        return tuple((g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]) for g in self.opt.param_groups)

    def _publish(self, loss):
        """write the loss into pinned, device-mapped host memory from inside the
        step (a kernel of the step itself, captured with it), so that the host's
        per-step read (main.py:64) needs no device-to-host copy launch. Two
        slots, picked by the model's device step counter: step c writes slot
        c & 1, so step c's value can be read while step c + 1 runs."""
        self._last = loss.detach()
        if not loss.is_cuda:
            return
        counter = getattr(self.model, "step_counter", None)
        slot_ok = torch.is_tensor(counter) and counter.is_cuda and counter.dtype == torch.int64
        if self._host is None:
            from . import kernels as K
            self._host = K.HostScalars(1, slots=2 if slot_ok else 1)
        self._host.publish(loss.detach().reshape(1).float(), counter if slot_ok else None)

    def _slot(self, c):
        return (c & 1) if self._host is not None and self._host.slots == 2 else 0

    def _mark(self):
        """after a step is queued: an event at its end and its step count"""
        if self._host is not None:
            ev = torch.cuda.Event()
            ev.record()
            self._done.append((ev, int(getattr(self.model, "step", 0))))
            del self._done[:-2]

    def loss_value(self) -> float:
        """The last step's loss as a Python float (the reference's loss.item(),
        main.py:64): waits for that step, then reads the value it published --
        no copy kernel."""
        if self._host is None or not self._done:
            return float(self._last.item())
        ev, c = self._done[-1]
        ev.synchronize()
        return self._host.values(self._slot(c))[0]

    def previous_loss(self):
        """The loss of the step before the last one queued (None after the first
        step): call it right after step() to read step k's loss while step k + 1
        runs -- the per-step read of main.py:64 without a GPU bubble at the step
        boundary (the host's graph launch of step k + 1 is already queued)."""
        if self._host is None or len(self._done) < 2:
            return None
        ev, c = self._done[-2]
        ev.synchronize()
        return self._host.values(self._slot(c))[0]

    def _eager(self, batch):
        self.opt.zero_grad(set_to_none=True)
        loss = self.model(batch)
        loss.backward()
        if self.dp is not None:
            self.dp.sync_gradients()
        self.opt.step()
        self._publish(loss)
        # detached: a caller holding the loss must not keep this step's autograd
        # graph (and its AccumulateGrad nodes, bound to the eager stream) alive
        # into the capture
        return loss.detach()

    def _capture(self, batch):
        self.graph = None
        self.static = {k: v.clone() for k, v in batch.items()}
        model_step = self.model.step
        # grads are re-created inside the graph's private pool: drop the eager ones
        self.opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # backward seed allocated outside the graph: loss.backward() would fill
        # a fresh ones tensor inside every replay
        one = torch.ones((), device=next(self.model.parameters()).device, dtype=torch.float32)
        replay = torch.cuda.current_stream().cuda_stream
        with torch.cuda.graph(g, capture_error_mode="relaxed"):
            cap = torch.cuda.current_stream().cuda_stream
            K.alias_stream(cap, replay)
            try:
                loss = self.model(self.static)
                torch.autograd.backward(loss, grad_tensors=one.expand_as(loss) if loss.dim() else one)
                if self.dp is not None:
                    self.dp.sync_gradients()
                self.opt.step()
                self._publish(loss)
            finally:
                K.alias_stream(cap, None)
        # capture recorded the work without running it: undo its host-side counting
        self.model.step = model_step
        self.opt._advance_host_steps(-1)
        # detached: the captured loss must not keep the capture's autograd graph
        # (and its AccumulateGrad nodes, bound to the capture stream) alive into
        # later eager fallback steps or a re-capture (torch's AccumulateGrad
        # stream-mismatch hazard); the replays still refresh its storage
        self.graph, self.loss = g, loss.detach()
        self._seed = one
        self.hp_key = self._hparams()
        self.graph_grads = [(p, p.grad) for grp in self.opt.param_groups for p in grp["params"]]
        self.state_key = self._state_key()
        self.captures += 1

    def _fits(self, batch):
        return all(k in self.static and v.shape == self.static[k].shape and v.dtype == self.static[k].dtype
                   and v.device == self.static[k].device for k, v in batch.items()) and len(batch) == len(self.static)

    def step(self, batch):
        """One training step on `batch` (dict of device tensors); returns the loss tensor.
        (The step is queued; loss_value() / previous_loss() read its published loss.)"""
        loss = self._step(batch)
        self._mark()
        return loss

    def _step(self, batch):
        """One training step on `batch` (dict of device tensors); returns the loss tensor.

        A batch whose shapes differ from the captured ones (e.g. the last,
        partial batch of an epoch: the reference's DataLoader keeps it,
        main.py:42-47) runs as an eager step; a change of lr / betas / eps /
        weight_decay (e.g. by a scheduler, main.py:104) re-captures the graph."""
        if self.graph is not None and self._state_key() != self.state_key:
            self.invalidate()   # parameters / optimizer state changed outside the graph
        self.calls += 1
        if not self.enabled or self.calls <= self.eager_steps:
            return self._eager(batch)
        if self.graph is not None and not self._fits(batch):
            loss = self._eager(batch)
            # p.grad of the eager step is not the graph's: point back at the
            # buffers the next replay fills
            for p, gr in self.graph_grads:
                p.grad = gr
            return loss
        if self.graph is None or self._hparams() != self.hp_key:
            self._capture(batch)
        else:
            for k, v in batch.items():
                if v.data_ptr() != self.static[k].data_ptr():
                    self.static[k].copy_(v, non_blocking=True)
        self.graph.replay()
        self.model.step += 1
        self.opt._advance_host_steps(1)
        return self.loss
