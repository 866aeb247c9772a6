"""Checkpoint / resume for the training step.

The reference saves the bare model weights after each improving epoch,
`torch.save(model.state_dict(), "best.pt")` (main.py:118-122), and inference
loads them back with `model.load_state_dict(torch.load(model_path))`
(inference.py:18). CLIPModel keeps the reference's parameter names (timm /
HF DistilBERT / modules.py layouts, tests/test_boundary_cpu.py), so those two
lines work unchanged on mae_clip_amd.CLIPModel. Across the two codebases the
keys match exactly only for the reference's own model family -- a ViT image
encoder (the reference defaults to resnet50, config.py) with mask_ratio = 0
(no MAE decoder). A reference best.pt loaded into an MAE model (mask_ratio > 0)
lacks the mae_decoder.* keys: load_checkpoint(strict="reference") accepts
exactly that case, keeps the decoder's own initialisation and reports the keys
it did not find (missing_out).

For resuming a run this module adds what the bare state_dict cannot carry:
  * the optimizer state (AdamW exp_avg / exp_avg_sq / step, torch.optim format),
  * the model's training step, which keys the MAE mask noise and every dropout
    mask (CLIPModel.step / the device step_counter), so a resumed run draws
    exactly the masks the uninterrupted run would have drawn.
Files are plain tensors and ints: `load_checkpoint` reads them with
torch.load(weights_only=True) -- nothing in a checkpoint is executed.
"""
from __future__ import annotations

import os

import torch

FORMAT = "mae_clip_amd.checkpoint/1"


def save_checkpoint(path, model, optimizer=None, extra=None):
    """Write model weights (reference state_dict keys), optimizer state and the
    training step to `path` (atomically: a temporary file is renamed)."""
    ckpt = {
        "format": FORMAT,
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "step": int(getattr(model, "step", 0)),
    }
    if optimizer is not None:
        ckpt["optimizer"] = _to_cpu(optimizer.state_dict())
    if extra:
        ckpt["extra"] = extra
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, model, optimizer=None, map_location="cpu", strict=True, missing_out=None):
    """Restore a file written by save_checkpoint -- or a bare reference
    `best.pt` (main.py:121: just model.state_dict()). Returns the step restored
    (0 for a bare state_dict) and sets model.step / model.step_counter.

    strict=True: every key must match. strict="reference": a bare reference
    state_dict may lack the MAE head (keys under mae_decoder.), nothing else;
    the missing keys are appended to `missing_out` (a list) when given."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(ckpt, dict) and ckpt.get("format") == FORMAT:
        state, step = ckpt["model"], int(ckpt.get("step", 0))
        opt_state = ckpt.get("optimizer")
    else:
        state, step, opt_state = ckpt, 0, None
    if strict == "reference":
        res = model.load_state_dict(state, strict=False)
        bad = [k for k in res.missing_keys if not k.startswith("mae_decoder.")]
        if bad or res.unexpected_keys:
            raise RuntimeError(f"load_checkpoint: state_dict mismatch beyond the MAE head: missing {bad}, "
                               f"unexpected {list(res.unexpected_keys)}")
        if missing_out is not None:
            missing_out.extend(res.missing_keys)
    else:
        model.load_state_dict(state, strict=strict)
    set_step(model, step)
    if optimizer is not None and opt_state is not None:
        optimizer.load_state_dict(opt_state)
        for st in optimizer.state.values():   # torch keeps the saved dtype; AdamW's host step is an int
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"] = int(st["step"].item())
    return step


def set_step(model, step):
    """Host step and device step_counter of a CLIPModel (the RNG key of the
    MAE masks and dropout masks)."""
    if hasattr(model, "step"):
        model.step = int(step)
    sc = getattr(model, "step_counter", None)
    if sc is not None:
        with torch.no_grad():
            sc.fill_(int(step))


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
