"""Calibrate the CPU oracle (bench.py's cpu_baseline, kind "port") against the
reference itself, in THIS container (the restatement must be
within +-10% of the reference's own CPU step rate).

Both models are timed in one process on the same synthetic inputs with the
same optimizer (AdamW lr 1e-3, wd 1e-3, main.py:101-103), median of the timed
steps after one warm-up, torch.set_num_threads(os.cpu_count()):
  * reference: /root/reference CLIP.py + modules.py, imported with the timm stub
    of SURVEY.md §8c (its create_model returns the oracle's timm-semantics ViT,
    because timm 0.9.12 is not installed) and a random-init frozen DistilBERT;
  * oracle:    oracle/ref_model.CLIPModel (mask_ratio 0: the CLIP-only path the
    reference has), fp32.
Configs = SURVEY.md §6's probes: ViT-Tiny/16 @32, 2-layer text, B=8, T=32; and
ViT-B/16 @224, 6-layer text, B=32, T=32.

Writes profiles/r02/cpu_calibration.json. Needs /root/reference (build
container only); never runs on the GPU box.
"""
from __future__ import annotations

import json
import os
import platform
import statistics
import sys
import time
import types

import torch

import transformers  # noqa: F401  (before the timm stub)
from transformers import DistilBertConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.ref_model import CLIPModel as OracleCLIP, OracleConfig, VisionTransformer  # noqa: E402

REF = "/root/reference"


class StubViT(torch.nn.Module):
    """timm.create_model(name, pretrained, num_classes=0, global_pool='avg')."""

    def __init__(self, name, img):
        super().__init__()
        self.vit = VisionTransformer(name, img)

    def forward(self, x):
        return self.vit(x)


def import_reference(model_name, img, text_layers):
    stub = types.ModuleType("timm")
    stub.create_model = lambda name, pretrained=False, num_classes=0, global_pool="avg": StubViT(model_name, img)
    sys.modules["timm"] = stub
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import modules as RM
    import CLIP as RC
    RM.DistilBertConfig = lambda: DistilBertConfig(n_layers=text_layers)
    RM.TextEncoder.__init__.__defaults__ = ("distilbert-base-uncased", False, False)
    RM.ImageEncoder.__init__.__defaults__ = (model_name, False, True)
    return RC


def batch(B, S, T):
    g = torch.Generator().manual_seed(0)
    px = torch.randint(0, 256, (B, 3, S, S), generator=g, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return {"image": ((px.float() / 255.0) - mean) / std,
            "input_ids": torch.randint(5, 300, (B, T), generator=g),
            "attention_mask": torch.ones(B, T, dtype=torch.int64)}


def time_steps(model, b, steps):
    model.train()
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    ts = []
    for _ in range(steps + 1):
        t0 = time.perf_counter()
        opt.zero_grad()
        model(b).backward()
        opt.step()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts[1:])


def main():
    torch.set_num_threads(os.cpu_count())
    cases = [("vit_tiny_patch16_224", 32, 192, 2, 8, 32, 8, 96.0),
             ("vit_base_patch16_224", 224, 768, 6, 32, 32, 2, 6.8)]
    out = {"threads": torch.get_num_threads(), "cpu": platform.processor() or None, "cases": []}
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            out["cpu"] = line.split(":", 1)[1].strip()
            break
    for name, S, D, tl, B, T, steps, survey in cases:
        b = batch(B, S, T)
        RC = import_reference(name, S, tl)
        torch.manual_seed(0)
        ref = RC.CLIPModel(image_embedding=D)
        torch.manual_seed(0)
        orc = OracleCLIP(OracleConfig(model_name=name, img_size=S, text_layers=tl, mask_ratio=0.0))
        # alternate the two models (3 rounds) so host noise hits both alike
        tr, to = [], []
        for _ in range(3):
            tr.append(time_steps(ref, b, steps))
            to.append(time_steps(orc, b, steps))
        t_ref, t_orc = statistics.median(tr), statistics.median(to)
        for m in ("modules", "CLIP", "config"):
            sys.modules.pop(m, None)
        rec = {"config": f"{name} @{S}, {tl}-layer text, B={B}, T={T}, CLIP-only, fp32, AdamW",
               "reference_img_s": round(B / t_ref, 2), "oracle_img_s": round(B / t_orc, 2),
               "oracle_over_reference": round(t_ref / t_orc, 3), "survey_reference_img_s": survey,
               "timed_steps": f"3 alternating rounds x {steps} steps (+1 warm-up each), median"}
        print(json.dumps(rec), flush=True)
        out["cases"].append(rec)
    out["within_10pct"] = all(abs(c["oracle_over_reference"] - 1) <= 0.10 for c in out["cases"])
    os.makedirs(os.path.join(ROOT, "profiles", "r02"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r02", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
