"""Where does the product's C0 fp32 training curve leave the oracle's envelope?

test_reference_training_curve_fp32 runs 20 AdamW steps of the reference's loop
(main.py:54-66, AdamW lr 1e-3 wd 1e-3 as main.py:101-103) at C0, mask 0, and
compares the losses with the fp64 curve the reference itself produced
(tests/golden/train_curve.npz). This script runs the same 20 steps as

  A  product (fp32 parity mode) + HIP AdamW          (the test)
  B  product (fp32 parity mode) + torch.optim.AdamW  (same forward / backward, torch's update on the GPU)
  D  oracle fp32 on the CPU + torch.optim.AdamW
  F  oracle fp32 on the GPU (torch's own kernels) + torch.optim.AdamW
  E  oracle fp64 on the CPU + torch.optim.AdamW       (must reproduce the golden curve)

and prints, per step, |dloss| / loss vs the golden curve, plus the step-0
gradient deviation of A and D from E per parameter (max-rel and rel-L2), so
the first op or optimizer detail that departs from fp64 can be named.

    python tools/curve_diag.py [--out gpurun_out/curve_diag.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.helpers import C0, make_batch, product_config, oracle_config  # noqa: E402


def build(kind, dev):
    from mae_clip_amd.CLIP import CLIPModel
    from oracle.ref_model import CLIPModel as RefCLIP
    kw = dict(C0, mask_ratio=0.0)
    kw.pop("batch_size")
    torch.manual_seed(0)
    with product_config(precision="fp32", **kw):
        m = CLIPModel()
    if kind == "product":
        return m.to(dev).eval()
    if kind == "fp32gpu":
        ref = RefCLIP(oracle_config(**kw))
        ref.load_state_dict({k: v.detach().clone() for k, v in m.state_dict().items()}, strict=True)
        return ref.float().to(dev).eval()
    ref = RefCLIP(oracle_config(**kw))
    ref.load_state_dict({k: v.detach().clone() for k, v in m.state_dict().items()}, strict=True)
    return (ref.double() if kind == "fp64" else ref.float()).eval()


def run(kind, opt_kind, dev, steps, grads0=None):
    m = build(kind, dev)
    params = [p for p in m.parameters() if p.requires_grad]
    if opt_kind == "hip":
        from mae_clip_amd.optim import AdamW
        opt = AdamW(params, lr=1e-3, weight_decay=1e-3)
    else:
        opt = torch.optim.AdamW(params, lr=1e-3, weight_decay=1e-3, foreach=False)
    losses, g0 = [], None
    for k in range(steps):
        b = make_batch(8, 32, seed=300 + k)
        if kind in ("product", "fp32gpu"):
            b = {kk: v.to(dev) for kk, v in b.items()}
        else:
            b = dict(b, image=b["image"].to(torch.float64 if kind == "fp64" else torch.float32))
        loss = m(b)
        opt.zero_grad()
        loss.backward()
        if k == 0:
            g0 = {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters() if p.grad is not None}
        opt.step()
        losses.append(float(loss.item()))
    return losses, g0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(ROOT, "tests", "golden", "train_curve.npz"))
    gold = [float(x) for x in z["losses"]][:a.steps]
    res = {}
    for name, kind, optk in [("A_product_hipadamw", "product", "hip"), ("B_product_torchadamw", "product", "torch"),
                             ("D_oracle_fp32", "fp32", "torch"), ("F_oracle_fp32_gpu_torch", "fp32gpu", "torch"),
                             ("E_oracle_fp64", "fp64", "torch")]:
        losses, g0 = run(kind, optk, dev, a.steps)
        rel = [abs(l - g) / abs(g) for l, g in zip(losses, gold)]
        res[name] = {"losses": losses, "rel": rel, "worst": max(rel), "worst_step": int(np.argmax(rel)), "g0": g0}
        print(f"{name:24s} worst {max(rel):.3e} at step {int(np.argmax(rel))}; "
              + " ".join(f"{r:.1e}" for r in rel), flush=True)
    ref_g = res["E_oracle_fp64"]["g0"]
    out = {k: {kk: vv for kk, vv in v.items() if kk != "g0"} for k, v in res.items()}
    for name in ("A_product_hipadamw", "D_oracle_fp32"):
        rows = []
        for n, g in res[name]["g0"].items():
            r = ref_g[n]
            maxrel = ((g - r).abs().max() / (r.abs().max() + 1e-30)).item()
            rel2 = ((g - r).norm() / (r.norm() + 1e-30)).item()
            rows.append((maxrel, rel2, n))
        rows.sort(reverse=True)
        out[name]["grad0_worst"] = rows[:12]
        print(f"{name}: step-0 gradient deviation vs fp64 (max-rel, rel-L2), worst 8:")
        for r in rows[:8]:
            print(f"   {r[0]:.2e} {r[1]:.2e} {r[2]}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
