"""C4-shape fp32 parity triage: the image / text embeddings and their CLIP-loss
gradients of the product vs the fp64 oracle, and the product's fused CLIP loss
gradient vs fp64 autograd on the product's own embeddings."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import build_pair, make_batch
import mae_clip_amd.CLIP as PC
import oracle.ref_model as RM

cap = {}
pcl, rcl = PC.clip_loss, RM.clip_loss


def p_hook(I, T, *a, **k):
    I.retain_grad(); T.retain_grad(); cap["pI"], cap["pT"] = I, T
    return pcl(I, T, *a, **k)


def r_hook(I, T, *a, **k):
    I.retain_grad(); T.retain_grad(); cap["rI"], cap["rT"] = I, T
    return rcl(I, T, *a, **k)


PC.clip_loss, RM.clip_loss = p_hook, r_hook
kw = dict(model_name="vit_large_patch14_336", size=336, image_embedding=1024, text_layers=2, mask_ratio=0.75,
          decoder_embed_dim=512, decoder_depth=int(os.environ.get("DD", "8")), decoder_num_heads=16,
          vit_depth=4)
if os.environ.get("CFG") == "C2":
    kw = dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, text_layers=2, mask_ratio=0.75,
              decoder_embed_dim=512, decoder_depth=2, decoder_num_heads=16)
prod, ref = build_pair("fp32", **kw)
prod.eval(); ref.eval()
b = make_batch(2, kw["size"], seed=int(os.environ.get("SEED", "13")))
lp = prod({k: v.cuda() for k, v in b.items()}); lp.backward()
lr = ref(dict(b, image=b["image"].double())); lr.backward()
print("loss", lp.item(), lr.item())


def d(name, a, r):
    a = a.detach().double().cpu(); r = r.detach().double().cpu()
    print(f"{name:10s} maxabs={(a - r).abs().max().item():.3e} scale={r.abs().max().item():.3e} "
          f"colsum_err={(a.sum(0) - r.sum(0)).abs().max().item():.3e} colsum_scale={r.sum(0).abs().max().item():.3e}")


d("I", cap["pI"], cap["rI"]); d("T", cap["pT"], cap["rT"])
d("dI", cap["pI"].grad, cap["rI"].grad); d("dT", cap["pT"].grad, cap["rT"].grad)
I64 = cap["pI"].detach().double().cpu().requires_grad_(True)
T64 = cap["pT"].detach().double().cpu().requires_grad_(True)
rcl(I64, T64).backward()
d("dI(own)", cap["pI"].grad, I64.grad); d("dT(own)", cap["pT"].grad, T64.grad)
print("logits", (cap["rT"] @ cap["rI"].T).detach())
if os.environ.get("SAVE"):
    import numpy as np
    np.savez(os.environ["SAVE"], I=cap["pI"].detach().cpu().numpy(), T=cap["pT"].detach().cpu().numpy(),
             dI=cap["pI"].grad.cpu().numpy(), dT=cap["pT"].grad.cpu().numpy())
