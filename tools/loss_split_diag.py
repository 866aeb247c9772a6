"""Where does the bf16 path's loss deviation at C2 model shapes come from?

bench.py's loss_delta_vs_ref_headline compares the whole loss (CLIP + MAE) of
the bf16 product with the fp64 CPU oracle (ViT-B/16 @224, mask .75, 8 x 512
decoder, 6-layer text, B = 4, eval forward). This splits it: the CLIP and MAE
terms separately, and the embeddings that feed the CLIP term (image / text
projection outputs, relative L2 vs the oracle's).

    python tools/loss_split_diag.py [B]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.helpers import build_pair, make_batch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    kw = dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, text_layers=6, mask_ratio=0.75,
              decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16)
    for prec in ("bf16", "fp32"):
        prod, ref = build_pair(prec, **kw)
        prod.eval()
        ref.eval()
        b = make_batch(B, 224, seed=12)
        emb = {}
        hooks = [prod.image_projection.register_forward_hook(lambda m, i, o: emb.__setitem__("pi", o.detach())),
                 prod.text_projection.register_forward_hook(lambda m, i, o: emb.__setitem__("pt", o.detach())),
                 ref.image_projection.register_forward_hook(lambda m, i, o: emb.__setitem__("ri", o.detach())),
                 ref.text_projection.register_forward_hook(lambda m, i, o: emb.__setitem__("rt", o.detach()))]
        with torch.no_grad():
            lp = prod({k: v.to(dev) for k, v in b.items()}).item()
            lr = ref(dict(b, image=b["image"].double())).item()
        for h in hooks:
            h.remove()
        out = {"total": (lp, lr)}
        for k in ("clip", "mae"):
            out[k] = (float(prod.last_losses[k]), float(ref.last_losses[k]))
        print(f"[{prec}] B={B}")
        for k, (p, r) in out.items():
            print(f"  {k:6s} product {p:.6f} oracle {r:.6f} abs {abs(p - r):.3e} rel {abs(p - r) / max(1.0, abs(r)):.3e}")
        for a, c, name in (("pi", "ri", "image embeddings"), ("pt", "rt", "text embeddings")):
            x, y = emb[a].double().cpu(), emb[c].double()
            print(f"  {name}: rel-L2 {((x - y).norm() / y.norm()).item():.3e}")


if __name__ == "__main__":
    main()
