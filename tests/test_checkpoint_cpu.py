"""Checkpoint / resume files (mae_clip_amd.checkpoint) on
CPU: reference-format state_dict round trip (main.py:121 save, inference.py:18
load), the extended format's optimizer state and training step."""
import torch

from tests.helpers import C0, product_config


def _model():
    from mae_clip_amd.CLIP import CLIPModel
    with product_config(**{k: v for k, v in C0.items() if k != "batch_size"}):
        torch.manual_seed(0)
        return CLIPModel()


def test_reference_best_pt_round_trip(tmp_path):
    """`torch.save(model.state_dict(), "best.pt")` then
    `model.load_state_dict(torch.load(path))` -- the reference's own two lines."""
    from mae_clip_amd.checkpoint import load_checkpoint
    a = _model()
    path = tmp_path / "best.pt"
    torch.save(a.state_dict(), path)
    b = _model()
    with torch.no_grad():
        for p in b.parameters():
            p.add_(1.0)
    b.load_state_dict(torch.load(path, weights_only=True))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb), ka
    c = _model()
    assert load_checkpoint(path, c) == 0      # bare state_dict: step 0
    assert all(torch.equal(x, y) for x, y in zip(a.state_dict().values(), c.state_dict().values()))


def test_extended_checkpoint_restores_optimizer_and_step(tmp_path):
    from mae_clip_amd.checkpoint import save_checkpoint, load_checkpoint
    a = _model()
    params = [p for p in a.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-3, weight_decay=1e-3)
    for p in params:
        p.grad = torch.randn_like(p)
    opt.step()
    a.step = 7
    path = tmp_path / "ckpt.pt"
    save_checkpoint(path, a, opt, extra={"epoch": 3})
    b = _model()
    opt_b = torch.optim.AdamW([p for p in b.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
    assert load_checkpoint(path, b, opt_b) == 7
    assert b.step == 7 and int(b.step_counter.item()) == 7
    for x, y in zip(a.state_dict().values(), b.state_dict().values()):
        assert torch.equal(x, y)
    sa, sb = opt.state_dict()["state"], opt_b.state_dict()["state"]
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k]["exp_avg"], sb[k]["exp_avg"])
        assert torch.equal(sa[k]["exp_avg_sq"], sb[k]["exp_avg_sq"])
    assert torch.load(path, weights_only=True)["extra"] == {"epoch": 3}


def test_reference_clip_only_state_dict_into_mae_model(tmp_path):
    """A reference best.pt comes from the CLIP-only model (no MAE head): loading
    it into an MAE model needs strict="reference", which tolerates exactly the
    missing mae_decoder.* keys (reported) and nothing else."""
    import pytest
    from mae_clip_amd.CLIP import CLIPModel
    from mae_clip_amd.checkpoint import load_checkpoint
    kw = {k: v for k, v in C0.items() if k != "batch_size"}
    with product_config(**dict(kw, mask_ratio=0.0)):
        torch.manual_seed(1)
        ref_like = CLIPModel()
    path = tmp_path / "best.pt"
    torch.save(ref_like.state_dict(), path)
    mae = _model()
    with pytest.raises(RuntimeError):
        load_checkpoint(path, mae)                       # strict: the decoder keys are missing
    missing = []
    assert load_checkpoint(path, mae, strict="reference", missing_out=missing) == 0
    assert missing and all(k.startswith("mae_decoder.") for k in missing)
    sd = mae.state_dict()
    for k, v in ref_like.state_dict().items():
        assert torch.equal(sd[k], v), k
    bad = dict(ref_like.state_dict())
    bad.pop("image_projection.fc.weight")
    torch.save(bad, path)
    with pytest.raises(RuntimeError):
        load_checkpoint(path, _model(), strict="reference")
