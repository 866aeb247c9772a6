"""The product's data-parallel branch on the GPU box: two ranks (two
processes on cuda:0, gloo process group -- one MI355X, and RCCL refuses two
ranks on one device) run mae_clip_amd.CLIPModel under
distributed.DataParallel on B rows each; the result must equal one process
running the same model on the 2B rows:
  * CLIPModel.forward's world > 1 branch: embeddings all-gathered in rank
    order, the fused CLIP loss of the gathered batch with the gradient of the
    local rows only (grad_rows), MAE term scaled by 1/world, masks keyed by
    the global sample index (sample_offset = rank * B);
  * gradients written straight into the GradArena slots by the product's
    autograd Functions and SUM-all-reduced in place (no flatten copies)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B_LOCAL = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# C3 = BASELINE.json configs[3] per-rank model: ViT-B/16 @224 (12 blocks, n = 50
# visible tokens), 8 x 512-d decoder (n = 197), 6-layer frozen text
C3 = dict(model_name="vit_base_patch16_224", size=224, image_embedding=768, text_layers=6, mask_ratio=0.75,
          decoder_embed_dim=512, decoder_depth=8, decoder_num_heads=16)
SHAPES = {"C0": (B_LOCAL, 32, 0.5), "C3": (2, 224, 64.0)}   # (B per rank, image size, bucket MB)


def _model(precision="fp32", cfg="C0"):
    from tests.helpers import product_config, C0
    from mae_clip_amd.CLIP import CLIPModel
    kw = {k: v for k, v in C0.items() if k != "batch_size"} if cfg == "C0" else dict(C3)
    with product_config(precision=precision, **kw):
        torch.manual_seed(0)
        m = CLIPModel()
    return m.cuda().eval()


def _batch(cfg="C0"):
    from tests.helpers import make_batch
    B, S, _ = SHAPES[cfg]
    return make_batch(2 * B, S, seed=3)


def _rank(rank, world, port, out, cfg="C0"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mae_clip_amd import _lib
        from mae_clip_amd.distributed import DataParallel
        _lib.load()
        B, _, bucket = SHAPES[cfg]
        m = _model(cfg=cfg)
        dp = DataParallel(m, bucket_mb=bucket)
        b = {k: v[rank * B:(rank + 1) * B].cuda() for k, v in _batch(cfg).items()}
        for p in m.parameters():
            p.grad = None
        loss = m(b)
        loss.backward()
        dp.sync_gradients()
        torch.cuda.synchronize()
        out[rank] = dict(clip=m.last_losses["clip"].item(), mae=m.last_losses["mae"].item(),
                         mask=m.last_mask[2].cpu(), adopted=dp.adopted, nparams=len(dp.params),
                         nbuckets=len(dp.buckets),
                         grads={n: p.grad.cpu() for n, p in m.named_parameters() if p.requires_grad})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", ["C0", "C3"])
def test_product_data_parallel_equals_full_batch(dev, cfg):
    """C0: ViT-Tiny @32, 4 samples per rank, 0.5 MB buckets (many buckets).
    C3: the BASELINE.json configs[3] model (ViT-B/16 MAE+CLIP, 8 x 512 decoder,
    6-layer text) at 2 samples per rank with the production 64 MB buckets and
    the chunked encoder / decoder Functions of world > 1 (dp_*_chunk): 2 ranks
    x 2 == one process on the 4 samples (fp32 parity mode)."""
    from tests.helpers import record_parity
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank, args=(2, _free_port(), out, cfg), nprocs=2, join=True)
    res = [out[r] for r in range(2)]
    B = SHAPES[cfg][0]
    m = _model(cfg=cfg)
    full = {k: v.to(dev) for k, v in _batch(cfg).items()}
    m(full).backward()
    ref_clip, ref_mae = m.last_losses["clip"].item(), m.last_losses["mae"].item()
    ref_mask = m.last_mask[2].cpu()
    for r, o in enumerate(res):
        assert abs(o["clip"] - ref_clip) < 1e-5 * max(1.0, abs(ref_clip)), (o["clip"], ref_clip)
        assert torch.equal(o["mask"], ref_mask[r * B:(r + 1) * B])
        # every trainable gradient was produced in its arena slot (no copy)
        assert o["adopted"] == o["nparams"], (o["adopted"], o["nparams"])
        assert o["nbuckets"] >= 2
    assert abs((res[0]["mae"] + res[1]["mae"]) / 2 - ref_mae) < 1e-5 * max(1.0, abs(ref_mae))
    worst = 0.0
    for n, p in m.named_parameters():
        if not p.requires_grad:
            continue
        g = p.grad.cpu()
        sc = g.abs().max().item() + 1e-30
        for o in res:
            e = (o["grads"][n] - g).abs().max().item() / sc
            worst = max(worst, e)
            assert e < 1e-4, (n, e)
        assert torch.equal(res[0]["grads"][n], res[1]["grads"][n]), n
    record_parity(f"dp2_gloo_{cfg}_vs_single_process", clip_rel=abs(res[0]["clip"] - ref_clip) / max(1.0, ref_clip),
                  worst_grad_maxrel=worst)



B_MB = 128   # samples per rank of the production-precision DP test (both stacks micro-batched)


def _bf16_dp_rank(rank, world, port, out, grad_dtype, precision="bf16"):
    """One gloo rank of the production-precision DP step: bf16 (or fp8) MFMA stacks run
    as two micro-batch chains each (B = 128 per rank: encoder 64 x 50, decoder
    64 x 197 rows per chain), the encoder / decoder cut into DP chunks
    (dp_*_chunk), gradients in the GradArena, all-reduced in fp32 or bf16
    buckets; the default GEMM path."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mae_clip_amd import _lib
        from mae_clip_amd import functions as Fn
        from mae_clip_amd.distributed import DataParallel
        from tests.helpers import make_batch
        _lib.load()
        m = _model(precision, cfg="C3")
        mb = [Fn.microbatch_count(Fn.StackSpec(B=B_MB, n=n, D=D, H=H, eps=1e-6, dtype=torch.bfloat16, wT=[]))
              for n, D, H in ((50, 768, 12), (197, 512, 16))]
        dp = DataParallel(m, bucket_mb=64.0, grad_dtype=torch.bfloat16 if grad_dtype == "bf16" else torch.float32)
        full = make_batch(world * B_MB, 224, seed=9)
        b = {k: v[rank * B_MB:(rank + 1) * B_MB].cuda() for k, v in full.items()}
        loss = m(b)
        loss.backward()
        dp.sync_gradients()
        torch.cuda.synchronize()
        out[rank] = dict(loss=loss.item(), clip=m.last_losses["clip"].item(), mae=m.last_losses["mae"].item(),
                         microbatches=mb, nbuckets=len(dp.buckets),
                         grads={n: p.grad.cpu() for n, p in m.named_parameters() if p.requires_grad})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision,grad_dtype", [("bf16", "fp32"), ("bf16", "bf16"), ("fp8", "fp32")])
def test_product_data_parallel_bf16_microbatched(dev, precision, grad_dtype):
    """The production DP step at world 2 (main.py:99-103's model and optimizer
    wrapped by distributed.DataParallel): C3 per-rank ViT-B/16 MAE+CLIP shapes
    in bf16 with micro-batched stacks and DP chunks, 2 gloo ranks on the one
    GPU, B = 128 per rank, vs one process on the 256 concatenated samples
    (bf16, default settings). Loss within BF16_TOL["C2"][0] relative,
    gradients identical on both ranks, every gradient within BF16_TOL["C2"][1]
    relative L2 of the single process's; grad_dtype bf16 = the opt-in bf16
    all-reduce buckets; precision fp8 = the C4 mode's fp8 stacks (encoder and
    decoder, per-row / per-block scales, which are row-local: a rank quantises
    its rows as the single process does) on the same DP path."""
    from tests.helpers import make_batch, record_parity
    from tests.test_model_gpu import BF16_TOL
    loss_tol, grad_tol = BF16_TOL["C2"]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bf16_dp_rank, args=(2, _free_port(), out, grad_dtype, precision), nprocs=2, join=True)
    res = [out[r] for r in range(2)]
    assert all(r["microbatches"] == [2, 2] for r in res), [r["microbatches"] for r in res]
    assert res[0]["nbuckets"] >= 2
    m = _model(precision, cfg="C3")
    full = {k: v.to(dev) for k, v in make_batch(2 * B_MB, 224, seed=9).items()}
    loss = m(full)
    loss.backward()
    ref_loss = loss.item()
    # every rank evaluates the gathered CLIP loss (identical); the MAE term is
    # each rank's own samples, so the global-batch loss is clip + w * mean(mae)
    assert res[0]["clip"] == res[1]["clip"]
    glob = res[0]["clip"] + m.mae_weight * (res[0]["mae"] + res[1]["mae"]) / 2
    dl = abs(glob - ref_loss) / max(1.0, abs(ref_loss))
    assert dl < loss_tol, (glob, ref_loss)
    worst, worst_name = 0.0, None
    for n, p in m.named_parameters():
        if not p.requires_grad:
            continue
        g = p.grad.cpu()
        assert torch.equal(res[0]["grads"][n], res[1]["grads"][n]), n
        e = ((res[0]["grads"][n] - g).norm() / (g.norm() + 1e-30)).item()
        if e > worst:
            worst, worst_name = e, n
    record_parity(f"dp2_gloo_C3_{precision}_microbatched_grad{grad_dtype}_vs_single_process", loss_rel=dl,
                  worst_grad_relL2=worst, worst_grad=worst_name)
    assert worst < grad_tol, (worst_name, worst)


def _captured_dp_rank(rank, world, port, out):
    """One RCCL rank (the box has one GPU): CapturedStep with DataParallel --
    the embedding all-gather and the bucketed gradient all-reduces are captured
    in the step's HIP graph -- against the same DP steps run eagerly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from mae_clip_amd import _lib
        from mae_clip_amd.distributed import DataParallel
        from mae_clip_amd.optim import AdamW
        from mae_clip_amd.graph import CapturedStep
        from tests.helpers import make_batch
        _lib.load()
        res = {}
        for captured in (False, True):
            m = _model("bf16").train()
            dp = DataParallel(m, bucket_mb=4.0)
            opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
            runner = CapturedStep(m, opt, enabled=captured, eager_steps=2, dp=dp)
            losses = []
            for it in range(5):
                b = {k: v.cuda() for k, v in make_batch(8, 32, seed=it).items()}
                losses.append(runner.step(b).item())
            torch.cuda.synchronize()
            res[captured] = dict(losses=losses, enabled=runner.enabled, captures=runner.captures,
                                 params={n: p.detach().cpu() for n, p in m.named_parameters()})
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_captured_step_with_rccl_data_parallel(dev):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_captured_dp_rank, args=(1, _free_port(), out), nprocs=1, join=True)
    eager, graph = out[0][False], out[0][True]
    assert graph["enabled"] and graph["captures"] == 1
    assert eager["losses"] == graph["losses"], (eager["losses"], graph["losses"])
    for n, p in eager["params"].items():
        assert torch.equal(p, graph["params"][n]), n


def _bf16_reduce_rank(rank, world, port, out):
    """the opt-in bf16 gradient all-reduce on the device path (the
    maeclip_cast_flat kernel both ways around an RCCL bf16 SUM). At world 1 the
    sum is the rank's own gradient, so every gradient must equal the fp32
    run's gradient rounded to bf16 (deterministic kernels: the two backward
    passes produce identical fp32 gradients)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from mae_clip_amd import _lib
        from mae_clip_amd.distributed import DataParallel
        from tests.helpers import make_batch
        _lib.load()
        res = {}
        for gd in (torch.float32, torch.bfloat16):
            m = _model("bf16").train()
            dp = DataParallel(m, bucket_mb=1.0, grad_dtype=gd)
            b = {k: v.cuda() for k, v in make_batch(8, 32, seed=3).items()}
            loss = m(b)
            loss.backward()
            dp.sync_gradients()
            torch.cuda.synchronize()
            res[str(gd)] = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters() if p.grad is not None}
            res[str(gd) + "_buckets"] = len(dp.buckets)
            res[str(gd) + "_offsets"] = [o for o, _, _ in dp.arena.offsets.values()]
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_bf16_gradient_allreduce_rccl_world1(dev):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bf16_reduce_rank, args=(1, _free_port(), out), nprocs=1, join=True)
    r = out[0]
    f32, b16 = r[str(torch.float32)], r[str(torch.bfloat16)]
    assert r[str(torch.bfloat16) + "_buckets"] > 1
    assert all(o % 4 == 0 for o in r[str(torch.bfloat16) + "_offsets"])   # 16-B aligned slots
    assert set(f32) == set(b16) and len(f32) > 10
    for n, g in f32.items():
        assert torch.equal(b16[n], g.to(torch.bfloat16).float()), n
