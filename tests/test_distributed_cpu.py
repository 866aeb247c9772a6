"""Data-parallel path on CPU: world_size 2, 4 and 8 over gloo
(SURVEY.md §4.4).

The product's CLIPModel (mae_clip_amd/CLIP.py) shards the batch across ranks,
all-gathers the projection embeddings (distributed.gather_rows), scales the
MAE term by 1/world and SUM-all-reduces gradients (distributed.DataParallel).
Here the same composition is driven with the oracle's CPU modules so the
claim "W ranks x B == 1 rank x WB, exactly" is checked without a GPU:
loss, every parameter gradient and the per-sample MAE masks must match the
single-process full-batch oracle."""
import functools
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import oracle_config, make_batch


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(max(1, 4 // world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = fn(rank, world)
    finally:
        dist.destroy_process_group()


def run_ranks(fn, world=2):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), fn, out), nprocs=world, join=True)
    return [out[r] for r in range(world)]


# ---------------------------------------------------------------- rank bodies
def _gather_body(rank, world):
    from mae_clip_amd.distributed import gather_rows
    x = torch.arange(6.0).reshape(3, 2).add(100 * rank).requires_grad_()
    y = gather_rows(x)
    (y * torch.arange(y.numel(), dtype=y.dtype).reshape(y.shape)).sum().backward()
    return y.detach(), x.grad


def test_gather_rows_forward_backward():
    res = run_ranks(_gather_body)
    for r, (y, g) in enumerate(res):
        assert y.shape == (6, 2)
        assert torch.equal(y[:3], torch.arange(6.0).reshape(3, 2))
        assert torch.equal(y[3:], torch.arange(6.0).reshape(3, 2) + 100)
        # backward keeps this rank's slice of the upstream gradient
        assert torch.equal(g, torch.arange(6.0).reshape(3, 2) + 6 * r)


B_LOCAL = 3


def _model_and_batch(world=2):
    from oracle.ref_model import CLIPModel
    torch.manual_seed(0)
    cfg = oracle_config(mask_ratio=0.75)
    m = CLIPModel(cfg).double().eval()   # eval: dropout off, so both sides are deterministic
    batch = make_batch(world * B_LOCAL, cfg.img_size, seed=3)
    batch["image"] = batch["image"].double()
    return m, cfg, batch


def _dp_forward(m, cfg, batch, rank, world):
    """CLIP.py:23-43 + MAE, distributed exactly as mae_clip_amd/CLIP.py does it."""
    from mae_clip_amd.distributed import gather_rows
    from oracle.ref_model import clip_loss, mae_loss
    vit = m.image_encoder.model
    img = batch["image"]
    B = img.shape[0]
    ids_shuffle, ids_restore, mask, keep = m.mask_for_batch(B, 0, rank * B)
    tokens = vit.forward_tokens(img, ids_shuffle[:, :keep])
    ie = m.image_projection(vit.pool(tokens))
    te = m.text_projection(m.text_encoder(batch["input_ids"], batch["attention_mask"]))
    loss = clip_loss(gather_rows(ie), gather_rows(te), m.temperature)
    ml = mae_loss(m.mae_decoder(tokens, ids_restore), img, mask, vit.patch_embed.patch_size, cfg.norm_pix_loss)
    return loss + cfg.mae_weight * ml / world, loss.detach(), ml.detach(), mask


def _dp_body(bucket_mb, overlap, rank, world, grad_dtype=torch.float32):
        from mae_clip_amd.distributed import DataParallel
        m, cfg, batch = _model_and_batch(world)
        if rank > 0:   # replicas start different; DataParallel broadcasts rank 0's weights
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(float(rank))
        dp = DataParallel(m, bucket_mb=bucket_mb, grad_dtype=grad_dtype)
        dp.overlap = overlap
        sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
        local = {k: v[sl] for k, v in batch.items()}
        total, clip, mae, mask = _dp_forward(m, cfg, local, rank, world)
        total.backward()
        dp.sync_gradients()
        grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        return clip, mae, mask, grads, len(dp.buckets)


@pytest.mark.parametrize("world,bucket_mb,overlap", [(2, 64.0, True), (2, 0.05, True), (2, 0.05, False),
                                                     (4, 0.05, True), (8, 0.05, True), (8, 64.0, False)])
def test_data_parallel_equals_full_batch(world, bucket_mb, overlap):
    res = run_ranks(functools.partial(_dp_body, bucket_mb, overlap), world=world)
    m, cfg, batch = _model_and_batch(world)
    ref_loss = m(batch, step=0)
    ref_loss.backward()
    ref_clip, ref_mae = m.last_losses["clip"], m.last_losses["mae"]
    ref_mask = m.mask_for_batch(world * B_LOCAL, 0, 0)[2]
    if bucket_mb < 1:
        assert res[0][4] > 2   # several buckets actually exercised
    for r, (clip, mae, mask, grads, _) in enumerate(res):
        assert torch.allclose(clip, ref_clip, atol=1e-6, rtol=1e-5)
        # masks keyed by the global sample index: shard r == rows of the full batch
        assert torch.equal(mask, ref_mask[r * B_LOCAL:(r + 1) * B_LOCAL])
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            assert torch.allclose(grads[n], p.grad, atol=2e-6, rtol=1e-4), n
    # global MAE loss is the mean of the per-rank losses (equal masked counts)
    assert torch.allclose(sum(r[1] for r in res) / world, ref_mae, atol=1e-6, rtol=1e-5)
    # every rank holds identical synchronised gradients
    for r in range(1, world):
        for n in res[0][3]:
            assert torch.equal(res[0][3][n], res[r][3][n]), (r, n)


def test_grad_arena_slot_handed_out_once():
    """A parameter reaching two backward Functions gets its arena slot once;
    the second request must get a fresh tensor (else autograd would sum two
    aliases of one buffer: 2*g2 instead of g1+g2). begin_forward re-arms."""
    from mae_clip_amd.distributed import GradArena
    p = torch.nn.Parameter(torch.zeros(4, 3))
    q = torch.nn.Parameter(torch.zeros(5))
    ar = GradArena([p, q], "cpu")
    s1 = ar.slot(p)
    assert s1 is not None and s1.data_ptr() == ar.flat.data_ptr()
    assert ar.slot(p) is None
    assert ar.slot(q) is not None
    ar.begin_forward()
    assert ar.slot(p) is not None


def _ragged_body(rank, world):
    from mae_clip_amd.distributed import check_equal_rows
    check_equal_rows(4, None, torch.device("cpu"))          # equal: passes
    try:
        check_equal_rows(4 + rank, None, torch.device("cpu"))
    except RuntimeError as e:
        return str(e)
    return None


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_rejects_ragged_batches(world):
    """ranks with different local B fail with a clear error, not a hang."""
    res = run_ranks(_ragged_body, world=world)
    assert all(r is not None and "different local batch sizes" in r for r in res)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_data_parallel_bf16_gradient_allreduce(world):
    """opt-in bf16 all-reduce buckets (DataParallel(grad_dtype=bfloat16)): every
    gradient within 1e-2 relative L2 of the fp32 single-process full batch
    (two bf16 roundings + world - 1 bf16 adds per element), ranks identical."""
    res = run_ranks(functools.partial(_dp_body, 0.05, True, grad_dtype=torch.bfloat16), world=world)
    m, cfg, batch = _model_and_batch(world)
    m(batch, step=0).backward()
    worst = 0.0
    for n, p in m.named_parameters():
        if p.grad is None:
            continue
        g = res[0][3][n].double()
        den = p.grad.double().norm().item()
        if den > 0:
            worst = max(worst, (g - p.grad.double()).norm().item() / den)
        for r in range(1, world):
            assert torch.equal(res[0][3][n], res[r][3][n]), n
    assert worst < 1e-2, worst


def test_grad_arena_slots_are_16b_aligned():
    """arena slots start on 4-float boundaries, so every all-reduce
    bucket slice handed to the flat cast kernel is 16-B aligned; the padding
    is zero."""
    from mae_clip_amd.distributed import GradArena
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (3, 5, 8, 1, 7)]
    ar = GradArena(ps, "cpu")
    offs = [ar.offsets[id(p)][0] for p in ps]
    assert offs == [0, 4, 12, 20, 24]
    for p in ps:
        ar.view(p).fill_(1.0)
    assert ar.flat.sum().item() == sum(p.numel() for p in ps)


def _bucket_body(rank, world):
    from mae_clip_amd.distributed import DataParallel
    m, cfg, batch = _model_and_batch(world)
    dp = DataParallel(m, bucket_mb=0.05, tail_mb=0.01)
    sizes = [sum(p.numel() * 4 for p in b) for b in dp.buckets]
    flat = [id(p) for b in dp.buckets for p in b]
    order = [id(p) for p in reversed([p for p in m.parameters() if p.requires_grad])]
    one = max(p.numel() * 4 for p in dp.buckets[-1])
    return sizes, flat == order, one


def test_data_parallel_tail_bucket_is_small():
    """The last all-reduce bucket (the gradients the backward produces last:
    bottom encoder block + patch embedding, exposed after the backward) is cut
    at tail_mb; buckets still cover every parameter once, in arena order."""
    (sizes, ordered, one), = run_ranks(_bucket_body, world=1)
    assert ordered
    assert sizes[-1] <= max(0.01 * 2 ** 20, one)
    assert max(sizes[:-1]) > 0.01 * 2 ** 20
