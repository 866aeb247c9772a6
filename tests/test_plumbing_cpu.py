"""Host-side plumbing of the product on CPU, with every kernel LAUNCH stubbed
out (the library's host-only query entry points -- workspace sizes, partial
row counts -- are the real ones from libmaeclip.so). It runs CLIPModel
forward/backward/AdamW through every autograd Function and ctypes wrapper,
and the data-parallel GradArena path on two gloo ranks, so signature or
bookkeeping errors surface here instead of on the GPU box. Numbers computed
with stubbed launches are meaningless; only shapes, call sequences, gradient
ownership and the all-reduce bucketing are checked. The real-kernel versions
of these tests are test_model_gpu.py / test_distributed_gpu.py."""
import contextlib
import ctypes
import functools
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import product_config, make_batch, C0

# host-only entry points (no device work): keep the real implementation
_QUERIES = {"maeclip_abi_version", "maeclip_last_error", "maeclip_device_count", "maeclip_gemm_colsum_rows",
            "maeclip_gemm_workspace", "maeclip_gemm_splitk", "maeclip_wgrad_grouped_workspace",
            "maeclip_ln_bwd_partial_rows", "maeclip_rows_colsum_partial_rows", "maeclip_mt_chunk",
            "maeclip_clip_loss_workspace", "maeclip_wallclock_khz", "maeclip_unshuffle_bwd_partial_rows",
            "maeclip_mae_loss_bwd_partial_rows"}


class _StubLib:
    def __init__(self, real):
        self._real = real
        self.calls = []

    def __getattr__(self, name):
        if name in _QUERIES:
            return getattr(self._real, name)
        fn = getattr(self._real, name)   # AttributeError for unknown symbols, like the real lib

        def launch(*args):
            assert len(args) == len(fn.argtypes), (name, len(args), len(fn.argtypes))
            self.calls.append(name)
            return 0
        return launch


class _Stream:
    cuda_stream = 0

    def wait_stream(self, other):
        pass


@contextlib.contextmanager
def stubbed_kernels(monkeypatch):
    from mae_clip_amd import _lib, kernels as K, modules as Mo, CLIP as CL, config as CFG
    real = _lib.load()
    monkeypatch.setattr(CFG, "side_stream", False)
    stub = _StubLib(real)
    monkeypatch.setattr(_lib, "lib", lambda: stub)
    monkeypatch.setattr(K, "_dev", lambda *ts: None)
    monkeypatch.setattr(Mo, "_require_device", lambda t, what: None)
    monkeypatch.setattr(CL, "_require_device", lambda t, what: None)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _Stream())
    monkeypatch.setattr(K, "_capturing", lambda: False)

    def stage(self, host_struct_array, device):
        raw = bytes(memoryview(host_struct_array).cast("B"))
        return torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    monkeypatch.setattr(K.PinnedStager, "stage", stage)
    yield stub


def _model(precision, **over):
    from mae_clip_amd.CLIP import CLIPModel
    kw = {k: v for k, v in C0.items() if k != "batch_size"}
    kw.update(over)
    with product_config(precision=precision, side_stream=False, **kw):
        torch.manual_seed(0)
        return CLIPModel()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("mask_ratio", [0.75, 0.0])
def test_training_step_plumbing(monkeypatch, precision, mask_ratio):
    from mae_clip_amd.optim import AdamW
    with stubbed_kernels(monkeypatch) as stub:
        m = _model(precision, mask_ratio=mask_ratio).train()
        opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-3)
        for B in (8, 5):
            opt.zero_grad(set_to_none=True)
            loss = m(make_batch(B, 32))
            assert loss.shape == ()
            loss.backward()
            for n, p in m.named_parameters():
                if p.requires_grad:
                    assert p.grad is not None and p.grad.shape == p.shape and p.grad.dtype == torch.float32, n
            opt.step()
        assert "maeclip_clip_loss" in stub.calls and "maeclip_adamw_multi" in stub.calls
        assert ("maeclip_mae_loss_bwd" in stub.calls) == (mask_ratio > 0)


def test_vitl14_padded_shapes_plumbing(monkeypatch):
    """patch 14 (K = 588 padded to 640, decoder_pred rows padded) bookkeeping."""
    with stubbed_kernels(monkeypatch):
        m = _model("bf16", model_name="vit_large_patch14_336", size=336, image_embedding=1024,
                   decoder_embed_dim=512, decoder_depth=1, decoder_num_heads=16)
        m.image_encoder.model.blocks = m.image_encoder.model.blocks[:1]
        m._cache = None
        loss = m(make_batch(2, 336))
        loss.backward()
        pe = m.image_encoder.model.patch_embed.proj.weight
        assert pe.grad.shape == pe.shape == (1024, 3, 14, 14)
        dp = m.mae_decoder.decoder_pred
        assert dp.weight.grad.shape == (588, 512) and dp.bias.grad.shape == (588,)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mp_ = pytest.MonkeyPatch()
        with stubbed_kernels(mp_):
            from mae_clip_amd.distributed import DataParallel
            m = _model("bf16").train()
            dp = DataParallel(m, bucket_mb=0.5)
            for _ in range(2):
                for p in m.parameters():
                    p.grad = None
                dp.reset_stats()
                m(make_batch(4, 32, seed=rank)).backward()
                dp.sync_gradients()
            owned = all(dp.arena.owns(p) for p in dp.params)
            out[rank] = (dp.adopted, len(dp.params), len(dp.buckets), owned)
        mp_.undo()
    finally:
        dist.destroy_process_group()


def test_data_parallel_arena_plumbing():
    """Under DataParallel every trainable gradient is produced in its GradArena
    slot by the product's Functions (adopted by autograd without a copy), and
    the bucketed all-reduce runs on arena slices."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_dp_rank, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        adopted, nparams, nbuckets, owned = out[r]
        assert adopted == nparams, (adopted, nparams)
        assert nbuckets > 2 and owned


def test_chunk_bounds():
    from mae_clip_amd.modules import chunk_bounds
    assert chunk_bounds(12, None) == [(0, 12)]
    assert chunk_bounds(12, 6) == [(0, 6), (6, 12)]
    assert chunk_bounds(12, (2, 4, 6)) == [(0, 2), (2, 6), (6, 12)]
    assert chunk_bounds(12, (1, 2, 3, 6)) == [(0, 1), (1, 3), (3, 6), (6, 12)]
    assert chunk_bounds(8, (2, 4, 6)) == [(0, 2), (2, 6), (6, 8)]
    assert chunk_bounds(5, (2,)) == [(0, 2), (2, 4), (4, 5)]
