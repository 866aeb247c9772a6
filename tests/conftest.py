import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm (gfx950) GPU and libmaeclip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    # a GPU test that runs without a GPU is a failure, not a skip
    assert torch.cuda.is_available(), "gpu-marked test but no ROCm device visible"
    from mae_clip_amd import _lib
    _lib.load()
    return torch.device("cuda:0")


@pytest.fixture
def opts():
    """set library plan options for one test (include/maeclip.h
    maeclip_set_option; the library reads the environment only once):
    opts(GEMM_BM=192, ...); every option set is restored afterwards"""
    from mae_clip_amd import kernels as K
    prev = {}

    def set_(**kw):
        for k, v in kw.items():
            old = K.set_option(k, v)
            prev.setdefault(k, old)

    yield set_
    for k, v in prev.items():
        K.set_option(k, v)
