"""Bit-exact numpy restatement of the MAE mask noise of libmaeclip
(mae_clip_amd/csrc/common.h mc_mix64 / mc_hash4, mae.hip mask_ids_kernel).
TEST INFRASTRUCTURE ONLY.

noise[b, l] = (hash(seed, step, sample_offset + b, l) >> 8) * 2**-24, a float32
that is exact (24-bit mantissa); ids_shuffle = argsort(noise, stable=True)
(HF ViTMAE random_masking, modeling_vit_mae.py:297-327, with an index tie-break).
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def hash4(seed, a, b, c):
    with np.errstate(over="ignore"):
        h = _mix64(np.asarray(seed, dtype=np.uint64))
        h = _mix64(h ^ np.asarray(a, dtype=np.uint64))
        h = _mix64(h ^ np.asarray(b, dtype=np.uint64))
        h = _mix64(h ^ np.asarray(c, dtype=np.uint64))
    return (h >> np.uint64(32)).astype(np.uint32)


def keys24(seed, step, sample_offset, B, L):
    b = (np.arange(B, dtype=np.uint64) + np.uint64(sample_offset))[:, None]
    l = np.arange(L, dtype=np.uint64)[None, :]
    return hash4(np.uint64(seed), np.uint64(step), b, l) >> np.uint32(8)


def noise(seed, step, sample_offset, B, L):
    return (keys24(seed, step, sample_offset, B, L).astype(np.float64) * 2.0 ** -24).astype(np.float32)
