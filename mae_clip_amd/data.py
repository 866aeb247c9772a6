"""Device-side input pipeline.

The reference's CLIPDataset.__getitem__ (dataset.py:24-37) decodes each image
with cv2 (BGR -> RGB), runs albumentations Resize + Normalize
(get_transforms, dataset.py:44-58) and permutes HWC -> CHW float32 on the host;
main.py:55 then copies the fp32 batch to the GPU. Here decoding stays on the
host (cv2 / PIL, unchanged); the decoded uint8 HWC images cross PCIe as they
are (any sizes, 4x fewer bytes than the fp32 batch), and libmaeclip resizes,
normalises and transposes them in HBM in one pass
(maeclip_image_preprocess_u8 = Resize + Normalize + permute), producing
exactly the tensor the model takes. normalize_u8 is the resize-free variant
for batches already at the model's size.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from .kernels import _dev, _call, _stream

# ImageNet statistics of albumentations' A.Normalize defaults (dataset.py:49)
from .kernels import IMAGENET_MEAN, IMAGENET_STD  # noqa: E402


def normalize_u8(images: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD, max_pixel_value=255.0,
                 out: torch.Tensor = None) -> torch.Tensor:
    """uint8 [B, H, W, 3] (RGB, HWC) on the device -> float32 [B, 3, H, W]:
    (x - mean * max_pixel_value) / (std * max_pixel_value), albumentations'
    normalize() arithmetic in fp32 (dataset.py:49, 34)."""
    _dev(images, out)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
        raise ValueError(f"normalize_u8: expected uint8 [B, H, W, 3], got {images.dtype} {tuple(images.shape)}")
    images = images.contiguous()
    B, H, W, _ = images.shape
    if out is None:
        out = torch.empty((B, 3, H, W), device=images.device, dtype=torch.float32)
    elif out.shape != (B, 3, H, W) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("normalize_u8: out must be a dense float32 [B, 3, H, W]")
    a = L.ImageU8Args(src=images.data_ptr(), dst=out.data_ptr(), B=B, H=H, W=W,
                      mean=(C.c_float * 3)(*mean), std=(C.c_float * 3)(*std), max_pixel=max_pixel_value)
    _call("maeclip_image_normalize_u8", C.byref(a), _stream())
    return out


def preprocess_images(images, size, mean=IMAGENET_MEAN, std=IMAGENET_STD, max_pixel_value=255.0, out=None):
    """get_transforms() of dataset.py:44-58 (+ the permute of :34) on the device:
    a list of uint8 HWC RGB images of any sizes (device tensors; row-strided
    views allowed) -> float32 [B, 3, size, size]: A.Resize(size, size) with
    cv2.INTER_LINEAR semantics, then A.Normalize."""
    if not images:
        raise ValueError("preprocess_images: empty image list")
    dev = images[0].device
    descs = (L.ImageSrc * len(images))()
    for i, im in enumerate(images):
        _dev(im)
        if im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3 or im.stride(2) != 1 or im.stride(1) != 3:
            raise ValueError(f"preprocess_images: image {i} must be uint8 [H, W, 3] with packed pixels")
        if im.device != dev:
            raise ValueError("preprocess_images: images on different devices")
        descs[i].src, descs[i].H, descs[i].W, descs[i].row_stride = im.data_ptr(), im.shape[0], im.shape[1], im.stride(0)
    B = len(images)
    if out is None:
        out = torch.empty((B, 3, size, size), device=dev, dtype=torch.float32)
    elif out.shape != (B, 3, size, size) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("preprocess_images: out must be a dense float32 [B, 3, size, size]")
    d = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    a = L.PreprocessArgs(images=d.data_ptr(), dst=out.data_ptr(), B=B, S=size, mean=(C.c_float * 3)(*mean),
                         std=(C.c_float * 3)(*std), max_pixel=max_pixel_value)
    _call("maeclip_image_preprocess_u8", C.byref(a), _stream())
    return out


def to_device_batch(images_u8, input_ids, attention_mask, device, non_blocking=True):
    """The dict main.train_epoch feeds the model (main.py:55), built from a
    host uint8 HWC batch: upload uint8, normalise on the device."""
    imgs = images_u8.to(device, non_blocking=non_blocking)
    return {"image": normalize_u8(imgs), "input_ids": input_ids.to(device, non_blocking=non_blocking),
            "attention_mask": attention_mask.to(device, non_blocking=non_blocking)}
