"""CPU restatement of the reference's image transform (test infrastructure only:
imported by tests/, never by the product).

dataset.py:44-58 builds A.Compose([A.Resize(size, size), A.Normalize(max_pixel_value=255.0)])
and dataset.py:34 turns the result into torch.tensor(image).permute(2, 0, 1).float().
albumentations (pinned 1.3.1 in requirements.txt) is not installed here; its
published normalize() is restated:
    mean = np.array(mean, dtype=np.float32) * max_pixel_value
    std = np.array(std, dtype=np.float32) * max_pixel_value
    denominator = np.reciprocal(std, dtype=np.float32)
    img = (img.astype(np.float32) - mean) * denominator
Parity of this restatement with the library itself is unpinned (no fixture in
the reference exercises the transform); the GPU kernel is checked bit-exactly
against it."""
import numpy as np


def normalize_u8_ref(images_u8_nhwc, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), max_pixel_value=255.0):
    m = np.array(mean, dtype=np.float32) * np.float32(max_pixel_value)
    s = np.array(std, dtype=np.float32) * np.float32(max_pixel_value)
    den = np.reciprocal(s, dtype=np.float32)
    img = (images_u8_nhwc.astype(np.float32) - m) * den          # HWC, per-channel broadcast
    return np.ascontiguousarray(img.transpose(0, 3, 1, 2))       # permute(2, 0, 1) per image
