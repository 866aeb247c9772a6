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


# ---------------------------------------------------------------- Resize
# dataset.py:48 A.Resize(size, size) = cv2.resize(img, (size, size),
# interpolation=cv2.INTER_LINEAR) (albumentations 1.3.1 default). OpenCV
# (opencv-python is absent here: parity unpinned) restated from its published
# resize.cpp for CV_8UC3:
#   * equal sizes: copy; exact 2x downscale on both axes: INTER_AREA fast path,
#     dst = (a + b + c + d + 2) >> 2;
#   * otherwise fixed point, INTER_RESIZE_COEF_BITS = 11:
#       scale = 1 / (dst / src)  (double);  f = float((d + 0.5) * scale - 0.5)
#       s = floor(f); f -= s; s < 0 -> (s, f) = (0, 0); s >= n - 1 -> (n - 1, 0)
#       a0 = rint((1 - f) * 2048), a1 = rint(f * 2048)   (saturate_cast<short>)
#       horizontal (int32): h = S[sx] a0 + S[sx + 1] a1   (S[sx] * 2048 at the right border)
#       vertical, the SIMD VResizeLinearVec_32s8u form every x86 / ARM build runs
#       on these row widths:  u8((((h0 >> 4) b0) >> 16) + (((h1 >> 4) b1) >> 16) + 2) >> 2)
def _linear_coefs(n_src, n_dst):
    scale = 1.0 / (float(n_dst) / float(n_src))
    d = np.arange(n_dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo], f[lo] = 0, 0
    hi = s >= n_src - 1
    s[hi], f[hi] = n_src - 1, 0
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    s1 = np.minimum(s + 1, n_src - 1)
    a1 = np.where(hi, 0, a1)
    return s, s1, a0, a1


def resize_u8_linear_ref(img_hwc, size):
    """cv2.resize(img, (size, size), interpolation=INTER_LINEAR) for uint8 HWC."""
    H, W, C = img_hwc.shape
    if H == size and W == size:
        return img_hwc.copy()
    src = img_hwc.astype(np.int64)
    if H == 2 * size and W == 2 * size:
        return ((src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    xs0, xs1, xa0, xa1 = _linear_coefs(W, size)
    ys0, ys1, yb0, yb1 = _linear_coefs(H, size)
    h = src[:, xs0, :] * xa0[None, :, None] + src[:, xs1, :] * xa1[None, :, None]     # [H, size, C]
    h0, h1 = h[ys0], h[ys1]
    v = ((((h0 >> 4) * yb0[:, None, None]) >> 16) + (((h1 >> 4) * yb1[:, None, None]) >> 16) + 2) >> 2
    return np.clip(v, 0, 255).astype(np.uint8)


def preprocess_ref(images, size, **norm):
    """dataset.py:44-58 + :34 for a list of uint8 HWC images of any sizes:
    Resize -> Normalize -> CHW float32, stacked [B, 3, size, size]."""
    return np.concatenate([normalize_u8_ref(resize_u8_linear_ref(im, size)[None], **norm) for im in images])
