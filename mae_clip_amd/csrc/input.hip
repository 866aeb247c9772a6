// Input pipeline on the device.
//
// Replaces the per-image host transform of dataset.py:44-58: the decoded RGB
// uint8 HWC image (cv2.imread + cvtColor, dataset.py:30-33) goes through
// albumentations Normalize(max_pixel_value=255) (dataset.py:49) and
// torch.tensor(image).permute(2, 0, 1).float() (dataset.py:34). The batch is
// uploaded as uint8 (a quarter of the fp32 bytes over PCIe) and normalised
// here, in HBM, straight into the model's NCHW fp32 input.
//
// maeclip_image_preprocess_u8 adds the resize in the same pass: images of any
// size (one descriptor each) -> A.Resize(S, S) = cv2.resize INTER_LINEAR
// (dataset.py:48; OpenCV's fixed-point uint8 algorithm, see oracle/input_ref.py)
// -> Normalize -> NCHW fp32 [B, 3, S, S]: the whole get_transforms() pipeline.
//
// Arithmetic is albumentations' normalize(): mean32 = f32(mean) * max_pixel,
// den32 = 1 / (f32(std) * max_pixel) (both fp32, computed on the host with
// IEEE division), out = (f32(x) - mean32) * den32 -- two roundings, no FMA.
// HBM-bound: 3 B read + 12 B written per pixel.
#include "common.h"
#include "../../include/maeclip.h"

namespace {
constexpr int NTH = 256;

// 4 consecutive pixels of one row per thread: three 4-B loads of interleaved
// RGB, one 16-B store per plane (W % 4 == 0)
__global__ void __launch_bounds__(NTH) normalize_u8_x4_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                               int64_t npix4, int64_t HW, NormConst k) {
  const int64_t q = (int64_t)blockIdx.x * NTH + threadIdx.x;
  if (q >= npix4) return;
  const int64_t pix = q * 4;              // global pixel index b*HW + y*W + x
  const int64_t b = pix / HW, off = pix % HW;
  const uint32_t* s = (const uint32_t*)(src + pix * 3);
  const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];
  const uint8_t v[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                         (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                         (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    v4f o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = mc_norm_px(v[3 * j + c], k, c);
    }
    *(v4f*)(dst + (b * 3 + c) * HW + off) = o;
  }
}

__global__ void __launch_bounds__(NTH) normalize_u8_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                            int64_t npix, int64_t HW, NormConst k) {
  const int64_t pix = (int64_t)blockIdx.x * NTH + threadIdx.x;
  if (pix >= npix) return;
  const int64_t b = pix / HW, off = pix % HW;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    dst[(b * 3 + c) * HW + off] = mc_norm_px(src[pix * 3 + c], k, c);
  }
}
// OpenCV INTER_LINEAR source index / fixed-point weights of output coordinate d
// (resize.cpp, CV_8U: float f from double arithmetic, weights
// saturate_cast<short>(w * 2048) = rint, borders clamp with weight 0)
struct Lin {
  int s0, s1, a0, a1;
};
__device__ __forceinline__ Lin lin_coef(int d, int n_src, int n_dst) {
  const double scale = 1.0 / ((double)n_dst / (double)n_src);
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  bool hi = false;
  if (s < 0) { s = 0; f = 0.f; }
  if (s >= n_src - 1) { s = n_src - 1; f = 0.f; hi = true; }
  Lin r;
  r.s0 = s;
  r.s1 = min(s + 1, n_src - 1);
  r.a0 = (int)rintf((1.f - f) * 2048.f);
  r.a1 = hi ? 0 : (int)rintf(f * 2048.f);
  return r;
}

// one output pixel (3 channels) per thread; grid (pixel blocks, image)
__global__ void __launch_bounds__(NTH) preprocess_u8_kernel(const maeclip_image_src* __restrict__ imgs, float* __restrict__ dst,
                                                             int S, NormConst k) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * NTH + threadIdx.x;
  if (p >= S * S) return;
  const int dy = p / S, dx = p % S;
  const maeclip_image_src im = imgs[b];
  const uint8_t* src = im.src;
  const int H = im.H, W = im.W;
  const int64_t rs = im.row_stride;
  int v[3];
  if (H == S && W == S) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = src[dy * rs + dx * 3 + c];
  } else if (H == 2 * S && W == 2 * S) {   // cv2: exact 2x -> INTER_AREA fast path
    const uint8_t* r0 = src + (int64_t)(2 * dy) * rs + 2 * dx * 3;
    const uint8_t* r1 = r0 + rs;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (r0[c] + r0[3 + c] + r1[c] + r1[3 + c] + 2) >> 2;
  } else {
    const Lin x = lin_coef(dx, W, S), y = lin_coef(dy, H, S);
    const uint8_t* r0 = src + (int64_t)y.s0 * rs;
    const uint8_t* r1 = src + (int64_t)y.s1 * rs;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int h0 = r0[x.s0 * 3 + c] * x.a0 + r0[x.s1 * 3 + c] * x.a1;
      const int h1 = r1[x.s0 * 3 + c] * x.a0 + r1[x.s1 * 3 + c] * x.a1;
      // VResizeLinearVec_32s8u: mul_hi of (h >> 4) by the int16 weight, round by 2 bits
      const int t = (((h0 >> 4) * y.a0) >> 16) + (((h1 >> 4) * y.a1) >> 16);
      v[c] = min(max((t + 2) >> 2, 0), 255);
    }
  }
  const int64_t plane = (int64_t)S * S;
#pragma unroll
  for (int c = 0; c < 3; ++c) dst[((int64_t)b * 3 + c) * plane + p] = mc_norm_px(v[c], k, c);
}
}  // namespace

extern "C" int32_t maeclip_image_preprocess_u8(const maeclip_preprocess_args* a, void* stream) {
  MC_CHECK_ARG(a && a->images && a->dst, "maeclip_image_preprocess_u8: null pointer");
  MC_CHECK_ARG(a->B >= 0 && a->S > 0 && a->S <= 8192 && a->B <= 65535, "maeclip_image_preprocess_u8: bad sizes");
  NormConst k;
  MC_CHECK_ARG(mc_norm_const(a->mean, a->std, a->max_pixel, k),
               "maeclip_image_preprocess_u8: std and max_pixel must be > 0");
  if (a->B == 0) return 0;
  const int S = (int)a->S;
  hipLaunchKernelGGL(preprocess_u8_kernel, dim3((unsigned)((S * S + NTH - 1) / NTH), (unsigned)a->B), dim3(NTH), 0,
                     (hipStream_t)stream, a->images, a->dst, S, k);
  MC_CHECK_LAUNCH("maeclip_image_preprocess_u8");
  return 0;
}

extern "C" int32_t maeclip_image_normalize_u8(const maeclip_image_u8_args* a, void* stream) {
  MC_CHECK_ARG(a && a->src && a->dst, "maeclip_image_normalize_u8: null pointer");
  MC_CHECK_ARG(a->B >= 0 && a->H > 0 && a->W > 0, "maeclip_image_normalize_u8: bad sizes");
  NormConst k;
  MC_CHECK_ARG(mc_norm_const(a->mean, a->std, a->max_pixel, k),
               "maeclip_image_normalize_u8: std and max_pixel must be > 0");
  const int64_t HW = a->H * a->W, npix = a->B * HW;
  if (npix == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = a->W % 4 == 0 && ((uintptr_t)a->src & 3) == 0 && ((uintptr_t)a->dst & 15) == 0;
  if (vec) {
    const int64_t n4 = npix / 4;
    hipLaunchKernelGGL(normalize_u8_x4_kernel, dim3((unsigned)((n4 + NTH - 1) / NTH)), dim3(NTH), 0, s, a->src, a->dst,
                       n4, HW, k);
  } else {
    hipLaunchKernelGGL(normalize_u8_kernel, dim3((unsigned)((npix + NTH - 1) / NTH)), dim3(NTH), 0, s, a->src, a->dst,
                       npix, HW, k);
  }
  MC_CHECK_LAUNCH("maeclip_image_normalize_u8");
  return 0;
}
