// Shared device/host helpers for libmaeclip (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this library:
//   * bf16 tensors are passed as raw uint16 bit patterns (bf16_t); fp32 as float.
//   * Every entry point receives the caller's hipStream_t and never allocates:
//     workspaces are carved by the Python host from the torch caching allocator.
//   * Errors are reported through a negative return code plus a thread-local
//     message (maeclip_last_error), mirroring torch's RuntimeError convention
//     that the reference's main.py relies on (main.py:54-66 has no handling).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

typedef uint16_t bf16_t;

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));

#define MAECLIP_F32 0
#define MAECLIP_BF16 1

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ---------------------------------------------------------------- host errors
namespace maeclip {
void set_error(const char* fmt, ...);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for a kernel only when a
// launch needs more dynamic LDS than was allowed before (runtime.hip): one
// call per kernel in practice, none per launch
void allow_lds(const void* kernel, int bytes);
// plan option `key` (MAECLIP_OPT_*), or dflt when unset (runtime.hip)
int option(int key, int dflt);
}

#define MC_CHECK_ARG(cond, ...)                  \
  do {                                           \
    if (!(cond)) {                               \
      maeclip::set_error(__VA_ARGS__);           \
      return -1;                                 \
    }                                            \
  } while (0)

#define MC_CHECK_LAUNCH(name)                                                   \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      maeclip::set_error("%s: launch failed: %s", name, hipGetErrorString(_e)); \
      return -2;                                                                \
    }                                                                           \
  } while (0)

// ------------------------------------------------------------- device helpers
// XCD-chunked workgroup id. The dispatcher deals consecutive workgroups
// round-robin over the 8 XCDs; this bijective remap hands each XCD a contiguous
// range of logical ids, so workgroups that read the same rows (e.g. the heads
// of one sample) share that XCD's L2 (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_chunk_id(int bid, int G) {
  const int q = G >> 3, r = G & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float bf2f(bf16_t u) {
  return __uint_as_float(((unsigned)u) << 16);
}
// Round-to-nearest-even; NaN stays NaN (hipcc lowers the cast to v_cvt_pk_bf16_f32).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}
// two f32 -> packed bf16 pair (a low) in ONE v_cvt_pk_bf16_f32 (the
// or-of-two-casts form costs two conversions and a v_or_b32_sdwa)
typedef __bf16 mc_bf16x2 __attribute__((ext_vector_type(2)));
typedef float mc_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2bf(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((mc_f32x2){a, b}, mc_bf16x2));
}

template <typename T> __device__ __forceinline__ float ld_as_f(const T* p);
template <> __device__ __forceinline__ float ld_as_f<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_as_f<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename T> __device__ __forceinline__ void st_from_f(T* p, float v);
template <> __device__ __forceinline__ void st_from_f<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st_from_f<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// 4 consecutive elements <-> float4 (vectorised: 16 B for f32, 8 B for bf16)
template <typename T> __device__ __forceinline__ v4f ld4(const T* p);
template <> __device__ __forceinline__ v4f ld4<float>(const float* p) { return *(const v4f*)p; }
template <> __device__ __forceinline__ v4f ld4<bf16_t>(const bf16_t* p) {
  v2u u = *(const v2u*)p;
  v4f r;
  r[0] = __uint_as_float(u[0] << 16);
  r[1] = __uint_as_float(u[0] & 0xffff0000u);
  r[2] = __uint_as_float(u[1] << 16);
  r[3] = __uint_as_float(u[1] & 0xffff0000u);
  return r;
}
template <typename T> __device__ __forceinline__ void st4(T* p, v4f v);
template <> __device__ __forceinline__ void st4<float>(float* p, v4f v) { *(v4f*)p = v; }
template <> __device__ __forceinline__ void st4<bf16_t>(bf16_t* p, v4f v) {
  v2u u;
  u[0] = pack2bf(v[0], v[1]);
  u[1] = pack2bf(v[2], v[3]);
  *(v2u*)p = u;
}

// OCP fp8 (gfx950 v_cvt_pk_fp8_f32 = e4m3fn, v_cvt_pk_bf8_f32 = e5m2, RNE) of
// four values -> one dword; row quantisation "q = rne(x / s), s = amax / MAX"
// (fp8.hip, layernorm.hip)
constexpr float MC_E4M3_MAX = 448.f;
constexpr float MC_E5M2_MAX = 57344.f;
template <bool E5> __device__ __forceinline__ unsigned mc_cvt4_fp8(float a, float b, float c, float d) {
  int r;
  if (E5) {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  }
  return (unsigned)r;
}

// fp8 BLOCKS (MX-style operands of v_mfma_scale_f32_16x16x128_f8f6f4; maeclip.h
// "fp8 blocks"): one e8m0 exponent per 32 consecutive K-elements of a row.
// The exponent is the smallest power of two 2^(e-127) with amax / 2^(e-127) <=
// FMT_MAX (448 = 1.75 * 2^8 for e4m3, 57344 = 1.75 * 2^15 for e5m2), taken from
// the bits of amax: no division, and x * 2^(127-e) is exact, so q =
// rne(x * 2^(127-e)) never overflows. amax = 0 gives e = 0 (q = 0).
__device__ __forceinline__ unsigned mc_e8m0(float amax, bool e5) {
  const unsigned u = __float_as_uint(amax);
  int e = (int)(u >> 23) - (e5 ? 15 : 8) + ((u & 0x7fffffu) > 0x600000u ? 1 : 0);
  return (unsigned)(e < 0 ? 0 : e);
}
// 2^(127 - e): the quantisation multiplier of exponent e (e <= 253)
__device__ __forceinline__ float mc_e8m0_inv(unsigned e) { return __uint_as_float((254u - e) << 23); }
// byte offset of the scale of row r, K-block b (32 elements) in a scale tensor
// for K = 128 T: [row / 64][K-tile b / 4][block b % 4][row % 16][(row / 16) % 4].
// The GEMM reads, per K-tile, one 256-byte run per 64-row group: lane (row
// fragment r % 16, block g) the dword holding the scales of rows r, r + 16,
// r + 32, r + 48, selected by the MFMA's scale byte select.
__host__ __device__ __forceinline__ int64_t mc_fp8b_off(int64_t r, int64_t b, int64_t T) {
  return ((((r >> 6) * T + (b >> 2)) << 8) | ((b & 3) << 6) | ((r & 15) << 2) | ((r >> 4) & 3));
}
__host__ __device__ __forceinline__ int64_t mc_fp8b_bytes(int64_t rows, int64_t K) {
  return (rows + 63) / 64 * 64 * (K / 32);
}

// erf-GELU (nn.GELU() / HF "gelu" / timm default) and its derivative sharing
// one exp: Phi(x) = 0.5 erfc(-x/sqrt2) with erfc by Abramowitz & Stegun 7.1.26
// (|err| <= 1.5e-7; |gelu err| <= 4.2e-7 over [-12,12], the same as f32 erff),
// phi(x) = exp(-x^2/2)/sqrt(2 pi). The tail is taken from erfc directly, so
// gelu(x) for x << 0 has no cancellation.
__device__ __forceinline__ void gelu_pair(float x, float& y, float& dy) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float e = __expf(-0.5f * x * x);
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float ht = 0.5f * p * t * e;           // 0.5 erfc(|x|/sqrt2)
  const float cdf = x < 0.f ? ht : 1.0f - ht;
  y = x * cdf;
  dy = fmaf(x * e, 0.39894228040143268f, cdf);
}
// The same pair for two values at once: every add / mul / fma of the erfc
// polynomial on a float2, which gfx950 issues as one v_pk_* instruction for
// both (no MFMA beside it in a GEMM epilogue, where the GELU math is the
// VALU-bound part); the two rcp / exp stay per value. Same formula, so the
// result is the scalar pair's to within the packed ops' rounding (identical
// operations: bitwise equal on gfx950).
__device__ __forceinline__ void gelu_pair2(mc_f32x2 x, mc_f32x2& y, mc_f32x2& dy) {
  const mc_f32x2 ax = {fabsf(x[0]), fabsf(x[1])};
  const mc_f32x2 z = ax * 0.70710678118654752f;
  const mc_f32x2 den = __builtin_elementwise_fma(z, (mc_f32x2){0.3275911f, 0.3275911f}, (mc_f32x2){1.0f, 1.0f});
  const mc_f32x2 t = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
  const mc_f32x2 h = (x * x) * -0.5f;
  const mc_f32x2 e = {__expf(h[0]), __expf(h[1])};
  mc_f32x2 p = __builtin_elementwise_fma(t, (mc_f32x2){1.061405429f, 1.061405429f}, (mc_f32x2){-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(t, p, (mc_f32x2){1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(t, p, (mc_f32x2){-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(t, p, (mc_f32x2){0.254829592f, 0.254829592f});
  const mc_f32x2 ht = ((p * t) * e) * 0.5f;              // 0.5 erfc(|x|/sqrt2)
  const mc_f32x2 cdf = {x[0] < 0.f ? ht[0] : 1.0f - ht[0], x[1] < 0.f ? ht[1] : 1.0f - ht[1]};
  y = x * cdf;
  dy = __builtin_elementwise_fma(x * e, (mc_f32x2){0.39894228040143268f, 0.39894228040143268f}, cdf);
}
// The GEMM epilogue's form of the same pair over NP value pairs at once, each
// step applied to every pair before the next (the dependent packed ops of one
// pair would otherwise stand back to back and take a wait state each), with
// the constants folded:
//   t   = 1 / (1 + (p / sqrt2) |x|)                 (|x| as an fma source modifier)
//   phi = 2^(x (x (-log2(e) / 2)) + log2(1 / sqrt(2 pi)))  = exp(-x^2/2) / sqrt(2 pi)
//   ht  = t P'(t) phi,  P' = sqrt(pi / 2) P          = 0.5 erfc(|x| / sqrt2)
//   cdf = x < 0 ? ht : 1 - ht                       (sign mask + bit select, no compare)
//   y = x cdf,  dy = x phi + cdf
// The same approximation as gelu_pair; the result differs from it only by the
// rounding of the folded constants (a few f32 ulp, far below the bf16 output).
template <int NP>
__device__ __forceinline__ void gelu_pairs(const mc_f32x2 (&x)[NP], mc_f32x2 (&y)[NP], mc_f32x2 (&dy)[NP]) {
  constexpr float KD = 0.3275911f * 0.70710678118654752f;
  constexpr float KE = -0.72134752044448170f;          // -log2(e) / 2
  constexpr float KC = -1.3257480647361593f;           // log2(1 / sqrt(2 pi))
  constexpr float S = 1.2533141373155003f;             // sqrt(pi / 2) = 0.5 sqrt(2 pi)
  mc_f32x2 t[NP], e[NP], p[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) t[i][h] = fmaf(fabsf(x[i][h]), KD, 1.0f);
#pragma unroll
  for (int i = 0; i < NP; ++i) e[i] = x[i] * KE;
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) t[i][h] = __builtin_amdgcn_rcpf(t[i][h]);
#pragma unroll
  for (int i = 0; i < NP; ++i) e[i] = __builtin_elementwise_fma(e[i], x[i], (mc_f32x2){KC, KC});
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) e[i][h] = __builtin_amdgcn_exp2f(e[i][h]);
#pragma unroll
  for (int i = 0; i < NP; ++i)
    p[i] = __builtin_elementwise_fma(t[i], (mc_f32x2){1.061405429f * S, 1.061405429f * S},
                                     (mc_f32x2){-1.453152027f * S, -1.453152027f * S});
#pragma unroll
  for (int i = 0; i < NP; ++i) p[i] = __builtin_elementwise_fma(t[i], p[i], (mc_f32x2){1.421413741f * S, 1.421413741f * S});
#pragma unroll
  for (int i = 0; i < NP; ++i) p[i] = __builtin_elementwise_fma(t[i], p[i], (mc_f32x2){-0.284496736f * S, -0.284496736f * S});
#pragma unroll
  for (int i = 0; i < NP; ++i) p[i] = __builtin_elementwise_fma(t[i], p[i], (mc_f32x2){0.254829592f * S, 0.254829592f * S});
#pragma unroll
  for (int i = 0; i < NP; ++i) p[i] = p[i] * t[i];
#pragma unroll
  for (int i = 0; i < NP; ++i) p[i] = p[i] * e[i];                      // ht
#pragma unroll
  for (int i = 0; i < NP; ++i) t[i] = (mc_f32x2){1.0f, 1.0f} - p[i];      // 1 - ht
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // all ones for x < 0; one v_bfi_b32 (written out: as C the select
      // becomes a compare into an SGPR pair + v_cndmask, with wait states)
      const int m = __float_as_int(x[i][h]) >> 31;
      float r;
      asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(p[i][h]), "v"(t[i][h]));
      t[i][h] = r;
    }
#pragma unroll
  for (int i = 0; i < NP; ++i) y[i] = x[i] * t[i];
#pragma unroll
  for (int i = 0; i < NP; ++i) dy[i] = __builtin_elementwise_fma(x[i], e[i], t[i]);
}
// gelu and gelu' of the 4 lanes of v: v <- gelu(v), returns gelu'(v)
__device__ __forceinline__ v4f gelu4_inplace(v4f& v) {
  v4f d;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float y, dy;
    gelu_pair(v[r], y, dy);
    v[r] = y;
    d[r] = dy;
  }
  return d;
}
__device__ __forceinline__ float gelu_f(float x) {
  float y, dy;
  gelu_pair(x, y, dy);
  return y;
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float y, dy;
  gelu_pair(x, y, dy);
  return dy;
}

// Sum over the 16 lanes of each row (lanes 16r .. 16r+15) with four DPP adds
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror): VALU only,
// no ds_bpermute round trips. Every lane of the row gets the row's sum, in a
// fixed order (deterministic).
template <int CTRL> __device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}

__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// whole-wave sum / max: DPP within each 16-lane row, then the four row
// results combined through v_readlane (no LDS round trips); every lane gets
// the same value, in a fixed order
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// fp8 copy (per-row scale) of a row held by one wave (lane: NC chunks of 4 at c * 256 + 4 lane),
// bit-identical to maeclip_quant_rows_fp8 of the stored row: s = amax / MAX
// (1 if amax = 0), q = rne(v / s)
template <int NC>
__device__ __forceinline__ void quant_row_fp8(const float (&v)[NC][4], float amax, bool e5, uint8_t* q, float* scale,
                                              int D, int lane) {
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / (e5 ? MC_E5M2_MAX : MC_E4M3_MAX) : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) *scale = s;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e = c * 256 + lane * 4;
    if (e < D)
      *(unsigned*)(q + e) = e5 ? mc_cvt4_fp8<true>(v[c][0] * inv, v[c][1] * inv, v[c][2] * inv, v[c][3] * inv)
                               : mc_cvt4_fp8<false>(v[c][0] * inv, v[c][1] * inv, v[c][2] * inv, v[c][3] * inv);
  }
}

// Counter-based hash used for dropout keep-masks and MAE mask noise.
// splitmix64 finaliser; restated bit-exactly in oracle/maskrng.py.
__host__ __device__ __forceinline__ uint64_t mc_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// seed of a dropout / noise draw at the current device step (MAECLIP_STEP_MULT, maeclip.h)
__device__ __forceinline__ uint64_t mc_step_seed(uint64_t seed, const int64_t* step_ptr) {
  return step_ptr ? seed + (uint64_t)(*step_ptr) * 0x9E3779B97F4A7C15ull : seed;
}
__host__ __device__ __forceinline__ uint32_t mc_hash4(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = mc_mix64(seed);
  h = mc_mix64(h ^ a);
  h = mc_mix64(h ^ b);
  h = mc_mix64(h ^ c);
  return (uint32_t)(h >> 32);
}

// albumentations Normalize(mean, std, max_pixel_value) (dataset.py:49) as fp32
// constants: m = f32(mean) * max_pixel, d = 1 / (f32(std) * max_pixel) (IEEE
// fp32 product then reciprocal, on the host); a pixel x maps to
// __fmul_rn(f32(x) - m, d) -- two roundings, no FMA. Shared by the input
// pipeline (input.hip) and the kernels that read uint8 HWC pixels directly
// (patch gather, MAE targets in mae.hip), so both routes give identical floats.
struct NormConst {
  float m[3], d[3];
};
// returns false on a non-positive std / max_pixel
inline bool mc_norm_const(const float* mean, const float* stdv, float max_pixel, NormConst& k) {
  if (!(max_pixel > 0.f)) return false;
  for (int c = 0; c < 3; ++c) {
    if (!(stdv[c] > 0.f)) return false;
    k.m[c] = mean[c] * max_pixel;
    const volatile float sd = stdv[c] * max_pixel;
    k.d[c] = 1.0f / sd;
  }
  return true;
}
__device__ __forceinline__ float mc_norm_px(unsigned x, const NormConst& k, int c) {
  return __fmul_rn((float)x - k.m[c], k.d[c]);
}
