// OCP fp8 quantisation for the fp8 GEMM path (C4, BASELINE.json configs[4]).
//
// Scaling recipe (SURVEY.md §8 row "fp8 MFMA path"): dequantisation scales per
// GEMM row -- per token for activations and gradients, per output channel for
// the forward weight W [N, K] and per input channel for the dgrad weight W^T
// [K, N] -- so every scale sits on the M or N side of the product and the GEMM
// applies s_a[m] * s_b[n] to its fp32 accumulator (maeclip_gemm_fp8). A row is
// quantised as q = rne(x / s), s = amax(row) / FMT_MAX (amax = 0 -> s = 1):
// "current" scaling, one pass, no amax history and no first-step special case.
//
//   maeclip_quant_rows_fp8 : [rows, cols] (bf16 or f32, row stride ld) ->
//                            fp8 [rows, ldq] + f32 scales [rows].
//                            One wave per row; the row stays in registers
//                            between the amax and the quantisation (cols <=
//                            4096, longer rows re-read from L2).
//   maeclip_quant_cols_fp8 : f32 [rows, cols] (the fp32 master of W) ->
//                            fp8 [cols, ldq] = quantised W^T, scales [cols]
//                            (per column of W): a partial-column-max pass and
//                            a quantise pass, both over 256 x 64 tiles of W,
//                            the transpose through LDS.
// Conversion: v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 (gfx950: OCP e4m3fn / e5m2,
// round to nearest even); |x / s| <= FMT_MAX by construction.
#include "common.h"
#include "../../include/maeclip.h"

namespace {

constexpr float E4M3_MAX = MC_E4M3_MAX;
constexpr float E5M2_MAX = MC_E5M2_MAX;

template <bool E5> __device__ __forceinline__ unsigned cvt4(float a, float b, float c, float d) {
  return mc_cvt4_fp8<E5>(a, b, c, d);
}

template <typename T> struct Row8;   // 8 consecutive elements as f32
template <> struct Row8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[8]) {
    const v4u u = *(const v4u*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(u[j] << 16);
      v[2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
    }
  }
};
template <> struct Row8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const v4f a = *(const v4f*)p, b = *(const v4f*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a[j];
      v[4 + j] = b[j];
    }
  }
};

constexpr int RCH = 8;   // row chunks of 512 elements kept in registers (cols <= 4096)

template <typename T, bool E5>
__global__ void __launch_bounds__(256) quant_rows_kernel(const T* __restrict__ x, int64_t rows, int cols, int64_t ld,
                                                         uint8_t* __restrict__ q, int64_t ldq,
                                                         float* __restrict__ scales) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * ld;
  const int nchunk = (cols + 511) / 512;
  float v[RCH][8];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < RCH; ++c) {
    const int e = c * 512 + lane * 8;
    if (c < nchunk && e < cols) {
      Row8<T>::load(xr + e, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[c][j]));
    }
  }
  for (int c = RCH; c < nchunk; ++c) {   // rows longer than 4096
    const int e = c * 512 + lane * 8;
    if (e < cols) {
      float w[8];
      Row8<T>::load(xr + e, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(w[j]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const float fmax_ = E5 ? E5M2_MAX : E4M3_MAX;
  const float s = amax > 0.f ? amax / fmax_ : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scales[row] = s;
  uint8_t* qr = q + row * ldq;
  for (int c = 0; c < nchunk; ++c) {
    const int e = c * 512 + lane * 8;
    if (e >= cols) continue;
    float w[8];
    if (c < RCH) {
#pragma unroll
      for (int cc = 0; cc < RCH; ++cc)
        if (cc == c) {
#pragma unroll
          for (int j = 0; j < 8; ++j) w[j] = v[cc][j];
        }
    } else {
      Row8<T>::load(xr + e, w);
    }
    v2u o;
    o[0] = cvt4<E5>(w[0] * inv, w[1] * inv, w[2] * inv, w[3] * inv);
    o[1] = cvt4<E5>(w[4] * inv, w[5] * inv, w[6] * inv, w[7] * inv);
    *(v2u*)(qr + e) = o;
  }
}

// W^T quantisation, two fully parallel passes over 64-column x 256-row tiles of
// W (grid = column strips x row chunks):
//   pass 1: partial column maxima of each tile -> part[chunk][col]
//   pass 2: every tile reduces its strip's partials (fixed order), writes the
//           column scales (chunk 0) and its 256 x 64 tile of W^T through LDS.
constexpr int QC_ROWS = 256;

__global__ void __launch_bounds__(256) quant_cols_amax_kernel(const float* __restrict__ w, int rows, int cols,
                                                              int64_t ld, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * QC_ROWS;
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;
  const int col = c0 + tc;
  float amax = 0.f;
  if (col < cols)
    for (int r = r0 + tr; r < min(rows, r0 + QC_ROWS); r += 4) amax = fmaxf(amax, fabsf(w[(int64_t)r * ld + col]));
  red[tr][tc] = amax;
  __syncthreads();
  if (tr == 0 && col < cols)
    part[(int64_t)blockIdx.y * cols + col] = fmaxf(fmaxf(red[0][tc], red[1][tc]), fmaxf(red[2][tc], red[3][tc]));
}

__global__ void __launch_bounds__(256) quant_cols_kernel(const float* __restrict__ w, int rows, int cols, int64_t ld,
                                                         const float* __restrict__ part, uint8_t* __restrict__ qt,
                                                         int64_t ldq, float* __restrict__ scales) {
  __shared__ float tile[64][65];
  __shared__ float inv_s[64];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * QC_ROWS;
  const int nchunks = gridDim.y;
  if (threadIdx.x < 64) {
    const int col = c0 + threadIdx.x;
    float a = 0.f;
    if (col < cols)
      for (int k = 0; k < nchunks; ++k) a = fmaxf(a, part[(int64_t)k * cols + col]);
    const float s = a > 0.f ? a / E4M3_MAX : 1.f;
    inv_s[threadIdx.x] = 1.f / s;
    if (blockIdx.y == 0 && col < cols) scales[col] = s;
  }
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;
  const int col = c0 + tc;
  for (int rb = r0; rb < min(rows, r0 + QC_ROWS); rb += 64) {
    __syncthreads();
    for (int rr = tr; rr < 64; rr += 4) {
      const int r = rb + rr;
      tile[rr][tc] = (r < rows && col < cols) ? w[(int64_t)r * ld + col] : 0.f;
    }
    __syncthreads();
    // thread -> (W^T row = strip column tc2, 16 consecutive W rows)
    const int tc2 = threadIdx.x >> 2, seg = threadIdx.x & 3;
    const float inv = inv_s[tc2];
    if (c0 + tc2 < cols && rb + seg * 16 < rows) {
      uint8_t* dst = qt + (int64_t)(c0 + tc2) * ldq + rb + seg * 16;
      v4u o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rr = seg * 16 + 4 * k;
        o[k] = cvt4<false>(tile[rr][tc2] * inv, tile[rr + 1][tc2] * inv, tile[rr + 2][tc2] * inv,
                           tile[rr + 3][tc2] * inv);
      }
      if (rb + seg * 16 + 16 <= rows) {
        *(v4u*)dst = o;
      } else {
        for (int k = 0; k < 16 && rb + seg * 16 + k < rows; ++k) dst[k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

// ---- all stack weights of a step in two launches (maeclip_quant_weights_fp8)
// entry lookup: the last entry whose prefix start is <= u (n <= a few hundred)
__device__ __forceinline__ int wentry(const maeclip_fp8w_entry* __restrict__ e, int n, int64_t u, bool strips) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((strips ? e[mid].unit_begin : e[mid].row_begin) <= u) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Launch 1: W rows (per output channel) AND the column partial maxima of W^T
// from ONE read of W. A workgroup owns WQ_G consecutive rows of one entry (16
// per wave, one row at a time in registers: cols <= 512 * RCH); every lane keeps
// the running |max| of its 8 columns per 512-column chunk over the wave's rows,
// the four waves' maxima meet in LDS, and the group writes one partial row
// part[part_begin + g * cols + col] (g = the entry's group index). Entries'
// row spaces are padded to WQ_G rows (row_begin), so no group straddles two.
constexpr int WQ_G = 64;

__global__ void __launch_bounds__(256) wq_rows_kernel(const maeclip_fp8w_entry* __restrict__ e, int n,
                                                      float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t grow0 = (int64_t)blockIdx.x * WQ_G;
  const maeclip_fp8w_entry& w = e[wentry(e, n, grow0, false)];
  const int r0 = (int)(grow0 - w.row_begin);
  const int cols = w.cols, nchunk = (cols + 511) / 512;
  float cm[RCH][8];
#pragma unroll
  for (int c = 0; c < RCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) cm[c][j] = 0.f;
  for (int i = 0; i < WQ_G / 4; ++i) {
    const int r = r0 + wave * (WQ_G / 4) + i;
    if (r >= w.rows) break;   // wave-uniform
    const float* xr = w.w + (int64_t)r * w.ld;
    float v[RCH][8];
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < RCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (c < nchunk && col < cols) {
        Row8<float>::load(xr + col, v[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = fabsf(v[c][j]);
          amax = fmaxf(amax, a);
          cm[c][j] = fmaxf(cm[c][j], a);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    const float s = amax > 0.f ? amax / E4M3_MAX : 1.f;
    const float inv = 1.f / s;
    if (lane == 0) w.sq[r] = s;
    uint8_t* qr = (uint8_t*)w.q + (int64_t)r * cols;
#pragma unroll
    for (int c = 0; c < RCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (c < nchunk && col < cols) {
        v2u o;
        o[0] = cvt4<false>(v[c][0] * inv, v[c][1] * inv, v[c][2] * inv, v[c][3] * inv);
        o[1] = cvt4<false>(v[c][4] * inv, v[c][5] * inv, v[c][6] * inv, v[c][7] * inv);
        *(v2u*)(qr + col) = o;
      }
    }
  }
  float* pr = part + w.part_begin + (int64_t)(r0 / WQ_G) * cols;
#pragma unroll
  for (int c = 0; c < RCH; ++c) {
    if (c >= nchunk) break;   // block-uniform
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = cm[c][j];
    __syncthreads();
    for (int t = threadIdx.x; t < 512; t += 256) {
      const int col = c * 512 + t;
      if (col < cols) pr[col] = fmaxf(fmaxf(red[0][t], red[1][t]), fmaxf(red[2][t], red[3][t]));
    }
    __syncthreads();
  }
}

// Launch 2: W^T. Units = (entry, 64-column strip, 256-row chunk), chunk
// fastest; each reduces its strip's partials (fixed order) and writes its
// 256 x 64 tile of W^T through LDS (the second and last read of W).
__global__ void __launch_bounds__(256) wq_cols_kernel(const maeclip_fp8w_entry* __restrict__ e, int n,
                                                      const float* __restrict__ part) {
  __shared__ float tile[64][65];
  __shared__ float inv_s[64];
  __shared__ float pmax[4][64];
  const int64_t gu = blockIdx.x;
  const maeclip_fp8w_entry& w = e[wentry(e, n, gu, true)];
  const int lu = (int)(gu - w.unit_begin), nch = (w.rows + QC_ROWS - 1) / QC_ROWS;
  const int npart = (w.rows + WQ_G - 1) / WQ_G;
  const int c0 = (lu / nch) * 64, r0 = (lu % nch) * QC_ROWS;
  const int rows = w.rows, cols = w.cols;
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6, col = c0 + tc;
  {
    // the strip's column maxima: wave tr reduces partials tr, tr + 4, ...
    // (4 loads in flight per lane), then the four meet in LDS (fixed order)
    float a = 0.f;
    if (col < cols) {
      const float* pc = part + w.part_begin + col;
      int k = tr;
      for (; k + 12 < npart; k += 16)
        a = fmaxf(fmaxf(a, fmaxf(pc[(int64_t)k * cols], pc[(int64_t)(k + 4) * cols])),
                  fmaxf(pc[(int64_t)(k + 8) * cols], pc[(int64_t)(k + 12) * cols]));
      for (; k < npart; k += 4) a = fmaxf(a, pc[(int64_t)k * cols]);
    }
    pmax[tr][tc] = a;
    __syncthreads();
    if (threadIdx.x < 64) {
      const float m = fmaxf(fmaxf(pmax[0][tc], pmax[1][tc]), fmaxf(pmax[2][tc], pmax[3][tc]));
      const float s = m > 0.f ? m / E4M3_MAX : 1.f;
      inv_s[tc] = 1.f / s;
      if (r0 == 0 && col < cols) w.sqt[col] = s;
    }
  }
  uint8_t* qt = (uint8_t*)w.qt;
  // 64 x 64 sub-tiles of W, 16-B loads (lane: 4 columns of rows t / 16 + 16 k),
  // the next sub-tile's loads in flight while this one is transposed
  const int lr = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;
  const int rend = min(rows, r0 + QC_ROWS);
  auto ld4 = [&](int rb, v4f (&x)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = rb + lr + 16 * k;
      x[k] = (r < rend && c0 + lc < cols) ? *(const v4f*)(w.w + (int64_t)r * w.ld + c0 + lc) : v4f{0.f, 0.f, 0.f, 0.f};
    }
  };
  v4f nx[4];
  ld4(r0, nx);
  for (int rb = r0; rb < rend; rb += 64) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[lr + 16 * k][lc + j] = nx[k][j];
    if (rb + 64 < rend) ld4(rb + 64, nx);
    __syncthreads();
    const int tc2 = threadIdx.x >> 2, seg = threadIdx.x & 3;
    const float inv = inv_s[tc2];
    if (c0 + tc2 < cols && rb + seg * 16 < rows) {
      uint8_t* dst = qt + (int64_t)(c0 + tc2) * w.ldqt + rb + seg * 16;
      v4u o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rr = seg * 16 + 4 * k;
        o[k] = cvt4<false>(tile[rr][tc2] * inv, tile[rr + 1][tc2] * inv, tile[rr + 2][tc2] * inv,
                           tile[rr + 3][tc2] * inv);
      }
      if (rb + seg * 16 + 16 <= rows) {
        *(v4u*)dst = o;
      } else {
        for (int k = 0; k < 16 && rb + seg * 16 + k < rows; ++k) dst[k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

// fp8 blocks (maeclip_quant_blocks_fp8): one wave per row, 8 consecutive
// elements per lane and 512-column chunk, so a 32-element block is the 4 lanes
// of a DPP quad: its amax is two quad-permute max steps, its e8m0 exponent
// mc_e8m0, written by the quad's first lane at mc_fp8b_off.
template <typename T, bool E5>
__global__ void __launch_bounds__(256) quant_blocks_kernel(const T* __restrict__ x, int64_t rows, int cols, int64_t ld,
                                                           uint8_t* __restrict__ q, int64_t ldq,
                                                           uint8_t* __restrict__ sc) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int KT = cols / 128;
  const T* xr = x + row * ld;
  uint8_t* qr = q + row * ldq;
  for (int c0 = 0; c0 < cols; c0 += 512) {
    const int e = c0 + lane * 8;
    float w[8];
    float amax = 0.f;
    if (e < cols) {
      Row8<T>::load(xr + e, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(w[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = 0.f;
    }
    amax = fmaxf(amax, dpp_mov<0xB1>(amax));   // quad_perm [1,0,3,2]
    amax = fmaxf(amax, dpp_mov<0x4E>(amax));   // quad_perm [2,3,0,1]
    const unsigned ex = mc_e8m0(amax, E5);
    const float inv = mc_e8m0_inv(ex);
    if (e < cols) {
      v2u o;
      o[0] = cvt4<E5>(w[0] * inv, w[1] * inv, w[2] * inv, w[3] * inv);
      o[1] = cvt4<E5>(w[4] * inv, w[5] * inv, w[6] * inv, w[7] * inv);
      *(v2u*)(qr + e) = o;
      if ((lane & 3) == 0) sc[mc_fp8b_off(row, e >> 5, KT)] = (uint8_t)ex;
    }
  }
}

}  // namespace

extern "C" int64_t maeclip_fp8b_scale_bytes(int64_t rows, int64_t K) {
  return rows > 0 && K > 0 && K % 128 == 0 ? mc_fp8b_bytes(rows, K) : 0;
}

extern "C" int32_t maeclip_quant_blocks_fp8(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ld,
                                            void* q, int64_t ldq, uint8_t* scales, int32_t fmt, void* stream) {
  MC_CHECK_ARG(x && q && scales && rows >= 0 && cols > 0, "maeclip_quant_blocks_fp8: bad arguments");
  MC_CHECK_ARG(x_dtype == MAECLIP_BF16 || x_dtype == MAECLIP_F32, "maeclip_quant_blocks_fp8: x dtype bf16 or f32");
  MC_CHECK_ARG(fmt == MAECLIP_FP8_E4M3 || fmt == MAECLIP_FP8_E5M2, "maeclip_quant_blocks_fp8: bad fp8 format");
  MC_CHECK_ARG(cols % 128 == 0 && ld % 8 == 0 && ldq % 8 == 0 && ld >= cols && ldq >= cols,
               "maeclip_quant_blocks_fp8: cols %% 128, ld and ldq %% 8");
  MC_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0, "maeclip_quant_blocks_fp8: alignment");
  MC_CHECK_ARG(cols < (1 << 30), "maeclip_quant_blocks_fp8: row too long");
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const bool e5 = fmt == MAECLIP_FP8_E5M2;
  if (x_dtype == MAECLIP_BF16) {
    if (e5) hipLaunchKernelGGL((quant_blocks_kernel<bf16_t, true>), grid, dim3(256), 0, s, (const bf16_t*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
    else hipLaunchKernelGGL((quant_blocks_kernel<bf16_t, false>), grid, dim3(256), 0, s, (const bf16_t*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
  } else {
    if (e5) hipLaunchKernelGGL((quant_blocks_kernel<float, true>), grid, dim3(256), 0, s, (const float*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
    else hipLaunchKernelGGL((quant_blocks_kernel<float, false>), grid, dim3(256), 0, s, (const float*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
  }
  MC_CHECK_LAUNCH("maeclip_quant_blocks_fp8");
  return 0;
}

// host side of the batched weight quantisation: prefix sums filled here (row
// spaces padded to WQ_G rows; one partial row of column maxima per WQ_G rows)
extern "C" int64_t maeclip_quant_weights_fp8_prepare(maeclip_fp8w_entry* host, int32_t n) {
  int64_t rows = 0, units = 0, part = 0;
  for (int i = 0; i < n; ++i) {
    maeclip_fp8w_entry& w = host[i];
    const int nch = (w.rows + QC_ROWS - 1) / QC_ROWS, ng = (w.rows + WQ_G - 1) / WQ_G;
    w.row_begin = rows;
    w.unit_begin = units;
    w.part_begin = part;
    rows += (int64_t)ng * WQ_G;
    units += (int64_t)((w.cols + 63) / 64) * nch;
    part += (int64_t)ng * w.cols;
  }
  return part * 4;   // workspace bytes (column partial maxima)
}

extern "C" int32_t maeclip_quant_weights_fp8(const maeclip_fp8w_entry* dev, const maeclip_fp8w_entry* host, int32_t n,
                                             float* workspace, int64_t ws_bytes, void* stream) {
  MC_CHECK_ARG(dev && host && n > 0, "maeclip_quant_weights_fp8: bad arguments");
  int64_t rows = 0, units = 0, part = 0;
  for (int i = 0; i < n; ++i) {
    const maeclip_fp8w_entry& w = host[i];
    MC_CHECK_ARG(w.w && ((uintptr_t)w.w & 15) == 0 && w.q && w.sq && w.qt && w.sqt && w.rows > 0 && w.cols > 0 && w.cols % 8 == 0 &&
                     w.cols <= 512 * RCH && w.ld >= w.cols && w.ld % 8 == 0 && w.ldqt >= w.rows && w.ldqt % 16 == 0,
                 "maeclip_quant_weights_fp8: bad entry %d (16-B aligned w, cols %% 8, cols <= %d)", i, 512 * RCH);
    MC_CHECK_ARG(w.row_begin == rows && w.unit_begin == units && w.part_begin == part,
                 "maeclip_quant_weights_fp8: entries not prepared (maeclip_quant_weights_fp8_prepare)");
    const int nch = (w.rows + QC_ROWS - 1) / QC_ROWS, ng = (w.rows + WQ_G - 1) / WQ_G;
    rows += (int64_t)ng * WQ_G;
    units += (int64_t)((w.cols + 63) / 64) * nch;
    part += (int64_t)ng * w.cols;
  }
  MC_CHECK_ARG(workspace && ws_bytes >= part * 4, "maeclip_quant_weights_fp8: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wq_rows_kernel, dim3((unsigned)(rows / WQ_G)), dim3(256), 0, s, dev, n, workspace);
  MC_CHECK_LAUNCH("maeclip_quant_weights_fp8(rows + column maxima)");
  hipLaunchKernelGGL(wq_cols_kernel, dim3((unsigned)units), dim3(256), 0, s, dev, n, (const float*)workspace);
  MC_CHECK_LAUNCH("maeclip_quant_weights_fp8(cols)");
  return 0;
}

extern "C" int32_t maeclip_quant_rows_fp8(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ld,
                                          void* q, int64_t ldq, float* scales, int32_t fmt, void* stream) {
  MC_CHECK_ARG(x && q && scales && rows >= 0 && cols > 0, "maeclip_quant_rows_fp8: bad arguments");
  MC_CHECK_ARG(x_dtype == MAECLIP_BF16 || x_dtype == MAECLIP_F32, "maeclip_quant_rows_fp8: x dtype bf16 or f32");
  MC_CHECK_ARG(fmt == MAECLIP_FP8_E4M3 || fmt == MAECLIP_FP8_E5M2, "maeclip_quant_rows_fp8: bad fp8 format");
  MC_CHECK_ARG(cols % 8 == 0 && ld % 8 == 0 && ldq % 8 == 0 && ld >= cols && ldq >= cols,
               "maeclip_quant_rows_fp8: cols, ld, ldq must be multiples of 8");
  MC_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0, "maeclip_quant_rows_fp8: alignment");
  MC_CHECK_ARG(cols < (1 << 30), "maeclip_quant_rows_fp8: row too long");
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const bool e5 = fmt == MAECLIP_FP8_E5M2;
  if (x_dtype == MAECLIP_BF16) {
    if (e5) hipLaunchKernelGGL((quant_rows_kernel<bf16_t, true>), grid, dim3(256), 0, s, (const bf16_t*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
    else hipLaunchKernelGGL((quant_rows_kernel<bf16_t, false>), grid, dim3(256), 0, s, (const bf16_t*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
  } else {
    if (e5) hipLaunchKernelGGL((quant_rows_kernel<float, true>), grid, dim3(256), 0, s, (const float*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
    else hipLaunchKernelGGL((quant_rows_kernel<float, false>), grid, dim3(256), 0, s, (const float*)x, rows, (int)cols, ld, (uint8_t*)q, ldq, scales);
  }
  MC_CHECK_LAUNCH("maeclip_quant_rows_fp8");
  return 0;
}

extern "C" int64_t maeclip_quant_cols_fp8_workspace(int64_t rows, int64_t cols) {
  return rows > 0 && cols > 0 ? (rows + QC_ROWS - 1) / QC_ROWS * cols * 4 : 0;
}

extern "C" int32_t maeclip_quant_cols_fp8(const float* w, int64_t rows, int64_t cols, int64_t ld, void* qt,
                                          int64_t ldq, float* scales, float* workspace, int64_t ws_bytes,
                                          void* stream) {
  MC_CHECK_ARG(w && qt && scales && rows > 0 && cols > 0 && ld >= cols && ldq >= rows,
               "maeclip_quant_cols_fp8: bad arguments");
  MC_CHECK_ARG(ldq % 16 == 0 && ((uintptr_t)qt & 15) == 0, "maeclip_quant_cols_fp8: ldq %% 16, 16-B aligned output");
  MC_CHECK_ARG(rows < (1 << 30) && cols < (1 << 30), "maeclip_quant_cols_fp8: too large");
  MC_CHECK_ARG(workspace && ws_bytes >= maeclip_quant_cols_fp8_workspace(rows, cols),
               "maeclip_quant_cols_fp8: workspace too small");
  const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + QC_ROWS - 1) / QC_ROWS));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(quant_cols_amax_kernel, grid, dim3(256), 0, s, w, (int)rows, (int)cols, ld, workspace);
  MC_CHECK_LAUNCH("maeclip_quant_cols_fp8(amax)");
  hipLaunchKernelGGL(quant_cols_kernel, grid, dim3(256), 0, s, w, (int)rows, (int)cols, ld, (const float*)workspace,
                     (uint8_t*)qt, ldq, scales);
  MC_CHECK_LAUNCH("maeclip_quant_cols_fp8");
  return 0;
}
