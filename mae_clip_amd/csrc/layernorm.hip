// LayerNorm forward/backward, one wave per row (gfx950).
//
// Replaces nn.LayerNorm at every site of the hot path: timm Block norm1/norm2
// and fc_norm (eps 1e-6), ProjectionHead.layer_norm (modules.py:67, eps 1e-5),
// HF ViTMAE decoder layernorms (eps 1e-6 after config), DistilBERT
// Embeddings.LayerNorm / sa_layer_norm / output_layer_norm (eps 1e-12,
// modeling_distilbert.py:88,236,239).
//
// Fusions (each saves a full HBM pass over an [M,D] activation):
//   fwd: x' = dropout(x) + res       (post-LN residual of DistilBERT, ProjectionHead)
//        y  = LN(x') [+ dropout]     (Embeddings dropout after LN)
//        y2 = bf16 copy of y         (GEMM operand) ; x' saved for backward
//   bwd: dx = LN'(dy) + dres         (pre-LN residual stream gradient)
//        dx_bf = bf16 copy of dx     (next GEMM operand)
//        per-block partials of dgamma, dbeta and colsum(dx) (= the bias gradient
//        of the Linear that produced the residual branch), reduced by
//        maeclip_colsum_reduce -> deterministic.
// Statistics are fp32 two-pass (mean, then sum of squared deviations), as torch.
#include "common.h"
#include "../../include/maeclip.h"

namespace {

constexpr int NTH = 256;
constexpr int MAXC = 8;  // chunks of 4 elements per lane -> D <= 2048

// non-temporal streams (LN_NT bits): 1 the forward's saved residual-stream
// copy (xsum, read again only by the backward), 2 the backward's read of it,
// 4 the backward's f32 dx
#ifndef LN_NT
#define LN_NT 7
#endif
template <typename T> __device__ __forceinline__ v4f ld4_nt(const T* p);
template <> __device__ __forceinline__ v4f ld4_nt<float>(const float* p) { return __builtin_nontemporal_load((const v4f*)p); }
template <> __device__ __forceinline__ v4f ld4_nt<bf16_t>(const bf16_t* p) {
  const v2u u = __builtin_nontemporal_load((const v2u*)p);
  return v4f{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
             __uint_as_float(u[1] & 0xffff0000u)};
}

template <int NC, typename T, bool NT = false>
__device__ __forceinline__ void load_row(float (&v)[NC][4], const T* p, int D, int lane) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e = c * 256 + lane * 4;
    if (e < D) {
      v4f t = NT ? ld4_nt<T>(p + e) : ld4<T>(p + e);
      v[c][0] = t[0]; v[c][1] = t[1]; v[c][2] = t[2]; v[c][3] = t[3];
    } else {
      v[c][0] = v[c][1] = v[c][2] = v[c][3] = 0.f;
    }
  }
}

// the value a consumer reads back from a YT store of f
template <typename YT> __device__ __forceinline__ float as_stored(float f) {
  return sizeof(YT) == 2 ? bf2f(f2bf(f)) : f;
}

__device__ __forceinline__ float keepf(uint64_t seed, int64_t row, int col, uint32_t thr, float sc) {
  return mc_hash4(seed, (uint64_t)row, (uint64_t)col, 0x4c4eull) >= thr ? sc : 0.f;
}

template <int NC, typename XT, typename YT>
__global__ void __launch_bounds__(NTH) ln_fwd_kernel(const maeclip_ln_fwd_args a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NTH / 64) + (threadIdx.x >> 6);
  if (row >= a.M) return;
  const int D = (int)a.D;
  float v[NC][4];
  load_row<NC, XT>(v, (const XT*)a.x + row * a.ldx, D, lane);
  if (a.in_dropout_p > 0.f) {
    const uint32_t thr = (uint32_t)((double)a.in_dropout_p * 4294967296.0);
    const float sc = 1.f / (1.f - a.in_dropout_p);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[c][j] *= keepf(mc_step_seed(a.seed_in, a.step_ptr), row, c * 256 + lane * 4 + j, thr, sc);
  }
  if (a.res) {
    float r[NC][4];
    load_row<NC, float>(r, a.res + row * a.ldres, D, lane);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[c][j] += r[c][j];
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[c][j];
  const float mean = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c * 256 + lane * 4 < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[c][j] - mean; ss += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / D + a.eps);
  if (lane == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
  const bool odrop = a.out_dropout_p > 0.f;
  const uint32_t othr = (uint32_t)((double)a.out_dropout_p * 4294967296.0);
  const float osc = odrop ? 1.f / (1.f - a.out_dropout_p) : 1.f;
  float amax = 0.f;   // of the stored y (fp8 copy only)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e = c * 256 + lane * 4;
    if (e >= D) continue;
    if (a.xsum_out) {
      const v4f t = {v[c][0], v[c][1], v[c][2], v[c][3]};
      if (LN_NT & 1) __builtin_nontemporal_store(t, (v4f*)(a.xsum_out + row * a.ldxs + e));
      else *(v4f*)(a.xsum_out + row * a.ldxs + e) = t;
    }
    const v4f gm = *(const v4f*)(a.gamma + e);
    const v4f bt = *(const v4f*)(a.beta + e);
    v4f y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      y[j] = (v[c][j] - mean) * rstd * gm[j] + bt[j];
      if (odrop) y[j] *= keepf(mc_step_seed(a.seed_out, a.step_ptr), row, e + j, othr, osc);
      v[c][j] = as_stored<YT>(y[j]);
      amax = fmaxf(amax, fabsf(v[c][j]));
    }
    st4<YT>((YT*)a.y + row * a.ldy + e, y);
    if (a.y2) st4<bf16_t>((bf16_t*)a.y2 + row * a.ldy2 + e, y);
  }
  if (a.q8) quant_row_fp8<NC>(v, amax, a.q8_fmt == MAECLIP_FP8_E5M2, (uint8_t*)a.q8 + row * a.ldq8, a.q8_scale + row, D, lane);
}

template <int NC, typename GT, typename XT>
__global__ void __launch_bounds__(NTH) ln_bwd_kernel(const maeclip_ln_bwd_args a) {
  __shared__ float red[NTH / 64][NC * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D = (int)a.D;
  float pg[NC][4], pb[NC][4], pc[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) pg[c][j] = pb[c][j] = pc[c][j] = 0.f;

  float gm[NC][4];
  load_row<NC, float>(gm, a.gamma, D, lane);

  for (int64_t row = (int64_t)blockIdx.x * (NTH / 64) + wave; row < a.M; row += (int64_t)gridDim.x * (NTH / 64)) {
    // every load of the row issued together (one HBM round trip per row)
    float dy[NC][4], x[NC][4], dr[NC][4];
    load_row<NC, GT>(dy, (const GT*)a.dy + row * a.lddy, D, lane);
    load_row<NC, XT, (LN_NT & 2) != 0>(x, (const XT*)a.x + row * a.ldx, D, lane);
    if (a.dres) load_row<NC, float>(dr, a.dres + row * a.lddx, D, lane);
    const bool pool = a.dres_pool != nullptr;
    if (pool) {   // global_pool="avg" backward: 1/(n-1) of the pooled gradient, 0 for the cls row
      load_row<NC, float>(dr, a.dres_pool + (row / a.pool_n) * D, D, lane);
      const bool cls = row % a.pool_n == 0;
      const float den = (float)(a.pool_n - 1);
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) dr[c][j] = cls ? 0.f : dr[c][j] / den;
    }
    const float mean = a.mean[row], rstd = a.rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (x[c][j] - mean) * rstd;
        x[c][j] = xh;
        const float gdy = dy[c][j] * gm[c][j];
        s1 += gdy;
        s2 += gdy * xh;
        pg[c][j] += dy[c][j] * xh;
        pb[c][j] += dy[c][j];
      }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
    float amax = 0.f;   // of the bf16 dx copy (fp8 copy only)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int e = c * 256 + lane * 4;
      if (e >= D) continue;
      v4f o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d = rstd * (dy[c][j] * gm[c][j] - s1 - x[c][j] * s2);
        if (a.dres || pool) d += dr[c][j];
        o[j] = d;
        pc[c][j] += d;
        dy[c][j] = as_stored<bf16_t>(d);
        amax = fmaxf(amax, fabsf(dy[c][j]));
      }
      if (LN_NT & 4) __builtin_nontemporal_store(o, (v4f*)(a.dx + row * a.lddx + e));
      else *(v4f*)(a.dx + row * a.lddx + e) = o;
      if (a.dx_bf) st4<bf16_t>((bf16_t*)a.dx_bf + row * a.lddx_bf + e, o);
    }
    if (a.q8) quant_row_fp8<NC>(dy, amax, a.q8_fmt == MAECLIP_FP8_E5M2, (uint8_t*)a.q8 + row * a.ldq8, a.q8_scale + row, D, lane);
  }
  // cross-wave reduction of the three per-lane partial vectors
  float* outs[3] = {a.dgamma_partial, a.dbeta_partial, a.dx_colsum_partial};
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    if (!outs[w]) continue;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = c * 256 + lane * 4 + j;
        if (e < D) red[wave][e] = (w == 0 ? pg[c][j] : (w == 1 ? pb[c][j] : pc[c][j]));
      }
    __syncthreads();
    for (int e = threadIdx.x; e < D; e += NTH) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NTH / 64; ++k) s += red[k][e];
      outs[w][(int64_t)blockIdx.x * D + e] = s;
    }
    __syncthreads();
  }
}

// workgroups of the backward (each writes one partial row per output): 1024
// at D <= 512 (the decoder: 72 -> 65 us alone at 50432 rows, 2 -> 4 waves per
// SIMD), 512 above (D = 768 at 180 VGPRs holds 2 waves per SIMD anyway, and
// 1024 measured slower: 31 -> 35 us; profiles/r05/ln_bwd_grid_ab_r5am.txt).
// A next-row prefetch in the row loop measured slower alone (72 -> 83 us) and
// neutral on the step (profiles/r05/ln_bwd_prefetch_ab_r5al.txt).
#ifndef LN_BWD_GRID_CAP
#define LN_BWD_GRID_CAP 512
#endif
#ifndef LN_BWD_GRID_CAP_NARROW
#define LN_BWD_GRID_CAP_NARROW 1024
#endif
int ln_bwd_grid(int64_t M, int64_t D) {
  const int64_t g = (M + 3) / 4, cap = D <= 512 ? LN_BWD_GRID_CAP_NARROW : LN_BWD_GRID_CAP;
  return (int)(g < cap ? g : cap);
}

}  // namespace

extern "C" int32_t maeclip_ln_fwd(const maeclip_ln_fwd_args* a, void* stream) {
  MC_CHECK_ARG(a && a->x && a->y && a->gamma && a->beta, "maeclip_ln_fwd: null pointer");
  MC_CHECK_ARG(a->D > 0 && a->D <= MAXC * 256 && a->D % 4 == 0, "maeclip_ln_fwd: D=%lld unsupported", (long long)a->D);
  MC_CHECK_ARG(!a->q8 || (a->q8_scale && a->ldq8 >= a->D && a->ldq8 % 4 == 0 && ((uintptr_t)a->q8 & 3) == 0 &&
                          (a->q8_fmt == MAECLIP_FP8_E4M3 || a->q8_fmt == MAECLIP_FP8_E5M2)),
               "maeclip_ln_fwd: bad fp8 output");
  if (a->M == 0) return 0;
  dim3 grid((unsigned)((a->M + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int nc = (int)((a->D + 255) / 256);
  const int code = (a->x_dtype == MAECLIP_BF16 ? 2 : 0) + (a->y_dtype == MAECLIP_BF16 ? 1 : 0);
#define LNF(NCV)                                                                                         \
  case NCV:                                                                                              \
    if (code == 3) hipLaunchKernelGGL((ln_fwd_kernel<NCV, bf16_t, bf16_t>), grid, dim3(NTH), 0, s, *a);  \
    else if (code == 2) hipLaunchKernelGGL((ln_fwd_kernel<NCV, bf16_t, float>), grid, dim3(NTH), 0, s, *a); \
    else if (code == 1) hipLaunchKernelGGL((ln_fwd_kernel<NCV, float, bf16_t>), grid, dim3(NTH), 0, s, *a); \
    else hipLaunchKernelGGL((ln_fwd_kernel<NCV, float, float>), grid, dim3(NTH), 0, s, *a);              \
    break;
  switch (nc) { LNF(1) LNF(2) LNF(3) LNF(4) LNF(5) LNF(6) LNF(7) LNF(8) }
#undef LNF
  MC_CHECK_LAUNCH("maeclip_ln_fwd");
  return 0;
}

extern "C" int32_t maeclip_ln_bwd_partial_rows(int64_t M, int64_t D) { return ln_bwd_grid(M, D); }

extern "C" int32_t maeclip_ln_bwd(const maeclip_ln_bwd_args* a, void* stream) {
  MC_CHECK_ARG(a && a->dy && a->x && a->mean && a->rstd && a->gamma && a->dx, "maeclip_ln_bwd: null pointer");
  MC_CHECK_ARG(a->D > 0 && a->D <= MAXC * 256 && a->D % 4 == 0, "maeclip_ln_bwd: D unsupported");
  MC_CHECK_ARG(!a->q8 || (a->dx_bf && a->q8_scale && a->ldq8 >= a->D && a->ldq8 % 4 == 0 && ((uintptr_t)a->q8 & 3) == 0 &&
                          (a->q8_fmt == MAECLIP_FP8_E4M3 || a->q8_fmt == MAECLIP_FP8_E5M2)),
               "maeclip_ln_bwd: bad fp8 output (needs dx_bf)");
  MC_CHECK_ARG(!a->dres_pool || (!a->dres && a->pool_n > 1 && a->M % a->pool_n == 0),
               "maeclip_ln_bwd: dres_pool needs pool_n > 1 dividing M (and no dres)");
  if (a->M == 0) return 0;
  dim3 grid((unsigned)ln_bwd_grid(a->M, a->D));
  hipStream_t s = (hipStream_t)stream;
  const int nc = (int)((a->D + 255) / 256);
  const int code = (a->dy_dtype == MAECLIP_BF16 ? 2 : 0) + (a->x_dtype == MAECLIP_BF16 ? 1 : 0);
#define LNB(NCV)                                                                                         \
  case NCV:                                                                                              \
    if (code == 3) hipLaunchKernelGGL((ln_bwd_kernel<NCV, bf16_t, bf16_t>), grid, dim3(NTH), 0, s, *a);  \
    else if (code == 2) hipLaunchKernelGGL((ln_bwd_kernel<NCV, bf16_t, float>), grid, dim3(NTH), 0, s, *a); \
    else if (code == 1) hipLaunchKernelGGL((ln_bwd_kernel<NCV, float, bf16_t>), grid, dim3(NTH), 0, s, *a); \
    else hipLaunchKernelGGL((ln_bwd_kernel<NCV, float, float>), grid, dim3(NTH), 0, s, *a);              \
    break;
  switch (nc) { LNB(1) LNB(2) LNB(3) LNB(4) LNB(5) LNB(6) LNB(7) LNB(8) }
#undef LNB
  MC_CHECK_LAUNCH("maeclip_ln_bwd");
  return 0;
}
