// Retrieval: the embedding search of inference.py:40-45,
//   image_embeddings_n = F.normalize(image_embeddings, p=2, dim=-1)
//   text_embeddings_n  = F.normalize(text_embeddings, p=2, dim=-1)
//   dot_similarity     = text_embeddings_n @ image_embeddings_n.T   (maeclip_gemm, fp32)
//   _, indices         = torch.topk(dot_similarity.squeeze(0), n * 5)
// maeclip_l2_normalize: one wave per row, x / max(||x||_2, eps) (F.normalize's
// clamp_min(eps) semantics), fp32, fixed summation order.
// maeclip_topk_rows: one workgroup per row; k selection rounds, each a block
// arg-max over the row restricted to entries after the previous pick in the
// order (value descending, index ascending): sorted output, ties broken by the
// lower index, deterministic. The row is re-read from L2 every round
// (k <= 1024; the retrieval case is k = 45 over <= 1e5 candidates).
#include "common.h"
#include "../../include/maeclip.h"

namespace {

__global__ void __launch_bounds__(256) l2_normalize_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           int64_t M, int64_t P, int64_t ldx, int64_t ldy,
                                                           float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + row * ldx;
  float ss = 0.f;
  for (int64_t c = lane; c < P; c += 64) ss = fmaf(xr[c], xr[c], ss);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float nrm = fmaxf(sqrtf(ss), eps);
  float* yr = y + row * ldy;
  for (int64_t c = lane; c < P; c += 64) yr[c] = xr[c] / nrm;
}

// is (v, i) ranked before (bv, bi)?  value descending, index ascending
__device__ __forceinline__ bool before(float v, int64_t i, float bv, int64_t bi) {
  return v > bv || (v == bv && i < bi);
}

__global__ void __launch_bounds__(256) topk_rows_kernel(const float* __restrict__ s, int64_t N, int64_t lds, int k,
                                                        float* __restrict__ vals, int64_t* __restrict__ idx) {
  __shared__ float sv[4];
  __shared__ int64_t si[4];
  const int64_t row = blockIdx.x;
  const float* r = s + row * lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pv = INFINITY;
  int64_t pi = -1;   // previous pick; everything "after" it is eligible
  for (int t = 0; t < k; ++t) {
    float bv = -INFINITY;
    int64_t bi = INT64_MAX;
    for (int64_t i = threadIdx.x; i < N; i += 256) {
      const float v = r[i];
      const bool after = v < pv || (v == pv && i > pi);
      if (after && before(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int64_t oi = __shfl_xor(bi, o, 64);
      if (before(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      sv[wave] = bv;
      si[wave] = bi;
    }
    __syncthreads();
    bv = sv[0];
    bi = si[0];
    for (int w = 1; w < 4; ++w)
      if (before(sv[w], si[w], bv, bi)) {
        bv = sv[w];
        bi = si[w];
      }
    __syncthreads();
    if (threadIdx.x == 0) {
      vals[row * k + t] = bv;
      idx[row * k + t] = bi < N ? bi : -1;
    }
    pv = bv;
    pi = bi;
  }
}
}  // namespace

extern "C" int32_t maeclip_l2_normalize(const float* x, float* y, int64_t M, int64_t P, int64_t ldx, int64_t ldy,
                                        float eps, void* stream) {
  MC_CHECK_ARG(x && y && M >= 0 && P > 0 && ldx >= P && ldy >= P, "maeclip_l2_normalize: bad arguments");
  if (M == 0) return 0;
  hipLaunchKernelGGL(l2_normalize_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, y, M,
                     P, ldx, ldy, eps);
  MC_CHECK_LAUNCH("maeclip_l2_normalize");
  return 0;
}

extern "C" int32_t maeclip_topk_rows(const float* s, int64_t Q, int64_t N, int64_t lds, int32_t k, float* vals,
                                     int64_t* idx, void* stream) {
  MC_CHECK_ARG(s && vals && idx && Q >= 0 && N > 0 && lds >= N, "maeclip_topk_rows: bad arguments");
  MC_CHECK_ARG(k >= 1 && k <= N && k <= 1024, "maeclip_topk_rows: need 1 <= k <= min(N, 1024), got k=%d", k);
  if (Q == 0) return 0;
  hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)Q), dim3(256), 0, (hipStream_t)stream, s, N, lds, k, vals, idx);
  MC_CHECK_LAUNCH("maeclip_topk_rows");
  return 0;
}
