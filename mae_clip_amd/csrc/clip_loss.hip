// Soft-target symmetric CLIP loss, forward + closed-form backward, fp32 always.
//
// Reference: CLIP.py:34-43 and cross_entropy CLIP.py:46-52
//   L = T I^T / tau ; S = (I I^T + T T^T) / 2 * tau ; Y = softmax_row(S)
//   loss = mean_k[(CE_row(L,Y)_k + CE_col(L,Y)_k)/2]   (gradient flows through Y)
// Backward (verified vs autograd to 5.6e-17 in fp64):
//   G  = -(logsm_row(L) + logsm_col(L)) / 2N ;  loss = sum(Y .* G)
//   dS = Y .* (G - rowsum(G .* Y)) ; Dm = (dS + dS^T) tau/2
//   dL = (P_r - 2Y + P_c .* colsum(Y)) / 2N
//   dI = Dm I + dL^T T / tau ;  dT = Dm T + dL I / tau
// The N x N products run on the exact-f32 MFMA GEMM (v_mfma_f32_16x16x4_f32);
// the softmax/row/column statistics are wave-reduced, one workgroup per row.
// Gradients are produced during the forward (the loss is a leaf of the graph),
// the autograd backward only scales them by grad_output.
#include "common.h"
#include "../../include/maeclip.h"

namespace {
constexpr int NTH = 256;

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int k = 1; k < NTH / 64; ++k) r = is_max ? fmaxf(r, red[k]) : r + red[k];
  return r;
}

// Y[i,:] = softmax(S[i,:]) ; lse_r[i] = logsumexp(L[i,:])
__global__ void __launch_bounds__(NTH) rowstats_kernel(const float* __restrict__ S, const float* __restrict__ Lm,
                                                       float* __restrict__ Y, float* __restrict__ lse_r, int N) {
  __shared__ float red[NTH / 64];
  const int i = blockIdx.x;
  const float* s = S + (int64_t)i * N;
  const float* l = Lm + (int64_t)i * N;
  float ms = -INFINITY, ml = -INFINITY;
  for (int j = threadIdx.x; j < N; j += NTH) { ms = fmaxf(ms, s[j]); ml = fmaxf(ml, l[j]); }
  ms = block_reduce(ms, red, true);
  ml = block_reduce(ml, red, true);
  float zs = 0.f, zl = 0.f;
  for (int j = threadIdx.x; j < N; j += NTH) { zs += expf(s[j] - ms); zl += expf(l[j] - ml); }
  zs = block_reduce(zs, red, false);
  zl = block_reduce(zl, red, false);
  const float inv = 1.f / zs;
  for (int j = threadIdx.x; j < N; j += NTH) Y[(int64_t)i * N + j] = expf(s[j] - ms) * inv;
  if (threadIdx.x == 0) lse_r[i] = ml + logf(zl);
}

// lse_c[j] = logsumexp_i L[i,j] ; cy[j] = sum_i Y[i,j]
__global__ void __launch_bounds__(NTH) colstats_kernel(const float* __restrict__ Lm, const float* __restrict__ Y,
                                                       float* __restrict__ lse_c, float* __restrict__ cy, int N) {
  const int j = blockIdx.x * NTH + threadIdx.x;
  if (j >= N) return;
  float m = -INFINITY;
  for (int i = 0; i < N; ++i) m = fmaxf(m, Lm[(int64_t)i * N + j]);
  float z = 0.f, c = 0.f;
  for (int i = 0; i < N; ++i) {
    z += expf(Lm[(int64_t)i * N + j] - m);
    c += Y[(int64_t)i * N + j];
  }
  lse_c[j] = m + logf(z);
  cy[j] = c;
}

// row i: row_loss[i] = sum_j Y G ; dS (in place of S) and dL
__global__ void __launch_bounds__(NTH) grad_kernel(const float* __restrict__ Lm, const float* __restrict__ Y,
                                                   const float* __restrict__ lse_r, const float* __restrict__ lse_c,
                                                   const float* __restrict__ cy, float* __restrict__ dS,
                                                   float* __restrict__ dL, float* __restrict__ row_loss, int N,
                                                   int want_grad) {
  __shared__ float red[NTH / 64];
  const int i = blockIdx.x;
  const float inv2n = 0.5f / (float)N;
  const float lr = lse_r[i];
  const float* l = Lm + (int64_t)i * N;
  const float* y = Y + (int64_t)i * N;
  float acc = 0.f;
  for (int j = threadIdx.x; j < N; j += NTH) {
    const float G = -((l[j] - lr) + (l[j] - lse_c[j])) * inv2n;
    acc += y[j] * G;
  }
  acc = block_reduce(acc, red, false);
  if (threadIdx.x == 0) row_loss[i] = acc;
  if (!want_grad) return;
  for (int j = threadIdx.x; j < N; j += NTH) {
    const float G = -((l[j] - lr) + (l[j] - lse_c[j])) * inv2n;
    dS[(int64_t)i * N + j] = y[j] * (G - acc);
    dL[(int64_t)i * N + j] = (expf(l[j] - lr) - 2.f * y[j] + expf(l[j] - lse_c[j]) * cy[j]) * inv2n;
  }
}

// Dm = (dS + dS^T) * tau/2, 32x32 tiles through LDS
__global__ void __launch_bounds__(NTH) symmetrize_kernel(const float* __restrict__ dS, float* __restrict__ Dm, int N,
                                                         float half_tau) {
  __shared__ float tile[32][33];
  const int bi = blockIdx.y * 32, bj = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int i = bj + r, j = bi + tx;  // transposed source block
    tile[r][tx] = (i < N && j < N) ? dS[(int64_t)i * N + j] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int i = bi + r, j = bj + tx;
    if (i < N && j < N) Dm[(int64_t)i * N + j] = (dS[(int64_t)i * N + j] + tile[tx][r]) * half_tau;
  }
}

int gemm_f32(const float* A, int64_t lda, int alay, const float* B, int64_t ldb, int blay, float* C, int64_t ldc,
             int64_t M, int64_t N, int64_t K, float alpha, float beta, hipStream_t s) {
  maeclip_gemm_args g = {};
  g.A = A; g.B = B; g.C = C;
  g.M = M; g.N = N; g.K = K;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.batch = 1;
  g.dtype = MAECLIP_F32; g.out_dtype = MAECLIP_F32;
  g.a_layout = alay; g.b_layout = blay;
  g.epilogue = 0;
  g.alpha = alpha; g.beta = beta;
  return maeclip_gemm(&g, s);
}

}  // namespace

extern "C" size_t maeclip_clip_loss_workspace(int64_t N) { return (size_t)(4 * N * N + 5 * N + 64) * sizeof(float); }

extern "C" int32_t maeclip_clip_loss(const maeclip_clip_args* a, void* stream) {
  MC_CHECK_ARG(a && a->I && a->T && a->loss && a->workspace, "maeclip_clip_loss: null pointer");
  MC_CHECK_ARG(a->N > 0 && a->P > 0 && a->P % 4 == 0 && a->N % 4 == 0, "maeclip_clip_loss: N, P must be multiples of 4");
  MC_CHECK_ARG(a->ws_bytes >= maeclip_clip_loss_workspace(a->N), "maeclip_clip_loss: workspace too small");
  MC_CHECK_ARG(a->temperature > 0.f, "maeclip_clip_loss: temperature must be > 0");
  const int64_t N = a->N, P = a->P;
  const bool grad = a->dI && a->dT;
  hipStream_t s = (hipStream_t)stream;
  float* ws = (float*)a->workspace;
  float* S = ws;             // S, later dS
  float* Lm = S + N * N;     // logits
  float* Y = Lm + N * N;     // targets, later Dm
  float* dL = Y + N * N;
  float* lse_r = dL + N * N;
  float* lse_c = lse_r + N;
  float* cy = lse_c + N;
  float* rl = cy + N;
  const float tau = a->temperature;
  const int64_t ldi = a->ld_I ? a->ld_I : P, ldt = a->ld_T ? a->ld_T : P;
  int e;
  // L = T I^T / tau  (CLIP.py:34)
  if ((e = gemm_f32(a->T, ldt, 0, a->I, ldi, 0, Lm, N, N, N, P, 1.f / tau, 0.f, s))) return e;
  // S = (I I^T + T T^T)/2 * tau  (CLIP.py:35-38)
  if ((e = gemm_f32(a->I, ldi, 0, a->I, ldi, 0, S, N, N, N, P, 0.5f * tau, 0.f, s))) return e;
  if ((e = gemm_f32(a->T, ldt, 0, a->T, ldt, 0, S, N, N, N, P, 0.5f * tau, 1.f, s))) return e;
  hipLaunchKernelGGL(rowstats_kernel, dim3((unsigned)N), dim3(NTH), 0, s, S, Lm, Y, lse_r, (int)N);
  hipLaunchKernelGGL(colstats_kernel, dim3((unsigned)((N + NTH - 1) / NTH)), dim3(NTH), 0, s, Lm, Y, lse_c, cy, (int)N);
  hipLaunchKernelGGL(grad_kernel, dim3((unsigned)N), dim3(NTH), 0, s, Lm, Y, lse_r, lse_c, cy, S, dL, rl, (int)N,
                     grad ? 1 : 0);
  MC_CHECK_LAUNCH("maeclip_clip_loss(stats)");
  if ((e = maeclip_colsum_reduce(rl, N, 1, a->loss, 0, 1.f, nullptr, s))) return e;
  if (a->row_loss_out) (void)hipMemcpyAsync(a->row_loss_out, rl, N * sizeof(float), hipMemcpyDeviceToDevice, s);
  if (!grad) return 0;
  float* Dm = Y;
  dim3 tg((unsigned)((N + 31) / 32), (unsigned)((N + 31) / 32));
  hipLaunchKernelGGL(symmetrize_kernel, tg, dim3(NTH), 0, s, S, Dm, (int)N, 0.5f * tau);
  MC_CHECK_LAUNCH("maeclip_clip_loss(sym)");
  const int64_t lddi = a->ld_dI ? a->ld_dI : P, lddt = a->ld_dT ? a->ld_dT : P;
  // dI = Dm I + dL^T T / tau
  if ((e = gemm_f32(Dm, N, 0, a->I, ldi, 1, a->dI, lddi, N, P, N, 1.f, 0.f, s))) return e;
  if ((e = gemm_f32(dL, N, 1, a->T, ldt, 1, a->dI, lddi, N, P, N, 1.f / tau, 1.f, s))) return e;
  // dT = Dm T + dL I / tau
  if ((e = gemm_f32(Dm, N, 0, a->T, ldt, 1, a->dT, lddt, N, P, N, 1.f, 0.f, s))) return e;
  if ((e = gemm_f32(dL, N, 0, a->I, ldi, 1, a->dT, lddt, N, P, N, 1.f / tau, 1.f, s))) return e;
  return 0;
}
