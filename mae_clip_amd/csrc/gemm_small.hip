// Small fp32 GEMM: 32x32 output tiles, 256 threads, 2x2 outputs per thread.
//
// The fp32 ProjectionHead (modules.py:69-76: projection 768->256, fc 256->256,
// and their dgrad / wgrad) and the CLIP-side GEMMs are [256 x 256..768] shapes:
// the 128x128-tile MFMA kernel of gemm.hip gets 4-12 workgroups there and runs
// latency-bound on a handful of CUs (25-70 us per launch). A 32x32 tile gives
// 64-192 workgroups; each K-chunk of 32 is staged k-major through LDS (padded
// rows, no bank conflicts on the broadcast reads) and every thread does 4 FMA
// per k. Epilogues and their semantics are those of gemm.hip (bias, GELU with
// pre-activation aux_out, residual, dGELU, GELU', mul-aux, alpha/beta).
#include "common.h"
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

constexpr int TS = 32;   // tile edge (m, n and k chunk)

// stage a 32 (rows) x 32 (k) chunk of an operand into s[k][row]
template <int LAY>
__device__ __forceinline__ void stage(float (*s)[TS + 1], const float* __restrict__ p, int64_t ld, int r0, int R,
                                      int k0, int K, int tid) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int id = it * 256 + tid;
    int r, k;
    if (LAY == LAY_KC) {   // p[r * ld + k]: consecutive threads walk k
      r = id >> 5;
      k = id & 31;
    } else {               // p[k * ld + r]: consecutive threads walk r
      k = id >> 5;
      r = id & 31;
    }
    const bool ok = (r0 + r < R) && (k0 + k < K);
    const int64_t off = LAY == LAY_KC ? (int64_t)(r0 + r) * ld + (k0 + k) : (int64_t)(k0 + k) * ld + (r0 + r);
    s[k][r] = ok ? p[off] : 0.f;
  }
}

// Apply alpha + epilogue EPI to the accumulated value v of output (m, n).
template <int EPI>
__device__ __forceinline__ void epi_store(const maeclip_gemm_args& args, int64_t z, int m, int n, float v) {
  const int64_t zo = z * args.strideC;
  v *= args.alpha;
  if (args.bias) v += args.bias[n];
  if (EPI == EPI_GELU) {
    if (args.aux_out) ((float*)args.aux_out)[zo + (int64_t)m * args.ldaux + n] = v;
    v = gelu_f(v);
  } else if (EPI == EPI_RESID) {
    v += args.resid[zo + (int64_t)m * args.ldr + n];
  } else if (EPI == EPI_DGELU) {
    v *= gelu_grad_f(((const float*)args.aux)[zo + (int64_t)m * args.ldaux + n]);
    if (args.resid) v += args.resid[zo + (int64_t)m * args.ldr + n];
  } else if (EPI == EPI_GELU_D) {
    float y, dy;
    gelu_pair(v, y, dy);
    v = y;
    if (args.aux_out) ((float*)args.aux_out)[zo + (int64_t)m * args.ldaux + n] = dy;
  } else if (EPI == EPI_MUL_AUX) {
    v *= ((const float*)args.aux)[zo + (int64_t)m * args.ldaux + n];
    if (args.resid) v += args.resid[zo + (int64_t)m * args.ldr + n];
  }
  float* cp = (float*)args.C + zo + (int64_t)m * args.ldc + n;
  if (args.beta != 0.f) v += args.beta * *cp;
  *cp = v;
}

// blockIdx.y = K slice (gridDim.y slices of whole 32-chunks). One slice: the
// epilogue is applied here; several: raw partials go to slab y of the
// workspace and small_reduce_kernel sums them in slice order.
template <int LA, int LB, int EPI>
__global__ void __launch_bounds__(256) gemm_small_kernel(const maeclip_gemm_args args) {
  __shared__ float sa[TS][TS + 1];
  __shared__ float sb[TS][TS + 1];
  const int tid = threadIdx.x;
  const int M = (int)args.M, N = (int)args.N, K = (int)args.K;
  const int gn = (N + TS - 1) / TS;
  const int m0 = (blockIdx.x / gn) * TS, n0 = (blockIdx.x % gn) * TS;
  const int S = gridDim.y;
  const int nch = (K + TS - 1) / TS;
  const int cps = (nch + S - 1) / S;
  const int kbeg = blockIdx.y * cps * TS, kend = min(K, kbeg + cps * TS);
  const int64_t z = blockIdx.z;
  const float* __restrict__ A = (const float*)args.A + z * args.strideA;
  const float* __restrict__ B = (const float*)args.B + z * args.strideB;
  const int tm = (tid >> 4) * 2, tn = (tid & 15) * 2;
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  for (int k0 = kbeg; k0 < kend; k0 += TS) {
    stage<LA>(sa, A, args.lda, m0, M, k0, kend, tid);
    stage<LB>(sb, B, args.ldb, n0, N, k0, kend, tid);
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < TS; ++k) {
      const float a0 = sa[k][tm], a1 = sa[k][tm + 1];
      const float b0 = sb[k][tn], b1 = sb[k][tn + 1];
      acc[0][0] = fmaf(a0, b0, acc[0][0]);
      acc[0][1] = fmaf(a0, b1, acc[0][1]);
      acc[1][0] = fmaf(a1, b0, acc[1][0]);
      acc[1][1] = fmaf(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + tm + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + tn + j;
      if (n >= N) continue;
      if (S == 1) epi_store<EPI>(args, z, m, n, acc[i][j]);
      else args.workspace[((z * S + blockIdx.y) * (int64_t)M + m) * N + n] = acc[i][j];
    }
  }
}

template <int EPI>
__global__ void __launch_bounds__(256) small_reduce_kernel(const maeclip_gemm_args args, int S) {
  const int64_t MN = args.M * args.N;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= MN) return;
  const int64_t z = blockIdx.z;
  const float* ws = args.workspace + z * S * MN + e;
  float v = ws[0];
  for (int s = 1; s < S; ++s) v += ws[s * MN];
  epi_store<EPI>(args, z, (int)(e / args.N), (int)(e % args.N), v);
}

// K slices: enough workgroups to cover the CUs twice, >= 2 chunks of 32 per slice
int small_splits(const maeclip_gemm_args& a) {
  const int64_t tiles = ((a.M + TS - 1) / TS) * ((a.N + TS - 1) / TS) * a.batch;
  const int64_t nch = (a.K + TS - 1) / TS;
  int64_t s = (512 + tiles - 1) / tiles;
  if (s > nch / 2) s = nch / 2;
  if (s > 32) s = 32;
  return (int)(s < 1 ? 1 : s);
}

template <int LA, int LB, int EPI>
int launch_small(const maeclip_gemm_args& a, hipStream_t s) {
  const int tiles = (int)(((a.M + TS - 1) / TS) * ((a.N + TS - 1) / TS));
  const int S = a.workspace ? small_splits(a) : 1;
  hipLaunchKernelGGL((gemm_small_kernel<LA, LB, EPI>), dim3(tiles, S, (unsigned)a.batch), dim3(256), 0, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(small f32)");
  if (S > 1) {
    const int64_t MN = a.M * a.N;
    hipLaunchKernelGGL((small_reduce_kernel<EPI>), dim3((unsigned)((MN + 255) / 256), 1, (unsigned)a.batch), dim3(256),
                       0, s, a, S);
    MC_CHECK_LAUNCH("maeclip_gemm(small f32 reduce)");
  }
  return 0;
}
template <int LA, int LB>
int epi_small(const maeclip_gemm_args& a, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_NONE: return launch_small<LA, LB, EPI_NONE>(a, s);
    case EPI_GELU: return launch_small<LA, LB, EPI_GELU>(a, s);
    case EPI_RESID: return launch_small<LA, LB, EPI_RESID>(a, s);
    case EPI_DGELU: return launch_small<LA, LB, EPI_DGELU>(a, s);
    case EPI_GELU_D: return launch_small<LA, LB, EPI_GELU_D>(a, s);
    default: return launch_small<LA, LB, EPI_MUL_AUX>(a, s);
  }
}

}  // namespace

namespace maeclip {
// fp32, no caller split-K, no column-sum partials, and few enough outputs that
// the 128x128 MFMA tiles would leave most CUs idle. a.workspace, when set
// (maeclip_gemm_workspace bytes), holds this path's own K-slice partials.
bool gemm_small_ok(const maeclip_gemm_args& a) {
  return a.dtype == MAECLIP_F32 && a.out_dtype == MAECLIP_F32 && a.splitk <= 1 && !a.colsum_partial &&
         a.M * a.N <= 256 * 1024 && a.K <= 8192;
}

// workspace bytes gemm_small uses for split-K partials (0: it runs unsplit)
int64_t gemm_small_workspace(const maeclip_gemm_args& a) {
  const int S = small_splits(a);
  return S > 1 ? (int64_t)S * a.M * a.N * a.batch * 4 : 0;
}

int gemm_small(const maeclip_gemm_args& a, hipStream_t s) {
  if (a.a_layout == LAY_KC && a.b_layout == LAY_KC) return epi_small<LAY_KC, LAY_KC>(a, s);
  if (a.a_layout == LAY_KC && a.b_layout == LAY_RC) return epi_small<LAY_KC, LAY_RC>(a, s);
  if (a.a_layout == LAY_RC && a.b_layout == LAY_KC) return epi_small<LAY_RC, LAY_KC>(a, s);
  return epi_small<LAY_RC, LAY_RC>(a, s);
}
}  // namespace maeclip
