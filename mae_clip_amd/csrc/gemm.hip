// MFMA GEMM for every Linear on the hot path (gfx950).
//
// Replaces the cuBLAS calls that torch dispatches for the reference's
// nn.Linear / Conv2d-as-patch-GEMM (timm Block qkv/proj/fc1/fc2, PatchEmbed,
// modules.py:64-66 ProjectionHead, DistilBERT q/k/v/out/lin1/lin2) and the
// N x N x P products of the CLIP loss (CLIP.py:34-38).
//
//   C[M,N] = alpha * sum_k A(m,k) B(k,n)  (+ epilogue)
//
// Operand layouts (per operand, template):
//   KC : element (r,k) at p[r*ld + k]   (k contiguous; nn.Linear weight [N,K])
//   RC : element (r,k) at p[k*ld + r]   (row index contiguous)
// so Y = X W^T is (KC,KC), dX = dY W is (KC,RC), dW = dY^T X is (RC,RC).
//
// Tile: 128x128 per 256-thread workgroup (4 waves, 2x2, 64x64 per wave),
// K-tile = 128 bytes of K (64 bf16 / 32 f32); double-buffered LDS, register
// staging (16-B global loads, tile t+1 written after the compute of tile t),
// one barrier per K-tile.
// KC tiles: [128 rows][128 B], 16-B chunks XOR-swizzled by (row>>1)&7 so the
//   ds_read_b128 fragment reads are conflict-free.
// RC tiles (bf16): [64 k][128 cols], 8-B units XOR-swizzled by 4*swz(k); read
//   with ds_read_b64_tr_b16 (hardware transpose) -> conflict-free.
// MFMA: v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32 (fp32
//   parity mode, exact f32). The product is issued operand-swapped (B tile as
//   the A operand) so each lane ends up owning 4 consecutive columns of one
//   output row -> vectorised epilogue loads/stores along N.
#include "common.h"
#include "../../include/maeclip.h"
#include <stdlib.h>

namespace maeclip {
int gemm_v2(const maeclip_gemm_args& a, hipStream_t s, int variant);
int gemm_v4(const maeclip_gemm_args& a, hipStream_t s);
bool gemm_v4_ok(const maeclip_gemm_args& a);
int check_q8(const maeclip_gemm_args& a, const char* who);
int64_t gemm_v4_workspace(const maeclip_gemm_args& a);
int gemm_small(const maeclip_gemm_args& a, hipStream_t s);
bool gemm_small_ok(const maeclip_gemm_args& a);
int64_t gemm_small_workspace(const maeclip_gemm_args& a);
}

namespace {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int TILE_BYTES = 16384;  // one operand, one stage

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

template <typename T> struct Tr;
template <> struct Tr<bf16_t> { static constexpr int BK = 64; static constexpr int EPC = 8; };
template <> struct Tr<float> { static constexpr int BK = 32; static constexpr int EPC = 4; };

__device__ __forceinline__ int swz_rc(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

// ---- staging: global -> registers (4 x 16 B per thread per operand)
template <typename T, int LAY>
__device__ __forceinline__ void stage_load(v4u (&r)[4], const T* __restrict__ p, int64_t ld, int r0,
                                           int R, int k0, int K, int tid) {
  constexpr int EPC = Tr<T>::EPC;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int id = it * NT + tid;
    int row, kk;
    if (LAY == LAY_KC) {
      row = id >> 3;
      kk = (id & 7) * EPC;
      const bool ok = (r0 + row < R) && (k0 + kk < K);
      r[it] = ok ? *(const v4u*)(p + (int64_t)(r0 + row) * ld + (k0 + kk)) : v4u{0, 0, 0, 0};
    } else {
      constexpr int CPR = 128 / EPC;  // 16B chunks per k-row of the tile
      const int krow = id / CPR;
      const int col = (id % CPR) * EPC;
      const bool ok = (k0 + krow < K) && (r0 + col < R);
      r[it] = ok ? *(const v4u*)(p + (int64_t)(k0 + krow) * ld + (r0 + col)) : v4u{0, 0, 0, 0};
    }
  }
}

template <typename T, int LAY>
__device__ __forceinline__ void stage_store(char* lds, const v4u (&r)[4], int tid) {
  constexpr int EPC = Tr<T>::EPC;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int id = it * NT + tid;
    int off;
    if (LAY == LAY_KC) {
      const int row = id >> 3, c = id & 7;
      off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
    } else if (sizeof(T) == 2) {
      const int krow = id >> 4, c = id & 15;
      off = krow * 256 + (((2 * c) ^ swz_rc(krow)) << 3);
    } else {
      const int krow = id >> 5, c = id & 31;
      off = krow * 512 + c * 16;
    }
    *(v4u*)(lds + off) = r[it];
  }
  (void)EPC;
}

// ---- fragment: 8 consecutive k (k = 8*g + j, g = lane>>4) of tile row rs + (lane&15)
template <typename T, int LAY> struct Frag;

template <> struct Frag<bf16_t, LAY_KC> {
  v8s v;
  __device__ __forceinline__ void load(const char* lds, int rs, int ks, int lane) {
    const int row = rs + (lane & 15);
    const int chunk = 4 * ks + (lane >> 4);
    v = *(const v8s*)(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  }
};
template <> struct Frag<bf16_t, LAY_RC> {
  v8s v;
  __device__ __forceinline__ void load(const char* lds, int rs, int ks, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int unit = (rs >> 2) + p;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int krow = 32 * ks + 8 * g + 4 * h + q;
      const char* a = lds + krow * 256 + ((unit ^ swz_rc(krow)) << 3);
      v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
      v[4 * h + 0] = t[0];
      v[4 * h + 1] = t[1];
      v[4 * h + 2] = t[2];
      v[4 * h + 3] = t[3];
    }
  }
};
template <> struct Frag<float, LAY_KC> {
  float v[8];
  __device__ __forceinline__ void load(const char* lds, int rs, int ks, int lane) {
    const int row = rs + (lane & 15);
    const int g = lane >> 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int chunk = 2 * g + h;
      v4f t = *(const v4f*)(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
      v[4 * h + 0] = t[0];
      v[4 * h + 1] = t[1];
      v[4 * h + 2] = t[2];
      v[4 * h + 3] = t[3];
    }
    (void)ks;
  }
};
template <> struct Frag<float, LAY_RC> {
  float v[8];
  __device__ __forceinline__ void load(const char* lds, int rs, int ks, int lane) {
    const int col = rs + (lane & 15);
    const int g = lane >> 4;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *(const float*)(lds + (8 * g + j) * 512 + col * 4);
    (void)ks;
  }
};

// D[n][m] += sum_k B(k,n) A(m,k) : operand-swapped product (see header)
template <int LA, int LB>
__device__ __forceinline__ v4f mma(const Frag<bf16_t, LB>& b, const Frag<bf16_t, LA>& a, v4f acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b.v, a.v, acc, 0, 0, 0);
}
template <int LA, int LB>
__device__ __forceinline__ v4f mma(const Frag<float, LB>& b, const Frag<float, LA>& a, v4f acc) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(b.v[s], a.v[s], acc, 0, 0, 0);
  return acc;
}

template <typename T, typename OutT, int LA, int LB, int EPI>
__global__ void __launch_bounds__(NT, 2)
gemm_kernel(const maeclip_gemm_args args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BK = Tr<T>::BK;
  constexpr int KSTEPS = sizeof(T) == 2 ? 2 : 1;  // 32-deep MFMA k-steps per K-tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = (int)args.M, N = (int)args.N, K = (int)args.K;

  // XCD-aware remap: consecutive tiles (sharing A rows) land on one XCD.
  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int bm = bid / gn, bn = bid % gn;
  const int m0 = bm * BM, n0 = bn * BN;

  const int64_t z = blockIdx.z;
  const T* __restrict__ A = (const T*)args.A + z * args.strideA;
  const T* __restrict__ B = (const T*)args.B + z * args.strideB;
  OutT* __restrict__ C = (OutT*)args.C + z * args.strideC;

  // stage s: A at smem + 2*s*TILE, B at smem + (2*s+1)*TILE
#define LDS_A(s) (smem + (2 * (s)) * TILE_BYTES)
#define LDS_B(s) (smem + (2 * (s) + 1) * TILE_BYTES)

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  v4u ra[4], rb[4];
  // split-K slice [kbeg, kend) (whole K when splitk == 1)
  const int S = args.splitk > 1 ? args.splitk : 1;
  const int klen = ((K + S - 1) / S + BK - 1) / BK * BK;
  const int kbeg = blockIdx.y * klen;
  const int kend = min(K, kbeg + klen);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  stage_load<T, LA>(ra, A, args.lda, m0, M, kbeg, kend, tid);
  stage_load<T, LB>(rb, B, args.ldb, n0, N, kbeg, kend, tid);
  stage_store<T, LA>(LDS_A(0), ra, tid);
  stage_store<T, LB>(LDS_B(0), rb, tid);
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < nt;
    if (more) {
      stage_load<T, LA>(ra, A, args.lda, m0, M, kbeg + (t + 1) * BK, kend, tid);
      stage_load<T, LB>(rb, B, args.ldb, n0, N, kbeg + (t + 1) * BK, kend, tid);
    }
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      Frag<T, LA> fa[4];
      Frag<T, LB> fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i].load(LDS_A(cur), wm * 64 + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j].load(LDS_B(cur), wn * 64 + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma<LA, LB>(fb[j], fa[i], acc[i][j]);
    }
    if (more) {
      stage_store<T, LA>(LDS_A(cur ^ 1), ra, tid);
      stage_store<T, LB>(LDS_B(cur ^ 1), rb, tid);
    }
    __syncthreads();
  }

  // ---------------- epilogue: lane owns C[m][n..n+3]
  const int g = lane >> 4;
  if (S > 1) {  // split-K: raw fp32 partial tile -> workspace slab (reduced by splitk_reduce_kernel)
    float* slab = args.workspace + ((int64_t)z * S + blockIdx.y) * (int64_t)M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + 4 * g;
        if (m < M && n < N) *(v4f*)(slab + (int64_t)m * N + n) = acc[i][j] * args.alpha;
      }
    }
    return;
  }
  const float alpha = args.alpha, beta = args.beta;
  const float* __restrict__ bias = args.bias;
  float csum[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + 16 * i + (lane & 15);
    const bool mok = m < M;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + 16 * j + 4 * g;
      if (!mok || n >= N) continue;
      v4f v = acc[i][j] * alpha;
      if (bias) {
        const v4f bb = *(const v4f*)(bias + n);
        v += bb;
      }
      if (EPI == EPI_GELU) {
        if (args.aux_out) st4<T>((T*)args.aux_out + z * args.strideC + (int64_t)m * args.ldaux + n, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
      } else if (EPI == EPI_RESID) {
        v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      } else if (EPI == EPI_DGELU) {
        const v4f pre = ld4<T>((const T*)args.aux + z * args.strideC + (int64_t)m * args.ldaux + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_f(pre[r]);
        if (args.resid) v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      } else if (EPI == EPI_GELU_D) {
        const v4f d = gelu4_inplace(v);
        if (args.aux_out) st4<T>((T*)args.aux_out + z * args.strideC + (int64_t)m * args.ldaux + n, d);
      } else if (EPI == EPI_MUL_AUX) {
        v *= ld4<T>((const T*)args.aux + z * args.strideC + (int64_t)m * args.ldaux + n);
        if (args.resid) v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      }
      OutT* cp = C + (int64_t)m * args.ldc + n;
      if (beta != 0.f) v += beta * ld4<OutT>(cp);
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[j][r] += v[r];
      st4<OutT>(cp, v);
    }
  }
  if (args.colsum_partial) {
    // reduce over the 16 rows held by lanes sharing (lane>>4), then write one
    // partial row per (block row, wave row): deterministic bias gradients.
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = csum[j][r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        csum[j][r] = s;
      }
    const int mrow = m0 + wm * 64;
    if ((lane & 15) == 0 && mrow < M) {  // one partial row per 64-row group
      float* prow = args.colsum_partial + ((int64_t)z * ((M + 63) / 64) + mrow / 64) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + 4 * g;
        if (n < N) *(v4f*)(prow + n) = v4f{csum[j][0], csum[j][1], csum[j][2], csum[j][3]};
      }
    }
  }
}

// C[z] = sum_s slab[z][s] (+bias) (+beta*C), fixed summation order
template <typename OutT>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const maeclip_gemm_args a) {
  const int64_t MN = a.M * a.N;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= MN) return;
  const int64_t z = blockIdx.y;
  const float* ws = a.workspace + z * a.splitk * MN + e;
  v4f v = *(const v4f*)ws;
  for (int s = 1; s < a.splitk; ++s) v += *(const v4f*)(ws + s * MN);
  const int64_t m = e / a.N, n = e % a.N;
  if (a.bias) v += *(const v4f*)(a.bias + n);
  OutT* cp = (OutT*)a.C + z * a.strideC + m * a.ldc + n;
  if (a.beta != 0.f) v += a.beta * ld4<OutT>(cp);
  st4<OutT>(cp, v);
}

template <typename OutT>
int splitk_reduce_t(const maeclip_gemm_args& a, hipStream_t s) {
  const int64_t MN = a.M * a.N;
  dim3 g2((unsigned)((MN / 4 + 255) / 256), (unsigned)a.batch);
  hipLaunchKernelGGL((splitk_reduce_kernel<OutT>), g2, dim3(256), 0, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(splitk reduce)");
  return 0;
}

int splitk_reduce(const maeclip_gemm_args& a, hipStream_t s) {
  return a.out_dtype == MAECLIP_BF16 ? splitk_reduce_t<bf16_t>(a, s) : splitk_reduce_t<float>(a, s);
}

template <typename T, typename OutT, int LA, int LB, int EPI>
int launch(const maeclip_gemm_args& a, hipStream_t s) {
  const int gm = (int)((a.M + BM - 1) / BM), gn = (int)((a.N + BN - 1) / BN);
  const int S = a.splitk > 1 ? a.splitk : 1;
  dim3 grid(gm * gn, S, (unsigned)a.batch);
  hipLaunchKernelGGL((gemm_kernel<T, OutT, LA, LB, EPI>), grid, dim3(NT), 4 * TILE_BYTES, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm");
  if (S > 1) return splitk_reduce_t<OutT>(a, s);
  return 0;
}

template <typename T, typename OutT, int LA, int LB>
int dispatch_epi(const maeclip_gemm_args& a, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_NONE: return launch<T, OutT, LA, LB, EPI_NONE>(a, s);
    case EPI_GELU: return launch<T, OutT, LA, LB, EPI_GELU>(a, s);
    case EPI_RESID: return launch<T, OutT, LA, LB, EPI_RESID>(a, s);
    case EPI_DGELU: return launch<T, OutT, LA, LB, EPI_DGELU>(a, s);
    case EPI_GELU_D: return launch<T, OutT, LA, LB, EPI_GELU_D>(a, s);
    case EPI_MUL_AUX: return launch<T, OutT, LA, LB, EPI_MUL_AUX>(a, s);
  }
  maeclip::set_error("maeclip_gemm: bad epilogue %d", a.epilogue);
  return -1;
}
template <typename T, typename OutT>
int dispatch_lay(const maeclip_gemm_args& a, hipStream_t s) {
  if (a.a_layout == LAY_KC && a.b_layout == LAY_KC) return dispatch_epi<T, OutT, LAY_KC, LAY_KC>(a, s);
  if (a.a_layout == LAY_KC && a.b_layout == LAY_RC) return dispatch_epi<T, OutT, LAY_KC, LAY_RC>(a, s);
  if (a.a_layout == LAY_RC && a.b_layout == LAY_KC) return dispatch_epi<T, OutT, LAY_RC, LAY_KC>(a, s);
  return dispatch_epi<T, OutT, LAY_RC, LAY_RC>(a, s);
}

}  // namespace

extern "C" int32_t maeclip_gemm(const maeclip_gemm_args* a, void* stream) {
  MC_CHECK_ARG(a != nullptr, "maeclip_gemm: null args");
  MC_CHECK_ARG(a->M >= 0 && a->N >= 0 && a->K >= 0 && a->batch >= 1, "maeclip_gemm: bad sizes");
  if (a->M == 0 || a->N == 0) return 0;
  MC_CHECK_ARG(a->M < (1ll << 31) && a->N < (1ll << 31) && a->K < (1ll << 31), "maeclip_gemm: dims too large");
  MC_CHECK_ARG(a->dtype == MAECLIP_F32 || a->dtype == MAECLIP_BF16, "maeclip_gemm: bad dtype %d", a->dtype);
  MC_CHECK_ARG(a->out_dtype == MAECLIP_F32 || a->out_dtype == MAECLIP_BF16, "maeclip_gemm: bad out dtype");
  const int epc = a->dtype == MAECLIP_BF16 ? 8 : 4;
  // 16-B vector loads along the contiguous dimension of each operand
  MC_CHECK_ARG(a->a_layout == LAY_KC ? (a->K % epc == 0 && a->lda % epc == 0)
                                     : (a->M % epc == 0 && a->lda % epc == 0),
               "maeclip_gemm: A contiguous dim / lda must be a multiple of %d", epc);
  MC_CHECK_ARG(a->b_layout == LAY_KC ? (a->K % epc == 0 && a->ldb % epc == 0)
                                     : (a->N % epc == 0 && a->ldb % epc == 0),
               "maeclip_gemm: B contiguous dim / ldb must be a multiple of %d", epc);
  MC_CHECK_ARG(a->N % 4 == 0 && a->ldc % 4 == 0, "maeclip_gemm: N and ldc must be multiples of 4");
  MC_CHECK_ARG(((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->B & 15) == 0 && ((uintptr_t)a->C & 7) == 0,
               "maeclip_gemm: operands must be 16-byte aligned");
  MC_CHECK_ARG((a->epilogue != EPI_DGELU && a->epilogue != EPI_MUL_AUX) || a->aux,
               "maeclip_gemm: DGELU / MUL_AUX epilogue needs aux");
  MC_CHECK_ARG(a->epilogue != EPI_RESID || (a->resid && a->out_dtype == MAECLIP_F32),
               "maeclip_gemm: RESID epilogue needs fp32 resid and fp32 output");
  if (a->splitk > 1) {
    MC_CHECK_ARG(a->workspace && a->epilogue == EPI_NONE && !a->colsum_partial && a->splitk <= 64,
                 "maeclip_gemm: split-K needs a workspace, epilogue 0 and no colsum");
    MC_CHECK_ARG(a->ldc == a->N, "maeclip_gemm: split-K output must be dense (ldc == N)");
  }
  if (int e = maeclip::check_q8(*a, "maeclip_gemm")) return e;
  hipStream_t s = (hipStream_t)stream;
  // v2 (LDS-DMA, larger tiles) for every bf16 shape with 64-aligned K
  static const int forced = getenv("MAECLIP_GEMM_VARIANT") ? atoi(getenv("MAECLIP_GEMM_VARIANT")) : 0;
  // v4/v2 write raw fp32 split-K slabs and leave the reduction to
  // splitk_reduce (v1's launch() reduces by itself)
  if (forced != 99 && maeclip::gemm_small_ok(*a)) return maeclip::gemm_small(*a, s);
  int rc = 1;
  // v4 (8-wave ping-pong 256x256 / 192x256, persistent, buffer-descriptor DMA,
  // split tiles with an in-launch fix-up when the tiles leave most of the grid
  // idle) wherever its shape conditions hold; MAECLIP_GEMM_VARIANT=1..7 pins a
  // v2 tile, 99 v1
  const bool v4 = (forced == 0 || forced == 8) && maeclip::gemm_v4_ok(*a);
  // every path but v4 (whose epilogue writes it): the fp8-blocks copy of C
  // (q8) by a second pass
  if (a->q8 && !v4) {
    maeclip_gemm_args b = *a;
    b.q8 = nullptr;
    if (int e = maeclip_gemm(&b, stream)) return e;
    return maeclip_quant_blocks_fp8(a->C, MAECLIP_BF16, a->M, a->N, a->ldc, a->q8, a->ldq8, a->q8_scale, a->q8_fmt,
                                    stream);
  }
  if (v4)
    rc = maeclip::gemm_v4(*a, s);
  else if (a->dtype == MAECLIP_BF16 && forced != 99 && a->K % 64 == 0 && a->K > 0 && a->lda % 8 == 0 && a->ldb % 8 == 0 &&
           (a->a_layout == LAY_KC || a->M >= 8) && (a->b_layout == LAY_KC || a->N >= 8))
    rc = maeclip::gemm_v2(*a, s, forced == 8 ? 0 : forced);
  if (rc != 1) return (rc == 0 && a->splitk > 1) ? splitk_reduce(*a, s) : rc;
  if (a->dtype == MAECLIP_BF16)
    return a->out_dtype == MAECLIP_BF16 ? dispatch_lay<bf16_t, bf16_t>(*a, s) : dispatch_lay<bf16_t, float>(*a, s);
  return a->out_dtype == MAECLIP_BF16 ? dispatch_lay<float, bf16_t>(*a, s) : dispatch_lay<float, float>(*a, s);
}

extern "C" int64_t maeclip_gemm_colsum_rows(int64_t M) { return (M + 63) / 64; }

// Every GEMM runs on this library's kernels (ABI v9 kept the query; the
// round-4 vendor path was removed in round 5).
extern "C" int32_t maeclip_gemm_impl(const maeclip_gemm_args* a) {
  (void)a;
  return 0;
}

// Scratch bytes maeclip_gemm may use for this call when the caller asks for no
// split-K itself (splitk <= 1): the small-fp32 path's K-slice partials, or the
// v4 split plan's arrival counters + fp32 partial tiles (one workspace per
// stream: launches on one stream run in order; the counters must be zero
// before the first launch, and every completed launch leaves them zero).
extern "C" int64_t maeclip_gemm_workspace(const maeclip_gemm_args* a) {
  if (!a || a->splitk > 1) return 0;
  static const int forced = getenv("MAECLIP_GEMM_VARIANT") ? atoi(getenv("MAECLIP_GEMM_VARIANT")) : 0;
  if (forced != 99 && maeclip::gemm_small_ok(*a)) return maeclip::gemm_small_workspace(*a);
  return (forced == 0 || forced == 8) ? maeclip::gemm_v4_workspace(*a) : 0;
}

// Slice count for split-K (the wgrad shapes of the hot path have only 4-36
// output tiles of 256x256 but 12.8k-50k deep K). For shapes the v4 kernel takes
// (one 128-KiB-LDS block per CU) fill the 256 CUs exactly once: S = 256/tiles,
// at least 8 K-tiles of 64 per slice -- every extra slice costs an fp32 slab
// write + read in splitk_reduce. Other shapes (v1 128x128 tiles, several blocks
// per CU): ~1024 workgroups, >= 16 K-tiles per slice.
extern "C" int32_t maeclip_gemm_splitk(int64_t M, int64_t N, int64_t K) {
  int64_t s;
  if (M >= 256 && N >= 256 && K % 64 == 0) {
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
    s = 256 / tiles;
    if (s > K / 512) s = K / 512;
  } else {
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    s = 1024 / (tiles > 0 ? tiles : 1);
    if (s > K / 1024) s = K / 1024;
  }
  if (s > 64) s = 64;
  return (int32_t)(s < 1 ? 1 : s);
}
