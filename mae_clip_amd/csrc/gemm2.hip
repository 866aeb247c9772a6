// GEMM v2 (bf16 operands, fp32 accumulate) for K % 64 == 0 -- the production
// path of every Linear on the hot path (see gemm.hip for the op mapping).
//
// Differences from v1 (gemm.hip, kept for fp32 parity mode and odd shapes):
//   * operands go HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA): no staging
//     VGPRs, no ds_write pass; the LDS image is lane-linear per wave
//     instruction, so the bank-conflict XOR swizzle is applied to the SOURCE
//     address and undone on the ds_read (cdna_hip_programming.md §5.4 rule 21);
//   * block tile BM x BN chosen per shape (128x128 / 256x128 / 128x256 /
//     256x256), 64x64 per wave, 16x16x32 bf16 MFMA, BK = 64, two LDS stages:
//     the DMA for K-tile t+1 is in flight while tile t is on the MFMAs, one
//     barrier per K-tile;
//   * out-of-range rows/columns are clamped to valid addresses (their results
//     are never stored) -> no per-load predicates.
// Epilogue semantics are identical to v1 (bias, GELU, residual, dGELU,
// column-sum partials, split-K slabs).
#include "common.h"
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

__device__ __forceinline__ int swz_rc(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

typedef __attribute__((address_space(3))) void lds_void;

// Issue the LDS-DMA of one operand tile: R rows (M or N) x 64 k, 128*R bytes,
// as R/8 wave-instructions of 1 KiB distributed over NW waves.
template <int LAY, int R, int NW>
__device__ __forceinline__ void issue_operand(const bf16_t* __restrict__ p, int64_t ld, int r0, int Rtot, int k0,
                                              char* lds, int wave, int lane) {
  constexpr int NI = R / 8 / NW;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int q = i * NW + wave;
    const bf16_t* src;
    if (LAY == LAY_KC) {
      const int r = q * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int rr = min(r0 + r, Rtot - 1);
      src = p + (int64_t)rr * ld + k0 + c * 8;
    } else {
      constexpr int CPR = R / 8;           // 16-B chunks per k-row (row = 2R bytes)
      constexpr int RPI = 64 / CPR;        // k-rows per wave-instruction
      const int kr = q * RPI + lane / CPR;
      const int c = (lane % CPR) ^ (swz_rc(kr) >> 1);
      const int col = min(r0 + c * 8, Rtot - 8);
      src = p + (int64_t)(k0 + kr) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + q * 1024), 16, 0, 0);
  }
}

template <int LAY, int R>
__device__ __forceinline__ v8s load_frag(const char* lds, int rs, int ks, int lane) {
  if (LAY == LAY_KC) {
    const int row = rs + (lane & 15);
    const int chunk = 4 * ks + (lane >> 4);
    return *(const v8s*)(lds + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int unit = (rs >> 2) + p;
    v8s v;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int krow = 32 * ks + 8 * g + 4 * h + q;
      const char* a = lds + krow * (2 * R) + ((unit ^ swz_rc(krow)) << 3);
      v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
      v[4 * h + 0] = t[0];
      v[4 * h + 1] = t[1];
      v[4 * h + 2] = t[2];
      v[4 * h + 3] = t[3];
    }
    return v;
  }
}

template <int BM, int BN, int WM, int WN, int LA, int LB, typename OutT, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) gemm2_kernel(const maeclip_gemm_args args) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int M = (int)args.M, N = (int)args.N, K = (int)args.K;

  const int gm = (M + BM - 1) / BM, gn = (N + BN - 1) / BN;
  const int nwg = gm * gn;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap: consecutive tiles (same A rows) share an XCD's L2
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int bm = bid / gn, bn = bid % gn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int64_t z = blockIdx.z;
  const bf16_t* __restrict__ A = (const bf16_t*)args.A + z * args.strideA;
  const bf16_t* __restrict__ B = (const bf16_t*)args.B + z * args.strideB;

  const int S = args.splitk > 1 ? args.splitk : 1;
  const int klen = ((K + S - 1) / S + 63) / 64 * 64;
  const int kbeg = blockIdx.y * klen;
  const int kend = min(K, kbeg + klen);
  const int nt = kend > kbeg ? (kend - kbeg) / 64 : 0;

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    issue_operand<LA, BM, NW>(A, args.lda, m0, M, kbeg, smem, wave, lane);
    issue_operand<LB, BN, NW>(B, args.ldb, n0, N, kbeg, smem + A_BYTES, wave, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const char* sA = smem + (t & 1) * STAGE;
    const char* sB = sA + A_BYTES;
    if (t + 1 < nt) {
      char* nA = smem + ((t + 1) & 1) * STAGE;
      issue_operand<LA, BM, NW>(A, args.lda, m0, M, kbeg + (t + 1) * 64, nA, wave, lane);
      issue_operand<LB, BN, NW>(B, args.ldb, n0, N, kbeg + (t + 1) * 64, nA + A_BYTES, wave, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = load_frag<LA, BM>(sA, wm * TM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = load_frag<LB, BN>(sB, wn * TN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---------------- epilogue: lane owns C[m][n..n+3]
  const int g = lane >> 4;
  if (S > 1) {
    float* slab = args.workspace + ((int64_t)z * S + blockIdx.y) * (int64_t)M * N;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + 16 * j + 4 * g;
        if (m < M && n < N) *(v4f*)(slab + (int64_t)m * N + n) = acc[i][j] * args.alpha;
      }
    }
    return;
  }
  OutT* __restrict__ C = (OutT*)args.C + z * args.strideC;
  const float alpha = args.alpha, beta = args.beta;
  const float* __restrict__ bias = args.bias;
  constexpr int NH = TM / 64;  // 64-row groups per wave (column-sum partial rows)
  float csum[NH][FN][4];
#pragma unroll
  for (int hh = 0; hh < NH; ++hh)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[hh][j][r] = 0.f;
  v4f bias4[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = min(n0 + wn * TN + 16 * j + 4 * g, N - 4);
    bias4[j] = bias ? *(const v4f*)(bias + n) : v4f{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + 16 * i + (lane & 15);
    const bool mok = m < M;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + 16 * j + 4 * g;
      if (!mok || n >= N) continue;
      v4f v = acc[i][j] * alpha + bias4[j];
      if (EPI == EPI_GELU) {
        if (args.aux_out) st4<bf16_t>((bf16_t*)args.aux_out + z * args.strideC + (int64_t)m * args.ldaux + n, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
      } else if (EPI == EPI_RESID) {
        v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      } else if (EPI == EPI_DGELU) {
        const v4f pre = ld4<bf16_t>((const bf16_t*)args.aux + z * args.strideC + (int64_t)m * args.ldaux + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_f(pre[r]);
        if (args.resid) v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      } else if (EPI == EPI_GELU_D) {
        const v4f d = gelu4_inplace(v);
        if (args.aux_out) st4<bf16_t>((bf16_t*)args.aux_out + z * args.strideC + (int64_t)m * args.ldaux + n, d);
      } else if (EPI == EPI_MUL_AUX) {
        v *= ld4<bf16_t>((const bf16_t*)args.aux + z * args.strideC + (int64_t)m * args.ldaux + n);
        if (args.resid) v += *(const v4f*)(args.resid + z * args.strideC + (int64_t)m * args.ldr + n);
      }
      OutT* cp = C + (int64_t)m * args.ldc + n;
      if (beta != 0.f) v += beta * ld4<OutT>(cp);
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[i / 4][j][r] += v[r];
      st4<OutT>(cp, v);
    }
  }
  if (args.colsum_partial) {  // one partial row per 64-row group
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = csum[hh][j][r];
          s += __shfl_xor(s, 1, 64);
          s += __shfl_xor(s, 2, 64);
          s += __shfl_xor(s, 4, 64);
          s += __shfl_xor(s, 8, 64);
          csum[hh][j][r] = s;
        }
      const int mrow = m0 + wm * TM + 64 * hh;
      if ((lane & 15) == 0 && mrow < M) {
        float* prow = args.colsum_partial + ((int64_t)z * ((M + 63) / 64) + mrow / 64) * N;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0 + wn * TN + 16 * j + 4 * g;
          if (n < N) *(v4f*)(prow + n) = v4f{csum[hh][j][0], csum[hh][j][1], csum[hh][j][2], csum[hh][j][3]};
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int LA, int LB, typename OutT, int EPI>
int launch2(const maeclip_gemm_args& a, hipStream_t s) {
  const int gm = (int)((a.M + BM - 1) / BM), gn = (int)((a.N + BN - 1) / BN);
  const int S = a.splitk > 1 ? a.splitk : 1;
  const size_t lds = (size_t)2 * (BM + BN) * 128;
  auto kern = gemm2_kernel<BM, BN, WM, WN, LA, LB, OutT, EPI>;
  if (lds > 65536) maeclip::allow_lds((const void*)kern, (int)lds);
  hipLaunchKernelGGL(kern, dim3(gm * gn, S, (unsigned)a.batch), dim3(WM * WN * 64), lds, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(v2)");
  return 0;
}

template <int BM, int BN, int WM, int WN, int LA, int LB, typename OutT>
int epi2(const maeclip_gemm_args& a, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_NONE: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_NONE>(a, s);
    case EPI_GELU: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_GELU>(a, s);
    case EPI_RESID: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_RESID>(a, s);
    case EPI_GELU_D: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_GELU_D>(a, s);
    case EPI_MUL_AUX: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_MUL_AUX>(a, s);
    default: return launch2<BM, BN, WM, WN, LA, LB, OutT, EPI_DGELU>(a, s);
  }
}

template <int BM, int BN, int WM, int WN, int LA, int LB>
int out2(const maeclip_gemm_args& a, hipStream_t s) {
  return a.out_dtype == MAECLIP_BF16 ? epi2<BM, BN, WM, WN, LA, LB, bf16_t>(a, s)
                                     : epi2<BM, BN, WM, WN, LA, LB, float>(a, s);
}

template <int BM, int BN, int WM, int WN>
int lay2(const maeclip_gemm_args& a, hipStream_t s) {
  if (a.a_layout == LAY_KC && a.b_layout == LAY_KC) return out2<BM, BN, WM, WN, LAY_KC, LAY_KC>(a, s);
  if (a.a_layout == LAY_KC && a.b_layout == LAY_RC) return out2<BM, BN, WM, WN, LAY_KC, LAY_RC>(a, s);
  if (a.a_layout == LAY_RC && a.b_layout == LAY_KC) return out2<BM, BN, WM, WN, LAY_RC, LAY_KC>(a, s);
  return out2<BM, BN, WM, WN, LAY_RC, LAY_RC>(a, s);
}

}  // namespace

namespace maeclip {
// variant: 0 auto, 1 = 128x128 (4 waves), 2 = 256x128 (8), 3 = 128x256 (8), 4 = 256x256 (16)
int gemm_v2(const maeclip_gemm_args& a, hipStream_t s, int variant) {
  if (variant == 0) {
    // measured on the C2 shapes (tools/gemm_variants.sh): the 256x256 / 16-wave
    // tile wins every fwd, dgrad and split-K wgrad shape; 128x128 below 256.
    variant = (a.M >= 256 && a.N >= 256) ? 4 : 1;
  }
  switch (variant) {
    case 2: return lay2<256, 128, 4, 2>(a, s);
    case 3: return lay2<128, 256, 2, 4>(a, s);
    case 4: return lay2<256, 256, 4, 4>(a, s);
    case 6: return lay2<256, 256, 2, 4>(a, s);
    case 7: return lay2<256, 128, 2, 2>(a, s);
    default: return lay2<128, 128, 2, 2>(a, s);
  }
}
}  // namespace maeclip
