// GEMM v3 (bf16, K % 32 == 0): persistent 256x256 tiles with a 4-deep LDS-DMA
// ring that runs continuously across output tiles.
//
// Why (profiles/r01): v2 issues the DMA of K-tile t+1 while tile t is on the
// MFMAs and then drains vmcnt(0) at a barrier every K-tile, so any DMA latency
// beyond one K-tile of math stalls all 16 waves; and every workgroup pays a
// cold prologue + an epilogue during which its CU streams nothing.
// v3:
//   * BK = 32 -> a 256x256 K-tile is 32 KiB; 4 ring slots = 128 KiB of LDS;
//     three K-tiles are in flight while the fourth is consumed;
//   * counted `s_waitcnt vmcnt(N)` + raw s_barrier: each wave waits only for its
//     own DMA of the NEXT K-tile (2 wave-instructions per K-tile per wave), never
//     vmcnt(0) in steady state (cdna_hip_programming.md §5 "Pipelining across
//     barriers");
//   * persistent grid (one 16-wave workgroup per CU): the ring prefetches the
//     first K-tiles of the next output tile while the current tile's epilogue
//     is stored;
//   * XCD-aware tile order: workgroups that share an XCD walk consecutive tiles
//     (same A row-block) so A panels are L2 hits.
// LDS images: KC [256 rows][64 B], 16-B chunk ^ (((row>>2)&1)<<1); RC [32 k][512 B],
// 8-B unit ^ 4*swz(k) -- both conflict-free (tools/lds_bank_sim.py), swizzle
// applied to the DMA source address and undone on the ds_read.
#include "common.h"
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3 };
constexpr int BM = 256, BN = 256, NW = 16, NT = NW * 64;

__device__ __forceinline__ int swz_rc(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }
typedef __attribute__((address_space(3))) void lds_void;

// BK*R*2 bytes per operand tile = BK*R/512 wave-instructions of 1 KiB over NW waves
template <int LAY, int R, int BK>
__device__ __forceinline__ void issue3(const bf16_t* __restrict__ p, int64_t ld, int r0, int Rtot, int k0, char* lds,
                                       int wave, int lane) {
  constexpr int NI = BK * R / 512 / NW;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int q = i * NW + wave;
    const bf16_t* src;
    if (LAY == LAY_KC) {
      constexpr int RB = BK * 2, RPI = 1024 / RB, CPR = RB / 16;  // row bytes, rows / instruction
      const int row = q * RPI + lane / CPR;
      const int c = BK == 32 ? ((lane & 3) ^ (((row >> 2) & 1) << 1)) : ((lane & 7) ^ ((row >> 1) & 7));
      const int rr = min(r0 + row, Rtot - 1);
      src = p + (int64_t)rr * ld + k0 + c * 8;
    } else {
      constexpr int CPR = R / 8, RPI = 64 / CPR;
      const int kr = q * RPI + lane / CPR;
      const int c = (lane % CPR) ^ (swz_rc(kr) >> 1);
      const int col = min(r0 + c * 8, Rtot - 8);
      src = p + (int64_t)(k0 + kr) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + q * 1024), 16, 0, 0);
  }
}

template <int LAY, int R, int BK>
__device__ __forceinline__ v8s frag3(const char* lds, int rs, int ks, int lane) {
  if (LAY == LAY_KC) {
    const int row = rs + (lane & 15);
    if (BK == 32) {
      const int chunk = lane >> 4;
      return *(const v8s*)(lds + row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4));
    }
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

__device__ __forceinline__ void wait_vm(int n) {
  // n = DMA instructions of this wave that may stay in flight
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BK>
struct Work {
  int M, N, K, S, tiles, gm, gn, klen;
  int64_t items;
  // item -> (z, split, bm, bn, kbeg, nkt)
  __device__ __forceinline__ void decode(int64_t item, int& z, int& s, int& bm, int& bn, int& kbeg, int& nkt) const {
    const int tile = (int)(item % tiles);
    const int64_t rest = item / tiles;
    s = (int)(rest % S);
    z = (int)(rest / S);
    bm = tile / gn;
    bn = tile % gn;
    kbeg = s * klen;
    const int kend = min(K, kbeg + klen);
    nkt = kend > kbeg ? (kend - kbeg) / BK : 0;
  }
};

template <int LA, int LB, typename OutT, int EPI, int BK, int NST>
__global__ void __launch_bounds__(NT) gemm3_kernel(const maeclip_gemm_args args) {
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int IPT = 2 * BK * BM / 512 / NW;  // DMA instructions per wave per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  Work<BK> W;
  W.M = (int)args.M; W.N = (int)args.N; W.K = (int)args.K;
  W.S = args.splitk > 1 ? args.splitk : 1;
  W.gm = (W.M + BM - 1) / BM;
  W.gn = (W.N + BN - 1) / BN;
  W.tiles = W.gm * W.gn;
  W.klen = ((W.K + W.S - 1) / W.S + BK - 1) / BK * BK;
  W.items = (int64_t)W.tiles * W.S * args.batch;

  // logical block id: workgroups sharing an XCD (blockIdx % 8) get consecutive ids
  const int G = gridDim.x;
  int lb = blockIdx.x;
  {
    const int q = G / 8, r = G % 8, x = lb % 8;
    lb = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lb / 8;
  }

  // producer cursor (DMA) and consumer cursor (MFMA) over this block's items
  int64_t p_item = lb, c_item = lb;
  int p_k = 0, c_k = 0;
  int pz = 0, ps = 0, pbm = 0, pbn = 0, pkbeg = 0, pnkt = 0;
  int cz, cs, cbm, cbn, ckbeg, cnkt;
  if (p_item < W.items) W.decode(p_item, pz, ps, pbm, pbn, pkbeg, pnkt); else pnkt = 0;
  cz = pz; cs = ps; cbm = pbm; cbn = pbn; ckbeg = pkbeg; cnkt = pnkt;
  // skip empty split slices (only possible when klen*S overshoots K)
  int issued = 0, consumed = 0;

  auto produce = [&]() -> bool {
    while (p_item < W.items && p_k >= pnkt) {
      p_item += G;
      p_k = 0;
      if (p_item < W.items) W.decode(p_item, pz, ps, pbm, pbn, pkbeg, pnkt);
    }
    if (p_item >= W.items) return false;
    char* st = smem + (issued % NST) * STAGE;
    const bf16_t* A = (const bf16_t*)args.A + (int64_t)pz * args.strideA;
    const bf16_t* B = (const bf16_t*)args.B + (int64_t)pz * args.strideB;
    const int k0 = pkbeg + p_k * BK;
    issue3<LA, BM, BK>(A, args.lda, pbm * BM, W.M, k0, st, wave, lane);
    issue3<LB, BN, BK>(B, args.ldb, pbn * BN, W.N, k0, st + A_BYTES, wave, lane);
    ++p_k;
    ++issued;
    return true;
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  for (int i = 0; i < NST - 1; ++i) produce();
  wait_vm(IPT * (issued - 1));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  while (c_item < W.items) {
    if (c_k >= cnkt) {  // (empty slice) advance without computing
      c_item += G;
      c_k = 0;
      if (c_item < W.items) W.decode(c_item, cz, cs, cbm, cbn, ckbeg, cnkt);
      continue;
    }
    const bool last = (c_k + 1 == cnkt);
    if (!last) produce();
    const char* sA = smem + (consumed % NST) * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      v8s fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag3<LA, BM, BK>(sA, wm * 64 + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag3<LB, BN, BK>(sB, wn * 64 + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    ++consumed;
    ++c_k;
    if (last) {
      // Drain the ring's DMA (the next K-tiles have had a full K-tile of MFMAs to
      // land) so the epilogue's loads/stores are counted exactly by the compiler
      // instead of each load waiting vmcnt(0) behind every earlier store.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ---------------- epilogue of (cz, cs, cbm, cbn): lane owns C[m][n..n+3]
      const int M = W.M, N = W.N, S = W.S;
      const int m0 = cbm * BM, n0 = cbn * BN;
      const int g = lane >> 4;
      if (S > 1) {
        float* slab = args.workspace + ((int64_t)cz * S + cs) * (int64_t)M * N;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * 64 + 16 * i + (lane & 15);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + 16 * j + 4 * g;
            if (m < M && n < N) *(v4f*)(slab + (int64_t)m * N + n) = acc[i][j] * args.alpha;
          }
        }
      } else {
        OutT* __restrict__ C = (OutT*)args.C + (int64_t)cz * args.strideC;
        v4f bias4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = min(n0 + wn * 64 + 16 * j + 4 * g, N - 4);
          bias4[j] = args.bias ? *(const v4f*)(args.bias + n) : v4f{0.f, 0.f, 0.f, 0.f};
        }
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
            v4f v = acc[i][j] * args.alpha + bias4[j];
            if (EPI == EPI_GELU) {
              st4<bf16_t>((bf16_t*)args.aux_out + (int64_t)cz * args.strideC + (int64_t)m * args.ldaux + n, v);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
            } else if (EPI == EPI_RESID) {
              v += *(const v4f*)(args.resid + (int64_t)cz * args.strideC + (int64_t)m * args.ldr + n);
            } else if (EPI == EPI_DGELU) {
              const v4f pre = ld4<bf16_t>((const bf16_t*)args.aux + (int64_t)cz * args.strideC + (int64_t)m * args.ldaux + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] *= gelu_grad_f(pre[r]);
              if (args.resid) v += *(const v4f*)(args.resid + (int64_t)cz * args.strideC + (int64_t)m * args.ldr + n);
            }
            OutT* cp = C + (int64_t)m * args.ldc + n;
            if (args.beta != 0.f) v += args.beta * ld4<OutT>(cp);
#pragma unroll
            for (int r = 0; r < 4; ++r) csum[j][r] += v[r];
            st4<OutT>(cp, v);
          }
        }
        if (args.colsum_partial) {
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
          if ((lane & 15) == 0 && mrow < M) {
            float* prow = args.colsum_partial + ((int64_t)cz * ((M + 63) / 64) + mrow / 64) * N;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int n = n0 + wn * 64 + 16 * j + 4 * g;
              if (n < N) *(v4f*)(prow + n) = v4f{csum[j][0], csum[j][1], csum[j][2], csum[j][3]};
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
      c_item += G;
      c_k = 0;
      if (c_item < W.items) W.decode(c_item, cz, cs, cbm, cbn, ckbeg, cnkt);
      const int issued_before = issued;
      produce();
      // with >= 3 ring slots the next K-tile was issued before the drain and has
      // landed; with 2 slots it was issued just now -> wait for it
      if (consumed >= issued_before) wait_vm(IPT * (issued - consumed - 1));
    } else {
      wait_vm(IPT * (issued - consumed - 1));
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
}

template <int LA, int LB, typename OutT, int EPI, int BK, int NST>
int launch3(const maeclip_gemm_args& a, hipStream_t s) {
  constexpr int STAGE = (BM + BN) * BK * 2;
  const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int64_t items = tiles * (a.splitk > 1 ? a.splitk : 1) * a.batch;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int grid = (int)(items < ncu ? items : ncu);
  const size_t lds = (size_t)NST * STAGE;
  auto kern = gemm3_kernel<LA, LB, OutT, EPI, BK, NST>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(v3)");
  return 0;
}

#ifndef MAECLIP_G3_BK
#define MAECLIP_G3_BK 64
#define MAECLIP_G3_NST 2
#endif
template <int LA, int LB, typename OutT>
int epi3(const maeclip_gemm_args& a, hipStream_t s) {
  constexpr int BK = MAECLIP_G3_BK, NS = MAECLIP_G3_NST;
  switch (a.epilogue) {
    case EPI_NONE: return launch3<LA, LB, OutT, EPI_NONE, BK, NS>(a, s);
    case EPI_GELU: return launch3<LA, LB, OutT, EPI_GELU, BK, NS>(a, s);
    case EPI_RESID: return launch3<LA, LB, OutT, EPI_RESID, BK, NS>(a, s);
    default: return launch3<LA, LB, OutT, EPI_DGELU, BK, NS>(a, s);
  }
}
template <int LA, int LB>
int out3(const maeclip_gemm_args& a, hipStream_t s) {
  return a.out_dtype == MAECLIP_BF16 ? epi3<LA, LB, bf16_t>(a, s) : epi3<LA, LB, float>(a, s);
}

}  // namespace

namespace maeclip {
int gemm_v3(const maeclip_gemm_args& a, hipStream_t s) {
  if (a.a_layout == LAY_KC && a.b_layout == LAY_KC) return out3<LAY_KC, LAY_KC>(a, s);
  if (a.a_layout == LAY_KC && a.b_layout == LAY_RC) return out3<LAY_KC, LAY_RC>(a, s);
  if (a.a_layout == LAY_RC && a.b_layout == LAY_KC) return out3<LAY_RC, LAY_KC>(a, s);
  return out3<LAY_RC, LAY_RC>(a, s);
}
}  // namespace maeclip
