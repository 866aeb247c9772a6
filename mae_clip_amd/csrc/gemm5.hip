// GEMM v5: 256x256x64 bf16 tiles, ONE wave per SIMD.
//
// Four waves (2 x 2) per workgroup, each owning a 128 x 128 output block =
// 8 x 8 fragments of 16x16: 256 fp32 accumulators per lane, which at one wave
// per SIMD live in the AGPR half of the 512-entry unified register file (the
// v4 kernel's 8-wave ping-pong gives each wave 128 x 64 and needs twice the
// LDS fragment reads per MFMA). Per 64-deep K-tile a wave reads 32 fragments
// (16-B ds_read_b128, or two ds_read_b64_tr_b16 for row-contiguous operands)
// for 128 MFMA 16x16x32 (2048 cycles of matrix pipe): the LDS array is far
// from saturated, and the latency of the next fragments is covered by the
// current MFMAs instead of by a partner wave.
//
// Operand staging: two LDS stages of 64 KiB (A rows 0-127 | A rows 128-255 |
// B 0-127 | B 128-255, each 16 KiB in the v4 kernel's swizzled half-image
// formats), filled by buffer-descriptor LDS-DMA (16 wave-instructions of 1 KiB
// per wave per stage). The K-tiles of all of a block's output tiles form ONE
// stream of stages g = 0, 1, 2, ... (stage g in buffer g & 1), so the first
// two stages of the next tile are in flight while the current tile's last
// K-tile and its epilogue run. Per K-tile (stage g in buffer b):
//   1. ds_read fragments F1 <- (g, k 32..63)        [F0 <- (g, k 0..31) already in VGPRs]
//   2. 64 MFMAs on F0
//   3. wait F1 (lgkmcnt(0)); barrier       -- every wave is done reading b
//   4. DMA stage g+2 -> b; wait this wave's stage g+1 DMA (counted vmcnt); barrier
//   5. ds_read F0 <- (g+1, k 0..31)         (buffer b ^ 1)
//   6. 64 MFMAs on F1
// so a stage's DMA has one K-tile (~1 us) to land and no MFMA waits for LDS.
#include "common.h"
#include <stdlib.h>
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

typedef __attribute__((address_space(3))) void lds_void;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int HALF = 16384;          // 128 rows (cols) x 64 k x bf16
constexpr int STAGE = 4 * HALF;      // A0 A1 B0 B1
constexpr int LDS5 = 2 * STAGE;      // 128 KiB
constexpr int NTH5 = 256;

__device__ __forceinline__ int swz_rc(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

__device__ __forceinline__ rsrc_t make_rsrc(const char* base, int64_t bytes) {
  const int nrec = (int)(bytes < 0x7fffffff ? (bytes > 0 ? bytes : 0) : 0x7fffffff);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);
}

// per-lane byte offset of DMA wave-instruction q (0..15) of half `sub` of an
// operand whose halves are contiguous 128-row (KC) / 128-column (RC) slabs
template <int LAY>
__device__ __forceinline__ int voff5(int64_t ld, int sub, int q, int lane) {
  if (LAY == LAY_KC) {
    const int r = q * 8 + (lane >> 3);                 // local row of the half
    const int c = (lane & 7) ^ ((r >> 1) & 7);         // 16-B chunk, XOR-swizzled
    return (int)((int64_t)(128 * sub + r) * ld * 2) + c * 16;
  } else {
    const int kr = q * 4 + (lane >> 4);                // k-row of the half
    const int c = (lane & 15) ^ (swz_rc(kr) >> 1);     // 16-B unit of the 256-B k-row
    return (int)((int64_t)kr * ld * 2) + (128 * sub + 8 * c) * 2;
  }
}

// voff5(ld, s, 4 i + wave, lane) - voff5(ld, 0, wave, lane): the XOR swizzle
// term is the same for every (s, i) of a lane (KC: (r >> 1) & 7 with r = 32 i +
// 8 wave + lane / 8; RC: kr & 3 and (kr >> 3) & 1 with kr = 16 i + 4 wave +
// lane / 16), so the difference is uniform
template <int LAY>
__device__ __forceinline__ int dsoff5(int64_t ld, int s, int i) {
  return LAY == LAY_KC ? (int)((int64_t)(128 * s + 32 * i) * ld * 2) : (int)((int64_t)(16 * i) * ld * 2) + 256 * s;
}

// 16x32 fragment (rows rs..rs+15 of a half, k 32ks..32ks+31) as an MFMA operand
template <int LAY>
__device__ __forceinline__ v8s frag5(const char* lds, int rs, int ks, int lane) {
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
      const char* a = lds + krow * 256 + ((unit ^ swz_rc(krow)) << 3);
      v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
      v[4 * h + 0] = t[0];
      v[4 * h + 1] = t[1];
      v[4 * h + 2] = t[2];
      v[4 * h + 3] = t[3];
    }
    return v;
  }
}

#define BARRIER5()                           \
  do {                                       \
    asm volatile("" ::: "memory");           \
    __builtin_amdgcn_sched_barrier(0);       \
    __builtin_amdgcn_s_barrier();            \
    __builtin_amdgcn_sched_barrier(0);       \
    asm volatile("" ::: "memory");           \
  } while (0)

struct Frags {
  v8s a[8], b[8];
};

template <int LA, int LB>
__device__ __forceinline__ void read_frags(Frags& f, const char* stage, int ks, int wm, int wn, int lane) {
  const char* ha = stage + wm * HALF;
  const char* hb = stage + (2 + wn) * HALF;
#pragma unroll
  for (int j = 0; j < 8; ++j) f.b[j] = frag5<LB>(hb, 16 * j, ks, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) f.a[i] = frag5<LA>(ha, 16 * i, ks, lane);
}

// The 256 accumulators are pinned to AGPRs ("+a"): with the builtin, the
// register allocator splits them across VGPRs/AGPRs and spills hundreds of
// them. ZERO starts a tile (src C = inline 0, no AGPR clears). The hazard
// recogniser does not see into asm: the dependence distance between MFMAs on
// one accumulator is 64 issues, and the epilogue starts after s_nops.
__device__ __forceinline__ void mma64(v4f (&acc)[8][8], const Frags& f) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)   // the host pass cannot type-check AGPR constraints
      asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(f.b[j]), "v"(f.a[i]));
#endif
    }
}

// Epilogue of a wave's 128 x 128 block. Fragment (i, j): rows m0 + 128 wm +
// 16 i + (lane & 15); after the permlane16 swap of column fragments (2p,
// 2p+1) lane group g holds 8 consecutive columns n0 + 128 wn + 32 p + 16 (g&1)
// + 8 (g>>1) .. +7 of fragment row i (16-B bf16 / 2 x 16-B f32 accesses).
// after_loads() is called once the last global load is issued (the kernel
// issues its deferred stage DMA there: vmcnt retires in issue order, so a load
// issued after the DMA would wait for the whole stage).
template <typename OutT, int EPI, typename Hook>
__device__ __forceinline__ void epilogue5(const maeclip_gemm_args& args, v4f (&acc)[8][8], int m0, int n0, int wm,
                                          int wn, int lane, Hook&& after_loads) {
  constexpr bool LOAD_AUX = EPI == EPI_DGELU || EPI == EPI_MUL_AUX;
  constexpr bool LOAD_RES = EPI == EPI_RESID || EPI == EPI_DGELU || EPI == EPI_MUL_AUX;
  const int M = (int)args.M, N = (int)args.N;
  const int g = lane >> 4;
  OutT* C = (OutT*)args.C;
  const int rbase = m0 + 128 * wm + (lane & 15);
  const int cb0 = n0 + 128 * wn + 16 * (g & 1) + 8 * (g >> 1);
  const bool has_res = LOAD_RES && args.resid != nullptr;
  v4f bias8[4][2];
  {
    const float* bias = args.bias;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = min(cb0 + 32 * p, N - 8);
      bias8[p][0] = bias ? *(const v4f*)(bias + n) : v4f{0.f, 0.f, 0.f, 0.f};
      bias8[p][1] = bias ? *(const v4f*)(bias + n + 4) : v4f{0.f, 0.f, 0.f, 0.f};
    }
  }
  // aux / residual of row fragment i + 1 loaded while fragment i is finished
  v4u ax[2][4];
  v4f rs[2][4][2];
  auto load_row = [&](int i, int buf) {
    const int m = min(rbase + 16 * i, M - 1);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = min(cb0 + 32 * p, N - 8);
      if (LOAD_AUX) ax[buf][p] = *(const v4u*)((const bf16_t*)args.aux + (int64_t)m * args.ldaux + n);
      if (LOAD_RES && has_res) {
        const float* rp = args.resid + (int64_t)m * args.ldr + n;
        rs[buf][p][0] = *(const v4f*)rp;
        rs[buf][p][1] = *(const v4f*)(rp + 4);
      }
    }
  };
  if (LOAD_AUX || LOAD_RES) load_row(0, 0);
  // uniform scalars re-read from the kernel arguments here (s_load): kept live
  // across the K-loop they would sit in spilled VGPRs
  float alpha = args.alpha, beta = args.beta;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(alpha), "+s"(beta));
#endif
  // column sums only for the MLP dgrad (mul-aux) epilogue, their one user:
  // 32 more live VGPRs would push the other epilogues into spills
  constexpr bool CSUM = EPI == EPI_MUL_AUX;
  float csum[4][8];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int r = 0; r < 8; ++r) csum[p][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if ((LOAD_AUX || LOAD_RES) && i + 1 < 8) load_row(i + 1, (i + 1) & 1);
    if ((LOAD_AUX || LOAD_RES) ? i == 6 : i == 0) after_loads();
    __builtin_amdgcn_sched_barrier(0);
    // this row fragment's 32 accumulators only (the rest stay in AGPRs)
    v4f t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = acc[i][j];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(t[2 * p][r]), __float_as_uint(t[2 * p + 1][r]),
                                                   false, false);
        t[2 * p][r] = __uint_as_float(sw[0]);
        t[2 * p + 1][r] = __uint_as_float(sw[1]);
      }
    const int m = rbase + 16 * i;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = cb0 + 32 * p;
      v4f lo = t[2 * p] * alpha + bias8[p][0];
      v4f hi = t[2 * p + 1] * alpha + bias8[p][1];
      if (EPI == EPI_GELU || EPI == EPI_GELU_D) {
        v4f dlo = lo, dhi = hi;
        if (EPI == EPI_GELU_D) {
          dlo = gelu4_inplace(lo);
          dhi = gelu4_inplace(hi);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = gelu_f(lo[r]);
            hi[r] = gelu_f(hi[r]);
          }
        }
        if (args.aux_out && m < M && n < N) {
          v4u pk;
          pk[0] = pack2bf(dlo[0], dlo[1]);
          pk[1] = pack2bf(dlo[2], dlo[3]);
          pk[2] = pack2bf(dhi[0], dhi[1]);
          pk[3] = pack2bf(dhi[2], dhi[3]);
          *(v4u*)((bf16_t*)args.aux_out + (int64_t)m * args.ldaux + n) = pk;
        }
      }
      if (LOAD_AUX) {
        const v4u pk = ax[i & 1][p];
        if (EPI == EPI_MUL_AUX) {
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            lo[2 * r] *= __uint_as_float(pk[r] << 16);
            lo[2 * r + 1] *= __uint_as_float(pk[r] & 0xffff0000u);
            hi[2 * r] *= __uint_as_float(pk[2 + r] << 16);
            hi[2 * r + 1] *= __uint_as_float(pk[2 + r] & 0xffff0000u);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            lo[2 * r] *= gelu_grad_f(__uint_as_float(pk[r] << 16));
            lo[2 * r + 1] *= gelu_grad_f(__uint_as_float(pk[r] & 0xffff0000u));
            hi[2 * r] *= gelu_grad_f(__uint_as_float(pk[2 + r] << 16));
            hi[2 * r + 1] *= gelu_grad_f(__uint_as_float(pk[2 + r] & 0xffff0000u));
          }
        }
      }
      if (LOAD_RES && has_res) {
        lo += rs[i & 1][p][0];
        hi += rs[i & 1][p][1];
      }
      if (m < M && n < N) {
        OutT* cp = C + (int64_t)m * args.ldc + n;
        if (beta != 0.f) {
          lo += beta * ld4<OutT>(cp);
          hi += beta * ld4<OutT>(cp + 4);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (CSUM) {
            csum[p][r] += lo[r];
            csum[p][4 + r] += hi[r];
          }
        }
        if (sizeof(OutT) == 2) {
          v4u pk;
          pk[0] = pack2bf(lo[0], lo[1]);
          pk[1] = pack2bf(lo[2], lo[3]);
          pk[2] = pack2bf(hi[0], hi[1]);
          pk[3] = pack2bf(hi[2], hi[3]);
          *(v4u*)cp = pk;
        } else {
          *(v4f*)cp = lo;
          *(v4f*)((float*)cp + 4) = hi;
        }
      }
    }
    if (CSUM && (i & 3) == 3 && args.colsum_partial) {   // one partial row per 64-row group
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) csum[p][r] = row16_sum(csum[p][r]);
      const int mrow = m0 + 128 * wm + 64 * (i >> 2);
      if ((lane & 15) == 0 && mrow < M) {
        float* prow = args.colsum_partial + (int64_t)(mrow / 64) * N;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int n = cb0 + 32 * p;
          if (n < N) {
            *(v4f*)(prow + n) = v4f{csum[p][0], csum[p][1], csum[p][2], csum[p][3]};
            *(v4f*)(prow + n + 4) = v4f{csum[p][4], csum[p][5], csum[p][6], csum[p][7]};
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) csum[p][r] = 0.f;
    }
  }
}

template <int LA, int LB, typename OutT, int EPI>
__device__ __forceinline__ void gemm5_body(const maeclip_gemm_args& args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int M = (int)args.M, N = (int)args.N, K = (int)args.K;
  const int gm = (M + 255) / 256, gn = (N + 255) / 256, T = gm * gn;
  const int nt = K / 64;
  // persistent XCD-chunked tile order (blocks b and b + 8 share an XCD): XCD
  // x works the contiguous tile range [cbeg, cend), so neighbouring tiles
  // (same A panel) run on one L2
  const int G = gridDim.x, x8 = blockIdx.x % 8, li = blockIdx.x / 8;
  const int nbx = (G - x8 + 7) / 8;
  const int cq = T / 8, cr = T % 8;
  const int cbeg = x8 < cr ? x8 * (cq + 1) : cr * (cq + 1) + (x8 - cr) * cq;
  const int cend = cbeg + cq + (x8 < cr ? 1 : 0);
  const int njobs = cbeg + li < cend ? (cend - (cbeg + li) + nbx - 1) / nbx : 0;
  if (njobs == 0) return;
  const int total = njobs * nt;   // stages of this block (32-bit: 64-bit division would leave VALU)

  auto tile_of = [&](int g, int& m0, int& n0) {
    const int u = cbeg + li + (g / nt) * nbx;
    m0 = (u / gn) * 256;
    n0 = (u % gn) * 256;
  };
  // DMA of stage g (K-tile g % nt of job g / nt) into buffer g & 1
  auto issue_stage = [&](int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int k0 = (g % nt) * 64;
    char* dst = smem + (g & 1) * STAGE;
    const char* A = (const char*)args.A;
    const char* B = (const char*)args.B;
    const rsrc_t ra = LA == LAY_KC ? make_rsrc(A + (int64_t)m0 * args.lda * 2, ((int64_t)M - m0) * args.lda * 2)
                                   : make_rsrc(A + (int64_t)m0 * 2, ((int64_t)K * args.lda - m0) * 2);
    const rsrc_t rb = LB == LAY_KC ? make_rsrc(B + (int64_t)n0 * args.ldb * 2, ((int64_t)N - n0) * args.ldb * 2)
                                   : make_rsrc(B + (int64_t)n0 * 2, ((int64_t)K * args.ldb - n0) * 2);
    const int sa = LA == LAY_KC ? k0 * 2 : (int)(k0 * args.lda * 2);
    const int sb = LB == LAY_KC ? k0 * 2 : (int)(k0 * args.ldb * 2);
    // The swizzled 16-B chunk of a lane does not depend on the instruction
    // index (s, i): one VGPR offset per operand, the rest a scalar delta
    // (dsoff5). Recomputed per stage from an opaque copy of the lane id (a
    // few VALU ops) rather than kept live across the loop nest, where the
    // allocator spills it and the reload would wait behind the DMA in vmcnt.
    int ln = lane;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(ln));
#endif
    const int vA = voff5<LA>(args.lda, 0, wave, ln);
    const int vB = voff5<LB>(args.ldb, 0, wave, ln);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + s * HALF + (4 * i + wave) * 1024), 16, vA,
                                                 sa + dsoff5<LA>(args.lda, s, i), 0, 0);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(dst + (2 + s) * HALF + (4 * i + wave) * 1024), 16, vB,
                                                 sb + dsoff5<LB>(args.ldb, s, i), 0, 0);
  };

  issue_stage(0);
  if (total > 1) issue_stage(1);
  if (total > 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  BARRIER5();

  Frags f0, f1;
  read_frags<LA, LB>(f0, smem, 0, wm, wn, lane);
  // Loop nest tile { acc = 0; K-tiles; epilogue }: the accumulators are born
  // at the top of each tile and die in its epilogue, so the only phi on them
  // is the K-loop's own (a conditional zeroing or a second MFMA site makes a
  // phi the coalescer cannot merge, and the allocator then copies all 256 of
  // them through VGPRs every K-tile).
  int g = 0;
  // stores the previous epilogue left in flight (younger than stage g+1's DMA)
  bool after_epi = false;
  for (int job = 0; job < njobs; ++job) {
    v4f acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    auto ktile = [&](bool last) {
      const char* st = smem + (g & 1) * STAGE;
      read_frags<LA, LB>(f1, st, 1, wm, wn, lane);                   // 1
      mma64(acc, f0);                                                // 2
      // lgkmcnt(0) through the builtin: the compiler's waitcnt pass sees it
      // (16 outstanding reads exceed the 4-bit counter it would otherwise use)
      __builtin_amdgcn_s_waitcnt(0xc07f);                            // 3
      BARRIER5();
      if (!last && g + 2 < total) {                                  // 4
        issue_stage(g + 2);
        // this wave's stage g+1 DMA done: all but the 16 just issued (and the
        // previous epilogue's stores, counted conservatively: vmcnt caps at 63)
        if (after_epi) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      after_epi = false;
      BARRIER5();
      // (the last K-tile of a tile reads the next tile's F0 after the
      // epilogue: 64 fragment VGPRs live across it would spill)
      if (!last) read_frags<LA, LB>(f0, smem + ((g + 1) & 1) * STAGE, 0, wm, wn, lane);   // 5
      mma64(acc, f1);                                                // 6
      __builtin_amdgcn_s_waitcnt(0xc07f);   // F0 landed long ago; keeps the counter exact
      ++g;
    };
    // not peeled: a peeled last K-tile is scheduled into ~150 spills
    for (int kt = 0; kt < nt; ++kt) ktile(kt == nt - 1);
    int m0, n0;
    tile_of(g - 1, m0, n0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    // the last K-tile's stage DMA (g + 1 here), deferred until the epilogue has
    // issued its loads: vmcnt retires in issue order, so a load issued after
    // the DMA would wait for the whole stage
    epilogue5<OutT, EPI>(args, acc, m0, n0, wm, wn, lane, [&] {
      if (g + 1 < total) issue_stage(g + 1);
    });
    // past the last stage this reads stale LDS (never used)
    read_frags<LA, LB>(f0, smem + (g & 1) * STAGE, 0, wm, wn, lane);
    after_epi = true;
  }
}

// thin kernel over a device body (the host pass then instantiates the kernel
// stub; with the body inline in the __global__ template it did not)
template <int LA, int LB, typename OutT, int EPI>
__global__ void __launch_bounds__(NTH5, 1) gemm5_kernel(const maeclip_gemm_args args) {
  gemm5_body<LA, LB, OutT, EPI>(args);
}

int ncu5() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const char* e = getenv("MAECLIP_GEMM_GRID");   // diagnostic grid cap (contention scans)
  const int cap = (e && *e) ? atoi(e) : 0;
  return cap > 0 && cap < ncu ? cap : ncu;
}

template <int LA, int LB, typename OutT, int EPI>
int launch5(const maeclip_gemm_args& a, hipStream_t s) {
  auto kern = gemm5_kernel<LA, LB, OutT, EPI>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS5);
  const int tiles = (int)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  const int ncu = ncu5();
  hipLaunchKernelGGL(kern, dim3(tiles < ncu ? tiles : ncu), dim3(NTH5), LDS5, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(v5)");
  return 0;
}

template <int LA, int LB, typename OutT>
int epi5(const maeclip_gemm_args& a, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_NONE: return launch5<LA, LB, OutT, EPI_NONE>(a, s);
    case EPI_GELU: return launch5<LA, LB, OutT, EPI_GELU>(a, s);
    case EPI_RESID: return launch5<LA, LB, OutT, EPI_RESID>(a, s);
    case EPI_GELU_D: return launch5<LA, LB, OutT, EPI_GELU_D>(a, s);
    case EPI_MUL_AUX: return launch5<LA, LB, OutT, EPI_MUL_AUX>(a, s);
    default: return launch5<LA, LB, OutT, EPI_DGELU>(a, s);
  }
}

template <int LA, int LB>
int out5(const maeclip_gemm_args& a, hipStream_t s) {
  return a.out_dtype == MAECLIP_BF16 ? epi5<LA, LB, bf16_t>(a, s) : epi5<LA, LB, float>(a, s);
}

}  // namespace

namespace maeclip {
// v5 takes plain bf16 launches (no split-K, batch 1) with A K-contiguous
// (forward and dgrad GEMMs) and the v4 epilogue's 16-B access conditions
bool gemm_v5_ok(const maeclip_gemm_args& a) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a.dtype != MAECLIP_BF16 || a.a_layout != LAY_KC || a.splitk > 1 || a.batch != 1) return false;
  if (a.K % 64 != 0 || a.K <= 0 || a.lda % 8 || a.ldb % 8) return false;
  if (a.M < 256 || a.N < 256 || a.N % 8) return false;
  const int64_t lim = 0x7fffffffLL;
  if (a.M * a.lda * 2 >= lim || (a.b_layout == LAY_KC ? a.N * a.ldb : a.K * a.ldb) * 2 >= lim) return false;
  if (!al16(a.C) || (a.out_dtype == MAECLIP_BF16 ? a.ldc % 8 : a.ldc % 4)) return false;
  const bool wa = a.epilogue == EPI_GELU || a.epilogue == EPI_GELU_D;
  const bool ra = a.epilogue == EPI_DGELU || a.epilogue == EPI_MUL_AUX;
  if ((wa && a.aux_out && (!al16(a.aux_out) || a.ldaux % 8)) || (ra && (!al16(a.aux) || a.ldaux % 8))) return false;
  if (a.resid && (!al16(a.resid) || a.ldr % 4)) return false;
  if (a.bias && !al16(a.bias)) return false;
  if (a.colsum_partial && a.epilogue != EPI_MUL_AUX) return false;
  return true;
}

int gemm_v5(const maeclip_gemm_args& a, hipStream_t s) {
  return a.b_layout == LAY_KC ? out5<LAY_KC, LAY_KC>(a, s) : out5<LAY_KC, LAY_RC>(a, s);
}
}  // namespace maeclip
