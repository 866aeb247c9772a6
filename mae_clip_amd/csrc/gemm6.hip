// GEMM v6: 256x256x64 bf16 tile on FOUR waves (2 x 2), each wave owning a
// 128 x 128 output block = 8 x 8 fragments of 16x16 (256 accumulator
// registers, one wave per SIMD), for the long-K forward / dgrad shapes.
//
// Why (profiles/r04/gemm_sq_vs_hipblaslt.jsonl, hipblaslt_kernels_*.txt): the
// 8-wave v4 tile (128 x 64 per wave) reads 192 KiB of LDS fragments per
// K-tile in bursts between ping-pong barriers; its main loop runs at ~3.2k
// cycles per K-tile against a 2.05k MFMA floor, and hipBLASLt's 4-wave
// 128 x 128-per-wave tiles (MIWT8_8) are 1.3x faster at K = 8192. Here a
// wave reads 32 KiB per K-tile (128 KiB per CU) spread one ds_read per four
// MFMAs, and the workgroup meets at ONE barrier per K-tile.
//
// Schedule (stage of K-tile t = (sb + t) & 1, two 64-KiB stages A | B):
//   half 1 of K-tile t : 64 MFMAs on the ks = 0 fragments (registers), while
//                        the ks = 1 fragments of t are read from LDS
//   M(t)               : lgkmcnt(0) (this wave's reads of stage t done) +
//                        vmcnt for DMA(t+1) + s_barrier -- after it the stage
//                        of t is free and DMA(t+1) is visible to every wave
//   after M(t)         : DMA(t+2) into the stage of t (or, at the tile's end,
//                        the next tile's K-tiles 0 and 1 at M(nt-2), M(nt-1))
//   half 2 of K-tile t : 64 MFMAs on the ks = 1 fragments, while the ks = 0
//                        fragments of t+1 are read
// so an LDS-DMA has one K-tile (~2k cycles) to land and every fragment read
// has half a K-tile. Operand images are the v4 ones (KC: 128-byte rows with
// the 16-byte chunk XOR-swizzled by (row >> 1) & 7; RC: two 128-column
// [64 k-rows][256 B] images), filled through buffer descriptors with the
// swizzle applied to the source address.
//
// Epilogue: each 16-row chunk of the wave's block goes through an 8-KiB
// per-wave LDS scratch (the fourth 32 KiB of LDS) in fp32 and comes back in
// row layout (2 rows x 512 B per wave instruction): bias, alpha, the fp32
// residual (RESID) and full-line stores of C. The stores are never waited
// for in the epilogue: the next tile's first two K-tiles were issued before
// them (counted vmcnt at the tile start).
#include "common.h"
#include <stdlib.h>
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

typedef __attribute__((address_space(3))) void lds_void;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int OPB = 256 * 128;               // one operand image of a stage: 256 rows (KC) x 128 B = 32 KiB
constexpr int STAGE = 2 * OPB;                // A | B
constexpr int SCR = 8192;                     // epilogue scratch per wave
constexpr int LDS_ALL = 2 * STAGE + 4 * SCR;  // 160 KiB

__device__ __forceinline__ rsrc_t make_rsrc6(const char* base, int64_t bytes) {
  const int nrec = (int)(bytes < 0x7fffffff ? (bytes > 0 ? bytes : 0) : 0x7fffffff);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);
}
__device__ __forceinline__ int swz_rc6(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

// fragment reads (the v4 images): KC rows of 128 B; RC [64 k-rows][256 B] of 128 columns
__device__ __forceinline__ v8s frag_kc(const char* img, int rs, int ks, int lane) {
  const int row = rs + (lane & 15);
  const int chunk = 4 * ks + (lane >> 4);
  return *(const v8s*)(img + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}
__device__ __forceinline__ v8s frag_rc(const char* img, int rs, int ks, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int unit = (rs >> 2) + p;
  v8s v;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int krow = 32 * ks + 8 * g + 4 * h + q;
    const char* a = img + krow * 256 + ((unit ^ swz_rc6(krow)) << 3);
    v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
    v[4 * h + 0] = t[0];
    v[4 * h + 1] = t[1];
    v[4 * h + 2] = t[2];
    v[4 * h + 3] = t[3];
  }
  return v;
}
template <int LAY>
__device__ __forceinline__ v8s frag6(const char* img, int rs, int ks, int lane) {
  if constexpr (LAY == LAY_KC) return frag_kc(img, rs, ks, lane);
  else return frag_rc(img + (rs >> 7) * 16384, rs & 127, ks, lane);
}

#define V6_BARRIER()                   \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
    asm volatile("" ::: "memory");     \
  } while (0)

// s_waitcnt vmcnt(N) with N a compile-time constant <= 63
template <int N> __device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vector-memory instructions a wave's epilogue issues per tile (fixed: buffer
// descriptors drop / zero out-of-range rows and columns instead of branches)
template <typename OutT, int EPI> constexpr int epi_vm() {
  if (sizeof(OutT) == 4) return 64 + (EPI == EPI_RESID ? 64 : 0) + 2;   // C, residual loads, 2 colsum rows
  return 32 + ((EPI == EPI_GELU || EPI == EPI_GELU_D || EPI == EPI_MUL_AUX) ? 32 : 0) + 4;
}
constexpr int cmin(int a, int b) { return a < b ? a : b; }

// diagnostic builds only (tools/build_variant.sh ... -DV6_NO_MFMA / -DV6_NO_READ):
// drop the MFMAs (operands kept live) or the fragment reads (MFMAs on stale
// registers) to time the DMA / LDS-read / MFMA streams of the main loop apart
#ifdef V6_NO_MFMA
#define V6_MMA(c, x, y) asm volatile("" ::"v"(x), "v"(y))
#else
#define V6_MMA(c, x, y) (c) = __builtin_amdgcn_mfma_f32_16x16x32_bf16((x), (y), (c), 0, 0, 0)
#endif
#ifdef V6_NO_READ
template <typename T> __device__ __forceinline__ v8s v6_keep(T) {
  v8s z;
  asm volatile("" : "=v"(z));
  return z;
}
#define V6_RD(e) v6_keep(0)
#else
#define V6_RD(e) (e)
#endif

// After a 16-byte buffer store, the store may read its data VGPRs late: a
// following VALU write of them needs wait states (cdna_hip_programming.md §5.7
// item 1). hipcc did not pad a v_pk_add_f32 that reused the registers right
// behind a buffer_store_dwordx4 here (tools/gemm6_probe.py: corrupted columns
// 4k+3), so every epilogue store carries its own pad.
#define V6_STORE_PAD()                 \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    asm volatile("s_nop 1");           \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

struct Tile6 {
  int m0, n0;
};

template <int LB, typename OutT, int EPI>
__global__ void __launch_bounds__(256) gemm6_kernel(const maeclip_gemm_args args) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  char* const scr = smem + 2 * STAGE + wave * SCR;
  const int M = (int)args.M, N = (int)args.N, K = (int)args.K;
  const int64_t lda = args.lda, ldb = args.ldb;
  const char* const Ab = (const char*)args.A;
  const char* const Bb = (const char*)args.B;
  const int gn = (N + 255) >> 8, T = ((M + 255) >> 8) * gn, nt = K >> 6;

  // persistent, XCD-chunked tile list (v4): tiles [cbeg, cend) for the
  // blocks with blockIdx.x % 8 == x8, strided by the number of such blocks
  const int G = gridDim.x, x8 = blockIdx.x % 8, li = blockIdx.x / 8;
  const int nbx = (G - x8 + 7) / 8;
  const int cq = T / 8, cr = T % 8;
  const int cbeg = x8 < cr ? x8 * (cq + 1) : cr * (cq + 1) + (x8 - cr) * cq;
  const int cend = cbeg + cq + (x8 < cr ? 1 : 0);
  auto tile = [&](int u) { return Tile6{((cbeg + li + u * nbx) / gn) * 256, ((cbeg + li + u * nbx) % gn) * 256}; };
  const int ntiles = cbeg + li < cend ? (cend - (cbeg + li) + nbx - 1) / nbx : 0;
  if (ntiles == 0) return;

  // per-lane DMA byte offsets: A KC rows 8q.. (q = wave + 4i); B KC likewise,
  // B RC: image i >> 2, k-rows 4qq.. (qq = 4 (i & 3) + wave). The swizzle term
  // does not depend on i (rows / k-rows of instruction i are those of
  // instruction 0 shifted by a multiple of 16), so one VGPR per operand plus a
  // uniform per-instruction offset (V6_OA(i), V6_OB(i): SGPR soffset) cover all 8.
  int vA0, vB0;
  {
    const int r = 8 * wave + (lane >> 3), p = lane & 7;
    vA0 = (int)(r * lda * 2) + ((p ^ ((r >> 1) & 7)) << 4);
    if constexpr (LB == LAY_KC) {
      vB0 = (int)(r * ldb * 2) + ((p ^ ((r >> 1) & 7)) << 4);
    } else {
      const int kr = 4 * wave + (lane >> 4);
      const int c = (lane & 15) ^ (swz_rc6(kr) >> 1);
      vB0 = (int)(kr * ldb * 2) + 8 * c * 2;
    }
  }
  // (plain expressions: a lambda call inside these builtins' arguments made the
  // host pass drop the kernel stubs without a diagnostic, ROCm 7.2)
  const int sA = (int)(64 * lda), sB = LB == LAY_KC ? (int)(64 * ldb) : (int)(32 * ldb);
#define V6_OA(i) ((i) * sA)
#define V6_OB(i) (LB == LAY_KC ? (i) * sB : ((i) & 3) * sB + ((i) >> 2) * 256)
  auto dma = [&](const Tile6& tl, int t, int st) {
    char* sa = smem + st * STAGE;
    char* sbp = sa + OPB;
    const rsrc_t ra = make_rsrc6(Ab + (int64_t)tl.m0 * lda * 2, ((int64_t)M - tl.m0) * lda * 2);
    const int k0 = t * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(sa + (wave + 4 * i) * 1024), 16, vA0, k0 * 2 + V6_OA(i), 0, 0);
    if constexpr (LB == LAY_KC) {
      const rsrc_t rb = make_rsrc6(Bb + (int64_t)tl.n0 * ldb * 2, ((int64_t)N - tl.n0) * ldb * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sbp + (wave + 4 * i) * 1024), 16, vB0, k0 * 2 + V6_OB(i), 0, 0);
    } else {
      const rsrc_t rb = make_rsrc6(Bb + (int64_t)tl.n0 * 2, ((int64_t)K * ldb - tl.n0) * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(sbp + (i >> 2) * 16384 + (4 * (i & 3) + wave) * 1024),
                                                 16, vB0, (int)(k0 * ldb * 2) + V6_OB(i), 0, 0);
    }
  };

#ifdef V6_REG
  // register-staged variant (diagnostic build, -DV6_REG): item g = K-tile
  // g % nt of the block's tile g / nt goes global -> 64 VGPRs -> ds_write into
  // stage g & 1, the same lane-linear images the LDS-DMA writes. Items past the
  // block's last tile read zeros through an empty descriptor.
  v4u rA[8], rB[8];
  auto gload = [&](int g) {
    const int uu = g / nt, t = g - uu * nt;
    const Tile6 tl = tile(uu);
    const bool live = uu < ntiles;
    const rsrc_t ra = make_rsrc6(Ab + (int64_t)tl.m0 * lda * 2, live ? ((int64_t)M - tl.m0) * lda * 2 : 0);
    const int k0 = t * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) rA[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, vA0, k0 * 2 + V6_OA(i), 0);
    if constexpr (LB == LAY_KC) {
      const rsrc_t rb = make_rsrc6(Bb + (int64_t)tl.n0 * ldb * 2, live ? ((int64_t)N - tl.n0) * ldb * 2 : 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) rB[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, vB0, k0 * 2 + V6_OB(i), 0);
    } else {
      const rsrc_t rb = make_rsrc6(Bb + (int64_t)tl.n0 * 2, live ? ((int64_t)K * ldb - tl.n0) * 2 : 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) rB[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, vB0, (int)(k0 * ldb * 2) + V6_OB(i), 0);
    }
  };
  auto swrite = [&](int st) {
    char* sa = smem + st * STAGE;
    char* sbp = sa + OPB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      *(v4u*)(sa + (wave + 4 * i) * 1024 + lane * 16) = rA[i];
      if constexpr (LB == LAY_KC) *(v4u*)(sbp + (wave + 4 * i) * 1024 + lane * 16) = rB[i];
      else *(v4u*)(sbp + (i >> 2) * 16384 + (4 * (i & 3) + wave) * 1024 + lane * 16) = rB[i];
    }
  };
#endif
  const int64_t ldc = args.ldc;
  const float alpha = args.alpha;
  int sb = 0;
  Tile6 cur = tile(0);
#ifdef V6_REG
  gload(0);
  swrite(0);
  gload(1);
  swrite(1);
  gload(2);
#else
  dma(cur, 0, 0);
  dma(cur, 1, 1);
#endif
  bool stores_pending = false;

  for (int u = 0; u < ntiles; ++u) {
    const bool has_next = u + 1 < ntiles;
    const Tile6 nxt = has_next ? tile(u + 1) : cur;
    // DMA(0) of this tile landed (DMA(1) and the last tile's epilogue may be in flight)
    constexpr int EV = epi_vm<OutT, EPI>();
#ifdef V6_REG
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
    if (stores_pending) wait_vm<cmin(63, 16 + EV)>();
    else wait_vm<16>();
#endif
    V6_BARRIER();

    v4f acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    v8s fa0[8], fb0[8], fa1[8], fb1[8];
    {
      const char* sa = smem + sb * STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        fa0[i] = frag_kc(sa, 128 * wr + 16 * i, 0, lane);
        fb0[i] = frag6<LB>(sa + OPB, 128 * wc + 16 * i, 0, lane);
      }
    }
    for (int t = 0; t < nt; ++t) {
      const int st = (sb + t) & 1;
      const char* sa = smem + st * STAGE;
      // ---- half 1: ks = 0 MFMAs; ks = 1 fragments of t. Eight groups of 8
      // MFMAs, each followed by two fragment reads (B fragments first: row i = 0
      // of the next half needs all eight of them); sched_barrier pins the order
      // so the compiler neither hoists the reads nor waits for them early.
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) V6_MMA(acc[i][j], fb0[j], fa0[i]);
        if (i < 4) {
          fb1[2 * i] = V6_RD(frag6<LB>(sa + OPB, 128 * wc + 32 * i, 1, lane));
          fb1[2 * i + 1] = V6_RD(frag6<LB>(sa + OPB, 128 * wc + 32 * i + 16, 1, lane));
        } else {
          fa1[2 * i - 8] = V6_RD(frag_kc(sa, 128 * wr + 32 * (i - 4), 1, lane));
          fa1[2 * i - 7] = V6_RD(frag_kc(sa, 128 * wr + 32 * (i - 4) + 16, 1, lane));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- M(t)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef V6_REG
      V6_BARRIER();
      swrite(st);                      // item g + 2, loaded one K-tile ago
      __builtin_amdgcn_sched_barrier(0);
      gload(u * nt + t + 3);
#else
      if (t + 1 < nt) {
        if (t == 0 && stores_pending) wait_vm<cmin(63, EV)>();   // DMA(1) is older than the last tile's epilogue
        else wait_vm<0>();
      }
      V6_BARRIER();
      if (t + 2 < nt) {
        dma(cur, t + 2, st);
      } else if (has_next) {
        // the next tile's K-tile 0 (at M(nt-2)) / 1 (at M(nt-1)) into the stage just freed
        dma(nxt, t + 2 - nt, st);
      }
#endif
      // ---- half 2: ks = 1 MFMAs; ks = 0 fragments of t + 1 (read even in the
      // last K-tile: the values are dead, the stage holds the next tile's data)
      const char* sn = smem + (st ^ 1) * STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) V6_MMA(acc[i][j], fb1[j], fa1[i]);
        if (i < 4) {
          fb0[2 * i] = V6_RD(frag6<LB>(sn + OPB, 128 * wc + 32 * i, 0, lane));
          fb0[2 * i + 1] = V6_RD(frag6<LB>(sn + OPB, 128 * wc + 32 * i + 16, 0, lane));
        } else {
          fa0[2 * i - 8] = V6_RD(frag_kc(sn, 128 * wr + 32 * (i - 4), 0, lane));
          fa0[2 * i - 7] = V6_RD(frag_kc(sn, 128 * wr + 32 * (i - 4) + 16, 0, lane));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    sb = (sb + nt) & 1;

    // ---- epilogue: 16-row chunks through the fp32 scratch (16-B unit u of row r
    // at u ^ r), read back in row layout; loads / stores through buffer
    // descriptors (rows >= M and columns >= N fall outside the range and read 0 /
    // are dropped), so every wave issues the same number of vector-memory
    // instructions per tile (EPI_VM) and the counted waits above stay exact
    const int mb = cur.m0 + 128 * wr, nb = cur.n0 + 128 * wc;
    constexpr int ES = sizeof(OutT);
    // per-lane offset (one VGPR; huge for columns >= N so the access falls
    // outside the descriptor) + per-instruction uniform row offset (SGPR soffset)
    auto rs_i = [&](const void* base, int64_t ld, int esz, int i) {   // rows mb + 16 i .. of a row-major operand
      return make_rsrc6(base ? (const char*)base + (int64_t)(mb + 16 * i) * ld * esz : nullptr,
                        base ? ((int64_t)M - mb - 16 * i) * ld * esz : 0);
    };
    const bool want_cs = args.colsum_partial != nullptr;
    // colsum partial row (one per 64-row group) of group h of the wave's 128 rows
    auto cs_rsrc = [&](int h) {
      const int mrow = mb + 64 * h;
      return make_rsrc6(want_cs && mrow < M ? (const char*)(args.colsum_partial + (int64_t)(mrow / 64) * N) : nullptr,
                        want_cs && mrow < M ? (int64_t)N * 4 : 0);
    };
    if constexpr (ES == 4) {
      // fp32: 8 instructions per chunk, lane -> row 2q + (lane >> 5), columns 4 (lane & 31) ..
      const int rr = lane >> 5, c = lane & 31;
      const int n = nb + 4 * c;
      const bool nok = n < N;                              // N % 8 == 0
      const v4f bias = (args.bias && nok) ? *(const v4f*)(args.bias + n) : v4f{0.f, 0.f, 0.f, 0.f};
      const int vo = nok ? (rr * (int)ldc + n) * 4 : 0x7ffffff0;
      const int ldr = (int)args.ldr;
      const int vr = nok ? (rr * ldr + n) * 4 : 0x7ffffff0;
      v4f rs[2][8];
      auto load_res = [&](int i, int b) {
        const rsrc_t rres = rs_i(EPI == EPI_RESID ? args.resid : nullptr, ldr, 4, i);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          rs[b][q] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rres, vr, 2 * q * ldr * 4, 2));
      };
      if constexpr (EPI == EPI_RESID) load_res(0, 0);
      v4f csum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const rsrc_t rci = rs_i(args.C, ldc, 4, i);
        if constexpr (EPI == EPI_RESID) {
          if (i + 1 < 8) load_res(i + 1, (i + 1) & 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = lane & 15, u = 4 * j + (lane >> 4);
          *(v4f*)(scr + row * 512 + ((u ^ row) << 4)) = acc[i][j];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int row = 2 * q + rr;
          v4f x = *(const v4f*)(scr + row * 512 + ((c ^ row) << 4));
          x = x * alpha + bias;
          if constexpr (EPI == EPI_RESID) x += rs[i & 1][q];
          if (mb + 16 * i + row < M) csum += x;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, x), rci, vo, 2 * q * (int)ldc * 4, 2);
          V6_STORE_PAD();
        }
        if ((i & 3) == 3) {   // 64-row group done: lanes c and c + 32 hold the same columns
          v4f t;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(csum[e]), __float_as_uint(csum[e]), false, false);
            t[e] = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, t), cs_rsrc(i >> 2),
                                                 (lane < 32 && nok) ? n * 4 : 0x7ffffff0, 0, 0);
          V6_STORE_PAD();
          csum = v4f{0.f, 0.f, 0.f, 0.f};
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // bf16: 4 instructions per chunk, lane -> row 4q + (lane >> 4), columns 8 (lane & 15) ..
      constexpr bool GEL = EPI == EPI_GELU || EPI == EPI_GELU_D;
      const int rr = lane >> 4, c = lane & 15;
      const int n = nb + 8 * c;
      const bool nok = n < N;
      v4f b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
      if (args.bias && nok) {
        b0 = *(const v4f*)(args.bias + n);
        b1 = *(const v4f*)(args.bias + n + 4);
      }
      const int vo = nok ? (rr * (int)ldc + n) * 2 : 0x7ffffff0;
      const int ldx = (int)args.ldaux;
      const int vx = nok ? (rr * ldx + n) * 2 : 0x7ffffff0;
      v4u ax[2][4];
      auto load_aux = [&](int i, int b) {
        const rsrc_t ra = rs_i(args.aux, ldx, 2, i);
#pragma unroll
        for (int q = 0; q < 4; ++q) ax[b][q] = __builtin_amdgcn_raw_buffer_load_b128(ra, vx, 4 * q * ldx * 2, 2);
      };
      if constexpr (EPI == EPI_MUL_AUX) load_aux(0, 0);
      float csum[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const rsrc_t rci = rs_i(args.C, ldc, 2, i);
        const rsrc_t rao = rs_i(GEL ? args.aux_out : nullptr, ldx, 2, i);
        if constexpr (EPI == EPI_MUL_AUX) {
          if (i + 1 < 8) load_aux(i + 1, (i + 1) & 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = lane & 15, u = 4 * j + (lane >> 4);
          *(v4f*)(scr + row * 512 + ((u ^ row) << 4)) = acc[i][j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 4 * q + rr;
          const v4f x0 = *(const v4f*)(scr + row * 512 + (((2 * c) ^ row) << 4));
          const v4f x1 = *(const v4f*)(scr + row * 512 + (((2 * c + 1) ^ row) << 4));
          float x[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            x[e] = fmaf(x0[e], alpha, b0[e]);
            x[4 + e] = fmaf(x1[e], alpha, b1[e]);
          }
          if constexpr (GEL) {
            float d[8];   // GELU: aux_out <- pre-activation; GELU_D: aux_out <- gelu'(pre)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float y, dy;
              gelu_pair(x[e], y, dy);
              d[e] = EPI == EPI_GELU_D ? dy : x[e];
              x[e] = y;
            }
            const v4u pd = {pack2bf(d[0], d[1]), pack2bf(d[2], d[3]), pack2bf(d[4], d[5]), pack2bf(d[6], d[7])};
            __builtin_amdgcn_raw_buffer_store_b128(pd, rao, vx, 4 * q * ldx * 2, 2);
          V6_STORE_PAD();
          }
          if constexpr (EPI == EPI_MUL_AUX) {
            const v4u a = ax[i & 1][q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              x[2 * e] *= __uint_as_float(a[e] << 16);
              x[2 * e + 1] *= __uint_as_float(a[e] & 0xffff0000u);
            }
          }
          if (mb + 16 * i + row < M) {
#pragma unroll
            for (int e = 0; e < 8; ++e) csum[e] += x[e];
          }
          const v4u pk = {pack2bf(x[0], x[1]), pack2bf(x[2], x[3]), pack2bf(x[4], x[5]), pack2bf(x[6], x[7])};
          __builtin_amdgcn_raw_buffer_store_b128(pk, rci, vo, 4 * q * (int)ldc * 2, 2);
          V6_STORE_PAD();
        }
        if ((i & 3) == 3) {   // 64-row group done: lanes c + 16 k hold the same columns
          float t[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(csum[e]), __float_as_uint(csum[e]), false, false);
            const float u = __uint_as_float(p[0]) + __uint_as_float(p[1]);
            const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(u), __float_as_uint(u), false, false);
            t[e] = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
            csum[e] = 0.f;
          }
          const rsrc_t rcs = cs_rsrc(i >> 2);
          const int vcs = (lane < 16 && nok) ? n * 4 : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{t[0], t[1], t[2], t[3]}), rcs, vcs, 0, 0);
          V6_STORE_PAD();
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{t[4], t[5], t[6], t[7]}), rcs, vcs, 16, 0);
          V6_STORE_PAD();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stores_pending = true;
    cur = nxt;
  }
}

}  // namespace

namespace maeclip {

// v6 shapes: bf16 A (KC) and B (KC or RC), K % 64 == 0 and K >= 128, fp32 /
// bf16 C (GELU / GELU_D / MUL_AUX: bf16), no split-K / batch / beta;
// MAECLIP_GEMM_V6=1 turns it on (A/B against v4 until it is the measured default)
bool gemm_v6_ok(const maeclip_gemm_args& a) {
  static const int on = getenv("MAECLIP_GEMM_V6") ? atoi(getenv("MAECLIP_GEMM_V6")) : 0;
  if (!on) return false;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a.dtype != MAECLIP_BF16 || a.a_layout != LAY_KC || a.K % 64 != 0 || a.K < 128) return false;
  const int e = a.epilogue;
  if (e == EPI_DGELU) return false;
  if ((e == EPI_GELU || e == EPI_GELU_D || e == EPI_MUL_AUX) && a.out_dtype != MAECLIP_BF16) return false;
  if (a.splitk > 1 || a.batch != 1 || a.beta != 0.f) return false;
  if (a.M < 256 || a.N < 256 || a.N % 8 || a.lda % 8 || a.ldb % 8) return false;
  if (!al16(a.A) || !al16(a.B) || !al16(a.C) || (a.bias && !al16(a.bias))) return false;
  if (a.out_dtype == MAECLIP_BF16 ? a.ldc % 8 : a.ldc % 4) return false;
  if (a.resid && (!al16(a.resid) || a.ldr % 4)) return false;
  if ((e == EPI_MUL_AUX && (!al16(a.aux) || a.ldaux % 8)) ||
      ((e == EPI_GELU || e == EPI_GELU_D) && a.aux_out && (!al16(a.aux_out) || a.ldaux % 8)))
    return false;
  if (a.colsum_partial && !al16(a.colsum_partial)) return false;
  const int64_t lim = 0x7fffffffLL;
  if (a.M * a.lda * 2 >= lim || a.M * a.ldc * 4 >= lim || (a.resid && a.M * a.ldr * 4 >= lim) ||
      (a.ldaux && a.M * a.ldaux * 2 >= lim))
    return false;
  if ((a.b_layout == LAY_KC ? a.N * a.ldb : a.K * a.ldb) * 2 >= lim) return false;
  return true;
}

template <int LB, typename OutT, int EPI>
static int launch6(const maeclip_gemm_args& a, hipStream_t s) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  auto kern = gemm6_kernel<LB, OutT, EPI>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_ALL);
  const int tiles = (int)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  hipLaunchKernelGGL(kern, dim3(tiles < ncu ? tiles : ncu), dim3(256), LDS_ALL, s, a);
  MC_CHECK_LAUNCH("maeclip_gemm(v6)");
  return 0;
}

template <int LB>
static int gemm_v6_lb(const maeclip_gemm_args& a, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_RESID: return launch6<LB, float, EPI_RESID>(a, s);
    case EPI_GELU: return launch6<LB, bf16_t, EPI_GELU>(a, s);
    case EPI_GELU_D: return launch6<LB, bf16_t, EPI_GELU_D>(a, s);
    case EPI_MUL_AUX: return launch6<LB, bf16_t, EPI_MUL_AUX>(a, s);
    default:
      return a.out_dtype == MAECLIP_F32 ? launch6<LB, float, EPI_NONE>(a, s) : launch6<LB, bf16_t, EPI_NONE>(a, s);
  }
}

int gemm_v6(const maeclip_gemm_args& a, hipStream_t s) {
  return a.b_layout == LAY_RC ? gemm_v6_lb<LAY_RC>(a, s) : gemm_v6_lb<LAY_KC>(a, s);
}

}  // namespace maeclip
