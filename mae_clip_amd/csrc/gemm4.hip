// GEMM v4: 256x256x64 bf16 tile, 8 waves in two ping-pong groups, LDS-DMA
// prefetch kept in flight across raw barriers (the 256² 8-phase structure of
// cdna_hip_programming.md §5, restated for this library's operand layouts and
// epilogues).
//
// Geometry: waves (wm, wn) = 2 x 4, each wave owns a 128 x 64 output block as
// 8 x 4 fragments of 16x16 (acc = 128 VGPRs). A K-tile is split into four
// 16-KiB "halves" so that each half's last LDS read lands at a different phase:
//   Am0 = A rows {0-63, 128-191}  (mi = 0 sub-rows of both wave rows)
//   Am1 = A rows {64-127, 192-255}
//   Bn0 = B cols {0-31, 64-95, 128-159, 192-223} (ni = 0 sub-cols of all wn)
//   Bn1 = the other 128 columns
// Per K-tile every wave runs four phases, each one 64x32 output quadrant x K 64
// = 16 MFMA 16x16x32:
//   p0 (mi0,ni0): read A-sub0 + B-sub0     p1 (mi0,ni1): read B-sub1
//   p2 (mi1,ni1): read A-sub1              p3 (mi1,ni0): B-sub0 still in VGPRs
// so the last LDS reads are Am0,Bn0 @p0, Bn1 @p1, Am1 @p2.
// DMA schedule (2 glds per wave per phase = one half):
//   p0 of tile t issues half Am1 of tile t+1;  p1,p2,p3 issue Am0,Bn0,Bn1 of
//   tile t+2 into the buffer tile t is still being read -- each one phase after
//   that half's last read (the reads are retired by lgkmcnt(0) before the
//   barrier that ends the reading segment).
//   p3 waits vmcnt(6): everything but the three youngest halves (tile t+2's)
//   has landed, i.e. all of tile t+1, before the barrier that precedes its
//   first read.
// Ping-pong: group 1 (wm == 1) executes one extra barrier up front, so in every
// barrier-delimited segment one group issues its ds_reads/DMA while the other
// group's 16 MFMAs run (one wave of each group per SIMD).
#include "common.h"
#include <stdlib.h>
#include "../../include/maeclip.h"

namespace maeclip {
int check_q8(const maeclip_gemm_args& a, const char* who);
}

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_DGELU = 3, EPI_GELU_D = 4, EPI_MUL_AUX = 5 };

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int swz_rc(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

#ifndef GEMM4_EPI_PF_AUX
#define GEMM4_EPI_PF_AUX 2
#endif
#ifndef GEMM4_EPI_PF
#define GEMM4_EPI_PF 2
#endif

#ifdef GEMM4_STAMPS
__device__ uint64_t g_stamps[256 * 8 * 2 * 4];
#endif

constexpr int HALF = 16384;          // bytes per half image (128 rows/cols x 64 k x bf16)
// BM = 192 (plain launches, KC A operand): 96-row A halves (12 KiB), waves own
// 96 x 64 output blocks (3 x 4 fragments per quadrant row), 6 row fragments;
// chosen when it needs fewer full-tile rounds of the grid (encoder N = 768
// shapes: 201 tiles of 192 x 256 instead of 150 of 256 x 256 on 256 CUs)
template <int BM> struct TileM {
  static constexpr int MI = BM / 64;                 // A fragments per wave per half
  static constexpr int HALF_A = BM / 2 * 128;        // bytes per A half image
  static constexpr int BUF_T = 2 * HALF_A + 2 * HALF;
  static constexpr int LDS_T = 2 * BUF_T;                      // operand stages
  // BM = 192: fp8-blocks A scales, one 1 KiB image per K-tile stage (the 3
  // 64-row groups of the tile + a dummy slot, 256 B each)
  static constexpr int SC_T = BM == 192 ? 2048 : 0;
  static constexpr int SCR_OFF = LDS_T + SC_T;
  static constexpr int LDS_ALL = SCR_OFF + 8 * 4096;             // + epilogue scratch (8 waves x 4 KiB)
  __device__ static __forceinline__ int hoff(int h) { return h < 2 ? h * HALF_A : 2 * HALF_A + (h - 2) * HALF; }
};

// local index l (0..127) of a half -> offset inside the 256-wide block tile
// (BM = 192: local row l of a 96-row half; BM = 128: of a 64-row half; the
// wave row group wm owns rows [BM/2 wm, BM/2 (wm + 1)), half `sub` its
// sub-rows BM/4 sub .. +BM/4)
template <int BM = 256>
__device__ __forceinline__ int amap(int l, int sub) {
  if constexpr (BM == 256) return (l & 63) + ((l >> 6) << 7) + (sub << 6);
  else return (l % (BM / 4)) + (l / (BM / 4)) * (BM / 2) + sub * (BM / 4);
}
__device__ __forceinline__ int bmap(int l, int sub) { return (l & 31) + ((l >> 5) << 6) + (sub << 5); }

// Operand DMA through buffer descriptors (buffer_load_dwordx4 ... lds): the
// tile base and extent live in SGPRs, the per-lane byte offsets of the two
// wave-instructions this wave issues per half are loop invariants (8 VGPRs for
// both operands), and the K-tile advance is the scalar soffset. Rows (KC) past
// the operand's end read as zero through the descriptor's range check, so no
// clamping is needed; RC columns past N read neighbouring (finite) data whose
// results are never stored.
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const char* base, int64_t bytes) {
  const int nrec = (int)(bytes < 0x7fffffff ? (bytes > 0 ? bytes : 0) : 0x7fffffff);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nrec, 0x00020000);
}

// per-lane byte offset of wave-instruction i (0, 1) of half `sub` (0, 1) of an operand
template <int LAY, bool ISA, int ESZ = 2, int BM = 256>
__device__ __forceinline__ int half_voffset(int64_t ld, int sub, int i, int wave, int lane) {
  const int q = i * 8 + wave;
  if (LAY == LAY_KC) {
    const int r = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int g = ISA ? amap<BM>(r, sub) : bmap(r, sub);
    return (int)(g * ld * ESZ) + c * 16;
  } else {
    const int kr = q * 4 + (lane >> 4);
    const int c = (lane & 15) ^ (swz_rc(kr) >> 1);
    const int g = ISA ? amap(c * 8, sub) : bmap(c * 8, sub);
    return (int)(kr * ld * 2) + g * 2;
  }
}

// One half = 16 wave-instructions of 1 KiB; this wave issues 2 of them.
__device__ __forceinline__ void issue_half(rsrc_t rs, int v0, int v1, int soff, char* lds, int wave) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + wave * 1024), 16, v0, soff, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + (8 + wave) * 1024), 16, v1, soff, 0, 0);
}

template <int LAY>
__device__ __forceinline__ v8s frag(const char* lds, int rs, int ks, int lane) {
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

// p1 / p2 reads (Bn1, Am1) are restaged two phases after they are read, so
// they need not be retired before the barrier that ends their segment
// (cdna_hip_programming.md §5, 256^2 template, WAR rule); GEMM4_LATE_LGKM
// leaves their wait to the compiler's, right before the first MFMA that uses
// them, so the read latency overlaps the barrier. p0's reads (Am0, restaged
// one phase later) keep the early wait.
#ifdef GEMM4_LATE_LGKM
#define LGKM_EARLY() do {} while (0)
#else
#define LGKM_EARLY() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#endif

#define SEG_BARRIER()                        \
  do {                                       \
    asm volatile("" ::: "memory");           \
    __builtin_amdgcn_sched_barrier(0);       \
    __builtin_amdgcn_s_barrier();            \
    __builtin_amdgcn_sched_barrier(0);       \
    asm volatile("" ::: "memory");           \
  } while (0)

// The 16 MFMAs of one quadrant: rows i0.. of acc (4 A fragments), columns j0..
// (2 B fragments). Each operand fragment is two 16-B LDS chunks of a row (k
// chunks g and 4 + g of the 128-byte K-tile row). bf16: two 16x16x32 MFMAs
// (ks = 0, 1). fp8 (F8 = 1: A e4m3, F8 = 2: A e5m2; B e4m3): the same 32 bytes
// are one 16x16x128 block-scaled MFMA operand (all block scales 2^0; the
// per-row / per-column dequantisation scales are applied in the epilogue). A
// and B fragments put identical k's at identical lane/byte positions, so the
// hardware's k order inside the 128 need not be known.
__device__ __forceinline__ v8i cat_frag(v8s a, v8s b) {
  const v4i x = __builtin_bit_cast(v4i, a), y = __builtin_bit_cast(v4i, b);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}
// Keep a quadrant's MFMAs inside their segment: an empty asm that reads and
// writes the quadrant's accumulators cannot be reordered with the asm barrier
// that follows, so every MFMA of the cluster is emitted before it. Without
// it hipcc (ROCm 7.2) moved 10 of the 16 MFMAs of p0 and of p1 past the
// segment's closing s_barrier into the next read segment (tools/isa_gemm4.sh
// + the per-segment MFMA count), undoing the ping-pong (GEMM4_NO_PIN restores
// that schedule for A/B). Measured (profiles/r05/gemm_pin_ab_r5n.txt): every
// plain shape 1.02-1.17x (4096^3 1109 -> 1292 TF/s), the C2 step 9963 ->
// 10221 img/s. In the grouped weight-gradient body GEMM4_PIN_GRP is a bit
// mask of the phases p0..p3 pinned: all four make its RC x RC fragment
// addresses spill inside the K loop (2790 instead of 2450 us per launch);
// p0 + p1 (the two clusters the compiler split) alone keep every cluster
// whole with the unpinned body's spills (one scratch reload per K-tile):
// step 10150 -> 10254 img/s on one box (profiles/r05/step_pinmask_ab_r5p.txt).
#ifndef GEMM4_PIN_GRP
#define GEMM4_PIN_GRP 3
#endif
template <int MI>
__device__ __forceinline__ void pin_quad(v4f (&acc)[2 * MI][4], int i0, int j0) {
#ifndef GEMM4_NO_PIN
#pragma unroll
  for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(acc[i0 + i][j0]), "+v"(acc[i0 + i][j0 + 1]));
#endif
}

// F8 = 3 / 4 (fp8-blocks A, e4m3 / e5m2): the A fragment i of the half takes
// its e8m0 block scale from byte i of `sc` (the MFMA's scale byte select), B's
// scale is 2^0 (its per-column scale is applied in the epilogue). Measured
// operand layout of the 16x16x128 form (tools/mfma_scale_probe.py,
// profiles/r06/mfma_scale_probe.json): lane group g holds K [16 g, 16 g + 16)
// in its first four VGPRs and K [64 + 16 g, ...) in the last four -- the two
// 16-B chunks g and 4 + g of the K-tile row that frag() reads -- and the scale
// of lane l applies to row l % 16 and K-block l / 16 = K [32 (l / 16), +32):
// a K-block's 32 elements sit in two lane groups, its scale in a third lane's
// VGPR, which is what the scale tensor's layout hands each lane.
template <int AF, int I>
__device__ __forceinline__ v4f mfma_blk(v8i b, v8i a, v4f c, unsigned sc) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, 0, AF, 0, 127, I, (int)sc);
}
template <int F8, int MI>
__device__ __forceinline__ void quad_mma(v4f (&acc)[2 * MI][4], int i0, int j0, const v8s (&fbq)[2][2],
                                         const v8s (&fa)[MI][2], unsigned sc = 0) {
  if constexpr (F8 >= 3) {
    constexpr int AF = F8 == 4 ? 1 : 0;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const v8i a8 = cat_frag(fa[i][0], fa[i][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const v8i b8 = cat_frag(fbq[j][0], fbq[j][1]);
        v4f& c = acc[i0 + i][j0 + j];
        switch (i) {
          case 0: c = mfma_blk<AF, 0>(b8, a8, c, sc); break;
          case 1: c = mfma_blk<AF, 1>(b8, a8, c, sc); break;
          case 2: c = mfma_blk<AF, 2>(b8, a8, c, sc); break;
          default: c = mfma_blk<AF, 3>(b8, a8, c, sc); break;
        }
      }
    }
  } else if constexpr (F8 == 0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbq[j][ks], fa[i][ks], acc[i0 + i][j0 + j], 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const v8i a8 = cat_frag(fa[i][0], fa[i][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            cat_frag(fbq[j][0], fbq[j][1]), a8, acc[i0 + i][j0 + j], 0, F8 == 2 ? 1 : 0, 0, 127, 0, 127);
    }
  }
}

// Epilogue. Fragment (i, j) of the wave covers rows m0 + 128 wm + 64 (i>>2) +
// 16 (i&3) and columns n0 + 64 wn + 32 (j>>1) + 16 (j&1); the MFMA leaves lane
// l with C[row l&15][4 (l>>4) .. +3] of each fragment. A permlane16 swap of the
// column pair (2 ni, 2 ni + 1) hands every lane 8 CONSECUTIVE columns of one
// fragment (lane group g: fragment g&1, columns 8 (g>>1) .. +7), so a row
// segment is one 16-B access per lane (bf16) instead of two 8-B ones
// (cdna_hip_programming.md T21).
//
// vmcnt is in-order on CDNA: a load issued after a store can only be waited
// for together with that store. So every load (bias, aux, resid) of a chunk of
// two row fragments is issued BEFORE the stores of the previous chunk, and the
// stores themselves are never waited for here (they drain behind the next
// tile's main loop, see the counted wait at the tile start).
template <int NI8 = 8>
__device__ __forceinline__ void swap_pairs(v4f (&acc)[NI8][4]) {
#pragma unroll
  for (int i = 0; i < NI8; ++i)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * ni][r]),
                                                  __float_as_uint(acc[i][2 * ni + 1][r]), false, false);
        acc[i][2 * ni][r] = __uint_as_float(p[0]);
        acc[i][2 * ni + 1][r] = __uint_as_float(p[1]);
      }
}

// split-K slab: fp32 partial of this K slice (dense [M, N]), no epilogue
__device__ __forceinline__ void epilogue4_slab(float* __restrict__ slab, int M, int N, float alpha, v4f (&acc)[8][4],
                                               int m0, int n0, int wm, int wn, int lane) {
  const int g = lane >> 4;
  swap_pairs(acc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + 128 * wm + 64 * (i >> 2) + 16 * (i & 3) + (lane & 15);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int n = n0 + 64 * wn + 32 * ni + 16 * (g & 1) + 8 * (g >> 1);
      if (m < M && n < N) {
        float* d = slab + (int64_t)m * N + n;
        *(v4f*)d = acc[i][2 * ni] * alpha;
        *(v4f*)(d + 4) = acc[i][2 * ni + 1] * alpha;
      }
    }
  }
}

// whole 256x256 fp32 tile (stream-K partial) into a dense slot [256][256]
__device__ __forceinline__ void epilogue4_tile(float* __restrict__ t, v4f (&acc)[8][4], int wm, int wn, int lane) {
  const int g = lane >> 4;
  swap_pairs(acc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ml = 128 * wm + 64 * (i >> 2) + 16 * (i & 3) + (lane & 15);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      float* d = t + ml * 256 + 64 * wn + 32 * ni + 16 * (g & 1) + 8 * (g >> 1);
      *(v4f*)d = acc[i][2 * ni];
      *(v4f*)(d + 4) = acc[i][2 * ni + 1];
    }
  }
}

// Epilogue in full-line row layout. The MFMA fragments (16 rows x 16 columns,
// 4 consecutive columns per lane) would be stored / loaded as 16 rows x 64 B
// per wave-instruction; tools/micro/store_layout.hip measured 2.3x the
// per-CU rate for whole 128-B lines (8 rows x 128 B per instruction: 12.4 vs
// 28.8 us for the same bytes on 64 CUs, loads alike), and the epilogue of
// this kernel is bound by its CU's memory-instruction rate
// (tools/gemm_grid_scan.py). So each 16-row chunk of the wave's 64-column
// block goes through a 4 KiB per-wave LDS scratch (beside the operand stages:
// the next tile's DMA is in flight in those) and comes back row-major:
//   bf16 output (L8): lane -> row lane / 8 (+ 8 q), columns 8 (lane % 8) .. +7
//                     = 16 B per lane, 8 rows x 128 B per instruction
//   f32 output  (L4): lane -> row lane / 16 (+ 4 q), columns 4 (lane % 16) .. +3
//                     = 16 B per lane, 4 rows x 256 B per instruction
// and every epilogue operand (bias, aux, residual, C for beta, aux_out) is
// read / written in that layout. Scratch: 16 rows x 256 B, 16-B unit u of
// row r at unit u ^ r (conflict-free for the fragment writes and both read
// layouts). The wave reads back only what it wrote (LDS is in order per wave).
//
// vmcnt is in-order on CDNA: a load issued after a store can only be waited
// for together with that store. So every load (aux, resid) of a chunk is
// issued BEFORE the stores of the previous chunk, and the stores themselves
// are never waited for here (they drain behind the next tile's main loop, see
// the counted wait at the tile start: 2 bf16 / 4 f32 store instructions per
// chunk, as many more for the GELU epilogues' aux_out).
//
// sa / sb (fp8 only): per-row dequantisation scale of A [M] and per-column
// scale of B [N]; the product scales the accumulator before alpha / bias.
constexpr int EPI_SCR = 4096;   // bytes of epilogue scratch per wave
// epilogue streams (aux / residual reads, C / aux_out writes) touch each byte
// once: non-temporal, so they do not evict the A / B panels the XCD's tiles share
#ifndef GEMM4_EPI_NT
#define GEMM4_EPI_NT 3   // 1: loads, 2: stores
#endif
#if GEMM4_EPI_NT & 1
#define NT_LD(p) __builtin_nontemporal_load(p)
#else
#define NT_LD(p) (*(p))
#endif
#if GEMM4_EPI_NT & 2
#define NT_ST(v, p) __builtin_nontemporal_store(v, p)
#else
#define NT_ST(v, p) (*(p) = (v))
#endif
__device__ __forceinline__ int scr_off(int r, int u) { return r * 256 + ((u ^ r) << 4); }

template <typename OutT, int EPI, bool F8 = false, int BM = 256>
__device__ __forceinline__ void epilogue4(const maeclip_gemm_args& args, v4f (&acc)[BM / 32][4], int64_t z, int m0,
                                          int n0, int wm, int wn, int lane, char* __restrict__ scr,
                                          const float* __restrict__ sa = nullptr,
                                          const float* __restrict__ sb = nullptr) {
  constexpr int NCH = BM / 32;               // 16-row chunks per wave: 8 (BM 256) or 6 (BM 192)
  constexpr bool L8 = sizeof(OutT) == 2;
  constexpr int RPI = L8 ? 8 : 4;            // rows per instruction
  constexpr int NQ = 16 / RPI;               // instructions per chunk
  constexpr int VPL = L8 ? 8 : 4;            // values per lane per instruction
  constexpr bool LOAD_AUX = EPI == EPI_DGELU || EPI == EPI_MUL_AUX;
  constexpr bool LOAD_RES = EPI == EPI_RESID || EPI == EPI_DGELU || EPI == EPI_MUL_AUX;
  const int M = (int)args.M, N = (int)args.N;
  const int g = lane >> 4;
  swap_pairs(acc);
  const int64_t off = z * args.strideC;
  OutT* __restrict__ C = (OutT*)args.C + off;
  const float alpha = args.alpha, beta = args.beta;
  const bool has_res = LOAD_RES && args.resid != nullptr;
  const int lr = L8 ? lane >> 3 : lane >> 4;                    // row of the lane within an instruction
  const int n = n0 + 64 * wn + (L8 ? 8 * (lane & 7) : 4 * (lane & 15));
  const bool nok = n < N;                                        // N % 8 == 0 on this path
  const int nc = nok ? n : N - VPL;
  const int rbase = m0 + (BM / 2) * wm + lr;                     // + 16 c + RPI q
  float bias[VPL], csc[VPL];
#pragma unroll
  for (int v = 0; v < VPL; v += 4) {
    const v4f bv = args.bias ? *(const v4f*)(args.bias + nc + v) : v4f{0.f, 0.f, 0.f, 0.f};
    const v4f sv = F8 ? *(const v4f*)(sb + nc + v) : v4f{1.f, 1.f, 1.f, 1.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bias[v + r] = bv[r];
      csc[v + r] = sv[r] * alpha;
    }
  }
  // aux / residual of chunk c + PF - 1 issued before chunk c is finished;
  // the aux ring (8 VGPRs a chunk) may run deeper than the residual one
  // (16 / 32 VGPRs a chunk)
  constexpr int PF = GEMM4_EPI_PF;
  constexpr int PFA = LOAD_AUX ? GEMM4_EPI_PF_AUX : 1;
  typedef unsigned int auxv_t __attribute__((ext_vector_type(L8 ? 4 : 2)));
  auxv_t ax[PFA][NQ];
  v4f rs[PF][NQ][VPL / 4];
  auto load_aux = [&](int c) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int m = min(rbase + 16 * c + RPI * q, M - 1);
      ax[c % PFA][q] = NT_LD((const auxv_t*)((const bf16_t*)args.aux + off + (int64_t)m * args.ldaux + nc));
    }
  };
  auto load_res = [&](int c) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int m = min(rbase + 16 * c + RPI * q, M - 1);
      const float* rp = args.resid + off + (int64_t)m * args.ldr + nc;
#pragma unroll
      for (int v = 0; v < VPL / 4; ++v) rs[c % PF][q][v] = NT_LD((const v4f*)(rp + 4 * v));
    }
  };
  float csum[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) csum[v] = 0.f;
  if constexpr (LOAD_AUX) {
#pragma unroll
    for (int c = 0; c < PFA - 1; ++c) load_aux(c);
  }
  if (LOAD_RES && has_res) {
#pragma unroll
    for (int c = 0; c < PF - 1; ++c) load_res(c);
  }
  // fragment -> scratch offsets of this lane (row lane & 15; units 8 ni + 4 (g & 1) + 2 (g >> 1) + e)
  int wo[4];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int e = 0; e < 2; ++e) wo[2 * ni + e] = scr_off(lane & 15, 8 * ni + 4 * (g & 1) + 2 * (g >> 1) + e);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (LOAD_AUX && c + PFA - 1 < NCH) load_aux(c + PFA - 1);
    if (LOAD_RES && has_res && c + PF - 1 < NCH) load_res(c + PF - 1);
    __builtin_amdgcn_sched_barrier(0);   // keep chunk c+1's loads ahead of chunk c's stores
#pragma unroll
    for (int j = 0; j < 4; ++j) *(v4f*)(scr + wo[j]) = acc[c][j];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int R = lr + RPI * q;           // row within the chunk
      const int m = rbase + 16 * c + RPI * q;
      float x[VPL];
#pragma unroll
      for (int v = 0; v < VPL / 4; ++v) {
        const v4f t = *(const v4f*)(scr + scr_off(R, L8 ? 2 * (lane & 7) + v : (lane & 15)));
#pragma unroll
        for (int r = 0; r < 4; ++r) x[4 * v + r] = t[r];
      }
      const float rsc = (F8 && sa) ? sa[min(m, M - 1)] : 1.f;   // fp8-blocks A: scaled in the MFMA
#pragma unroll
      for (int v = 0; v < VPL; ++v) x[v] = F8 ? fmaf(x[v] * rsc, csc[v], bias[v]) : fmaf(x[v], alpha, bias[v]);
      const bool ok = m < M && nok;
      if (EPI == EPI_GELU || EPI == EPI_GELU_D) {
        float d[VPL];   // GELU: aux_out <- pre-activation; GELU_D: aux_out <- gelu'(pre)
        mc_f32x2 xv[VPL / 2], yv[VPL / 2], dv[VPL / 2];   // value pairs: packed f32 math
#pragma unroll
        for (int v = 0; v < VPL; v += 2) xv[v / 2] = mc_f32x2{x[v], x[v + 1]};
#ifdef GEMM4_OLD_GELU   // A/B builds only: the round-5 first form, pair by pair
#pragma unroll
        for (int v = 0; v < VPL / 2; ++v) gelu_pair2(xv[v], yv[v], dv[v]);
#else
        gelu_pairs<VPL / 2>(xv, yv, dv);
#endif
#pragma unroll
        for (int v = 0; v < VPL; v += 2) {
          d[v] = EPI == EPI_GELU_D ? dv[v / 2][0] : x[v];
          d[v + 1] = EPI == EPI_GELU_D ? dv[v / 2][1] : x[v + 1];
          x[v] = yv[v / 2][0];
          x[v + 1] = yv[v / 2][1];
        }
        if (args.aux_out && ok) {
          bf16_t* ap = (bf16_t*)args.aux_out + off + (int64_t)m * args.ldaux + n;
          if (L8) {
            const v4u pk = {pack2bf(d[0], d[1]), pack2bf(d[2], d[3]), pack2bf(d[4 % VPL], d[5 % VPL]),
                            pack2bf(d[6 % VPL], d[7 % VPL])};
            NT_ST(pk, (v4u*)ap);
          } else {
            const v2u pk = {pack2bf(d[0], d[1]), pack2bf(d[2], d[3])};
            NT_ST(pk, (v2u*)ap);
          }
        }
      }
      if (LOAD_AUX) {
        const auxv_t pk = ax[c % PFA][q];
#pragma unroll
        for (int r = 0; r < VPL / 2; ++r) {
          const float a0 = __uint_as_float(pk[r] << 16), a1 = __uint_as_float(pk[r] & 0xffff0000u);
          if (EPI == EPI_MUL_AUX) {
            x[2 * r] *= a0;
            x[2 * r + 1] *= a1;
          } else {
            x[2 * r] *= gelu_grad_f(a0);
            x[2 * r + 1] *= gelu_grad_f(a1);
          }
        }
      }
      if (LOAD_RES && has_res) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) x[v] += rs[c % PF][q][v / 4][v % 4];
      }
      if (L8 && args.q8) {
        // fp8-blocks copy of the bf16 row segment as stored (maeclip.h q8):
        // a 32-column block is the lane quad 4k .. 4k + 3 (8 columns each)
        float xs[VPL], am = 0.f;
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          xs[v] = bf2f(f2bf(x[v]));
          am = fmaxf(am, fabsf(xs[v]));
        }
        am = fmaxf(am, dpp_mov<0xB1>(am));
        am = fmaxf(am, dpp_mov<0x4E>(am));
        const bool e5 = args.q8_fmt == MAECLIP_FP8_E5M2;
        const unsigned ex = mc_e8m0(am, e5);
        const float inv = mc_e8m0_inv(ex);
#pragma unroll
        for (int v = 0; v < VPL; ++v) xs[v] *= inv;
        if (ok) {
          v2u o;
          if (e5) {
            o[0] = mc_cvt4_fp8<true>(xs[0], xs[1], xs[2], xs[3]);
            o[1] = mc_cvt4_fp8<true>(xs[4 % VPL], xs[5 % VPL], xs[6 % VPL], xs[7 % VPL]);
          } else {
            o[0] = mc_cvt4_fp8<false>(xs[0], xs[1], xs[2], xs[3]);
            o[1] = mc_cvt4_fp8<false>(xs[4 % VPL], xs[5 % VPL], xs[6 % VPL], xs[7 % VPL]);
          }
          NT_ST(o, (v2u*)((uint8_t*)args.q8 + (int64_t)m * args.ldq8 + n));
          if ((lane & 3) == 0) args.q8_scale[mc_fp8b_off(m, n >> 5, N >> 7)] = (uint8_t)ex;
        }
      }
      if (ok) {
        OutT* cp = C + (int64_t)m * args.ldc + n;
        if (beta != 0.f) {
#pragma unroll
          for (int v = 0; v < VPL; v += 4) {
            const v4f cv = ld4<OutT>(cp + v);
#pragma unroll
            for (int r = 0; r < 4; ++r) x[v + r] += beta * cv[r];
          }
        }
#pragma unroll
        for (int v = 0; v < VPL; ++v) csum[v] += x[v];
        if (L8) {
          const v4u pk = {pack2bf(x[0], x[1]), pack2bf(x[2], x[3]), pack2bf(x[4 % VPL], x[5 % VPL]),
                          pack2bf(x[6 % VPL], x[7 % VPL])};
          NT_ST(pk, (v4u*)cp);
        } else {
          NT_ST((v4f{x[0], x[1], x[2], x[3]}), (v4f*)cp);
        }
      }
    }
    if (BM == 256 && (c & 3) == 3 && args.colsum_partial) {   // one partial row per 64-row group
      // the lanes holding the same columns: L8 lanes k + 8 j (row_ror 8 inside
      // each 16-lane row, then the four rows), L4 lanes u + 16 j (the four rows)
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        float t = csum[v];
        if (L8) t += dpp_mov<0x128>(t);
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false, false);
        t = __uint_as_float(p[0]) + __uint_as_float(p[1]);
        const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
        csum[v] = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
      }
      const int mrow = m0 + 128 * wm + 64 * (c >> 2);
      if (lane < (L8 ? 8 : 16) && mrow < M && nok) {
        float* prow = args.colsum_partial + ((int64_t)z * ((M + 63) / 64) + mrow / 64) * N + n;
#pragma unroll
        for (int v = 0; v < VPL; v += 4) *(v4f*)(prow + v) = v4f{csum[v], csum[v + 1], csum[v + 2], csum[v + 3]};
      }
#pragma unroll
      for (int v = 0; v < VPL; ++v) csum[v] = 0.f;
    }
  }
}

// One unit of work of the persistent loop: a 256x256 output tile of one
// problem and its K range (a split-K slice or the whole K).
struct Unit4 {
  const char* A;
  const char* B;
  int64_t lda, ldb;
  int M, N, K;        // problem sizes (K = full reduction length)
  int m0, n0;
  int kbeg, nt;       // first k and number of 64-wide K-tiles of this unit
  int slice, prob;
  int slot;           // stream-K partial tile: workspace slot; -1 = final result
  int tl;             // stream-K: remainder tile index
};

// Split plan of a plain launch (maeclip_gemm with a workspace): every tile's
// K range is cut into S slices, one unit per (tile, slice), units tile-major
// and dealt out in XCD-contiguous chunks of the persistent grid, so a launch
// with fewer tiles than CUs still fills the chip (the micro-batch's 6400-row
// encoder shapes: 75 tiles of 256 x 256 for 256 CUs) and the blocks on one XCD
// work the same K-range of neighbouring tiles at the same time, sharing A rows
// / B columns in its L2. (Stream-K ranges -- every block an equal run of
// K-tiles across tile boundaries -- start every block at a different K and
// lose that reuse: 2.5x the K-tile time, profiles/r05/stream_k_diag_r5c.jsonl;
// removed.) The slices of a tile are summed IN THE SAME LAUNCH by the block
// that arrives last (sk_fixup): no second launch, no waiting, a fixed
// summation order. Slice 0 is the longest, by `lead` K-tiles per other slice
// (L0 = ceil((NT + (S - 1) lead) / S), the rest split evenly): the other
// slices finish first and publish while slice 0 still computes, so slice 0
// usually finds them all published and sums without publishing its own.
// Workspace: [SK_CNT_BYTES] arrival counters (zero before the first launch,
// left zero by every completed launch), then one SK_SLOT partial per unit
// (slot t * S + s), at most 2 per CU.
constexpr int SK_CNT_STRIDE = 16;                 // counter words apart (64 B)
constexpr int64_t SK_CNT_BYTES = 256 * SK_CNT_STRIDE * 4;
constexpr int64_t SK_SLOT = 256 * 256 * 4;        // one fp32 256x256 tile
constexpr int SPLIT_MAX = 2;   // the fix-up sums two partials
struct SkPlan {
  int NT;             // K-tiles of the whole K
  int S;              // slices per tile (0: no split)
  int L0;             // K-tiles of slice 0 (the others share NT - L0)
  int nsl;            // fp32 256x256 slots in the workspace
  unsigned* cnt;
  float* slots;
  __host__ __device__ bool on() const { return S > 0; }
};
struct Gemm4Args {
  maeclip_gemm_args a;
  SkPlan sk;
  const float* sa;    // fp8 only: per-row A / per-column B dequantisation scales
  const float* sb;
  const uint8_t* sab; // fp8-blocks A: e8m0 block scales (common.h mc_fp8b_off layout)
};

// Fix-up of one split tile (slice u.slot of S = 2): returns true in the block
// that arrives last, whose acc then holds the whole tile's sum and which runs
// the epilogue. Hand-off (MI355X_MICROARCH.md, publish-large / handoff-payload):
// every slice but the last to arrive is stored write-through (16-B sc1
// stores), each storing wave drains with vmcnt(0), a workgroup barrier, then
// ONE lane adds to the tile's agent-scope counter; the block whose add returns
// S - 1 (or whose poll already reads S - 1 and so skips its own store: slice
// 0, by its lead) reads the other slices with sc1 loads only. The summation
// order is fixed by slice index whichever block reduces: ((p0 + p1) + p2),
// the reducer's own partial entering at its position, so the output bits do
// not depend on arrival order (p0 + p1 == p1 + p0). Slot layout is fragment-native (the accumulator
// registers as they stand, 1 KiB per wave-instruction): [wave][row
// fragment][col fragment][lane] x 16 B.
template <int NF>
__device__ __forceinline__ bool sk_fixup(v4f (&acc)[NF][4], const SkPlan& sk, const Unit4& u, int* flag, int tid,
                                         int wave, int lane) {
  const int np = sk.S, r = u.slot;
  unsigned* cnt = sk.cnt + u.tl * SK_CNT_STRIDE;
  const unsigned last_count = (unsigned)(np - 1);
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sk.slots, (short)0, (int)((int64_t)sk.nsl * SK_SLOT),
                                                      0x00020000);
  const int vo = lane * 16 + wave * NF * 4 * 1024;
  const int sbase = u.tl * np * (int)SK_SLOT;
  if (tid == 0) *flag = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == last_count ? 1 : 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  SEG_BARRIER();
  bool last = *flag == 1;
  if (!last) {
#ifndef SKX_NO_PUBLISH   // diagnostic builds only: time without the partial stores
    const int so = sbase + r * (int)SK_SLOT;
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[i][j]), rs, vo, so + (i * 4 + j) * 1024, 16);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SEG_BARRIER();
    if (tid == 0)
      *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == last_count ? 1 : 2;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SEG_BARRIER();
    last = *flag == 1;
  }
  if (!last) return false;
#ifndef SKX_NO_REDUCE
  auto ld4 = [&](int p, int i, v4f (&L)[4]) {
    const int so = sbase + p * (int)SK_SLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      L[j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so + (i * 4 + j) * 1024, 16));
  };
  // (the per-fragment offset rides in the scalar soffset: as a per-lane
  // voffset it would take one VGPR per fragment, past the immediate's range)
  // S = 2: the other slice's two row fragments at a time, 8 16-B loads per
  // lane in flight (the hand-off read is latency-bound below that)
  const int o = 1 - r;
#pragma unroll
  for (int i = 0; i < NF; i += 2) {
    v4f L[2][4];
    ld4(o, i, L[0]);
    ld4(o, i + 1, L[1]);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i + ii][j] += L[ii][j];   // p0 + p1 == p1 + p0
    // keep the next fragments' loads below this sum: hoisted, they would
    // hold the whole partial beside acc
    __builtin_amdgcn_sched_barrier(0);
  }
#endif
  if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Grouped weight gradients (maeclip_wgrad_grouped): dW_p[N_p, K_p] (+)=
// dy_p[Mtok, N_p]^T x_p[Mtok, K_p] for up to WG_MAX problems in one persistent
// launch, so the 4 x layers weight-gradient GEMMs of a transformer stack share
// one grid instead of each needing an fp32 split-K slab round trip to fill the
// chip. In GEMM terms M = N_p, N = K_p, K = Mtok, both operands RC.
constexpr int WG_MAX = 48;
struct WgProb {
  const bf16_t* dy;
  const bf16_t* x;
  float* dw;
  int N, K, ldy, ldx;
  int tile_begin;     // prefix sum of tiles
  int slab_off;       // floats, S > 1 only
};
struct WgGroup {
  int np, S, T, Mtok;
  // stream-K remainder (skw > 0): tiles [0, Tdp) run whole (Tdp a multiple of
  // the grid), the K-tiles of tiles [Tdp, T) are dealt out evenly, skw per
  // block in block-position order; a tile cut between blocks leaves fp32
  // partials in 256x256 slots (2 per block) summed by wgrad4_sk_reduce_kernel
  int Tdp, skw, NT;
  float beta;
  float* ws;
  WgProb p[WG_MAX];
};

// F8: 0 = bf16 operands (K-tile 64); 1 / 2 = fp8 operands, A e4m3 / e5m2 and
// B e4m3 (K-tile 128 = the same 128 bytes per row), per-row A scales sa[M] and
// per-column B scales sb[N] applied in the epilogue.
template <int LA, int LB, typename OutT, int EPI, bool SPLIT, bool GRP, int F8 = 0, int BM = 256, bool SK = false>
__device__ __forceinline__ void gemm4_body(const maeclip_gemm_args& args, const WgGroup* __restrict__ gp,
                                           const float* __restrict__ sa = nullptr,
                                           const float* __restrict__ sb = nullptr, const SkPlan* skp_ = nullptr,
                                           const uint8_t* __restrict__ sab = nullptr) {
  static_assert(F8 == 0 || (LA == LAY_KC && LB == LAY_KC && !SPLIT && !GRP), "fp8: KC x KC plain launches only");
  // fp8-blocks A (F8 3 / 4): 192-row tiles, no split plan. The three 64-row
  // scale groups of a K-tile ride with its Bn1 half: waves 4-6 issue one
  // 256-B LDS-DMA each (wave 7 a dummy copy), so every wave keeps 6 DMA
  // instructions in the three youngest halves (waves 0-3: 2 + 2 + 2, waves
  // 4-7: 1 + 2 + 3) and one counted wait serves all.
  constexpr bool F8B = F8 >= 3;
  static_assert(!F8B || (BM == 192 && !SK), "fp8-blocks A: 192-row tiles without a split plan");
  static_assert(BM == 256 || ((BM == 192 || BM == 128) && LA == LAY_KC && !SPLIT && !GRP),
                "BM 192 / 128: KC A, plain launches only");
  static_assert(!SK || (!SPLIT && !GRP), "stream-K: plain launches only");
  using TM = TileM<BM>;
  constexpr int MI = TM::MI;
  constexpr int ESZ = F8 ? 1 : 2;      // operand bytes per element
  constexpr int KT = 128 / ESZ;        // elements per K-tile (128 bytes per row)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  char* const scr = smem + TM::SCR_OFF + wave * EPI_SCR;   // this wave's epilogue scratch
  const int64_t z = GRP ? 0 : blockIdx.z;

  // units: standard = output tiles (this block's slice is blockIdx.y);
  // grouped = slice-major (slice, tile) pairs, so neighbouring units share operands
  int T, gn = 1, klen = 0;
  if (GRP) {
    T = gp->skw > 0 ? gp->Tdp : gp->T * gp->S;
    klen = ((gp->Mtok + gp->S - 1) / gp->S + KT - 1) / KT * KT;
  } else {
    const int gm = ((int)args.M + BM - 1) / BM;
    gn = ((int)args.N + 255) / 256;
    T = gm * gn;
    const int S = SPLIT ? args.splitk : 1;
    klen = (((int)args.K + S - 1) / S + KT - 1) / KT * KT;
  }
  // stream-K remainder (grouped launches: gp): tiles [Tdp, Ttot) are dealt out
  // by K-tiles, skw per block
  int Ttot = T, Tdp = T, skw = 0, NTr = 1;
  if (GRP && gp->skw > 0) {
    Ttot = gp->T;
    Tdp = gp->Tdp;
    skw = gp->skw;
    NTr = gp->NT;
  }
  int skS = 0;   // aligned split: units = (tile, slice)
  if (SK) {
    skS = skp_->S;
    Ttot = Tdp = T = T * skS;
  }
  auto unit = [&](int u) {
    Unit4 w;
    if (GRP) {
      const int tile = u % gp->T, sl = u / gp->T;
      int p = 0;
      while (p + 1 < gp->np && gp->p[p + 1].tile_begin <= tile) ++p;
      const WgProb& q = gp->p[p];
      const int local = tile - q.tile_begin, gnp = (q.K + 255) / 256;
      w.A = (const char*)q.dy;
      w.B = (const char*)q.x;
      w.lda = q.ldy;
      w.ldb = q.ldx;
      w.M = q.N;
      w.N = q.K;
      w.K = gp->Mtok;
      w.m0 = (local / gnp) * 256;
      w.n0 = (local % gnp) * 256;
      w.slice = sl;
      w.prob = p;
    } else {
      w.A = (const char*)args.A + z * args.strideA * ESZ;
      w.B = (const char*)args.B + z * args.strideB * ESZ;
      w.lda = args.lda;
      w.ldb = args.ldb;
      w.M = (int)args.M;
      w.N = (int)args.N;
      w.K = (int)args.K;
      const int tile = skS > 0 ? u / skS : u;
      w.m0 = (tile / gn) * BM;
      w.n0 = (tile % gn) * 256;
      w.slice = skS > 0 ? u - tile * skS : (int)blockIdx.y;
      w.prob = 0;
    }
    if (SK && skS > 0) {
      // slice 0: K-tiles [0, L0); slice s >= 1: its share of the rest
      const int L0 = skp_->L0, rem = skp_->NT - L0, q = rem / (skS - 1), rr = rem % (skS - 1);
      const int s1 = w.slice - 1;
      const int kb = w.slice == 0 ? 0 : L0 + s1 * q + min(s1, rr);
      w.nt = w.slice == 0 ? L0 : q + (s1 < rr ? 1 : 0);
      w.kbeg = kb * KT;
    } else {
      w.kbeg = w.slice * klen;
      const int kend = min(w.K, w.kbeg + klen);
      w.nt = kend > w.kbeg ? (kend - w.kbeg) / KT : 0;
    }
    w.slot = skS > 0 ? w.slice : -1;   // aligned split: every unit is a piece
    w.tl = skS > 0 ? u / skS : 0;
    return w;
  };

  // Persistent over units: the units are cut into 8 contiguous chunks, chunk
  // x worked by the blocks with blockIdx.x % 8 == x (round-robin dispatch puts
  // them on one XCD, so concurrently running tiles share A rows in that XCD's
  // L2; placement is a speed assumption only).
  const int G = gridDim.x, x8 = blockIdx.x % 8, li = blockIdx.x / 8;
  const int nbx = (G - x8 + 7) / 8;
  const int cq = T / 8, cr = T % 8;
  const int cbeg = x8 < cr ? x8 * (cq + 1) : cr * (cq + 1) + (x8 - cr) * cq;
  const int cend = cbeg + cq + (x8 < cr ? 1 : 0);
  // this block's jobs: its whole tiles, then (grouped stream-K) its K range of
  // the remainder tiles
  const int ndp = cbeg + li < cend ? (cend - (cbeg + li) + nbx - 1) / nbx : 0;
  // this block's stream-K range [ska, skb) of (remainder tile, K-tile)
  // iterations: tiles t0 (from K-tile k0) .. t1 (up to K-tile k1); the
  // divisions stay out of the K loop, where job() is also called
  int nsk = 0, skp = 0, sk_t0 = 0, sk_k0 = 0, sk_t1 = 0, sk_k1 = 0;
  if (skw > 0) {
    skp = G % 8 == 0 ? x8 * (G / 8) + li : (int)blockIdx.x;   // XCD-contiguous positions
    const int tot = (Ttot - Tdp) * NTr;
    const int ska = min(skp * skw, tot), skb = min(ska + skw, tot);
    if (skb > ska) {
      sk_t0 = ska / NTr;
      sk_k0 = ska - sk_t0 * NTr;
      sk_t1 = (skb - 1) / NTr;
      sk_k1 = skb - sk_t1 * NTr;
      nsk = sk_t1 - sk_t0 + 1;
    }
  }
  auto job = [&](int j) -> Unit4 {
    if (j < ndp) return unit(cbeg + li + j * nbx);
    const int s = j - ndp, NT = NTr;
    const int tl = sk_t0 + s;
    const int k0 = s == 0 ? sk_k0 : 0;
    const int k1 = tl == sk_t1 ? sk_k1 : NT;
    Unit4 w = unit(Tdp + tl);
    w.kbeg = k0 * KT;
    w.nt = k1 - k0;
    w.slot = (k0 == 0 && k1 == NT) ? -1 : 2 * skp + (s == 0 ? 0 : 1);
    w.tl = tl;
    return w;
  };
  const int njobs = ndp + nsk;

  // per-lane DMA byte offsets of a unit's operands (loop invariants of its K loop)
  auto offsets = [&](const Unit4& w, int (&vA)[2][2], int (&vB)[2][2]) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        vA[sub][i] = half_voffset<LA, true, ESZ, BM>(w.lda, sub, i, wave, lane);
        vB[sub][i] = half_voffset<LB, false, ESZ>(w.ldb, sub, i, wave, lane);
      }
  };
  // half h of K-tile t of unit w: 0 = Am0, 1 = Am1, 2 = Bn0, 3 = Bn1. The
  // K-tile advance is along the row (KC) or down the k-rows (RC).
  auto issue = [&](const Unit4& w, const int (&vA)[2][2], const int (&vB)[2][2], int t, int h) {
    char* dst = smem + (t & 1) * TM::BUF_T + TM::hoff(h);
    const int k0 = w.kbeg + t * KT;
    if (h < 2) {
      const rsrc_t rs = LA == LAY_KC ? make_rsrc(w.A + (int64_t)w.m0 * w.lda * ESZ, ((int64_t)w.M - w.m0) * w.lda * ESZ)
                                     : make_rsrc(w.A + (int64_t)w.m0 * ESZ, ((int64_t)w.K * w.lda - w.m0) * ESZ);
      if constexpr (BM == 256) {
        issue_half(rs, vA[h][0], vA[h][1], k0 * (LA == LAY_KC ? ESZ : (int)(w.lda * ESZ)), dst, wave);
      } else {
        // a 96-row A half is 12 wave-instructions (waves 0-3 issue two, 4-7
        // one), a 64-row half 8 (one per wave)
        const int soff = k0 * ESZ;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + wave * 1024), 16, vA[h][0], soff, 0, 0);
        if (BM == 192 && wave < 4)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + (8 + wave) * 1024), 16, vA[h][1], soff, 0, 0);
      }
    } else {
      const rsrc_t rs = LB == LAY_KC ? make_rsrc(w.B + (int64_t)w.n0 * w.ldb * ESZ, ((int64_t)w.N - w.n0) * w.ldb * ESZ)
                                     : make_rsrc(w.B + (int64_t)w.n0 * ESZ, ((int64_t)w.K * w.ldb - w.n0) * ESZ);
      issue_half(rs, vB[h - 2][0], vB[h - 2][1], k0 * (LB == LAY_KC ? ESZ : (int)(w.ldb * ESZ)), dst, wave);
      if constexpr (F8B) {
        if (h == 3 && wave >= 4) {
          const int T8 = w.K / KT;
          const int G = w.m0 / 64 + min(wave - 4, 2);
          const rsrc_t rsc = make_rsrc((const char*)sab, mc_fp8b_bytes(w.M, w.K));
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsc, (lds_void*)(smem + TM::LDS_T + (t & 1) * 1024 + (wave - 4) * 256),
                                                   4, lane * 4, (G * T8 + w.kbeg / KT + t) * 256, 0, 0);
        }
      }
    }
  };
  // K-tile 0 whole + three halves of K-tile 1 (its Am1 follows in p0)
  auto prologue = [&](const Unit4& w) {
    int vA[2][2], vB[2][2];
    offsets(w, vA, vB);
    issue(w, vA, vB, 0, 0);
    issue(w, vA, vB, 0, 2);
    issue(w, vA, vB, 0, 3);
    issue(w, vA, vB, 0, 1);
    if (w.nt > 1) {
      issue(w, vA, vB, 1, 0);
      issue(w, vA, vB, 1, 2);
      issue(w, vA, vB, 1, 3);
    }
  };

  bool primed = false, first = true, prev_full = false;
  // everything but the three youngest halves (Am0, Bn0, Bn1 of one K-tile):
  // 2 + 2 + 2 wave-instructions, or 1 + 2 + 2 for waves 4-7 at BM 192 and
  // every wave at BM 128
  auto wait_halves = [&]() {
    if (BM == 256 || (BM == 192 && (wave < 4 || F8B))) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  };
#ifdef GEMM4_STAMPS
  // diagnostic build only: s_memtime at tile start / after the DMA wait /
  // after the K-loop / after the epilogue, waves 0 and 4 of every block
  int ntile = 0;
  const bool stamp = blockIdx.y == 0 && blockIdx.z == 0 && (wave == 0 || wave == 4) && lane == 0 && blockIdx.x < 256;
  uint64_t* sp = g_stamps + ((int64_t)blockIdx.x * 8 * 2 + (wave >> 2)) * 4;
#define STAMP(k) do { if (stamp && ntile < 8) sp[ntile * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define STAMP(k) do {} while (0)
#endif
  for (int jb = 0; jb < njobs; ++jb) {
    STAMP(0);
    const Unit4 u = job(jb);
    const int m0 = u.m0, n0 = u.n0, nt = u.nt;
    int voA[2][2], voB[2][2];
    offsets(u, voA, voB);
    if (nt > 0 && !primed) prologue(u);
    if (first && nt > 1) {
      wait_halves();
    } else if (prev_full) {
      // This tile's DMA was issued before the previous tile's epilogue, whose
      // C stores (at least NST per wave for a full tile: 8 row fragments x 2
      // x 16-B, twice that for fp32) are the youngest vector-memory ops: wait
      // for everything older and let the stores drain behind this tile's
      // MFMAs instead of stalling every CU on HBM writes at once.
      // GELU epilogues with aux_out also store a bf16 pre-activation / GELU'
      // per chunk: twice the bf16 stores, all younger than this tile's DMA
      const bool two_out = (EPI == EPI_GELU || EPI == EPI_GELU_D) && args.aux_out != nullptr && !GRP;
      // an fp8-blocks copy (q8) adds two stores per bf16 store instruction
      // (the fp8 bytes, the quad's scale byte)
      const bool q8 = sizeof(OutT) == 2 && args.q8 != nullptr && !GRP;
      if (q8) {
        if (BM == 256) {
          if (two_out) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        } else if (BM == 128) {
          if (two_out) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        } else {
          if (two_out) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
        }
      } else if (BM == 256) {
        if (sizeof(OutT) == 2 && two_out) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else if (sizeof(OutT) == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      } else if (BM == 128) {   // 4 row fragments x 2 (bf16) or x 4 (fp32) stores
        if (sizeof(OutT) == 2 && two_out) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else if (sizeof(OutT) == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else if (sizeof(OutT) == 2 && two_out) {
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      } else {   // 6 row fragments x 2 (bf16) or x 4 (fp32) stores
        if (sizeof(OutT) == 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    first = false;
    prev_full = !SPLIT && m0 + BM <= u.M && n0 + 256 <= u.N;
    primed = false;
    SEG_BARRIER();
    if (wm == 1) SEG_BARRIER();
    STAMP(1);

    v4f acc[2 * MI][4];
#pragma unroll
    for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    v8s fa[MI][2], fb[2][2][2];
    // fp8-blocks: the A scale dword of half `sub` for this lane (row lane % 16,
    // block lane / 16): the 16-row groups 6 wm + 3 sub .. +2 of the tile, byte i
    // = fragment i after the byte align
    auto read_sc = [&](const char* img, int sub) -> unsigned {
      const int g16 = 6 * wm + 3 * sub;
      const int o = (lane >> 4) * 64 + (lane & 15) * 4;
      const unsigned lo = *(const unsigned*)(img + (g16 >> 2) * 256 + o);
      const unsigned hi = *(const unsigned*)(img + ((g16 + 2) >> 2) * 256 + o);
      return __builtin_amdgcn_alignbyte(hi, lo, (unsigned)(g16 & 3));
    };
    unsigned sc0 = 0, sc1 = 0;
    for (int t = 0; t < nt; ++t) {
      const char* buf = smem + (t & 1) * TM::BUF_T;
      const char* scimg = smem + TM::LDS_T + (t & 1) * 1024;
      const char* hA0 = buf;
      const char* hA1 = buf + TM::HALF_A;
      const char* hB0 = buf + 2 * TM::HALF_A;
      const char* hB1 = hB0 + HALF;
      const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
      // ---- p0: quadrant (0,0)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb[0][j][ks] = frag<LB>(hB0, 32 * wn + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(hA0, (BM / 4) * wm + 16 * i, ks, lane);
      if constexpr (F8B) sc0 = read_sc(scimg, 0);
      if (more1) issue(u, voA, voB, t + 1, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      SEG_BARRIER();
      __builtin_amdgcn_s_setprio(1);
      quad_mma<F8, MI>(acc, 0, 0, fb[0], fa, sc0);
      if constexpr (!GRP || (GEMM4_PIN_GRP >> 0) & 1) pin_quad<MI>(acc, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      SEG_BARRIER();
      // ---- p1: quadrant (0,1)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb[1][j][ks] = frag<LB>(hB1, 32 * wn + 16 * j, ks, lane);
      if (more2) issue(u, voA, voB, t + 2, 0);
      LGKM_EARLY();
      SEG_BARRIER();
      __builtin_amdgcn_s_setprio(1);
      quad_mma<F8, MI>(acc, 0, 2, fb[1], fa, sc0);
      if constexpr (!GRP || (GEMM4_PIN_GRP >> 1) & 1) pin_quad<MI>(acc, 0, 2);
      __builtin_amdgcn_s_setprio(0);
      SEG_BARRIER();
      // ---- p2: quadrant (1,1)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(hA1, (BM / 4) * wm + 16 * i, ks, lane);
      if constexpr (F8B) sc1 = read_sc(scimg, 1);
      if (more2) issue(u, voA, voB, t + 2, 2);
      LGKM_EARLY();
      SEG_BARRIER();
      __builtin_amdgcn_s_setprio(1);
      quad_mma<F8, MI>(acc, MI, 2, fb[1], fa, sc1);
      if constexpr (!GRP || (GEMM4_PIN_GRP >> 2) & 1) pin_quad<MI>(acc, MI, 2);
      __builtin_amdgcn_s_setprio(0);
      SEG_BARRIER();
      // ---- p3: quadrant (1,0), operands already in VGPRs. Every LDS read of
      // this tile has been retired behind an earlier barrier, so the last
      // K-tile starts the next unit's DMA here.
      if (more2) {
        issue(u, voA, voB, t + 2, 3);
        wait_halves();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!more1 && jb + 1 < njobs) {
          const Unit4 un = job(jb + 1);
          if (un.nt > 0) {
            prologue(un);
            primed = true;
          }
        }
      }
      SEG_BARRIER();
      __builtin_amdgcn_s_setprio(1);
      quad_mma<F8, MI>(acc, MI, 0, fb[0], fa, sc1);
      if constexpr (!GRP || (GEMM4_PIN_GRP >> 3) & 1) pin_quad<MI>(acc, MI, 0);
      __builtin_amdgcn_s_setprio(0);
      if (wm == 0 || more1) SEG_BARRIER();   // group 1 skips its very last one (it took one extra up front)
    }
    if (nt == 0 && wm == 0) SEG_BARRIER();
    STAMP(2);
    // cut tile (stream-K): the epilogue runs once, in the block that sums the
    // pieces (one epilogue call site either way). Flag word: the Am1 half of
    // LDS buffer 1, which no DMA writes before the next unit's first K-tile
    // (the prologue fills buffer 0 and the other three halves of buffer 1)
    bool run_epi = true;
    if (SK && u.slot >= 0)
      run_epi = sk_fixup<2 * MI>(acc, *skp_, u, (int*)(smem + TM::BUF_T + TM::HALF_A), tid, wave, lane);
    if (!run_epi) {
    } else if constexpr (BM != 256) {
      epilogue4<OutT, EPI, F8 != 0, BM>(args, acc, z, m0, n0, wm, wn, lane, scr, sa, sb);
    } else if (GRP) {
      const WgProb& q = gp->p[u.prob];
      if (u.slot >= 0) {
        epilogue4_tile(gp->ws + (int64_t)u.slot * 65536, acc, wm, wn, lane);
      } else if (SPLIT) {
        epilogue4_slab(gp->ws + q.slab_off + (int64_t)u.slice * q.N * q.K, q.N, q.K, 1.f, acc, m0, n0, wm, wn, lane);
      } else {
        maeclip_gemm_args ea = args;
        ea.M = q.N;
        ea.N = q.K;
        ea.C = q.dw;
        ea.ldc = q.K;
        ea.alpha = 1.f;
        ea.beta = gp->beta;
        epilogue4<OutT, EPI>(ea, acc, 0, m0, n0, wm, wn, lane, scr);
      }
    } else if (SPLIT) {
      epilogue4_slab(args.workspace + ((int64_t)z * args.splitk + blockIdx.y) * args.M * args.N, (int)args.M,
                     (int)args.N, args.alpha, acc, m0, n0, wm, wn, lane);
    } else {
      epilogue4<OutT, EPI, F8 != 0>(args, acc, z, m0, n0, wm, wn, lane, scr, sa, sb);
    }
    STAMP(3);
#ifdef GEMM4_STAMPS
    ++ntile;
#endif
  }
}

template <int LA, int LB, typename OutT, int EPI, bool SPLIT, int BM = 256, bool SK = false>
__global__ void __launch_bounds__(512) gemm4_kernel(const Gemm4Args g) {
  gemm4_body<LA, LB, OutT, EPI, SPLIT, false, 0, BM, SK>(g.a, nullptr, nullptr, nullptr, &g.sk);
}

// fp8 operands (maeclip_gemm_fp8): KC x KC, per-row / per-column scales
template <typename OutT, int EPI, int F8, int BM = 256, bool SK = false>
__global__ void __launch_bounds__(512) gemm4_f8_kernel(const Gemm4Args g) {
  gemm4_body<LAY_KC, LAY_KC, OutT, EPI, false, false, F8, BM, SK>(g.a, nullptr, g.sa, g.sb, &g.sk, g.sab);
}

// grouped weight gradients: RC x RC, fp32 out, no epilogue (beta only)
template <bool SPLIT>
__global__ void __launch_bounds__(512) wgrad4_kernel(const WgGroup grp) {
  maeclip_gemm_args a = {};
  a.alpha = 1.f;
  gemm4_body<LAY_RC, LAY_RC, float, EPI_NONE, SPLIT, true>(a, &grp);
}

// S slabs of every problem -> dW (fixed summation order)
__global__ void __launch_bounds__(256) wgrad4_reduce_kernel(const WgGroup grp) {
  const WgProb& q = grp.p[blockIdx.y];
  const int64_t NK = (int64_t)q.N * q.K;
  const float* ws = grp.ws + q.slab_off;
  for (int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; e < NK; e += (int64_t)gridDim.x * 1024) {
    v4f v = *(const v4f*)(ws + e);
    for (int s = 1; s < grp.S; ++s) v += *(const v4f*)(ws + s * NK + e);
    float* d = q.dw + e;
    if (grp.beta != 0.f) v += grp.beta * *(const v4f*)d;
    *(v4f*)d = v;
  }
}

// stream-K remainder tile blockIdx.x, element chunk blockIdx.y (of SKR_CHUNKS):
// the partial slots of the blocks that shared its K range, in block-position
// order (fixed summation order), + beta dW. Chunking the tile over SKR_CHUNKS
// workgroups keeps the reduce at HBM rate when only a few tiles are cut (the
// encoder's 16 remainder tiles each carry ~17 slots).
constexpr int SKR_CHUNKS = 16;
__global__ void __launch_bounds__(256) wgrad4_sk_reduce_kernel(const WgGroup grp) {
  const int r = blockIdx.x, NT = grp.NT, w = grp.skw;
  const int p0 = r * NT / w, p1 = ((r + 1) * NT - 1) / w;
  if (p0 == p1) return;   // one block ran the whole tile and wrote dW itself
  const int tile = grp.Tdp + r;
  int p = 0;
  while (p + 1 < grp.np && grp.p[p + 1].tile_begin <= tile) ++p;
  const WgProb& q = grp.p[p];
  const int local = tile - q.tile_begin, gnp = (q.K + 255) / 256;
  const int m0 = (local / gnp) * 256, n0 = (local % gnp) * 256;
  constexpr int CH = 65536 / SKR_CHUNKS;
  for (int e = blockIdx.y * CH + threadIdx.x * 4; e < (int)(blockIdx.y + 1) * CH; e += 1024) {
    const int m = m0 + (e >> 8), n = n0 + (e & 255);
    if (m >= q.N || n >= q.K) continue;   // K % 8 == 0: a 4-group is all in or all out
    v4f v = {0.f, 0.f, 0.f, 0.f};
    for (int c = p0; c <= p1; ++c) {
      const int slot = 2 * c + ((c * w) / NT == r ? 0 : 1);
      v += *(const v4f*)(grp.ws + (int64_t)slot * 65536 + e);
    }
    float* d = q.dw + (int64_t)m * q.K + n;
    if (grp.beta != 0.f) v += grp.beta * *(const v4f*)d;
    *(v4f*)d = v;
  }
}

int gemm4_ncu() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  // diagnostic: option GEMM_GRID caps the persistent grid of plain launches
  // (contention scans, tools/gemm_grid_scan.py); unset in production
  const int cap = maeclip::option(MAECLIP_OPT_GEMM_GRID, 0);
  return cap > 0 && cap < ncu ? cap : ncu;
}

// Tile height and split plan of a plain launch (one batch, no caller
// split-K), from a cost model in units of one 256-row K-tile (~2.9k cycles, 64
// KiB of operand DMA per CU): a 192-row K-tile costs 0.89 of it (measured,
// encoder fc2 fwd, one round each); a tile's epilogue ~EPI_C; a split costs
// slice 0's K-tiles (its lead hides the others' publish) + F1 per other slice
// the last block reads back. MAECLIP_GEMM_BM=256 / 192 forces a tile height;
// MAECLIP_GEMM_SK=1 enables the cost model's split (default off, see below);
// MAECLIP_GEMM_SPLIT=S forces a split of S wherever it fits (A/B, tests).
struct TileChoice {
  int bm;
  SkPlan sk;
};
int64_t sk_workspace_bytes(int ncu) { return SK_CNT_BYTES + 2 * (int64_t)ncu * SK_SLOT; }

TileChoice choose_tiles(const maeclip_gemm_args& a, int KT, int ncu) {
  const int force_bm = maeclip::option(MAECLIP_OPT_GEMM_BM, 0);
  // default off: in the micro-batched step every split cost whole-step
  // throughput although it wins alone (profiles/r05/gemm_split_minK_step_ab_r5i.txt)
  const int sk_mode = maeclip::option(MAECLIP_OPT_GEMM_SK, 0);   // 0 off, 1 cost model
  const int force_split = maeclip::option(MAECLIP_OPT_GEMM_SPLIT, 0);
  // the cost model's split only at K >= GEMM_SPLIT_MINK (step A/B)
  const int64_t split_min_k = maeclip::option(MAECLIP_OPT_GEMM_SPLIT_MINK, 0);
  const bool plain = a.splitk <= 1 && a.batch == 1;
  const bool allow192 = force_bm != 256 && force_bm != 128 && plain && a.a_layout == LAY_KC && !a.colsum_partial;
  // 128-row tiles: bf16 only (KT 64); chosen by the cost model only when
  // MAECLIP_GEMM_BM128=1 (A/B) or forced by MAECLIP_GEMM_BM=128
  const bool allow128 = KT == 64 && plain && a.a_layout == LAY_KC && !a.colsum_partial &&
                        (force_bm == 128 || (force_bm == 0 && maeclip::option(MAECLIP_OPT_GEMM_BM128, 0) == 1));
  const bool allow256 = (force_bm != 192 || !allow192) && (force_bm != 128 || !allow128);
  const bool allow_sk = plain && (sk_mode != 0 || force_split > 0) && a.workspace != nullptr && ncu <= 256;
  const int64_t gn = (a.N + 255) / 256, NT = a.K / KT;
  constexpr double EPI_C = 2.5, F1 = 2.0;
  const SkPlan none = {0, 0, 0, 0, nullptr, nullptr};
  // slice 0's lead per other slice (aligned split): about one publish of a
  // 256 x 256 fp32 partial; MAECLIP_GEMM_SPLIT_D overrides
  const int lead = maeclip::option(MAECLIP_OPT_GEMM_SPLIT_D, 4);
  TileChoice best = {256, none};
  double best_cost = 1e30;
  // the best data-parallel choice: the result whenever no split plan is taken
  // (also when a forced split S does not fit the shape)
  TileChoice best_dp = {256, none};
  double best_dp_cost = 1e30;
  auto l0 = [&](int S) {
    // slice 0 longer by `lead` per other slice, every other slice >= 1 K-tile
    const int64_t L0 = (NT + (int64_t)(S - 1) * lead + S - 1) / S;
    return (int)std::max<int64_t>(std::min<int64_t>(L0, NT - (S - 1)), (NT + S - 1) / S);
  };
  auto plan = [&](int S) {
    SkPlan p = none;
    p.NT = (int)NT;
    p.S = S;
    p.L0 = l0(S);
    p.nsl = 2 * ncu;
    p.cnt = (unsigned*)a.workspace;
    p.slots = (float*)((char*)a.workspace + SK_CNT_BYTES);
    return p;
  };
  for (int bm : {256, 192, 128}) {
    if ((bm == 256 && !allow256) || (bm == 192 && !allow192) || (bm == 128 && !allow128)) continue;
    const double c = bm == 192 ? 0.89 : bm == 128 ? 0.72 : 1.0;
    const int64_t T = (a.M + bm - 1) / bm * gn, R = T % ncu;
    const double dp = (double)((T + ncu - 1) / ncu) * (NT * c + EPI_C);
    if (dp < best_dp_cost - 1e-9) {
      best_dp_cost = dp;
      best_dp = {bm, none};
    }
    if (dp < best_cost - 1e-9 && force_split == 0) {
      best_cost = dp;
      best = {bm, none};
    }
    // split: 192-row tiles only (the 256-row body has no registers left for
    // the fix-up: its split instantiation spilled inside the K loop)
    if (!allow_sk || bm != 192 || (force_split == 0 && (R == 0 || a.K < split_min_k))) continue;
    for (int S = 2; S <= SPLIT_MAX; ++S) {
      if ((force_split > 0 && S != force_split) || T * S > 2 * ncu || T > 256 || NT < 2 * S) continue;
      const int64_t rounds = (T * S + ncu - 1) / ncu;
      // the publish of slices >= 1 runs while slice 0 computes its lead
      const double cost = (double)rounds * l0(S) * c + EPI_C + F1 * (S - 1);
      if (force_split > 0 || cost < best_cost - 1e-9) {
        best_cost = force_split > 0 ? -1.0 : cost;
        best = {bm, plan(S)};
      }
    }
  }
  return best.sk.on() ? best : best_dp;
}

template <typename KernT, typename ArgT>
void launch_persistent(KernT kern, int lds, int64_t tiles, int ncu, bool sk, const ArgT& g, hipStream_t s) {
  maeclip::allow_lds((const void*)kern, lds);
  // one block per CU: persistent over tiles (stream-K: the whole grid, the
  // block positions the plan was made for)
  const int grid = sk ? ncu : (int)(tiles < ncu ? tiles : ncu);
  hipLaunchKernelGGL(kern, dim3(grid, 1, 1), dim3(512), lds, s, g);
}

template <int LA, int LB, typename OutT, int EPI>
int launch4(const maeclip_gemm_args& a, hipStream_t s) {
  const int gn = (int)((a.N + 255) / 256);
  const int S = a.splitk > 1 ? a.splitk : 1;
  const int ncu = gemm4_ncu();
  Gemm4Args g = {};
  g.a = a;
  if (S == 1 && a.batch == 1) {
    const TileChoice tc = choose_tiles(a, 64, ncu);
    g.sk = tc.sk;
    const bool sk = tc.sk.on();
    if constexpr (LA == LAY_KC) {
      if (tc.bm == 192) {
        const int64_t tiles = (a.M + 191) / 192 * gn;
        if (sk) launch_persistent(gemm4_kernel<LA, LB, OutT, EPI, false, 192, true>, TileM<192>::LDS_ALL, tiles, ncu, true, g, s);
        else launch_persistent(gemm4_kernel<LA, LB, OutT, EPI, false, 192>, TileM<192>::LDS_ALL, tiles, ncu, false, g, s);
        MC_CHECK_LAUNCH("maeclip_gemm(v4, 192-row tiles)");
        return 0;
      }
      if (tc.bm == 128) {
        const int64_t tiles = (a.M + 127) / 128 * gn;
        launch_persistent(gemm4_kernel<LA, LB, OutT, EPI, false, 128>, TileM<128>::LDS_ALL, tiles, ncu, false, g, s);
        MC_CHECK_LAUNCH("maeclip_gemm(v4, 128-row tiles)");
        return 0;
      }
    }
  }
  const int gm = (int)((a.M + 255) / 256);
  auto kern = S > 1 ? gemm4_kernel<LA, LB, OutT, EPI, true> : gemm4_kernel<LA, LB, OutT, EPI, false>;
  maeclip::allow_lds((const void*)kern, TileM<256>::LDS_ALL);
  // one block per CU (128 KiB LDS): persistent over tiles for plain launches;
  // split-K / batched launches get one block per (tile, slice, batch)
  const int tiles = gm * gn;
  const int grid = (S * a.batch > 1 || tiles < ncu) ? tiles : ncu;
  hipLaunchKernelGGL(kern, dim3(grid, S, (unsigned)a.batch), dim3(512), TileM<256>::LDS_ALL, s, g);
  MC_CHECK_LAUNCH("maeclip_gemm(v4)");
  return 0;
}

template <int LA, int LB, typename OutT>
int epi4(const maeclip_gemm_args& a, hipStream_t s) {
#ifdef GEMM4_DEV_SUBSET   // register / ISA inspection builds only: one epilogue
#ifndef GEMM4_DEV_EPI
#define GEMM4_DEV_EPI EPI_NONE
#endif
  return launch4<LA, LB, OutT, GEMM4_DEV_EPI>(a, s);
#else
  switch (a.epilogue) {
    case EPI_NONE: return launch4<LA, LB, OutT, EPI_NONE>(a, s);
    case EPI_GELU: return launch4<LA, LB, OutT, EPI_GELU>(a, s);
    case EPI_RESID: return launch4<LA, LB, OutT, EPI_RESID>(a, s);
    case EPI_GELU_D: return launch4<LA, LB, OutT, EPI_GELU_D>(a, s);
    case EPI_MUL_AUX: return launch4<LA, LB, OutT, EPI_MUL_AUX>(a, s);
    default: return launch4<LA, LB, OutT, EPI_DGELU>(a, s);
  }
#endif
}

template <int LA, int LB>
int out4(const maeclip_gemm_args& a, hipStream_t s) {
  return a.out_dtype == MAECLIP_BF16 ? epi4<LA, LB, bf16_t>(a, s) : epi4<LA, LB, float>(a, s);
}

}  // namespace

#ifdef GEMM4_STAMPS
extern "C" int maeclip_debug_gemm4_stamps(uint64_t* host, int n) {
  // n < 0: zero the stamp buffer (host unused)
  if (n < 0) {
    static uint64_t zero[256 * 8 * 2 * 4] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(uint64_t) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

namespace maeclip {
// Shapes the v4 epilogue supports: 8 consecutive output columns per lane with
// 16-B accesses on C / aux / resid.
bool gemm_v4_ok(const maeclip_gemm_args& a) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a.dtype != MAECLIP_BF16 || a.K % 64 != 0 || a.K <= 0 || a.lda % 8 || a.ldb % 8) return false;
  if (a.M < 256 || a.N < 256 || a.N % 8) return false;
  // buffer-descriptor DMA: every operand byte offset must fit 31 bits
  const int64_t lim = 0x7fffffffLL;
  if ((a.a_layout == LAY_KC ? a.M * a.lda : a.K * a.lda) * 2 >= lim) return false;
  if ((a.b_layout == LAY_KC ? a.N * a.ldb : a.K * a.ldb) * 2 >= lim) return false;
  if (a.splitk > 1) return al16(a.workspace);
  if (!al16(a.C) || (a.out_dtype == MAECLIP_BF16 ? a.ldc % 8 : a.ldc % 4)) return false;
  const bool wa = a.epilogue == EPI_GELU || a.epilogue == EPI_GELU_D;
  const bool ra = a.epilogue == EPI_DGELU || a.epilogue == EPI_MUL_AUX;
  if ((wa && a.aux_out && (!al16(a.aux_out) || a.ldaux % 8)) || (ra && (!al16(a.aux) || a.ldaux % 8))) return false;
  if (a.resid && (!al16(a.resid) || a.ldr % 4)) return false;
  if (a.bias && !al16(a.bias)) return false;
  return true;
}

// scratch bytes of a stream-K launch of this shape (0: none chosen)
int64_t gemm_v4_workspace(const maeclip_gemm_args& a) {
  const bool f8 = a.dtype == MAECLIP_FP8_E4M3 || a.dtype == MAECLIP_FP8_E5M2;
  if (f8 ? (a.K % 128 != 0 || a.M < 256 || a.N < 256) : !gemm_v4_ok(a)) return 0;
  if (a.splitk > 1 || a.batch != 1) return 0;
  if (!f8 && a.a_layout != LAY_KC) return 0;
  maeclip_gemm_args b = a;
  b.workspace = (float*)(uintptr_t)256;   // any non-null: "a workspace is offered"
  const int ncu = gemm4_ncu();
  return choose_tiles(b, f8 ? 128 : 64, ncu).sk.on() ? sk_workspace_bytes(ncu) : 0;
}

int gemm_v4(const maeclip_gemm_args& a, hipStream_t s) {
  if (a.a_layout == LAY_KC && a.b_layout == LAY_KC) return out4<LAY_KC, LAY_KC>(a, s);
  if (a.a_layout == LAY_KC && a.b_layout == LAY_RC) return out4<LAY_KC, LAY_RC>(a, s);
  if (a.a_layout == LAY_RC && a.b_layout == LAY_KC) return out4<LAY_RC, LAY_KC>(a, s);
  return out4<LAY_RC, LAY_RC>(a, s);
}
}  // namespace maeclip

// ------------------------------------------------------------ fp8 operands

namespace {

template <typename OutT, int EPI, int F8>
int launch_f8(const maeclip_gemm_args& a, const float* sa, const float* sb, hipStream_t s) {
  const int ncu = gemm4_ncu();
  Gemm4Args g = {};
  g.a = a;
  g.sa = sa;
  g.sb = sb;
  const int gn = (int)((a.N + 255) / 256);
  if (a.batch == 1) {
    const TileChoice tc = choose_tiles(a, 128, ncu);
    g.sk = tc.sk;
    const bool sk = tc.sk.on();
    const int64_t tiles = (a.M + tc.bm - 1) / tc.bm * gn;
    if (tc.bm == 192) {
      if (sk) launch_persistent(gemm4_f8_kernel<OutT, EPI, F8, 192, true>, TileM<192>::LDS_ALL, tiles, ncu, true, g, s);
      else launch_persistent(gemm4_f8_kernel<OutT, EPI, F8, 192>, TileM<192>::LDS_ALL, tiles, ncu, false, g, s);
      MC_CHECK_LAUNCH("maeclip_gemm_fp8(192-row tiles)");
      return 0;
    }
  }
  auto kern = gemm4_f8_kernel<OutT, EPI, F8>;
  maeclip::allow_lds((const void*)kern, TileM<256>::LDS_ALL);
  const int tiles = (int)(((a.M + 255) / 256) * gn);
  const int grid = (a.batch > 1 || tiles < ncu) ? tiles : ncu;
  hipLaunchKernelGGL(kern, dim3(grid, 1, (unsigned)a.batch), dim3(512), TileM<256>::LDS_ALL, s, g);
  MC_CHECK_LAUNCH("maeclip_gemm_fp8");
  return 0;
}

template <typename OutT, int F8>
int epi_f8(const maeclip_gemm_args& a, const float* sa, const float* sb, hipStream_t s) {
#ifdef GEMM4_DEV_SUBSET
  return launch_f8<OutT, EPI_NONE, F8>(a, sa, sb, s);
#else
  switch (a.epilogue) {
    case EPI_NONE: return launch_f8<OutT, EPI_NONE, F8>(a, sa, sb, s);
    case EPI_GELU: return launch_f8<OutT, EPI_GELU, F8>(a, sa, sb, s);
    case EPI_RESID: return launch_f8<OutT, EPI_RESID, F8>(a, sa, sb, s);
    case EPI_GELU_D: return launch_f8<OutT, EPI_GELU_D, F8>(a, sa, sb, s);
    case EPI_MUL_AUX: return launch_f8<OutT, EPI_MUL_AUX, F8>(a, sa, sb, s);
    default: return launch_f8<OutT, EPI_DGELU, F8>(a, sa, sb, s);
  }
#endif
}

// fp8-blocks A (maeclip_gemm_fp8_blocks): 192-row tiles (the scale images fit
// beside their operand stages there), no split plan
template <typename OutT, int EPI, int F8>
int launch_f8b(const maeclip_gemm_args& a, const uint8_t* sab, const float* sb, hipStream_t s) {
  const int ncu = gemm4_ncu();
  Gemm4Args g = {};
  g.a = a;
  g.sb = sb;
  g.sab = sab;
  const int64_t tiles = (a.M + 191) / 192 * ((a.N + 255) / 256);
  launch_persistent(gemm4_f8_kernel<OutT, EPI, F8, 192>, TileM<192>::LDS_ALL, tiles, ncu, false, g, s);
  MC_CHECK_LAUNCH("maeclip_gemm_fp8_blocks");
  return 0;
}

template <typename OutT, int F8>
int epi_f8b(const maeclip_gemm_args& a, const uint8_t* sab, const float* sb, hipStream_t s) {
  switch (a.epilogue) {
    case EPI_NONE: return launch_f8b<OutT, EPI_NONE, F8>(a, sab, sb, s);
    case EPI_RESID: return launch_f8b<OutT, EPI_RESID, F8>(a, sab, sb, s);
    case EPI_GELU_D: return launch_f8b<OutT, EPI_GELU_D, F8>(a, sab, sb, s);
    case EPI_MUL_AUX: return launch_f8b<OutT, EPI_MUL_AUX, F8>(a, sab, sb, s);
    default: MC_CHECK_ARG(false, "maeclip_gemm_fp8_blocks: epilogue %d not built (0, 2, 4, 5)", a.epilogue);
  }
}

// argument checks shared by the two fp8 entries
int check_f8(const maeclip_gemm_args* a, const char* who) {
  MC_CHECK_ARG(a->dtype == MAECLIP_FP8_E4M3 || a->dtype == MAECLIP_FP8_E5M2,
               "%s: dtype (A format) must be MAECLIP_FP8_E4M3 or MAECLIP_FP8_E5M2", who);
  MC_CHECK_ARG(a->a_layout == LAY_KC && a->b_layout == LAY_KC, "%s: KC x KC operands only", who);
  MC_CHECK_ARG(a->K > 0 && a->K % 128 == 0, "%s: K=%lld must be a positive multiple of 128", who, (long long)a->K);
  MC_CHECK_ARG(a->M >= 256 && a->N >= 256 && a->N % 8 == 0, "%s: M, N >= 256 and N %% 8 == 0", who);
  MC_CHECK_ARG(a->splitk <= 1, "%s: no split-K", who);
  MC_CHECK_ARG(a->batch >= 1, "%s: batch >= 1", who);
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  MC_CHECK_ARG(al16(a->A) && al16(a->B) && a->lda % 16 == 0 && a->ldb % 16 == 0 && a->lda >= a->K && a->ldb >= a->K,
               "%s: operands need 16-B aligned rows (lda, ldb %% 16 == 0, >= K)", who);
  MC_CHECK_ARG(al16(a->C) && (a->out_dtype == MAECLIP_BF16 ? a->ldc % 8 : a->ldc % 4) == 0, "%s: C alignment", who);
  const bool wa = a->epilogue == EPI_GELU || a->epilogue == EPI_GELU_D;
  const bool ra = a->epilogue == EPI_DGELU || a->epilogue == EPI_MUL_AUX;
  MC_CHECK_ARG(!(wa && a->aux_out && (!al16(a->aux_out) || a->ldaux % 8)) && !(ra && (!al16(a->aux) || a->ldaux % 8)),
               "%s: aux alignment", who);
  MC_CHECK_ARG(!a->resid || (al16(a->resid) && a->ldr % 4 == 0), "%s: resid alignment", who);
  MC_CHECK_ARG(!a->bias || al16(a->bias), "%s: bias alignment", who);
  const int64_t lim = 0x7fffffffLL;
  MC_CHECK_ARG(a->M * a->lda < lim && a->N * a->ldb < lim, "%s: operand exceeds 2^31 bytes", who);
  return maeclip::check_q8(*a, who);
}

}  // namespace

namespace maeclip {
// the optional fp8-blocks output of a GEMM (maeclip_gemm_args q8)
int check_q8(const maeclip_gemm_args& a, const char* who) {
  if (!a.q8) return 0;
  MC_CHECK_ARG(a.out_dtype == MAECLIP_BF16 && a.batch == 1 && a.beta == 0.f && a.splitk <= 1 && a.N % 128 == 0 &&
                   a.ldq8 >= a.N && a.ldq8 % 8 == 0 && ((uintptr_t)a.q8 & 7) == 0 && a.q8_scale &&
                   (a.q8_fmt == MAECLIP_FP8_E4M3 || a.q8_fmt == MAECLIP_FP8_E5M2),
               "%s: fp8-blocks output (q8) needs bf16 C, batch 1, beta 0, N %% 128 == 0, ldq8 %% 8, a scale buffer "
               "and an fp8 format", who);
  return 0;
}
}  // namespace maeclip

extern "C" int32_t maeclip_gemm_fp8_blocks(const maeclip_gemm_args* a, const uint8_t* scale_a, const float* scale_b,
                                           void* stream) {
  MC_CHECK_ARG(a != nullptr && scale_a != nullptr && scale_b != nullptr, "maeclip_gemm_fp8_blocks: null argument");
  if (int e = check_f8(a, "maeclip_gemm_fp8_blocks")) return e;
  MC_CHECK_ARG(a->batch == 1 && ((uintptr_t)scale_b & 15) == 0, "maeclip_gemm_fp8_blocks: batch 1, 16-B aligned scale_b");
  hipStream_t s = (hipStream_t)stream;
  const bool e5 = a->dtype == MAECLIP_FP8_E5M2;
  if (a->out_dtype == MAECLIP_BF16)
    return e5 ? epi_f8b<bf16_t, 4>(*a, scale_a, scale_b, s) : epi_f8b<bf16_t, 3>(*a, scale_a, scale_b, s);
  return e5 ? epi_f8b<float, 4>(*a, scale_a, scale_b, s) : epi_f8b<float, 3>(*a, scale_a, scale_b, s);
}

extern "C" int32_t maeclip_gemm_fp8(const maeclip_gemm_args* a, const float* scale_a, const float* scale_b,
                                    void* stream) {
  MC_CHECK_ARG(a != nullptr && scale_a != nullptr && scale_b != nullptr, "maeclip_gemm_fp8: null argument");
  if (int e = check_f8(a, "maeclip_gemm_fp8")) return e;
  MC_CHECK_ARG(((uintptr_t)scale_b & 15) == 0, "maeclip_gemm_fp8: 16-B aligned scale_b");
  hipStream_t s = (hipStream_t)stream;
  const bool e5 = a->dtype == MAECLIP_FP8_E5M2;
  if (a->out_dtype == MAECLIP_BF16)
    return e5 ? epi_f8<bf16_t, 2>(*a, scale_a, scale_b, s) : epi_f8<bf16_t, 1>(*a, scale_a, scale_b, s);
  return e5 ? epi_f8<float, 2>(*a, scale_a, scale_b, s) : epi_f8<float, 1>(*a, scale_a, scale_b, s);
}

// ------------------------------------------------- grouped weight gradients
namespace {

int wg_ncu() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

bool wg_v4_ok(const maeclip_wgrad_problem* pr, int n, int64_t M, int32_t dtype) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (dtype != MAECLIP_BF16 || M <= 0 || M % 64 != 0 || M >= (1ll << 31)) return false;
  for (int i = 0; i < n; ++i) {
    const maeclip_wgrad_problem& q = pr[i];
    if (q.N < 256 || q.K < 256 || q.N % 8 || q.K % 8 || q.ldy % 8 || q.ldx % 8) return false;
    if (q.ldy < q.N || q.ldx < q.K) return false;
    if (!al16(q.dy) || !al16(q.x) || !al16(q.dw)) return false;
    if (M * q.ldy * 2 >= 0x7fffffffLL || M * q.ldx * 2 >= 0x7fffffffLL) return false;
  }
  return true;
}

int wg_tiles(const maeclip_wgrad_problem& q) { return (int)(((q.N + 255) / 256) * ((q.K + 255) / 256)); }

// Slices per tile for one launch of T tiles: the S minimising the number of
// waves of units per tile-K, ceil(T*S/ncu)/S, where S > 1 must beat S = 1 by
// 15% to pay for the fp32 slab write + reduce, and S <= 4 (the slab traffic
// grows with S while the wave quantisation it fixes does not); every slice
// keeps >= 16 K-tiles. The encoder's 48 dW (1296 tiles: 5.06 waves) take S = 1, the
// decoder's 32 (384 tiles: 1.5 waves) S = 2.
int wg_splits(int T, int64_t M) {
  const int ncu = wg_ncu();
  const double c1 = (double)((T + ncu - 1) / ncu);
  int best = 1;
  double best_cost = c1;
  for (int S = 2; S <= 4; ++S) {
    if (M / 64 / S < 16) break;
    const double cost = (double)((T * S + ncu - 1) / ncu) / S;
    if (cost < 0.85 * c1 && cost < best_cost - 1e-9) {
      best = S;
      best_cost = cost;
    }
  }
  return best;
}

// Stream-K remainder: K-tiles per block when the T tiles leave a partial last
// wave on the grid (0 = none). Each block then runs floor(T / ncu) whole tiles
// plus skw K-tiles of the remainder, so every block does the same work; a
// block's range cuts at most two tiles (two 256 KB fp32 slots). Below 8
// K-tiles per block the slot write + reduce outweighs the balance.
int wg_skw(int T, int64_t M) {
  const bool enabled = maeclip::option(MAECLIP_OPT_WG_SK, 1) != 0;   // 0: uniform split-K slices instead (A/B)
  const int G = wg_ncu(), R = T % G;
  if (R == 0 || !enabled) return 0;
  const int64_t skw = ((int64_t)R * (M / 64) + G - 1) / G;
  return skw >= 8 ? (int)skw : 0;
}

int64_t wg_chunk_ws(const maeclip_wgrad_problem* pr, int n, int64_t M) {
  int T = 0;
  int64_t nk = 0;
  for (int i = 0; i < n; ++i) {
    T += wg_tiles(pr[i]);
    nk += pr[i].N * pr[i].K;
  }
  if (wg_skw(T, M) > 0) return (int64_t)2 * wg_ncu() * 65536 * 4;
  const int S = wg_splits(T, M);
  return S > 1 ? (int64_t)S * nk * 4 : 0;
}

}  // namespace

extern "C" int64_t maeclip_wgrad_grouped_workspace(const maeclip_wgrad_problem* probs, int32_t nprob, int64_t M,
                                                   int32_t dtype) {
  if (!probs || nprob <= 0 || !wg_v4_ok(probs, nprob, M, dtype)) return 0;
  int64_t ws = 0;
  for (int c = 0; c < nprob; c += WG_MAX) ws = std::max(ws, wg_chunk_ws(probs + c, std::min(WG_MAX, nprob - c), M));
  return ws;
}

extern "C" int32_t maeclip_wgrad_grouped(const maeclip_wgrad_problem* probs, int32_t nprob, int64_t M, int32_t dtype,
                                         float beta, void* workspace, int64_t ws_bytes, void* stream) {
  MC_CHECK_ARG(probs != nullptr && nprob >= 0, "maeclip_wgrad_grouped: bad problem list");
  MC_CHECK_ARG(M >= 0, "maeclip_wgrad_grouped: bad token count");
  if (nprob == 0 || M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (!wg_v4_ok(probs, nprob, M, dtype)) {
    // shapes / dtypes outside the grouped kernel: one maeclip_gemm per problem
    for (int i = 0; i < nprob; ++i) {
      const maeclip_wgrad_problem& q = probs[i];
      maeclip_gemm_args a = {};
      a.A = q.dy;
      a.B = q.x;
      a.C = q.dw;
      a.M = q.N;
      a.N = q.K;
      a.K = M;
      a.lda = q.ldy;
      a.ldb = q.ldx;
      a.ldc = q.K;
      a.batch = 1;
      a.dtype = dtype;
      a.out_dtype = MAECLIP_F32;
      a.a_layout = LAY_RC;
      a.b_layout = LAY_RC;
      a.alpha = 1.f;
      a.beta = beta;
      a.splitk = 1;
      const int rc = maeclip_gemm(&a, stream);
      if (rc != 0) return rc;
    }
    return 0;
  }
  MC_CHECK_ARG(ws_bytes >= maeclip_wgrad_grouped_workspace(probs, nprob, M, dtype) &&
                   (ws_bytes == 0 || ((uintptr_t)workspace & 15) == 0),
               "maeclip_wgrad_grouped: workspace too small or misaligned");
  for (int c = 0; c < nprob; c += WG_MAX) {
    const int n = std::min(WG_MAX, nprob - c);
    WgGroup g = {};
    g.np = n;
    g.Mtok = (int)M;
    g.beta = beta;
    g.ws = (float*)workspace;
    int T = 0;
    int64_t so = 0;
    for (int i = 0; i < n; ++i) {
      const maeclip_wgrad_problem& q = probs[c + i];
      WgProb& w = g.p[i];
      w.dy = (const bf16_t*)q.dy;
      w.x = (const bf16_t*)q.x;
      w.dw = q.dw;
      w.N = (int)q.N;
      w.K = (int)q.K;
      w.ldy = (int)q.ldy;
      w.ldx = (int)q.ldx;
      w.tile_begin = T;
      T += wg_tiles(q);
    }
    g.T = T;
    g.skw = wg_skw(T, M);
    if (g.skw > 0) {
      g.S = 1;
      g.NT = (int)(M / 64);
      g.Tdp = T - T % wg_ncu();
      maeclip::allow_lds((const void*)wgrad4_kernel<false>, TileM<256>::LDS_ALL);
      hipLaunchKernelGGL(wgrad4_kernel<false>, dim3(wg_ncu()), dim3(512), TileM<256>::LDS_ALL, s, g);
      MC_CHECK_LAUNCH("maeclip_wgrad_grouped(stream-k)");
      hipLaunchKernelGGL(wgrad4_sk_reduce_kernel, dim3(T - g.Tdp, SKR_CHUNKS), dim3(256), 0, s, g);
      MC_CHECK_LAUNCH("maeclip_wgrad_grouped(stream-k reduce)");
      continue;
    }
    g.S = wg_splits(T, M);
    if (g.S > 1) {
      for (int i = 0; i < n; ++i) {
        MC_CHECK_ARG(so < (1ll << 31), "maeclip_wgrad_grouped: workspace offsets exceed 2^31 floats");
        g.p[i].slab_off = (int)so;
        so += (int64_t)g.S * g.p[i].N * g.p[i].K;
      }
    }
    const int units = T * g.S, grid = std::min(units, wg_ncu());
    if (g.S > 1) {
      maeclip::allow_lds((const void*)wgrad4_kernel<true>, TileM<256>::LDS_ALL);
      hipLaunchKernelGGL(wgrad4_kernel<true>, dim3(grid), dim3(512), TileM<256>::LDS_ALL, s, g);
      MC_CHECK_LAUNCH("maeclip_wgrad_grouped");
      int64_t maxnk = 0;
      for (int i = 0; i < n; ++i) maxnk = std::max(maxnk, (int64_t)g.p[i].N * g.p[i].K);
      const int gx = (int)std::min<int64_t>((maxnk / 4 + 255) / 256, 1024);
      hipLaunchKernelGGL(wgrad4_reduce_kernel, dim3(gx, n), dim3(256), 0, s, g);
      MC_CHECK_LAUNCH("maeclip_wgrad_grouped(reduce)");
    } else {
      maeclip::allow_lds((const void*)wgrad4_kernel<false>, TileM<256>::LDS_ALL);
      hipLaunchKernelGGL(wgrad4_kernel<false>, dim3(grid), dim3(512), TileM<256>::LDS_ALL, s, g);
      MC_CHECK_LAUNCH("maeclip_wgrad_grouped");
    }
  }
  return 0;
}
