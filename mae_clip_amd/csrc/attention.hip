// Multi-head attention forward/backward (gfx950 MFMA).
//
// Replaces F.scaled_dot_product_attention inside timm's Attention (ViT encoder
// blocks, timm 0.9.12), HF ViTMAE decoder layers (modeling_vit_mae.py:455-580)
// and DistilBERT's self-attention with additive key-padding mask
// (modeling_distilbert.py:125-145, 174-205).
//
// Input is the fused qkv activation [B*n, ld_qkv] (token rows; q at column
// h*HD, k at H*HD + h*HD, v at 2*H*HD + h*HD) exactly as the qkv GEMM wrote
// it, so no permute/copy kernels sit between the GEMM and attention.
//
// One workgroup (8 waves) owns one (sample, head): the whole K/V (and for the
// backward Q/dO) slice of that head lives in LDS (n <= ~600 tokens fits for
// every config: ViT-B 197/50, decoder 197/577 at HD=32, text 25).
//   forward : waves take 16-query tiles; S^T = K Q^T on MFMA (key on the
//             register axis, query on the lane) -> online softmax entirely
//             lane-local, P stays in registers and feeds P.V as the B operand;
//             V^T fragments come from ds_read_b64_tr_b16.
//   backward: phase 1 -- waves own 16-key tiles, sweep queries: S, dP, then
//             dV^T += dO^T P, dK^T += Q^T dS (accumulator-as-operand, no LDS
//             round trip). phase 2 -- waves own 16-query tiles, sweep keys:
//             S^T, dP^T, dQ^T += K^T dS^T. No atomics, deterministic.
// LDS images (bf16): [rows][HD] with 16-B chunk index XOR-swizzled by f(row)
// = row&6 (HD=64) or (row>>1)&2 (HD=32): conflict-free for both the
// ds_read_b128 row reads and the ds_read_b64_tr_b16 transposed reads
// (checked with tools/lds_bank_sim.py). fp32 parity mode uses padded rows and
// exact-f32 MFMA (v_mfma_f32_16x16x4_f32).
// Softmax statistics are kept in log2 units: lse2 = log2(sum 2^(s*scale*log2e)).
#include "common.h"
#include "../../include/maeclip.h"
#include <type_traits>
#include <stdlib.h>

namespace {

constexpr int MAXW = 8;          // max waves per workgroup (sized per launch to the tile count)
// forward waves per SIMD the register allocator must keep: the bf16 HD 32
// body with the MFMA row sum fits 80 VGPRs (6 waves per SIMD, 3 workgroups of
// 7 waves per CU at n = 197); the others are left to the compiler
template <typename T, int HD, bool DROP> constexpr int fwd_wpe() {
#ifdef FWD_WPE
  return FWD_WPE;
#else
  return (sizeof(T) == 2 && HD == 32 && !DROP) ? 6 : 1;
#endif
}

// Q / K / V / O / dO are read once per (sample, head): non-temporal loads, so
// they do not evict what the next kernels reuse (ATTN_NT=0 turns it off)
#ifndef ATTN_NT
#define ATTN_NT 1
#endif
#if ATTN_NT
#define ANT(p) __builtin_nontemporal_load(p)
#else
#define ANT(p) (*(p))
#endif
#define NW ((int)(blockDim.x >> 6))
#define NTH ((int)blockDim.x)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;

#ifdef ATTN_STAMPS
// diagnostic build only: s_memtime per wave of the first 4096 backward
// workgroups at start / prologue done / phase 1 done / phase 2 start / phase 2
// done / exit
__device__ uint64_t g_attn_stamps[4096 * MAXW * 8];
#define ASTAMP(k) do { if (lane == 0 && blockIdx.x < 4096) g_attn_stamps[((int64_t)blockIdx.x * MAXW + wave) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define ASTAMP(k) do {} while (0)
#endif

template <typename T, int HD> struct Img {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int ROWB = BF ? HD * 2 : HD * 4 + 16;
  __device__ static __forceinline__ int f(int row) { return HD == 64 ? (row & 6) : ((row >> 1) & 2); }
  // byte offset of 16-byte chunk c of a row
  __device__ static __forceinline__ int chunk(int row, int c) {
    return BF ? row * ROWB + ((c ^ f(row)) << 4) : row * ROWB + (c << 4);
  }
  static constexpr int CPR = BF ? HD / 8 : HD / 4;  // 16-B chunks per row
};

// NI head slices of the same token rows (global [n rows, stride ld]) -> NI
// LDS images, zero rows >= n up to npad. Every thread keeps 2*NI 16-B loads in
// flight before it writes LDS (the loop is latency-, not bandwidth-bound).
template <typename T, int HD, int NI>
__device__ __forceinline__ void load_imgs(char* const (&lds)[NI], const T* const (&g)[NI], int64_t ld, int n,
                                          int npad) {
  using I = Img<T, HD>;
  const int total = npad * I::CPR;
  for (int id0 = threadIdx.x; id0 < total; id0 += 2 * NTH) {
    v4u v[2][NI];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = id0 + u * NTH;
      const int row = id / I::CPR, c = id % I::CPR;
      const bool ok = id < total && row < n;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        v[u][i] = ok ? ANT((const v4u*)(g[i] + (int64_t)row * ld + c * (16 / sizeof(T)))) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = id0 + u * NTH;
      const int row = id / I::CPR, c = id % I::CPR;
      if (id < total) {
#pragma unroll
        for (int i = 0; i < NI; ++i) *(v4u*)(lds[i] + I::chunk(row, c)) = v[u][i];
      }
    }
  }
}

// bf16 K / V images by LDS-DMA (buffer_load_dwordx4 ... lds): one
// wave-instruction fills 1 KiB of an image, lane L the 16-B slot L of it, so
// the XOR swizzle goes into the SOURCE address (slot s of row r holds chunk
// s ^ f(r)); rows >= n read as zero through the descriptor's range check (its
// extent ends with row n - 1's slice). No VGPR round trip and no per-chunk
// address VALU beyond one row / chunk split per instruction; the wave waits for
// its own DMA, the caller's barrier for everyone's. ATTN_NT: non-temporal
// (aux bit 1) like the register path's loads.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
#ifndef ATTN_DMA
#define ATTN_DMA 1
#endif
#ifndef ATTN_QIMG
#define ATTN_QIMG 1
#endif
// forward: Q as a third LDS image (bf16 DMA path) only while two workgroups
// per CU still fit with it: with one, the longer prologue has nothing to
// overlap (C1 encoder n = 197 at hd 64: 95.6 -> 116.2 us; C4 decoder n = 577:
// 233 -> 249 us), with two it saves a global round trip per query tile (C2
// decoder 74.2 -> 67.6 us, C4 encoder 49.9 -> 47.3; profiles/r06/attn_fwd_qimg_ab_r6aa.txt)
template <typename T, int HD> __host__ __device__ __forceinline__ bool fwd_qimg(int npad) {
  return std::is_same<T, bf16_t>::value && ATTN_DMA && ATTN_QIMG &&
         2 * (3 * npad * Img<T, HD>::ROWB + npad * 4) <= 163840;
}

template <int HD, int NI>
__device__ __forceinline__ void dma_imgs(char* const (&dst)[NI], const bf16_t* const (&src)[NI], int64_t ld, int n,
                                         int npad) {
  using I = Img<bf16_t, HD>;
  const int64_t span = ((int64_t)(n - 1) * ld + HD) * 2;
  const int nrec = (int)(span < 0x7fffffff ? span : 0x7fffffff);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nw = (int)(blockDim.x >> 6);
  const int ninst = npad * I::CPR / 64;   // npad is a multiple of 64
  for (int k = wave; k < ninst; k += nw) {
    const int id = k * 64 + lane;
    const int row = id / I::CPR, sl = id % I::CPR;
    const int voff = row * (int)ld * 2 + ((sl ^ I::f(row)) << 4);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src[i], (short)0, nrec, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst[i] + k * 1024), 16, voff, 0, 0, ATTN_NT ? 2 : 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// dot product of two 16-B chunks in f32
template <typename T> __device__ __forceinline__ float chunk_dot(v4u a, v4u b);
template <> __device__ __forceinline__ float chunk_dot<bf16_t>(v4u a, v4u b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s = fmaf(__uint_as_float(a[j] << 16), __uint_as_float(b[j] << 16), s);
    s = fmaf(__uint_as_float(a[j] & 0xffff0000u), __uint_as_float(b[j] & 0xffff0000u), s);
  }
  return s;
}
template <> __device__ __forceinline__ float chunk_dot<float>(v4u a, v4u b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s = fmaf(__uint_as_float(a[j]), __uint_as_float(b[j]), s);
  return s;
}

// Backward prologue: Q, K, V, dO images + Dv[q] = -rowsum(dO * O) (f32) +
// L2[q] = -lse / c (-1e30 on padding rows), all rows in one pass with every load of an iteration in flight.
// A row's CPR chunks sit on CPR consecutive lanes of one wave (CPR | 64, NTH a
// multiple of 64, total a multiple of 64), so the row sum is an xor-shuffle.
template <typename T, int HD, bool KV>
__device__ __forceinline__ void bwd_prologue(char* Qi, char* Ki, char* Vi, char* Di, float* L2, float* Dv,
                                             const T* q, const T* k, const T* v, int64_t ld_qkv, const T* O,
                                             const T* dO, int64_t ld_o, const float* lse, float inv_c, int n,
                                             int npad) {
  using I = Img<T, HD>;
  constexpr int CPR = I::CPR, EPC = 16 / (int)sizeof(T);
  const int total = npad * CPR;
  for (int id0 = threadIdx.x; id0 < total; id0 += 2 * NTH) {
    v4u vq[2], vk[2], vv[2], vd[2], vo[2];
    float ls[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = id0 + u * NTH;
      const int row = id / CPR, c = id % CPR;
      const bool ok = id < total && row < n;
      const int64_t oq = (int64_t)row * ld_qkv + c * EPC, oo = (int64_t)row * ld_o + c * EPC;
      const v4u z = {0, 0, 0, 0};
      vq[u] = ok ? ANT((const v4u*)(q + oq)) : z;
      if (KV) {
        vk[u] = ok ? ANT((const v4u*)(k + oq)) : z;
        vv[u] = ok ? ANT((const v4u*)(v + oq)) : z;
      }
      vd[u] = ok ? ANT((const v4u*)(dO + oo)) : z;
      vo[u] = ok ? ANT((const v4u*)(O + oo)) : z;
      ls[u] = (ok && c == 0) ? -lse[row] * inv_c : -1.0e30f;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = id0 + u * NTH;
      if (id >= total) break;  // wave-uniform
      const int row = id / CPR, c = id % CPR;
      *(v4u*)(Qi + I::chunk(row, c)) = vq[u];
      if (KV) {
        *(v4u*)(Ki + I::chunk(row, c)) = vk[u];
        *(v4u*)(Vi + I::chunk(row, c)) = vv[u];
      }
      *(v4u*)(Di + I::chunk(row, c)) = vd[u];
      float d = chunk_dot<T>(vd[u], vo[u]);
#pragma unroll
      for (int o = 1; o < CPR; o <<= 1) d += __shfl_xor(d, o, 64);
      if (c == 0) {
        Dv[row] = -d;
        L2[row] = ls[u];
      }
    }
  }
}

// ---- row fragment: 8 consecutive d (d = 32ks + 8g + j) of LDS row r0 + (lane&15)
template <typename T, int HD> struct RowFrag;
template <int HD> struct RowFrag<bf16_t, HD> {
  v8s v;
  __device__ __forceinline__ void lds(const char* img, int r0, int ks, int lane) {
    const int row = r0 + (lane & 15);
    v = *(const v8s*)(img + Img<bf16_t, HD>::chunk(row, 4 * ks + (lane >> 4)));
  }
  __device__ __forceinline__ void glob(const bf16_t* p, int ks, int lane, bool ok) {
    v = ok ? ANT((const v8s*)(p + 32 * ks + 8 * (lane >> 4))) : v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
};
template <int HD> struct RowFrag<float, HD> {
  float v[8];
  __device__ __forceinline__ void lds(const char* img, int r0, int ks, int lane) {
    const int row = r0 + (lane & 15);
    const int c0 = 8 * ks + 2 * (lane >> 4);
    v4f a = *(const v4f*)(img + Img<float, HD>::chunk(row, c0));
    v4f b = *(const v4f*)(img + Img<float, HD>::chunk(row, c0 + 1));
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
  __device__ __forceinline__ void glob(const float* p, int ks, int lane, bool ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ok ? p[32 * ks + 8 * (lane >> 4) + j] : 0.f;
  }
};

// D += X Y over a 32-deep k-step; X, Y row fragments (X rows on lane for A operand).
__device__ __forceinline__ v4f mma32(const RowFrag<bf16_t, 64>& x, const RowFrag<bf16_t, 64>& y, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.v, y.v, c, 0, 0, 0);
}
__device__ __forceinline__ v4f mma32(const RowFrag<bf16_t, 32>& x, const RowFrag<bf16_t, 32>& y, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.v, y.v, c, 0, 0, 0);
}
template <int HD>
__device__ __forceinline__ v4f mma32(const RowFrag<float, HD>& x, const RowFrag<float, HD>& y, v4f c) {
#pragma unroll
  for (int s = 0; s < 8; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(x.v[s], y.v[s], c, 0, 0, 0);
  return c;
}

// bf16 transposed fragment: element j <-> row rb + 16*(j>>2) + 4*g + (j&3),
// column c0 + (lane&15): the A operand "X^T" of a product that sums over rows.
template <int HD>
__device__ __forceinline__ v8s tr_frag(const char* img, int rb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int unit = (c0 >> 2) + p;  // 8-byte unit within the row
  v8s r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = rb + 16 * h + 4 * g + q;
    const char* a = img + Img<bf16_t, HD>::chunk(row, unit >> 1) + ((unit & 1) << 3);
    v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, a));
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * h + e] = t[e];
  }
  return r;
}
__device__ __forceinline__ v8s pack_p(const v4f& a, const v4f& b) {
  // four v_cvt_pk_bf16_f32 (RNE), one per pair
  const v4u u = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(v8s, u);
}

// D[c][col] += sum over 32 rows (rb..rb+31) of X[row][c] * P[row][col], where
// P is held as two accumulator tiles (rows rb+4g+i and rb+16+4g+i on lane col).
template <typename T, int HD>
__device__ __forceinline__ v4f mma_rowsum(const char* img, int rb, int c0, const v4f& p0, const v4f& p1,
                                          v4f acc, int lane) {
  if constexpr (std::is_same<T, bf16_t>::value) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag<HD>(img, rb, c0, lane), pack_p(p0, p1), acc, 0, 0, 0);
  } else {
    const int g = lane >> 4, col = c0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x0 = *(const float*)(img + (rb + 4 * g + i) * Img<float, HD>::ROWB + col * 4);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, p0[i], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x1 = *(const float*)(img + (rb + 16 + 4 * g + i) * Img<float, HD>::ROWB + col * 4);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x1, p1[i], acc, 0, 0, 0);
    }
    return acc;
  }
}

__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t bh, int q, int k, uint32_t thr) {
  return mc_hash4(seed, bh, (uint64_t)q, (uint64_t)k) >= thr;
}

// ============================================================== forward
// max over the four 16-lane rows (the lanes l, l^16, l^32, l^48 of a query):
// two permlane swaps (VALU) instead of two ds_bpermute round trips
// (ATTN_RAWMAX: a plain v_max_f32 of the two halves -- fmaxf would first
// canonicalise each permlane result, two more VALU ops per swap; the scores
// are never signalling NaNs)
#ifndef ATTN_RAWMAX
#define ATTN_RAWMAX 0   // measured: the asm pins the schedule (C4 decoder fwd 255 -> 280 us)
#endif
__device__ __forceinline__ float vmax_raw(float a, float b) {
#if ATTN_RAWMAX
  float r;
  asm volatile("v_max_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmaxf(a, b);
#endif
}
__device__ __forceinline__ float max4rows(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = vmax_raw(__uint_as_float(p[0]), __uint_as_float(p[1]));
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum4rows(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct FwdDrop {
  uint64_t seed, bh;
  uint32_t thr;
  float scale;
};

// One 64-key chunk of a 16-query tile with its shape fixed at compile time, so
// the body is straight-line code the scheduler can interleave (the runtime
// per-32-key / mask / dropout branches of a generic body split it into ~30
// basic blocks with an MFMA or a few VALU ops each). NT: 16-key S tiles that
// hold real keys (4 for a whole chunk; the tail chunk of n = 197, keys
// 192..196, runs one tile instead of two -- its PV product takes a zero
// second half); MASKED: add the key bias (padding keys, DistilBERT's key mask)
// -- the scale c > 0 then rides in the bias fma, otherwise in the exponent's
// fma and the running max is taken on the raw scores.
// bf16 without dropout: the row sum of P comes out of the MFMA as a
// 17th..32nd "V column" of ones (lsum accumulator `ol`, every element the
// lane's query's sum of the bf16 P the PV product uses) instead of 16 VALU
// adds per chunk -- the kernel is VALU-bound at HD 32, the MFMA pipe is not;
// lsum is then the exact weight sum of O = sum P V (both over bf16(P)).
// With dropout the normalisation needs the sum BEFORE the mask: VALU adds.
// bf16 rescales lazily: the running max m only moves (alpha exp + the O / lsum
// multiplies) when some query of the wave sees a chunk max more than LAZY_TH
// (log2 units) above it; otherwise P = exp2(s' - m) <= 2^LAZY_TH. bf16(P) has
// the same relative rounding at any exponent, O and lsum accumulate in f32,
// and lse = m + log2(lsum) holds for any m, so only the f32 roundings of the
// final O / lsum change. Wave-uniform branch (ballot), taken on the first
// chunk (m = -1e30) and then rarely.
#ifndef LAZY_TH
#define LAZY_TH 8.0f
#endif
#ifndef ATTN_BWD_FLAGS
#define ATTN_BWD_FLAGS 1
#endif
// HD 32 with the round flags: each wave fills its own 32-row chunk of the Q /
// dO images, Dv, L2 and the dQ image and publishes it; no prologue barrier
#ifndef ATTN_BWD_CHUNKED
#define ATTN_BWD_CHUNKED 0   // measured: decoder bwd 186.4 -> 191.8 us (bitwise-identical): opt-in
#endif
#ifndef ATTN_PKFMA
#define ATTN_PKFMA 0   // measured: neutral to -3 % (dec 75 -> 77-80 us)
#endif
#ifndef ATTN_LAZY
#define ATTN_LAZY 0   // measured slower (the branch splits the chunk body): opt-in
#endif
template <typename T, int HD, int NT, bool MASKED, bool DROP>
__device__ __forceinline__ void fwd_chunk(const char* Kimg, const char* Vimg, const float* kmask, int kc,
                                          const RowFrag<T, HD> (&qf)[HD / 32], float c, float& m, float& lsum,
                                          v4f (&o)[HD / 16], v4f& ol, int lane, const FwdDrop& dr, int q) {
  constexpr bool BF = std::is_same<T, bf16_t>::value;
  constexpr bool MSUM = BF && !DROP;
  constexpr int NP = (NT + 1) / 2;   // 32-key halves of the PV product
  const int g = lane >> 4;
  v4f s[2 * NP];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    s[t] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HD / 32; ++ks) {
      RowFrag<T, HD> kf;
      kf.lds(Kimg, kc + 16 * t, ks, lane);
      s[t] = mma32(kf, qf[ks], s[t]);
    }
  }
  float mloc = NEG_BIG;
  if (MASKED) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const v4f km = *(const v4f*)(kmask + kc + 16 * t + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[t][i] = fmaf(s[t][i], c, km[i]);
        mloc = fmaxf(mloc, s[t][i]);
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) mloc = fmaxf(mloc, s[t][i]);
    mloc *= c;
  }
  mloc = max4rows(mloc);
  float lsc = 1.f;
  bool resc = true;
  if (BF && ATTN_LAZY) resc = __builtin_amdgcn_ballot_w64(mloc > m + LAZY_TH) != 0;
  if (resc) {
    const float mnew = fmaxf(m, mloc);
    lsc = __builtin_amdgcn_exp2f(m - mnew);
    if (MSUM) ol[0] *= lsc;   // only element 0 is read back
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[dt] *= lsc;
    m = mnew;
  }
  const float cc = MASKED ? 1.f : c, nm = -m;
  float lp = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#if ATTN_PKFMA   // exponent arguments of a value pair in one v_pk_fma_f32 (A/B builds)
    if (MSUM) {
      typedef float f2_t __attribute__((ext_vector_type(2)));
      const f2_t c2 = {cc, cc}, n2 = {nm, nm};
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const f2_t e = __builtin_elementwise_fma(f2_t{s[t][i], s[t][i + 1]}, c2, n2);
        s[t][i] = __builtin_amdgcn_exp2f(e[0]);
        s[t][i + 1] = __builtin_amdgcn_exp2f(e[1]);
      }
      continue;
    }
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = __builtin_amdgcn_exp2f(fmaf(s[t][i], cc, nm));
      if (!MSUM) lp += p;
      s[t][i] = p;
    }
  }
  if (NT & 1) s[NT] = v4f{0.f, 0.f, 0.f, 0.f};
  if (!MSUM) lsum = fmaf(lsum, lsc, lp);
  if (DROP) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kc + 16 * t + 4 * g + i;
        s[t][i] = dropout_keep(dr.seed, dr.bh, q, key, dr.thr) ? s[t][i] * dr.scale : 0.f;
      }
  }
#pragma unroll
  for (int s2 = 0; s2 < NP; ++s2) {
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
      o[dt] = mma_rowsum<T, HD>(Vimg, kc + 32 * s2, 16 * dt, s[2 * s2], s[2 * s2 + 1], o[dt], lane);
    if constexpr (MSUM) {
      const v8s ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
      ol = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pack_p(s[2 * s2], s[2 * s2 + 1]), ol, 0, 0, 0);
    }
  }
}

// fp8-blocks copy (maeclip_attn_args q8) of the HD columns [col0, col0 + HD)
// of output row `row` this lane's 16-row tile stores: lane (row, g = lane / 16)
// holds v[dt] = columns 16 dt + 4 g .. +3 as stored in bf16, so the 32-column
// block j is dt = 2j, 2j + 1 of the four lanes l % 16 + 16 g: its amax is two
// permlane swaps (every lane of the wave takes part; `ok` gates the stores).
template <int HD>
__device__ __forceinline__ void q8_store(const maeclip_attn_args& a, int64_t row, bool ok, int col0, int rowlen,
                                         const v4f (&v)[HD / 16], int lane) {
  const int g = lane >> 4;
  const bool e5 = a.q8_fmt == MAECLIP_FP8_E5M2;
#pragma unroll
  for (int j = 0; j < HD / 32; ++j) {
    float x[8], am = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] = bf2f(f2bf(v[2 * j][i]));
      x[4 + i] = bf2f(f2bf(v[2 * j + 1][i]));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(x[i]));
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(am), __float_as_uint(am), false, false);
    am = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    p = __builtin_amdgcn_permlane32_swap(__float_as_uint(am), __float_as_uint(am), false, false);
    am = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    const unsigned ex = mc_e8m0(am, e5);
    const float inv = mc_e8m0_inv(ex);
    if (ok) {
      uint8_t* q = (uint8_t*)a.q8 + row * a.ldq8 + col0 + 32 * j + 4 * g;
      unsigned w0, w1;
      if (e5) {
        w0 = mc_cvt4_fp8<true>(x[0] * inv, x[1] * inv, x[2] * inv, x[3] * inv);
        w1 = mc_cvt4_fp8<true>(x[4] * inv, x[5] * inv, x[6] * inv, x[7] * inv);
      } else {
        w0 = mc_cvt4_fp8<false>(x[0] * inv, x[1] * inv, x[2] * inv, x[3] * inv);
        w1 = mc_cvt4_fp8<false>(x[4] * inv, x[5] * inv, x[6] * inv, x[7] * inv);
      }
      *(unsigned*)q = w0;
      *(unsigned*)(q + 16) = w1;
      if (g == 0) a.q8_scale[mc_fp8b_off(row, (col0 >> 5) + j, rowlen >> 7)] = (uint8_t)ex;
    }
  }
}

// WG = 16: up to 16 waves when the K / V images leave room for one workgroup
// per CU only (the C4 decoder, n = 577: 37 query tiles in 3 rounds of 13
// waves instead of 5 rounds of 8)
template <int A, int B> constexpr int cmax() { return A > B ? A : B; }
// Q8: the fp8-blocks copy of o (maeclip_attn_args q8) from the kernel's own
// stores -- its own instantiation, so the plain kernels keep their registers
// QI: Q as a third LDS image (fwd_qimg; bf16, 8-wave launches only)
template <typename T, int HD, bool DROP, int WG = MAXW, bool Q8 = false, bool QI = false>
__global__ void __launch_bounds__(WG * 64)
__attribute__((amdgpu_waves_per_eu(WG > MAXW ? cmax<fwd_wpe<T, HD, DROP>(), 4>() : fwd_wpe<T, HD, DROP>())))
attn_fwd_kernel(const maeclip_attn_args a) {
  static_assert(!QI || (std::is_same<T, bf16_t>::value && WG == MAXW), "QI: bf16, 8-wave launches");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using I = Img<T, HD>;
  const int n = a.n, H = a.H;
  const int bid = xcd_chunk_id(blockIdx.x, gridDim.x);
  const int b = bid / H, h = bid % H;
  const int npad = (n + 63) & ~63;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  ASTAMP(0);
  char* Kimg = smem;
  char* Vimg = smem + npad * I::ROWB;
  float* kmask = (float*)(smem + 2 * npad * I::ROWB);

  const T* qkv = (const T*)a.qkv + (int64_t)b * n * a.ld_qkv;
  const int HH = H * HD;
  // bf16: the Q rows come as a third LDS image with K and V when two
  // workgroups per CU still fit (fwd_qimg), so a query tile reads its Q
  // fragments from LDS instead of a global round trip per tile
  constexpr bool qimg = QI;
  char* Qimg = smem + 2 * npad * I::ROWB + npad * 4;
  if constexpr (qimg) {
    char* const dst[3] = {Kimg, Vimg, Qimg};
    const bf16_t* const src[3] = {(const bf16_t*)qkv + HH + h * HD, (const bf16_t*)qkv + 2 * HH + h * HD,
                                  (const bf16_t*)qkv + h * HD};
    dma_imgs<HD, 3>(dst, src, a.ld_qkv, n, npad);
  } else if constexpr (std::is_same<T, bf16_t>::value && ATTN_DMA) {
    char* const dst[2] = {Kimg, Vimg};
    const bf16_t* const src[2] = {qkv + HH + h * HD, qkv + 2 * HH + h * HD};
    dma_imgs<HD, 2>(dst, src, a.ld_qkv, n, npad);
  } else {
    char* const dst[2] = {Kimg, Vimg};
    const T* const src[2] = {qkv + HH + h * HD, qkv + 2 * HH + h * HD};
    load_imgs<T, HD, 2>(dst, src, a.ld_qkv, n, npad);
  }
  for (int k = threadIdx.x; k < npad; k += NTH) {
    float mk = (k < n) ? 0.f : NEG_BIG;
    if (k < n && a.key_mask && a.key_mask[(int64_t)b * n + k] == 0.f) mk = NEG_BIG;
    kmask[k] = mk;
  }
  __syncthreads();
  ASTAMP(1);

  const float c = a.scale * LOG2E;
  FwdDrop dr{};
  if (DROP) {
    dr.seed = mc_step_seed(a.seed, a.step_ptr);
    dr.bh = (uint64_t)b * H + h;
    dr.thr = (uint32_t)((double)a.dropout_p * 4294967296.0);
    dr.scale = 1.f / (1.f - a.dropout_p);
  }
  // chunks whose 64 keys are all real and unmasked run the bias-free body
  const int nfull = a.key_mask ? 0 : n >> 6;

  const int nqt = (n + 15) >> 4;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int q = qt * 16 + (lane & 15);
    const bool qok = q < n;
    RowFrag<T, HD> qf[HD / 32];
#pragma unroll
    for (int ks = 0; ks < HD / 32; ++ks) {
      if constexpr (qimg) qf[ks].lds(Qimg, qt * 16, ks, lane);
      else qf[ks].glob(qkv + (int64_t)q * a.ld_qkv + h * HD, ks, lane, qok);
    }

    float m = NEG_BIG, lsum = 0.f;
    v4f o[HD / 16], ol = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};

    int kc = 0;
    for (; kc < 64 * nfull; kc += 64)
      fwd_chunk<T, HD, 4, false, DROP>(Kimg, Vimg, kmask, kc, qf, c, m, lsum, o, ol, lane, dr, q);
    for (; kc < npad; kc += 64) {
      // 16-key tiles of this chunk that hold real keys (wave-uniform; n > kc)
      const int rem = n - kc;
      if (rem > 48) fwd_chunk<T, HD, 4, true, DROP>(Kimg, Vimg, kmask, kc, qf, c, m, lsum, o, ol, lane, dr, q);
      else if (rem > 32) fwd_chunk<T, HD, 3, true, DROP>(Kimg, Vimg, kmask, kc, qf, c, m, lsum, o, ol, lane, dr, q);
      else if (rem > 16) fwd_chunk<T, HD, 2, true, DROP>(Kimg, Vimg, kmask, kc, qf, c, m, lsum, o, ol, lane, dr, q);
      else fwd_chunk<T, HD, 1, true, DROP>(Kimg, Vimg, kmask, kc, qf, c, m, lsum, o, ol, lane, dr, q);
    }
    // the MFMA row sum (bf16, no dropout) is whole in every lane of the query
    if (std::is_same<T, bf16_t>::value && !DROP) lsum = ol[0];
    else lsum = sum4rows(lsum);
    const float inv = 1.f / lsum;
    if constexpr (Q8 && std::is_same<T, bf16_t>::value) {
      {
        v4f ov[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) ov[dt] = o[dt] * inv;
        q8_store<HD>(a, (int64_t)b * n + q, qok, h * HD, HH, ov, lane);
      }
    }
    if (qok) {
      T* orow = (T*)a.o + ((int64_t)b * n + q) * a.ld_o + h * HD;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) st4<T>(orow + 16 * dt + 4 * g, o[dt] * inv);
      if (g == 0 && a.lse) a.lse[((int64_t)b * H + h) * n + q] = m + log2f(lsum);
    }
    if (qt == wave) ASTAMP(2);
  }
  ASTAMP(3);
}

// ============================================================== backward
// TWO_ (bf16; always on for fp32): two [npad][HD] images in LDS instead of four --
// phase 1 keeps Q, dO and reads each wave's K/V tile from HBM, phase 2 reloads
// the slots with K, V. Chosen when it fits more workgroups per CU (C4: decoder
// n = 577, encoder n = 145 at HD = 64).
// OCC > 1 asks the compiler for that many resident 8-wave workgroups per CU
// (register budget 512 / (2 OCC)); used with TWO_ at HD = 32, where the
// two-image LDS footprint would allow three.
// WG = 16: up to 16 waves in the one workgroup a CU holds (the C4 decoder,
// n = 577: 37 tiles, at most 3 per wave instead of 5; register budget 128).
template <typename T, int HD, bool TWO_ = false, int OCC = 1, int WG = MAXW, bool Q8 = false>
__global__ void __launch_bounds__(WG * 64) __attribute__((amdgpu_waves_per_eu(WG > MAXW ? 4 : 2 * OCC)))
attn_bwd_kernel(const maeclip_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using I = Img<T, HD>;
  const int n = a.n, H = a.H;
  const int bid = xcd_chunk_id(blockIdx.x, gridDim.x);
  const int b = bid / H, h = bid % H;
  const int npad = (n + 31) & ~31;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  ASTAMP(0);
  // bf16: Q, K, V, dO images resident together. fp32 parity mode (rows twice
  // as wide) holds two at a time so that n = 197 at HD = 64 fits: phase 1
  // keeps Q, dO in LDS and reads each wave's K/V tile from HBM, phase 2
  // reloads the two slots with K, V and reads Q/dO tiles from HBM.
  constexpr bool TWO = TWO_ || !std::is_same<T, bf16_t>::value;
  const int img = npad * I::ROWB;
  char* Qi = smem;
  char* Di = smem + (TWO ? 1 : 3) * img;
  char* Ki = TWO ? smem : smem + img;
  char* Vi = TWO ? smem + img : smem + 2 * img;
  float* L2 = (float*)(smem + (TWO ? 2 : 4) * img);
  float* Dv = L2 + npad;
  float* cs = Dv + npad;  // [NW][3*HD] bias-grad partials

  const int HH = H * HD;
  const T* qkv = (const T*)a.qkv + (int64_t)b * n * a.ld_qkv;
  const T* O = (const T*)a.o + (int64_t)b * n * a.ld_o + h * HD;
  const T* dO = (const T*)a.dout + (int64_t)b * n * a.ld_o + h * HD;
  bwd_prologue<T, HD, !TWO>(Qi, Ki, Vi, Di, L2, Dv, qkv + h * HD, qkv + HH + h * HD, qkv + 2 * HH + h * HD, a.ld_qkv,
                            O, dO, a.ld_o, a.lse + ((int64_t)b * H + h) * n, 1.f / (a.scale * LOG2E), n, npad);
  for (int i = threadIdx.x; i < NW * 3 * HD; i += NTH) cs[i] = 0.f;
  const int nkt = (n + 15) >> 4;
  __syncthreads();
  ASTAMP(1);
  if (a.colsum_partial && threadIdx.x < NW * HD) {
    // v-bias gradient: sum over keys of dV = sum over queries of dO (softmax
    // rows sum to 1; the backward runs without attention dropout). Row group
    // r0 of column d -> cs[r0][2 HD + d]; the k-bias gradient is identically
    // zero (softmax is invariant to a per-query constant) and stays 0.
    constexpr int EPC = 16 / (int)sizeof(T);
    const int d = threadIdx.x % HD, r0 = threadIdx.x / HD;
    float sv = 0.f;
    for (int r = r0; r < n; r += NW)
      sv += ld_as_f<T>((const T*)(Di + I::chunk(r, d / EPC) + (d % EPC) * (int)sizeof(T)));
    cs[r0 * 3 * HD + 2 * HD + d] = sv;
  }

  const float c = a.scale * LOG2E;
  T* dqkv = (T*)a.dqkv + (int64_t)b * n * a.ld_dqkv;

  // ---------------- phase 1: dK, dV (wave owns 16-key tiles)
  for (int kt = wave; kt < nkt; kt += NW) {
    const int k0 = kt * 16;
    const int key = k0 + (lane & 15);
    const bool kok = key < n;
    RowFrag<T, HD> kf[HD / 32], vf[HD / 32];
#pragma unroll
    for (int ks = 0; ks < HD / 32; ++ks) {
      if (TWO) {
        const T* kr = qkv + (int64_t)(kok ? key : 0) * a.ld_qkv + HH + h * HD;
        kf[ks].glob(kr, ks, lane, kok);
        vf[ks].glob(kr + HH, ks, lane, kok);
      } else {
        kf[ks].lds(Ki, k0, ks, lane);
        vf[ks].lds(Vi, k0, ks, lane);
      }
    }
    v4f dv[HD / 16], dk[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) { dv[dt] = v4f{0, 0, 0, 0}; dk[dt] = v4f{0, 0, 0, 0}; }

    for (int qc = 0; qc < npad; qc += 32) {
      v4f P[2], dS[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q0 = qc + 16 * u;
        // row constants as the initial accumulators: s' = S - lse/c, dp' = dP - Dv
        v4f s = *(const v4f*)(L2 + q0 + 4 * g), dp = *(const v4f*)(Dv + q0 + 4 * g);
#pragma unroll
        for (int ks = 0; ks < HD / 32; ++ks) {
          RowFrag<T, HD> qf, df;
          qf.lds(Qi, q0, ks, lane);
          df.lds(Di, q0, ks, lane);
          s = mma32(qf, kf[ks], s);    // S[q=4g+i][key=lane&15]
          dp = mma32(df, vf[ks], dp);  // dP[q][key]
        }
        // padding keys (lane >= n) only pollute their own dK/dV columns, which
        // are never stored; padding queries have p = 0 (L2 = -1e30)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(s[i] * c);
          P[u][i] = p;
          dS[u][i] = p * dp[i];
        }
      }
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        dv[dt] = mma_rowsum<T, HD>(Di, qc, 16 * dt, P[0], P[1], dv[dt], lane);
        dk[dt] = mma_rowsum<T, HD>(Qi, qc, 16 * dt, dS[0], dS[1], dk[dt], lane);
      }
    }
    // lane holds dV[key][16dt+4g+i], dK likewise
    if constexpr (Q8 && std::is_same<T, bf16_t>::value) {
      {
        v4f kv[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) kv[dt] = dk[dt] * a.scale;
        q8_store<HD>(a, (int64_t)b * n + key, kok, HH + h * HD, 3 * HH, kv, lane);
        q8_store<HD>(a, (int64_t)b * n + key, kok, 2 * HH + h * HD, 3 * HH, dv, lane);
      }
    }
    if (kok) {
      T* rowp = dqkv + (int64_t)key * a.ld_dqkv + h * HD;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        st4<T>(rowp + HH + 16 * dt + 4 * g, dk[dt] * a.scale);
        st4<T>(rowp + 2 * HH + 16 * dt + 4 * g, dv[dt]);
      }
    }
  }

  ASTAMP(2);
  if (TWO) {
    // phase-1 reads of the Q / dO images are done: K, V take their slots
    __syncthreads();
    char* const dst[2] = {Ki, Vi};
    const T* const src[2] = {qkv + HH + h * HD, qkv + 2 * HH + h * HD};
    load_imgs<T, HD, 2>(dst, src, a.ld_qkv, n, npad);
    __syncthreads();
  }
  // ---------------- phase 2: dQ (wave owns 16-query tiles)
  ASTAMP(3);
  float cq[HD / 16][4];  // per-lane running sum of this wave's dQ rows (q-bias gradient)
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) cq[dt][i] = 0.f;
  for (int qt = wave; qt < nkt; qt += NW) {
    const int q0 = qt * 16;
    const int q = q0 + (lane & 15);
    const bool qok = q < n;
    v4f dq[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = v4f{0, 0, 0, 0};
    RowFrag<T, HD> qf[HD / 32], df[HD / 32];
#pragma unroll
    for (int ks = 0; ks < HD / 32; ++ks) {
      if (TWO) {
        qf[ks].glob(qkv + (int64_t)(qok ? q : 0) * a.ld_qkv + h * HD, ks, lane, qok);
        df[ks].glob(dO + (int64_t)(qok ? q : 0) * a.ld_o, ks, lane, qok);
      } else {
        qf[ks].lds(Qi, q0, ks, lane);
        df[ks].lds(Di, q0, ks, lane);
      }
    }
    const float lq = L2[q], dq_ = Dv[q];
    for (int kc = 0; kc < npad; kc += 32) {
      v4f dST[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kb = kc + 16 * u;
        v4f s = {lq, lq, lq, lq}, dp = {dq_, dq_, dq_, dq_};
#pragma unroll
        for (int ks = 0; ks < HD / 32; ++ks) {
          RowFrag<T, HD> kf, vf;
          kf.lds(Ki, kb, ks, lane);
          vf.lds(Vi, kb, ks, lane);
          s = mma32(kf, qf[ks], s);    // S^T[key=4g+i][q=lane&15]
          dp = mma32(vf, df[ks], dp);  // dP^T
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dST[u][i] = __builtin_amdgcn_exp2f(s[i] * c) * dp[i];
        // padding keys (last chunk only): K rows are zero, but an overflowing
        // exp2(-lse) would turn 0 * inf into NaN in dQ, so zero them explicitly
        if (kb + 16 > n) {
#pragma unroll
          for (int i = 0; i < 4; ++i) dST[u][i] = (kb + 4 * g + i < n) ? dST[u][i] : 0.f;
        }
      }
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = mma_rowsum<T, HD>(Ki, kc, 16 * dt, dST[0], dST[1], dq[dt], lane);
    }
    if constexpr (Q8 && std::is_same<T, bf16_t>::value) {
      {
        v4f qv[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) qv[dt] = dq[dt] * a.scale;
        q8_store<HD>(a, (int64_t)b * n + q, qok, h * HD, 3 * HH, qv, lane);
      }
    }
    if (qok) {
      T* rowp = dqkv + (int64_t)q * a.ld_dqkv + h * HD;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) st4<T>(rowp + 16 * dt + 4 * g, dq[dt] * a.scale);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) cq[dt][i] += dq[dt][i];
    }
  }
  if (a.colsum_partial) {
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sq = cq[dt][i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) sq += __shfl_xor(sq, o, 64);
        if ((lane & 15) == 0) cs[wave * 3 * HD + 16 * dt + 4 * g + i] = sq * a.scale;
      }
  }
  ASTAMP(4);
  if (a.colsum_partial) {
    __syncthreads();
    // colsum_partial row b: [3*H*HD], this head's q/k/v column slices
    for (int i = threadIdx.x; i < 3 * HD; i += NTH) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += cs[w * 3 * HD + i];
      const int part = i / HD, d = i % HD;
      a.colsum_partial[(int64_t)b * 3 * HH + part * HH + h * HD + d] = s;
    }
  }
  ASTAMP(5);
}

// ======================================================= backward, diagonal
// bf16, HD = 32 with npad <= 256 (the C2/C3 MAE decoder: n = 197) and HD = 64
// with npad <= 224 (the ViT encoders: C1 n = 197, C2 n = 50, C4 n = 145): one pass
// instead of two. Wave w owns key chunk w (32 keys, K/V fragments in
// registers) and in round r works query chunk c = (w + r) % NC, so in every
// round each query chunk is touched by exactly one wave. Per (key chunk, query
// chunk) block it computes S, dP, P, dS once, accumulates dK/dV in registers,
// transposes dS through a 2 KB per-wave LDS tile (ds_read_b64_tr_b16) and adds
// dQ^T = K^T dS^T into an fp32 dQ image in LDS (read-modify-write by the one
// wave that owns the chunk this round; a barrier ends the round). The order
// in which the waves add to a query chunk is fixed by the schedule, so the
// result is deterministic, and S / dP / exp are not recomputed for dQ.
// LDS: Q, dO images, L2 / Dv, dQ f32 [npad][HD] (16-B chunks XOR-swizzled by
// the row), NW dS tiles, bias partials: ~78 KB at n = 197, HD = 32 (two
// workgroups per CU); ~142 KB at HD = 64 (one).
// dQ image: HD f32 per row, 16-B chunk ^ (row & 7) (128-B rows) / (row & 15)
// (256-B rows): conflict-free b128 reads and writes of the (16 rows x 4
// chunks) tiles of one MFMA output
template <int HD> __device__ __forceinline__ int dq_off(int row, int c16) {
  return row * (4 * HD) + ((c16 ^ (row & (HD / 4 - 1))) << 4);
}
// dS tile [32 keys][32 q] bf16, 64-B rows, 8-B unit ^ F(row) with F linear in
// row bits 1..3 (found by tools/lds_bank_sim.py): conflict-free for both the
// ds_write_b64 of the MFMA output (row = key, unit = 4u + g) and the
// ds_read_b64_tr_b16 of the dQ B operand
__device__ __forceinline__ int dst_off(int row, int unit) {
  const int f = ((row >> 1) & 1) ^ (((row >> 2) & 1) << 2) ^ (((row >> 3) & 1) << 1);
  return row * 64 + ((unit ^ f) << 3);
}
// B operand dS^T[key][q] for keys 0..31 (permuted order of pack_p), q = c0 + (lane & 15)
__device__ __forceinline__ v8s dst_frag(const char* t, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  v8s r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    v4s x = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, t + dst_off(16 * h + 4 * g + q, (c0 >> 2) + p)));
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * h + e] = x[e];
  }
  return r;
}

// 8 f32 -> the v8s bf16 operand (elements 0-3 from a, 4-7 from b), one
// v_cvt_pk_bf16_f32 per pair and no lane shuffles
__device__ __forceinline__ v8s pack8(const v4f& a, const v4f& b) {
  const v4u u = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(v8s, u);
}

template <int HD>
__global__ void __launch_bounds__(MAXW * 64) __attribute__((amdgpu_waves_per_eu(HD == 32 ? 4 : 2)))
attn_bwd_diag_kernel(const maeclip_attn_args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = HD / 32, DT = HD / 16, CPR = HD / 8, ROWB = Img<bf16_t, HD>::ROWB, DQB = 4 * HD;
  using I = Img<bf16_t, HD>;
  const int n = a.n, H = a.H;
  const int bid = xcd_chunk_id(blockIdx.x, gridDim.x);
  const int b = bid / H, h = bid % H;
  const int npad = (n + 31) & ~31, NC = npad >> 5;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, l15 = lane & 15;
  const int img = npad * I::ROWB;
  char* Qi = smem;
  char* Di = smem + img;
  float* L2 = (float*)(smem + 2 * img);
  float* Dv = L2 + npad;
  char* dQi = (char*)(Dv + npad);                 // f32 [npad][HD]
  char* dst = dQi + npad * DQB;                   // NW x [32 keys][32 q] bf16
  float* csv = (float*)(dst + NW * 2048);         // [4 NW][HD] v-bias partials (one row per 16-lane row)
  float* csq = csv + 4 * NW * HD;                 // [4 NW][HD] q-bias partials
  char* myds = dst + wave * 2048;
  // rflag[w]: 1 once wave w's prologue is in (CHUNKED: its chunk of the
  // images), r + 2 once its round-r dQ add is
  constexpr bool CHUNKED = ATTN_BWD_FLAGS && ATTN_BWD_CHUNKED && HD == 32;
  int* rflag = (int*)(csq + 4 * NW * HD);
  if (threadIdx.x < NW) rflag[threadIdx.x] = 0;   // stale LDS of an earlier workgroup
  if (CHUNKED) __syncthreads();                   // nothing in flight yet: a cheap barrier
  ASTAMP(0);

  const int HH = H * HD;
  const float c = a.scale * LOG2E;
  const bf16_t* qkv = (const bf16_t*)a.qkv + (int64_t)b * n * a.ld_qkv;
  const bf16_t* O = (const bf16_t*)a.o + (int64_t)b * n * a.ld_o + h * HD;
  const bf16_t* dO = (const bf16_t*)a.dout + (int64_t)b * n * a.ld_o + h * HD;
  const float* lse = a.lse + ((int64_t)b * H + h) * n;

  // ---- prologue: every global load of the workgroup issued before the first
  // use (row indices clamped, out-of-range values selected to zero afterwards)
  // this wave's key chunk: K (scaled by c: S comes out in log2 units), V as
  // B-operand row fragments, K^T as the A operand of dQ^T in the permuted key
  // order of pack8 / dst_frag
  const int kbase = 32 * wave;
  v8s kf[2][KS], vf[2][KS], kT[DT];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = min(kbase + 16 * kt + l15, n - 1);
    const bf16_t* kr = qkv + (int64_t)key * a.ld_qkv + HH + h * HD + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[kt][ks] = ANT((const v8s*)(kr + 32 * ks));
      vf[kt][ks] = ANT((const v8s*)(kr + HH + 32 * ks));
    }
  }
  // Q, dO, O chunks: thread -> chunk slots tid + u NTH (CPR per row); CHUNKED:
  // wave w's lanes -> rows 32 w + (64 / CPR) u + lane / CPR (its own chunk)
  constexpr int U = CPR / 2;   // npad CPR chunks over NTH = 2 npad threads
  auto prow = [&](int u) {
    return CHUNKED ? 32 * wave + (64 / CPR) * u + lane / CPR : (int)(threadIdx.x + u * NTH) / CPR;
  };
  v4u vq[U], vd[U], vo[U];
  float ls[U];
  const int cc = threadIdx.x % CPR;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int row = prow(u), rc = min(row, n - 1);
    vq[u] = ANT((const v4u*)(qkv + (int64_t)rc * a.ld_qkv + h * HD + 8 * cc));
    vd[u] = ANT((const v4u*)(dO + (int64_t)rc * a.ld_o + 8 * cc));
    vo[u] = ANT((const v4u*)(O + (int64_t)rc * a.ld_o + 8 * cc));
    ls[u] = lse[rc];
  }
  if (CHUNKED) {   // this wave's 32 dQ rows (contiguous: the swizzle stays inside a row)
#pragma unroll
    for (int i = lane * 4; i < 32 * HD; i += 256) *(v4f*)(dQi + (32 * wave * HD + i) * 4) = v4f{0.f, 0.f, 0.f, 0.f};
  } else if (HD == 32) {   // (HD = 64: the region first holds the K images for K^T, below)
    for (int i = threadIdx.x * 4; i < npad * HD; i += 4 * NTH) *(v4f*)(dQi + i * 4) = v4f{0.f, 0.f, 0.f, 0.f};
  }
  ASTAMP(6);
  float vs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // v-bias: column sums of dO
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int row = prow(u);
    const bool ok = row < n;
    const v4u z = {0, 0, 0, 0};
    const v4u q = ok ? vq[u] : z, d = ok ? vd[u] : z;
    *(v4u*)(Qi + I::chunk(row, cc)) = q;
    *(v4u*)(Di + I::chunk(row, cc)) = d;
    float dd = chunk_dot<bf16_t>(d, ok ? vo[u] : z);
    dd += dpp_mov<0xB1>(dd);   // the row's CPR chunks are one lane quad (HD 32) or two
    dd += dpp_mov<0x4E>(dd);
    if (CPR == 8) dd += dpp_mov<0x141>(dd);   // row_half_mirror: the other quad
    if (cc == 0) {
      Dv[row] = -dd;
      L2[row] = ok ? -ls[u] : -1.0e30f;   // S' = c S: the exponent is S' - lse2
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vs[2 * j] += __uint_as_float(d[j] << 16);
      vs[2 * j + 1] += __uint_as_float(d[j] & 0xffff0000u);
    }
  }
  // lanes cc, cc + CPR, ... of each 16-lane row: row_shr 4, 8 (DPP) leave the
  // row's sum for chunk cc in lane 16 - CPR + cc
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (CPR == 4) vs[j] += dpp_mov<0x114>(vs[j]);
    vs[j] += dpp_mov<0x118>(vs[j]);
  }
  // K^T (the A operand of dQ^T) through LDS: the wave's 32 K rows as a
  // [32][HD] image (padding keys zero), read back transposed -- instead of
  // 16 DT two-byte global loads per lane. HD 32: this wave's dS tile, free
  // until the first round; HD 64 (4 KB): the wave's slice of the dQ image,
  // zeroed afterwards
  char* kimg = HD == 32 ? myds : dQi + wave * 4096;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const bool kok = kbase + 16 * kt + l15 < n;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      *(v8s*)(kimg + I::chunk(16 * kt + l15, 4 * ks + g)) = kok ? kf[kt][ks] : v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) kT[dt] = tr_frag<HD>(kimg, 0, 16 * dt, lane);
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const bool kok = kbase + 16 * kt + l15 < n;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      v8s t;
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = kok ? (short)f2bf(c * bf2f((bf16_t)kf[kt][ks][j])) : (short)0;
      kf[kt][ks] = t;
      vf[kt][ks] = kok ? vf[kt][ks] : v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  if (HD != 32) {
    __syncthreads();   // every wave has read its K^T back
    for (int i = threadIdx.x * 4; i < npad * HD; i += 4 * NTH) *(v4f*)(dQi + i * 4) = v4f{0.f, 0.f, 0.f, 0.f};
  }
  ASTAMP(7);
  if (CHUNKED) __hip_atomic_store(&rflag[wave], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __syncthreads();
  if (a.colsum_partial && (lane & 15) >= 16 - CPR)
#pragma unroll
    for (int j = 0; j < 8; ++j) csv[(4 * wave + (lane >> 4)) * HD + 8 * cc + j] = vs[j];
  ASTAMP(1);

  // per-lane LDS offsets; a round adds its query-chunk base (q0 is a multiple
  // of 32, so every swizzle below depends on the lane only)
  const int p_ = lane & 3;
  const int qq_ = (lane >> 2) & 3;
  int o_rf[KS];                                          // Q / dO row fragment, + 16 ROWB for u = 1
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) o_rf[ks] = I::chunk(l15, 4 * ks + g);
  int o_tr[DT];                                          // Q / dO transposed, + 16 ROWB for h = 1
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int unit = 4 * dt + p_;
    o_tr[dt] = I::chunk(4 * g + qq_, unit >> 1) + ((unit & 1) << 3);
  }
  int o_dq[DT];                                          // dQ f32, + 16 DQB for u = 1
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o_dq[dt] = dq_off<HD>(l15, 4 * dt + g);
  int o_sw[2], o_sr[2];                                  // dS tile write (+ 1024 kt = 1) / read (+ 1024 h = 1)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    o_sw[u] = dst_off(l15, 4 * u + g);
    o_sr[u] = dst_off(4 * g + qq_, 4 * u + p_);
  }

  v4f dv[2][DT], dk[2][DT];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) { dv[kt][dt] = v4f{0, 0, 0, 0}; dk[kt][dt] = v4f{0, 0, 0, 0}; }

  for (int r = 0; r < NC; ++r) {
    int qc = wave + r;
    qc = qc >= NC ? qc - NC : qc;
    const int q0 = qc * 32;
    if (CHUNKED && r > 0)   // chunk qc's images, Dv, L2, dQ rows are wave qc's
      while (__hip_atomic_load(&rflag[qc], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 1)
        __builtin_amdgcn_s_sleep(1);
    const char* Qr = Qi + q0 * ROWB;
    const char* Dr = Di + q0 * ROWB;
    v8s qf[2][KS], df[2][KS];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qf[u][ks] = *(const v8s*)(Qr + o_rf[ks] + 16 * ROWB * u);
        df[u][ks] = *(const v8s*)(Dr + o_rf[ks] + 16 * ROWB * u);
      }
    // transposed Q / dO fragments (A operands of dK^T / dV^T): rows q0..q0+31
    v8s qT[DT], dT[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, Qr + o_tr[dt]));
      v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, Qr + o_tr[dt] + 16 * ROWB));
      v4s y0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, Dr + o_tr[dt]));
      v4s y1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, Dr + o_tr[dt] + 16 * ROWB));
      qT[dt] = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
      dT[dt] = __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    v4f l2[2], dvr[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      l2[u] = *(const v4f*)(L2 + q0 + 16 * u + 4 * g);
      dvr[u] = *(const v4f*)(Dv + q0 + 16 * u + 4 * g);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      v4f P[2], dS[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // S' - lse2 [q = 4g+i][key = lane&15] and dP - Dv, row constants as the
        // initial accumulators
        v4f s = l2[u], dp = dvr[u];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[u][ks], kf[kt][ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(df[u][ks], vf[kt][ks], dp, 0, 0, 0);
        }
        // P clamped to [0, 1] by the exp's output modifier (free): softmax
        // probabilities never exceed 1, and a padding key (zero K row: S' = 0,
        // P = 2^-lse2) can then never overflow into 0 * inf = NaN in dQ
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          P[u][i] = fminf(fmaxf(__builtin_amdgcn_exp2f(s[i]), 0.f), 1.f);
          dS[u][i] = P[u][i] * dp[i];
        }
        const v2u pk = {pack2bf(dS[u][0], dS[u][1]), pack2bf(dS[u][2], dS[u][3])};
        *(v2u*)(myds + o_sw[u] + 1024 * kt) = pk;
      }
      const v8s pp = pack8(P[0], P[1]), ps = pack8(dS[0], dS[1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dv[kt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dT[dt], pp, dv[kt][dt], 0, 0, 0);
        dk[kt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qT[dt], ps, dk[kt][dt], 0, 0, 0);
      }
    }
    // dQ^T[d][q] += K^T[d][keys] dS^T[keys][q] for this wave's 32 keys.
    // ATTN_BWD_FLAGS: instead of a workgroup barrier per round, wave w waits
    // only for the wave that added into this query chunk in the round before
    // ((w + 1) mod NC, one LDS flag); every other phase of the round depends on
    // no other wave, so the waves drift apart by at most a round each and their
    // exp / MFMA / LDS phases interleave. The order of the adds per chunk (and
    // so the result) is the barrier schedule's.
#if ATTN_BWD_FLAGS
    if (r > 0) {
      const int src = wave + 1 == NW ? 0 : wave + 1;
      while (__hip_atomic_load(&rflag[src], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < r + 1)
        __builtin_amdgcn_s_sleep(1);
    }
#endif
    char* dQr = dQi + q0 * DQB;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v4s x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, myds + o_sr[u]));
      v4s x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, myds + o_sr[u] + 1024));
      const v8s bds = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        v4f* pq = (v4f*)(dQr + o_dq[dt] + 16 * DQB * u);
        *pq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kT[dt], bds, *pq, 0, 0, 0);
      }
    }
#if ATTN_BWD_FLAGS
    __hip_atomic_store(&rflag[wave], r + 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
    __syncthreads();
#endif
  }
  ASTAMP(2);

  bf16_t* dqkv = (bf16_t*)a.dqkv + (int64_t)b * a.n * a.ld_dqkv;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = kbase + 16 * kt + l15;
    if (key < n) {
      bf16_t* rowp = dqkv + (int64_t)key * a.ld_dqkv + h * HD;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        st4<bf16_t>(rowp + HH + 16 * dt + 4 * g, dk[kt][dt] * a.scale);
        st4<bf16_t>(rowp + 2 * HH + 16 * dt + 4 * g, dv[kt][dt]);
      }
    }
  }
  ASTAMP(3);
#if ATTN_BWD_FLAGS
  __syncthreads();   // every wave's last dQ update is in
#endif
  // dQ rows: thread -> (row, 4 columns); q-bias partial per (row group, column)
  float cq[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int C4N = HD / 4;   // 16-B chunks per dQ row
  const int c4 = threadIdx.x % C4N, rg = threadIdx.x / C4N, nrg = NTH / C4N;
  for (int row = rg; row < n; row += nrg) {
    const v4f v = *(const v4f*)(dQi + dq_off<HD>(row, c4)) * a.scale;
    st4<bf16_t>(dqkv + (int64_t)row * a.ld_dqkv + h * HD + 4 * c4, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) cq[i] += v[i];
  }
  ASTAMP(4);
  if (a.colsum_partial) {
    // reduce the row groups of a wave (lanes with equal c4) by shuffles, then
    // one partial row per wave in cs
    // HD 32: lanes c4 and c4 + 8 of each 16-lane row (row_shr 8): the row's
    // sum in lane 8 + c4; HD 64: a 16-lane row is one dQ row already
    if (HD == 32)
#pragma unroll
      for (int i = 0; i < 4; ++i) cq[i] += dpp_mov<0x118>(cq[i]);
    if ((lane & 15) >= (HD == 32 ? 8 : 0))
#pragma unroll
      for (int i = 0; i < 4; ++i) csq[(4 * wave + (lane >> 4)) * HD + 4 * c4 + i] = cq[i];
    __syncthreads();
    // q | k | v bias partials of this (sample, head); k is identically zero
    for (int i = threadIdx.x; i < 3 * HD; i += NTH) {
      const int part = i / HD, d = i % HD;
      float sum = 0.f;
      if (part != 1) {
        const float* src = part == 0 ? csq : csv;
        for (int w = 0; w < 4 * NW; ++w) sum += src[w * HD + d];
      }
      a.colsum_partial[(int64_t)b * 3 * HH + part * HH + h * HD + d] = sum;
    }
  }
  ASTAMP(5);
}

// ============================================ fp32 parity mode, long sequences
// The fp32 images of the MFMA kernels take 2 npad (4 HD + 16) bytes of LDS (the
// forward's K / V, the backward's two-image slots): past n ~ 540 at HD = 32 --
// the C4 decoder, n = 577 -- they do not fit in 160 KiB. These kernels stream
// 64-row blocks of the other side through LDS instead: one thread per query
// (forward, dQ) or key (dK, dV) row, exact f32 FMA, and the conventions of the
// MFMA kernels (scores in log2 units, lse2 = m + log2 l, Dv = -rowsum(dO O),
// dS = P (dP + Dv), the bias partials' zero k slice), so both agree to f32
// rounding. Parity mode only: the bf16 path never comes here.
constexpr int RB = 64;   // rows per streamed block = threads per workgroup

template <int HD>
__device__ __forceinline__ void load_row(float (&r)[HD], const float* p, bool ok) {
#pragma unroll
  for (int d = 0; d < HD; d += 4) {
    const v4f v = ok ? *(const v4f*)(p + d) : v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) r[d + j] = v[j];
  }
}
template <int HD>
__device__ __forceinline__ float dot_row(const float (&r)[HD], const float* l) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < HD; ++d) s = fmaf(r[d], l[d], s);
  return s;
}
// rows r0 .. r0 + RB - 1 of one head slice -> LDS [RB][HD] (zero past n)
template <int HD>
__device__ __forceinline__ void stage_rows(float (*dst)[HD], const float* src, int64_t ld, int r0, int n) {
  for (int i = threadIdx.x; i < RB * HD / 4; i += RB) {
    const int r = i / (HD / 4), c = 4 * (i % (HD / 4));
    *(v4f*)&dst[r][c] = r0 + r < n ? *(const v4f*)(src + (int64_t)(r0 + r) * ld + c) : v4f{0.f, 0.f, 0.f, 0.f};
  }
}
__device__ __forceinline__ float key_bias(const maeclip_attn_args& a, int b, int k) {
  return k < a.n && !(a.key_mask && a.key_mask[(int64_t)b * a.n + k] == 0.f) ? 0.f : NEG_BIG;
}

template <int HD>
__global__ void __launch_bounds__(RB) attn_fwd_rows_kernel(const maeclip_attn_args a) {
  __shared__ __attribute__((aligned(16))) float Kb[RB][HD], Vb[RB][HD];
  __shared__ float mb[RB];
  const int n = a.n, H = a.H, HH = H * HD;
  const int b = blockIdx.y / H, h = blockIdx.y % H;
  const int q = blockIdx.x * RB + threadIdx.x;
  const bool qok = q < n;
  const float* qkv = (const float*)a.qkv + (int64_t)b * n * a.ld_qkv;
  float qv[HD], o[HD];
  load_row<HD>(qv, qkv + (int64_t)(qok ? q : 0) * a.ld_qkv + h * HD, qok);
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.f;
  const float c = a.scale * LOG2E;
  float m = NEG_BIG, l = 0.f;
  for (int k0 = 0; k0 < n; k0 += RB) {
    __syncthreads();
    stage_rows<HD>(Kb, qkv + HH + h * HD, a.ld_qkv, k0, n);
    stage_rows<HD>(Vb, qkv + 2 * HH + h * HD, a.ld_qkv, k0, n);
    mb[threadIdx.x] = key_bias(a, b, k0 + threadIdx.x);
    __syncthreads();
    const int kn = min(RB, n - k0);
    for (int j = 0; j < kn; ++j) {
      const float s = fmaf(dot_row<HD>(qv, Kb[j]), c, mb[j]);
      const float mn = fmaxf(m, s);
      const float corr = __builtin_amdgcn_exp2f(m - mn), p = __builtin_amdgcn_exp2f(s - mn);
      l = fmaf(l, corr, p);
#pragma unroll
      for (int d = 0; d < HD; ++d) o[d] = fmaf(o[d], corr, p * Vb[j][d]);
      m = mn;
    }
  }
  if (qok) {
    const float inv = 1.f / l;
    float* orow = (float*)a.o + ((int64_t)b * n + q) * a.ld_o + h * HD;
#pragma unroll
    for (int d = 0; d < HD; d += 4) *(v4f*)(orow + d) = v4f{o[d], o[d + 1], o[d + 2], o[d + 3]} * inv;
    if (a.lse) a.lse[((int64_t)b * H + h) * n + q] = m + log2f(l);
  }
}

// dQ: one thread per query row, 64-key blocks of K, V through LDS
template <int HD>
__global__ void __launch_bounds__(RB) attn_bwd_rows_dq_kernel(const maeclip_attn_args a) {
  __shared__ __attribute__((aligned(16))) float Kb[RB][HD], Vb[RB][HD];
  __shared__ float mb[RB];
  const int n = a.n, H = a.H, HH = H * HD;
  const int b = blockIdx.y / H, h = blockIdx.y % H;
  const int q = blockIdx.x * RB + threadIdx.x;
  const bool qok = q < n;
  const int qr = qok ? q : 0;
  const float* qkv = (const float*)a.qkv + (int64_t)b * n * a.ld_qkv;
  float qv[HD], dov[HD], dq[HD];
  load_row<HD>(qv, qkv + (int64_t)qr * a.ld_qkv + h * HD, qok);
  load_row<HD>(dov, (const float*)a.dout + ((int64_t)b * n + qr) * a.ld_o + h * HD, qok);
  const float Dq = -dot_row<HD>(dov, (const float*)a.o + ((int64_t)b * n + qr) * a.ld_o + h * HD);
  const float L = qok ? a.lse[((int64_t)b * H + h) * n + q] : 1.0e30f;
#pragma unroll
  for (int d = 0; d < HD; ++d) dq[d] = 0.f;
  const float c = a.scale * LOG2E;
  for (int k0 = 0; k0 < n; k0 += RB) {
    __syncthreads();
    stage_rows<HD>(Kb, qkv + HH + h * HD, a.ld_qkv, k0, n);
    stage_rows<HD>(Vb, qkv + 2 * HH + h * HD, a.ld_qkv, k0, n);
    mb[threadIdx.x] = key_bias(a, b, k0 + threadIdx.x);
    __syncthreads();
    const int kn = min(RB, n - k0);
    for (int j = 0; j < kn; ++j) {
      const float p = __builtin_amdgcn_exp2f(fmaf(dot_row<HD>(qv, Kb[j]), c, mb[j]) - L);
      const float ds = p * (dot_row<HD>(dov, Vb[j]) + Dq);
#pragma unroll
      for (int d = 0; d < HD; ++d) dq[d] = fmaf(ds, Kb[j][d], dq[d]);
    }
  }
  if (qok) {
    float* row = (float*)a.dqkv + ((int64_t)b * n + q) * a.ld_dqkv + h * HD;
#pragma unroll
    for (int d = 0; d < HD; d += 4) *(v4f*)(row + d) = v4f{dq[d], dq[d + 1], dq[d + 2], dq[d + 3]} * a.scale;
  }
}

// dK, dV: one thread per key row, 64-query blocks of Q, dO (+ lse2, Dv) through LDS
template <int HD>
__global__ void __launch_bounds__(RB) attn_bwd_rows_dkv_kernel(const maeclip_attn_args a) {
  __shared__ __attribute__((aligned(16))) float Qb[RB][HD], Db[RB][HD];
  __shared__ float Lb[RB], Dvb[RB];
  const int n = a.n, H = a.H, HH = H * HD;
  const int b = blockIdx.y / H, h = blockIdx.y % H;
  const int k = blockIdx.x * RB + threadIdx.x;
  const bool kok = k < n;
  const int kr = kok ? k : 0;
  const float* qkv = (const float*)a.qkv + (int64_t)b * n * a.ld_qkv;
  const float* O = (const float*)a.o + (int64_t)b * n * a.ld_o + h * HD;
  const float* dO = (const float*)a.dout + (int64_t)b * n * a.ld_o + h * HD;
  float kv[HD], vv[HD], dk[HD], dv[HD];
  load_row<HD>(kv, qkv + (int64_t)kr * a.ld_qkv + HH + h * HD, kok);
  load_row<HD>(vv, qkv + (int64_t)kr * a.ld_qkv + 2 * HH + h * HD, kok);
  const float mk = key_bias(a, b, k);
#pragma unroll
  for (int d = 0; d < HD; ++d) dk[d] = dv[d] = 0.f;
  const float c = a.scale * LOG2E;
  for (int q0 = 0; q0 < n; q0 += RB) {
    __syncthreads();
    stage_rows<HD>(Qb, qkv + h * HD, a.ld_qkv, q0, n);
    stage_rows<HD>(Db, dO, a.ld_o, q0, n);
    {
      const int q = q0 + threadIdx.x;
      const bool ok = q < n;
      float dr[HD];
      load_row<HD>(dr, dO + (int64_t)(ok ? q : 0) * a.ld_o, ok);
      Dvb[threadIdx.x] = ok ? -dot_row<HD>(dr, O + (int64_t)q * a.ld_o) : 0.f;
      Lb[threadIdx.x] = ok ? a.lse[((int64_t)b * H + h) * n + q] : 1.0e30f;
    }
    __syncthreads();
    const int qn = min(RB, n - q0);
    for (int j = 0; j < qn; ++j) {
      const float p = __builtin_amdgcn_exp2f(fmaf(dot_row<HD>(kv, Qb[j]), c, mk) - Lb[j]);
      const float ds = p * (dot_row<HD>(vv, Db[j]) + Dvb[j]);
#pragma unroll
      for (int d = 0; d < HD; ++d) {
        dv[d] = fmaf(p, Db[j][d], dv[d]);
        dk[d] = fmaf(ds, Qb[j][d], dk[d]);
      }
    }
  }
  if (kok) {
    float* row = (float*)a.dqkv + ((int64_t)b * n + k) * a.ld_dqkv + h * HD;
#pragma unroll
    for (int d = 0; d < HD; d += 4) {
      *(v4f*)(row + HH + d) = v4f{dk[d], dk[d + 1], dk[d + 2], dk[d + 3]} * a.scale;
      *(v4f*)(row + 2 * HH + d) = v4f{dv[d], dv[d + 1], dv[d + 2], dv[d + 3]};
    }
  }
}

// bias partials of the rows path: column sums of this sample's dqkv rows (the
// q and v slices of every head; the k slice is identically zero, as above)
__global__ void __launch_bounds__(256) attn_rows_colsum_kernel(const maeclip_attn_args a, int HH) {
  const int b = blockIdx.y, col = blockIdx.x * 256 + threadIdx.x;
  if (col >= 3 * HH) return;
  float s = 0.f;
  if (col < HH || col >= 2 * HH) {
    const float* p = (const float*)a.dqkv + (int64_t)b * a.n * a.ld_dqkv + col;
    for (int r = 0; r < a.n; ++r) s += p[(int64_t)r * a.ld_dqkv];
  }
  a.colsum_partial[(int64_t)b * 3 * HH + col] = s;
}

template <int HD>
int run_rows(const maeclip_attn_args& a, bool bwd, hipStream_t s) {
  MC_CHECK_ARG(bwd || a.dropout_p == 0.f, "maeclip_attn_fwd: the fp32 long-sequence path has no attention dropout");
  const dim3 grid((unsigned)((a.n + RB - 1) / RB), (unsigned)(a.B * a.H));
  if (!bwd) {
    hipLaunchKernelGGL(attn_fwd_rows_kernel<HD>, grid, dim3(RB), 0, s, a);
    MC_CHECK_LAUNCH("maeclip_attn_fwd(f32 rows)");
    return 0;
  }
  hipLaunchKernelGGL(attn_bwd_rows_dq_kernel<HD>, grid, dim3(RB), 0, s, a);
  hipLaunchKernelGGL(attn_bwd_rows_dkv_kernel<HD>, grid, dim3(RB), 0, s, a);
  if (a.colsum_partial) {
    const int HH = a.H * HD;
    hipLaunchKernelGGL(attn_rows_colsum_kernel, dim3((unsigned)((3 * HH + 255) / 256), (unsigned)a.B), dim3(256), 0,
                       s, a, HH);
  }
  MC_CHECK_LAUNCH("maeclip_attn_bwd(f32 rows)");
  return 0;
}

template <int HD> size_t bwd_diag_lds(int n) {
  const int npad = (n + 31) & ~31, nw = npad / 32;
  return (size_t)2 * npad * Img<bf16_t, HD>::ROWB + (size_t)2 * npad * 4 + (size_t)npad * 4 * HD +
         (size_t)nw * 2048 + (size_t)8 * nw * HD * 4 + (size_t)nw * 4;
}

template <typename T, int HD> size_t fwd_lds(int n) {
  const int npad = (n + 63) & ~63;
  const int nimg = fwd_qimg<T, HD>(npad) ? 3 : 2;   // K, V (+ Q; the 16-wave launches ignore the third)
  return (size_t)nimg * npad * Img<T, HD>::ROWB + (size_t)npad * 4;
}
template <typename T, int HD> size_t bwd_lds(int n, int nw, bool two = false) {
  const int npad = (n + 31) & ~31;
  const int nimg = (std::is_same<T, bf16_t>::value && !two) ? 4 : 2;
  return (size_t)nimg * npad * Img<T, HD>::ROWB + (size_t)2 * npad * 4 + (size_t)nw * 3 * HD * 4;
}

template <typename T, int HD, bool TWO = false, int OCC = 1, int WG = MAXW, bool Q8 = false>
void launch_bwd(const maeclip_attn_args& a, dim3 grid, int nthreads, size_t lds, hipStream_t s) {
  if (lds > 65536)
    maeclip::allow_lds((const void*)attn_bwd_kernel<T, HD, TWO, OCC, WG, Q8>, (int)lds);
  hipLaunchKernelGGL((attn_bwd_kernel<T, HD, TWO, OCC, WG, Q8>), grid, dim3(nthreads), lds, s, a);
}

// resident workgroups per CU of a bwd variant (registers, waves and LDS)
template <typename T, int HD, bool TWO, int OCC = 1>
int bwd_occupancy(int nthreads, size_t lds) {
  if (lds > 65536)
    maeclip::allow_lds((const void*)attn_bwd_kernel<T, HD, TWO, OCC>, (int)lds);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)attn_bwd_kernel<T, HD, TWO, OCC>,
                                                   nthreads, lds) != hipSuccess)
    return 0;
  return nb;
}

// bf16: use the two-image backward when it keeps more workgroups per CU
// resident (option ATTN_TWO = 0 / 1 / 3 forces it); cached per shape.
// returns 0 (four images), 1 (two images) or 3 (two images, 3 workgroups / CU)
template <int HD>
int bwd_two(int n, int nw, size_t lds4, size_t lds2) {
  const int forced = maeclip::option(MAECLIP_OPT_ATTN_TWO, -1);
  if (forced >= 0) return forced == 0 ? 0 : forced == 3 && HD == 32 ? 3 : 1;
  static int cache[2][64][MAXW + 1] = {};   // (npad / 32) x nw -> variant + 1
  const int key = ((n + 31) >> 5) & 63;
  int& c = cache[HD == 64][key][nw];
  if (c == 0) {
    const int occ4 = lds4 <= 163840 ? bwd_occupancy<bf16_t, HD, false>(64 * nw, lds4) : 0;
    const int occ2 = bwd_occupancy<bf16_t, HD, true>(64 * nw, lds2);
    const int occ3 = HD == 32 ? bwd_occupancy<bf16_t, HD, true, 3>(64 * nw, lds2) : 0;
    c = occ3 > occ2 && occ3 > occ4 ? 4 : occ2 > occ4 ? 2 : 1;
  }
  return c - 1;
}

// q8_done: set when the launched kernel wrote the fp8-blocks copy itself
template <typename T, int HD>
int run(const maeclip_attn_args& a, bool bwd, hipStream_t s, bool& q8_done) {
  q8_done = false;
  // one wave per 16-row tile (no idle waves), at most MAXW; the forward
  // spreads its tiles evenly over the rounds it needs (n = 197: 13 tiles on 7
  // waves, not 8 waves of which 3 idle for the second round)
  const int tiles = (a.n + 15) / 16;
  const int rounds = (tiles + MAXW - 1) / MAXW;
  const int nw = bwd ? (tiles < MAXW ? tiles : MAXW) : (tiles + rounds - 1) / rounds;
  const int nthreads = 64 * nw;
  size_t lds = bwd ? bwd_lds<T, HD>(a.n, nw) : fwd_lds<T, HD>(a.n);
  bool two = false;
  int variant = 0;
  if constexpr (std::is_same<T, bf16_t>::value) {
    if (bwd) {
      const size_t lds2 = bwd_lds<T, HD>(a.n, nw, true);
      variant = lds2 <= 163840 ? bwd_two<HD>(a.n, nw, lds, lds2) : 0;
      two = variant != 0;
      if (two) lds = lds2;
    }
  }
  if constexpr (!std::is_same<T, bf16_t>::value) {
    // fp32 beyond the LDS images (option ATTN_ROWS = 1 forces it: tests)
    if (lds > 163840 || maeclip::option(MAECLIP_OPT_ATTN_ROWS, 0) != 0) return run_rows<HD>(a, bwd, s);
  }
  MC_CHECK_ARG(lds <= 163840, "maeclip_attn: n=%d needs %zu B of LDS (> 160 KiB)", a.n, lds);
  MC_CHECK_ARG(!bwd || !a.key_mask, "maeclip_attn_bwd: key_mask is supported by the fp32 rows path only");
  dim3 grid((unsigned)(a.B * a.H));
  if constexpr (std::is_same<T, bf16_t>::value) {
    // one-pass diagonal backward: the default at HD 32 up to npad 256
    // (MAECLIP_ATTN_DIAG=0 turns it off). HD 64 (LDS fits up to npad 224): the
    // 56 KB f32 dQ image leaves one workgroup per CU, whose ~140 KB prologue
    // has nothing to overlap with -- slower everywhere with a barrier per
    // round (profiles/r03/attn_diag64_ab.txt); with the per-wave round flags
    // it wins at the long rows only (C1 encoder n = 197: 299 -> 289 us; C2
    // encoder n = 50: 52 -> 55; C4 n = 145 even; profiles/r05/attn_diag64_ab_r5ag.txt),
    // so it is the default for npad >= 192 (option ATTN_DIAG = 1 / 0 forces it on / off).
    const int od = maeclip::option(MAECLIP_OPT_ATTN_DIAG, -1);
    const int npad = (a.n + 31) & ~31;
    const size_t ld = bwd_diag_lds<HD>(a.n);
    const bool want = HD == 32 ? od != 0 : (od >= 0 ? od == 1 : npad >= 192);
    if (bwd && npad <= 256 && ld <= 163840 && want && !a.key_mask) {
      if (ld > 65536)
        maeclip::allow_lds((const void*)attn_bwd_diag_kernel<HD>, (int)ld);
      hipLaunchKernelGGL(attn_bwd_diag_kernel<HD>, grid, dim3(2 * npad), ld, s, a);
      MC_CHECK_LAUNCH("maeclip_attn_bwd(diag)");
      return 0;
    }
  }
  if constexpr (std::is_same<T, bf16_t>::value) {
    // bf16 rows beyond the diagonal kernel with more 16-row tiles than MAXW
    // waves: the two-image layout with up to 16 waves, default at HD 32 (C4
    // decoder n = 577: 604 -> 555 us; at HD 64 the C4 encoder, n = 145, loses:
    // 147 -> 168; profiles/r05/attn_bw16_ab_r5ah.txt). Option ATTN_BW16 = 1 / 0
    // forces it on / off.
    const int o16 = maeclip::option(MAECLIP_OPT_ATTN_BW16, -1);
    const bool bw16 = o16 >= 0 ? o16 != 0 : HD == 32;
    if (bwd && tiles > MAXW && bw16) {
      const int nw16 = tiles < 16 ? tiles : 16;
      const size_t lds16 = bwd_lds<T, HD>(a.n, nw16, true);
      if (lds16 <= 163840) {
        if (a.q8) launch_bwd<T, HD, true, 1, 16, true>(a, grid, 64 * nw16, lds16, s);
        else launch_bwd<T, HD, true, 1, 16>(a, grid, 64 * nw16, lds16, s);
        q8_done = a.q8 != nullptr;
        MC_CHECK_LAUNCH("maeclip_attn_bwd(16 waves)");
        return 0;
      }
    }
  }
  if (bwd) {
    // (round 2 also had a bf16 variant that kept dS in LDS between the two
    // phases instead of recomputing S / dP for dQ: 355 vs 224 us at the
    // decoder shape, the n x n image halving the workgroups per CU; removed)
    const bool q8 = std::is_same<T, bf16_t>::value && a.q8 != nullptr;
    if constexpr (std::is_same<T, bf16_t>::value) {
      if (variant == 3) launch_bwd<T, HD, true, HD == 32 ? 3 : 1>(a, grid, nthreads, lds, s);   // (no q8: pass)
      else if (two && q8) launch_bwd<T, HD, true, 1, MAXW, true>(a, grid, nthreads, lds, s);
      else if (two) launch_bwd<T, HD, true>(a, grid, nthreads, lds, s);
      else if (q8) launch_bwd<T, HD, false, 1, MAXW, true>(a, grid, nthreads, lds, s);
      q8_done = q8 && variant != 3;
    }
    if (!two && !q8) launch_bwd<T, HD, false>(a, grid, nthreads, lds, s);
  } else {
    // the fused fp8 copy: bf16 without dropout (the fp8 stacks' case)
    const bool q8 = std::is_same<T, bf16_t>::value && a.q8 != nullptr && a.dropout_p == 0.f;
    auto kern = a.dropout_p > 0.f ? attn_fwd_kernel<T, HD, true>
                                  : (q8 ? attn_fwd_kernel<T, HD, false, MAXW, true> : attn_fwd_kernel<T, HD, false>);
    if constexpr (std::is_same<T, bf16_t>::value) {
      // (n <= 48: at most three query tiles, one per wave -- the DMA'd Q saves no
      // round trip and lengthens the prologue: text n = 25 13.5 -> 15.5 us)
      if (a.n > 48 && fwd_qimg<T, HD>((a.n + 63) & ~63))
        kern = a.dropout_p > 0.f ? attn_fwd_kernel<T, HD, true, MAXW, false, true>
                                 : (q8 ? attn_fwd_kernel<T, HD, false, MAXW, true, true>
                                       : attn_fwd_kernel<T, HD, false, MAXW, false, true>);
    }
    int nth = nthreads;
    // one workgroup per CU by LDS and more tiles than MAXW waves: up to 16
    // waves (option ATTN_FW16 = 0 turns it off)
    if (tiles > MAXW && 2 * lds > 163840 && maeclip::option(MAECLIP_OPT_ATTN_FW16, 1) != 0) {
      const int r16 = (tiles + 15) / 16;
      nth = 64 * ((tiles + r16 - 1) / r16);
      kern = a.dropout_p > 0.f ? attn_fwd_kernel<T, HD, true, 16>
                               : (q8 ? attn_fwd_kernel<T, HD, false, 16, true> : attn_fwd_kernel<T, HD, false, 16>);
    }
    if (lds > 65536) maeclip::allow_lds((const void*)kern, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(nth), lds, s, a);
    q8_done = q8;
  }
  MC_CHECK_LAUNCH(bwd ? "maeclip_attn_bwd" : "maeclip_attn_fwd");
  return 0;
}

int check(const maeclip_attn_args* a, bool bwd) {
  MC_CHECK_ARG(a && a->qkv && a->o, "maeclip_attn: null pointer");
  MC_CHECK_ARG(a->head_dim == 32 || a->head_dim == 64, "maeclip_attn: head_dim must be 32 or 64 (got %d)", a->head_dim);
  MC_CHECK_ARG(a->B > 0 && a->n > 0 && a->H > 0, "maeclip_attn: bad sizes");
  MC_CHECK_ARG(a->dtype == MAECLIP_F32 || a->dtype == MAECLIP_BF16, "maeclip_attn: bad dtype");
  const int epc = a->dtype == MAECLIP_BF16 ? 8 : 4;
  MC_CHECK_ARG(a->ld_qkv % epc == 0 && a->ld_o % epc == 0, "maeclip_attn: row strides must be 16-byte multiples");
  if (bwd) {
    MC_CHECK_ARG(a->dout && a->dqkv && a->lse, "maeclip_attn_bwd: null pointer");
    MC_CHECK_ARG(a->ld_dqkv % epc == 0, "maeclip_attn_bwd: ld_dqkv");
  }
  if (a->q8) {
    const int64_t len = (int64_t)a->H * a->head_dim * (bwd ? 3 : 1);
    MC_CHECK_ARG(len % 128 == 0 && a->ldq8 >= len && a->ldq8 % 16 == 0 && ((uintptr_t)a->q8 & 15) == 0 &&
                     a->q8_scale && (a->q8_fmt == MAECLIP_FP8_E4M3 || a->q8_fmt == MAECLIP_FP8_E5M2),
                 "maeclip_attn: fp8-blocks output needs a row length %% 128, ldq8 %% 16, a scale buffer and a format");
  }
  return 0;
}

int dispatch(const maeclip_attn_args* a, bool bwd, void* stream) {
  if (int e = check(a, bwd)) return e;
  hipStream_t s = (hipStream_t)stream;
  bool q8_done = false;
  int rc;
  if (a->dtype == MAECLIP_BF16)
    rc = a->head_dim == 64 ? run<bf16_t, 64>(*a, bwd, s, q8_done) : run<bf16_t, 32>(*a, bwd, s, q8_done);
  else
    rc = a->head_dim == 64 ? run<float, 64>(*a, bwd, s, q8_done) : run<float, 32>(*a, bwd, s, q8_done);
  if (rc != 0 || !a->q8 || q8_done) return rc;
  // variants without the fused copy: the standalone pass over the output
  const int64_t HH = (int64_t)a->H * a->head_dim;
  return bwd ? maeclip_quant_blocks_fp8(a->dqkv, a->dtype, (int64_t)a->B * a->n, 3 * HH, a->ld_dqkv, a->q8, a->ldq8,
                                        a->q8_scale, a->q8_fmt, stream)
             : maeclip_quant_blocks_fp8(a->o, a->dtype, (int64_t)a->B * a->n, HH, a->ld_o, a->q8, a->ldq8,
                                        a->q8_scale, a->q8_fmt, stream);
}

}  // namespace

#ifdef ATTN_STAMPS
extern "C" int maeclip_debug_attn_stamps(uint64_t* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), sizeof(uint64_t) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int32_t maeclip_attn_fwd(const maeclip_attn_args* a, void* stream) { return dispatch(a, false, stream); }
extern "C" int32_t maeclip_attn_bwd(const maeclip_attn_args* a, void* stream) { return dispatch(a, true, stream); }
