// MAE head kernels (gfx950). The reference names MAE but ships no code for it
// (SURVEY.md §0.2); semantics follow HF transformers ViTMAE
// (models/vit_mae/modeling_vit_mae.py):
//   random_masking  :297-327  per-sample argsort of noise, keep the first
//                             int(L*(1-r)), ids_restore = argsort(ids_shuffle),
//                             mask 1 = removed
//   patchify        :706-745  [B,C,h*p,w*p] -> [B,h*w,p*p*C], in-patch (ky,kx,c)
//   decoder unshuffle :548-566 cat(tokens[:,1:], mask_tokens) gathered by
//                             ids_restore, cls re-prepended, + decoder_pos_embed
//   loss            :852-859  optional norm_pix (unbiased var, eps 1e-6),
//                             mean over p*p*C, (l*mask).sum()/mask.sum()
// The encoder side follows timm's PatchEmbed/_pos_embed applied FLIP-style to
// the visible patches only.
//
// Mask noise is a counter-based hash (common.h mc_hash4) of (seed, step,
// global sample index, patch): key24 = hash>>8, noise = key24 * 2^-24, sorted
// ascending with the patch index as tie-break == torch.argsort(noise,
// stable=True). Restated bit-exactly in oracle/maskrng.py.
#include "common.h"
#include "../../include/maeclip.h"

namespace {
constexpr int NTH = 256;

__global__ void __launch_bounds__(NTH) mask_ids_kernel(const maeclip_mask_args a) {
  __shared__ uint64_t keys[1024];
  const int b = blockIdx.x, L = a.L;
  int S2 = 1;
  while (S2 < L) S2 <<= 1;
  const uint64_t gb = (uint64_t)a.sample_offset + b;
  const uint64_t step = a.step + (a.step_ptr ? (uint64_t)*a.step_ptr : 0ull);
  for (int i = threadIdx.x; i < S2; i += NTH) {
    if (i < L) {
      const uint64_t k24 = mc_hash4(a.seed, step, gb, (uint64_t)i) >> 8;
      keys[i] = (k24 << 10) | (uint64_t)i;
      if (a.noise) a.noise[(int64_t)b * L + i] = (float)k24 * (1.0f / 16777216.0f);
    } else {
      keys[i] = ~0ull;
    }
  }
  __syncthreads();
  for (int k = 2; k <= S2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < S2; i += NTH) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = keys[i], y = keys[ixj];
          const bool asc = (i & k) == 0;
          if (asc ? (x > y) : (x < y)) {
            keys[i] = y;
            keys[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < L; i += NTH) {
    const int idx = (int)(keys[i] & 1023u);
    a.ids_shuffle[(int64_t)b * L + i] = idx;
    a.ids_restore[(int64_t)b * L + idx] = i;
    if (a.mask) a.mask[(int64_t)b * L + idx] = i >= a.len_keep ? 1.f : 0.f;
  }
}

// patch rows of the visible patches in conv-weight order (c, ky, kx)
template <typename OT>
__global__ void __launch_bounds__(NTH) patch_gather_kernel(const maeclip_patch_args a) {
  const int64_t seg = (int64_t)blockIdx.x * NTH + threadIdx.x;  // one (row, c, ky) run of p pixels
  const int p = a.p, C = a.C, S = a.S, w = S / p, L = w * w;
  const int64_t nseg = (int64_t)a.B * a.keep * C * p;
  if (seg >= nseg) return;
  const int ky = (int)(seg % p);
  const int c = (int)((seg / p) % C);
  const int64_t row = seg / ((int64_t)p * C);
  const int b = (int)(row / a.keep), j = (int)(row % a.keep);
  const int l = a.ids_shuffle ? a.ids_shuffle[(int64_t)b * L + j] : j;
  const int py = l / w, px = l % w;
  const float* src = a.img + (((int64_t)b * C + c) * S + (py * p + ky)) * S + px * p;
  OT* dst = (OT*)a.out + row * a.ld_out + (int64_t)c * p * p + ky * p;
  if ((p & 3) == 0) {
    for (int kx = 0; kx < p; kx += 4) st4<OT>(dst + kx, *(const v4f*)(src + kx));
  } else {
    for (int kx = 0; kx < p; ++kx) st_from_f<OT>(dst + kx, src[kx]);
  }
  if (c == 0 && ky == 0) {
    OT* prow = (OT*)a.out + row * a.ld_out;
    for (int64_t k = (int64_t)C * p * p; k < a.ld_out; ++k) st_from_f<OT>(prow + k, 0.f);
  }
}

// The same rows with one lane per 4 pixels (p % 4 == 0): lane -> (segment,
// quarter), segments (row j, c, ky) ordered with ky fastest, so the p/4 lanes
// of a segment read one contiguous 4p-byte run of an image row together, and
// at p = 16 one wave covers a whole (row, c) block: 16 image-row runs of 64 B
// in, 256 consecutive output elements out (the one-lane-per-run kernel below
// touches 64 rows with 16 B per lane per load instruction)
template <typename OT>
__global__ void __launch_bounds__(NTH) patch_gather4_kernel(const maeclip_patch_args a) {
  const int64_t t = (int64_t)blockIdx.x * NTH + threadIdx.x;
  const int p = a.p, C = a.C, S = a.S, w = S / p, L = w * w, Q = p >> 2;
  const int64_t nt = (int64_t)a.B * a.keep * C * p * Q;
  if (t >= nt) return;
  const int qr = (int)(t % Q);
  const int64_t seg = t / Q;
  const int ky = (int)(seg % p);
  const int c = (int)((seg / p) % C);
  const int64_t row = seg / ((int64_t)p * C);
  const int b = (int)(row / a.keep), j = (int)(row % a.keep);
  const int l = a.ids_shuffle ? a.ids_shuffle[(int64_t)b * L + j] : j;
  const int py = l / w, px = l % w;
  const float* src = a.img + (((int64_t)b * C + c) * S + (py * p + ky)) * S + px * p + 4 * qr;
  OT* dst = (OT*)a.out + row * a.ld_out + (int64_t)c * p * p + ky * p + 4 * qr;
  st4<OT>(dst, *(const v4f*)src);
  if (c == 0 && ky == 0) {   // zero pad columns [C*p*p, ld_out): the segment's lanes share them
    OT* prow = (OT*)a.out + row * a.ld_out;
    for (int64_t k = (int64_t)C * p * p + qr; k < a.ld_out; k += Q) st_from_f<OT>(prow + k, 0.f);
  }
}

// patch rows of the visible patches from the decoded uint8 HWC pixels, with
// A.Normalize + the HWC->CHW permute (dataset.py:49, :34) folded in: one
// thread per (row, ky) reads the p*C contiguous bytes of that patch row
// (p = 16, C = 3: three 16-B loads) and writes the C channel runs of p values
// (c, ky, kx order) -- 1 B read per 2 B (bf16) written instead of the fp32
// image's 4 B read
template <typename OT, bool VEC>
__global__ void __launch_bounds__(NTH) patch_gather_u8_kernel(const maeclip_patch_args a, NormConst k) {
  const int64_t seg = (int64_t)blockIdx.x * NTH + threadIdx.x;  // (row, ky)
  const int p = a.p, C = a.C, S = a.S, w = S / p, L = w * w;
  if (seg >= (int64_t)a.B * a.keep * p) return;
  const int ky = (int)(seg % p);
  const int64_t row = seg / p;
  const int b = (int)(row / a.keep), j = (int)(row % a.keep);
  const int l = a.ids_shuffle ? a.ids_shuffle[(int64_t)b * L + j] : j;
  const int py = l / w, px = l % w;
  const uint8_t* src = a.img_u8 + (((int64_t)b * S + py * p + ky) * S + (int64_t)px * p) * C;
  OT* dst = (OT*)a.out + row * a.ld_out + ky * p;
  if constexpr (VEC) {   // p = 16, C = 3: 48 bytes, 16-B aligned
    const v4u q0 = *(const v4u*)src, q1 = *(const v4u*)(src + 16), q2 = *(const v4u*)(src + 32);
    const unsigned wd[12] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3], q2[0], q2[1], q2[2], q2[3]};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      v4f o[4];
#pragma unroll
      for (int kx = 0; kx < 16; ++kx) {
        const int byte = kx * 3 + c;
        o[kx >> 2][kx & 3] = mc_norm_px((wd[byte >> 2] >> (8 * (byte & 3))) & 0xffu, k, c);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) st4<OT>(dst + c * 256 + 4 * q, o[q]);
    }
  } else {
    for (int c = 0; c < C; ++c)
      for (int kx = 0; kx < p; ++kx) st_from_f<OT>(dst + (int64_t)c * p * p + kx, mc_norm_px(src[kx * C + c], k, c));
  }
  if (ky == 0) {
    OT* prow = (OT*)a.out + row * a.ld_out;
    for (int64_t kk = (int64_t)C * p * p; kk < a.ld_out; ++kk) st_from_f<OT>(prow + kk, 0.f);
  }
}

// x[b,0] = cls + pos[0]; x[b,1+j] = Y[b*keep+j] + pos[1+ids_shuffle[b,j]]   (f32 out)
template <typename YT>
__global__ void __launch_bounds__(NTH) tokens_fwd_kernel(const maeclip_tokens_args a) {
  const int64_t row = blockIdx.y;  // b*(1+keep) + t
  const int d = (blockIdx.x * NTH + threadIdx.x) * 4;
  if (d >= a.D) return;
  const int nt = a.keep + 1;
  const int b = (int)(row / nt), t = (int)(row % nt);
  v4f v;
  if (t == 0) {
    v = *(const v4f*)(a.cls + d) + *(const v4f*)(a.pos + d);
  } else {
    const int j = t - 1;
    const int l = a.ids_shuffle ? a.ids_shuffle[(int64_t)b * a.L + j] : j;
    v = ld4<YT>((const YT*)a.y + ((int64_t)b * a.keep + j) * a.ldy + d) + *(const v4f*)(a.pos + (int64_t)(1 + l) * a.D + d);
  }
  *(v4f*)(a.x + row * a.D + d) = v;
}

// dY[b*keep+j] = dx[b,1+j] (as GEMM operand dtype)
template <typename YT>
__global__ void __launch_bounds__(NTH) tokens_bwd_dy_kernel(const maeclip_tokens_args a) {
  const int64_t r = blockIdx.y;  // b*keep + j
  const int d = (blockIdx.x * NTH + threadIdx.x) * 4;
  if (d >= a.D) return;
  const int b = (int)(r / a.keep), j = (int)(r % a.keep);
  const v4f v = *(const v4f*)(a.dx + ((int64_t)b * (a.keep + 1) + 1 + j) * a.D + d);
  st4<YT>((YT*)a.dy + r * a.ldy + d, v);
}
#ifndef TBP_UNROLL
#define TBP_UNROLL 8
#endif
// dpos[1+l] = sum_b [kept] dx[b,1+restore[b,l]] ; dpos[0] = dcls = sum_b dx[b,0]
// One workgroup per (position, 256-column chunk): wave w sums the samples
// b = w, w+4, ... in ascending order. The wave first loads the restore index
// of 64 of its samples (one per lane) and ballots which keep this position,
// then issues the dx rows of only those, TBP_UNROLL 16-B loads in flight per lane
// (no dependent index load per row, no loads for masked samples). The four
// wave partials are added in a fixed order through LDS (deterministic).
__global__ void __launch_bounds__(NTH) tokens_bwd_pos_kernel(const maeclip_tokens_args a) {
  __shared__ v4f red[NTH / 64][64];
  const int pr = blockIdx.x;  // 0..L
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d = (blockIdx.y * 64 + lane) * 4;
  const int nt = a.keep + 1;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  // Lane `lane` plays two roles: the 4-column chunk d of the sums, and sample
  // b0 + wave + 4*lane of the restore-index ballot. The ballot must therefore
  // run with all 64 lanes active whatever D is; only the dx loads are guarded
  // by the column bound.
  const bool dok = d < a.D;
  for (int b0 = 0; b0 < a.B; b0 += 4 * 64) {
    const int bl = b0 + wave + 4 * lane;
    // token row t = 1 + r of sample bl (r = -1: the cls row, for pr = 0)
    int r = a.keep;
    if (bl < a.B) r = pr == 0 ? -1 : (a.ids_restore ? a.ids_restore[(int64_t)bl * a.L + pr - 1] : pr - 1);
    uint64_t m = __ballot(r < a.keep);
    while (m) {
      v4f v[TBP_UNROLL];
      bool ok[TBP_UNROLL];
#pragma unroll
      for (int u = 0; u < TBP_UNROLL; ++u) {
        ok[u] = m != 0;
        const int i = ok[u] ? (int)__builtin_ctzll(m) : 0;
        m &= m - 1;
        const int t = 1 + __builtin_amdgcn_readlane(r, i);
        const int bb = b0 + wave + 4 * i;
        ok[u] = ok[u] && dok;
        if (ok[u]) v[u] = *(const v4f*)(a.dx + ((int64_t)bb * nt + t) * a.D + d);
      }
#pragma unroll
      for (int u = 0; u < TBP_UNROLL; ++u)
        if (ok[u]) acc += v[u];
    }
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && d < a.D) {
    const v4f sum = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    *(v4f*)(a.dpos + (int64_t)pr * a.D + d) = sum;
    if (pr == 0 && a.dcls) *(v4f*)(a.dcls + d) = sum;
  }
}

// decoder input: out[b,0] = y[b,0] + pos[0]; out[b,1+l] = (restore<keep ? y[b,1+restore] : mask_token) + pos[1+l]
__global__ void __launch_bounds__(NTH) unshuffle_fwd_kernel(const maeclip_unshuffle_args a) {
  const int64_t row = blockIdx.y;  // b*(1+L) + t
  const int d = (blockIdx.x * NTH + threadIdx.x) * 4;
  if (d >= a.D) return;
  const int b = (int)(row / (a.L + 1)), t = (int)(row % (a.L + 1));
  v4f v;
  if (t == 0) {
    v = *(const v4f*)(a.y + (int64_t)b * (a.keep + 1) * a.ldy + d);
  } else {
    const int r = a.ids_restore[(int64_t)b * a.L + t - 1];
    v = r < a.keep ? *(const v4f*)(a.y + ((int64_t)b * (a.keep + 1) + 1 + r) * a.ldy + d) : *(const v4f*)(a.mask_token + d);
  }
  v += *(const v4f*)(a.pos + (int64_t)t * a.D + d);
  *(v4f*)(a.out + row * a.D + d) = v;
}

// dy[b,0] = dout[b,0]; dy[b,1+r] = dout[b,1+l] for r = restore[b,l] < keep;
// partials: dmask = sum of dout rows of masked positions, colsum = sum of the
// dy rows. Workgroup (b, q) reads rows t = q, q+UQ, ... of sample b in natural
// order (coalesced 16-B loads; rows scattered only on the dy write side), wave
// w takes every 4th of them, lane = 4-column chunk; partial row b*UQ + q.
constexpr int UQ = 4;   // workgroups per sample
template <typename YT>
__global__ void __launch_bounds__(NTH) unshuffle_bwd_kernel(const maeclip_unshuffle_args a) {
  constexpr int MC = 4;   // <= 4 x 64 four-column chunks: D <= 1024
  __shared__ v4f red[2][NTH / 64][MC * 64];
  const int b = blockIdx.x, q = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nc = a.D / 4;
  v4f cs[MC], dm[MC];
#pragma unroll
  for (int i = 0; i < MC; ++i) cs[i] = dm[i] = v4f{0.f, 0.f, 0.f, 0.f};
  const float* base = a.dout + (int64_t)b * (a.L + 1) * a.D;
  YT* dyb = (YT*)a.dy + (int64_t)b * (a.keep + 1) * a.ldy;
  for (int t = q + UQ * wave; t < a.L + 1; t += UQ * (NTH / 64)) {
    int r = 0;
    bool kept = true;
    if (t > 0) {
      r = a.ids_restore[(int64_t)b * a.L + t - 1];
      kept = r < a.keep;
      r += 1;
    }
#pragma unroll
    for (int i = 0; i < MC; ++i) {
      const int c = lane + 64 * i;
      if (c < nc) {
        const v4f v = *(const v4f*)(base + (int64_t)t * a.D + 4 * c);
        if (kept) {
          st4<YT>(dyb + (int64_t)r * a.ldy + 4 * c, v);
          cs[i] += v;
        } else {
          dm[i] += v;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MC; ++i) {
    red[0][wave][lane + 64 * i] = cs[i];
    red[1][wave][lane + 64 * i] = dm[i];
  }
  __syncthreads();
  const int64_t prow = (int64_t)b * UQ + q;
  for (int c = threadIdx.x; c < nc; c += NTH) {
    const v4f s0 = ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    const v4f s1 = ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
    if (a.colsum_partial) *(v4f*)(a.colsum_partial + prow * a.D + 4 * c) = s0;
    if (a.dmask_partial) *(v4f*)(a.dmask_partial + prow * a.D + 4 * c) = s1;
  }
}

constexpr int PMAX = 1024;   // p*p*C <= 1024 (ViT-B/16: 768, ViT-L/14: 588)

// Target pixels of patch l of sample b into the wave's LDS row tg[P] in the
// HF patchify order k = (ky*p + kx)*C + c (modeling_vit_mae.py:739). The image
// is read in its own (c, ky, kx) order -- VW-float vectors along kx, so
// consecutive lanes read consecutive bytes of one pixel row -- and the
// channel interleave happens on the LDS write.
template <int VW>
__device__ __forceinline__ void load_target(const maeclip_mae_loss_args& a, int b, int l, float* tg, int lane) {
  const int C = a.C, p = a.p, w = a.S / p;
  const int py = l / w, px = l % w;
  const int vpr = p / VW, nv = C * p * vpr;
  const float* img = a.img + (int64_t)b * C * a.S * a.S + (int64_t)(py * p) * a.S + px * p;
  for (int v = lane; v < nv; v += 64) {
    const int r = v / vpr, kx = (v - r * vpr) * VW;
    const int c = r / p, ky = r - c * p;
    const float* src = img + ((int64_t)c * a.S + ky) * a.S + kx;
    float t[VW];
    if constexpr (VW == 4) {
      const v4f x = *(const v4f*)src;
      t[0] = x[0]; t[1] = x[1]; t[2] = x[2]; t[3] = x[3];
    } else if constexpr (VW == 2) {
      const float2 x = *(const float2*)src;
      t[0] = x.x; t[1] = x.y;
    } else {
      t[0] = src[0];
    }
#pragma unroll
    for (int e = 0; e < VW; ++e) tg[(ky * p + kx + e) * C + c] = t[e];
  }
}

// The same target row from the uint8 HWC pixels: HF's patchify order
// (ky, kx, c) IS the HWC byte order, so patch row ky is p*C contiguous bytes
// of image row py*p + ky, copied to tg[ky*p*C ..] normalised (A.Normalize,
// dataset.py:49; channel c = byte index mod C). VB = 16: 16-B loads (p*C and
// S*C multiples of 16), else bytes.
template <int VB>
__device__ __forceinline__ void load_target_u8(const maeclip_mae_loss_args& a, const NormConst& k, int b, int l,
                                               float* tg, int lane) {
  const int C = a.C, p = a.p, w = a.S / p, R = p * C;
  const int py = l / w, px = l % w;
  const uint8_t* img = a.img_u8 + (((int64_t)b * a.S + py * p) * a.S + (int64_t)px * p) * C;
  const int64_t rs = (int64_t)a.S * C;
  if constexpr (VB == 16) {
    const int vpr = R / 16;
    for (int v = lane; v < p * vpr; v += 64) {
      const int ky = v / vpr, off = (v - ky * vpr) * 16;
      const v4u q = *(const v4u*)(img + ky * rs + off);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kk = off + e;
        tg[ky * R + kk] = mc_norm_px((q[e >> 2] >> (8 * (e & 3))) & 0xffu, k, kk % C);
      }
    }
  } else {
    for (int v = lane; v < p * R; v += 64) {
      const int ky = v / R, kk = v - ky * R;
      tg[v] = mc_norm_px(img[ky * rs + kk], k, kk % C);
    }
  }
}

// norm_pix_loss: targets -> (t - mean) / sqrt(var + 1e-6), unbiased var (HF)
__device__ __forceinline__ void norm_target(float* tg, int P, int lane) {
  float s = 0.f;
  for (int k = lane; k < P; k += 64) s += tg[k];
  const float mean = wave_sum(s) / (float)P;
  float ss = 0.f;
  for (int k = lane; k < P; k += 64) {
    const float d = tg[k] - mean;
    ss += d * d;
  }
  const float inv = 1.f / sqrtf(wave_sum(ss) / (float)(P - 1) + 1.0e-6f);
  for (int k = lane; k < P; k += 64) tg[k] = (tg[k] - mean) * inv;
}

// VW > 0: fp32 NCHW image, VW floats per load; VW < 0: uint8 HWC pixels,
// -VW bytes per load
template <int VW>
__device__ __forceinline__ void load_target_any(const maeclip_mae_loss_args& a, const NormConst& k, int b, int l,
                                                float* tg, int lane) {
  if constexpr (VW > 0) load_target<VW>(a, b, l, tg, lane);
  else load_target_u8<-VW>(a, k, b, l, tg, lane);
  if (a.norm_pix) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    norm_target(tg, a.C * a.p * a.p, lane);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per patch (b, l); only masked patches (mask 1) read anything.
template <typename PT, int VW>
__global__ void __launch_bounds__(NTH) mae_loss_fwd_kernel(const maeclip_mae_loss_args a, NormConst nk) {
  __shared__ float tgs[NTH / 64][PMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t wid = (int64_t)blockIdx.x * (NTH / 64) + wave;
  if (wid >= (int64_t)a.B * a.L) return;
  const float mk = a.mask[wid];
  if (mk == 0.f) {
    if (lane == 0) a.row_loss[wid] = 0.f;
    return;
  }
  const int b = (int)(wid / a.L), l = (int)(wid % a.L);
  const int P = a.C * a.p * a.p;
  float* tg = tgs[wave];
  load_target_any<VW>(a, nk, b, l, tg, lane);
  const PT* pred = (const PT*)a.pred + ((int64_t)b * (a.L + 1) + 1 + l) * a.ldp;
  float s = 0.f;
  for (int k = 4 * lane; k < P; k += 256) {
    const v4f pv = ld4<PT>(pred + k);
    const v4f tv = *(const v4f*)(tg + k);
    const v4f d = pv - tv;
    s += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
  }
  s = wave_sum(s);
  if (lane == 0) a.row_loss[wid] = mk * s / (float)P;
}

// dpred rows of a sample: workgroup (b, chunk of RB = 16 rows of 1+L), wave w
// takes rows r0 + w + 4i; row 0 (cls) and unmasked rows are written as zeros
// without reading. Pad columns [P, lddp) are zeroed. Per-workgroup column sums
// (decoder_pred bias gradient) -> colsum_partial[b * nchunk + chunk][P].
constexpr int RB = 16;
template <typename PT, int VW>
__global__ void __launch_bounds__(NTH) mae_loss_bwd_kernel(const maeclip_mae_loss_args a, NormConst nk) {
  __shared__ float tgs[NTH / 64][PMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x, chunk = blockIdx.y;
  const int P = a.C * a.p * a.p;
  const float gscale = (a.grad_out ? a.grad_out[0] : 1.f) * a.loss_scale * 2.f / ((float)P * a.mask_count);
  v4f cs[PMAX / 256];
#pragma unroll
  for (int i = 0; i < PMAX / 256; ++i) cs[i] = v4f{0.f, 0.f, 0.f, 0.f};
  float* tg = tgs[wave];
  for (int rr = wave; rr < RB; rr += NTH / 64) {
    const int r = chunk * RB + rr;
    if (r > a.L) break;
    PT* drow = (PT*)a.dpred + ((int64_t)b * (a.L + 1) + r) * a.lddp;
    const float mk = r > 0 ? a.mask[(int64_t)b * a.L + r - 1] : 0.f;
    if (mk == 0.f) {
      for (int k = 4 * lane; k < (int)a.lddp; k += 256) st4<PT>(drow + k, v4f{0.f, 0.f, 0.f, 0.f});
      continue;
    }
    const PT* prow = (const PT*)a.pred + ((int64_t)b * (a.L + 1) + r) * a.ldp;
    load_target_any<VW>(a, nk, b, r - 1, tg, lane);
    const float g = gscale * mk;
#pragma unroll
    for (int i = 0; i < PMAX / 256; ++i) {
      const int k = 4 * lane + 256 * i;
      if (k < P) {
        const v4f d = (ld4<PT>(prow + k) - *(const v4f*)(tg + k)) * g;
        st4<PT>(drow + k, d);
        cs[i] += d;
      } else if (k < (int)a.lddp) {
        st4<PT>(drow + k, v4f{0.f, 0.f, 0.f, 0.f});
      }
    }
    // the next row's target overwrites tg: every lane's reads of it are done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (!a.colsum_partial) return;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PMAX / 256; ++i) *(v4f*)(tg + 4 * lane + 256 * i) = cs[i];
  __syncthreads();
  float* prow = a.colsum_partial + ((int64_t)b * gridDim.y + chunk) * P;
  for (int k = threadIdx.x; k < P; k += NTH)
    prow[k] = ((tgs[0][k] + tgs[1][k]) + tgs[2][k]) + tgs[3][k];
}

}  // namespace

extern "C" int32_t maeclip_mask_ids(const maeclip_mask_args* a, void* stream) {
  MC_CHECK_ARG(a && a->ids_shuffle && a->ids_restore, "maeclip_mask_ids: null pointer");
  MC_CHECK_ARG(a->L > 0 && a->L <= 1024 && a->len_keep >= 0 && a->len_keep <= a->L && a->B > 0,
               "maeclip_mask_ids: bad sizes (L<=1024)");
  hipLaunchKernelGGL(mask_ids_kernel, dim3(a->B), dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_mask_ids");
  return 0;
}

extern "C" int32_t maeclip_patch_gather(const maeclip_patch_args* a, void* stream) {
  MC_CHECK_ARG(a && (a->img || a->img_u8) && a->out, "maeclip_patch_gather: null pointer");
  MC_CHECK_ARG(a->p > 0 && a->S % a->p == 0 && a->keep > 0 && a->ld_out >= (int64_t)a->C * a->p * a->p,
               "maeclip_patch_gather: bad sizes");
  if (a->img_u8) {
    NormConst k;
    MC_CHECK_ARG(a->C == 3, "maeclip_patch_gather: uint8 pixels need C == 3 (RGB)");
    MC_CHECK_ARG(mc_norm_const(a->u8_mean, a->u8_std, a->u8_max_pixel, k),
                 "maeclip_patch_gather: u8_std and u8_max_pixel must be > 0");
    const int64_t nseg = (int64_t)a->B * a->keep * a->p;
    dim3 grid((unsigned)((nseg + NTH - 1) / NTH));
    const bool vec = a->p == 16 && ((uintptr_t)a->img_u8 & 15) == 0 && (a->S * 3) % 16 == 0;
    hipStream_t st = (hipStream_t)stream;
    if (a->dtype == MAECLIP_BF16) {
      if (vec) hipLaunchKernelGGL((patch_gather_u8_kernel<bf16_t, true>), grid, dim3(NTH), 0, st, *a, k);
      else hipLaunchKernelGGL((patch_gather_u8_kernel<bf16_t, false>), grid, dim3(NTH), 0, st, *a, k);
    } else {
      if (vec) hipLaunchKernelGGL((patch_gather_u8_kernel<float, true>), grid, dim3(NTH), 0, st, *a, k);
      else hipLaunchKernelGGL((patch_gather_u8_kernel<float, false>), grid, dim3(NTH), 0, st, *a, k);
    }
    MC_CHECK_LAUNCH("maeclip_patch_gather(u8)");
    return 0;
  }
  const int64_t nseg = (int64_t)a->B * a->keep * a->C * a->p;
  hipStream_t st = (hipStream_t)stream;
  const int ob = a->dtype == MAECLIP_BF16 ? 2 : 4;
  if (a->p % 4 == 0 && a->S % 4 == 0 && ((uintptr_t)a->img & 15) == 0 && ((uintptr_t)a->out & 7) == 0 &&
      (a->ld_out * ob) % 8 == 0) {
    const int64_t nt = nseg * (a->p / 4);
    dim3 grid((unsigned)((nt + NTH - 1) / NTH));
    if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((patch_gather4_kernel<bf16_t>), grid, dim3(NTH), 0, st, *a);
    else hipLaunchKernelGGL((patch_gather4_kernel<float>), grid, dim3(NTH), 0, st, *a);
    MC_CHECK_LAUNCH("maeclip_patch_gather");
    return 0;
  }
  dim3 grid((unsigned)((nseg + NTH - 1) / NTH));
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((patch_gather_kernel<bf16_t>), grid, dim3(NTH), 0, st, *a);
  else hipLaunchKernelGGL((patch_gather_kernel<float>), grid, dim3(NTH), 0, st, *a);
  MC_CHECK_LAUNCH("maeclip_patch_gather");
  return 0;
}

extern "C" int32_t maeclip_tokens_fwd(const maeclip_tokens_args* a, void* stream) {
  MC_CHECK_ARG(a && a->y && a->pos && a->cls && a->x && a->D % 4 == 0, "maeclip_tokens_fwd: bad args");
  dim3 grid((unsigned)((a->D / 4 + NTH - 1) / NTH), (unsigned)((int64_t)a->B * (a->keep + 1)));
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((tokens_fwd_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((tokens_fwd_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_tokens_fwd");
  return 0;
}

extern "C" int32_t maeclip_tokens_bwd(const maeclip_tokens_args* a, void* stream) {
  MC_CHECK_ARG(a && a->dx && a->dpos && a->D % 4 == 0, "maeclip_tokens_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (a->dy) {
    dim3 grid((unsigned)((a->D / 4 + NTH - 1) / NTH), (unsigned)((int64_t)a->B * a->keep));
    if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((tokens_bwd_dy_kernel<bf16_t>), grid, dim3(NTH), 0, s, *a);
    else hipLaunchKernelGGL((tokens_bwd_dy_kernel<float>), grid, dim3(NTH), 0, s, *a);
    MC_CHECK_LAUNCH("maeclip_tokens_bwd(dy)");
  }
  MC_CHECK_ARG(((uintptr_t)a->dx & 15) == 0 && ((uintptr_t)a->dpos & 15) == 0 && (!a->dcls || ((uintptr_t)a->dcls & 15) == 0),
               "maeclip_tokens_bwd: dx / dpos / dcls must be 16-byte aligned");
  dim3 g2((unsigned)(a->L + 1), (unsigned)((a->D / 4 + 63) / 64));
  hipLaunchKernelGGL(tokens_bwd_pos_kernel, g2, dim3(NTH), 0, s, *a);
  MC_CHECK_LAUNCH("maeclip_tokens_bwd(pos)");
  return 0;
}

extern "C" int32_t maeclip_unshuffle_fwd(const maeclip_unshuffle_args* a, void* stream) {
  MC_CHECK_ARG(a && a->y && a->ids_restore && a->mask_token && a->pos && a->out && a->D % 4 == 0,
               "maeclip_unshuffle_fwd: bad args");
  dim3 grid((unsigned)((a->D / 4 + NTH - 1) / NTH), (unsigned)((int64_t)a->B * (a->L + 1)));
  hipLaunchKernelGGL(unshuffle_fwd_kernel, grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_unshuffle_fwd");
  return 0;
}

extern "C" int32_t maeclip_unshuffle_bwd(const maeclip_unshuffle_args* a, void* stream) {
  MC_CHECK_ARG(a && a->dout && a->ids_restore && a->dy, "maeclip_unshuffle_bwd: bad args");
  MC_CHECK_ARG(a->D % 4 == 0 && a->D <= 1024 && a->ldy % 4 == 0 && ((uintptr_t)a->dout & 15) == 0 &&
                   ((uintptr_t)a->dy & 7) == 0,
               "maeclip_unshuffle_bwd: D must be a multiple of 4 (<= 1024), rows aligned");
  dim3 grid((unsigned)a->B, UQ);
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((unshuffle_bwd_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((unshuffle_bwd_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_unshuffle_bwd");
  return 0;
}

extern "C" int32_t maeclip_unshuffle_bwd_partial_rows(int32_t B) { return B * UQ; }

namespace {
int check_loss(const maeclip_mae_loss_args* a, bool bwd, NormConst& k) {
  MC_CHECK_ARG(a && a->pred && (a->img || a->img_u8) && a->mask, "maeclip_mae_loss: null pointer");
  const int P = a->C * a->p * a->p;
  MC_CHECK_ARG(P <= PMAX && P % 4 == 0 && a->ldp % 4 == 0 && a->ldp >= P && a->S % a->p == 0,
               "maeclip_mae_loss: p*p*C must be a multiple of 4, <= %d", PMAX);
  if (a->img_u8) {
    MC_CHECK_ARG(a->C == 3, "maeclip_mae_loss: uint8 pixels need C == 3 (RGB)");
    MC_CHECK_ARG(mc_norm_const(a->u8_mean, a->u8_std, a->u8_max_pixel, k),
                 "maeclip_mae_loss: u8_std and u8_max_pixel must be > 0");
  } else {
    k = NormConst{};
    MC_CHECK_ARG(((uintptr_t)a->img & 15) == 0 && a->S % 4 == 0, "maeclip_mae_loss: misaligned image");
  }
  MC_CHECK_ARG(((uintptr_t)a->pred & 7) == 0, "maeclip_mae_loss: misaligned pred");
  if (bwd) MC_CHECK_ARG(a->dpred && a->lddp % 4 == 0 && a->lddp >= P && a->mask_count > 0.f,
                        "maeclip_mae_loss_bwd: bad dpred / mask_count");
  else MC_CHECK_ARG(a->row_loss != nullptr, "maeclip_mae_loss_fwd: null row_loss");
  return 0;
}

// load width of the target read: fp32 NCHW floats (4 / 2 / 1) or, for uint8
// HWC pixels, 16-B vectors (-16) when every patch row is 16-B aligned, else bytes (-1)
int loss_vw(const maeclip_mae_loss_args& a) {
  if (a.img_u8)
    return ((a.p * a.C) % 16 == 0 && ((int64_t)a.S * a.C) % 16 == 0 && ((uintptr_t)a.img_u8 & 15) == 0) ? -16 : -1;
  return a.p % 4 == 0 ? 4 : (a.p % 2 == 0 ? 2 : 1);
}

}  // namespace

extern "C" int32_t maeclip_mae_loss_bwd_partial_rows(int32_t B, int32_t L) { return B * ((L + 1 + RB - 1) / RB); }

extern "C" int32_t maeclip_mae_loss_fwd(const maeclip_mae_loss_args* a, void* stream) {
  NormConst k;
  if (int e = check_loss(a, false, k)) return e;
  const int64_t nw = (int64_t)a->B * a->L;
  dim3 grid((unsigned)((nw + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int vw = loss_vw(*a);
#define FWD(PT, VW) hipLaunchKernelGGL((mae_loss_fwd_kernel<PT, VW>), grid, dim3(NTH), 0, s, *a, k)
  if (a->dtype == MAECLIP_BF16) {
    switch (vw) { case 4: FWD(bf16_t, 4); break; case 2: FWD(bf16_t, 2); break; case 1: FWD(bf16_t, 1); break;
                  case -16: FWD(bf16_t, -16); break; default: FWD(bf16_t, -1); }
  } else {
    switch (vw) { case 4: FWD(float, 4); break; case 2: FWD(float, 2); break; case 1: FWD(float, 1); break;
                  case -16: FWD(float, -16); break; default: FWD(float, -1); }
  }
#undef FWD
  MC_CHECK_LAUNCH("maeclip_mae_loss_fwd");
  return 0;
}

extern "C" int32_t maeclip_mae_loss_bwd(const maeclip_mae_loss_args* a, void* stream) {
  NormConst k;
  if (int e = check_loss(a, true, k)) return e;
  dim3 grid((unsigned)a->B, (unsigned)((a->L + 1 + RB - 1) / RB));
  hipStream_t s = (hipStream_t)stream;
  const int vw = loss_vw(*a);
#define BWD(PT, VW) hipLaunchKernelGGL((mae_loss_bwd_kernel<PT, VW>), grid, dim3(NTH), 0, s, *a, k)
  if (a->dtype == MAECLIP_BF16) {
    switch (vw) { case 4: BWD(bf16_t, 4); break; case 2: BWD(bf16_t, 2); break; case 1: BWD(bf16_t, 1); break;
                  case -16: BWD(bf16_t, -16); break; default: BWD(bf16_t, -1); }
  } else {
    switch (vw) { case 4: BWD(float, 4); break; case 2: BWD(float, 2); break; case 1: BWD(float, 1); break;
                  case -16: BWD(float, -16); break; default: BWD(float, -1); }
  }
#undef BWD
  MC_CHECK_LAUNCH("maeclip_mae_loss_bwd");
  return 0;
}
