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
// dpos[1+l] = sum_b [kept] dx[b,1+restore[b,l]] ; dpos[0] = dcls = sum_b dx[b,0]
__global__ void __launch_bounds__(NTH) tokens_bwd_pos_kernel(const maeclip_tokens_args a) {
  const int pr = blockIdx.y;  // 0..L
  const int d = blockIdx.x * NTH + threadIdx.x;
  if (d >= a.D) return;
  const int nt = a.keep + 1;
  float s = 0.f;
  for (int b = 0; b < a.B; ++b) {
    int t;
    if (pr == 0) {
      t = 0;
    } else {
      const int l = pr - 1;
      const int r = a.ids_restore ? a.ids_restore[(int64_t)b * a.L + l] : l;
      if (r >= a.keep) continue;
      t = 1 + r;
    }
    s += a.dx[((int64_t)b * nt + t) * a.D + d];
  }
  a.dpos[(int64_t)pr * a.D + d] = s;
  if (pr == 0 && a.dcls) a.dcls[d] = s;
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

// dy[b,0] = dout[b,0]; dy[b,1+j] = dout[b,1+shuffle[b,j]];  partials per sample:
// dmask[b] = sum_{j>=keep} dout[b,1+shuffle[b,j]],  colsum[b] = sum_t dy[b,t]
template <typename YT>
__global__ void __launch_bounds__(NTH) unshuffle_bwd_kernel(const maeclip_unshuffle_args a) {
  const int b = blockIdx.y;
  const int d = (blockIdx.x * NTH + threadIdx.x);
  if (d >= a.D) return;
  const float* base = a.dout + (int64_t)b * (a.L + 1) * a.D + d;
  YT* dyb = (YT*)a.dy + (int64_t)b * (a.keep + 1) * a.ldy + d;
  float v0 = base[0];
  st_from_f<YT>(dyb, v0);
  float cs = v0, dm = 0.f;
  for (int j = 0; j < a.L; ++j) {
    const int l = a.ids_shuffle[(int64_t)b * a.L + j];
    const float v = base[(int64_t)(1 + l) * a.D];
    if (j < a.keep) {
      st_from_f<YT>(dyb + (int64_t)(1 + j) * a.ldy, v);
      cs += v;
    } else {
      dm += v;
    }
  }
  if (a.dmask_partial) a.dmask_partial[(int64_t)b * a.D + d] = dm;
  if (a.colsum_partial) a.colsum_partial[(int64_t)b * a.D + d] = cs;
}

constexpr int MAXK = 16;  // elements per lane -> p*p*C <= 1024

// target element k = (ky*p + kx)*C + c of patch l of sample b
__device__ __forceinline__ float target_px(const maeclip_mae_loss_args& a, int b, int l, int k) {
  const int C = a.C, p = a.p, w = a.S / p;
  const int c = k % C, pix = k / C;
  const int ky = pix / p, kx = pix % p;
  const int py = l / w, px = l % w;
  return a.img[(((int64_t)b * C + c) * a.S + py * p + ky) * a.S + px * p + kx];
}

template <typename PT>
__device__ __forceinline__ void patch_diff(const maeclip_mae_loss_args& a, int b, int l, int lane, float (&df)[MAXK]) {
  const int P = a.C * a.p * a.p;
  const PT* pred = (const PT*)a.pred + ((int64_t)b * (a.L + 1) + 1 + l) * a.ldp;
  float t[MAXK];
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    const int k = lane + 64 * i;
    t[i] = k < P ? target_px(a, b, l, k) : 0.f;
  }
  if (a.norm_pix) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) s += t[i];
    const float mean = wave_sum(s) / P;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXK; ++i)
      if (lane + 64 * i < P) ss += (t[i] - mean) * (t[i] - mean);
    const float var = wave_sum(ss) / (P - 1);
    const float inv = 1.f / sqrtf(var + 1.0e-6f);
#pragma unroll
    for (int i = 0; i < MAXK; ++i) t[i] = (t[i] - mean) * inv;
  }
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    const int k = lane + 64 * i;
    df[i] = k < P ? ld_as_f<PT>(pred + k) - t[i] : 0.f;
  }
}

template <typename PT>
__global__ void __launch_bounds__(NTH) mae_loss_fwd_kernel(const maeclip_mae_loss_args a) {
  const int64_t wid = (int64_t)blockIdx.x * (NTH / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wid >= (int64_t)a.B * a.L) return;
  const int b = (int)(wid / a.L), l = (int)(wid % a.L);
  const float mk = a.mask[wid];
  float df[MAXK];
  patch_diff<PT>(a, b, l, lane, df);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) s += df[i] * df[i];
  s = wave_sum(s);
  if (lane == 0) a.row_loss[wid] = mk * s / (float)(a.C * a.p * a.p);
}

// one workgroup per sample; waves stride over its 1+L rows (row 0 = cls -> 0)
template <typename PT>
__global__ void __launch_bounds__(NTH) mae_loss_bwd_kernel(const maeclip_mae_loss_args a) {
  __shared__ float red[NTH / 64][MAXK * 64];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int P = a.C * a.p * a.p;
  const float gscale = (a.grad_out ? a.grad_out[0] : 1.f) * a.loss_scale * 2.f / ((float)P * a.mask_count);
  float cs[MAXK];
#pragma unroll
  for (int i = 0; i < MAXK; ++i) cs[i] = 0.f;
  for (int r = wave; r < a.L + 1; r += NTH / 64) {
    PT* drow = (PT*)a.dpred + ((int64_t)b * (a.L + 1) + r) * a.lddp;
    float df[MAXK];
    float mk = 0.f;
    if (r > 0) {
      mk = a.mask[(int64_t)b * a.L + r - 1];
      patch_diff<PT>(a, b, r - 1, lane, df);
    }
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const int k = lane + 64 * i;
      if (k < P) {
        const float g = (r > 0) ? gscale * mk * df[i] : 0.f;
        st_from_f<PT>(drow + k, g);
        cs[i] += g;
      }
    }
  }
  if (a.colsum_partial) {
#pragma unroll
    for (int i = 0; i < MAXK; ++i) red[wave][lane + 64 * i] = cs[i];
    __syncthreads();
    for (int k = threadIdx.x; k < P; k += NTH) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NTH / 64; ++w) s += red[w][k];
      a.colsum_partial[(int64_t)b * P + k] = s;
    }
  }
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
  MC_CHECK_ARG(a && a->img && a->out, "maeclip_patch_gather: null pointer");
  MC_CHECK_ARG(a->p > 0 && a->S % a->p == 0 && a->keep > 0 && a->ld_out >= (int64_t)a->C * a->p * a->p,
               "maeclip_patch_gather: bad sizes");
  const int64_t nseg = (int64_t)a->B * a->keep * a->C * a->p;
  dim3 grid((unsigned)((nseg + NTH - 1) / NTH));
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((patch_gather_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((patch_gather_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
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
  dim3 g2((unsigned)((a->D + NTH - 1) / NTH), (unsigned)(a->L + 1));
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
  MC_CHECK_ARG(a && a->dout && a->ids_shuffle && a->dy, "maeclip_unshuffle_bwd: bad args");
  dim3 grid((unsigned)((a->D + NTH - 1) / NTH), (unsigned)a->B);
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((unshuffle_bwd_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((unshuffle_bwd_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_unshuffle_bwd");
  return 0;
}

extern "C" int32_t maeclip_mae_loss_fwd(const maeclip_mae_loss_args* a, void* stream) {
  MC_CHECK_ARG(a && a->pred && a->img && a->mask && a->row_loss, "maeclip_mae_loss_fwd: null pointer");
  MC_CHECK_ARG(a->C * a->p * a->p <= MAXK * 64, "maeclip_mae_loss_fwd: patch too large");
  const int64_t nw = (int64_t)a->B * a->L;
  dim3 grid((unsigned)((nw + 3) / 4));
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((mae_loss_fwd_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((mae_loss_fwd_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_mae_loss_fwd");
  return 0;
}

extern "C" int32_t maeclip_mae_loss_bwd(const maeclip_mae_loss_args* a, void* stream) {
  MC_CHECK_ARG(a && a->pred && a->img && a->mask && a->dpred, "maeclip_mae_loss_bwd: null pointer");
  MC_CHECK_ARG(a->C * a->p * a->p <= MAXK * 64 && a->mask_count > 0.f, "maeclip_mae_loss_bwd: bad sizes");
  dim3 grid((unsigned)a->B);
  if (a->dtype == MAECLIP_BF16) hipLaunchKernelGGL((mae_loss_bwd_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  else hipLaunchKernelGGL((mae_loss_bwd_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, *a);
  MC_CHECK_LAUNCH("maeclip_mae_loss_bwd");
  return 0;
}
