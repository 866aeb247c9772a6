// HBM-bound helper kernels: deterministic column reductions (bias/LN-param
// gradients), timm global_pool="avg" (modules.py:17-19 -> VisionTransformer
// forward_head), dropout masks, DistilBERT embedding gather, multi-tensor
// fp32->bf16 weight casts and the fused multi-tensor AdamW step that replaces
// torch.optim.AdamW (main.py:101-103,59).
#include "common.h"
#include "../../include/maeclip.h"

namespace {
constexpr int NTH = 256;

// out[n] (+)= sum_p partial[p][n]  -- fixed summation order, vectorised over n
__global__ void __launch_bounds__(NTH) colsum_reduce_kernel(const float* __restrict__ part, int64_t P, int64_t N,
                                                            float* __restrict__ out, int accumulate, float scale) {
  const int64_t n = (int64_t)blockIdx.x * NTH + threadIdx.x;
  if (n >= N) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int64_t p = 0;
  for (; p + 3 < P; p += 4) {
    s0 += part[(p + 0) * N + n];
    s1 += part[(p + 1) * N + n];
    s2 += part[(p + 2) * N + n];
    s3 += part[(p + 3) * N + n];
  }
  for (; p < P; ++p) s0 += part[p * N + n];
  const float s = ((s0 + s1) + (s2 + s3)) * scale;
  out[n] = accumulate ? out[n] + s : s;
}

// pass 1 of a tall reduction: block (64 columns x 64 rows) -> one row of scratch
__global__ void __launch_bounds__(NTH) colsum_pass1_kernel(const float* __restrict__ part, int64_t P, int64_t N,
                                                           float* __restrict__ scratch) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + c;
  const int64_t r0 = (int64_t)blockIdx.y * 64;
  float s = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int i = ph; i < 64; i += 4) {
      const int64_t r = r0 + i;
      if (r < P) s += part[r * N + n];
    }
  }
  red[ph][c] = s;
  __syncthreads();
  if (ph == 0 && n < N) scratch[(int64_t)blockIdx.y * N + n] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// single-vector sum, pass 1 (P > VS_CHUNK): block b sums x[b*VS_CHUNK ..
// +VS_CHUNK) in a fixed order (16 B per lane per iteration) -> scratch[b]
constexpr int VS_CHUNK = NTH * 16;
__global__ void __launch_bounds__(NTH) vec_sum_pass1_kernel(const float* __restrict__ x, int64_t P,
                                                            float* __restrict__ scratch) {
  __shared__ float red[NTH / 64];
  const int64_t base = (int64_t)blockIdx.x * VS_CHUNK;
  const int64_t end = min(base + (int64_t)VS_CHUNK, P);
  float s = 0.f;
  if (end - base == VS_CHUNK && ((uintptr_t)(x + base) & 15) == 0) {
#pragma unroll
    for (int i = 0; i < VS_CHUNK / (NTH * 4); ++i) {
      const v4f v = *(const v4f*)(x + base + (int64_t)(i * NTH + threadIdx.x) * 4);
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
  } else {
    for (int64_t i = base + threadIdx.x; i < end; i += NTH) s += x[i];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) scratch[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// single-vector sum (N == 1): one workgroup, fixed-order tree (after pass 1
// when P > VS_CHUNK, so the one workgroup reads at most a few hundred floats)
__global__ void __launch_bounds__(NTH) vec_sum_kernel(const float* __restrict__ x, int64_t P, float* __restrict__ out,
                                                      int accumulate, float scale) {
  __shared__ float red[NTH / 64];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < P; i += NTH) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NTH / 64; ++w) t += red[w];
    t *= scale;
    out[0] = accumulate ? out[0] + t : t;
  }
}

// feat[b] = mean_{t=1..n-1} x[b,t,:]   (timm global_pool="avg", num_prefix_tokens=1)
__global__ void __launch_bounds__(NTH) pool_fwd_kernel(const float* __restrict__ x, int n, int D, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int d = blockIdx.x * NTH + threadIdx.x;
  if (d >= D) return;
  const float* p = x + (int64_t)b * n * D + d;
  float s = 0.f;
  for (int t = 1; t < n; ++t) s += p[(int64_t)t * D];
  out[(int64_t)b * D + d] = s / (float)(n - 1);
}
__global__ void __launch_bounds__(NTH) pool_bwd_kernel(const float* __restrict__ dout, int n, int D, float* __restrict__ dx,
                                                       int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x;
  const int64_t total = (int64_t)gridDim.y * n * D;
  (void)total;
  const int b = blockIdx.y;
  if (i >= (int64_t)n * D) return;
  const int t = (int)(i / D), d = (int)(i % D);
  const float v = t == 0 ? 0.f : dout[(int64_t)b * D + d] / (float)(n - 1);
  float* o = dx + (int64_t)b * n * D + i;
  *o = accumulate ? *o + v : v;
}

// y = x * keep/(1-p) with the same mask function as the LayerNorm input dropout
__global__ void __launch_bounds__(NTH) dropout_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t M, int D,
                                                      int64_t ld, float p, uint64_t seed, const int64_t* step_ptr) {
  const int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x;
  if (i >= M * D) return;
  const int64_t r = i / D;
  const int c = (int)(i % D);
  const uint32_t thr = (uint32_t)((double)p * 4294967296.0);
  const float k = mc_hash4(mc_step_seed(seed, step_ptr), (uint64_t)r, (uint64_t)c, 0x4c4eull) >= thr ? 1.f / (1.f - p) : 0.f;
  y[r * ld + c] = x[r * ld + c] * k;
}

// DistilBERT Embeddings (modeling_distilbert.py:92-117) up to the LayerNorm:
// out[b*T+t] = word[ids[b,t]] + pos[t]
__global__ void __launch_bounds__(NTH) embed_kernel(const int64_t* __restrict__ ids, const float* __restrict__ word,
                                                    const float* __restrict__ pos, int T, int D, int64_t V,
                                                    float* __restrict__ out, const int64_t* __restrict__ mask_in,
                                                    float* __restrict__ mask_out) {
  const int64_t row = blockIdx.y;
  const int d = (blockIdx.x * NTH + threadIdx.x) * 4;
  if (mask_out && d == 0) mask_out[row] = (float)mask_in[row];
  if (d >= D) return;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const int t = (int)(row % T);
  v4f w = *(const v4f*)(word + id * D + d);
  v4f pp = *(const v4f*)(pos + (int64_t)t * D + d);
  *(v4f*)(out + row * D + d) = w + pp;
}


// colsum partials of a row matrix (bias gradient of a Linear whose output
// gradient arrives un-reduced), optionally emitting a bf16 copy of the rows.
constexpr int RC_MAXC = 8;  // D <= 2048
// Q8 (with out_bf): also the fp8 rows of the bf16 copy, bit-identical to
// maeclip_quant_rows_fp8 of it (the fp8 stack's top fc2-dgrad operand)
template <typename T, bool Q8 = false>
__global__ void __launch_bounds__(NTH) rows_colsum_kernel(const T* __restrict__ x, int64_t M, int D, int64_t ld,
                                                          bf16_t* __restrict__ out_bf, float* __restrict__ partial,
                                                          uint8_t* __restrict__ q8 = nullptr, int64_t ldq8 = 0,
                                                          float* __restrict__ q8_scale = nullptr, bool e5 = false) {
  __shared__ float red[NTH / 64][RC_MAXC * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[RC_MAXC][4];
#pragma unroll
  for (int c = 0; c < RC_MAXC; ++c) acc[c][0] = acc[c][1] = acc[c][2] = acc[c][3] = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * (NTH / 64) + wave; r < M; r += (int64_t)gridDim.x * (NTH / 64)) {
    float rv[Q8 ? RC_MAXC : 1][4];
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < RC_MAXC; ++c) {
      const int e = c * 256 + lane * 4;
      if (e < D) {
        const v4f v = ld4<T>(x + r * ld + e);
        acc[c][0] += v[0]; acc[c][1] += v[1]; acc[c][2] += v[2]; acc[c][3] += v[3];
        if (out_bf) st4<bf16_t>(out_bf + r * D + e, v);
        if constexpr (Q8) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            rv[c][j] = bf2f(f2bf(v[j]));
            amax = fmaxf(amax, fabsf(rv[c][j]));
          }
        }
      } else if constexpr (Q8) {
        rv[c][0] = rv[c][1] = rv[c][2] = rv[c][3] = 0.f;
      }
    }
    if constexpr (Q8) quant_row_fp8<RC_MAXC>(rv, amax, e5, q8 + r * ldq8, q8_scale + r, D, lane);
  }
#pragma unroll
  for (int c = 0; c < RC_MAXC; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = c * 256 + lane * 4 + j;
      if (e < D) red[wave][e] = acc[c][j];
    }
  __syncthreads();
  for (int e = threadIdx.x; e < D; e += NTH) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NTH / 64; ++k) s += red[k][e];
    partial[(int64_t)blockIdx.x * D + e] = s;
  }
}
int rows_colsum_grid(int64_t M) {
  const int64_t g = (M + 3) / 4;
  return (int)(g < 512 ? (g < 1 ? 1 : g) : 512);
}

// Many column reductions in ONE launch: block -> (entry, 64-column chunk),
// 4 row phases x 64 columns, fixed summation order.
__global__ void __launch_bounds__(NTH) colsum_multi_kernel(const maeclip_colsum_entry* __restrict__ e, int ne) {
  __shared__ float red[4][64];
  int lo = 0, hi = ne - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (e[mid].block_start <= (int64_t)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const maeclip_colsum_entry en = e[lo];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int64_t n = (blockIdx.x - en.block_start) * 64 + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (n < en.N) {
    const float* p = en.partial + n;
    int64_t r = ph;
    for (; r + 12 < en.P; r += 16) {
      s0 += p[r * en.N];
      s1 += p[(r + 4) * en.N];
      s2 += p[(r + 8) * en.N];
      s3 += p[(r + 12) * en.N];
    }
    for (; r < en.P; r += 4) s0 += p[r * en.N];
  }
  red[ph][c] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ph == 0 && n < en.N) {
    const float v = ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) * en.scale;
    en.out[n] = en.accumulate ? en.out[n] + v : v;
  }
}

// ---- multi-tensor: one block per CHUNK elements, entries located by binary search
constexpr int64_t CHUNK = 4096;

__device__ __forceinline__ int find_entry(const maeclip_mt_entry* e, int ne, int64_t blk) {
  int lo = 0, hi = ne - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (e[mid].chunk_start <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(NTH) cast_multi_kernel(const maeclip_mt_entry* __restrict__ e, int ne) {
  const int k = find_entry(e, ne, blockIdx.x);
  const int64_t base = (blockIdx.x - e[k].chunk_start) * CHUNK;
  const float* src = (const float*)e[k].p0;
  bf16_t* dst = (bf16_t*)e[k].p4;
  const int64_t n = e[k].n;
  for (int64_t i = base + threadIdx.x * 4; i < base + CHUNK && i < n; i += NTH * 4) {
    if (i + 3 < n) {
      st4<bf16_t>(dst + i, *(const v4f*)(src + i));
    } else {
      for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
    }
  }
}

// flat dtype conversion dst = scale * src (f32 <-> bf16, RNE): the bf16
// gradient all-reduce buckets of data parallelism (distributed.py)
template <typename ST, typename DT>
__global__ void __launch_bounds__(NTH) cast_flat_kernel(const ST* __restrict__ src, DT* __restrict__ dst, int64_t n,
                                                        float scale) {
  const int64_t i = ((int64_t)blockIdx.x * NTH + threadIdx.x) * 4;
  if (i + 3 < n) {
    st4<DT>(dst + i, ld4<ST>(src + i) * scale);
  } else {
    for (int64_t j = i; j < n; ++j) st_from_f<DT>(dst + j, ld_as_f<ST>(src + j) * scale);
  }
}

// torch.optim.AdamW (decoupled weight decay), torch/optim/adamw.py _single_tensor_adamw:
//   p *= 1 - lr*wd ; m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void __launch_bounds__(NTH) adamw_multi_kernel(const maeclip_mt_entry* __restrict__ e, int ne,
                                                          maeclip_adamw_hparams hp) {
  const int k = find_entry(e, ne, blockIdx.x);
  const int64_t base = (blockIdx.x - e[k].chunk_start) * CHUNK;
  float* p = (float*)e[k].p0;
  const float* gr = (const float*)e[k].p1;
  float* m = (float*)e[k].p2;
  float* v = (float*)e[k].p3;
  bf16_t* sh = (bf16_t*)e[k].p4;
  const int64_t n = e[k].n;
  const float decay = 1.f - hp.lr * hp.weight_decay;
  const float b1 = hp.beta1, b2 = hp.beta2;
  float step_size = hp.step_size, bc2_sqrt = hp.bc2_sqrt;
  if (hp.step_ptr) {   // device step count t: bias corrections of torch's _single_tensor_adamw
    const float t = (float)*hp.step_ptr;
    step_size = hp.lr / (1.f - powf(b1, t));
    bc2_sqrt = sqrtf(1.f - powf(b2, t));
  }
  auto upd = [&](float g, float& pi, float& mi, float& vi) {
    g *= hp.grad_scale;
    pi *= decay;
    mi = b1 * mi + (1.f - b1) * g;
    vi = b2 * vi + (1.f - b2) * g * g;
    pi -= step_size * mi / (sqrtf(vi) / bc2_sqrt + hp.eps);
  };
  // 16-B vectors when the entry allows (every tensor of the path does); the
  // fp32 streams are non-temporal -- read and written once per step, they would
  // otherwise evict the next forward's operands -- the bf16 shadow is not
  const bool vec = (n & 3) == 0 && ((((uintptr_t)p) | ((uintptr_t)gr) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (!sh || (((uintptr_t)sh) & 7) == 0);
  if (vec) {
    for (int64_t i = base + 4 * threadIdx.x; i < base + CHUNK && i < n; i += 4 * NTH) {
      const v4f g = __builtin_nontemporal_load((const v4f*)(gr + i));
      v4f pv = __builtin_nontemporal_load((const v4f*)(p + i));
      v4f mv = __builtin_nontemporal_load((const v4f*)(m + i));
      v4f vv = __builtin_nontemporal_load((const v4f*)(v + i));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = pv[j], mj = mv[j], vj = vv[j];
        upd(g[j], pj, mj, vj);
        pv[j] = pj;
        mv[j] = mj;
        vv[j] = vj;
      }
      __builtin_nontemporal_store(pv, (v4f*)(p + i));
      __builtin_nontemporal_store(mv, (v4f*)(m + i));
      __builtin_nontemporal_store(vv, (v4f*)(v + i));
      if (sh) *(v2u*)(sh + i) = v2u{pack2bf(pv[0], pv[1]), pack2bf(pv[2], pv[3])};
    }
    return;
  }
  for (int64_t i = base + threadIdx.x; i < base + CHUNK && i < n; i += NTH) {
    float pi = p[i], mi = m[i], vi = v[i];
    upd(gr[i], pi, mi, vi);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (sh) sh[i] = f2bf(pi);
  }
}

int64_t mt_blocks(const maeclip_mt_entry* host_entries, int ne) {
  if (ne <= 0) return 0;
  return host_entries[ne - 1].chunk_start + (host_entries[ne - 1].n + CHUNK - 1) / CHUNK;
}

}  // namespace

extern "C" int64_t maeclip_mt_chunk(void) { return CHUNK; }

extern "C" int32_t maeclip_colsum_multi(const maeclip_colsum_entry* dev_entries, const maeclip_colsum_entry* host_entries,
                                        int32_t ne, void* stream) {
  MC_CHECK_ARG(dev_entries && host_entries && ne > 0, "maeclip_colsum_multi: bad args");
  const int64_t nb = host_entries[ne - 1].block_start + (host_entries[ne - 1].N + 63) / 64;
  hipLaunchKernelGGL(colsum_multi_kernel, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, dev_entries, ne);
  MC_CHECK_LAUNCH("maeclip_colsum_multi");
  return 0;
}

extern "C" int32_t maeclip_colsum_reduce(const float* partial, int64_t P, int64_t N, float* out, int32_t accumulate,
                                         float scale, float* scratch, void* stream) {
  MC_CHECK_ARG(partial && out && P >= 1 && N >= 1, "maeclip_colsum_reduce: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (N > 1 && P > 64) {
    MC_CHECK_ARG(scratch != nullptr, "maeclip_colsum_reduce: P > 64 needs scratch [ceil(P/64)][N]");
    dim3 g1((unsigned)((N + 63) / 64), (unsigned)((P + 63) / 64));
    hipLaunchKernelGGL(colsum_pass1_kernel, g1, dim3(NTH), 0, s, partial, P, N, scratch);
    MC_CHECK_LAUNCH("maeclip_colsum_reduce(pass1)");
    partial = scratch;
    P = (P + 63) / 64;
  }
  if (N == 1) {
    if (P > VS_CHUNK) {
      MC_CHECK_ARG(scratch != nullptr, "maeclip_colsum_reduce: N == 1, P > %d needs scratch [ceil(P/%d)]", VS_CHUNK,
                   VS_CHUNK);
      const int64_t G = (P + VS_CHUNK - 1) / VS_CHUNK;
      hipLaunchKernelGGL(vec_sum_pass1_kernel, dim3((unsigned)G), dim3(NTH), 0, s, partial, P, scratch);
      MC_CHECK_LAUNCH("maeclip_colsum_reduce(vec pass1)");
      partial = scratch;
      P = G;
    }
    hipLaunchKernelGGL(vec_sum_kernel, dim3(1), dim3(NTH), 0, s, partial, P, out, accumulate, scale);
  } else {
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((unsigned)((N + NTH - 1) / NTH)), dim3(NTH), 0, s, partial, P, N, out,
                       accumulate, scale);
  }
  MC_CHECK_LAUNCH("maeclip_colsum_reduce");
  return 0;
}


extern "C" int32_t maeclip_rows_colsum_partial_rows(int64_t M) { return rows_colsum_grid(M); }

extern "C" int32_t maeclip_rows_colsum_q8(const void* x, int32_t dtype, int64_t M, int64_t D, int64_t ld,
                                          void* out_bf16, float* partial, void* q8, int64_t ldq8, float* q8_scale,
                                          int32_t q8_fmt, void* stream) {
  MC_CHECK_ARG(x && partial && out_bf16 && q8 && q8_scale && M >= 0 && D > 0 && D <= RC_MAXC * 256 && D % 4 == 0 &&
                   ld >= D && ldq8 >= D && ldq8 % 4 == 0 && ((uintptr_t)q8 & 3) == 0 &&
                   (dtype == MAECLIP_F32 || dtype == MAECLIP_BF16) &&
                   (q8_fmt == MAECLIP_FP8_E4M3 || q8_fmt == MAECLIP_FP8_E5M2),
               "maeclip_rows_colsum_q8: bad args");
  if (M == 0) return 0;
  dim3 grid((unsigned)rows_colsum_grid(M));
  const bool e5 = q8_fmt == MAECLIP_FP8_E5M2;
  if (dtype == MAECLIP_BF16)
    hipLaunchKernelGGL((rows_colsum_kernel<bf16_t, true>), grid, dim3(NTH), 0, (hipStream_t)stream, (const bf16_t*)x, M,
                       (int)D, ld, (bf16_t*)out_bf16, partial, (uint8_t*)q8, ldq8, q8_scale, e5);
  else
    hipLaunchKernelGGL((rows_colsum_kernel<float, true>), grid, dim3(NTH), 0, (hipStream_t)stream, (const float*)x, M,
                       (int)D, ld, (bf16_t*)out_bf16, partial, (uint8_t*)q8, ldq8, q8_scale, e5);
  MC_CHECK_LAUNCH("maeclip_rows_colsum_q8");
  return 0;
}

// scratch floats maeclip_colsum_reduce needs for a [P, N] partial matrix
extern "C" int64_t maeclip_colsum_scratch(int64_t P, int64_t N) {
  if (N == 1) return P > VS_CHUNK ? (P + VS_CHUNK - 1) / VS_CHUNK : 0;
  return P > 64 ? (P + 63) / 64 * N : 0;
}

extern "C" int32_t maeclip_rows_colsum(const void* x, int32_t dtype, int64_t M, int64_t D, int64_t ld, void* out_bf16,
                                       float* partial, void* stream) {
  MC_CHECK_ARG(x && partial && M >= 1 && D > 0 && D <= RC_MAXC * 256 && D % 4 == 0 && ld % 4 == 0,
               "maeclip_rows_colsum: bad args");
  dim3 grid((unsigned)rows_colsum_grid(M));
  if (dtype == MAECLIP_BF16)
    hipLaunchKernelGGL((rows_colsum_kernel<bf16_t>), grid, dim3(NTH), 0, (hipStream_t)stream, (const bf16_t*)x, M, (int)D,
                       ld, (bf16_t*)out_bf16, partial);
  else
    hipLaunchKernelGGL((rows_colsum_kernel<float>), grid, dim3(NTH), 0, (hipStream_t)stream, (const float*)x, M, (int)D, ld,
                       (bf16_t*)out_bf16, partial);
  MC_CHECK_LAUNCH("maeclip_rows_colsum");
  return 0;
}

extern "C" int32_t maeclip_pool_fwd(const float* x, int32_t B, int32_t n, int32_t D, float* out, void* stream) {
  MC_CHECK_ARG(x && out && B > 0 && n > 1 && D > 0, "maeclip_pool_fwd: bad args");
  hipLaunchKernelGGL(pool_fwd_kernel, dim3((D + NTH - 1) / NTH, B), dim3(NTH), 0, (hipStream_t)stream, x, n, D, out);
  MC_CHECK_LAUNCH("maeclip_pool_fwd");
  return 0;
}

extern "C" int32_t maeclip_pool_bwd(const float* dout, int32_t B, int32_t n, int32_t D, float* dx, int32_t accumulate,
                                    void* stream) {
  MC_CHECK_ARG(dout && dx && B > 0 && n > 1 && D > 0, "maeclip_pool_bwd: bad args");
  const int64_t per = (int64_t)n * D;
  hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)((per + NTH - 1) / NTH), B), dim3(NTH), 0, (hipStream_t)stream, dout,
                     n, D, dx, accumulate);
  MC_CHECK_LAUNCH("maeclip_pool_bwd");
  return 0;
}

extern "C" int32_t maeclip_dropout(const float* x, float* y, int64_t M, int32_t D, int64_t ld, float p, uint64_t seed,
                                   const int64_t* step_ptr, void* stream) {
  MC_CHECK_ARG(x && y && M >= 0 && D > 0 && p >= 0.f && p < 1.f, "maeclip_dropout: bad args");
  if (M == 0) return 0;
  const int64_t total = M * D;
  hipLaunchKernelGGL(dropout_kernel, dim3((unsigned)((total + NTH - 1) / NTH)), dim3(NTH), 0, (hipStream_t)stream, x, y, M,
                     D, ld, p, seed, step_ptr);
  MC_CHECK_LAUNCH("maeclip_dropout");
  return 0;
}

extern "C" int32_t maeclip_embed_fwd(const int64_t* ids, const float* word, const float* pos, int32_t B, int32_t T,
                                     int32_t D, int64_t V, float* out, const int64_t* mask_in, float* mask_out,
                                     void* stream) {
  MC_CHECK_ARG(ids && word && pos && out && D % 4 == 0, "maeclip_embed_fwd: bad args");
  MC_CHECK_ARG((mask_in == nullptr) == (mask_out == nullptr), "maeclip_embed_fwd: mask_in and mask_out go together");
  hipLaunchKernelGGL(embed_kernel, dim3((D / 4 + NTH - 1) / NTH, (unsigned)(B * T)), dim3(NTH), 0, (hipStream_t)stream, ids,
                     word, pos, T, D, V, out, mask_in, mask_out);
  MC_CHECK_LAUNCH("maeclip_embed_fwd");
  return 0;
}

extern "C" int32_t maeclip_cast_multi(const maeclip_mt_entry* dev_entries, const maeclip_mt_entry* host_entries, int32_t ne,
                                      void* stream) {
  MC_CHECK_ARG(dev_entries && host_entries && ne > 0, "maeclip_cast_multi: bad args");
  const int64_t nb = mt_blocks(host_entries, ne);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(cast_multi_kernel, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, dev_entries, ne);
  MC_CHECK_LAUNCH("maeclip_cast_multi");
  return 0;
}

extern "C" int32_t maeclip_adamw_multi(const maeclip_mt_entry* dev_entries, const maeclip_mt_entry* host_entries,
                                       int32_t ne, const maeclip_adamw_hparams* hp, void* stream) {
  MC_CHECK_ARG(dev_entries && host_entries && hp && ne > 0, "maeclip_adamw_multi: bad args");
  const int64_t nb = mt_blocks(host_entries, ne);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(adamw_multi_kernel, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, dev_entries, ne, *hp);
  MC_CHECK_LAUNCH("maeclip_adamw_multi");
  return 0;
}

namespace {
__global__ void counter_add_kernel(int64_t* c, int64_t delta, int64_t* snap) {
  if (threadIdx.x == 0) {
    const int64_t v = *c;
    if (snap) *snap = v;
    *c = v + delta;
  }
}
__global__ void scalar_axpy_kernel(const float* a, const float* b, float w, float* out) {
  if (threadIdx.x == 0) out[0] = fmaf(w, b[0], a[0]);
}
// src_i == dst_i (in place) is allowed, so the src / dst pairs are not __restrict__
__global__ void __launch_bounds__(NTH) scale2_kernel(const float* s0, float* d0, int64_t n0,
                                                     const float* s1, float* d1, int64_t n1,
                                                     const float* __restrict__ sc, float w, int64_t nb0) {
  const float f = w * sc[0];
  const bool second = blockIdx.x >= nb0;
  const float* src = second ? s1 : s0;
  float* dst = second ? d1 : d0;
  const int64_t n = second ? n1 : n0;
  const int64_t i = ((second ? blockIdx.x - nb0 : blockIdx.x) * (int64_t)NTH + threadIdx.x) * 4;
  if (i + 3 < n && ((((uintptr_t)dst) | ((uintptr_t)(src ? src : dst))) & 15) == 0) {
    const v4f v = src ? *(const v4f*)(src + i) : v4f{1.f, 1.f, 1.f, 1.f};
    *(v4f*)(dst + i) = v * f;
  } else {
    for (int64_t j = i; j < n && j < i + 4; ++j) dst[j] = (src ? src[j] : 1.f) * f;
  }
}
}  // namespace

extern "C" int32_t maeclip_counter_add_snap(int64_t* counter, int64_t delta, int64_t* snap, void* stream) {
  MC_CHECK_ARG(counter != nullptr && snap != nullptr, "maeclip_counter_add_snap: null pointer");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, delta, snap);
  MC_CHECK_LAUNCH("maeclip_counter_add_snap");
  return 0;
}

extern "C" int32_t maeclip_scalar_axpy(const float* a, const float* b, float w, float* out, void* stream) {
  MC_CHECK_ARG(a && b && out, "maeclip_scalar_axpy: null pointer");
  hipLaunchKernelGGL(scalar_axpy_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, w, out);
  MC_CHECK_LAUNCH("maeclip_scalar_axpy");
  return 0;
}

__global__ void __launch_bounds__(NTH) copy_f32_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTH) dst[i] = src[i];
}

extern "C" int32_t maeclip_copy_f32(const float* src, float* dst, int64_t n, void* stream) {
  MC_CHECK_ARG(n >= 0 && (n == 0 || (src && dst)), "maeclip_copy_f32: bad args");
  if (n == 0) return 0;
  const int64_t nb = (n + NTH - 1) / NTH;
  hipLaunchKernelGGL(copy_f32_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(NTH), 0, (hipStream_t)stream, src,
                     dst, n);
  MC_CHECK_LAUNCH("maeclip_copy_f32");
  return 0;
}

__global__ void __launch_bounds__(NTH) copy_f32_slot_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                             int64_t n, const int64_t* __restrict__ counter) {
  float* d = dst + (counter[0] & 1) * n;
  for (int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTH) d[i] = src[i];
}

extern "C" int32_t maeclip_copy_f32_slot(const float* src, float* dst, int64_t n, const int64_t* counter, void* stream) {
  MC_CHECK_ARG(n >= 0 && (n == 0 || (src && dst && counter)), "maeclip_copy_f32_slot: bad args");
  if (n == 0) return 0;
  const int64_t nb = (n + NTH - 1) / NTH;
  hipLaunchKernelGGL(copy_f32_slot_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(NTH), 0, (hipStream_t)stream,
                     src, dst, n, counter);
  MC_CHECK_LAUNCH("maeclip_copy_f32_slot");
  return 0;
}

extern "C" int32_t maeclip_host_mapped_alloc(int64_t bytes, void** host_ptr, void** dev_ptr) {
  MC_CHECK_ARG(bytes > 0 && host_ptr && dev_ptr, "maeclip_host_mapped_alloc: bad args");
  void* h = nullptr;
  void* d = nullptr;
  MC_CHECK_ARG(hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped) == hipSuccess && h,
               "maeclip_host_mapped_alloc: hipHostMalloc(%lld) failed", (long long)bytes);
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    MC_CHECK_ARG(false, "maeclip_host_mapped_alloc: no device mapping");
  }
  *host_ptr = h;
  *dev_ptr = d;
  return 0;
}

extern "C" int32_t maeclip_host_mapped_free(void* host_ptr) {
  if (host_ptr) (void)hipHostFree(host_ptr);
  return 0;
}

extern "C" int32_t maeclip_scale_by_scalar2(const float* src0, float* dst0, int64_t n0, const float* src1, float* dst1,
                                            int64_t n1, const float* s, float w, void* stream) {
  MC_CHECK_ARG(s != nullptr && n0 >= 0 && n1 >= 0 && (n0 == 0 || dst0) && (n1 == 0 || dst1),
               "maeclip_scale_by_scalar2: bad args");
  const int64_t nb0 = (n0 + 4 * NTH - 1) / (4 * NTH), nb1 = (n1 + 4 * NTH - 1) / (4 * NTH);
  if (nb0 + nb1 == 0) return 0;
  hipLaunchKernelGGL(scale2_kernel, dim3((unsigned)(nb0 + nb1)), dim3(NTH), 0, (hipStream_t)stream, src0, dst0, n0, src1,
                     dst1, n1, s, w, nb0);
  MC_CHECK_LAUNCH("maeclip_scale_by_scalar2");
  return 0;
}

extern "C" int32_t maeclip_counter_add(int64_t* counter, int64_t delta, void* stream) {
  MC_CHECK_ARG(counter != nullptr, "maeclip_counter_add: null counter");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, delta, (int64_t*)nullptr);
  MC_CHECK_LAUNCH("maeclip_counter_add");
  return 0;
}

extern "C" int32_t maeclip_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  MC_CHECK_ARG(dst && src, "maeclip_memcpy_h2d: null pointer");
  if (bytes == 0) return 0;
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
  if (e != hipSuccess) {
    maeclip::set_error("maeclip_memcpy_h2d: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

extern "C" int32_t maeclip_cast_flat(const void* src, int32_t src_dtype, void* dst, int32_t dst_dtype, int64_t n,
                                     float scale, void* stream) {
  MC_CHECK_ARG(src && dst && n >= 0, "maeclip_cast_flat: bad args");
  MC_CHECK_ARG((src_dtype == MAECLIP_F32 || src_dtype == MAECLIP_BF16) &&
                   (dst_dtype == MAECLIP_F32 || dst_dtype == MAECLIP_BF16),
               "maeclip_cast_flat: dtypes must be f32 / bf16");
  MC_CHECK_ARG(((uintptr_t)src & 7) == 0 && ((uintptr_t)dst & 7) == 0, "maeclip_cast_flat: 8-B aligned buffers");
  if (n == 0) return 0;
  dim3 grid((unsigned)((n + 4 * NTH - 1) / (4 * NTH)));
  hipStream_t s = (hipStream_t)stream;
  if (src_dtype == MAECLIP_F32 && dst_dtype == MAECLIP_BF16)
    hipLaunchKernelGGL((cast_flat_kernel<float, bf16_t>), grid, dim3(NTH), 0, s, (const float*)src, (bf16_t*)dst, n, scale);
  else if (src_dtype == MAECLIP_BF16 && dst_dtype == MAECLIP_F32)
    hipLaunchKernelGGL((cast_flat_kernel<bf16_t, float>), grid, dim3(NTH), 0, s, (const bf16_t*)src, (float*)dst, n, scale);
  else if (src_dtype == MAECLIP_F32)
    hipLaunchKernelGGL((cast_flat_kernel<float, float>), grid, dim3(NTH), 0, s, (const float*)src, (float*)dst, n, scale);
  else
    hipLaunchKernelGGL((cast_flat_kernel<bf16_t, bf16_t>), grid, dim3(NTH), 0, s, (const bf16_t*)src, (bf16_t*)dst, n,
                       scale);
  MC_CHECK_LAUNCH("maeclip_cast_flat");
  return 0;
}
