// Soft-target symmetric CLIP loss, forward + closed-form backward, fp32 always.
//
// Reference: CLIP.py:34-43 and cross_entropy CLIP.py:46-52
//   L = T I^T / tau ; S = (I I^T + T T^T) / 2 * tau ; Y = softmax_row(S)
//   loss = mean_k[(CE_row(L,Y)_k + CE_col(L,Y)_k)/2]   (gradient flows through Y)
// Backward (verified vs autograd to 5.6e-17 in fp64):
//   G  = -(logsm_row(L) + logsm_col(L)) / 2N ;  rl_i = sum_j Y G ; loss = sum_i rl_i
//   dS = Y .* (G - rl) ; Dm = (dS + dS^T) tau/2 ; c_j = sum_i Y_ij
//   dL = (P_r - 2Y + P_c .* c) / 2N
//   dI = Dm I + dL^T T / tau ;  dT = Dm T + dL I / tau
//
// No N x N matrix ever reaches HBM. The all-pairs products are recomputed per
// (16-row i-block, 16-column j-tile) on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32, bitwise an f32 fma chain) in three phases, each a
// launch over (i-block, j-split) workgroups, with fixed-order partials between
// them (deterministic):
//   phase 1: online (max, sumexp) over j of the rows of S, L and L^T
//            (a row of L^T = a column of L)                    -> part1
//   phase 2: lse vectors (combined from part1); c_i = sum_j exp(S_ij - lseS_j)
//            (S symmetric: the column sums of Y), q_i = sum_j Y_ij (2 L_ij - lse_col(L)_j)
//            so that rl_i = -(q_i - lse_row(L)_i) / 2N                 -> part2
//   phase 3: per j-tile Dm, dL, dL^T in registers, then dI^T / dT^T += X_j^T (.)
//            on the same MFMA, only for the gradient rows [grad_row0, +grad_rows)
//            (data parallel: the local slice)                          -> part3
//   reduce : dI, dT = sum over j-splits of part3; loss = sum_i rl_i (one block,
//            fixed order).
// Workgroup = 4 waves; wave w computes one of the four 16x16 dot tiles of a
// j-tile (S1 = I_j.I_i, S2 = T_j.T_i, L = I_j.T_i, L^T = T_j.I_i), tiles are laid
// out transposed (row = j on the accumulator registers, column = i on the
// lane) so that row statistics over j are lane-local and the tiles feed the
// phase-3 contraction over j as MFMA B operands with no data movement.
// MFMA k mapping: in sub-step s of k-group b, hardware k = lane>>4 carries real
// k = 16b + 4(lane>>4) + s, so each lane reads its operands as 16-byte vectors.
#include "common.h"
#include "../../include/maeclip.h"

namespace {
constexpr int NT = 256;
constexpr float NEG = -1.0e30f;

struct ClipK {
  const float* I;
  const float* T;
  int64_t ldI, ldT;
  int N, P, nrep, Js;  // this phase: j-tiles per workgroup, number of j-splits
  int Js1, Js2;        // j-splits of phases 1 and 2 (partials read by 2, 3 and the reduce)
  float tau;
  float* part1;        // [Js1][3][N] (max, sumexp)
  float* part2;        // [Js2][2][N] (c, q)
  float* lse;          // [3][N]  lse of rows of S, rows of L, columns of L (phase 2, js == 0)
  float* part3;        // [Js][2][Ng][P]
  int g0, Ng;          // gradient rows
};

__device__ __forceinline__ v4f mma4(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ void merge_ms(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

// lse from partials [js * stride + idx] (max, sumexp pairs), js < n
__device__ __forceinline__ float lse_of(const float* part, int64_t stride, int64_t idx, int n) {
  float M = NEG;
  for (int s = 0; s < n; ++s) M = fmaxf(M, part[(s * stride + idx) * 2]);
  float z = 0.f;
  for (int s = 0; s < n; ++s) z += part[(s * stride + idx) * 2 + 1] * expf(part[(s * stride + idx) * 2] - M);
  return M + logf(z);
}

// i-side B operand of wave role ty: rows i0 + (lane&15), 16-B vector b at k = 16b + 4(lane>>4)
template <int NB>
__device__ __forceinline__ void load_iside(const ClipK& a, int ty, int i0, int lane, v4f (&r)[4 * NB]) {
  const bool useT = ty == 1 || ty == 2;
  const float* X = useT ? a.T : a.I;
  const int64_t ld = useT ? a.ldT : a.ldI;
  const int i = i0 + (lane & 15);
  const bool ok = i < a.N;
  const float* row = X + (int64_t)(ok ? i : 0) * ld + 4 * (lane >> 4);
#pragma unroll
  for (int b = 0; b < 4 * NB; ++b) r[b] = ok ? *(const v4f*)(row + 16 * b) : v4f{0.f, 0.f, 0.f, 0.f};
}

// I_j, T_j rows of j-tile jb -> LDS [2][16][P+4] (zero rows past N)
template <int NB>
__device__ __forceinline__ void stage_j(const ClipK& a, int jb, float* Xj) {
  constexpr int P = 64 * NB, RS = P + 4, V = 2 * 16 * P / 4;  // 16-B vectors
#pragma unroll
  for (int u = 0; u < (V + NT - 1) / NT; ++u) {
    const int v = threadIdx.x + u * NT;
    if (v < V) {
      const int m = v / (16 * P / 4), rem = v % (16 * P / 4), r = rem / (P / 4), c = (rem % (P / 4)) * 4;
      const int j = jb + r;
      const float* X = m ? a.T : a.I;
      const int64_t ld = m ? a.ldT : a.ldI;
      const v4f val = j < a.N ? *(const v4f*)(X + (int64_t)j * ld + c) : v4f{0.f, 0.f, 0.f, 0.f};
      *(v4f*)(Xj + (m * 16 + r) * RS + c) = val;
    }
  }
}

// 16x16 dot tile of role ty: D[j = 4(lane>>4) + reg][i = lane&15]
template <int NB>
__device__ __forceinline__ v4f score_tile(const float* Xj, int ty, const v4f (&ir)[4 * NB], int lane) {
  constexpr int RS = 64 * NB + 4;
  const float* rowp = Xj + ((ty & 1) * 16 + (lane & 15)) * RS + 4 * (lane >> 4);
  v4f c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 4 * NB; ++b) {
    const v4f x = *(const v4f*)(rowp + 16 * b);
    c0 = mma4(x[0], ir[b][0], c0);
    c1 = mma4(x[1], ir[b][1], c1);
    c0 = mma4(x[2], ir[b][2], c0);
    c1 = mma4(x[3], ir[b][3], c1);
  }
  return c0 + c1;
}

// ------------------------------------------------------------------ phases
template <int PH, int NB>
__global__ void __launch_bounds__(NT) clip_phase_kernel(const ClipK a) {
  constexpr int P = 64 * NB, RS = P + 4;
  __shared__ __attribute__((aligned(16))) float Xj[2 * 16 * RS];
  __shared__ __attribute__((aligned(16))) float sc[4][16][16];   // [role][j][i]
  __shared__ float ist[5][16];                                   // i rows: lseS, lseLr, lseLc, c, rl
  __shared__ float jst[5][16];                                   // j tile: lseS, lseLr, lseLc, c, rl
  const int lane = threadIdx.x & 63, g = lane >> 4, il = lane & 15;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i0 = PH == 3 ? a.g0 + 16 * (int)blockIdx.x : 16 * (int)blockIdx.x;
  const int js = blockIdx.y;
  const int jt0 = js * a.nrep, njt = (a.N + 15) / 16;
  const int jt1 = min(jt0 + a.nrep, njt);
  const float tau = a.tau, itau = 1.f / tau, inv2n = 0.5f / (float)a.N;
  const int N = a.N;

  v4f ir[4 * NB];
  load_iside<NB>(a, ty, i0, lane, ir);

  if (PH >= 2 && threadIdx.x < 16) {
    const int i = min(i0 + (int)threadIdx.x, N - 1);
    if (PH == 2) {
      ist[0][threadIdx.x] = lse_of(a.part1, 3LL * N, i, a.Js1);
      ist[1][threadIdx.x] = lse_of(a.part1, 3LL * N, N + i, a.Js1);
      ist[2][threadIdx.x] = lse_of(a.part1, 3LL * N, 2LL * N + i, a.Js1);
      if (js == 0 && i0 + (int)threadIdx.x < N)
        for (int t = 0; t < 3; ++t) a.lse[(int64_t)t * N + i] = ist[t][threadIdx.x];
    } else {
      float c = 0.f, q = 0.f;
      for (int s = 0; s < a.Js2; ++s) {
        c += a.part2[((int64_t)s * 2) * N + i];
        q += a.part2[((int64_t)s * 2 + 1) * N + i];
      }
      const float lr = a.lse[(int64_t)N + i];
      ist[0][threadIdx.x] = a.lse[i];
      ist[1][threadIdx.x] = lr;
      ist[2][threadIdx.x] = a.lse[2LL * N + i];
      ist[3][threadIdx.x] = c;
      ist[4][threadIdx.x] = -(q - lr) * inv2n;
    }
  }

  // phase 1 / 2 lane-local accumulators (row i = lane&15 over this lane's j)
  float m0 = NEG, s0 = 0.f;   // ph1: S rows (wave 0), L rows (wave 2), L^T rows (wave 3)
  float cacc = 0.f, qacc = 0.f;
  // phase 3 accumulators: wave ty owns p-tiles pq = ty + 4u
  v4f accI[NB], accT[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    accI[u] = v4f{0.f, 0.f, 0.f, 0.f};
    accT[u] = v4f{0.f, 0.f, 0.f, 0.f};
  }

  for (int jt = jt0; jt < jt1; ++jt) {
    const int jb = 16 * jt;
    __syncthreads();   // previous tile's LDS reads are done
    stage_j<NB>(a, jb, Xj);
    if (PH == 2 && threadIdx.x < 32) {
      const int t = threadIdx.x >> 4, j = min(jb + (int)(threadIdx.x & 15), N - 1);
      jst[t == 0 ? 0 : 2][threadIdx.x & 15] = lse_of(a.part1, 3LL * N, (t == 0 ? 0LL : 2LL * N) + j, a.Js1);
    }
    if (PH == 3 && threadIdx.x < 16) {
      const int j = min(jb + (int)threadIdx.x, N - 1);
      float c = 0.f, q = 0.f;
      for (int s = 0; s < a.Js2; ++s) {
        c += a.part2[((int64_t)s * 2) * N + j];
        q += a.part2[((int64_t)s * 2 + 1) * N + j];
      }
      const float lr = a.lse[(int64_t)N + j];
      jst[0][threadIdx.x] = a.lse[j];
      jst[1][threadIdx.x] = lr;
      jst[2][threadIdx.x] = a.lse[2LL * N + j];
      jst[3][threadIdx.x] = c;
      jst[4][threadIdx.x] = -(q - lr) * inv2n;
    }
    __syncthreads();
    // every role publishes its tile sc[ty][j][i] (phase 2 needs S1, S2, L only)
    const bool active = !(PH == 2 && ty == 3);
    v4f d = {0.f, 0.f, 0.f, 0.f};
    if (active) {
      d = score_tile<NB>(Xj, ty, ir, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[ty][4 * g + r][il] = d[r];
    }
    __syncthreads();

    if (PH == 1) {
      // wave 0: rows of S; wave 2: rows of L; wave 3: rows of L^T (columns of L)
      if (ty != 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = jb + 4 * g + r;
          const float x = ty == 0 ? (d[r] + sc[1][4 * g + r][il]) * (0.5f * tau) : d[r] * itau;
          if (j < N) merge_ms(m0, s0, x, 1.f);
        }
      }
    } else if (PH == 2) {
      if (ty == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int jl = 4 * g + r;
          if (jb + jl < N) {
            const float S = (d[r] + sc[1][jl][il]) * (0.5f * tau);
            const float Lij = sc[2][jl][il] * itau;
            cacc += __expf(S - jst[0][jl]);
            const float Y = __expf(S - ist[0][il]);
            qacc = fmaf(Y, 2.f * Lij - jst[2][jl], qacc);
          }
        }
      }
    } else {
      // phase 3: B operands of the contraction over j (k = j = 4g + r)
      float bD[4], bLt[4], bL[4];
      const float lsi = ist[0][il], lri = ist[1][il], lci = ist[2][il], ci = ist[3][il], rli = ist[4][il];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jl = 4 * g + r;
        const float S = (sc[0][jl][il] + sc[1][jl][il]) * (0.5f * tau);
        const float Lij = sc[2][jl][il] * itau, Lji = sc[3][jl][il] * itau;
        const float lsj = jst[0][jl], lrj = jst[1][jl], lcj = jst[2][jl], cj = jst[3][jl], rlj = jst[4][jl];
        const float Yij = __expf(S - lsi), Yji = __expf(S - lsj);
        const float Gij = -(2.f * Lij - lri - lcj) * inv2n, Gji = -(2.f * Lji - lrj - lci) * inv2n;
        const float Dm = (Yij * (Gij - rli) + Yji * (Gji - rlj)) * (0.5f * tau);
        const float dLij = (__expf(Lij - lri) - 2.f * Yij + __expf(Lij - lcj) * cj) * inv2n;
        const float dLji = (__expf(Lji - lrj) - 2.f * Yji + __expf(Lji - lci) * ci) * inv2n;
        const bool ok = jb + jl < N;
        bD[r] = ok ? Dm : 0.f;
        bLt[r] = ok ? dLji * itau : 0.f;
        bL[r] = ok ? dLij * itau : 0.f;
      }
      // dI^T[p][i] += sum_j I_j[j][p] Dm[i][j] + T_j[j][p] dL[j][i]/tau ; dT^T likewise
      const float* Ij = Xj + (4 * g) * RS + il;
      const float* Tj = Xj + (16 + 4 * g) * RS + il;
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int pc = 16 * (ty + 4 * u);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xi = Ij[r * RS + pc], xt = Tj[r * RS + pc];
          accI[u] = mma4(xi, bD[r], accI[u]);
          accI[u] = mma4(xt, bLt[r], accI[u]);
          accT[u] = mma4(xt, bD[r], accT[u]);
          accT[u] = mma4(xi, bL[r], accT[u]);
        }
      }
    }
  }

  if (PH == 1) {
    if (ty != 1) {
      float m2 = __shfl_xor(m0, 16, 64), s2 = __shfl_xor(s0, 16, 64);
      merge_ms(m0, s0, m2, s2);
      m2 = __shfl_xor(m0, 32, 64);
      s2 = __shfl_xor(s0, 32, 64);
      merge_ms(m0, s0, m2, s2);
      const int t = ty == 0 ? 0 : ty - 1;   // 0: S rows, 1: L rows, 2: L^T rows
      const int i = i0 + il;
      if (g == 0 && i < N) {
        float* dst = a.part1 + (((int64_t)js * 3 + t) * N + i) * 2;
        dst[0] = m0;
        dst[1] = s0;
      }
    }
  } else if (PH == 2) {
    if (ty == 0) {
      cacc += __shfl_xor(cacc, 16, 64);
      cacc += __shfl_xor(cacc, 32, 64);
      qacc += __shfl_xor(qacc, 16, 64);
      qacc += __shfl_xor(qacc, 32, 64);
      const int i = i0 + il;
      if (g == 0 && i < N) {
        a.part2[((int64_t)js * 2) * N + i] = cacc;
        a.part2[((int64_t)js * 2 + 1) * N + i] = qacc;
      }
    }
  } else {
    // accI[u]: lane holds dI^T[p = pc + 4g + r][i = il] -> row i, 4 consecutive p
    const int i = i0 + il;
    if (i < N && i < a.g0 + a.Ng) {
      const int64_t row = i - a.g0;
      float* dI = a.part3 + (((int64_t)js * 2) * a.Ng + row) * P;
      float* dT = a.part3 + (((int64_t)js * 2 + 1) * a.Ng + row) * P;
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int p = 16 * (ty + 4 * u) + 4 * g;
        *(v4f*)(dI + p) = accI[u];
        *(v4f*)(dT + p) = accT[u];
      }
    }
  }
}

// dI / dT rows = fixed-order sums of the phase-3 slabs; block 0 also writes
// loss = sum_i rl_i and the optional per-row rl.
__global__ void __launch_bounds__(NT) clip_reduce_kernel(const ClipK a, int Js3, float* loss, float* row_loss,
                                                         float* dI, int64_t lddI, float* dT, int64_t lddT) {
  const int N = a.N, P = a.P;
  if (blockIdx.x == 0) {
    __shared__ float red[NT / 64];
    const float inv2n = 0.5f / (float)N;
    float acc = 0.f;
    for (int i = threadIdx.x; i < N; i += NT) {
      float q = 0.f;
      for (int s = 0; s < a.Js2; ++s) q += a.part2[((int64_t)s * 2 + 1) * N + i];
      const float rl = -(q - a.lse[(int64_t)N + i]) * inv2n;
      if (row_loss) row_loss[i] = rl;
      acc += rl;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < NT / 64; ++w) t += red[w];
      *loss = t;
    }
  }
  if (!dI) return;
  const int64_t nv = (int64_t)a.Ng * P / 4;
  for (int64_t v = (int64_t)blockIdx.x * NT + threadIdx.x; v < nv; v += (int64_t)gridDim.x * NT) {
    const int64_t row = v / (P / 4), c = (v % (P / 4)) * 4;
    v4f si = {0.f, 0.f, 0.f, 0.f}, st = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < Js3; ++s) {
      si += *(const v4f*)(a.part3 + (((int64_t)s * 2) * a.Ng + row) * P + c);
      st += *(const v4f*)(a.part3 + (((int64_t)s * 2 + 1) * a.Ng + row) * P + c);
    }
    *(v4f*)(dI + row * lddI + c) = si;
    *(v4f*)(dT + row * lddT + c) = st;
  }
}

// ------------------------------------------------------------ geometry
struct Geo {
  int nrep1, Js1, nrep3, Js3, Ng;
};

Geo geometry(int64_t N, int64_t grad_rows) {
  Geo g;
  const int64_t nb = (N + 15) / 16;
  // phases 1/2: ~1024 workgroups over nb i-blocks x nb j-tiles
  int64_t r = (nb * nb + 1023) / 1024;
  if (r < 1) r = 1;
  if (r > nb) r = nb;
  g.nrep1 = (int)r;
  g.Js1 = (int)((nb + r - 1) / r);
  // phase 3: ~512 workgroups over the gradient rows' i-blocks
  g.Ng = (int)grad_rows;
  const int64_t ngb = (grad_rows + 15) / 16;
  int64_t js = ngb > 0 ? 512 / ngb : 1;
  if (js < 1) js = 1;
  if (js > nb) js = nb;
  g.nrep3 = (int)((nb + js - 1) / js);
  g.Js3 = (int)((nb + g.nrep3 - 1) / g.nrep3);
  return g;
}

size_t ws_floats(int64_t N, int64_t P, int64_t grad_rows) {
  const Geo g = geometry(N, grad_rows);
  return (size_t)g.Js1 * 3 * N * 2 + (size_t)g.Js1 * 2 * N + 3 * (size_t)N + (size_t)g.Js3 * 2 * grad_rows * P + 64;
}

template <int NB>
int run(const maeclip_clip_args& a, hipStream_t s) {
  const int64_t N = a.N;
  const bool grad = a.dI && a.dT;
  const int64_t Ng = grad ? (a.grad_rows > 0 ? a.grad_rows : N - a.grad_row0) : 0;
  const Geo geo = geometry(N, Ng);
  float* ws = (float*)a.workspace;
  ClipK k = {};
  k.I = a.I;
  k.T = a.T;
  k.ldI = a.ld_I ? a.ld_I : a.P;
  k.ldT = a.ld_T ? a.ld_T : a.P;
  k.N = (int)N;
  k.P = (int)a.P;
  k.tau = a.temperature;
  k.Js1 = geo.Js1;
  k.Js2 = geo.Js1;
  k.part1 = ws;
  k.part2 = k.part1 + (size_t)geo.Js1 * 3 * N * 2;
  k.lse = k.part2 + (size_t)geo.Js1 * 2 * N;
  k.part3 = k.lse + 3 * N;
  k.g0 = grad ? (int)a.grad_row0 : 0;
  k.Ng = (int)Ng;
  const unsigned nb = (unsigned)((N + 15) / 16);
  k.nrep = geo.nrep1;
  k.Js = geo.Js1;
  hipLaunchKernelGGL((clip_phase_kernel<1, NB>), dim3(nb, geo.Js1), dim3(NT), 0, s, k);
  hipLaunchKernelGGL((clip_phase_kernel<2, NB>), dim3(nb, geo.Js1), dim3(NT), 0, s, k);
  MC_CHECK_LAUNCH("maeclip_clip_loss(stats)");
  int red_grid = 1;
  if (grad && Ng > 0) {
    k.nrep = geo.nrep3;
    k.Js = geo.Js3;
    hipLaunchKernelGGL((clip_phase_kernel<3, NB>), dim3((unsigned)((Ng + 15) / 16), geo.Js3), dim3(NT), 0, s, k);
    MC_CHECK_LAUNCH("maeclip_clip_loss(grad)");
    const int64_t nv = Ng * a.P / 4;
    red_grid = (int)std::min<int64_t>((nv + NT - 1) / NT, 1024);
    if (red_grid < 1) red_grid = 1;
  }
  hipLaunchKernelGGL(clip_reduce_kernel, dim3(red_grid), dim3(NT), 0, s, k, geo.Js3, a.loss, a.row_loss_out,
                     grad && Ng > 0 ? a.dI : nullptr, a.ld_dI ? a.ld_dI : a.P, a.dT, a.ld_dT ? a.ld_dT : a.P);
  MC_CHECK_LAUNCH("maeclip_clip_loss(reduce)");
  return 0;
}

}  // namespace

extern "C" size_t maeclip_clip_loss_workspace(int64_t N, int64_t P, int64_t grad_rows) {
  if (N <= 0 || P <= 0) return 64 * sizeof(float);
  if (grad_rows < 0 || grad_rows > N) grad_rows = N;
  return ws_floats(N, P, grad_rows) * sizeof(float);
}

extern "C" int32_t maeclip_clip_loss(const maeclip_clip_args* a, void* stream) {
  MC_CHECK_ARG(a && a->I && a->T && a->loss && a->workspace, "maeclip_clip_loss: null pointer");
  MC_CHECK_ARG(a->N > 0 && a->N < (1LL << 30), "maeclip_clip_loss: bad N %lld", (long long)a->N);
  MC_CHECK_ARG(a->P == 64 || a->P == 128 || a->P == 256 || a->P == 512,
               "maeclip_clip_loss: P must be 64, 128, 256 or 512 (got %lld)", (long long)a->P);
  MC_CHECK_ARG(a->temperature > 0.f, "maeclip_clip_loss: temperature must be > 0");
  const int64_t ldi = a->ld_I ? a->ld_I : a->P, ldt = a->ld_T ? a->ld_T : a->P;
  MC_CHECK_ARG(ldi >= a->P && ldt >= a->P && ldi % 4 == 0 && ldt % 4 == 0 && ((uintptr_t)a->I & 15) == 0 &&
                   ((uintptr_t)a->T & 15) == 0,
               "maeclip_clip_loss: I/T rows must be 16-byte aligned");
  const bool grad = a->dI && a->dT;
  int64_t gr = 0;
  if (grad) {
    MC_CHECK_ARG(a->grad_row0 >= 0 && a->grad_row0 < a->N && a->grad_rows >= 0 && a->grad_row0 + a->grad_rows <= a->N,
                 "maeclip_clip_loss: gradient rows out of range");
    gr = a->grad_rows > 0 ? a->grad_rows : a->N - a->grad_row0;
    const int64_t lddi = a->ld_dI ? a->ld_dI : a->P, lddt = a->ld_dT ? a->ld_dT : a->P;
    MC_CHECK_ARG(lddi % 4 == 0 && lddt % 4 == 0 && ((uintptr_t)a->dI & 15) == 0 && ((uintptr_t)a->dT & 15) == 0,
                 "maeclip_clip_loss: dI/dT rows must be 16-byte aligned");
  }
  MC_CHECK_ARG(a->ws_bytes >= maeclip_clip_loss_workspace(a->N, a->P, gr) && ((uintptr_t)a->workspace & 15) == 0,
               "maeclip_clip_loss: workspace too small or misaligned");
  hipStream_t s = (hipStream_t)stream;
  switch (a->P) {
    case 64: return run<1>(*a, s);
    case 128: return run<2>(*a, s);
    case 256: return run<4>(*a, s);
    default: return run<8>(*a, s);
  }
}
