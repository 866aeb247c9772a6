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
// Three launches, deterministic (fixed-order sums everywhere, no atomics):
//   products: the all-pairs products ONCE per (16-row i-block, 16-column
//             j-tile) on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32, bitwise an
//             f32 fma chain); the scaled N x N matrices S, L and L^T go to the
//             workspace (3 N^2 f32: 0.8 MB at N = 256, 48 MB at N = 2048), and
//             the online (max, sumexp) over the workgroup's j range of the rows
//             of S, L and L^T (a row of L^T = a column of L) -> part1.
//   stats:    per row i: (max M, log sumexp z) of S / L / L^T rows (part1
//             combined; kept apart, x - lse is taken as (x - M) - z), c_i =
//             sum_j exp(S_ij - lseS_j) (S symmetric: the column sums of Y) and
//             rl_i = -sum_j Y_ij ((L_ij - lse_row(L)_i) + (L_ij - lse_col(L)_j)) / 2N
//             (log-probabilities as differences: 2 L - lse - lse, or an lse
//             rounded to f32, loses ~1e-6 absolute at |L| ~ 30, which the nearly
//             cancelling G - rl and P_r - 2Y + P_c c then amplify: a 16x larger
//             error than torch's f32 autograd at ViT-L C4 shapes, B = 2),
//             one pass over the stored S / L rows -> stat[8][N].
//   grad:     workgroup (16 gradient rows, 16 columns of P): wave w takes the
//             j-tiles w, w + 4, ...; per tile Dm, dL, dL^T from the stored
//             tiles and stat, then dI^T / dT^T += X_j^T (.) on the MFMA; the
//             four waves' sums are added in wave order and written (only the
//             rows [grad_row0, +grad_rows): data parallel, the local slice).
//             Workgroup (0, 0) writes loss = sum_i rl_i (and the per-row rl).
// No partial-gradient slabs and no reduction launch.
// Products workgroup = 4 waves; wave w computes one of the four 16x16 dot tiles
// of a j-tile (S1 = I_j.I_i, S2 = T_j.T_i, L = I_j.T_i, L^T = T_j.I_i), laid
// out transposed (row = j on the accumulator registers, column = i on the lane)
// so that row statistics over j are lane-local. In the later passes lane
// (i = lane & 15, j = 4 (lane >> 4) + r) reads its four consecutive j of row i
// of a stored matrix as one 16-B load: the B-operand layout of the contraction.
// MFMA k mapping: in sub-step s of k-group b, hardware k = lane>>4 carries real
// k = 16b + 4(lane>>4) + s, so each lane reads its operands as 16-byte vectors.
#include "common.h"
#include "../../include/maeclip.h"

namespace {
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int NT = 256;
constexpr float NEG = -1.0e30f;

struct ClipK {
  const float* I;
  const float* T;
  int64_t ldI, ldT;
  int N, P, NP;        // NP: row stride of the stored matrices (N rounded up to 16)
  int nrep, Js;        // products: j-tiles per workgroup, number of j-splits
  float tau;
  float* part1;        // [Js][3][N] (max, sumexp)
  float* stat;         // [8][N]: (max, log sumexp) of S rows, L rows, L^T rows; c; rl
  float* Sm;           // [N][NP] S = (I I^T + T T^T) tau / 2
  float* Lm;           // [N][NP] L = T I^T / tau
  float* Ltm;          // [N][NP] L^T
  int g0, Ng;          // gradient rows
};

__device__ __forceinline__ v4f mma4(float a, float b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ void merge_ms(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

// (max, log sumexp) from partials [js * stride + idx] (max, sumexp pairs), js <
// n, read 16 at a time with every load in flight. The two parts stay separate:
// lse = M + log z rounded to f32 is off by up to ulp(|M|) / 2 (1e-6 at |x| ~ 30),
// which the nearly cancelling gradient terms then amplify; x - lse is taken as
// (x - M) - log z, both exact or small where it matters.
__device__ __forceinline__ void lse_parts(const float* part, int64_t stride, int64_t idx, int n, float& M, float& lz) {
  M = NEG;
  float z = 0.f;
  for (int s0 = 0; s0 < n; s0 += 16) {
    v2f v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      v[u] = s0 + u < n ? *(const v2f*)(part + ((s0 + u) * stride + idx) * 2) : v2f{NEG, 0.f};
#pragma unroll
    for (int u = 0; u < 16; ++u) merge_ms(M, z, v[u][0], v[u][1]);
  }
  lz = logf(z);
}
__device__ __forceinline__ float lsub(float x, float M, float lz) { return (x - M) - lz; }

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

// I_j, T_j rows of a j-tile: the thread's 16-B pieces, loaded into registers
// (issued one tile ahead) and then written to LDS [2][16][P+4] (zero rows past N)
template <int NB> struct JStage {
  static constexpr int P = 64 * NB, RS = P + 4, V = 2 * 16 * P / 4, U = (V + NT - 1) / NT;
  v4f val[U];
  __device__ __forceinline__ void load(const ClipK& a, int jb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = threadIdx.x + u * NT;
      const int m = v / (16 * P / 4), rem = v % (16 * P / 4), r = rem / (P / 4), c = (rem % (P / 4)) * 4;
      const int j = jb + r;
      const float* X = m ? a.T : a.I;
      const int64_t ld = m ? a.ldT : a.ldI;
      val[u] = (v < V && j < a.N) ? *(const v4f*)(X + (int64_t)j * ld + c) : v4f{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store(float* Xj) const {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = threadIdx.x + u * NT;
      if (v < V) {
        const int m = v / (16 * P / 4), rem = v % (16 * P / 4), r = rem / (P / 4), c = (rem % (P / 4)) * 4;
        *(v4f*)(Xj + (m * 16 + r) * RS + c) = val[u];
      }
    }
  }
};

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

// ------------------------------------------------------------------ products
template <int NB>
__global__ void __launch_bounds__(NT) clip_products_kernel(const ClipK a) {
  constexpr int P = 64 * NB, RS = P + 4;
  __shared__ __attribute__((aligned(16))) float Xj[2 * 16 * RS];
  __shared__ __attribute__((aligned(16))) float sc[4][16][16];   // [role][j][i]
  const int lane = threadIdx.x & 63, g = lane >> 4, il = lane & 15;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i0 = 16 * (int)blockIdx.x;
  const int js = blockIdx.y;
  const int jt0 = js * a.nrep, njt = (a.N + 15) / 16;
  const int jt1 = min(jt0 + a.nrep, njt);
  const float tau = a.tau, itau = 1.f / tau;
  const int N = a.N;

  v4f ir[4 * NB];
  load_iside<NB>(a, ty, i0, lane, ir);
  JStage<NB> st;
  st.load(a, 16 * jt0);
  float m0 = NEG, s0 = 0.f;   // S rows (wave 0), L rows (wave 2), L^T rows (wave 3)
  for (int jt = jt0; jt < jt1; ++jt) {
    const int jb = 16 * jt;
    __syncthreads();   // the previous tile's LDS reads are done
    st.store(Xj);
    __syncthreads();
    // the next tile's operands are loaded now: their loads are older than this
    // tile's matrix stores, so waiting for them never waits for the stores
    if (jt + 1 < jt1) st.load(a, jb + 16);
    const v4f d = score_tile<NB>(Xj, ty, ir, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) sc[ty][4 * g + r][il] = d[r];
    __syncthreads();
    {
      // the three scaled matrices, row stride NP (64-B row pieces per tile)
      const int jl = threadIdx.x & 15, irr = threadIdx.x >> 4, i = i0 + irr, j = jb + jl;
      if (i < N && j < N) {
        const int64_t o = (int64_t)i * a.NP + j;
        a.Sm[o] = (sc[0][jl][irr] + sc[1][jl][irr]) * (0.5f * tau);
        a.Lm[o] = sc[2][jl][irr] * itau;
        a.Ltm[o] = sc[3][jl][irr] * itau;
      }
    }
    if (ty != 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb + 4 * g + r;
        const float x = ty == 0 ? (d[r] + sc[1][4 * g + r][il]) * (0.5f * tau) : d[r] * itau;
        if (j < N) merge_ms(m0, s0, x, 1.f);
      }
    }
  }
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
}

// ------------------------------------------------------------------ stats
// Workgroup = 8 rows; wave w takes rows 2w, 2w + 1 over all j (lane: 4
// consecutive j per 16-B load), j in chunks of JC whose column statistics (S
// rows = Y columns by symmetry, L columns) the workgroup first combines from
// part1 into LDS.
constexpr int JC = 2048;
__global__ void __launch_bounds__(NT) clip_stats_kernel(const ClipK a) {
  __shared__ float jm[4][JC];   // (M, log z) of S rows and of L columns, j of the chunk
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = a.N, NP = a.NP;
  const float inv2n = 0.5f / (float)N;
  const int i0 = 8 * (int)blockIdx.x + 2 * w;
  // row statistics of L (L rows); those of S rows and L^T rows are column
  // statistics (S symmetric, L^T rows = L columns): read from the first staged
  // chunk, or combined here for rows past it
  float ms[2], zs[2], mr[2], zr[2], mc[2], zc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) lse_parts(a.part1, 3LL * N, (int64_t)N + min(i0 + u, N - 1), a.Js, mr[u], zr[u]);
  float c[2] = {0.f, 0.f}, q[2] = {0.f, 0.f};
  for (int jc0 = 0; jc0 < N; jc0 += JC) {
    const int jn = min(JC, N - jc0);
    __syncthreads();   // the previous chunk's reads are done
    for (int t = threadIdx.x; t < 2 * jn; t += NT) {
      const int j = t % jn, which = t / jn;
      float M, lz;
      lse_parts(a.part1, 3LL * N, (which ? 2LL * N : 0LL) + jc0 + j, a.Js, M, lz);
      jm[2 * which][j] = M;
      jm[2 * which + 1][j] = lz;
    }
    __syncthreads();
    if (jc0 == 0) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = min(i0 + u, N - 1);
        if (i < jn) {
          ms[u] = jm[0][i];
          zs[u] = jm[1][i];
          mc[u] = jm[2][i];
          zc[u] = jm[3][i];
        } else {
          lse_parts(a.part1, 3LL * N, i, a.Js, ms[u], zs[u]);
          lse_parts(a.part1, 3LL * N, 2LL * N + i, a.Js, mc[u], zc[u]);
        }
      }
    }
    for (int jb = 4 * lane; jb < jn; jb += 512) {
      v4f Sv[2][2], Lv[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t o = (int64_t)min(i0 + u, N - 1) * NP + min(jc0 + jb + 256 * h, NP - 4);
          Sv[u][h] = *(const v4f*)(a.Sm + o);
          Lv[u][h] = *(const v4f*)(a.Lm + o);
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int jl = jb + 256 * h + r;
          if (jl < jn) {
            const float msj = jm[0][jl], zsj = jm[1][jl], mcj = jm[2][jl], zcj = jm[3][jl];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              c[u] += __expf(lsub(Sv[u][h][r], msj, zsj));
              // log P_row + log P_col: G - rl then vanishes where Y is one-hot
              q[u] = fmaf(__expf(lsub(Sv[u][h][r], ms[u], zs[u])),
                          lsub(Lv[u][h][r], mr[u], zr[u]) + lsub(Lv[u][h][r], mcj, zcj), q[u]);
            }
          }
        }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float cs = wave_sum(c[u]), qs = wave_sum(q[u]);
    const int i = i0 + u;
    if (lane == 0 && i < N) {
      const float v[8] = {ms[u], zs[u], mr[u], zr[u], mc[u], zc[u], cs, -qs * inv2n};
#pragma unroll
      for (int k = 0; k < 8; ++k) a.stat[k * (int64_t)N + i] = v[k];
    }
  }
}

// ------------------------------------------------------------------ grad
// grid (gradient 16-row blocks, P / 16), or (1, 1) for the loss alone.
__global__ void __launch_bounds__(NT) clip_grad_kernel(const ClipK a, float* loss, float* row_loss, float* dI,
                                                       int64_t lddI, float* dT, int64_t lddT) {
  __shared__ __attribute__((aligned(16))) v4f accs[2][4][64];
  __shared__ float red[NT / 64];
  const int lane = threadIdx.x & 63, g = lane >> 4, il = lane & 15;
  const int w = threadIdx.x >> 6;
  const int N = a.N;
  const float tau = a.tau, itau = 1.f / tau, inv2n = 0.5f / (float)N;
  const float* st = a.stat;   // [8][N]: mS, zS, mR, zR, mC, zC, c, rl
  const float* rlv = a.stat + 7LL * N;
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    float acc = 0.f;
    for (int k = threadIdx.x; k < N; k += NT) {
      acc += rlv[k];
      if (row_loss) row_loss[k] = rlv[k];
    }
    acc = wave_sum(acc);
    if (lane == 0) red[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) *loss = (red[0] + red[1]) + (red[2] + red[3]);
  }
  if (!dI || a.Ng <= 0) return;
  const int i0 = a.g0 + 16 * (int)blockIdx.x;
  const int irow = min(i0 + il, N - 1);
  const int pc = 16 * (int)blockIdx.y;
  float si[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) si[k] = st[k * (int64_t)N + irow];
  const float ci = si[6], rli = si[7];
  const int64_t rowo = (int64_t)irow * a.NP;
  v4f accI = {0.f, 0.f, 0.f, 0.f}, accT = {0.f, 0.f, 0.f, 0.f};
  const int njt = (N + 15) / 16;
  // two j-tiles per step, every load of both issued before any is used
  for (int jt0 = w; jt0 < njt; jt0 += 8) {
    v4f Sv[2], Lv[2], Ltv[2];
    float sj[2][4][8], xi[2][4], xt[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int jt = min(jt0 + 4 * h, njt - 1);
      const int jb = 16 * jt + 4 * g;   // the lane's 4 j
      Sv[h] = *(const v4f*)(a.Sm + rowo + jb);
      Lv[h] = *(const v4f*)(a.Lm + rowo + jb);
      Ltv[h] = *(const v4f*)(a.Ltm + rowo + jb);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = min(jb + r, N - 1);
#pragma unroll
        for (int k = 0; k < 8; ++k) sj[h][r][k] = st[k * (int64_t)N + j];
        xi[h][r] = a.I[(int64_t)j * a.ldI + pc + il];
        xt[h][r] = a.T[(int64_t)j * a.ldT + pc + il];
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int jt = jt0 + 4 * h;
      if (jt < njt) {   // wave-uniform
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = 16 * jt + 4 * g + r;
          const float S = Sv[h][r], Lij = Lv[h][r], Lji = Ltv[h][r];
          const float* J = sj[h][r];
          const float Yij = __expf(lsub(S, si[0], si[1])), Yji = __expf(lsub(S, J[0], J[1]));
          // log-probabilities of L under its row / column softmax, (x - M) - log z
          const float rij = lsub(Lij, si[2], si[3]), cij = lsub(Lij, J[4], J[5]);
          const float rji = lsub(Lji, J[2], J[3]), cji = lsub(Lji, si[4], si[5]);
          const float Gij = -(rij + cij) * inv2n, Gji = -(rji + cji) * inv2n;
          const float Dm = (Yij * (Gij - rli) + Yji * (Gji - J[7])) * (0.5f * tau);
          const float dLij = (__expf(rij) - 2.f * Yij + __expf(cij) * J[6]) * inv2n;
          const float dLji = (__expf(rji) - 2.f * Yji + __expf(cji) * ci) * inv2n;
          const bool ok = j < N;
          const float bD = ok ? Dm : 0.f, bLt = ok ? dLji * itau : 0.f, bL = ok ? dLij * itau : 0.f;
          // dI^T[p][i] += I_j[p] Dm[i][j] + T_j[p] dL[j][i] / tau ; dT^T likewise
          accI = mma4(xi[h][r], bD, accI);
          accI = mma4(xt[h][r], bLt, accI);
          accT = mma4(xt[h][r], bD, accT);
          accT = mma4(xi[h][r], bL, accT);
        }
      }
    }
  }
  accs[0][w][lane] = accI;
  accs[1][w][lane] = accT;
  __syncthreads();
  if (w < 2) {
    // lane holds dI^T[p = pc + 4g + r][i = il] -> row i, 4 consecutive p
    const v4f s = (accs[w][0][lane] + accs[w][1][lane]) + (accs[w][2][lane] + accs[w][3][lane]);
    const int i = i0 + il;
    if (i < N && i < a.g0 + a.Ng) {
      const int64_t row = i - a.g0;
      float* dst = w == 0 ? dI + row * lddI : dT + row * lddT;
      *(v4f*)(dst + pc + 4 * g) = s;
    }
  }
}

// ------------------------------------------------------------ geometry
int64_t stride16(int64_t N) { return (N + 15) / 16 * 16; }

// products: ~1024 workgroups over nb i-blocks x nb j-tiles
void products_geometry(int64_t N, int& nrep, int& Js) {
  const int64_t nb = (N + 15) / 16;
  int64_t r = (nb * nb + 1023) / 1024;
  if (r < 1) r = 1;
  if (r > nb) r = nb;
  nrep = (int)r;
  Js = (int)((nb + r - 1) / r);
}

size_t off_matrices(int64_t N, int Js) { return ((size_t)Js * 3 * N * 2 + 8 * (size_t)N + 3) / 4 * 4; }

size_t ws_floats(int64_t N) {
  int nrep, Js;
  products_geometry(N, nrep, Js);
  return off_matrices(N, Js) + 3 * (size_t)N * stride16(N);
}

template <int NB>
int run(const maeclip_clip_args& a, hipStream_t s) {
  const int64_t N = a.N;
  const bool grad = a.dI && a.dT;
  const int64_t Ng = grad ? (a.grad_rows > 0 ? a.grad_rows : N - a.grad_row0) : 0;
  float* ws = (float*)a.workspace;
  ClipK k = {};
  k.I = a.I;
  k.T = a.T;
  k.ldI = a.ld_I ? a.ld_I : a.P;
  k.ldT = a.ld_T ? a.ld_T : a.P;
  k.N = (int)N;
  k.P = (int)a.P;
  k.NP = (int)stride16(N);
  k.tau = a.temperature;
  products_geometry(N, k.nrep, k.Js);
  k.part1 = ws;
  k.stat = k.part1 + (size_t)k.Js * 3 * N * 2;
  k.Sm = ws + off_matrices(N, k.Js);   // 16-B aligned
  k.Lm = k.Sm + (size_t)N * k.NP;
  k.Ltm = k.Lm + (size_t)N * k.NP;
  k.g0 = grad ? (int)a.grad_row0 : 0;
  k.Ng = (int)Ng;
  const unsigned nb = (unsigned)((N + 15) / 16);
  hipLaunchKernelGGL((clip_products_kernel<NB>), dim3(nb, k.Js), dim3(NT), 0, s, k);
  MC_CHECK_LAUNCH("maeclip_clip_loss(products)");
  hipLaunchKernelGGL(clip_stats_kernel, dim3((unsigned)((N + 7) / 8)), dim3(NT), 0, s, k);
  MC_CHECK_LAUNCH("maeclip_clip_loss(stats)");
  const bool g = grad && Ng > 0;
  const int64_t lddI = a.ld_dI ? a.ld_dI : a.P, lddT = a.ld_dT ? a.ld_dT : a.P;
  hipLaunchKernelGGL(clip_grad_kernel, dim3(g ? (unsigned)((Ng + 15) / 16) : 1u, g ? (unsigned)(a.P / 16) : 1u),
                     dim3(NT), 0, s, k, a.loss, a.row_loss_out, g ? a.dI : nullptr, lddI, a.dT, lddT);
  MC_CHECK_LAUNCH("maeclip_clip_loss(grad)");
  return 0;
}

}  // namespace

extern "C" size_t maeclip_clip_loss_workspace(int64_t N, int64_t P, int64_t grad_rows) {
  (void)grad_rows;
  if (N <= 0 || P <= 0) return 64 * sizeof(float);
  return ws_floats(N) * sizeof(float);
}

extern "C" int32_t maeclip_clip_loss(const maeclip_clip_args* a, void* stream) {
  MC_CHECK_ARG(a && a->I && a->T && a->loss && a->workspace, "maeclip_clip_loss: null pointer");
  MC_CHECK_ARG(a->N > 0 && a->N <= 16384, "maeclip_clip_loss: N must be in [1, 16384] (got %lld)", (long long)a->N);
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
