/* libmaeclip -- C-ABI of the MI355X (gfx950) kernels behind the mae_clip hot path.
 *
 * The reference (ykojima4020/mae_clip) has no FFI: its boundary is the PyTorch
 * nn.Module API of modules.ImageEncoder / TextEncoder / ProjectionHead
 * (modules.py:8-76) and CLIP.CLIPModel (CLIP.py:9-52), which calls into
 * timm / HF transformers / torch ops. Each entry point below replaces the op
 * those modules dispatch (cited per function); the Python package
 * mae_clip_amd binds them with ctypes.
 *
 * Conventions
 *   - plain pointers + sizes; every pointer is device memory unless noted;
 *     bf16 tensors are uint16 bit patterns; strides are in elements.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream).
 *   - no entry point allocates, frees or synchronises (graph-capture safe);
 *     workspaces are provided by the caller.
 *   - return 0 on success, <0 on error; maeclip_last_error() gives the
 *     message (thread-local).
 */
#ifndef MAECLIP_H
#define MAECLIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAECLIP_ABI_VERSION 11
#ifndef MAECLIP_F32
#define MAECLIP_F32 0
#define MAECLIP_BF16 1
#endif
#define MAECLIP_FP8_E4M3 2   /* OCP float8 e4m3fn (gfx950), max 448 */
#define MAECLIP_FP8_E5M2 3   /* OCP float8 e5m2, max 57344 */

int32_t maeclip_abi_version(void);
const char* maeclip_last_error(void);
/* number of gfx950 devices visible (0 when no GPU); does not create a context */
int32_t maeclip_device_count(void);

/* Plan options (A/B and test knobs of the kernels' launch planning). The
 * library reads every MAECLIP_<name> environment variable ONCE, at the first
 * call of any entry point below, into this table; launches read the table,
 * never the environment. maeclip_set_option overrides one entry (value -1 =
 * the built-in default). Defaults are the measured-fastest plans; no option
 * changes results beyond the bf16 rounding of a different tile / split.
 *   GEMM_BM          force a tile height of plain GEMMs (256 / 192 / 128; 0 auto)
 *   GEMM_SK          1: the cost model may pick the aligned split plan (0 off)
 *   GEMM_SPLIT       force a split of S slices (192-row tiles) where it fits
 *   GEMM_SPLIT_D     slice 0's lead in K-tiles per other slice (default 4)
 *   GEMM_SPLIT_MINK  the cost model's split only at K >= this (default 0)
 *   GEMM_BM128       1: 128-row tiles enter the cost model (default 0)
 *   GEMM_GRID        cap of the persistent GEMM grid (diagnostic; 0 = #CUs)
 *   WG_SK            0: grouped weight gradients use uniform split-K slices
 *                    instead of the stream-K remainder (default 1)
 *   ATTN_TWO         bf16 attention backward layout: 0 four images, 1 two, 3
 *                    two at 3 workgroups / CU (hd 32); -1 by occupancy
 *   ATTN_ROWS        1: fp32 attention on the streaming rows path
 *   ATTN_DIAG        diagonal backward (hd 32 on, hd 64 at npad >= 192); 0 / 1
 *   ATTN_BW16        16-wave backward beyond MAXW tiles (default hd 32); 0 / 1
 *   ATTN_FW16        16-wave forward when LDS leaves one workgroup (default 1) */
enum {
  MAECLIP_OPT_GEMM_BM = 0,
  MAECLIP_OPT_GEMM_SK = 1,
  MAECLIP_OPT_GEMM_SPLIT = 2,
  MAECLIP_OPT_GEMM_SPLIT_D = 3,
  MAECLIP_OPT_GEMM_SPLIT_MINK = 4,
  MAECLIP_OPT_GEMM_BM128 = 5,
  MAECLIP_OPT_GEMM_GRID = 6,
  MAECLIP_OPT_WG_SK = 7,
  MAECLIP_OPT_ATTN_TWO = 8,
  MAECLIP_OPT_ATTN_ROWS = 9,
  MAECLIP_OPT_ATTN_DIAG = 10,
  MAECLIP_OPT_ATTN_BW16 = 11,
  MAECLIP_OPT_ATTN_FW16 = 12,
  MAECLIP_OPT_COUNT = 13
};
/* returns the previous value, or INT32_MIN for an unknown key */
int32_t maeclip_set_option(int32_t key, int32_t value);
/* current value (-1: default), INT32_MIN for an unknown key */
int32_t maeclip_get_option(int32_t key);

/* ------------------------------------------------------------------ GEMM
 * Replaces torch.nn.functional.linear (cuBLAS) for every nn.Linear on the
 * hot path (timm Block qkv/proj/fc1/fc2, PatchEmbed conv-as-GEMM,
 * modules.py:64-66 ProjectionHead, DistilBERT q/k/v/out/lin1/lin2, HF ViTMAE
 * decoder_embed/decoder_pred) in forward, dgrad and wgrad form, and the
 * N x N x P products of the CLIP loss (CLIP.py:34-38).
 *   C[z][m][n] = alpha * sum_k A(m,k) B(k,n) (+bias[n]) (epilogue) (+beta*C)
 * layouts: 0 = K-contiguous (A[m*lda+k], B[n*ldb+k]); 1 = row-contiguous
 * (A[k*lda+m], B[k*ldb+n]).
 * epilogue: 0 none; 1 GELU (aux_out <- pre-activation, C <- gelu(pre));
 *           2 residual (C(f32) <- resid + acc (+bias)); 3 dGELU (C <- acc *
 *           gelu'(aux) (+ resid if resid != NULL)); 4 GELU' (C <- gelu(pre),
 *           aux_out <- gelu'(pre): the backward then needs no transcendental);
 *           5 mul-aux (C <- acc * aux (+ resid if resid != NULL)).
 *           For 1 and 4 aux_out may be NULL (forward-only callers).
 *           aux / aux_out have the operand dtype on the fp32 path, bf16 on the
 *           bf16 path.
 * colsum_partial (optional, f32 [batch*maeclip_gemm_colsum_rows(M)][N]):
 *   per-block column sums of the final C, reduce with maeclip_colsum_reduce.
 * splitk > 1 (epilogue 0, no colsum): K is cut into splitk slices whose fp32
 *   partial tiles go to workspace [batch][splitk][M][N]; a second launch sums
 *   them in fixed order (+bias, +beta*C) -> deterministic. Use
 *   maeclip_gemm_splitk(M,N,K) for the slice count. */
typedef struct {
  const void* A;
  const void* B;
  void* C;
  int64_t M, N, K;
  int64_t lda, ldb, ldc;
  int64_t batch, strideA, strideB, strideC;
  int32_t dtype;     /* MAECLIP_F32 = 0 / MAECLIP_BF16 = 1 (A, B, aux) */
  int32_t out_dtype; /* C */
  int32_t a_layout, b_layout;
  int32_t epilogue;
  float alpha, beta;
  const float* bias;
  const void* aux;
  void* aux_out;
  int64_t ldaux;
  const float* resid;
  int64_t ldr;
  float* colsum_partial;
  int32_t splitk;
  float* workspace;
  /* optional fp8-blocks copy of the output (bf16 C only, N % 128 == 0): q8
   * [M, ldq8] bytes of format q8_fmt and e8m0 block scales q8_scale
   * (maeclip_fp8b_scale_bytes(M, N) bytes), the quantisation of the bf16 C as
   * stored (bit-identical to maeclip_quant_blocks_fp8 of C): the next fp8
   * GEMM's A operand without a separate pass */
  void* q8;
  int64_t ldq8;
  uint8_t* q8_scale;
  int32_t q8_fmt;
} maeclip_gemm_args;
int32_t maeclip_gemm(const maeclip_gemm_args* args, void* stream);
/* fp8 GEMM (C4 path; replaces the nn.Linear matmuls of the timm / ViTMAE
 * blocks, modules.py:17-19, when precision = "fp8"). A [M, lda] and B [N, ldb]
 * are OCP fp8 bytes, both KC (K contiguous, K % 128 == 0, lda, ldb % 16 == 0);
 * args->dtype is A's format (MAECLIP_FP8_E4M3 / _E5M2), B is e4m3. The
 * block-scaled 16x16x128 MFMA accumulates in fp32 and the epilogue applies
 * scale_a[m] * scale_b[n] * alpha before bias / epilogue (args->epilogue as
 * maeclip_gemm; no split-K, beta must be 0). M, N >= 256, N % 8 == 0. */
int32_t maeclip_gemm_fp8(const maeclip_gemm_args* args, const float* scale_a, const float* scale_b, void* stream);
/* fp8 BLOCKS (the MX layout of the block-scaled MFMA): a row of K elements is
 * cut into K / 32 blocks, each quantised with its own power-of-two scale
 * 2^(e - 127), e an e8m0 byte: e = the smallest exponent with amax(block) /
 * 2^(e - 127) <= FMT_MAX, q = rne(x * 2^(127 - e)); x ~= q * 2^(e - 127). A
 * producer that owns only part of a row (a GEMM epilogue tile, an attention
 * head) can quantise it without the whole-row amax a per-row scale needs.
 * Scale bytes are laid out for the GEMM's reads (K % 128 == 0):
 *   byte (r, b) at (((r / 64) * (K / 128) + b / 4) * 256 + (b % 4) * 64 +
 *                   (r % 16) * 4 + (r / 16) % 4)
 * maeclip_fp8b_scale_bytes(rows, K) = ceil(rows / 64) * 64 * K / 32. */
int64_t maeclip_fp8b_scale_bytes(int64_t rows, int64_t K);
/* x (bf16 / f32 [rows, ld]) -> fp8 blocks q [rows, ldq] + scales (cols % 128 == 0) */
int32_t maeclip_quant_blocks_fp8(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ld, void* q,
                                 int64_t ldq, uint8_t* scales, int32_t fmt, void* stream);
/* fp8 GEMM with an fp8-blocks A operand: as maeclip_gemm_fp8, the A block
 * scales (e8m0, the layout above, K = args->K) applied by the MFMA itself,
 * B (e4m3) scaled per column by scale_b in the epilogue. */
int32_t maeclip_gemm_fp8_blocks(const maeclip_gemm_args* args, const uint8_t* scale_a, const float* scale_b,
                                void* stream);
/* Row-wise fp8 quantisation: q[r, :] = rne(x[r, :] / s[r]), s[r] = amax(x[r, :]) /
 * FMT_MAX (1 when the row is zero). x bf16 or f32 [rows, ld]; q [rows, ldq]
 * bytes; fmt MAECLIP_FP8_E4M3 (activations, weights) or _E5M2 (gradients). */
int32_t maeclip_quant_rows_fp8(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ld, void* q,
                               int64_t ldq, float* scales, int32_t fmt, void* stream);
/* W^T quantisation (e4m3) from the fp32 master W [rows, ld]: qt [cols, ldq]
 * (ldq % 16 == 0), one scale per column of W (per row of W^T). */
/* Every fp8 stack weight of a step at once (two launches): for each entry,
 * q = rows of W quantised per output channel (scales sq [rows]) and qt = W^T
 * quantised per input channel (scales sqt [cols], rows of ldqt bytes), from
 * the fp32 master W [rows, ld], cols <= 4096 (the first launch keeps a row in
 * registers: it quantises the rows and takes the column maxima from that one
 * read; the second reads W again for W^T). The host array is filled in by
 * maeclip_quant_weights_fp8_prepare (prefix sums; returns the workspace
 * bytes); dev is its device copy. */
typedef struct {
  const float* w;
  void* q;
  float* sq;
  void* qt;
  float* sqt;
  int32_t rows, cols, ld, ldqt;
  int64_t row_begin, unit_begin, part_begin;
} maeclip_fp8w_entry;
int64_t maeclip_quant_weights_fp8_prepare(maeclip_fp8w_entry* host, int32_t n);
int32_t maeclip_quant_weights_fp8(const maeclip_fp8w_entry* dev, const maeclip_fp8w_entry* host, int32_t n,
                                  float* workspace, int64_t ws_bytes, void* stream);
int64_t maeclip_quant_cols_fp8_workspace(int64_t rows, int64_t cols);
int32_t maeclip_quant_cols_fp8(const float* w, int64_t rows, int64_t cols, int64_t ld, void* qt, int64_t ldq,
                               float* scales, float* workspace, int64_t ws_bytes, void* stream);
int64_t maeclip_gemm_colsum_rows(int64_t M);
/* scratch bytes maeclip_gemm may use for *args when args->splitk <= 1 (pass
 * them as args->workspace; a NULL workspace is always valid, just slower) */
int64_t maeclip_gemm_workspace(const maeclip_gemm_args* args);
/* which implementation maeclip_gemm runs for *args: always 0 = this library's
 * kernels (kept from ABI v9; the round-4 vendor-library path was removed) */
int32_t maeclip_gemm_impl(const maeclip_gemm_args* args);
int32_t maeclip_gemm_splitk(int64_t M, int64_t N, int64_t K);

/* Grouped weight gradients. Replaces the weight-gradient half of autograd's
 * nn.Linear backward (torch.nn.functional.linear's backward, reached from
 * loss.backward() at main.py:58) for all Linears of a transformer stack at
 * once (timm Block qkv/proj/fc1/fc2, HF ViTMAE decoder layers):
 *   dw_p[n][k] = sum_m dy_p[m*ldy + n] * x_p[m*ldx + k]  (+ beta * dw_p[n][k])
 * for p < nprob, m < M (tokens, shared by every problem). dw is fp32 dense
 * [N][K]; dy/x have `dtype`. bf16 problems with M % 64 == 0 and N, K >= 256
 * share one persistent launch per 48 problems (split-K slabs, S <= 4, only when
 * they cut the waves of output tiles by >= 15%); others run one maeclip_gemm
 * each.
 * Deterministic (fixed summation order). workspace: >= the bytes
 * maeclip_wgrad_grouped_workspace() returns (0 is common), 16-B aligned. */
typedef struct {
  const void* dy;
  const void* x;
  float* dw;
  int64_t N, K, ldy, ldx;
} maeclip_wgrad_problem;
int64_t maeclip_wgrad_grouped_workspace(const maeclip_wgrad_problem* probs, int32_t nprob, int64_t M,
                                        int32_t dtype);
int32_t maeclip_wgrad_grouped(const maeclip_wgrad_problem* probs, int32_t nprob, int64_t M, int32_t dtype,
                              float beta, void* workspace, int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------- attention
 * Replaces F.scaled_dot_product_attention in timm Attention / HF ViTMAE
 * decoder layers and DistilBERT attention with key-padding mask
 * (modeling_distilbert.py:125-145). qkv: [B*n, ld_qkv] token rows with q at
 * column h*hd, k at H*hd + h*hd, v at 2*H*hd + h*hd. o: [B*n, ld_o].
 * lse: [B, H, n] f32, log2-domain row log-sum-exp of scale*q.k (bwd input).
 * key_mask (optional, f32 [B, n]): 0 = padding key (forward; the backward
 * takes it only in fp32 at n beyond the LDS images -- the streamed "rows"
 * path -- and rejects it otherwise: the frozen text tower has no backward).
 * dropout_p applies to the probabilities in the forward only (DistilBERT
 * attention dropout; no bwd). fp32 forward / backward at any n: past the LDS
 * images (n ~ 540 at hd 32) 64-row blocks are streamed (no dropout there).
 * bwd: dout [B*n, ld_o], dqkv [B*n, ld_dqkv]; colsum_partial optional
 * [B, 3*H*hd] per-sample column sums of dqkv (qkv bias gradient). */
typedef struct {
  const void* qkv;
  void* o;
  float* lse;
  const void* dout;
  void* dqkv;
  const float* key_mask;
  float* colsum_partial;
  int64_t ld_qkv, ld_o, ld_dqkv;
  int32_t B, n, H, head_dim, dtype;
  float scale, dropout_p;
  uint64_t seed;
  /* optional device step counter: dropout seed = seed + (*step_ptr) * MAECLIP_STEP_MULT
   * (so a captured HIP graph draws fresh masks every replay) */
  const int64_t* step_ptr;
  /* optional fp8-blocks copy of the main output (maeclip_fp8b_scale_bytes
   * layout; o [B*n, H*head_dim] for the forward, dqkv [B*n, 3*H*head_dim] for
   * the backward, whose row length must be a multiple of 128): the bytes of
   * maeclip_quant_blocks_fp8 of the bf16 output as stored. Written by the
   * bf16 MFMA kernels' own stores; the other variants (fp32, the diagonal and
   * row-streaming backward) run the standalone pass after the kernel. */
  void* q8;
  int64_t ldq8;
  uint8_t* q8_scale;
  int32_t q8_fmt;
} maeclip_attn_args;
int32_t maeclip_attn_fwd(const maeclip_attn_args* args, void* stream);
int32_t maeclip_attn_bwd(const maeclip_attn_args* args, void* stream);

/* ------------------------------------------------------------- LayerNorm
 * Replaces nn.LayerNorm (timm norm1/norm2/fc_norm, modules.py:67, DistilBERT
 * LayerNorms, decoder_norm). fwd: x' = dropout(x; in_dropout_p) + res;
 * y = LN(x') (* out dropout); y2 optional bf16 copy; xsum_out optional x'. */
typedef struct {
  const void* x;
  int32_t x_dtype;
  const float* res;
  int64_t ldres;
  float in_dropout_p;
  const float* gamma;
  const float* beta;
  void* y;
  int32_t y_dtype;
  void* y2;
  int64_t ldy2;
  float* xsum_out;
  int64_t ldxs;
  float* mean;
  float* rstd;
  float out_dropout_p;
  uint64_t seed_in, seed_out;
  const int64_t* step_ptr; /* optional: both seeds + (*step_ptr) * MAECLIP_STEP_MULT */
  int64_t M, D, ldx, ldy;
  float eps;
  /* optional fp8 copy of y for an fp8 GEMM (C4): q8 [M, ldq8] quantised per
   * row exactly as maeclip_quant_rows_fp8 would quantise the stored y (format
   * q8_fmt, scales q8_scale [M]) -- the quantisation pass fused into the LN */
  void* q8;
  int64_t ldq8;
  float* q8_scale;
  int32_t q8_fmt;
} maeclip_ln_fwd_args;
int32_t maeclip_ln_fwd(const maeclip_ln_fwd_args* args, void* stream);

/* bwd: dx(f32) = LN'(dy) + dres; dx_bf optional bf16 copy; partials
 * [maeclip_ln_bwd_partial_rows(M, D)][D] of dgamma, dbeta, colsum(dx) (ABI 10: the
 * count depends on D -- up to 1024 workgroups at D <= 512, 512 above).
 * dres_pool (instead of dres, optional): the residual gradient is the
 * backward of timm's global_pool="avg" over pool_n tokens per sample, read
 * from dres_pool [M / pool_n][D]: row r gets dres_pool[r / pool_n] / (pool_n - 1)
 * for r % pool_n != 0 and 0 for the prefix (cls) token -- the pool backward
 * fused into the LN backward, no [M, D] residual tensor in HBM. */
typedef struct {
  const void* dy;
  int32_t dy_dtype;
  const void* x;
  int32_t x_dtype;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* dres;
  float* dx;
  void* dx_bf;
  int64_t lddx_bf;
  float* dgamma_partial;
  float* dbeta_partial;
  float* dx_colsum_partial;
  int64_t M, D, ldx, lddy, lddx;
  const float* dres_pool;
  int64_t pool_n;
  /* optional fp8 copy of dx_bf (required with it) for an fp8 dgrad GEMM, as
   * maeclip_quant_rows_fp8 of dx_bf with format q8_fmt (fused) */
  void* q8;
  int64_t ldq8;
  float* q8_scale;
  int32_t q8_fmt;
} maeclip_ln_bwd_args;
int32_t maeclip_ln_bwd(const maeclip_ln_bwd_args* args, void* stream);
int32_t maeclip_ln_bwd_partial_rows(int64_t M, int64_t D);

/* ------------------------------------------------------------ reductions */
/* out[n] (+)= scale * sum_p partial[p*N + n]  (fixed order -> deterministic);
 * two passes when maeclip_colsum_scratch(P, N) > 0: scratch holds that many
 * floats (N > 1, P > 64: [ceil(P/64)][N]; N == 1, P > 4096: ceil(P/4096)),
 * may be NULL otherwise. */
int32_t maeclip_colsum_reduce(const float* partial, int64_t P, int64_t N, float* out, int32_t accumulate, float scale,
                              float* scratch, void* stream);
int64_t maeclip_colsum_scratch(int64_t P, int64_t N);
/* many independent column reductions in one launch (bias / LN-parameter
 * gradients of a whole transformer stack): out[n] (+)= scale * sum_p partial[p][n];
 * block_start = prefix sum of ceil(N/64) over the entries. */
typedef struct {
  const float* partial;
  float* out;
  int64_t P, N;
  float scale;
  int32_t accumulate;
  int64_t block_start;
} maeclip_colsum_entry;
int32_t maeclip_colsum_multi(const maeclip_colsum_entry* dev_entries, const maeclip_colsum_entry* host_entries,
                             int32_t ne, void* stream);
/* partial column sums of a [M, D] row matrix (dtype f32/bf16, row stride ld)
 * into partial [maeclip_rows_colsum_partial_rows(M)][D]; optional bf16 copy
 * out_bf16 [M, D]. */
int32_t maeclip_rows_colsum(const void* x, int32_t dtype, int64_t M, int64_t D, int64_t ld, void* out_bf16,
                            float* partial, void* stream);
/* the same with the fp8 rows of the bf16 copy (per-row scales, bit-identical
 * to maeclip_quant_rows_fp8 of out_bf16; the fp8 stack's top operand) */
int32_t maeclip_rows_colsum_q8(const void* x, int32_t dtype, int64_t M, int64_t D, int64_t ld, void* out_bf16,
                               float* partial, void* q8, int64_t ldq8, float* q8_scale, int32_t q8_fmt, void* stream);
int32_t maeclip_rows_colsum_partial_rows(int64_t M);
/* timm global_pool="avg": out[b] = mean_{t>=1} x[b,t,:] ; bwd scatters 1/(n-1) */
int32_t maeclip_pool_fwd(const float* x, int32_t B, int32_t n, int32_t D, float* out, void* stream);
int32_t maeclip_pool_bwd(const float* dout, int32_t B, int32_t n, int32_t D, float* dx, int32_t accumulate, void* stream);
/* nn.Dropout with the library's counter-based mask (same as LN in_dropout) */
int32_t maeclip_dropout(const float* x, float* y, int64_t M, int32_t D, int64_t ld, float p, uint64_t seed,
                        const int64_t* step_ptr, void* stream);
/* DistilBERT Embeddings word+position gather (modeling_distilbert.py:92-117);
 * mask_in (optional, int64 [B*T], the tokenizer's attention_mask) -> mask_out
 * (f32 [B*T], the attention kernels' key mask) in the same launch */
int32_t maeclip_embed_fwd(const int64_t* ids, const float* word, const float* pos, int32_t B, int32_t T, int32_t D,
                          int64_t V, float* out, const int64_t* mask_in, float* mask_out, void* stream);

/* ---------------------------------------------------------- multi-tensor */
typedef struct {
  void* p0; /* param (f32) / cast source */
  void* p1; /* grad (f32) */
  void* p2; /* exp_avg */
  void* p3; /* exp_avg_sq */
  void* p4; /* bf16 shadow / cast destination (optional for adamw) */
  int64_t n;
  int64_t chunk_start; /* prefix sum of ceil(n / maeclip_mt_chunk()) */
} maeclip_mt_entry;
typedef struct {
  float lr, beta1, beta2, eps, weight_decay;
  float step_size; /* lr / (1 - beta1^t) */
  float bc2_sqrt;  /* sqrt(1 - beta2^t) */
  float grad_scale;
  /* optional device step count t (>= 1): when set, step_size and bc2_sqrt are
   * recomputed in the kernel from lr, beta1, beta2 and *step_ptr */
  const int64_t* step_ptr;
} maeclip_adamw_hparams;
int64_t maeclip_mt_chunk(void);
/* dev_entries: device copy of host_entries (host pointer used for the grid size) */
int32_t maeclip_cast_multi(const maeclip_mt_entry* dev_entries, const maeclip_mt_entry* host_entries, int32_t ne,
                           void* stream);
/* flat conversion dst[i] = scale * src[i], dtypes MAECLIP_F32 / MAECLIP_BF16
 * (RNE): the bf16 gradient all-reduce buckets of data parallelism */
int32_t maeclip_cast_flat(const void* src, int32_t src_dtype, void* dst, int32_t dst_dtype, int64_t n, float scale,
                          void* stream);
/* torch.optim.AdamW step (main.py:101-103,59) fused over all parameters */
int32_t maeclip_adamw_multi(const maeclip_mt_entry* dev_entries, const maeclip_mt_entry* host_entries, int32_t ne,
                            const maeclip_adamw_hparams* hp, void* stream);

/* ------------------------------------------------------------------- MAE */
/* HF ViTMAE random_masking (modeling_vit_mae.py:297-327) with counter-based
 * noise: ids int32 [B, L]; mask f32 [B, L] (1 = removed); noise optional. */
typedef struct {
  int32_t* ids_shuffle;
  int32_t* ids_restore;
  float* mask;
  float* noise;
  int32_t B, L, len_keep;
  uint64_t seed, step, sample_offset;
  const int64_t* step_ptr; /* optional: step used = step + *step_ptr */
} maeclip_mask_args;
int32_t maeclip_mask_ids(const maeclip_mask_args* args, void* stream);

/* visible-patch rows for the patch-embed GEMM (timm PatchEmbed Conv2d(k=s=p)
 * as GEMM): out[(b*keep+j), c*p*p+ky*p+kx] = img[b,c,py*p+ky,px*p+kx] for
 * patch l = ids_shuffle[b,j] (identity if NULL); columns >= C*p*p zeroed.
 * Image source: fp32 NCHW img, or -- when img_u8 is set (img ignored) -- the
 * decoded uint8 RGB HWC pixels [B][S][S][C] (C = 3) with albumentations
 * Normalize(u8_mean, u8_std, u8_max_pixel) (dataset.py:49) and the HWC->CHW
 * permute (dataset.py:34) applied in the gather: the fp32 image is never
 * materialised (same floats as maeclip_image_normalize_u8 + the fp32 gather). */
typedef struct {
  const float* img;
  const int32_t* ids_shuffle;
  void* out;
  int64_t ld_out;
  int32_t B, C, S, p, keep, dtype;
  const uint8_t* img_u8;
  float u8_mean[3], u8_std[3], u8_max_pixel;
} maeclip_patch_args;
int32_t maeclip_patch_gather(const maeclip_patch_args* args, void* stream);

/* Input pipeline. Replaces dataset.py:44-58 on the host: albumentations
 * Normalize(mean, std, max_pixel_value) of the decoded RGB uint8 HWC image
 * (dataset.py:49) and permute(2, 0, 1).float() (dataset.py:34), for a batch:
 * src uint8 [B][H][W][3] dense -> dst fp32 [B][3][H][W] dense,
 * dst = (float(src) - mean*max_pixel) * (1 / (std*max_pixel)) in fp32. */
typedef struct {
  const uint8_t* src;
  float* dst;
  int64_t B, H, W;
  float mean[3], std[3];
  float max_pixel;
} maeclip_image_u8_args;
int32_t maeclip_image_normalize_u8(const maeclip_image_u8_args* args, void* stream);
/* The whole get_transforms() pipeline of dataset.py:44-58 + the permute of
 * :34 in one pass, for decoded RGB uint8 HWC images of ANY sizes: A.Resize(S,
 * S) (cv2.resize INTER_LINEAR: OpenCV's fixed-point uint8 algorithm, equal
 * size = copy, exact 2x = INTER_AREA) then A.Normalize as above, into dst fp32
 * [B][3][S][S]. images: DEVICE array of B descriptors (src rows of row_stride
 * bytes, 3 interleaved channels). */
typedef struct {
  const uint8_t* src;
  int32_t H, W;
  int64_t row_stride;
} maeclip_image_src;
typedef struct {
  const maeclip_image_src* images;
  float* dst;
  int64_t B, S;
  float mean[3], std[3];
  float max_pixel;
} maeclip_preprocess_args;
int32_t maeclip_image_preprocess_u8(const maeclip_preprocess_args* args, void* stream);

/* Retrieval (inference.py:40-45). l2_normalize replaces F.normalize(x, p=2,
 * dim=-1): y = x / max(||x||_2, eps), fp32 [M][P] rows (strides ldx / ldy).
 * topk_rows replaces torch.topk(dot_similarity, k) row-wise: s fp32 [Q][N]
 * (row stride lds) -> vals [Q][k] descending, idx [Q][k] (int64), ties broken
 * by the lower index; 1 <= k <= min(N, 1024). The similarity itself is an
 * fp32 maeclip_gemm (text_n @ image_n^T). */
int32_t maeclip_l2_normalize(const float* x, float* y, int64_t M, int64_t P, int64_t ldx, int64_t ldy, float eps,
                             void* stream);
int32_t maeclip_topk_rows(const float* s, int64_t Q, int64_t N, int64_t lds, int32_t k, float* vals, int64_t* idx,
                          void* stream);

/* timm _pos_embed on the visible tokens: x[b,0] = cls + pos[0];
 * x[b,1+j] = y[b*keep+j] + pos[1+ids_shuffle[b,j]]; bwd: dy rows, dpos, dcls. */
typedef struct {
  const void* y;
  int64_t ldy;
  const int32_t* ids_shuffle;
  const int32_t* ids_restore;
  const float* pos;
  const float* cls;
  float* x;
  const float* dx;
  void* dy;
  float* dpos;
  float* dcls;
  int32_t B, L, keep, D, dtype;
} maeclip_tokens_args;
int32_t maeclip_tokens_fwd(const maeclip_tokens_args* args, void* stream);
int32_t maeclip_tokens_bwd(const maeclip_tokens_args* args, void* stream);

/* HF ViTMAEDecoder mask-token append + unshuffle + pos (modeling_vit_mae.py:548-566).
 * fwd: y f32 [B, 1+keep, ldy] -> out f32 [B, 1+L, D]. bwd (reads ids_restore):
 * dout f32 -> dy (dtype) [B, 1+keep, ldy]; dmask_partial / colsum_partial f32
 * [maeclip_unshuffle_bwd_partial_rows(B), D] (column-reduce them: mask_token
 * and decoder_embed bias gradients). D % 4 == 0, D <= 1024. */
typedef struct {
  const float* y;
  int64_t ldy;
  const int32_t* ids_shuffle;
  const int32_t* ids_restore;
  const float* mask_token;
  const float* pos;
  float* out;
  const float* dout;
  void* dy;
  float* dmask_partial;
  float* colsum_partial;
  int32_t B, L, keep, D, dtype;
} maeclip_unshuffle_args;
int32_t maeclip_unshuffle_fwd(const maeclip_unshuffle_args* args, void* stream);
int32_t maeclip_unshuffle_bwd(const maeclip_unshuffle_args* args, void* stream);
int32_t maeclip_unshuffle_bwd_partial_rows(int32_t B);

/* MAE reconstruction loss (modeling_vit_mae.py:706-745 patchify, :852-859).
 * pred: decoder output rows [B, 1+L, ldp] (row 0 = cls, ignored); targets are
 * patchified from img on the fly (only for masked patches) -- fp32 NCHW img,
 * or the uint8 HWC pixels img_u8 normalised in-kernel exactly as in
 * maeclip_patch_args (u8_mean / u8_std / u8_max_pixel). fwd: row_loss [B*L]
 * = mask * mean_k diff^2 (sum / mask_count outside). bwd: dpred [B, 1+L, lddp]
 * = grad_out[0] * loss_scale * 2 diff mask / (P * mask_count) (columns
 * [P, lddp) zeroed); colsum_partial [maeclip_mae_loss_bwd_partial_rows(B, L)][P]
 * optional. P = C*p*p <= 1024, P % 4 == 0. */
typedef struct {
  const void* pred;
  int64_t ldp;
  const float* img;
  const float* mask;
  float* row_loss;
  void* dpred;
  int64_t lddp;
  const float* grad_out;
  float* colsum_partial;
  float loss_scale, mask_count;
  int32_t B, C, S, p, L, norm_pix, dtype;
  const uint8_t* img_u8;
  float u8_mean[3], u8_std[3], u8_max_pixel;
} maeclip_mae_loss_args;
int32_t maeclip_mae_loss_fwd(const maeclip_mae_loss_args* args, void* stream);
int32_t maeclip_mae_loss_bwd(const maeclip_mae_loss_args* args, void* stream);
int32_t maeclip_mae_loss_bwd_partial_rows(int32_t B, int32_t L);

/* ------------------------------------------------------------- CLIP loss
 * CLIPModel.forward loss (CLIP.py:34-43) + cross_entropy (CLIP.py:46-52), fp32,
 * fused and deterministic, three launches at every N: the all-pairs products
 * once on the exact-f32 MFMA (S, L, L^T kept in the workspace, online row-LSE
 * partials), one statistics pass over the stored rows (row / column LSE, the
 * column sums of the soft targets, per-row losses and the loss), and the
 * gradient rows of the requested slice (no reduction launch). Above N = 2048
 * the statistics pass stages the column statistics per 2048-column chunk.
 * Any N >= 1; P in {64, 128, 256, 512}. I, T: [N, P] (row strides ld_I/ld_T, 0 = P, 16-B aligned rows).
 * loss: device scalar. row_loss_out (optional, [N]): rl_i with loss = sum rl_i.
 * dI, dT optional: d loss / d I, T for the rows [grad_row0, grad_row0 +
 * grad_rows) only (grad_rows 0 = to the end), stored from row 0 of dI / dT --
 * under data parallelism each rank asks for its own slice of the gathered batch.
 * workspace: >= maeclip_clip_loss_workspace(N, P, number of gradient rows). */
typedef struct {
  const float* I;
  const float* T;
  int64_t ld_I, ld_T;
  int64_t N, P;
  float temperature;
  float* loss;
  float* row_loss_out;
  float* dI;
  float* dT;
  int64_t ld_dI, ld_dT;
  int64_t grad_row0, grad_rows;
  void* workspace;
  size_t ws_bytes;
} maeclip_clip_args;
size_t maeclip_clip_loss_workspace(int64_t N, int64_t P, int64_t grad_rows);
int32_t maeclip_clip_loss(const maeclip_clip_args* args, void* stream);

/* ------------------------------------------------------------ step state
 * Device-resident step counters (model RNG step, optimizer step t) so that a
 * whole training step can be captured once in a HIP graph and replayed. */
#define MAECLIP_STEP_MULT 0x9E3779B97F4A7C15ull
int32_t maeclip_counter_add(int64_t* counter, int64_t delta, void* stream);
/* snap[0] = counter[0]; counter[0] += delta -- the step a forward used, kept for
 * its backward (dropout masks re-drawn there) without a separate copy */
int32_t maeclip_counter_add_snap(int64_t* counter, int64_t delta, int64_t* snap, void* stream);
/* loss combination on device scalars (CLIP.py total loss + MAE term):
 * out[0] = a[0] + w * b[0] */
int32_t maeclip_scalar_axpy(const float* a, const float* b, float w, float* out, void* stream);
/* Pinned, device-mapped host memory (hipHostMalloc mapped) for values the host
 * reads every step without a copy launch: *host_ptr for the CPU, *dev_ptr for
 * kernels (e.g. maeclip_copy_f32's dst). The reference reads its loss every
 * step (main.py:64 loss.item()); a kernel inside the captured step writes it
 * here instead of a device-to-host copy. */
int32_t maeclip_host_mapped_alloc(int64_t bytes, void** host_ptr, void** dev_ptr);
int32_t maeclip_host_mapped_free(void* host_ptr);
/* dst[0..n) = src[0..n) (f32, small n; dst may be device-mapped host memory) */
int32_t maeclip_copy_f32(const float* src, float* dst, int64_t n, void* stream);
/* dst[(counter[0] & 1) n + i] = src[i]: the step's loss into one of two host
 * slots picked by the device step counter, so the host can read step k's value
 * while step k + 1 (writing the other slot) is already running */
int32_t maeclip_copy_f32_slot(const float* src, float* dst, int64_t n, const int64_t* counter, void* stream);
/* dst_i[k] = w * s[0] * src_i[k] (src_i NULL: w * s[0]) for two dense f32
 * arrays in one launch (n_i = 0: unused); src_i == dst_i allowed. The
 * backward of a loss that scales stored gradients by the incoming grad_output
 * (a device scalar) without a host sync. */
int32_t maeclip_scale_by_scalar2(const float* src0, float* dst0, int64_t n0, const float* src1, float* dst1, int64_t n1,
                                 const float* s, float w, void* stream);
/* stream-ordered device timestamp (REALTIME counter, maeclip_wallclock_khz ticks/ms) */
int32_t maeclip_timestamp(int64_t* dst, void* stream);
int64_t maeclip_wallclock_khz(void);
/* stream-ordered host->device copy (pinned src), capturable into a HIP graph */
int32_t maeclip_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAECLIP_H */
