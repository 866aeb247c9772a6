// Library-shaped GEMMs through hipBLASLt, the vendor library -- the "plain
// library GEMM" case of the MI355X playbook: C = alpha A op(B) [+ bias] with a
// bf16 C, or the residual form C = alpha A op(B) + bias + R with fp32 R and C
// (the epilogues hipBLASLt runs itself: its BIAS epilogue, beta = 1 on an fp32
// C), at K > 512. Everything else -- GELU / GELU' / dGELU / mul-aux epilogues,
// column-sum partials, K = 512 (the MAE decoder's qkv / fc1 forward, proj
// dgrad: 0.83-0.98x here), fp8, the grouped weight gradients -- stays on this
// library's own kernels (gemm4.hip).
//
// Why (profiles/r04/plain_gemm_vendor_probe_r4u.jsonl, same box): at K >= 768
// the vendor's stream-K kernels run 1.00-1.84x of v4 on the step's plain shapes
// (1.84x: encoder fc1 dgrad at the micro-batch's 6400 rows, one partial round
// of v4 tiles), at K = 512 0.83-0.98x; the whole C2 step gains 2.1 % with the
// plain bf16 launches there (plain_gemm_vendor_ab_r4t.txt) and 4.2 % with the
// residual-form forwards as well (gemm_vendor_modes_ab_r4v.txt: 10032 -> 10456
// img/s, three rounds each on one box). MAECLIP_GEMM_LIB=0 keeps every GEMM on
// v4 (A/B, tests of the own kernels).
//
// Layout: row-major C[M,N] = A[M,K] op(B) is, column-major, C^T[N,M] =
// op(B)^T A^T, where A^T is A's storage read column-major ([K,M], ld lda) and
// op(B)^T is B's storage read column-major: [K,N] transposed (KC B, stored
// [N][K]) or [N,K] as is (RC B, stored [K][N]).
#include "common.h"
#include <hipblaslt/hipblaslt.h>
#include <stdlib.h>
#include <mutex>
#include <unordered_map>
#include "../../include/maeclip.h"

namespace {

enum { LAY_KC = 0, LAY_RC = 1 };
constexpr int64_t LIB_WS = 32ll << 20;   // workspace offered to hipBLASLt's heuristic (stream-K partials)

struct LibKey {
  int64_t M, N, K, lda, ldb, ldc, ldr;
  int lb, out, ws, bias, res, at;
  bool operator==(const LibKey& o) const {
    return M == o.M && N == o.N && K == o.K && lda == o.lda && ldb == o.ldb && ldc == o.ldc && ldr == o.ldr &&
           lb == o.lb && out == o.out && ws == o.ws && bias == o.bias && res == o.res && at == o.at;
  }
};
struct LibKeyHash {
  size_t operator()(const LibKey& k) const {
    size_t h = 1469598103934665603ull;
    for (int64_t v : {k.M, k.N, k.K, k.lda, k.ldb, k.ldc, k.ldr, (int64_t)k.lb, (int64_t)k.out, (int64_t)k.ws,
                      (int64_t)k.bias, (int64_t)k.res, (int64_t)k.at})
      h = (h ^ (size_t)v) * 1099511628211ull;
    return h;
  }
};
struct LibPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, lr = nullptr;   // lr: the residual C (fp32)
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
  // the heuristic's candidates (MAECLIP_GEMM_LIB_TUNE: the fastest of them,
  // timed once on the first call outside a graph capture)
  static constexpr int NCAND = 16;
  hipblasLtMatmulAlgo_t cand[NCAND];
  size_t cand_ws[NCAND] = {};
  int ncand = 0;
  bool tuned = false;
};

struct LibState {
  std::mutex mu;
  hipblasLtHandle_t handle[64] = {};
  std::unordered_map<LibKey, LibPlan, LibKeyHash> plans[64];
};
LibState& state() {
  static LibState s;
  return s;
}

// MAECLIP_GEMM_LIB: 0 = off (default: this library's kernels for every GEMM),
// 1 = vendor for the plain / residual forms at K > 512, 2 = bf16 outputs only
// (calibration A/B only)
int lib_mode() {
  const char* e = getenv("MAECLIP_GEMM_LIB");
  return (e && *e) ? atoi(e) : 0;
}

// MAECLIP_GEMM_LIB_TUNE=1: time the heuristic's candidates once per shape
bool tune_on() {
  const char* e = getenv("MAECLIP_GEMM_LIB_TUNE");
  return e && *e == '1';
}

// plan (descriptors + the heuristic's first algorithm) of one shape, cached per device
LibPlan* plan_for(const maeclip_gemm_args& a, bool have_ws, const float* scale_a = nullptr,
                        const float* scale_b = nullptr) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  LibState& st = state();
  std::lock_guard<std::mutex> lock(st.mu);
  if (!st.handle[dev] && hipblasLtCreate(&st.handle[dev]) != HIPBLAS_STATUS_SUCCESS) {
    st.handle[dev] = nullptr;
    return nullptr;
  }
  const bool res = a.epilogue == 2;   // EPI_RESID
  const LibKey key{a.M, a.N, a.K, a.lda, a.ldb, a.ldc, res ? a.ldr : 0, a.b_layout, a.out_dtype, have_ws ? 1 : 0,
                   a.bias ? 1 : 0, res ? 1 : 0, a.dtype};
  auto it = st.plans[dev].find(key);
  if (it != st.plans[dev].end()) return it->second.ok ? &it->second : nullptr;
  LibPlan& p = st.plans[dev][key];
  const hipDataType ct = a.out_dtype == MAECLIP_BF16 ? HIP_R_16BF : HIP_R_32F;
  bool ok = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  const hipblasOperation_t ta = a.b_layout == LAY_KC ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) == HIPBLAS_STATUS_SUCCESS;
  // first operand: op(B)^T, [N x K] after its op; second: A^T [K x M]; C / D: [N x M].
  // fp8 (maeclip_gemm_fp8): A e4m3 / e5m2, B e4m3, per-row A and per-column B
  // dequantisation scales as hipBLASLt's outer-vector scales (its first operand
  // is our B: N scales; its second our A: M scales)
  const bool f8 = a.dtype == MAECLIP_FP8_E4M3 || a.dtype == MAECLIP_FP8_E5M2;
  const hipDataType tB = f8 ? HIP_R_8F_E4M3 : HIP_R_16BF;
  const hipDataType tA = a.dtype == MAECLIP_FP8_E5M2 ? HIP_R_8F_E5M2 : f8 ? HIP_R_8F_E4M3 : HIP_R_16BF;
  if (a.b_layout == LAY_KC) ok = ok && hipblasLtMatrixLayoutCreate(&p.la, tB, a.K, a.N, a.ldb) == HIPBLAS_STATUS_SUCCESS;
  else ok = ok && hipblasLtMatrixLayoutCreate(&p.la, tB, a.N, a.K, a.ldb) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.lb, tA, a.K, a.M, a.lda) == HIPBLAS_STATUS_SUCCESS;
  if (f8) {
    const hipblasLtMatmulMatrixScale_t sm = HIPBLASLT_MATMUL_MATRIX_SCALE_OUTER_VEC_32F;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_A_SCALE_MODE, &sm, sizeof(sm)) == HIPBLAS_STATUS_SUCCESS;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_B_SCALE_MODE, &sm, sizeof(sm)) == HIPBLAS_STATUS_SUCCESS;
    const void* sp = scale_b;   // valid pointers for the heuristic; re-set at every call
    const void* sq = scale_a;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &sp, sizeof(sp)) == HIPBLAS_STATUS_SUCCESS;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &sq, sizeof(sq)) == HIPBLAS_STATUS_SUCCESS;
  }
  ok = ok && hipblasLtMatrixLayoutCreate(&p.lc, ct, a.N, a.M, a.ldc) == HIPBLAS_STATUS_SUCCESS;
  if (res) ok = ok && hipblasLtMatrixLayoutCreate(&p.lr, HIP_R_32F, a.N, a.M, a.ldr) == HIPBLAS_STATUS_SUCCESS;
  if (a.bias) {
    // bias per output column n = per row of the column-major D: hipBLASLt's BIAS epilogue
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) == HIPBLAS_STATUS_SUCCESS;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) ==
                   HIPBLAS_STATUS_SUCCESS;
    const void* bp = a.bias;   // a valid pointer for the heuristic; re-set at every call
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)) ==
                   HIPBLAS_STATUS_SUCCESS;
  }
  if (ok) {
    hipblasLtMatmulPreference_t pref = nullptr;
    const uint64_t wsb = have_ws ? (uint64_t)LIB_WS : 0;
    ok = hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)) ==
             HIPBLAS_STATUS_SUCCESS;
    hipblasLtMatmulHeuristicResult_t hr[LibPlan::NCAND];
    int n = 0;
    ok = ok && hipblasLtMatmulAlgoGetHeuristic(st.handle[dev], p.desc, p.la, p.lb, res ? p.lr : p.lc, p.lc, pref,
                                               tune_on() ? LibPlan::NCAND : 1, hr, &n) == HIPBLAS_STATUS_SUCCESS &&
         n > 0 && hr[0].state == HIPBLAS_STATUS_SUCCESS;
    if (ok) {
      p.algo = hr[0].algo;
      p.ws = hr[0].workspaceSize;
      ok = p.ws <= (size_t)wsb;
      for (int i = 0; i < n && i < LibPlan::NCAND; ++i)
        if (hr[i].state == HIPBLAS_STATUS_SUCCESS && hr[i].workspaceSize <= (size_t)wsb) {
          p.cand[p.ncand] = hr[i].algo;
          p.cand_ws[p.ncand++] = hr[i].workspaceSize;
        }
    }
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  }
  p.ok = ok;
  return ok ? &p : nullptr;
}

}  // namespace

namespace maeclip {

// GEMMs the vendor path takes: bf16 A (KC) and B, one batch, no split-K, no
// beta / column sums, K > 512; epilogue none (bf16 C) or the fp32 residual
// (fp32 R and C), each with or without bias. MAECLIP_GEMM_LIB: 0 = off,
// 2 = bf16-C launches only, 3 = every K (A/B)
bool lib_shape_ok(const maeclip_gemm_args& a) {
  const int mode = lib_mode();
  if (mode == 0) return false;
  if (a.a_layout != LAY_KC || a.colsum_partial || a.aux || a.aux_out) return false;
  if (a.beta != 0.f || a.batch != 1 || a.splitk > 1) return false;
  const bool plain = a.epilogue == 0 && !a.resid && a.out_dtype == MAECLIP_BF16;
  const bool res = a.epilogue == 2 && a.resid && a.out_dtype == MAECLIP_F32 && mode != 2;
  if (!plain && !res) return false;
  if (a.K <= 512 && mode != 3) return false;
  return a.M >= 256 && a.N >= 256;
}

bool gemm_lib_ok(const maeclip_gemm_args& a) { return a.dtype == MAECLIP_BF16 && lib_shape_ok(a); }

// fp8 operands (maeclip_gemm_fp8: KC x KC, B e4m3): the same epilogue forms
bool gemm_lib_fp8_ok(const maeclip_gemm_args& a) {
  if (a.dtype != MAECLIP_FP8_E4M3 && a.dtype != MAECLIP_FP8_E5M2) return false;
  const char* e = getenv("MAECLIP_GEMM_LIB_FP8");   // 0: fp8 GEMMs on the own kernel (A/B)
  if (e && *e == '0') return false;
  return a.b_layout == LAY_KC && lib_shape_ok(a);
}

int64_t gemm_lib_workspace(const maeclip_gemm_args& a) { return (gemm_lib_ok(a) || gemm_lib_fp8_ok(a)) ? LIB_WS : 0; }

// 0 = done, 1 = not taken (no plan for the shape: the caller falls back to the
// library's own kernels)
int gemm_lib(const maeclip_gemm_args& a, hipStream_t s, const float* scale_a, const float* scale_b) {
  const bool have_ws = a.workspace != nullptr;
  LibPlan* p = plan_for(a, have_ws, scale_a, scale_b);
  if (!p) return 1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const bool res = a.epilogue == 2;
  const float alpha = a.alpha, beta = res ? 1.f : 0.f;

  if (a.bias) {
    const void* bp = a.bias;
    MC_CHECK_ARG(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)) ==
                     HIPBLAS_STATUS_SUCCESS, "maeclip_gemm: hipBLASLt bias pointer");
  }
  if (scale_a) {
    const void* sp = scale_b;
    const void* sq = scale_a;
    MC_CHECK_ARG(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &sp, sizeof(sp)) ==
                         HIPBLAS_STATUS_SUCCESS &&
                     hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &sq, sizeof(sq)) ==
                         HIPBLAS_STATUS_SUCCESS,
                 "maeclip_gemm_fp8: hipBLASLt scale pointers");
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (!p->tuned && p->ncand > 1 && have_ws && (!res || (const void*)a.resid != a.C) &&
      hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
    // on this call's own operands (the final call below rewrites the outputs),
    // with the device drained first so that no other stream's kernels co-run
    hipEvent_t e0, e1;
    if (hipDeviceSynchronize() == hipSuccess && hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
      float best = 1e30f;
      int bi = 0;
      for (int i = 0; i < p->ncand; ++i) {
        bool good = true;
        for (int r = 0; r < 4 && good; ++r) {
          if (r == 1) good = hipEventRecord(e0, s) == hipSuccess;
          good = good && hipblasLtMatmul(state().handle[dev], p->desc, &alpha, a.B, p->la, a.A, p->lb, &beta,
                                         res ? (const void*)a.resid : a.C, res ? p->lr : p->lc, a.C, p->lc,
                                         &p->cand[i], (void*)a.workspace, p->cand_ws[i], s) == HIPBLAS_STATUS_SUCCESS;
        }
        float ms = 0.f;
        good = good && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
               hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
        if (good && ms < best) {
          best = ms;
          bi = i;
        }
      }
      p->algo = p->cand[bi];
      p->ws = p->cand_ws[bi];
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
    p->tuned = true;
  }
  const hipblasStatus_t r = hipblasLtMatmul(state().handle[dev], p->desc, &alpha, a.B, p->la, a.A, p->lb, &beta,
                                            res ? (const void*)a.resid : a.C, res ? p->lr : p->lc, a.C, p->lc, &p->algo,
                                            have_ws ? (void*)a.workspace : nullptr, p->ws, s);
  MC_CHECK_ARG(r == HIPBLAS_STATUS_SUCCESS, "maeclip_gemm: hipblasLtMatmul failed (status %d)", (int)r);
  return 0;
}

}  // namespace maeclip
