// Plain bf16 GEMMs on hipBLASLt (round 5): Y[M][N] (+)= X[M][K] W[N][K]^T (+ bias[N]), bf16
// operands, fp32 accumulation and output.  The recurrences' input projections and input
// gradients of the SeparateF0 encoder / decoders are plain GEMMs (no taps, no fused epilogue
// beyond the bias), M = 30 720 frames by N = 8H = 4 096 outputs, where the library's
// 256 x 256 macro tile with four 128 x 128 wave tiles and two global-read stages in flight
// (profiles/r5_gemm_library_anchor.txt) runs 1.3-1.6x the 128 x 128 implicit-GEMM kernel of
// gemm.hip; every fused / implicit-conv GEMM stays on gemm.hip.
//
// Row-major X (ldx), W (the GEMM engine's packed [Npad][Kp] bf16 rows, ldw = Kp) and Y (ldy) are
// the column-major matrices X^T (K x M), W^T (K x N) and Y^T (N x M); the call computes
// D = op(A) B with A = W^T (transposed: N x K), B = X^T, D = C = Y^T, and the bias epilogue
// adds bias[n] along D's rows.  One handle per device; one plan (descriptor, layouts, the
// heuristic's first algorithm) per shape, made on the first call -- the eager warm-up step, before
// any graph capture -- and reused, so a shape always runs the same kernel (deterministic: the
// algorithms these shapes get split no K).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "ensvs.h"

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

using Key = std::tuple<int, int, int, int, int, int, int, int>;  // dev M N K ldx ldw ldy bias

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<Key, Plan> g_plans;

#define BL_OK(x)                                 \
  do {                                           \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return 0; \
  } while (0)

// descriptor, layouts and algorithm of one shape (false: hipBLASLt has none)
bool make_plan(hipblasLtHandle_t h, int M, int N, int K, int ldx, int ldw, int ldy, bool bias,
               size_t max_ws, Plan& p) {
  BL_OK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  BL_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  BL_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    BL_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    BL_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt,
                                          sizeof(bt)));
  }
  BL_OK(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, ldw));
  BL_OK(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, ldx));
  BL_OK(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_32F, N, M, ldy));
  hipblasLtMatmulPreference_t pref;
  BL_OK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t mw = max_ws;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &mw,
                                        sizeof(mw));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.d, p.d, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return false;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  return true;
}

#undef BL_OK

}  // namespace

ENSVS_API int ensvs_blas_gemm(const void* x, int ldx, const void* w, int ldw, int M, int N, int K,
                              const float* bias, float* y, int ldy, int accum, void* ws,
                              long long ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldw < K || ldy < N) return ENSVS_E_SHAPE;
  if (!x || !w || !y || (ws_bytes > 0 && !ws) || ws_bytes < 0) return ENSVS_E_ARG;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return ENSVS_E_HIP;
  const Plan* plan = nullptr;
  hipblasLtHandle_t h = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto hi = g_handles.find(dev);
    if (hi == g_handles.end()) {
      if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return ENSVS_E_HIP;
      g_handles[dev] = h;
    } else {
      h = hi->second;
    }
    const Key key{dev, M, N, K, ldx, ldw, ldy, bias != nullptr};
    auto pi = g_plans.find(key);
    if (pi == g_plans.end()) {
      Plan p;
      if (!make_plan(h, M, N, K, ldx, ldw, ldy, bias != nullptr, (size_t)ws_bytes, p))
        return ENSVS_E_SHAPE;
      pi = g_plans.emplace(key, p).first;
    }
    plan = &pi->second;
    if ((long long)plan->ws > ws_bytes) return ENSVS_E_ARG;
    if (bias && hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER,
                                                &bias, sizeof(bias)) != HIPBLAS_STATUS_SUCCESS)
      return ENSVS_E_HIP;
    const float alpha = 1.f, beta = accum ? 1.f : 0.f;
    const hipblasStatus_t st =
        hipblasLtMatmul(h, plan->desc, &alpha, w, plan->a, x, plan->b, &beta, y, plan->d, y,
                        plan->d, &plan->algo, ws, (size_t)ws_bytes, (hipStream_t)stream);
    if (st != HIPBLAS_STATUS_SUCCESS) return ENSVS_E_HIP;
  }
  return ENSVS_OK;
}
