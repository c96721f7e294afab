// Plain bf16 GEMMs on hipBLASLt (round 5): Y[M][N] (+)= X[M][K] W[N][K]^T (+ bias[N]), bf16
// operands, fp32 accumulation and output.  The recurrences' input projections and input
// gradients of the SeparateF0 encoder / decoders are plain GEMMs (no taps, no fused epilogue
// beyond the bias), M = 30 720 frames by N = 8H = 4 096 outputs, where the library's
// 256 x 256 macro tile with four 128 x 128 wave tiles and two global-read stages in flight
// (profiles/r5_gemm_library_anchor.txt) runs 1.3-1.6x the 128 x 128 implicit-GEMM kernel of
// gemm.hip; every fused / implicit-conv GEMM and every weight gradient stays on gemm.hip.
//
// Row-major X (ldx), W (the GEMM engine's packed [Npad][Kp] bf16 rows, ldw = Kp) and Y (ldy) are
// the column-major matrices X^T (K x M), W^T (K x N) and Y^T (N x M); the call computes
// D = op(A) B with A = W^T (transposed: N x K), B = X^T, D = C = Y^T, and the bias epilogue
// adds bias[n] along D's rows.  One handle per device; one plan (descriptor, layouts, the
// heuristic's first algorithm) per shape, made on the first call -- the eager warm-up step, before
// any graph capture -- and reused, so a shape always runs the same kernel.
//
// Data-parallel grids only.  hipBLASLt's gfx950 kernels are stream-K ("_SK3_"): by default a
// persistent grid of ~one workgroup per CU walks the tiles and splits the last ones, whose
// owners wait for partial tiles of other workgroups.  Beside the cooperative recurrences --
// whose workgroups reserve whole CUs on other streams -- a waiting owner's producer may never
// become resident (a SeparateF0 step whose weight gradients ran on such a grid hung).  With
// TENSILE_STREAMK_DATA_PARALLEL=1 the same kernels launch one workgroup per tile and nothing
// waits (tools/blas_probe.py traces: 240-workgroup grids become 1 920 for the N = 4 096
// projections, at the same time).  The library sets it when it is loaded (unless the process
// set it), and makes no plan -- the caller keeps gemm.hip, ensvs_blas_supported says 0 -- when
// it is not "1".  Tensile reads it once, at the process's first hipBLASLt call: a process that
// ran hipBLASLt before loading this library and without the setting keeps stream-K grids.
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "ensvs.h"

namespace {

__attribute__((constructor)) void data_parallel_env() {
  setenv("TENSILE_STREAMK_DATA_PARALLEL", "1", 0);
}

bool data_parallel() {
  const char* v = getenv("TENSILE_STREAMK_DATA_PARALLEL");
  return v && strcmp(v, "1") == 0;
}

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
std::map<Key, bool> g_none;  // shapes without an algorithm

#define BL_OK(x)                                     \
  do {                                               \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return false; \
  } while (0)

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

// the plan of a shape (nullptr: none) and the device's handle; g_mu held
const Plan* find_plan(int M, int N, int K, int ldx, int ldw, int ldy, bool bias,
                      long long ws_bytes, hipblasLtHandle_t* hout) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipblasLtHandle_t h = nullptr;
  auto hi = g_handles.find(dev);
  if (hi == g_handles.end()) {
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    g_handles[dev] = h;
  } else {
    h = hi->second;
  }
  *hout = h;
  const Key key{dev, M, N, K, ldx, ldw, ldy, bias};
  auto pi = g_plans.find(key);
  if (pi != g_plans.end()) return &pi->second;
  if (g_none.count(key) || !data_parallel()) return nullptr;
  Plan p;
  if (!make_plan(h, M, N, K, ldx, ldw, ldy, bias, (size_t)ws_bytes, p)) {
    g_none[key] = true;
    return nullptr;
  }
  return &g_plans.emplace(key, p).first->second;
}

}  // namespace

ENSVS_API int ensvs_blas_supported(int M, int N, int K, int ldx, int ldw, int ldy, int bias,
                                   long long ws_bytes) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldw < K || ldy < N || ws_bytes < 0) return 0;
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h = nullptr;
  const Plan* p = find_plan(M, N, K, ldx, ldw, ldy, bias != 0, ws_bytes, &h);
  if (!h) return -ENSVS_E_HIP;
  return p && (long long)p->ws <= ws_bytes ? 1 : 0;
}

ENSVS_API int ensvs_blas_gemm(const void* x, int ldx, const void* w, int ldw, int M, int N, int K,
                              const float* bias, float* y, int ldy, int accum, void* ws,
                              long long ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldw < K || ldy < N) return ENSVS_E_SHAPE;
  if (!x || !w || !y || (ws_bytes > 0 && !ws) || ws_bytes < 0) return ENSVS_E_ARG;
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h = nullptr;
  const Plan* plan = find_plan(M, N, K, ldx, ldw, ldy, bias != nullptr, ws_bytes, &h);
  if (!h) return ENSVS_E_HIP;
  if (!plan) return ENSVS_E_SHAPE;
  if ((long long)plan->ws > ws_bytes) return ENSVS_E_ARG;
  if (bias && hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                              sizeof(bias)) != HIPBLAS_STATUS_SUCCESS)
    return ENSVS_E_HIP;
  const float alpha = 1.f, beta = accum ? 1.f : 0.f;
  if (hipblasLtMatmul(h, plan->desc, &alpha, w, plan->a, x, plan->b, &beta, y, plan->d, y, plan->d,
                      &plan->algo, ws, (size_t)ws_bytes, (hipStream_t)stream) != HIPBLAS_STATUS_SUCCESS)
    return ENSVS_E_HIP;
  return ENSVS_OK;
}
