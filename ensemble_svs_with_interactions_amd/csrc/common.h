// Shared definitions for the ensvs HIP kernels (gfx950 / CDNA4 only).
//
// Layout convention for every activation tensor on the path: channels-last
// frame rows, i.e. element (b, t, c) lives at  base + (b*T + t)*ld + c, with
// the row stride `ld` (floats) chosen by the host.  A "frame row" is the
// unit that the MFMA GEMMs tile over (M dimension), so HBM reads along the
// frame axis are 16-byte vector loads of contiguous channels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ENSVS_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

enum {
  ENSVS_OK = 0,
  ENSVS_E_SHAPE = 1,
  ENSVS_E_DTYPE = 2,
  ENSVS_E_HIP = 3,
  ENSVS_E_ARG = 4,
};

enum { PAD_ZERO = 0, PAD_REFLECT = 1, PAD_REPLICATE = 2 };
enum { DT_F32 = 0, DT_BF16 = 1 };

#define ENSVS_CHECK_LAUNCH()                               \
  do {                                                     \
    hipError_t _e = hipGetLastError();                     \
    if (_e != hipSuccess) return ENSVS_E_HIP;              \
  } while (0)

// Four fp32 values rounded to bf16 (nearest even) as one 8-B store: the rounding the GEMMs
// apply to fp32 operands, so a copy written here is the operand they would have staged.
__device__ __forceinline__ void store_bf16x4(__bf16* p, f32x4 v) {
  *(bf16x4*)p = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

// PyTorch ReflectionPad1d index map (valid for |pad| < n).
__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

// Map a source frame index under the given padding mode; returns -1 when the
// frame reads as zero.  Branch-free (selects): lanes of a wave hold different
// frames, and a divergent branch here sits between the staging loads.
__device__ __forceinline__ int pad_src(int s, int n, int mode) {
  const int refl = reflect_idx(s, n);
  const int repl = s < 0 ? 0 : n - 1;
  const int outside = mode == PAD_ZERO ? -1 : (mode == PAD_REFLECT ? refl : repl);
  return (s >= 0 && s < n) ? s : outside;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Fast gated-activation math for GEMM epilogues: hardware v_exp_f32 / v_rcp_f32 (about
// 1 ulp each) instead of IEEE division and libm tanhf (the DiffNet gate epilogue was
// VALU-bound on them).  tanh uses an odd polynomial below |x| = 1/16, where (1 - e)/(1 + e)
// would cancel, and saturates past |x| = 15.
__device__ __forceinline__ float fexpn_(float x) {  // exp(-x)
  return __builtin_amdgcn_exp2f(-1.44269504088896341f * x);
}
__device__ __forceinline__ float fsigmoid_(float x) {
  return __builtin_amdgcn_rcpf(1.f + fexpn_(x));
}
__device__ __forceinline__ float ftanh_(float x) {
  const float xc = fminf(fmaxf(x, -15.f), 15.f);
  const float e = fexpn_(2.f * xc);
  const float big = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  const float x2 = x * x;
  const float small = x * (1.f + x2 * (-0.333333333f + x2 * 0.133333333f));
  return fabsf(x) < 0.0625f ? small : big;
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// whether persistent recurrence workgroups reserve their CU's LDS (lstm.hip)
int ensvs_rec_exclusive();
