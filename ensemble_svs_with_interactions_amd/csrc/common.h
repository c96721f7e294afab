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

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
