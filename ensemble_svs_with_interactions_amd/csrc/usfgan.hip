// uSFGAN vocoder (synthesis path): the memory-bound kernels
// around the generator's convolutions.  Every convolution of the generator
// (conv_in, periodicity estimator, residual blocks, conv_last) runs on the MFMA
// implicit-GEMM engine of gemm.hip, where the adaptive blocks' pitch-dependent
// past/future taps are gathered inside the operand staging (no index tensors).
//
//   weight_norm   nn.utils.weight_norm folding w = v * (g / ||v||)     (generator.py:524-544)
//   usf_upsample  nearest x s + Conv2d(1,1,(1,2s+1)) along time          (upsample.py:15-44,111-128)
//   usf_dfactor   dilated_factor + repeat(hop)                           (features.py:56-75,
//                                                                          usfgan/__init__.py:50-58)
//   usf_source    SignalGenerator sine + noise with an fp64 phase scan   (features.py:112-164)
//   usf_mix       h = a h, n = (1 - a) n, s = h + n                     (generator.py:505-508)
//
// Layout: channels-last sample rows, element (b, i, c) at (b*L + i)*ld + c.
#include "common.h"
#include "ensvs.h"

namespace {

#define GRID_LOOP(i, n) \
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); \
       i += (long long)gridDim.x * blockDim.x)

inline int grid_for(long long n) { return (int)std::min<long long>(8192, (n + 255) / 256); }

// One block per output row n: w[n*sn + k*sk] = v[n][k] * (g[n] / ||v[n][:]||)
// (torch._weight_norm(v, g, 0)); a plain copy when g is null.
__global__ __launch_bounds__(256) void weight_norm_kernel(const float* __restrict__ g,
                                                          const float* __restrict__ v, int K,
                                                          float* __restrict__ w, long long sn,
                                                          long long sk) {
  __shared__ float red[256];
  const int n = blockIdx.x;
  const float* vr = v + (long long)n * K;
  float scale = 1.f;
  if (g) {
    float s = 0.f;
    for (int k = threadIdx.x; k < K; k += 256) s = fmaf(vr[k], vr[k], s);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
      __syncthreads();
    }
    scale = g[n] / sqrtf(red[0]);
  }
  for (int k = threadIdx.x; k < K; k += 256) w[n * sn + k * sk] = vr[k] * scale;
}

// y[b][u][c] = sum_k w[k] * up(u + k - s), k < 2s+1, with up(v) = x[b][src(v)][c] for
// 0 <= v < Tin*s (else 0: the Conv2d's zero padding) and src(v) = min(floor(float(v) *
// inv_s), Tin - 1) (F.interpolate(scale_factor=s, mode="nearest"): float(1/s) scale).
// Channels C..ld-1 of y are written as 0 so the GEMMs may read whole 16-B quads.
__global__ void usf_upsample_kernel(const float* __restrict__ x, int ld, int Tin, int C, int s,
                                    float inv_s, const float* __restrict__ w,
                                    float* __restrict__ y, long long total) {
  const int Tout = Tin * s;
  GRID_LOOP(i, total) {
    const int c = (int)(i % ld);
    const long long r = i / ld;
    const long long b = r / Tout;
    const int u = (int)(r - b * Tout);
    float acc = 0.f;
    if (c < C) {
      for (int k = 0; k <= 2 * s; ++k) {
        const int v = u + k - s;
        if (v < 0 || v >= Tout) continue;
        const int src = min((int)floorf(__fmul_rn((float)v, inv_s)), Tin - 1);
        acc = fmaf(w[k], x[(b * Tin + src) * ld + c], acc);
      }
    }
    y[i] = acc;
  }
}

// d[b*L + i] = float((fs / f) / dense), f = f0[b][i / hop] (f0 == 0 -> float(fs / dense)),
// numpy float64 arithmetic of dilated_factor followed by the float32 tensor cast.
__global__ void usf_dfactor_kernel(const float* __restrict__ f0, int T, int hop, double fs,
                                   double dense, float* __restrict__ d, long long total) {
  const long long L = (long long)T * hop;
  GRID_LOOP(i, total) {
    const long long b = i / L;
    const int t = (int)((i - b * L) / hop);
    float f = f0[b * T + t];
    if (f == 0.f) f = (float)(fs / dense);
    d[i] = (float)((fs / (double)f) / dense);
  }
}

// --------------------------------------------------------------- sine source
// rad(i) = (f0[src(i)] / fs) mod 1 in float32, src(i) = min(floor(float(i) * scale), T - 1)
// with scale = float(T) / float(L) (F.interpolate(size=L), mode nearest).  The phase is
// torch.cumsum of rad, which on the CPU accumulates float32 inputs in double and rounds each
// prefix to float32: here per-chunk fp64 sums, an fp64 scan of the chunk sums and an fp64
// in-chunk scan, rounded once per sample.
constexpr int SRC_CHUNK = 2048;  // samples per block: 256 threads x 8

__device__ __forceinline__ int src_frame(int i, float scale, int T) {
  return min((int)floorf(__fmul_rn((float)i, scale)), T - 1);
}

__device__ __forceinline__ float rad_of(float f, float fs) {
  float m = fmodf(__fdiv_rn(f, fs), 1.f);  // torch.remainder with divisor 1
  if (m < 0.f) m += 1.f;
  return m;
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) sh[threadIdx.x] += sh[threadIdx.x + st];
    __syncthreads();
  }
  return sh[0];
}

__global__ __launch_bounds__(256) void usf_phase_partial_kernel(const float* __restrict__ f0,
                                                                int T, int L, float scale,
                                                                float fs, int nch,
                                                                double* __restrict__ part) {
  __shared__ double sh[256];
  const int ch = blockIdx.x, b = blockIdx.y;
  const float* f = f0 + (long long)b * T;
  double s = 0.0;
  for (int k = threadIdx.x; k < SRC_CHUNK; k += 256) {
    const int i = ch * SRC_CHUNK + k;
    if (i < L) s += (double)rad_of(f[src_frame(i, scale, T)], fs);
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[(long long)b * nch + ch] = s;
}

// exclusive scan of the chunk sums, one thread per sequence (nch is small: L / 2048)
__global__ void usf_phase_scan_kernel(double* __restrict__ part, int nch, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double acc = 0.0;
  for (int c = 0; c < nch; ++c) {
    const double v = part[(long long)b * nch + c];
    part[(long long)b * nch + c] = acc;
    acc += v;
  }
}

// out[row][0] = vuv*sin(phase*2*pi)*sine_amp + sine_noise*(vuv*na + (1-vuv)*na/3),
// out[row][1] = noise   (SignalGenerator order: ["sine", "noise"], features.py:113-126)
__global__ __launch_bounds__(256) void usf_source_kernel(
    const float* __restrict__ f0, int T, int L, float scale, float fs, float sine_amp,
    float noise_amp, const double* __restrict__ part, int nch,
    const float* __restrict__ sine_noise, const float* __restrict__ noise,
    float* __restrict__ out, int ldo) {
  __shared__ double sh[256];
  const int ch = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const float* f = f0 + (long long)b * T;
  const int i0 = ch * SRC_CHUNK + tid * 8;
  float fv[8], r[8];
  double tsum = 0.0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int i = i0 + e;
    fv[e] = i < L ? f[src_frame(i, scale, T)] : 0.f;
    r[e] = i < L ? rad_of(fv[e], fs) : 0.f;
    tsum += (double)r[e];
  }
  sh[tid] = tsum;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {  // inclusive scan of the thread sums
    const double v = tid >= off ? sh[tid - off] : 0.0;
    __syncthreads();
    sh[tid] += v;
    __syncthreads();
  }
  double acc = part[(long long)b * nch + ch] + (tid > 0 ? sh[tid - 1] : 0.0);
  constexpr float PI_F = 3.14159265358979323846f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int i = i0 + e;
    if (i >= L) break;
    acc += (double)r[e];
    const float ph = (float)acc;
    const float vuv = fv[e] > 0.f ? 1.f : 0.f;
    const float sine = vuv * sinf(__fmul_rn(__fmul_rn(ph, 2.f), PI_F)) * sine_amp;
    const float amp = vuv * noise_amp + (1.f - vuv) * noise_amp / 3.f;
    const long long row = (long long)b * L + i;
    out[row * ldo] = sine + sine_noise[row] * amp;
    out[row * ldo + 1] = noise[row];
  }
}

__global__ void usf_mix_kernel(const float* __restrict__ a, float* __restrict__ h,
                               float* __restrict__ n, float* __restrict__ s, long long total,
                               int keep) {
  GRID_LOOP(i, total) {
    const float av = a[i];
    const float hv = av * h[i];
    const float nv = (1.f - av) * n[i];
    s[i] = hv + nv;
    if (keep) {
      h[i] = hv;
      n[i] = nv;
    }
  }
}

}  // namespace

// =================================================================== C ABI

ENSVS_API int ensvs_weight_norm(const float* g, const float* v, int N, int K, float* w,
                                long long sn, long long sk, void* stream) {
  if (N <= 0 || K <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(weight_norm_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, g, v, K, w,
                     sn, sk);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_usf_upsample(const float* x, int ld, int B, int Tin, int C, int s,
                                 float inv_s, const float* w, float* y, void* stream) {
  if (B <= 0 || Tin <= 0 || C <= 0 || C > ld || s <= 0) return ENSVS_E_SHAPE;
  const long long total = (long long)B * Tin * s * ld;
  hipLaunchKernelGGL(usf_upsample_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, x, ld, Tin, C, s, inv_s, w, y, total);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_usf_dfactor(const float* f0, int B, int T, int hop, double fs, double dense,
                                float* d, void* stream) {
  if (B <= 0 || T <= 0 || hop <= 0) return ENSVS_E_SHAPE;
  const long long total = (long long)B * T * hop;
  hipLaunchKernelGGL(usf_dfactor_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, f0, T, hop, fs, dense, d, total);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API long long ensvs_usf_source_workspace(int B, int T, int hop) {
  return (long long)B * cdiv((long long)T * hop, SRC_CHUNK);
}

ENSVS_API int ensvs_usf_source(const float* f0, int B, int T, int hop, float scale, float fs,
                               float sine_amp, float noise_amp, const float* sine_noise,
                               const float* noise, double* ws, float* out, int ldo,
                               void* stream) {
  const long long L = (long long)T * hop;
  if (B <= 0 || T <= 0 || hop <= 0 || L >= (1 << 24) || ldo < 2) return ENSVS_E_SHAPE;
  const int nch = cdiv(L, SRC_CHUNK);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(usf_phase_partial_kernel, dim3(nch, B), dim3(256), 0, st, f0, T, (int)L,
                     scale, fs, nch, ws);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(usf_phase_scan_kernel, dim3(cdiv(B, 64)), dim3(64), 0, st, ws, nch, B);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(usf_source_kernel, dim3(nch, B), dim3(256), 0, st, f0, T, (int)L, scale, fs,
                     sine_amp, noise_amp, ws, nch, sine_noise, noise, out, ldo);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_usf_mix(const float* a, float* h, float* n, float* s, long long total,
                            int keep, void* stream) {
  if (total <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(usf_mix_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, a,
                     h, n, s, total, keep);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
