// Post-acoustic feature processing of the synthesis path:
// nnsvs/gen.py postprocess_acoustic (:1314-1530) with gen_spsvs_static_features
// (:1899-2019), nnsvs/postfilters.py variance_scaling (:9-46), nnsvs/dsp.py lowpass_filter
// (:10-33, scipy.signal.butter + filtfilt), and the WORLD band-aperiodicity codec round trip
// that predict_waveform applies before uSFGAN (gen.py:1637-1670).
//
// Per-utterance arrays are small (T ~ 10^3..10^4 frames x 67 streams) and already in HBM
// after acoustic inference; these kernels keep them there (no host round trip between the
// acoustic model and the vocoder).  Features are frame rows [t * ld + c] (fp32); the
// reference runs these steps in float64 numpy where it does, and so do the kernels.
#include <algorithm>

#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ double bsum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < NT / 64; ++i) s += sh[i];
  return s;
}

// variance_scaling(gv, feats, offset, note_frame_indices): one block per column c >= offset.
// utt_mu / utt_gv are numpy float32 reductions (mean, var(ddof=0)) of the note frames; the
// scale sqrt(gv / utt_gv) and the affine map run in float64 on float32 operands as numpy's
// type promotion does (feats - utt_mu is a float32 subtraction).
__global__ __launch_bounds__(NT) void gv_scale_kernel(float* x, int ld, int T, int offset,
                                                      const unsigned char* note,
                                                      const double* gv) {
  __shared__ double sh[NT / 64];
  const int c = offset + blockIdx.x;
  double s = 0.0, n = 0.0;
  for (int t = threadIdx.x; t < T; t += NT)
    if (note[t]) {
      s += x[(long long)t * ld + c];
      n += 1.0;
    }
  s = bsum(s, sh);
  n = bsum(n, sh);
  if (n == 0.0) return;  // "if len(note_frame_indices) == 0: return feats"
  const float mu = (float)(s / n);
  double q = 0.0;
  for (int t = threadIdx.x; t < T; t += NT)
    if (note[t]) {
      const double d = (double)x[(long long)t * ld + c] - (double)mu;
      q += d * d;
    }
  q = bsum(q, sh);
  const float var = (float)(q / n);
  const double k = sqrt(gv[c] / (double)var);
  for (int t = threadIdx.x; t < T; t += NT)
    if (note[t]) {
      float* p = x + (long long)t * ld + c;
      const float d = *p - mu;
      *p = (float)(k * (double)d + (double)mu);
    }
}

// gen_spsvs_static_features, relative_f0 = False (gen.py:1988-1991, 2010-2016): f0 = lf0
// with f0[vuv < thr] = 0, exp then log of the non-zero frames (float32 numpy), then
// nnmnkwii.preprocessing.interp1d(kind="slinear"): frames <= 0 take the straight line between
// the neighbouring voiced frames, the ends hold the first / last voiced value.  Then
// + f0 shift (gen.py:1489-1491).  One block per track; frames in NT contiguous chunks, the
// voiced neighbours across chunks from a sequential pass over the NT chunk summaries.
// w: T floats of workspace (the thresholded track).
__global__ __launch_bounds__(NT) void world_lf0_kernel(float* lf0, int ldl, const float* vuv,
                                                       int ldv, int T, float thr, float shift,
                                                       float* w) {
  __shared__ int first_nz[NT], last_nz[NT], prev_nz[NT], next_nz[NT];
  const int chunk = (T + NT - 1) / NT;
  const int t0 = min(T, (int)threadIdx.x * chunk), t1 = min(T, t0 + chunk);
  int fnz = -1, lnz = -1;
  for (int t = t0; t < t1; ++t) {
    float f = lf0[(long long)t * ldl];
    if (vuv[(long long)t * ldv] < thr) f = 0.f;
    if (f != 0.f) {
      const float e = expf(f);
      f = e != 0.f ? logf(e) : 0.f;
    }
    w[t] = f;
    if (f > 0.f) {
      if (fnz < 0) fnz = t;
      lnz = t;
    }
  }
  first_nz[threadIdx.x] = fnz;
  last_nz[threadIdx.x] = lnz;
  __syncthreads();
  if (threadIdx.x == 0) {
    int p = -1;
    for (int i = 0; i < NT; ++i) {
      prev_nz[i] = p;
      if (last_nz[i] >= 0) p = last_nz[i];
    }
    int q = -1;
    for (int i = NT - 1; i >= 0; --i) {
      next_nz[i] = q;
      if (first_nz[i] >= 0) q = first_nz[i];
    }
  }
  __syncthreads();
  const int gfirst = first_nz[0] >= 0 ? first_nz[0] : next_nz[0];
  const int glast = last_nz[NT - 1] >= 0 ? last_nz[NT - 1] : prev_nz[NT - 1];
  if (gfirst < 0) {  // nothing voiced: interp1d returns its input
    for (int t = t0; t < t1; ++t) lf0[(long long)t * ldl] = w[t] + shift;
    return;
  }
  // knots: index 0 (value of the first voiced frame), every voiced frame, index T-1 (value
  // of the last voiced frame)
  const double vfirst = w[gfirst], vlast = w[glast];
  int prev = prev_nz[threadIdx.x];
  for (int t = t0; t < t1; ++t) {
    const float f = w[t];
    float v = f;
    if (t == 0) {
      v = (float)vfirst;
    } else if (t == T - 1) {
      v = (float)vlast;
    } else if (!(f > 0.f)) {
      int xl = prev, xr = -1;
      double yl, yr;
      if (xl <= 0) {
        xl = 0;
        yl = vfirst;
      } else {
        yl = w[xl];
      }
      for (int u = t + 1; u < t1; ++u)
        if (w[u] > 0.f) {
          xr = u;
          break;
        }
      if (xr < 0) xr = next_nz[threadIdx.x];
      if (xr < 0 || xr >= T - 1) {
        xr = T - 1;
        yr = vlast;
      } else {
        yr = w[xr];
      }
      const double a = (double)(t - xl) / (double)(xr - xl);
      v = (float)(yl * (1.0 - a) + yr * a);
    }
    if (f > 0.f) prev = t;
    lf0[(long long)t * ldl] = v + shift;
  }
}

// scipy.signal.filtfilt(b, a, x) with its defaults (padtype "odd", padlen 3 * max(len(a),
// len(b)), method "pad"): odd extension, lfilter with zi * first sample forward, again
// backwards, trimmed; float64 throughout (lfilter's direct form II transposed), one thread per
// channel.  Channels shorter than or equal to the lowpass_filter guard are left unchanged.
__global__ void filtfilt_kernel(float* x, int ld, int T, int C, const double* ba, int nb,
                                const double* zi, int padlen, int guard, double* work) {
#pragma clang fp contract(off)  // scipy's lfilter loop rounds every product and sum
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C || T <= guard) return;
  const double* b = ba;
  const double* a = ba + nb;
  const int n = T + 2 * padlen;
  double* e = work + (long long)c * n;
  // odd_ext is evaluated in the input's dtype (float32)
  const float x0 = x[c], xl = x[(long long)(T - 1) * ld + c];
  for (int i = 0; i < padlen; ++i) {
    e[i] = (double)(2.f * x0 - x[(long long)(padlen - i) * ld + c]);
    e[padlen + T + i] = (double)(2.f * xl - x[(long long)(T - 2 - i) * ld + c]);
  }
  for (int t = 0; t < T; ++t) e[padlen + t] = x[(long long)t * ld + c];
  double z[16];
  for (int pass = 0; pass < 2; ++pass) {
    const double s = pass == 0 ? e[0] : e[n - 1];
    for (int k = 0; k < nb - 1; ++k) z[k] = zi[k] * s;
    for (int j = 0; j < n; ++j) {
      const int i = pass == 0 ? j : n - 1 - j;
      const double xi = e[i];
      const double y = z[0] + b[0] * xi;
      for (int k = 0; k < nb - 2; ++k) z[k] = z[k + 1] + xi * b[k + 1] - y * a[k + 1];
      z[nb - 2] = xi * b[nb - 1] - y * a[nb - 1];
      e[i] = y;
    }
  }
  for (int t = 0; t < T; ++t) x[(long long)t * ld + c] = (float)e[padlen + t];
}

// The same filter for a compile-time coefficient count NB (the order-5 Butterworth of the
// recipe: NB = 6): state and coefficients in registers, the extended signal streamed through
// registers 16 samples at a time with the next chunk's loads issued before the current
// chunk's recursion -- the generic kernel keeps z in scratch (runtime-indexed) and pays a
// dependent memory round trip per sample (3.1 ms per call at T = 2 000).  The per-sample
// arithmetic is the generic kernel's, term for term (contraction off): the same bits.
// Up to 4 column groups of one feature matrix, each with its own filter, in one launch
// (blockIdx.y): the post-filter's lf0 / mgc / bap smoothing calls are independent and each
// is a latency-bound recursion on a few lanes, so they run side by side.
struct FFGroup {
  float* x;             // first column of the group
  const double* ba;     // b then a (NB each)
  const double* zi;     // lfilter_zi (NB - 1)
  double* work;         // C x (T + 2 padlen)
  int C, padlen, guard;
};
struct FFGroups {
  FFGroup g[4];
};

template <int NB>
__global__ void filtfilt_nb_kernel(FFGroups gs, int ld, int T) {
#pragma clang fp contract(off)
  constexpr int CH = 16;
  const FFGroup& G = gs.g[blockIdx.y];
  float* x = G.x;
  const double* ba = G.ba;
  const double* zi = G.zi;
  double* work = G.work;
  const int C = G.C, padlen = G.padlen, guard = G.guard;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C || T <= guard) return;
  double b[NB], a[NB], zi0[NB - 1];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    b[k] = ba[k];
    a[k] = ba[NB + k];
  }
#pragma unroll
  for (int k = 0; k < NB - 1; ++k) zi0[k] = zi[k];
  const int n = T + 2 * padlen;
  double* e = work + (long long)c * n;  // the forward pass's output
  const float x0 = x[c], xl = x[(long long)(T - 1) * ld + c];
  // sample i of the odd extension (evaluated in float32, as scipy's odd_ext on float input)
  auto ext = [&](int i) -> double {
    if (i < padlen) return (double)(2.f * x0 - x[(long long)(padlen - i) * ld + c]);
    if (i < padlen + T) return (double)x[(long long)(i - padlen) * ld + c];
    return (double)(2.f * xl - x[(long long)(T - 2 - (i - padlen - T)) * ld + c]);
  };
  // pass 0 reads the extension and writes e; pass 1 reads e backwards and writes the
  // trimmed result into x (the generic kernel's values, without its two copy loops)
#define FF_STEP(XI, Y)                                                                    \
  do {                                                                                    \
    const double xi_ = (XI);                                                              \
    Y = z[0] + b[0] * xi_;                                                                \
    _Pragma("unroll") for (int k = 0; k < NB - 2; ++k)                                    \
      z[k] = z[k + 1] + xi_ * b[k + 1] - Y * a[k + 1];                                    \
    z[NB - 2] = xi_ * b[NB - 1] - Y * a[NB - 1];                                          \
  } while (0)
  double z[NB - 1], cur[CH], nxt[CH];
  {
    const double s = ext(0);
#pragma unroll
    for (int k = 0; k < NB - 1; ++k) z[k] = zi0[k] * s;
#pragma unroll
    for (int q = 0; q < CH; ++q) cur[q] = q < n ? ext(q) : 0.0;
    for (int j0 = 0; j0 < n; j0 += CH) {
#pragma unroll
      for (int q = 0; q < CH; ++q) nxt[q] = j0 + CH + q < n ? ext(j0 + CH + q) : 0.0;
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        if (j0 + q >= n) break;
        double y;
        FF_STEP(cur[q], y);
        e[j0 + q] = y;
      }
#pragma unroll
      for (int q = 0; q < CH; ++q) cur[q] = nxt[q];
    }
  }
  {
    const double s = e[n - 1];
#pragma unroll
    for (int k = 0; k < NB - 1; ++k) z[k] = zi0[k] * s;
#pragma unroll
    for (int q = 0; q < CH; ++q) cur[q] = q < n ? e[n - 1 - q] : 0.0;
    for (int j0 = 0; j0 < n; j0 += CH) {
#pragma unroll
      for (int q = 0; q < CH; ++q) nxt[q] = j0 + CH + q < n ? e[n - 1 - (j0 + CH + q)] : 0.0;
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        if (j0 + q >= n) break;
        double y;
        FF_STEP(cur[q], y);
        const int t = n - 1 - (j0 + q) - padlen;
        if (t >= 0 && t < T) x[(long long)t * ld + c] = (float)y;
      }
#pragma unroll
      for (int q = 0; q < CH; ++q) cur[q] = nxt[q];
    }
  }
#undef FF_STEP
}

// bap clip to [-60, 0] (gen.py:1520-1522, band aperiodicity only) and the WORLD codec round
// trip of predict_waveform's uSFGAN branch (gen.py:1649-1670): DecodeAperiodicity turns a
// frame whose mean coded aperiodicity exceeds -0.5 into all (1 - 1e-12) (WORLD d4c.cpp
// CheckVUV), other frames into 10^(bap/20) on the FFT grid, whose band centres (multiples of
// 3 kHz) CodeAperiodicity reads back exactly; the clip to [0, 1] and the unvoiced bin-0 fill
// touch no band centre.  So: unvoiced-like frames -> 20 log10(1 - 1e-12), others unchanged.
__global__ void bap_post_kernel(float* bap, int ld, int T, int D, int clip, int codec) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  float* p = bap + (long long)t * ld;
  double m = 0.0;
  for (int d = 0; d < D; ++d) {
    float v = p[d];
    if (clip) v = fminf(fmaxf(v, -60.f), 0.f);
    p[d] = v;
    m += v;
  }
  if (codec && m / D > -0.5) {
    const float u = (float)(20.0 * log10(1.0 - 1e-12));
    for (int d = 0; d < D; ++d) p[d] = u;
  }
}

// sklearn scaler arithmetic on a float32 array with float64 statistics, column-wise and in
// place (numpy rounds each in-place op into float32): mode 0 x = (x * a) + b
// (StandardScaler.inverse_transform: a = scale_, b = mean_; MinMaxScaler.transform: a =
// scale_, b = min_), mode 1 x = (x - b) / a (StandardScaler.transform; MinMaxScaler
// .inverse_transform with b = min_, a = scale_).
__global__ void scale_cols_kernel(float* x, int ld, long long n, int C, const double* a,
                                  const double* b, int mode) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long t = e / C;
    const int c = (int)(e - t * C);
    float* p = x + t * ld + c;
    if (mode == 0) {
      const float u = (float)((double)*p * a[c]);
      *p = (float)((double)u + b[c]);
    } else {
      const float u = (float)((double)*p - b[c]);
      *p = (float)((double)u / a[c]);
    }
  }
}

// note[t] = score[t] > 0 (gen.py:1339-1340: GV on note frames, score = the linguistic
// features' pitch column)
__global__ void note_mask_kernel(const float* score, int lds, int T, unsigned char* note) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < T; t += gridDim.x * blockDim.x)
    note[t] = score[(long long)t * lds] > 0.f ? 1 : 0;
}

// f0[t] = exp(lf0[t]), 0 where vuv[t] < thr when zero_unvoiced (gen.py:1662-1666, sine_f0_type
// "f0"); expf: torch.exp's float32 arithmetic
__global__ void f0_from_lf0_kernel(const float* lf0, int ldl, const float* vuv, int ldv, int T,
                                   float thr, int zero_unvoiced, float* f0) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < T; t += gridDim.x * blockDim.x) {
    const float e = expf(lf0[(long long)t * ldl]);
    f0[t] = zero_unvoiced && vuv[(long long)t * ldv] < thr ? 0.f : e;
  }
}

}  // namespace

ENSVS_API int ensvs_note_mask(const float* score, int lds, int T, unsigned char* note,
                              void* stream) {
  if (T <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(note_mask_kernel, dim3(cdiv(T, 256)), dim3(256), 0, (hipStream_t)stream,
                     score, lds, T, note);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_f0_from_lf0(const float* lf0, int ldl, const float* vuv, int ldv, int T,
                                float thr, int zero_unvoiced, float* f0, void* stream) {
  if (T <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(f0_from_lf0_kernel, dim3(cdiv(T, 256)), dim3(256), 0, (hipStream_t)stream,
                     lf0, ldl, vuv, ldv, T, thr, zero_unvoiced, f0);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_scale_cols(float* x, int ld, int T, int C, const double* a, const double* b,
                               int mode, void* stream) {
  const long long n = (long long)T * C;
  if (n <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(scale_cols_kernel, dim3((int)std::min<long long>(4096, (n + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, x, ld, n, C, a, b, mode);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_gv_scale(float* x, int ld, int T, int D, int offset,
                             const unsigned char* note, const double* gv, void* stream) {
  if (T <= 0 || offset < 0 || offset >= D) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(gv_scale_kernel, dim3(D - offset), dim3(NT), 0, (hipStream_t)stream, x, ld,
                     T, offset, note, gv);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_world_lf0(float* lf0, int ldl, const float* vuv, int ldv, int T, float thr,
                              float shift, float* work, void* stream) {
  if (T <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(world_lf0_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, lf0, ldl, vuv,
                     ldv, T, thr, shift, work);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_filtfilt(float* x, int ld, int T, int C, const double* ba, int nb,
                             const double* zi, int padlen, int guard, double* work,
                             void* stream) {
  if (T <= 0 || C <= 0 || nb < 2 || nb > 17) return ENSVS_E_SHAPE;
  if (T > guard && T <= padlen) return ENSVS_E_SHAPE;  // filtfilt's own length check
  if (nb == 6) {
    FFGroups gs{};
    gs.g[0] = {x, ba, zi, work, C, padlen, guard};
    hipLaunchKernelGGL(filtfilt_nb_kernel<6>, dim3(cdiv(C, 64), 1), dim3(64), 0,
                       (hipStream_t)stream, gs, ld, T);
  } else
    hipLaunchKernelGGL(filtfilt_kernel, dim3(cdiv(C, 64)), dim3(64), 0, (hipStream_t)stream, x,
                       ld, T, C, ba, nb, zi, padlen, guard, work);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// ngroups (<= 4) independent ensvs_filtfilt calls on columns of one matrix (row stride ld, T
// rows) in one launch: group i filters cols[i] .. cols[i] + C[i] - 1 of x with ba[i] / zi[i]
// (nb = 6: order-5 Butterworth), workspace work[i] (C[i] x (T + 2 padlen[i]) doubles).
ENSVS_API int ensvs_filtfilt_multi(float* x, int ld, int T, int ngroups, const int* cols,
                                   const int* C, const double* const* ba, const double* const* zi,
                                   const int* padlen, const int* guard, double* const* work,
                                   void* stream) {
  if (T <= 0 || ngroups < 1 || ngroups > 4) return ENSVS_E_SHAPE;
  FFGroups gs{};
  int cmax = 1;
  for (int i = 0; i < ngroups; ++i) {
    if (C[i] <= 0 || (T > guard[i] && T <= padlen[i])) return ENSVS_E_SHAPE;
    gs.g[i] = {x + cols[i], ba[i], zi[i], work[i], C[i], padlen[i], guard[i]};
    cmax = std::max(cmax, C[i]);
  }
  hipLaunchKernelGGL(filtfilt_nb_kernel<6>, dim3(cdiv(cmax, 64), ngroups), dim3(64), 0,
                     (hipStream_t)stream, gs, ld, T);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_bap_post(float* bap, int ld, int T, int D, int clip, int codec,
                             void* stream) {
  if (T <= 0 || D <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(bap_post_kernel, dim3(cdiv(T, 256)), dim3(256), 0, (hipStream_t)stream, bap,
                     ld, T, D, clip, codec);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
