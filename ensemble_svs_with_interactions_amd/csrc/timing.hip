// Timing models: the MDN head / loss / most-probable selection
// (nnsvs/mdn.py) and the channel LayerNorm of MultiTrackVariancePredictor's conv stack
// (nnsvs/layers/layer_norm.py:10-35, nnsvs/model.py:1243-1260).  The convolutions and the
// linear heads run on the GEMM engine (gemm.hip).
//
// MDN arithmetic is per item = frame (or frame x output dim when dim_wise) over the G
// mixture components: a lane group of S = 2^ceil(log2 G) lanes (S <= 64) holds one item,
// lane g component g, and the max / log-sum-exp / first-argmax reductions over the mixture
// are xor-shuffles inside the wavefront (no LDS, no barriers).
//
// Layouts (frame rows m = b*T + t): log_pi [m][g] or, dim-wise, [m][g][d]; log_sigma and
// mu [m][g][d] (the reference's view(B, T, G, D)); targets [m][d] with row stride ldt.
#include "common.h"
#include "ensvs.h"

namespace {

__device__ __forceinline__ float grp_max(float v, int S) {
  for (int o = S >> 1; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float grp_sum(float v, int S) {
  for (int o = S >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int grp_min(int v, int S) {
  for (int o = S >> 1; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

struct Item {
  long long item, m;
  int d, g;
  bool act;
};

__device__ __forceinline__ Item item_of(long long items, int G, int D, int dim_wise, int S) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  Item it;
  it.item = t / S;
  it.g = (int)(t % S);
  it.m = dim_wise ? it.item / D : it.item;
  it.d = dim_wise ? (int)(it.item % D) : 0;
  it.act = it.item < items && it.g < G;
  return it;
}

__device__ __forceinline__ long long pi_idx(const Item& it, int G, int D, int dim_wise) {
  return dim_wise ? (it.m * G + it.g) * D + it.d : it.m * G + it.g;
}

// log_softmax over the mixture (mdn.py:64-70), in place: x - max - log(sum(exp(x - max)))
__global__ void mdn_log_softmax_kernel(float* __restrict__ lp, long long items, int G, int D,
                                       int dim_wise, int S) {
  const Item it = item_of(items, G, D, dim_wise, S);
  const long long i = pi_idx(it, G, D, dim_wise);
  const float a = it.act ? lp[i] : -INFINITY;
  const float mx = grp_max(a, S);
  const float s = grp_sum(it.act ? expf(a - mx) : 0.f, S);
  if (it.act) lp[i] = (a - mx) - logf(s);
}

// its backward, in place on g: g - exp(y) * sum(g)
__global__ void mdn_log_softmax_bwd_kernel(const float* __restrict__ y, float* __restrict__ g,
                                           long long items, int G, int D, int dim_wise, int S) {
  const Item it = item_of(items, G, D, dim_wise, S);
  const long long i = pi_idx(it, G, D, dim_wise);
  const float gv = it.act ? g[i] : 0.f;
  const float s = grp_sum(gv, S);
  if (it.act) g[i] = gv - expf(y[i]) * s;
}

constexpr float LOG_SQRT_2PI = 0.91893853320467274f;  // math.log(math.sqrt(2 * math.pi))

// mdn_loss (mdn.py:78-154) per item, reduce=False: loss = -logsumexp_g(s_g),
// s_g = max(log_pi, lp_min) + sum_d NormalLogProb(clip5(target - mu); exp(max(ls, ls_min))).
// With gloss: the gradients w.r.t. log_pi, log_sigma, mu of sum(gloss * loss).
__global__ void mdn_loss_kernel(const float* __restrict__ lp, const float* __restrict__ ls,
                                const float* __restrict__ mu, const float* __restrict__ tgt,
                                int ldt, long long items, int G, int D, int dim_wise, int S,
                                float lp_min, float ls_min, float* __restrict__ loss,
                                const float* __restrict__ gloss, float* __restrict__ dlp,
                                float* __restrict__ dls, float* __restrict__ dmu) {
  const Item it = item_of(items, G, D, dim_wise, S);
  const int d0 = dim_wise ? it.d : 0, d1 = dim_wise ? it.d + 1 : D;
  const long long pi = pi_idx(it, G, D, dim_wise);
  float s = -INFINITY, lpv = 0.f;
  if (it.act) {
    lpv = lp[pi];
    float acc = 0.f;
    for (int d = d0; d < d1; ++d) {
      const long long j = (it.m * G + it.g) * D + d;
      const float sc = expf(fmaxf(ls[j], ls_min));
      const float edge = 5.f * sc;
      float c = tgt[it.m * ldt + d] - mu[j];
      c = c > edge ? edge : c;
      c = c < -edge ? -edge : c;
      acc += -(c * c) / (2.f * (sc * sc)) - logf(sc) - LOG_SQRT_2PI;
    }
    s = acc + fmaxf(lpv, lp_min);
  }
  const float mx = grp_max(s, S);
  const float lse = logf(grp_sum(it.act ? expf(s - mx) : 0.f, S)) + mx;
  if (it.act && it.g == 0 && loss) loss[it.item] = -lse;
  if (!gloss || !it.act) return;
  const float ds = -gloss[it.item] * expf(s - lse);
  dlp[pi] = lpv >= lp_min ? ds : 0.f;
  for (int d = d0; d < d1; ++d) {
    const long long j = (it.m * G + it.g) * D + d;
    const float lsr = ls[j];
    const float sc = expf(fmaxf(lsr, ls_min));
    const float edge = 5.f * sc, var = sc * sc;
    const float c0 = tgt[it.m * ldt + d] - mu[j];
    const float c1 = c0 > edge ? edge : c0;
    const float c2 = c1 < -edge ? -edge : c1;
    const float dc2 = ds * (-c2 / var);
    float dsc = (ds * (c2 * c2) / (2.f * var * var)) * 2.f * sc - ds / sc;
    float dedge = 0.f, dc1 = dc2, dc0;
    if (c1 < -edge) {
      dedge -= dc2;
      dc1 = 0.f;
    }
    if (c0 > edge) {
      dedge += dc1;
      dc0 = 0.f;
    } else {
      dc0 = dc1;
    }
    dsc += 5.f * dedge;
    dls[j] = lsr >= ls_min ? dsc * sc : 0.f;
    dmu[j] = -dc0;
  }
}

// mdn_get_most_probable_sigma_and_mu (mdn.py:167-212): k = first argmax_g log_pi;
// sigma[m][d] = exp(log_sigma[m][k][d]), mu_out[m][d] = mu[m][k][d]
__global__ void mdn_most_probable_kernel(const float* __restrict__ lp, const float* __restrict__ ls,
                                         const float* __restrict__ mu, long long items, int G,
                                         int D, int dim_wise, int S, float* __restrict__ sigma,
                                         float* __restrict__ mu_out) {
  const Item it = item_of(items, G, D, dim_wise, S);
  const float v = it.act ? lp[pi_idx(it, G, D, dim_wise)] : -INFINITY;
  const float mx = grp_max(v, S);
  const int k = grp_min(it.act && v == mx ? it.g : (1 << 30), S);
  if (!it.act || it.g != k) return;
  const int d0 = dim_wise ? it.d : 0, d1 = dim_wise ? it.d + 1 : D;
  for (int d = d0; d < d1; ++d) {
    const long long j = (it.m * G + k) * D + d;
    sigma[it.m * D + d] = expf(ls[j]);
    mu_out[it.m * D + d] = mu[j];
  }
}

// ------------------------------------------------------------ LayerNorm
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wavefront per frame row, channels strided over the 64 lanes
__global__ __launch_bounds__(256) void layer_norm_fwd_kernel(
    const float* __restrict__ x, int ldx, long long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ y, int ldy,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + row * ldx;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  const float mean = wave_sum(s) / C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = xr[c] - mean;
    v = fmaf(d, d, v);
  }
  const float rstd = 1.f / sqrtf(wave_sum(v) / C + eps);
  float* yr = y + row * ldy;
  for (int c = lane; c < C; c += 64) yr[c] = (xr[c] - mean) * rstd * gamma[c] + beta[c];
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma;  dyxhat = dy * xhat
// (its column sums are the gamma gradient, the column sums of dy the beta gradient)
__global__ __launch_bounds__(256) void layer_norm_bwd_kernel(
    const float* __restrict__ dy, int lddy, const float* __restrict__ x, int ldx, long long M,
    int C, const float* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, float* __restrict__ dx, int lddx,
    float* __restrict__ dyxhat) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float mean = mean_in[row], rstd = rstd_in[row];
  const float* xr = x + row * ldx;
  const float* dr = dy + row * lddy;
  float a = 0.f, b = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float xh = (xr[c] - mean) * rstd;
    const float g = dr[c] * gamma[c];
    a += g;
    b = fmaf(g, xh, b);
    dyxhat[row * C + c] = dr[c] * xh;
  }
  a = wave_sum(a) / C;
  b = wave_sum(b) / C;
  for (int c = lane; c < C; c += 64) {
    const float xh = (xr[c] - mean) * rstd;
    dx[row * lddx + c] = rstd * (dr[c] * gamma[c] - a - xh * b);
  }
}

int group_size(int G) {
  int S = 1;
  while (S < G) S <<= 1;
  return S;
}

}  // namespace

// =================================================================== C ABI

#define MDN_LAUNCH(kernel, ...)                                                          \
  do {                                                                                   \
    if (M <= 0 || G <= 0 || G > 64 || D <= 0) return ENSVS_E_SHAPE;                      \
    const int S = group_size(G);                                                         \
    const long long items = dim_wise ? M * D : M;                                        \
    const long long threads = items * S;                                                 \
    hipLaunchKernelGGL(kernel, dim3((int)((threads + 255) / 256)), dim3(256), 0,         \
                       (hipStream_t)stream, __VA_ARGS__);                                \
    ENSVS_CHECK_LAUNCH();                                                                \
    return ENSVS_OK;                                                                     \
  } while (0)

ENSVS_API int ensvs_mdn_log_softmax(float* lp, long long M, int G, int D, int dim_wise,
                                    void* stream) {
  MDN_LAUNCH(mdn_log_softmax_kernel, lp, items, G, D, dim_wise, S);
}

ENSVS_API int ensvs_mdn_log_softmax_bwd(const float* y, float* g, long long M, int G, int D,
                                        int dim_wise, void* stream) {
  MDN_LAUNCH(mdn_log_softmax_bwd_kernel, y, g, items, G, D, dim_wise, S);
}

ENSVS_API int ensvs_mdn_loss(const float* lp, const float* ls, const float* mu, const float* tgt,
                             int ldt, long long M, int G, int D, int dim_wise, float lp_min,
                             float ls_min, float* loss, const float* gloss, float* dlp,
                             float* dls, float* dmu, void* stream) {
  if (gloss && (!dlp || !dls || !dmu)) return ENSVS_E_ARG;
  MDN_LAUNCH(mdn_loss_kernel, lp, ls, mu, tgt, ldt, items, G, D, dim_wise, S, lp_min, ls_min,
             loss, gloss, dlp, dls, dmu);
}

ENSVS_API int ensvs_mdn_most_probable(const float* lp, const float* ls, const float* mu,
                                      long long M, int G, int D, int dim_wise, float* sigma,
                                      float* mu_out, void* stream) {
  MDN_LAUNCH(mdn_most_probable_kernel, lp, ls, mu, items, G, D, dim_wise, S, sigma, mu_out);
}

ENSVS_API int ensvs_layer_norm_fwd(const float* x, int ldx, long long M, int C, const float* gamma,
                                   const float* beta, float eps, float* y, int ldy, float* mean,
                                   float* rstd, void* stream) {
  if (M <= 0 || C <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(layer_norm_fwd_kernel, dim3((int)((M + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, M, C, gamma, beta, eps, y, ldy, mean, rstd);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_layer_norm_bwd(const float* dy, int lddy, const float* x, int ldx, long long M,
                                   int C, const float* gamma, const float* mean,
                                   const float* rstd, float* dx, int lddx, float* dyxhat,
                                   void* stream) {
  if (M <= 0 || C <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(layer_norm_bwd_kernel, dim3((int)((M + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, dy, lddy, x, ldx, M, C, gamma, mean, rstd, dx, lddx,
                     dyxhat);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// ---------------------------------------------------------------- masked mean of the loss
// loss.masked_select(mask).mean() of the timing train step (bin/train_multitrack.py:113-121):
// per-block (sum, count) partials, then one block reduces them in double; out = {mean, count}.
// The backward spreads g / count over the selected items (zeros elsewhere).
namespace {
constexpr int MM_THREADS = 256, MM_MAX_BLOCKS = 512;

__global__ __launch_bounds__(MM_THREADS) void masked_sum_kernel(
    const float* __restrict__ x, const unsigned char* __restrict__ m, long long n,
    float* __restrict__ part) {
  __shared__ float rs[MM_THREADS], rc[MM_THREADS];
  float s = 0.f, c = 0.f;
  for (long long i = blockIdx.x * (long long)MM_THREADS + threadIdx.x; i < n;
       i += (long long)gridDim.x * MM_THREADS) {
    const bool on = m[i] != 0;
    s += on ? x[i] : 0.f;
    c += on ? 1.f : 0.f;
  }
  rs[threadIdx.x] = s;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int st = MM_THREADS / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      rs[threadIdx.x] += rs[threadIdx.x + st];
      rc[threadIdx.x] += rc[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = rs[0];
    part[2 * blockIdx.x + 1] = rc[0];
  }
}

__global__ __launch_bounds__(MM_THREADS) void masked_mean_final_kernel(
    const float* __restrict__ part, int nb, float* __restrict__ out) {
  __shared__ double rs[MM_THREADS], rc[MM_THREADS];
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < nb; i += MM_THREADS) {
    s += part[2 * i];
    c += part[2 * i + 1];
  }
  rs[threadIdx.x] = s;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int st = MM_THREADS / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      rs[threadIdx.x] += rs[threadIdx.x + st];
      rc[threadIdx.x] += rc[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (float)(rs[0] / rc[0]);  // empty selection: 0/0 = nan, as torch's mean
    out[1] = (float)rc[0];
  }
}

__global__ void masked_mean_bwd_kernel(const unsigned char* __restrict__ m, long long n,
                                       const float* __restrict__ g,
                                       const float* __restrict__ fwd_out,
                                       float* __restrict__ dx) {
  const float v = g[0] / fwd_out[1];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dx[i] = m[i] ? v : 0.f;
}
}  // namespace

ENSVS_API int ensvs_masked_mean(const float* x, const unsigned char* mask, long long n,
                                float* part, float* out, void* stream) {
  if (n < 0) return ENSVS_E_SHAPE;
  const int nb = (int)std::max(1LL, std::min<long long>(MM_MAX_BLOCKS, (n + 4095) / 4096));
  hipLaunchKernelGGL(masked_sum_kernel, dim3(nb), dim3(MM_THREADS), 0, (hipStream_t)stream, x,
                     mask, n, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(masked_mean_final_kernel, dim3(1), dim3(MM_THREADS), 0,
                     (hipStream_t)stream, part, nb, out);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_masked_mean_bwd(const unsigned char* mask, long long n, const float* gout,
                                    const float* fwd_out, float* dx, void* stream) {
  if (n <= 0) return n == 0 ? ENSVS_OK : ENSVS_E_SHAPE;
  const int nb = (int)std::min<long long>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(masked_mean_bwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, mask,
                     n, gout, fwd_out, dx);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
