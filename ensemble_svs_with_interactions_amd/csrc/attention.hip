// Relative-position multi-head self-attention of the VITS-style Transformer encoder
// (nnsvs/transformer/attentions.py:22-214, used by nnsvs.model.TransformerEncoder,
// model.py:1540-1671), forward and backward, fp32; plus the encoder's frame-mask and
// reduction-factor helpers (model.py:1655-1660).
//
// Layout: Q / K / V are frame rows [(b*T + t)*ld + h*dk + d] (the 1x1 projections write
// them side by side); scores / probabilities are [(b*H + h)][T][T].
//   S  = (Q / sqrt(dk)) K^T                                  (bgemm)
//   S += (Q / sqrt(dk)) . ek[j - i + w]    for |j - i| <= w  (relative keys, heads share)
//   S  = -1e4 where i >= L_b or j >= L_b                      (masked_fill(mask == 0, -1e4))
//   P  = softmax_j(S);  Pd = P * keep                         (dropout, optional)
//   O  = Pd V + sum_{|j - i| <= w} Pd[i][j] ev[j - i + w]     (bgemm + relative values)
// The backward runs the transposed products on the same batched GEMM.  The dense 1x1
// projections around this (q/k/v/o, FFN convs) are MFMA GEMMs of gemm.hip.
#include <algorithm>

#include "common.h"

namespace {

constexpr int TB = 64, TK = 16;

struct BG {  // batched operand: element (z, r, c) at p + zb*sb + zh*sh + r*sr + c*sc
  const float* p;
  long long sb, sh, sr, sc;
};

// C[z](m, n) (=|+=) alpha * sum_k A[z](m, k) B[z](k, n),  z = zb * H + zh.
// 64 x 64 tile per 256 threads (4 x 4 outputs each), K staged through LDS 16 deep.
__global__ __launch_bounds__(256) void bgemm_kernel(BG A, BG B, float* C, long long csb,
                                                    long long csh, long long csr, long long csc,
                                                    int H, int M, int N, int K, float alpha,
                                                    int accum) {
  __shared__ float As[TK][TB + 4], Bs[TK][TB + 4];
  const int z = blockIdx.z, zb = z / H, zh = z % H;
  const int m0 = blockIdx.x * TB, n0 = blockIdx.y * TB;
  const float* a = A.p + zb * A.sb + zh * A.sh;
  const float* b = B.p + zb * B.sb + zh * B.sh;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  // tile loads walk the operand's contiguous axis fastest (coalescing)
  const bool a_kfast = A.sc == 1;
  const bool b_nfast = B.sc == 1;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += TK) {
#pragma unroll
    for (int it = 0; it < TB * TK / 256; ++it) {
      const int e = threadIdx.x + it * 256;
      int r, kk;
      if (a_kfast) { r = e / TK; kk = e % TK; } else { kk = e / TB; r = e % TB; }
      const int m = m0 + r, k = k0 + kk;
      As[kk][r] = (m < M && k < K) ? a[m * A.sr + k * A.sc] : 0.f;
      int c, kb;
      if (b_nfast) { kb = e / TB; c = e % TB; } else { c = e / TK; kb = e % TK; }
      const int n = n0 + c, k2 = k0 + kb;
      Bs[kb][c] = (n < N && k2 < K) ? b[k2 * B.sr + n * B.sc] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* c = C + zb * csb + zh * csh;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= N) continue;
      float* p = c + m * csr + n * csc;
      const float v = alpha * acc[i][j];
      *p = accum ? *p + v : v;
    }
  }
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

struct RowIdx {
  int i, b, h;
};
__device__ __forceinline__ RowIdx row_idx(long long row, int H, int T) {
  const long long bh = row / T;
  return {(int)(row - bh * T), (int)(bh / H), (int)(bh % H)};
}

// y = x / s (attentions.py:93, :100 divide the query, they do not multiply by 1/sqrt(dk))
__global__ void div_kernel(const float* x, int ldx, float* y, int ldy, long long M, int C,
                           float s) {
  const long long n = M * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / C;
    const int c = (int)(e - r * C);
    y[r * ldy + c] = x[r * ldx + c] / s;
  }
}

// One wavefront per score row (b, h, i): relative-key band (lane r forms qs_i . ek[r] and the
// band element j = i + r - w takes it by a lane shuffle), key/query mask, softmax.  S is
// overwritten by P; with a keep mask Pd = P * keep goes to its own buffer.
__global__ __launch_bounds__(256) void softmax_kernel(float* S, const float* qs, int ldq,
                                                      const float* ek, const long long* lens,
                                                      long long rows, int H, int T, int dk,
                                                      int w, const float* keep, float* Pd) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform
  const RowIdx ri = row_idx(row, H, T);
  float* s = S + row * T;
  const int L = (int)lens[ri.b];
  const float* q = qs + ((long long)ri.b * T + ri.i) * ldq + ri.h * dk;
  float rel = 0.f;
  if (lane <= 2 * w) {
    const float* e = ek + (long long)lane * dk;
    for (int d = 0; d < dk; ++d) rel = fmaf(q[d], e[d], rel);
  }
  float m = -INFINITY;
  for (int j0 = 0; j0 < T; j0 += 64) {
    const int j = j0 + lane;
    const int r = j - ri.i + w;
    const float rv = __shfl(rel, min(max(r, 0), 63));
    if (j < T) {
      float v = s[j];
      if (r >= 0 && r <= 2 * w) v += rv;
      if (ri.i >= L || j >= L) v = -1e4f;
      s[j] = v;
      m = fmaxf(m, v);
    }
  }
  m = wmax(m);
  float sum = 0.f;
  for (int j = lane; j < T; j += 64) {
    const float e = __expf(s[j] - m);
    s[j] = e;
    sum += e;
  }
  sum = wsum(sum);
  for (int j = lane; j < T; j += 64) {
    const float p = s[j] / sum;
    s[j] = p;
    if (keep) Pd[row * T + j] = p * keep[row * T + j];
  }
}

// O[(b*T + i)*ldo + h*dk + d] += sum_{|j - i| <= w} P[row][j] ev[j - i + w][d]
__global__ void relv_kernel(const float* P, const float* ev, float* O, int ldo, long long rows,
                            int H, int T, int dk, int w) {
  const long long n = rows * dk;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long row = e / dk;
    const int d = (int)(e - row * dk);
    const RowIdx ri = row_idx(row, H, T);
    float acc = 0.f;
    for (int r = 0; r <= 2 * w; ++r) {
      const int j = ri.i + r - w;
      if (j >= 0 && j < T) acc = fmaf(P[row * T + j], ev[(long long)r * dk + d], acc);
    }
    O[((long long)ri.b * T + ri.i) * ldo + ri.h * dk + d] += acc;
  }
}

// D[row][i + r - w] += vec_i . tab[r]   (one wave per row; lanes r <= 2w form the dots)
__global__ __launch_bounds__(256) void band_dot_kernel(float* D, const float* vec, int ldv,
                                                       const float* tab, long long rows, int H,
                                                       int T, int dk, int w) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const RowIdx ri = row_idx(row, H, T);
  const int j = ri.i + lane - w;
  if (lane > 2 * w || j < 0 || j >= T) return;
  const float* v = vec + ((long long)ri.b * T + ri.i) * ldv + ri.h * dk;
  const float* e = tab + (long long)lane * dk;
  float dot = 0.f;
  for (int d = 0; d < dk; ++d) dot = fmaf(v[d], e[d], dot);
  D[row * T + j] += dot;
}

// part[chunk][r][d] = sum_{rows of chunk} A[row][i + r - w] * X_i[d]
// (gradient of a relative table shared by the heads: the rows of every (b, h) contribute)
__global__ void band_table_grad_kernel(const float* A, const float* X, int ldx, long long rows,
                                       int H, int T, int dk, int w, long long chunk,
                                       float* part) {
  const int r = blockIdx.x, c = blockIdx.y;
  const long long r0 = (long long)c * chunk, r1 = min(rows, r0 + chunk);
  for (int d = threadIdx.x; d < dk; d += blockDim.x) {
    float acc = 0.f;
    for (long long row = r0; row < r1; ++row) {
      const RowIdx ri = row_idx(row, H, T);
      const int j = ri.i + r - w;
      if (j < 0 || j >= T) continue;
      acc = fmaf(A[row * T + j], X[((long long)ri.b * T + ri.i) * ldx + ri.h * dk + d], acc);
    }
    part[((long long)c * (2 * w + 1) + r) * dk + d] = acc;
  }
}

__global__ void reduce_parts_kernel(const float* part, int nchunks, int n, float* out,
                                    int accum) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < nchunks; ++c) s += part[(long long)c * n + e];
    out[e] = accum ? out[e] + s : s;
  }
}

// Softmax backward, one wave per row: g = dPd * keep; dS = P (g - sum_j P g); scores that
// masked_fill replaced get no gradient.  In place on dS.
__global__ __launch_bounds__(256) void softmax_bwd_kernel(float* dS, const float* P,
                                                          const float* keep,
                                                          const long long* lens, long long rows,
                                                          int H, int T) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const RowIdx ri = row_idx(row, H, T);
  const int L = (int)lens[ri.b];
  float* g = dS + row * T;
  const float* p = P + row * T;
  const float* kp = keep ? keep + row * T : nullptr;
  float dot = 0.f;
  for (int j = lane; j < T; j += 64) {
    const float gj = kp ? g[j] * kp[j] : g[j];
    dot = fmaf(p[j], gj, dot);
  }
  dot = wsum(dot);
  for (int j = lane; j < T; j += 64) {
    const float gj = kp ? g[j] * kp[j] : g[j];
    g[j] = (ri.i >= L || j >= L) ? 0.f : p[j] * (gj - dot);
  }
}

// out_i[d] += sum_r A[row][i + r - w] tab[r][d]   (one thread per (row, d))
__global__ void band_rows_kernel(const float* A, const float* tab, float* out, int ldo,
                                 long long rows, int H, int T, int dk, int w) {
  const long long n = rows * dk;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long row = e / dk;
    const int d = (int)(e - row * dk);
    const RowIdx ri = row_idx(row, H, T);
    float acc = 0.f;
    for (int r = 0; r <= 2 * w; ++r) {
      const int j = ri.i + r - w;
      if (j >= 0 && j < T) acc = fmaf(A[row * T + j], tab[(long long)r * dk + d], acc);
    }
    out[((long long)ri.b * T + ri.i) * ldo + ri.h * dk + d] += acc;
  }
}

// y = x * x_mask: rows b*T + t with t >= L_b become 0 (y may alias x)
__global__ void mask_rows_kernel(const float* x, int ldx, float* y, int ldy, int T, int C,
                                 long long n, const long long* lens) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / C;
    const int c = (int)(e - r * C);
    const int b = (int)(r / T), t = (int)(r - (long long)b * T);
    y[r * ldy + c] = t < lens[b] ? x[r * ldx + c] : 0.f;
  }
}

// x[:, off::r] (forward, Tp rows per sequence) and its scatter-back (backward)
__global__ void stride_rows_kernel(const float* x, int ldx, float* y, int ldy, int T, int Tp,
                                   int C, int r, int off, long long n, int bwd) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / C;
    const int c = (int)(e - q * C);
    if (!bwd) {  // q = b*Tp + tp
      const int b = (int)(q / Tp), tp = (int)(q - (long long)b * Tp);
      y[q * ldy + c] = x[((long long)b * T + tp * r + off) * ldx + c];
    } else {  // q = b*T + t
      const int b = (int)(q / T), t = (int)(q - (long long)b * T);
      const int tp = (t - off) / r;
      const bool hit = t >= off && (t - off) % r == 0 && tp < Tp;
      y[q * ldy + c] = hit ? x[((long long)b * Tp + tp) * ldx + c] : 0.f;
    }
  }
}

// Depthwise Conv1d(C, C, kernel_size=r, stride=r, groups=C) (model.py:1610-1617, 1658)
__global__ void dwdown_fwd_kernel(const float* x, int ldx, const float* w, const float* bias,
                                  float* y, int ldy, int T, int Tp, int C, int r, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / C;
    const int c = (int)(e - q * C);
    const int b = (int)(q / Tp), tp = (int)(q - (long long)b * Tp);
    const float* xp = x + ((long long)b * T + (long long)tp * r) * ldx + c;
    float acc = 0.f;
    for (int k = 0; k < r; ++k) acc = fmaf(w[c * r + k], xp[(long long)k * ldx], acc);
    y[q * ldy + c] = acc + bias[c];
  }
}

// dx[b, tp*r + k, c] = w[c, k] dy[b, tp, c] (0 past Tp*r); prod[b*Tp + tp][c*r + k] =
// dy x (its column sums are the weight gradient)
__global__ void dwdown_bwd_kernel(const float* dy, int ldy, const float* x, int ldx,
                                  const float* w, float* dx, int lddx, float* prod, int T,
                                  int Tp, int C, int r, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / C;  // b*T + t
    const int c = (int)(e - q * C);
    const int b = (int)(q / T), t = (int)(q - (long long)b * T);
    const int tp = t / r, k = t - tp * r;
    float g = 0.f;
    if (tp < Tp) {
      const float d = dy[((long long)b * Tp + tp) * ldy + c];
      g = w[c * r + k] * d;
      prod[((long long)b * Tp + tp) * ((long long)C * r) + c * r + k] = d * x[q * ldx + c];
    }
    dx[q * lddx + c] = g;
  }
}

int grid1d(long long n) { return (int)std::min<long long>(16384, (n + 255) / 256); }

}  // namespace

ENSVS_API int ensvs_bgemm(const float* a, long long asb, long long ash, long long asr,
                          long long asc, const float* b, long long bsb, long long bsh,
                          long long bsr, long long bsc, float* c, long long csb, long long csh,
                          long long csr, long long csc, int Bn, int H, int M, int N, int K,
                          float alpha, int accum, void* stream) {
  if (Bn <= 0 || H <= 0 || M <= 0 || N <= 0 || K <= 0 || Bn * (long long)H > 65535)
    return ENSVS_E_SHAPE;
  BG A{a, asb, ash, asr, asc}, Bo{b, bsb, bsh, bsr, bsc};
  hipLaunchKernelGGL(bgemm_kernel, dim3(cdiv(M, TB), cdiv(N, TB), Bn * H), dim3(256), 0,
                     (hipStream_t)stream, A, Bo, c, csb, csh, csr, csc, H, M, N, K, alpha, accum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_div(const float* x, int ldx, float* y, int ldy, long long M, int C, float s,
                        void* stream) {
  if (M <= 0 || C <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(div_kernel, dim3(grid1d(M * C)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     y, ldy, M, C, s);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_softmax(float* S, const float* qs, int ldq, const float* ek,
                                 const long long* lens, int B, int H, int T, int dk, int w,
                                 const float* keep, float* Pd, void* stream) {
  if (w < 0 || 2 * w + 1 > 64 || T <= 0 || B <= 0 || H <= 0) return ENSVS_E_SHAPE;
  if ((keep == nullptr) != (Pd == nullptr)) return ENSVS_E_ARG;
  const long long rows = (long long)B * H * T;
  hipLaunchKernelGGL(softmax_kernel, dim3((int)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, S, qs, ldq, ek, lens, rows, H, T, dk, w, keep, Pd);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_relv(const float* P, const float* ev, float* O, int ldo, int B, int H,
                              int T, int dk, int w, void* stream) {
  const long long rows = (long long)B * H * T;
  if (rows <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(relv_kernel, dim3(grid1d(rows * dk)), dim3(256), 0, (hipStream_t)stream, P,
                     ev, O, ldo, rows, H, T, dk, w);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_band_dot(float* D, const float* vec, int ldv, const float* tab, int B,
                                  int H, int T, int dk, int w, void* stream) {
  if (w < 0 || 2 * w + 1 > 64) return ENSVS_E_SHAPE;
  const long long rows = (long long)B * H * T;
  if (rows <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(band_dot_kernel, dim3((int)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, D, vec, ldv, tab, rows, H, T, dk, w);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// floats of the `part` workspace ensvs_attn_table_grad needs
ENSVS_API long long ensvs_attn_table_grad_workspace(int dk, int w) {
  return 256LL * (2 * w + 1) * dk;
}

ENSVS_API int ensvs_attn_table_grad(const float* A, const float* X, int ldx, int B, int H, int T,
                                    int dk, int w, float* part, float* out, int accum,
                                    void* stream) {
  const long long rows = (long long)B * H * T;
  if (rows <= 0 || w < 0) return ENSVS_E_SHAPE;
  const int nch = (int)std::min<long long>(256, (rows + 63) / 64);
  const long long chunk = (rows + nch - 1) / nch;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(band_table_grad_kernel, dim3(2 * w + 1, nch), dim3(128), 0, st, A, X, ldx,
                     rows, H, T, dk, w, chunk, part);
  ENSVS_CHECK_LAUNCH();
  const int n = (2 * w + 1) * dk;
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, part, nch, n, out,
                     accum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_softmax_bwd(float* dS, const float* P, const float* keep,
                                     const long long* lens, int B, int H, int T, void* stream) {
  const long long rows = (long long)B * H * T;
  if (rows <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3((int)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, dS, P, keep, lens, rows, H, T);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_band_rows(const float* A, const float* tab, float* out, int ldo, int B,
                                   int H, int T, int dk, int w, void* stream) {
  const long long rows = (long long)B * H * T;
  if (rows <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(band_rows_kernel, dim3(grid1d(rows * dk)), dim3(256), 0,
                     (hipStream_t)stream, A, tab, out, ldo, rows, H, T, dk, w);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_mask_rows(const float* x, int ldx, float* y, int ldy, int B, int T, int C,
                              const long long* lens, void* stream) {
  const long long n = (long long)B * T * C;
  if (n <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(mask_rows_kernel, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, x,
                     ldx, y, ldy, T, C, n, lens);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_stride_rows(const float* x, int ldx, float* y, int ldy, int B, int T, int C,
                                int r, int off, int bwd, void* stream) {
  if (r <= 0 || off < 0 || off >= r || T <= 0 || C <= 0) return ENSVS_E_SHAPE;
  const int Tp = (T - off + r - 1) / r;
  const long long n = (long long)B * (bwd ? T : Tp) * C;
  if (n <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(stride_rows_kernel, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, x,
                     ldx, y, ldy, T, Tp, C, r, off, n, bwd);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_dwdown_fwd(const float* x, int ldx, const float* w, const float* bias,
                               float* y, int ldy, int B, int T, int C, int r, void* stream) {
  const int Tp = r > 0 ? T / r : 0;
  const long long n = (long long)B * Tp * C;
  if (n <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(dwdown_fwd_kernel, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, x,
                     ldx, w, bias, y, ldy, T, Tp, C, r, n);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_dwdown_bwd(const float* dy, int ldy, const float* x, int ldx, const float* w,
                               float* dx, int lddx, float* prod, int B, int T, int C, int r,
                               void* stream) {
  const int Tp = r > 0 ? T / r : 0;
  const long long n = (long long)B * T * C;
  if (n <= 0 || Tp <= 0) return ENSVS_E_SHAPE;
  hipLaunchKernelGGL(dwdown_bwd_kernel, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, dy,
                     ldy, x, ldx, w, dx, lddx, prod, T, Tp, C, r, n);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
