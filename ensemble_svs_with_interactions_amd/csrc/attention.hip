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

// ------------------------------------------------ batched GEMM, bf16 MFMA (production mode)
// The same products as bgemm_kernel with operands rounded to bf16 while staged and fp32
// accumulation on v_mfma_f32_16x16x32_bf16: 128 x 128 output tile per 256 threads (2 x 2 waves
// of 64 x 64), K in steps of 32, the next step's operands loaded into registers while the
// current one runs.  Each operand is staged in the layout of its contiguous axis, so every
// global load is a float4 run along it:
//  * k contiguous (A: sc == 1, B: sr == 1): image [128 rows][32 k], 80-B rows; a fragment is
//    one ds_read_b128 (8 k of one row);
//  * rows contiguous (A: sr == 1, B: sc == 1): image [32 k][128 rows], 256-B rows with XOR-
//    swizzled 16-B chunks; a fragment is two ds_read_b64_tr_b16 (transposed reads).
// Element (z, r, c) of an operand at p + zb*sb + zh*sh + r*sr + c*sc; for A (r, c) = (m, k),
// for B (r, c) = (k, n); the image row ("q") is m for A and n for B.
constexpr int QB = 128, KS = 32, IMGB = QB * 80;  // image bytes (the k-major one is 8 KB)

__device__ __forceinline__ int kmaj_off(int k, int ch) {  // [k][128 q] bf16, chunk ch = q / 8
  return 256 * k + 16 * (ch ^ (((k & 3) << 2) | ((k >> 2) & 3)));
}
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
__device__ __forceinline__ bf16x8 frag_kmaj(const char* img, int q0, int lane) {
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const int ch = (q0 >> 3) + (p >> 1);
  const int o0 = kmaj_off(8 * g + qq, ch) + 8 * (p & 1);
  const int o1 = kmaj_off(8 * g + 4 + qq, ch) + 8 * (p & 1);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(img + o0));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(img + o1));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 frag_qmaj(const char* img, int q0, int lane) {
  return *(const bf16x8*)(img + (q0 + (lane & 15)) * 80 + 16 * (lane >> 4));
}

struct Stage {  // one operand's staging: 16 consecutive elements along its contiguous axis
  const float* p;
  long long sq, sk;  // strides of q and k
  int Q, K;
  bool kfast;
};
// this thread's 16 elements of step k0: k-fast: q = tid/2, k = k0 + 16 (tid&1) ..;
// q-fast: k = k0 + tid/8, q = q0 + 16 (tid&7) ..; zeros outside [Q) x [K)
__device__ __forceinline__ void stage_load(const Stage& S, int q0, int k0, int tid, f32x4 (&v)[4]) {
  int q, k, n;
  const float* base;
  long long st;
  if (S.kfast) {
    q = q0 + (tid >> 1);
    k = k0 + 16 * (tid & 1);
    n = q < S.Q ? S.K - k : 0;
    base = S.p + q * S.sq + k;
    st = 1;
  } else {
    k = k0 + (tid >> 3);
    q = q0 + 16 * (tid & 7);
    n = k < S.K ? S.Q - q : 0;
    base = S.p + k * S.sk + q;
    st = 1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rem = n - 4 * i;
    if (rem >= 4) {
      v[i] = *(const f32x4*)(base + 4 * i);
    } else {
      f32x4 t = {0.f, 0.f, 0.f, 0.f};
      for (int e = 0; e < rem; ++e) t[e] = base[4 * i + e * st];
      v[i] = t;
    }
  }
}
__device__ __forceinline__ void stage_store(const Stage& S, char* img, int tid, const f32x4 (&v)[4]) {
  bf16x8 lo, hi;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    lo[e] = (__bf16)v[0][e];
    lo[4 + e] = (__bf16)v[1][e];
    hi[e] = (__bf16)v[2][e];
    hi[4 + e] = (__bf16)v[3][e];
  }
  if (S.kfast) {
    char* r = img + (tid >> 1) * 80 + 32 * (tid & 1);
    *(bf16x8*)r = lo;
    *(bf16x8*)(r + 16) = hi;
  } else {
    const int k = tid >> 3, ch = 2 * (tid & 7);
    *(bf16x8*)(img + kmaj_off(k, ch)) = lo;
    *(bf16x8*)(img + kmaj_off(k, ch + 1)) = hi;
  }
}

__global__ __launch_bounds__(256) void bgemm_b16_kernel(BG A, BG B, float* C, long long csb,
                                                        long long csh, long long csr,
                                                        long long csc, int H, int M, int N,
                                                        int K, float alpha, int accum) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][IMGB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int z = blockIdx.z, zb = z / H, zh = z % H;
  const int m0 = blockIdx.x * QB, n0 = blockIdx.y * QB;
  Stage SA{A.p + zb * A.sb + zh * A.sh + m0 * A.sr, A.sr, A.sc, M - m0, K, A.sc == 1};
  Stage SB{B.p + zb * B.sb + zh * B.sh + n0 * B.sc, B.sc, B.sr, N - n0, K, B.sr == 1};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 va[4], vb[4];
  const int nk = (K + KS - 1) / KS;
  stage_load(SA, 0, 0, tid, va);
  stage_load(SB, 0, 0, tid, vb);
  for (int it = 0; it < nk; ++it) {
    char* IA = smem[it & 1][0];
    char* IB = smem[it & 1][1];
    stage_store(SA, IA, tid, va);
    stage_store(SB, IB, tid, vb);
    __syncthreads();
    if (it + 1 < nk) {
      stage_load(SA, 0, (it + 1) * KS, tid, va);
      stage_load(SB, 0, (it + 1) * KS, tid, vb);
    }
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i] = SA.kfast ? frag_qmaj(IA, wr * 64 + 16 * i, lane) : frag_kmaj(IA, wr * 64 + 16 * i, lane);
      fb[i] = SB.kfast ? frag_qmaj(IB, wc * 64 + 16 * i, lane) : frag_kmaj(IB, wc * 64 + 16 * i, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
  float* c = C + zb * csb + zh * csh;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wr * 64 + 16 * i + 4 * (lane >> 4) + r;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + 16 * j + (lane & 15);
        if (n >= N) continue;
        float* p = c + m * csr + n * csc;
        const float v = alpha * acc[i][j][r];
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

// lane r <= 2w: v . tab[r] over dk (float4 runs when vec4: dk % 4 == 0, 16-B aligned rows)
__device__ __forceinline__ float band_lane_dot(const float* v, const float* tab, int dk, int w,
                                               int lane, int vec4) {
  float acc = 0.f;
  if (lane > 2 * w) return acc;
  const float* e = tab + (long long)lane * dk;
  if (vec4) {
    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
    for (int d = 0; d < dk; d += 4) {
      const f32x4 x = *(const f32x4*)(v + d), y = *(const f32x4*)(e + d);
      a4 = x * y + a4;
    }
    acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  } else {
    for (int d = 0; d < dk; ++d) acc = fmaf(v[d], e[d], acc);
  }
  return acc;
}

// softmax_kernel with the row held in registers (T <= 64 NJ): S read once and P written once
// (the three-pass form re-read and re-wrote the row in global memory: 159 us per 16 384 rows
// of 1 024, profiles/r4_tf_prof_before.txt).
template <int NJ>
__global__ __launch_bounds__(256) void softmax_reg_kernel(float* S, const float* qs, int ldq,
                                                          const float* ek, const long long* lens,
                                                          long long rows, int H, int T, int dk,
                                                          int w, const float* keep, float* Pd,
                                                          int vec4) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // wave-uniform
  const RowIdx ri = row_idx(row, H, T);
  float* s = S + row * T;
  const int L = (int)lens[ri.b];
  const float rel = band_lane_dot(qs + ((long long)ri.b * T + ri.i) * ldq + ri.h * dk, ek, dk, w,
                                  lane, vec4);
  float v[NJ];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    v[jj] = j < T ? s[j] : -INFINITY;
  }
  float m = -INFINITY;
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    const int r = j - ri.i + w;
    const float rv = __shfl(rel, min(max(r, 0), 63));
    if (j < T) {
      float x = v[jj];
      if (r >= 0 && r <= 2 * w) x += rv;
      if (ri.i >= L || j >= L) x = -1e4f;
      v[jj] = x;
      m = fmaxf(m, x);
    }
  }
  m = wmax(m);
  float sum = 0.f;
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    const float e = j < T ? __expf(v[jj] - m) : 0.f;
    v[jj] = e;
    sum += e;
  }
  sum = wsum(sum);
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    if (j < T) {
      const float p = v[jj] / sum;
      s[j] = p;
      if (keep) Pd[row * T + j] = p * keep[row * T + j];
    }
  }
}

// softmax_bwd_kernel with the row in registers (dS, P and keep read once, dS written once)
template <int NJ>
__global__ __launch_bounds__(256) void softmax_bwd_reg_kernel(float* dS, const float* P,
                                                              const float* keep,
                                                              const long long* lens,
                                                              long long rows, int H, int T) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const RowIdx ri = row_idx(row, H, T);
  const int L = (int)lens[ri.b];
  float* g = dS + row * T;
  const float* p = P + row * T;
  const float* kp = keep ? keep + row * T : nullptr;
  float gv[NJ], pv[NJ];
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    gv[jj] = j < T ? (kp ? g[j] * kp[j] : g[j]) : 0.f;
    pv[jj] = j < T ? p[j] : 0.f;
  }
  float dot = 0.f;
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) dot = fmaf(pv[jj], gv[jj], dot);
  dot = wsum(dot);
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = jj * 64 + lane;
    if (j < T) g[j] = (ri.i >= L || j >= L) ? 0.f : pv[jj] * (gv[jj] - dot);
  }
}

// band_table_grad_kernel as one workgroup per block of rows: each wave walks its rows with the
// band values in registers (loaded once per row) and accumulates all 2w + 1 table rows for its
// dk columns (lane d, d + 64, ...); the 4 waves' sums are combined in a fixed order through LDS.
// (The per-(r, chunk) form walked 64 rows per thread one dependent load pair at a time, and its
// 256-chunk reduction ran one thread per output: 65 + 60 us, profiles/r4_tf_prof_before.txt.)
constexpr int TG_W2 = 9;  // 2w + 1 <= 9 (the encoder's window_size 4)
template <int ND>
__global__ __launch_bounds__(256) void band_table_grad2_kernel(const float* A, const float* X,
                                                               int ldx, long long rows, int H,
                                                               int T, int dk, int w, int rpb,
                                                               float* part) {
  extern __shared__ float red[];  // [4][W2][dk]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, W2 = 2 * w + 1;
  float acc[TG_W2][ND];
#pragma unroll
  for (int r = 0; r < TG_W2; ++r)
#pragma unroll
    for (int q = 0; q < ND; ++q) acc[r][q] = 0.f;
  const long long r0 = (long long)blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  for (long long row = r0 + wid; row < r1; row += 4) {
    const RowIdx ri = row_idx(row, H, T);
    float av[TG_W2];
#pragma unroll
    for (int r = 0; r < TG_W2; ++r) {
      const int j = ri.i + r - w;
      av[r] = (r < W2 && j >= 0 && j < T) ? A[row * T + j] : 0.f;
    }
    const float* x = X + ((long long)ri.b * T + ri.i) * ldx + ri.h * dk;
    float xv[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) xv[q] = lane + 64 * q < dk ? x[lane + 64 * q] : 0.f;
#pragma unroll
    for (int r = 0; r < TG_W2; ++r)
#pragma unroll
      for (int q = 0; q < ND; ++q) acc[r][q] = fmaf(av[r], xv[q], acc[r][q]);
  }
#pragma unroll
  for (int r = 0; r < TG_W2; ++r)
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      const int d = lane + 64 * q;
      if (r < W2 && d < dk) red[(wid * W2 + r) * dk + d] = acc[r][q];
    }
  __syncthreads();
  for (int e = tid; e < W2 * dk; e += 256) {
    const float t = ((red[e] + red[W2 * dk + e]) + red[2 * W2 * dk + e]) + red[3 * W2 * dk + e];
    part[(long long)blockIdx.x * W2 * dk + e] = t;
  }
}

// out[e] (+)= sum_c part[c][e] in chunk order, 8 chunk loads in flight per step
__global__ void reduce_parts2_kernel(const float* part, int nchunks, int n, float* out,
                                     int accum) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float s = 0.f;
  int c = 0;
  for (; c + 8 <= nchunks; c += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[(long long)(c + k) * n + e];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  for (; c < nchunks; ++c) s += part[(long long)c * n + e];
  out[e] = accum ? out[e] + s : s;
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
                                                       int T, int dk, int w, int vec4) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const RowIdx ri = row_idx(row, H, T);
  const int j = ri.i + lane - w;
  if (lane > 2 * w || j < 0 || j >= T) return;
  const float dot = band_lane_dot(vec + ((long long)ri.b * T + ri.i) * ldv + ri.h * dk, tab, dk,
                                  w, lane, vec4);
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

// bf16-operand MFMA form of ensvs_bgemm (production precision).  Each operand needs a unit
// stride on its row or its reduction axis, 16-B aligned rows and the other strides multiples
// of 4 floats; other layouts run the exact kernel.
ENSVS_API int ensvs_bgemm_bf16(const float* a, long long asb, long long ash, long long asr,
                               long long asc, const float* b, long long bsb, long long bsh,
                               long long bsr, long long bsc, float* c, long long csb,
                               long long csh, long long csr, long long csc, int Bn, int H, int M,
                               int N, int K, float alpha, int accum, void* stream) {
  if (Bn <= 0 || H <= 0 || M <= 0 || N <= 0 || K <= 0 || Bn * (long long)H > 65535)
    return ENSVS_E_SHAPE;
  auto ok = [](const float* p, long long sb, long long sh, long long sr, long long sc) {
    const bool unit = sr == 1 || sc == 1;
    const long long other = sr == 1 ? sc : sr;
    return unit && (((uintptr_t)p) & 15) == 0 && other % 4 == 0 && sb % 4 == 0 && sh % 4 == 0;
  };
  if (!ok(a, asb, ash, asr, asc) || !ok(b, bsb, bsh, bsr, bsc))
    return ensvs_bgemm(a, asb, ash, asr, asc, b, bsb, bsh, bsr, bsc, c, csb, csh, csr, csc, Bn,
                       H, M, N, K, alpha, accum, stream);
  BG A{a, asb, ash, asr, asc}, Bo{b, bsb, bsh, bsr, bsc};
  hipLaunchKernelGGL(bgemm_b16_kernel, dim3(cdiv(M, QB), cdiv(N, QB), Bn * H), dim3(256), 0,
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
  const int vec4 = dk % 4 == 0 && ldq % 4 == 0 && ((((uintptr_t)qs) | (uintptr_t)ek) & 15) == 0;
  const dim3 grid((int)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define SMX(NJ)                                                                                  \
  hipLaunchKernelGGL(softmax_reg_kernel<NJ>, grid, dim3(256), 0, st, S, qs, ldq, ek, lens, rows, \
                     H, T, dk, w, keep, Pd, vec4)
  if (T <= 64) SMX(1);
  else if (T <= 128) SMX(2);
  else if (T <= 256) SMX(4);
  else if (T <= 512) SMX(8);
  else if (T <= 1024) SMX(16);
  else if (T <= 2048) SMX(32);
  else
    hipLaunchKernelGGL(softmax_kernel, grid, dim3(256), 0, st, S, qs, ldq, ek, lens, rows, H, T,
                       dk, w, keep, Pd);
#undef SMX
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
  const int vec4 = dk % 4 == 0 && ldv % 4 == 0 && ((((uintptr_t)vec) | (uintptr_t)tab) & 15) == 0;
  hipLaunchKernelGGL(band_dot_kernel, dim3((int)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, D, vec, ldv, tab, rows, H, T, dk, w, vec4);
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
  hipStream_t st = (hipStream_t)stream;
  const int n = (2 * w + 1) * dk;
  if (2 * w + 1 <= TG_W2 && dk <= 256) {
    // blocks of rpb rows (a multiple of the 4 waves), at most 256 partials (the workspace)
    const long long rpb = std::max<long long>(128, (cdiv(rows, 256) + 3) / 4 * 4);
    const int nch = cdiv(rows, rpb);
    const size_t lds = 4 * (size_t)n * sizeof(float);
#define TG(ND)                                                                                \
  hipLaunchKernelGGL(band_table_grad2_kernel<ND>, dim3(nch), dim3(256), lds, st, A, X, ldx, rows, \
                     H, T, dk, w, (int)rpb, part)
    if (dk <= 64) TG(1);
    else if (dk <= 128) TG(2);
    else TG(4);
#undef TG
    ENSVS_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_parts2_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, part, nch, n,
                       out, accum);
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  const int nch = (int)std::min<long long>(256, (rows + 63) / 64);
  const long long chunk = (rows + nch - 1) / nch;
  hipLaunchKernelGGL(band_table_grad_kernel, dim3(2 * w + 1, nch), dim3(128), 0, st, A, X, ldx,
                     rows, H, T, dk, w, chunk, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, part, nch, n, out,
                     accum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_attn_softmax_bwd(float* dS, const float* P, const float* keep,
                                     const long long* lens, int B, int H, int T, void* stream) {
  const long long rows = (long long)B * H * T;
  if (rows <= 0) return ENSVS_E_SHAPE;
  const dim3 grid((int)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define SMB(NJ) \
  hipLaunchKernelGGL(softmax_bwd_reg_kernel<NJ>, grid, dim3(256), 0, st, dS, P, keep, lens, rows, H, T)
  if (T <= 64) SMB(1);
  else if (T <= 128) SMB(2);
  else if (T <= 256) SMB(4);
  else if (T <= 512) SMB(8);
  else if (T <= 1024) SMB(16);
  else if (T <= 2048) SMB(32);
  else hipLaunchKernelGGL(softmax_bwd_kernel, grid, dim3(256), 0, st, dS, P, keep, lens, rows, H, T);
#undef SMB
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
