// Memory-bound kernels around the GEMMs and recurrences: phoneme argmax +
// embedding, BatchNorm1d (training statistics, apply+ReLU, backward), DiffNet
// step embedding / Mish, diffusion q_sample / p_sample, the masked L1 loss with
// its fused gradient, and the clip-by-global-norm + Adam update over the flat
// parameter buffer.  All are HBM-bound: grid-stride loops, one pass each.
#include <initializer_list>

#include "common.h"
#include "ensvs.h"

namespace {

#define GRID_LOOP(i, n) \
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); \
       i += (long long)gridDim.x * blockDim.x)

constexpr int BN_STATS_MAX_SPLITS = 256;

inline int grid_for(long long n) { return (int)std::min<long long>(8192, (n + 255) / 256); }

// ------------------------------------------------------------- embeddings
// ids[m] = argmax over x[m][ph0 .. ph0+nv) (first maximum; all-zero row -> 0),
// nnsvs/model.py:905 / tacotron_f0.py:939 torch.argmax semantics.
__global__ void phoneme_ids_kernel(const float* __restrict__ x, int ld, long long M, int ph0,
                                   int nv, int* __restrict__ ids) {
  GRID_LOOP(m, M) {
    const float* r = x + m * ld + ph0;
    float best = r[0];
    int bi = 0;
    for (int v = 1; v < nv; ++v) {
      const float z = r[v];
      if (z > best) { best = z; bi = v; }
    }
    ids[m] = bi;
  }
}

// The same with the block's 64 rows x nv columns staged through LDS by coalesced loads (the
// row-per-thread form reads each row's columns 4 * ld bytes apart across lanes: 18 us for
// 30 k rows).  Same comparisons in the same order, so the same ids.
constexpr int PH_ROWS = 64, PH_MAXV = 128;
__global__ __launch_bounds__(256) void phoneme_ids_tile_kernel(const float* __restrict__ x, int ld,
                                                               int M, int ph0, int nv,
                                                               int* __restrict__ ids) {
  __shared__ float t[PH_ROWS * (PH_MAXV + 1)];
  const int m0 = blockIdx.x * PH_ROWS;
  const int rows = min(PH_ROWS, M - m0);
  for (int i = threadIdx.x; i < rows * nv; i += 256) {
    const int r = i / nv, c = i - r * nv;
    t[r * (PH_MAXV + 1) + c] = x[(long long)(m0 + r) * ld + ph0 + c];
  }
  __syncthreads();
  if ((int)threadIdx.x < rows) {
    const float* r = t + threadIdx.x * (PH_MAXV + 1);
    float best = r[0];
    int bi = 0;
    for (int v = 1; v < nv; ++v) {
      const float z = r[v];
      if (z > best) { best = z; bi = v; }
    }
    ids[m0 + threadIdx.x] = bi;
  }
}

// Y[m][c] += sum_k emb[ids_k[m]][c] + spk_k[m / T][c]   (k over 1 or 2 tracks)
__global__ void embed_add_kernel(float* __restrict__ y, int ldy, long long M, int C, int T,
                                 const float* __restrict__ emb, const int* __restrict__ ids0,
                                 const int* __restrict__ ids1, const float* __restrict__ spk0,
                                 const float* __restrict__ spk1, int ldspk) {
  GRID_LOOP(i, M * C) {
    const long long m = i / C;
    const int c = (int)(i % C);
    const long long b = m / T;
    float v = y[m * ldy + c];
    if (ids0) v += emb[(long long)ids0[m] * C + c];
    if (ids1) v += emb[(long long)ids1[m] * C + c];
    if (spk0) v += spk0[b * ldspk + c];
    if (spk1) v += spk1[b * ldspk + c];
    y[m * ldy + c] = v;
  }
}

// The same, one row per 64-lane group (float4 lanes when VEC): no 64-bit division per element
// (the flat form above ran 32 us for 30 k x 256, VALU-bound on it).  Same adds in the same
// order per element.
template <bool VEC>
__global__ __launch_bounds__(256) void embed_add_rows_kernel(
    float* __restrict__ y, int ldy, int M, int C, int T, const float* __restrict__ emb,
    const int* __restrict__ ids0, const int* __restrict__ ids1, const float* __restrict__ spk0,
    const float* __restrict__ spk1, int ldspk) {
  const int lane = threadIdx.x & 63, sub = threadIdx.x >> 6;
  for (int m = blockIdx.x * 4 + sub; m < M; m += gridDim.x * 4) {
    const int b = m / T;
    const float* e0 = ids0 ? emb + (long long)ids0[m] * C : nullptr;
    const float* e1 = ids1 ? emb + (long long)ids1[m] * C : nullptr;
    const float* s0 = spk0 ? spk0 + (long long)b * ldspk : nullptr;
    const float* s1 = spk1 ? spk1 + (long long)b * ldspk : nullptr;
    float* yr = y + (long long)m * ldy;
    if constexpr (VEC) {
      for (int c = lane * 4; c < C; c += 256) {
        f32x4 v = *(const f32x4*)(yr + c);
        if (e0) v += *(const f32x4*)(e0 + c);
        if (e1) v += *(const f32x4*)(e1 + c);
        if (s0) v += *(const f32x4*)(s0 + c);
        if (s1) v += *(const f32x4*)(s1 + c);
        *(f32x4*)(yr + c) = v;
      }
    } else {
      for (int c = lane; c < C; c += 64) {
        float v = yr[c];
        if (e0) v += e0[c];
        if (e1) v += e1[c];
        if (s0) v += s0[c];
        if (s1) v += s1[c];
        yr[c] = v;
      }
    }
  }
}

// Embedding backward, deterministic.  Block (column block of 64, chunk of
// EMB_CHUNK frames): 4 sub-chunks x 64 columns; each thread walks its frames in
// order adding dy into an LDS table acc[sub][v][c]; the 4 sub-tables are summed in
// order into part[chunk][v][c]; embed_reduce sums the chunks in order into demb.
constexpr int EMB_CHUNK = 256;
__global__ __launch_bounds__(256) void embed_bwd_kernel(const float* __restrict__ dy, int ldy,
                                                        long long M, int C,
                                                        const int* __restrict__ ids, int V,
                                                        float* __restrict__ part) {
  extern __shared__ float acc[];  // [4][V][64]
  const int c = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  for (int i = threadIdx.x; i < 4 * V * 64; i += 256) acc[i] = 0.f;
  __syncthreads();
  const long long m0 = (long long)blockIdx.y * EMB_CHUNK + sub * (EMB_CHUNK / 4);
  const long long m1 = min(M, m0 + EMB_CHUNK / 4);
  float* a = acc + sub * V * 64 + c;
  // ids come in runs (a phoneme spans many frames): sum a run in a register and touch LDS
  // only when the id changes; four rows' loads in flight per step.
  if (col < C && m0 < m1) {
    int cur = ids[m0];
    float run = 0.f;
    long long m = m0;
    for (; m + 4 <= m1; m += 4) {
      int id[4];
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        id[j] = ids[m + j];
        v[j] = dy[(m + j) * ldy + col];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (id[j] != cur) {
          a[cur * 64] += run;
          cur = id[j];
          run = 0.f;
        }
        run += v[j];
      }
    }
    for (; m < m1; ++m) {
      const int i1 = ids[m];
      if (i1 != cur) {
        a[cur * 64] += run;
        cur = i1;
        run = 0.f;
      }
      run += dy[m * ldy + col];
    }
    a[cur * 64] += run;
  }
  __syncthreads();
  float* out = part + (long long)blockIdx.y * V * C;
  for (int i = threadIdx.x; i < V * 64; i += 256) {
    const int v = i >> 6, cc = i & 63;
    const int gc = blockIdx.x * 64 + cc;
    if (gc < C)
      out[(long long)v * C + gc] =
          (acc[i] + acc[V * 64 + i]) + (acc[2 * V * 64 + i] + acc[3 * V * 64 + i]);
  }
}

// chunk partials summed in chunk order, 16 loads in flight per thread (one at a time measured
// 37 us: V x C = 15 k threads each walking 120 dependent loads)
constexpr int EMB_ILP = 16;
__global__ void embed_reduce_kernel(const float* __restrict__ part, int nchunk, long long VC,
                                    float* __restrict__ demb) {
  GRID_LOOP(i, VC) {
    float s = 0.f;
    int k = 0;
    for (; k + EMB_ILP <= nchunk; k += EMB_ILP) {
      float t[EMB_ILP];
#pragma unroll
      for (int j = 0; j < EMB_ILP; ++j) t[j] = part[(k + j) * VC + i];
#pragma unroll
      for (int j = 0; j < EMB_ILP; ++j) s += t[j];
    }
    for (; k < nchunk; ++k) s += part[k * VC + i];
    demb[i] += s;
  }
}

// dtable[spk[b]][c] += sum over b' with spk[b'] == spk[b] of dseq[b'][c], written by the
// first such b (fixed summation order, no atomics).
__global__ void spk_scatter_kernel(const float* __restrict__ dseq, int B, int C,
                                   const long long* __restrict__ spk, float* __restrict__ dtab) {
  GRID_LOOP(i, (long long)B * C) {
    const int b = (int)(i / C), c = (int)(i % C);
    const long long r = spk[b];
    bool first = true;
    for (int q = 0; q < b; ++q) first &= spk[q] != r;
    if (!first) continue;
    float s = 0.f;
    for (int q = b; q < B; ++q)
      if (spk[q] == r) s += dseq[(long long)q * C + c];
    dtab[r * C + c] += s;
  }
}

// out[b][c] = table[spk[b]][c]
__global__ void gather_rows_kernel(const float* __restrict__ table, const long long* __restrict__ idx,
                                   int B, int C, float* __restrict__ out) {
  GRID_LOOP(i, (long long)B * C) {
    const int b = (int)(i / C), c = (int)(i % C);
    out[i] = table[idx[b] * C + c];
  }
}

// ------------------------------------------------------------- BatchNorm1d
// stats[g][0][c] = mean, stats[g][1][c] = rstd from (sum, sumsq-about-mean) already in
// mean/var buffers: var_biased = var_sum / M.
__global__ void bn_finalize_kernel(float* __restrict__ mean, float* __restrict__ var, int G, int C,
                                   long long Mg, float eps, float* __restrict__ rstd,
                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                   float momentum, int update) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float rm = update ? rmean[c] : 0.f, rv = update ? rvar[c] : 0.f;
  for (int g = 0; g < G; ++g) {
    const float mu = mean[g * C + c];
    const float vb = var[g * C + c];  // biased variance
    rstd[g * C + c] = 1.f / sqrtf(vb + eps);
    if (update) {
      const float vu = Mg > 1 ? vb * (float)Mg / (float)(Mg - 1) : vb;
      rm = (1.f - momentum) * rm + momentum * mu;
      rv = (1.f - momentum) * rv + momentum * vu;
    }
  }
  if (update) {
    rmean[c] = rm;
    rvar[c] = rv;
  }
}

// BatchNorm training statistics in two launches (round 5; were two column-sum launch pairs and
// bn_finalize).  bn_stats_partial: per (64-column block, row split s, group g) the split's
// column sums and its sums of squared deviations from the split's own mean (the split's rows
// are read twice, the second time from L2); part[g][s] = [sum (C) | M2 (C)].  bn_stats_final:
// per column, the group's mean (split sums added in a fixed order in double) and biased
// variance by Chan's merge of the splits (double, fixed order): var = (sum_s M2_s +
// n_s (mean_s - mean)^2) / Mg -- deterministic, and as exact as the two-pass form -- then
// bn_finalize's rstd and running-statistic updates (`updates` EMA steps per group, the
// module's num_batches_tracked advanced by G * updates).
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const float* __restrict__ y, int ld,
                                                               int Mg, int C, int rps, int vec,
                                                               float* __restrict__ part) {
  __shared__ f32x4 red[16][17];
  __shared__ f32x4 tot[16];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  const int s = blockIdx.y, S = gridDim.y;
  y += (long long)blockIdx.z * Mg * ld;
  float* pg = part + ((long long)blockIdx.z * S + s) * 2 * C;
  const int r0 = s * rps, r1 = min(Mg, r0 + rps);
  auto ld4 = [&](int r) -> f32x4 {
    const float* q = y + (long long)r * ld + col;
    f32x4 v;
    if (vec && col + 3 < C) {
      v = *(const f32x4*)q;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = col + e < C ? q[e] : 0.f;
    }
    return v;
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      const f32x4 v0 = ld4(r), v1 = ld4(r + 16), v2 = ld4(r + 32), v3 = ld4(r + 48);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; r < r1; r += 16) acc += ld4(r);
  }
  red[rl][cq] = acc;
  __syncthreads();
  if (rl == 0) {
    f32x4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cq];
    tot[cq] = t;
  }
  __syncthreads();
  const f32x4 sum = tot[cq];
  const float inv_n = 1.f / (float)max(r1 - r0, 1);
  const f32x4 mu = sum * inv_n;
  f32x4 q2 = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      const f32x4 v0 = ld4(r) - mu, v1 = ld4(r + 16) - mu, v2 = ld4(r + 32) - mu,
                  v3 = ld4(r + 48) - mu;
      q2 += (v0 * v0 + v1 * v1) + (v2 * v2 + v3 * v3);
    }
    for (; r < r1; r += 16) {
      const f32x4 v = ld4(r) - mu;
      q2 += v * v;
    }
  }
  red[rl][cq] = q2;  // every lane has read red (the sums) before the barrier above
  __syncthreads();
  if (rl == 0) {
    f32x4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cq];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (col + e < C) {
        pg[col + e] = sum[e];
        pg[C + col + e] = t[e];
      }
  }
}

// 16 columns x 16 split lanes per block: lane sl takes splits sl, sl + 16, ... (at most
// BN_STATS_MAX_SPLITS / 16 = 16: all its (sum, M2) pairs are loaded into registers at once,
// one round trip), and the 16 lane totals are added in lane order (fixed: deterministic)
__global__ __launch_bounds__(256) void bn_stats_final_kernel(
    const float* __restrict__ part, int S, int G, int C, int Mg, int rps, float eps,
    float* __restrict__ mean, float* __restrict__ var, float* __restrict__ rstd,
    float* __restrict__ rmean, float* __restrict__ rvar, float momentum, int updates,
    long long* __restrict__ nbt) {
  constexpr int PER = BN_STATS_MAX_SPLITS / 16;
  __shared__ double red[16][17];
  __shared__ double mus[16];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  if (blockIdx.x == 0 && threadIdx.x == 0 && updates > 0 && nbt) nbt[0] += (long long)G * updates;
  for (int g = 0; g < G; ++g) {
    const float* pg = part + (long long)g * S * 2 * C;
    float sv[PER], qv[PER];
    // unconditional loads at clamped (in-range) addresses, then the select: a predicated load
    // compiled to a branch and a wait per element (32 round trips, ~13 us per launch)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int s = sl + 16 * i;
      const bool ok = c < C && s < S;
      const float* q = pg + (long long)min(s, S - 1) * 2 * C + min(c, C - 1);
      const float a = q[0], b = q[C];
      sv[i] = ok ? a : 0.f;
      qv[i] = ok ? b : 0.f;
    }
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < PER; ++i) a += (double)sv[i];
    red[sl][cl] = a;
    __syncthreads();
    if (sl == 0) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[i][cl];
      mus[cl] = t / (double)Mg;
    }
    __syncthreads();
    const double mu = mus[cl];
    double m2 = 0.0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int s = sl + 16 * i;
      const int n = min(rps, Mg - s * rps);
      if (c < C && s < S && n > 0) {
        const double d = (double)sv[i] / (double)n - mu;
        m2 += (double)qv[i] + (double)n * d * d;
      }
    }
    __syncthreads();  // every lane has read red (the sums)
    red[sl][cl] = m2;
    __syncthreads();
    if (sl == 0 && c < C) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[i][cl];
      const float vb = (float)(t / (double)Mg);
      mean[g * C + c] = (float)mu;
      var[g * C + c] = vb;
      rstd[g * C + c] = 1.f / sqrtf(vb + eps);
    }
    __syncthreads();
  }
  if (sl == 0 && c < C && updates > 0) {  // bn_finalize's order: every group, `updates` times
    float rm = rmean[c], rv = rvar[c];
    for (int u = 0; u < updates; ++u)
      for (int g = 0; g < G; ++g) {
        const float mu = mean[g * C + c], vb = var[g * C + c];
        const float vu = Mg > 1 ? vb * (float)Mg / (float)(Mg - 1) : vb;
        rm = (1.f - momentum) * rm + momentum * mu;
        rv = (1.f - momentum) * rv + momentum * vu;
      }
    rmean[c] = rm;
    rvar[c] = rv;
  }
}

// out = relu((y - mean_g) * rstd_g * gamma + beta); group g = m / Mg
__global__ void bn_apply_relu_kernel(const float* __restrict__ y, int ldy, long long M, int C,
                                     long long Mg, const float* __restrict__ mean,
                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                     const float* __restrict__ beta, float* __restrict__ out,
                                     int ldo) {
  GRID_LOOP(i, M * C) {
    const long long m = i / C;
    const int c = (int)(i % C);
    const int g = (int)(m / Mg);
    const float v = (y[m * ldy + c] - mean[g * C + c]) * rstd[g * C + c] * gamma[c] + beta[c];
    out[m * ldo + c] = fmaxf(v, 0.f);
  }
}

// Four channels per lane (C, every ld % 4 == 0, 16-B aligned rows, M*C < 2^31): 16-B
// accesses and 32-bit index math; per element the same expression as the scalar kernel.
__global__ void bn_apply_relu4_kernel(const float* __restrict__ y, int ldy, int M, int C, int Mg,
                                      const float* __restrict__ mean,
                                      const float* __restrict__ rstd,
                                      const float* __restrict__ gamma,
                                      const float* __restrict__ beta, float* __restrict__ out,
                                      int ldo, __bf16* __restrict__ outb, int ldob) {
  const int C4 = C >> 2, n = M * C4;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int m = q / C4, c = (q - m * C4) * 4, g = m / Mg;
    const f32x4 v = *(const f32x4*)(y + (long long)m * ldy + c);
    const f32x4 mu = *(const f32x4*)(mean + g * C + c), rs = *(const f32x4*)(rstd + g * C + c);
    const f32x4 ga = *(const f32x4*)(gamma + c), be = *(const f32x4*)(beta + c);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaxf((v[j] - mu[j]) * rs[j] * ga[j] + be[j], 0.f);
    *(f32x4*)(out + (long long)m * ldo + c) = o;
    if (outb) store_bf16x4(outb + (long long)m * ldob + c, o);
  }
}

// Per-group column partials of dz and dz*xhat, dz = dout * (z > 0).
__global__ void bn_bwd_reduce_kernel(const float* __restrict__ dout, int ldd,
                                     const float* __restrict__ y, int ldy, long long Mg, int C,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                     int rps, float* __restrict__ part) {
  // grid: (ceil(C/64), S, G); part[g][s][2][C]
  __shared__ float red[2][4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int s = blockIdx.y, g = blockIdx.z, S = gridDim.y;
  const long long r0 = (long long)g * Mg + (long long)s * rps;
  const long long r1 = min((long long)g * Mg + Mg, r0 + rps);
  float a = 0.f, bsum = 0.f;
  if (col < C) {
    const float mu = mean[g * C + col], rs = rstd[g * C + col], ga = gamma[col], be = beta[col];
#pragma unroll 4
    for (long long r = r0 + w; r < r1; r += 4) {
      const float xh = (y[r * ldy + col] - mu) * rs;
      const float z = xh * ga + be;
      const float dz = z > 0.f ? dout[r * ldd + col] : 0.f;
      a += dz;
      bsum += dz * xh;
    }
  }
  red[0][w][threadIdx.x & 63] = a;
  red[1][w][threadIdx.x & 63] = bsum;
  __syncthreads();
  if (w == 0 && col < C) {
    float* p = part + (((long long)g * S + s) * 2) * C;
    p[col] = (red[0][0][threadIdx.x] + red[0][1][threadIdx.x]) +
             (red[0][2][threadIdx.x] + red[0][3][threadIdx.x]);
    p[C + col] = (red[1][0][threadIdx.x] + red[1][1][threadIdx.x]) +
                 (red[1][2][threadIdx.x] + red[1][3][threadIdx.x]);
  }
}

// bn_bwd_reduce_kernel with four channels per lane (the bn_vec4 conditions): a 256-thread
// block covers LPR = min(64, C / 4) lanes of 4 channels per row and 256 / LPR rows at a time,
// 16-B loads with 4 rows in flight per lane (the scalar form read 4 B per lane: 21 us per
// 30 720 x 256 launch, profiles/r4_train_kernel_stats.csv).  Rows r0 + rl + RB k per lane in
// order, then the RB row lanes folded in order: deterministic.
template <int LPR>
__global__ __launch_bounds__(256) void bn_bwd_reduce4_kernel(
    const float* __restrict__ dout, int ldd, const float* __restrict__ y, int ldy, long long Mg,
    int C, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int rps,
    float* __restrict__ part) {
  // grid: (ceil(C / (4 LPR)), S, G); part[g][s][2][C]
  constexpr int RB = 256 / LPR;
  __shared__ f32x4 red[2][RB][LPR + 1];
  const int cq = threadIdx.x % LPR, rl = threadIdx.x / LPR;
  const int col = (blockIdx.x * LPR + cq) * 4;
  const int s = blockIdx.y, g = blockIdx.z, S = gridDim.y;
  const long long r0 = (long long)g * Mg + (long long)s * rps;
  const long long r1 = min((long long)g * Mg + Mg, r0 + rps);
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, bs = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    const f32x4 mu = *(const f32x4*)(mean + g * C + col), rs = *(const f32x4*)(rstd + g * C + col);
    const f32x4 ga = *(const f32x4*)(gamma + col), be = *(const f32x4*)(beta + col);
    auto step = [&](f32x4 yv, f32x4 dv) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (yv[e] - mu[e]) * rs[e];
        const float z = xh * ga[e] + be[e];
        const float dz = z > 0.f ? dv[e] : 0.f;
        a[e] += dz;
        bs[e] += dz * xh;
      }
    };
    long long r = r0 + rl;
    for (; r + 3 * RB < r1; r += 4 * RB) {
      f32x4 yv[4], dv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        yv[k] = *(const f32x4*)(y + (r + k * RB) * ldy + col);
        dv[k] = *(const f32x4*)(dout + (r + k * RB) * ldd + col);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) step(yv[k], dv[k]);
    }
    for (; r < r1; r += RB)
      step(*(const f32x4*)(y + r * ldy + col), *(const f32x4*)(dout + r * ldd + col));
  }
  red[0][rl][cq] = a;
  red[1][rl][cq] = bs;
  __syncthreads();
  if (rl == 0 && col < C) {
    f32x4 ta = red[0][0][cq], tb = red[1][0][cq];
#pragma unroll
    for (int i = 1; i < RB; ++i) {
      ta += red[0][i][cq];
      tb += red[1][i][cq];
    }
    float* p = part + (((long long)g * S + s) * 2) * C;
    *(f32x4*)(p + col) = ta;
    *(f32x4*)(p + C + col) = tb;
  }
}

// sums[g][0|1][c] = sum_s part; dgamma[c] += sum_g sums1, dbeta[c] += sum_g sums0
// grid (ceil(C/64), G), 1024 threads: 16 lane rows split the S partials of 64 channels
// (s = row, row + 16, ...), then fold in a fixed order; one workgroup per group g (a
// single-workgroup serial sum over S ~ 480 splits took 63 us on the branch's chain).
__global__ __launch_bounds__(1024) void bn_bwd_final_kernel(
    const float* __restrict__ part, int S, int C, float* __restrict__ sums) {  // sums[g][2][C]
  __shared__ double red[2][16][65];
  const int cl = threadIdx.x & 63, row = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, g = blockIdx.y;
  double a = 0.0, b = 0.0;
  if (c < C)
#pragma unroll 4  // the loads of four splits in flight (the adds keep their order: same bits)
    for (int s = row; s < S; s += 16) {
      a += part[(((long long)g * S + s) * 2) * C + c];
      b += part[(((long long)g * S + s) * 2 + 1) * C + c];
    }
  red[0][row][cl] = a;
  red[1][row][cl] = b;
  __syncthreads();
  if (row == 0 && c < C) {
    double ta = 0.0, tb = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      ta += red[0][r][cl];
      tb += red[1][r][cl];
    }
    sums[(g * 2) * C + c] = (float)ta;
    sums[(g * 2 + 1) * C + c] = (float)tb;
  }
}

// dgamma[c] += sum_g sum dz*xhat, dbeta[c] += sum_g sum dz (groups in order)
__global__ void bn_param_grad_kernel(const float* __restrict__ sums, int G, int C,
                                     float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double tg = 0.0, tb = 0.0;
  for (int g = 0; g < G; ++g) {
    tb += sums[(g * 2) * C + c];
    tg += sums[(g * 2 + 1) * C + c];
  }
  dgamma[c] += (float)tg;
  dbeta[c] += (float)tb;
}

// dy = gamma * rstd / Mg * (Mg * dz - sum dz - xhat * sum dz*xhat)
__global__ void bn_bwd_apply_kernel(const float* __restrict__ dout, int ldd,
                                    const float* __restrict__ y, int ldy, long long M, int C,
                                    long long Mg, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, const float* __restrict__ sums,
                                    float* __restrict__ dy, int lddy) {
  GRID_LOOP(i, M * C) {
    const long long m = i / C;
    const int c = (int)(i % C);
    const int g = (int)(m / Mg);
    const float rs = rstd[g * C + c];
    const float xh = (y[m * ldy + c] - mean[g * C + c]) * rs;
    const float z = xh * gamma[c] + beta[c];
    const float dz = z > 0.f ? dout[m * ldd + c] : 0.f;
    const float s0 = sums[(g * 2) * C + c], s1 = sums[(g * 2 + 1) * C + c];
    dy[m * lddy + c] = gamma[c] * rs * (dz - (s0 + xh * s1) / (float)Mg);
  }
}

// Frozen (eval-mode) BatchNorm under training: mean / rstd are the running statistics,
// constants of the step, so dy = gamma * rstd * dz (dz = dout * (z > 0)).
__global__ void bn_bwd_apply_frozen_kernel(const float* __restrict__ dout, int ldd,
                                           const float* __restrict__ y, int ldy, long long M,
                                           int C, const float* __restrict__ mean,
                                           const float* __restrict__ rstd,
                                           const float* __restrict__ gamma,
                                           const float* __restrict__ beta,
                                           float* __restrict__ dy, int lddy) {
  GRID_LOOP(i, M * C) {
    const long long m = i / C;
    const int c = (int)(i % C);
    const float rs = rstd[c];
    const float z = (y[m * ldy + c] - mean[c]) * rs * gamma[c] + beta[c];
    const float dz = z > 0.f ? dout[m * ldd + c] : 0.f;
    dy[m * lddy + c] = gamma[c] * rs * dz;
  }
}

// bn_bwd_apply_kernel, four channels per lane (the bn_apply_relu4_kernel conditions)
__global__ void bn_bwd_apply4_kernel(const float* __restrict__ dout, int ldd,
                                     const float* __restrict__ y, int ldy, int M, int C, int Mg,
                                     const float* __restrict__ mean,
                                     const float* __restrict__ rstd,
                                     const float* __restrict__ gamma,
                                     const float* __restrict__ beta,
                                     const float* __restrict__ sums, float* __restrict__ dy,
                                     int lddy, __bf16* __restrict__ dyb, int lddyb) {
  const int C4 = C >> 2, n = M * C4;
  const float fMg = (float)Mg;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const int m = q / C4, c = (q - m * C4) * 4, g = m / Mg;
    const f32x4 yv = *(const f32x4*)(y + (long long)m * ldy + c);
    const f32x4 dv = *(const f32x4*)(dout + (long long)m * ldd + c);
    const f32x4 mu = *(const f32x4*)(mean + g * C + c), rs = *(const f32x4*)(rstd + g * C + c);
    const f32x4 ga = *(const f32x4*)(gamma + c), be = *(const f32x4*)(beta + c);
    const f32x4 s0 = *(const f32x4*)(sums + (g * 2) * C + c);
    const f32x4 s1 = *(const f32x4*)(sums + (g * 2 + 1) * C + c);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (yv[j] - mu[j]) * rs[j];
      const float z = xh * ga[j] + be[j];
      const float dz = z > 0.f ? dv[j] : 0.f;
      o[j] = ga[j] * rs[j] * (dz - (s0[j] + xh * s1[j]) / fMg);
    }
    *(f32x4*)(dy + (long long)m * lddy + c) = o;
    if (dyb) store_bf16x4(dyb + (long long)m * lddyb + c, o);
  }
}

// ------------------------------------------------------------- DiffNet head
// out[b][j] = sin(t_b * e_j) (j < C/2), cos(...) (j >= C/2); e_j = exp(-j ln(1e4)/(C/2-1))
__global__ void sinusoidal_kernel(const long long* __restrict__ t, int B, int C,
                                  float* __restrict__ out) {
  GRID_LOOP(i, (long long)B * C) {
    const int b = (int)(i / C), j = (int)(i % C);
    const int half = C / 2;
    const int jj = j < half ? j : j - half;
    const float scale = logf(10000.f) / (float)(half - 1);
    const float e = expf((float)jj * -scale);
    const float a = (float)t[b] * e;
    out[i] = j < half ? sinf(a) : cosf(a);
  }
}

__device__ __forceinline__ float softplus_(float x) {
  return x > 20.f ? x : log1pf(expf(x));  // torch softplus, beta 1, threshold 20
}

// y = x * tanh(softplus(x))  (denoiser.py:9-11)
__global__ void mish_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long long n) {
  GRID_LOOP(i, n) {
    const float v = x[i];
    y[i] = v * tanhf(softplus_(v));
  }
}

__global__ void mish_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                float* __restrict__ dx, long long n) {
  GRID_LOOP(i, n) {
    const float v = x[i];
    const float sp = softplus_(v);
    const float tsp = tanhf(sp);
    const float sig = v > 20.f ? 1.f : 1.f / (1.f + expf(-v));
    dx[i] = dy[i] * (tsp + v * (1.f - tsp * tsp) * sig);
  }
}

// ------------------------------------------------------------- diffusion
// xn[m][j] = sa[t_b] * y[m][j] / ns + s1ma[t_b] * noise[m][j]   (diffusion.py:261-267, 289-295)
__global__ void q_sample_kernel(const float* __restrict__ y, int ldy, const float* __restrict__ noise,
                                int ldn, const long long* __restrict__ t,
                                const float* __restrict__ sa, const float* __restrict__ s1ma,
                                long long M, int Mc, int T, float inv_ns, float* __restrict__ xn,
                                int ldx) {
  GRID_LOOP(i, M * Mc) {
    const long long m = i / Mc;
    const int j = (int)(i % Mc);
    const long long tb = t[m / T];
    xn[m * ldx + j] = sa[tb] * (y[m * ldy + j] * inv_ns) + s1ma[tb] * noise[m * ldn + j];
  }
}

// One reverse step (diffusion.py:170-204) at scalar step i:
// x_recon = clamp(sra*x - srm1*eps, -1, 1); x = c1*x_recon + c2*x + nz*exp(.5 logvar)*noise
__global__ void p_sample_kernel(float* __restrict__ x, const float* __restrict__ eps,
                                const float* __restrict__ noise, long long n, float sra,
                                float srm1, float c1, float c2, float sigma) {
  GRID_LOOP(i, n) {
    const float xv = x[i];
    float xr = sra * xv - srm1 * eps[i];
    xr = fminf(fmaxf(xr, -1.f), 1.f);
    x[i] = (c1 * xr + c2 * xv) + sigma * noise[i];
  }
}

// p_sample over M rows of Mc channels that also writes the next DiffNet input projection's
// bf16 operand: xb[m][k] = bf16(x[m][k]) for k < Mc, 0 for Mc <= k < ldb (the K padding the
// 16-B operand chunks read).  eps == nullptr: no update, only the copy (the first step's x).
__global__ void p_sample_bf16_kernel(float* __restrict__ x, const float* __restrict__ eps,
                                     const float* __restrict__ noise, long long M, int Mc,
                                     float sra, float srm1, float c1, float c2, float sigma,
                                     __bf16* __restrict__ xb, int ldb) {
  GRID_LOOP(i, M * ldb) {
    const long long m = i / ldb;
    const int k = (int)(i - m * ldb);
    float v = 0.f;
    if (k < Mc) {
      const long long j = m * Mc + k;
      v = x[j];
      if (eps) {
        float xr = sra * v - srm1 * eps[j];
        xr = fminf(fmaxf(xr, -1.f), 1.f);
        v = (c1 * xr + c2 * v) + sigma * noise[j];
        x[j] = v;
      }
    }
    xb[i] = (__bf16)v;
  }
}

// ------------------------------------------------------------- loss
struct LossStream {
  const float* a;  // prediction (or x_recon)
  const float* b;  // target (or noise)
  float* ga;       // gradient w.r.t. a (written)
  int lda, ldb, ldg, n;
};
struct LossArgs {
  LossStream s[4];
  int ns, T, B;
  float invN, gscale;
};

// loss partial sums of |a - b| over non-padded frames; ga = gscale * sign(a - b) (0 on padding).
__global__ void masked_l1_kernel(LossArgs a, const long long* __restrict__ lengths,
                                 float* __restrict__ part) {
  __shared__ float red[256];
  float acc = 0.f;
  const long long M = (long long)a.B * a.T;
  for (int k = 0; k < a.ns; ++k) {
    const LossStream& s = a.s[k];
    GRID_LOOP(i, M * s.n) {
      const long long m = i / s.n;
      const int j = (int)(i % s.n);
      const int t = (int)(m % a.T);
      const long long b = m / a.T;
      float g = 0.f;
      if (t < lengths[b]) {
        const float d = s.a[m * s.lda + j] - s.b[m * s.ldb + j];
        acc += fabsf(d);
        g = d > 0.f ? a.gscale : (d < 0.f ? -a.gscale : 0.f);
      }
      if (s.ga) s.ga[m * s.ldg + j] = g;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void sum_partials_kernel(const float* __restrict__ part, int n, float scale,
                                    float* __restrict__ out) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] * scale);
}

// ------------------------------------------------------------- optimizer
__global__ void sumsq_kernel(const float* __restrict__ x, long long n, float* __restrict__ part) {
  __shared__ float red[256];
  float acc = 0.f;
  GRID_LOOP(i, n) {
    const float v = x[i];
    acc = fmaf(v, v, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// The same over 16-B aligned x: float4 loads, two in flight per thread with their own
// accumulators (the scalar loop above walked ~90 dependent loads per thread: 42 us for the
// 94 MB gradient buffer)
__global__ __launch_bounds__(256) void sumsq4_kernel(const float* __restrict__ x, long long n,
                                                     float* __restrict__ part) {
  __shared__ float red[256];
  const long long n4 = n >> 2, stride = (long long)gridDim.x * 256;
  const f32x4* x4 = (const f32x4*)x;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const f32x4 u = x4[i], w = x4[i + stride];
    a += u * u;
    b += w * w;
  }
  if (i < n4) {
    const f32x4 u = x4[i];
    a += u * u;
  }
  float acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const float v = x[4 * n4 + threadIdx.x];
    acc = fmaf(v, v, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

static void launch_sumsq(const float* x, long long n, float* part, int blocks, hipStream_t st) {
  if (((uintptr_t)x & 15) == 0)
    hipLaunchKernelGGL(sumsq4_kernel, dim3(blocks), dim3(256), 0, st, x, n, part);
  else
    hipLaunchKernelGGL(sumsq_kernel, dim3(blocks), dim3(256), 0, st, x, n, part);
}

__global__ void norm_final_kernel(const float* __restrict__ part, int n, float* __restrict__ out,
                                  unsigned* __restrict__ err) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  // a failed cooperative recurrence (coop.h error word) makes the norm NaN: the update skips.
  // The word is snapshotted and cleared here, once per step: err[0] (the live word the
  // recurrences OR into) moves into err[1] (failed steps, cleared by the host when it raises),
  // so steps enqueued after a failure run their own updates normally.
  if (threadIdx.x == 0) {
    const unsigned e = err ? err[0] : 0u;
    out[0] = e ? __builtin_nanf("") : (float)sqrt(red[0]);
    if (e) {
      err[1] += 1u;
      err[0] = 0u;
    }
  }
}

// data parallel: a rank whose cooperative recurrence failed writes NaN into one gradient
// element before the all-reduce, so every rank's norm is NaN and every rank skips the update
__global__ void poison_kernel(const unsigned* __restrict__ err, float* __restrict__ x) {
  if (threadIdx.x == 0 && *err) x[0] = __builtin_nanf("");
}

// clip_grad_norm_(max_norm) then torch.optim.Adam (weight_decay 0, amsgrad off);
// skipped entirely when the norm is not finite (train_acoustic_multitrack.py:369-380).
// `st` (device-side optimizer state, see adam_prepare_kernel) replaces the host scalars
// lr / bc1 and sqrt_bc2 when given, so the update can be replayed from a HIP graph.
__global__ void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, const float* __restrict__ norm,
                            float max_norm, float lr, float b1, float b2, float eps, float bc1,
                            float sqrt_bc2, const double* __restrict__ st) {
  const float nv = norm[0];
  if (!isfinite(nv)) return;
  const float coef = fminf(max_norm / (nv + 1e-6f), 1.f);
  const float step = st ? (float)st[1] : lr / bc1;
  if (st) sqrt_bc2 = (float)st[2];
  GRID_LOOP(i, n) {
    const float gi = g[i] * coef;
    g[i] = gi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / sqrt_bc2 + eps;
    p[i] = p[i] - step * (mi / denom);
  }
}

// Device-side Adam step counter: st = {step, lr / (1 - b1^step), sqrt(1 - b2^step), lr}.
// The step only advances when the gradient norm is finite, like torch.optim.Adam whose
// step() the reference skips on a non-finite norm (train_acoustic_multitrack.py:365-380);
// the bias corrections are the reference's double-precision Python scalars.
__global__ void adam_prepare_kernel(const float* __restrict__ norm, double* __restrict__ st,
                                    double b1, double b2) {
  if (threadIdx.x != 0 || !isfinite(norm[0])) return;
  const double c = st[0] + 1.0;
  st[0] = c;
  st[1] = st[3] / (1.0 - pow(b1, c));
  st[2] = sqrt(1.0 - pow(b2, c));
}

__global__ void copy_cols_kernel(const float* __restrict__ src, int lds, float* __restrict__ dst,
                                 int ldd, long long M, int n) {
  GRID_LOOP(i, M * n) {
    const long long m = i / n;
    const int j = (int)(i % n);
    dst[m * ldd + j] = src[m * lds + j];
  }
}

// dst[m][b*dw + c] = c < sw ? src[m][b*sw + c] : 0 for b < nblk, c < dw: per-gate column blocks
// widened (zero pad) or narrowed (the LSTM hidden sizes run by a padded persistent kernel)
__global__ void regroup_cols_kernel(const float* __restrict__ src, int lds, float* __restrict__ dst,
                                    int ldd, long long M, int nblk, int sw, int dw) {
  const long long per = (long long)nblk * dw;
  GRID_LOOP(i, M * per) {
    const long long m = i / per;
    const int j = (int)(i % per), b = j / dw, c = j % dw;
    dst[m * ldd + j] = c < sw ? src[m * lds + (long long)b * sw + c] : 0.f;
  }
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, float a,
                            long long n) {
  GRID_LOOP(i, n) y[i] += a * x[i];
}

// y[g*ystride + j] += a * x[g*xstride + j], g < count, j < n: one launch for the same-shaped
// parameters of several layers (their gradients sit at a constant stride in the flat buffer)
__global__ void axpy_strided_kernel(float* __restrict__ y, long long ystride,
                                    const float* __restrict__ x, long long xstride, float a,
                                    int n, int count) {
  GRID_LOOP(i, (long long)n * count) {
    const long long g = i / n, j = i - g * n;
    y[g * ystride + j] += a * x[g * xstride + j];
  }
}

// y[g*ystride + r*yld + c] += a * x[g*xstride + r*xld + c]: one 2-D block per destination
__global__ void axpy_blocks2d_kernel(float* __restrict__ y, long long ystride, long long yld,
                                     const float* __restrict__ x, long long xstride,
                                     long long xld, float a, int rows, int cols, int count) {
  GRID_LOOP(i, (long long)rows * cols * count) {
    const long long per = (long long)rows * cols;
    const long long g = i / per, rc = i - g * per;
    const long long r = rc / cols, c = rc - r * cols;
    y[g * ystride + r * yld + c] += a * x[g * xstride + r * xld + c];
  }
}

// DiffNet residual-half output-projection bias grads from the per-block column sums of the
// dilated-conv input grads: s_l = colsum(dx_l) = a * s_l+1 + cdy[l], bias_l-1 += a * s_l
// (dx_l = a * dx_l+1 + dy_l, a = 1/sqrt2; block l-1's residual output feeds dx_l).
__global__ void res_bias_grad_kernel(const float* __restrict__ cdy, int L, int C,
                                     float* __restrict__ dst, long long dstride, float a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int l = L - 1; l >= 1; --l) {
    s = a * s + cdy[(long long)l * C + c];
    dst[(long long)(l - 1) * dstride + c] += a * s;
  }
}

__global__ void axpby_kernel(float* __restrict__ y, float a, const float* __restrict__ x, float b,
                             long long n) {
  GRID_LOOP(i, n) y[i] = __builtin_fmaf(a, y[i], b * x[i]);
}

// out = a * y + b * x (the same expression as axpby_kernel, out of place), and an
// optional bf16 shadow of out for the GEMM that reads it next
__global__ void axpby_to_kernel(float* __restrict__ out, __bf16* __restrict__ outb,
                                const float* __restrict__ y, float a, const float* __restrict__ x,
                                float b, long long n) {
  GRID_LOOP(i, n) {
    const float v = __builtin_fmaf(a, y[i], b * x[i]);  // = the GEMM ADDSCALE epilogue
    out[i] = v;
    if (outb) outb[i] = (__bf16)v;
  }
}

__global__ void mul_kernel(float* __restrict__ y, const float* __restrict__ x, long long n) {
  GRID_LOOP(i, n) y[i] *= x[i];
}

__global__ void relu_mask_kernel(float* __restrict__ out, const float* __restrict__ dy,
                                 const float* __restrict__ act, long long n) {
  GRID_LOOP(i, n) out[i] = act[i] > 0.f ? dy[i] : 0.f;
}

// the same, four elements per lane, plus the bf16 copy (n % 4 == 0, 16-B aligned)
__global__ void relu_mask4_kernel(float* __restrict__ out, __bf16* __restrict__ outb,
                                  const float* __restrict__ dy, const float* __restrict__ act,
                                  long long n4) {
  GRID_LOOP(q, n4) {
    const f32x4 a = *(const f32x4*)(act + 4 * q), d = *(const f32x4*)(dy + 4 * q);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = a[j] > 0.f ? d[j] : 0.f;
    *(f32x4*)(out + 4 * q) = o;
    store_bf16x4(outb + 4 * q, o);
  }
}

__global__ void mul_out_kernel(float* __restrict__ out, const float* __restrict__ a,
                               const float* __restrict__ b, long long n) {
  GRID_LOOP(i, n) out[i] = a[i] * b[i];
}

__global__ void reflect_fold_kernel(const float* __restrict__ dxp, int B, int T, int pad, int C,
                                    float* __restrict__ dx) {
  const int Tp = T + 2 * pad;
  GRID_LOOP(i, (long long)B * T * C) {
    const int c = (int)(i % C);
    const long long bt = i / C;
    const int t = (int)(bt % T);
    const long long b = bt / T;
    const float* src = dxp + b * Tp * C + c;
    float v = src[(long long)(t + pad) * C];
    if (t >= 1 && t <= pad) v += src[(long long)(pad - t) * C];
    if (t >= T - 1 - pad && t <= T - 2) v += src[(long long)(2 * (T - 1) - t + pad) * C];
    dx[i] = v;
  }
}

// ---- counter-based RNG: a 64-bit mix of (seed, index) (splitmix64 finaliser) ----
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Replay epoch of the RNG kernels: 0 (the eager default) leaves every seed as given; a
// captured training step advances it once per replay so each replay draws fresh numbers.
__device__ unsigned long long g_rng_epoch = 0ull;
__device__ __forceinline__ unsigned long long epoch_seed(unsigned long long seed) {
  const unsigned long long e = g_rng_epoch;
  return e ? seed ^ mix64(e * 0xD1B54A32D192ED03ull) : seed;
}
__device__ __forceinline__ float u01(unsigned long long r) {  // (0, 1]
  return ((float)(r >> 40) + 1.f) * (1.f / 16777216.f);
}

__global__ void rng_advance_kernel() {
  if (threadIdx.x == 0) g_rng_epoch += 1ull;
}

__global__ void randn_kernel(float* __restrict__ out, long long n, unsigned long long seed) {
  seed = epoch_seed(seed);
  GRID_LOOP(i, n) {
    const unsigned long long r = mix64(seed ^ mix64((unsigned long long)i));
    const float u1 = u01(r), u2 = u01(r << 24 | r >> 40);
    out[i] = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
  }
}

__global__ void dropout_mask_kernel(float* __restrict__ out, long long n, float p,
                                    unsigned long long seed) {
  const float keep = 1.f / (1.f - p);
  seed = epoch_seed(seed);
  GRID_LOOP(i, n) {
    const unsigned long long r = mix64(seed ^ mix64((unsigned long long)i));
    out[i] = u01(r) > p ? keep : 0.f;
  }
}

__global__ void randint_kernel(long long* __restrict__ out, long long n, long long hi,
                               unsigned long long seed) {
  seed = epoch_seed(seed);
  GRID_LOOP(i, n) {
    const unsigned long long r = mix64(seed ^ mix64((unsigned long long)i));
    out[i] = (long long)((r >> 11) % (unsigned long long)hi);
  }
}

}  // namespace

#define LAUNCH(kernel, n, ...)                                                                  \
  do {                                                                                          \
    hipLaunchKernelGGL(kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
    ENSVS_CHECK_LAUNCH();                                                                       \
  } while (0)

// four-channel lanes for the BatchNorm elementwise passes: see bn_apply_relu4_kernel
static bool bn_vec4(int C, std::initializer_list<int> lds, std::initializer_list<const void*> ps,
                    long long M) {
  if (C % 4 != 0 || M * (long long)C >= (1ll << 31)) return false;
  for (int l : lds)
    if (l % 4 != 0) return false;
  for (const void* p : ps)
    if ((uintptr_t)p % 16 != 0) return false;
  return true;
}

ENSVS_API int ensvs_phoneme_ids(const float* x, int ld, long long M, int ph0, int nv, int* ids,
                                void* stream) {
  if (M <= 0 || nv <= 0) return ENSVS_E_SHAPE;
  if (nv <= PH_MAXV && M < (1ll << 31)) {
    hipLaunchKernelGGL(phoneme_ids_tile_kernel, dim3((unsigned)((M + PH_ROWS - 1) / PH_ROWS)),
                       dim3(256), 0, (hipStream_t)stream, x, ld, (int)M, ph0, nv, ids);
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  LAUNCH(phoneme_ids_kernel, M, x, ld, M, ph0, nv, ids);
  return ENSVS_OK;
}

ENSVS_API int ensvs_embed_add(float* y, int ldy, long long M, int C, int T, const float* emb,
                              const int* ids0, const int* ids1, const float* spk0,
                              const float* spk1, int ldspk, void* stream) {
  if (M <= 0 || C <= 0 || T <= 0) return ENSVS_E_SHAPE;
  if (M < (1ll << 31)) {
    const bool vec = C % 4 == 0 && ldy % 4 == 0 && (!(spk0 || spk1) || ldspk % 4 == 0) &&
                     (((uintptr_t)y | (uintptr_t)emb | (uintptr_t)spk0 | (uintptr_t)spk1) & 15) == 0;
    const dim3 grid((unsigned)std::min<long long>(2048, (M + 3) / 4));
    if (vec)
      hipLaunchKernelGGL(embed_add_rows_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, y,
                         ldy, (int)M, C, T, emb, ids0, ids1, spk0, spk1, ldspk);
    else
      hipLaunchKernelGGL(embed_add_rows_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, y,
                         ldy, (int)M, C, T, emb, ids0, ids1, spk0, spk1, ldspk);
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  LAUNCH(embed_add_kernel, M * C, y, ldy, M, C, T, emb, ids0, ids1, spk0, spk1, ldspk);
  return ENSVS_OK;
}

ENSVS_API long long ensvs_embed_bwd_workspace(long long M, int C, int V) {
  return (M + EMB_CHUNK - 1) / EMB_CHUNK * (long long)V * C;
}

ENSVS_API int ensvs_embed_bwd(const float* dy, int ldy, long long M, int C, const int* ids, int V,
                              float* part, float* demb, void* stream) {
  if (V <= 0 || V > 128 || M <= 0 || C <= 0) return ENSVS_E_SHAPE;
  const int nchunk = (int)((M + EMB_CHUNK - 1) / EMB_CHUNK);
  if (nchunk > 65535) return ENSVS_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(cdiv(C, 64), nchunk), dim3(256),
                     4 * V * 64 * sizeof(float), st, dy, ldy, M, C, ids, V, part);
  ENSVS_CHECK_LAUNCH();
  const long long VC = (long long)V * C;
  LAUNCH(embed_reduce_kernel, VC, part, nchunk, VC, demb);
  return ENSVS_OK;
}

ENSVS_API int ensvs_spk_scatter(const float* dseq, int B, int C, const long long* spk, float* dtab,
                                void* stream) {
  LAUNCH(spk_scatter_kernel, (long long)B * C, dseq, B, C, spk, dtab);
  return ENSVS_OK;
}

ENSVS_API int ensvs_gather_rows(const float* table, const long long* idx, int B, int C, float* out,
                                void* stream) {
  LAUNCH(gather_rows_kernel, (long long)B * C, table, idx, B, C, out);
  return ENSVS_OK;
}

ENSVS_API int ensvs_bn_finalize(float* mean, float* var, int G, int C, long long Mg, float eps,
                                float* rstd, float* rmean, float* rvar, float momentum, int update,
                                void* stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream,
                     mean, var, G, C, Mg, eps, rstd, rmean, rvar, momentum, update);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// row splits of ensvs_bn_stats (as the column sums: >= ~2048 blocks, >= 128 rows per split)
static int bn_stats_splits(long long Mg, int C, int G) {
  return (int)std::max<long long>(
      1, std::min<long long>({(long long)BN_STATS_MAX_SPLITS, Mg / 128,
                              (long long)cdiv(2048, cdiv(C, 64) * G)}));
}

ENSVS_API long long ensvs_bn_stats_part_floats(long long M, int C, long long Mg) {
  if (M <= 0 || C <= 0 || Mg <= 0 || M % Mg) return 0;
  const int G = (int)(M / Mg);
  return (long long)G * bn_stats_splits(Mg, C, G) * 2 * C;
}

ENSVS_API int ensvs_bn_stats(const float* y, int ldy, long long M, int C, long long Mg,
                             float* part, long long part_floats, float eps, float* mean, float* var,
                             float* rstd, float* rmean, float* rvar, float momentum, int updates,
                             long long* nbt, void* stream) {
  if (M <= 0 || C <= 0 || Mg <= 0 || M % Mg || ldy < C || Mg > INT32_MAX) return ENSVS_E_SHAPE;
  const int G = (int)(M / Mg);
  const int S = bn_stats_splits(Mg, C, G);
  if (!part || part_floats < (long long)G * S * 2 * C || !mean || !var || !rstd) return ENSVS_E_ARG;
  if (updates > 0 && (!rmean || !rvar)) return ENSVS_E_ARG;
  const int rps = (int)cdiv(Mg, (long long)S);
  const int vec = (ldy % 4 == 0) && (((uintptr_t)y & 15) == 0);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_stats_partial_kernel, dim3(cdiv(C, 64), S, G), dim3(256), 0, st, y, ldy,
                     (int)Mg, C, rps, vec, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(cdiv(C, 16)), dim3(256), 0, st, part, S, G, C,
                     (int)Mg, rps, eps, mean, var, rstd, rmean, rvar, momentum, updates, nbt);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_bn_apply_relu(const float* y, int ldy, long long M, int C, long long Mg,
                                  const float* mean, const float* rstd, const float* gamma,
                                  const float* beta, float* out, int ldo, void* outb, int ldob,
                                  void* stream) {
  if (bn_vec4(C, {ldy, ldo}, {y, out, mean, rstd, gamma, beta}, M) &&
      (!outb || (ldob % 4 == 0 && (uintptr_t)outb % 8 == 0))) {
    LAUNCH(bn_apply_relu4_kernel, M * C / 4, y, ldy, (int)M, C, (int)Mg, mean, rstd, gamma, beta,
           out, ldo, (__bf16*)outb, ldob);
    return ENSVS_OK;
  }
  if (outb) return ENSVS_E_ARG;  // the bf16 copy needs the four-channel layout
  LAUNCH(bn_apply_relu_kernel, M * C, y, ldy, M, C, Mg, mean, rstd, gamma, beta, out, ldo);
  return ENSVS_OK;
}

// part: G*S*2*C floats (S <= max_splits), sums: G*2*C floats
ENSVS_API int ensvs_bn_bwd(const float* dout, int ldd, const float* y, int ldy, long long M, int C,
                           long long Mg, const float* mean, const float* rstd, const float* gamma,
                           const float* beta, float* part, int max_splits, float* sums,
                           float* dgamma, float* dbeta, float* dy, int lddy, void* dyb, int lddyb,
                           void* stream) {
  if (dyb && !(bn_vec4(C, {ldd, ldy, lddy}, {dout, y, dy, mean, rstd, gamma, beta, sums}, M) &&
               lddyb % 4 == 0 && (uintptr_t)dyb % 8 == 0))
    return ENSVS_E_ARG;  // the bf16 copy needs the four-channel layout
  hipStream_t st = (hipStream_t)stream;
  const int G = (int)(M / Mg);
  int S = (int)std::max<long long>(1, std::min<long long>(max_splits, Mg / 64));
  int rps = (int)((Mg + S - 1) / S);
  if (bn_vec4(C, {ldd, ldy}, {dout, y, mean, rstd, gamma, beta, part}, M)) {
    if (C >= 256)
      hipLaunchKernelGGL(bn_bwd_reduce4_kernel<64>, dim3(cdiv(C, 256), S, G), dim3(256), 0, st,
                         dout, ldd, y, ldy, Mg, C, mean, rstd, gamma, beta, rps, part);
    else if (C >= 128)
      hipLaunchKernelGGL(bn_bwd_reduce4_kernel<32>, dim3(cdiv(C, 128), S, G), dim3(256), 0, st,
                         dout, ldd, y, ldy, Mg, C, mean, rstd, gamma, beta, rps, part);
    else
      hipLaunchKernelGGL(bn_bwd_reduce4_kernel<16>, dim3(cdiv(C, 64), S, G), dim3(256), 0, st,
                         dout, ldd, y, ldy, Mg, C, mean, rstd, gamma, beta, rps, part);
  } else {
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(cdiv(C, 64), S, G), dim3(256), 0, st, dout, ldd,
                       y, ldy, Mg, C, mean, rstd, gamma, beta, rps, part);
  }
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, 64), G), dim3(1024), 0, st, part, S, C,
                     sums);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, G, C, dgamma,
                     dbeta);
  ENSVS_CHECK_LAUNCH();
  if (bn_vec4(C, {ldd, ldy, lddy}, {dout, y, dy, mean, rstd, gamma, beta, sums}, M)) {
    LAUNCH(bn_bwd_apply4_kernel, M * C / 4, dout, ldd, y, ldy, (int)M, C, (int)Mg, mean, rstd,
           gamma, beta, sums, dy, lddy, (__bf16*)dyb, lddyb);
    return ENSVS_OK;
  }
  LAUNCH(bn_bwd_apply_kernel, M * C, dout, ldd, y, ldy, M, C, Mg, mean, rstd, gamma, beta, sums, dy,
         lddy);
  return ENSVS_OK;
}

// BatchNorm1d in eval mode inside a training step (frozen statistics, e.g. the data-parallel
// parity definition of SURVEY 8(e)): dgamma / dbeta accumulate as in ensvs_bn_bwd (one group),
// the input gradient has no batch-statistic terms.
ENSVS_API int ensvs_bn_bwd_frozen(const float* dout, int ldd, const float* y, int ldy, long long M,
                                  int C, const float* mean, const float* rstd, const float* gamma,
                                  const float* beta, float* part, int max_splits, float* sums,
                                  float* dgamma, float* dbeta, float* dy, int lddy, void* stream) {
  if (M <= 0 || C <= 0) return ENSVS_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int S = (int)std::max<long long>(1, std::min<long long>(max_splits, M / 64));
  const int rps = (int)((M + S - 1) / S);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(cdiv(C, 64), S, 1), dim3(256), 0, st, dout, ldd, y,
                     ldy, M, C, mean, rstd, gamma, beta, rps, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, 64), 1), dim3(1024), 0, st, part, S, C,
                     sums);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, 1, C, dgamma,
                     dbeta);
  ENSVS_CHECK_LAUNCH();
  LAUNCH(bn_bwd_apply_frozen_kernel, M * C, dout, ldd, y, ldy, M, C, mean, rstd, gamma, beta, dy,
         lddy);
  return ENSVS_OK;
}

ENSVS_API int ensvs_sinusoidal(const long long* t, int B, int C, float* out, void* stream) {
  LAUNCH(sinusoidal_kernel, (long long)B * C, t, B, C, out);
  return ENSVS_OK;
}

ENSVS_API int ensvs_mish_fwd(const float* x, float* y, long long n, void* stream) {
  LAUNCH(mish_fwd_kernel, n, x, y, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_mish_bwd(const float* x, const float* dy, float* dx, long long n, void* stream) {
  LAUNCH(mish_bwd_kernel, n, x, dy, dx, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_q_sample(const float* y, int ldy, const float* noise, int ldn,
                             const long long* t, const float* sa, const float* s1ma, long long M,
                             int Mc, int T, float inv_ns, float* xn, int ldx, void* stream) {
  LAUNCH(q_sample_kernel, M * Mc, y, ldy, noise, ldn, t, sa, s1ma, M, Mc, T, inv_ns, xn, ldx);
  return ENSVS_OK;
}

ENSVS_API int ensvs_p_sample(float* x, const float* eps, const float* noise, long long n, float sra,
                             float srm1, float c1, float c2, float sigma, void* stream) {
  LAUNCH(p_sample_kernel, n, x, eps, noise, n, sra, srm1, c1, c2, sigma);
  return ENSVS_OK;
}

ENSVS_API int ensvs_p_sample_bf16(float* x, const float* eps, const float* noise, long long M,
                                  int Mc, float sra, float srm1, float c1, float c2, float sigma,
                                  void* xb, int ldb, void* stream) {
  if (ldb < Mc || ldb % 8 || ((uintptr_t)xb & 15)) return ENSVS_E_ARG;
  LAUNCH(p_sample_bf16_kernel, M * ldb, x, eps, noise, M, Mc, sra, srm1, c1, c2, sigma,
         (__bf16*)xb, ldb);
  return ENSVS_OK;
}

// streams: arrays of 4 (a, b, ga, lda, ldb, ldg, n); part >= 1024 floats; loss_out: 1 float
ENSVS_API int ensvs_masked_l1(const float* const* a, const float* const* b, float* const* ga,
                              const int* lda, const int* ldb, const int* ldg, const int* n, int ns,
                              const long long* lengths, int B, int T, float invN, float gscale,
                              float* part, float* loss_out, void* stream) {
  if (ns < 1 || ns > 4) return ENSVS_E_ARG;
  LossArgs args{};
  long long maxn = 0;
  for (int k = 0; k < ns; ++k) {
    args.s[k] = {a[k], b[k], ga[k], lda[k], ldb[k], ldg[k], n[k]};
    maxn = std::max<long long>(maxn, (long long)B * T * n[k]);
  }
  args.ns = ns;
  args.T = T;
  args.B = B;
  args.invN = invN;
  args.gscale = invN * gscale;
  int blocks = std::min(1024, grid_for(maxn));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(masked_l1_kernel, dim3(blocks), dim3(256), 0, st, args, lengths, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, part, blocks, invN, loss_out);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// norm_out[0] = ||x||_2 over n floats (part >= 1024 floats)
ENSVS_API int ensvs_l2norm(const float* x, long long n, float* part, float* norm_out, void* stream) {
  int blocks = std::min(1024, grid_for(n));
  hipStream_t st = (hipStream_t)stream;
  launch_sumsq(x, n, part, blocks, st);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(256), 0, st, part, blocks, norm_out,
                     (unsigned*)nullptr);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_l2norm_chk(const float* x, long long n, float* part, float* norm_out,
                               unsigned* err, void* stream) {
  int blocks = std::min(1024, grid_for(n));
  hipStream_t st = (hipStream_t)stream;
  launch_sumsq(x, n, part, blocks, st);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(256), 0, st, part, blocks, norm_out, err);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_poison_on_error(const unsigned* err, float* x, void* stream) {
  if (!err || !x) return ENSVS_E_ARG;
  hipLaunchKernelGGL(poison_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, err, x);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_adam(float* p, float* g, float* m, float* v, long long n, const float* norm,
                         float max_norm, float lr, float b1, float b2, float eps, float bc1,
                         float sqrt_bc2, void* stream) {
  LAUNCH(adam_kernel, n, p, g, m, v, n, norm, max_norm, lr, b1, b2, eps, bc1, sqrt_bc2,
         (const double*)nullptr);
  return ENSVS_OK;
}

ENSVS_API int ensvs_adam_step(float* p, float* g, float* m, float* v, long long n,
                              const float* norm, float max_norm, double b1, double b2, float eps,
                              double* state, void* stream) {
  if (!state) return ENSVS_E_ARG;
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, norm, state,
                     b1, b2);
  ENSVS_CHECK_LAUNCH();
  LAUNCH(adam_kernel, n, p, g, m, v, n, norm, max_norm, 0.f, (float)b1, (float)b2, eps, 1.f, 1.f,
         (const double*)state);
  return ENSVS_OK;
}

ENSVS_API int ensvs_rng_advance(void* stream) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_copy_cols(const float* src, int lds, float* dst, int ldd, long long M, int n,
                              void* stream) {
  LAUNCH(copy_cols_kernel, M * n, src, lds, dst, ldd, M, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_regroup_cols(const float* src, int lds, float* dst, int ldd, long long M,
                                 int nblk, int sw, int dw, void* stream) {
  if (M < 0 || nblk <= 0 || sw <= 0 || dw <= 0) return ENSVS_E_SHAPE;
  if (M == 0) return ENSVS_OK;
  LAUNCH(regroup_cols_kernel, M * nblk * dw, src, lds, dst, ldd, M, nblk, sw, dw);
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpy(float* y, const float* x, float a, long long n, void* stream) {
  LAUNCH(axpy_kernel, n, y, x, a, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpy_strided(float* y, long long ystride, const float* x, long long xstride,
                                 float a, int n, int count, void* stream) {
  if (n <= 0 || count <= 0) return ENSVS_OK;
  LAUNCH(axpy_strided_kernel, (long long)n * count, y, ystride, x, xstride, a, n, count);
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpy_blocks2d(float* y, long long ystride, long long yld, const float* x,
                                  long long xstride, long long xld, float a, int rows, int cols,
                                  int count, void* stream) {
  if (rows <= 0 || cols <= 0 || count <= 0) return ENSVS_OK;
  LAUNCH(axpy_blocks2d_kernel, (long long)rows * cols * count, y, ystride, yld, x, xstride, xld,
         a, rows, cols, count);
  return ENSVS_OK;
}

ENSVS_API int ensvs_res_bias_grad(const float* cdy, int L, int C, float* dst, long long dstride,
                                  float a, void* stream) {
  if (L <= 1 || C <= 0) return ENSVS_OK;
  hipLaunchKernelGGL(res_bias_grad_kernel, dim3((C + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, cdy, L, C, dst, dstride, a);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpby(float* y, float a, const float* x, float b, long long n, void* stream) {
  LAUNCH(axpby_kernel, n, y, a, x, b, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpby_to(float* out, const float* y, float a, const float* x, float b,
                             long long n, void* stream) {
  LAUNCH(axpby_to_kernel, n, out, (__bf16*)nullptr, y, a, x, b, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_axpby_to_bf16(float* out, void* outb, const float* y, float a, const float* x,
                                  float b, long long n, void* stream) {
  LAUNCH(axpby_to_kernel, n, out, (__bf16*)outb, y, a, x, b, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_mul(float* y, const float* x, long long n, void* stream) {
  LAUNCH(mul_kernel, n, y, x, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_reflect_fold(const float* dxp, int B, int T, int pad, int C, float* dx,
                                 void* stream) {
  if (pad >= T) return ENSVS_E_SHAPE;
  LAUNCH(reflect_fold_kernel, (long long)B * T * C, dxp, B, T, pad, C, dx);
  return ENSVS_OK;
}

ENSVS_API int ensvs_randn(float* out, long long n, unsigned long long seed, void* stream) {
  LAUNCH(randn_kernel, n, out, n, seed);
  return ENSVS_OK;
}

ENSVS_API int ensvs_dropout_mask(float* out, long long n, float p, unsigned long long seed,
                                 void* stream) {
  LAUNCH(dropout_mask_kernel, n, out, n, p, seed);
  return ENSVS_OK;
}

ENSVS_API int ensvs_randint(long long* out, long long n, long long hi, unsigned long long seed,
                            void* stream) {
  LAUNCH(randint_kernel, n, out, n, hi, seed);
  return ENSVS_OK;
}

ENSVS_API int ensvs_relu_mask(float* out, void* outb, const float* dy, const float* act,
                              long long n, void* stream) {
  if (outb) {
    if (n % 4 || (uintptr_t)out % 16 || (uintptr_t)dy % 16 || (uintptr_t)act % 16 ||
        (uintptr_t)outb % 8)
      return ENSVS_E_ARG;
    LAUNCH(relu_mask4_kernel, n / 4, out, (__bf16*)outb, dy, act, n / 4);
    return ENSVS_OK;
  }
  LAUNCH(relu_mask_kernel, n, out, dy, act, n);
  return ENSVS_OK;
}

ENSVS_API int ensvs_mul_out(float* out, const float* a, const float* b, long long n, void* stream) {
  LAUNCH(mul_out_kernel, n, out, a, b, n);
  return ENSVS_OK;
}

// ------------------------------------------------- log-F0 interaction loss
// bin/train_acoustic_multitrack.py:175-182 (logf0_diff_weight > 0, output_subtrack model):
//   sel(b, t) = t < len_b and vuv_main > 0 and vuv_sub > 0
//   L = mean_sel |(lf0_m - lf0_s) - (y_lf0_m - y_lf0_s)|,  loss_out += w * L
//   dL/dlf0_m = gscale * w * sign(.) / N_sel  (accumulated), dL/dlf0_s = - the same (written)
namespace {

__global__ __launch_bounds__(256) void lf0_int_partial_kernel(
    const float* __restrict__ pm, const float* __restrict__ ps, const float* __restrict__ ym,
    const float* __restrict__ ys, int ldy, int lf0_col, int vuv_col,
    const long long* __restrict__ lengths, int B, int T, float* __restrict__ part) {
  __shared__ float rs[256], rc[256];
  float s = 0.f, c = 0.f;
  GRID_LOOP(m, (long long)B * T) {
    const int t = (int)(m % T);
    const long long b = m / T;
    const float* a = ym + m * ldy;
    const float* q = ys + m * ldy;
    if (t < lengths[b] && a[vuv_col] > 0.f && q[vuv_col] > 0.f) {
      s += fabsf((pm[m] - ps[m]) - (a[lf0_col] - q[lf0_col]));
      c += 1.f;
    }
  }
  rs[threadIdx.x] = s;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
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

// one block: loss_out[0] += w * sum / count; coef[0] = gscale * w / count (inf when empty,
// as the reference's mean over an empty selection)
__global__ __launch_bounds__(256) void lf0_int_final_kernel(const float* __restrict__ part,
                                                            int n, float w, float gscale,
                                                            float* __restrict__ loss_out,
                                                            float* __restrict__ coef) {
  __shared__ double rs[256], rc[256];
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    s += part[2 * i];
    c += part[2 * i + 1];
  }
  rs[threadIdx.x] = s;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      rs[threadIdx.x] += rs[threadIdx.x + st];
      rc[threadIdx.x] += rc[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float cnt = (float)rc[0];
    loss_out[0] += w * ((float)rs[0] / cnt);
    coef[0] = gscale * w / cnt;
  }
}

__global__ void lf0_int_grad_kernel(const float* __restrict__ pm, const float* __restrict__ ps,
                                    const float* __restrict__ ym, const float* __restrict__ ys,
                                    int ldy, int lf0_col, int vuv_col,
                                    const long long* __restrict__ lengths, int B, int T,
                                    const float* __restrict__ coef, float* __restrict__ gm,
                                    float* __restrict__ gs) {
  const float k = coef[0];
  GRID_LOOP(m, (long long)B * T) {
    const int t = (int)(m % T);
    const long long b = m / T;
    const float* a = ym + m * ldy;
    const float* q = ys + m * ldy;
    float g = 0.f;
    if (t < lengths[b] && a[vuv_col] > 0.f && q[vuv_col] > 0.f) {
      const float d = (pm[m] - ps[m]) - (a[lf0_col] - q[lf0_col]);
      g = d > 0.f ? k : (d < 0.f ? -k : 0.f);
    }
    gm[m] += g;
    gs[m] = -g;
  }
}

}  // namespace

ENSVS_API int ensvs_lf0_interaction(const float* lf0_m, const float* lf0_s, const float* y_m,
                                    const float* y_s, int ldy, int lf0_col, int vuv_col,
                                    const long long* lengths, int B, int T, float weight,
                                    float gscale, float* part, float* loss_out, float* g_m,
                                    float* g_s, void* stream) {
  if (B <= 0 || T <= 0 || lf0_col >= ldy || vuv_col >= ldy) return ENSVS_E_SHAPE;
  const long long M = (long long)B * T;
  const int blocks = std::min(511, grid_for(M));  // part: 2*blocks partials + 1 coefficient
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lf0_int_partial_kernel, dim3(blocks), dim3(256), 0, st, lf0_m, lf0_s, y_m,
                     y_s, ldy, lf0_col, vuv_col, lengths, B, T, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(lf0_int_final_kernel, dim3(1), dim3(256), 0, st, part, blocks, weight,
                     gscale, loss_out, part + 1023);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(lf0_int_grad_kernel, dim3(grid_for(M)), dim3(256), 0, st, lf0_m, lf0_s, y_m,
                     y_s, ldy, lf0_col, vuv_col, lengths, B, T, part + 1023, g_m, g_s);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
