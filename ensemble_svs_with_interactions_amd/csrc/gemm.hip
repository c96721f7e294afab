// Implicit-GEMM engine for every dense contraction on the multi-track SVS
// path: Linear layers, Conv1d (any taps / dilation / zero-reflect-replicate
// padding), LSTM input projections, the DiffNet residual-block convolutions
// and their backward passes (dgrad = same kernel over transposed packed
// weights; wgrad = the frame-reduction kernel below).
//
//   fwd:   Y[m, n] = sum_seg sum_tap sum_k  X_seg[src(m, tap), k] * Wp[seg][tap][n][k]
//   wgrad: P[s, tap, n, k] = sum_{m in split s} dY[m, n] * X[src(m, tap), k]
//
// m = b*Tout + t is a frame row, src(m, tap) = b*Tin + pad(t + shift0 + tap*dil).
// Tiles are 128x128x32 on 4 waves (2x2, 64x64 per wave = 4x4 MFMA 16x16 tiles).
// MFMA type is a template parameter: __bf16 (v_mfma_f32_16x16x32_bf16) for
// the production path, float (v_mfma_f32_16x16x4_f32, exact fp32) for parity.
// Activations stay fp32 in HBM and are rounded to the MFMA type while staged
// into LDS, so one kernel serves both precisions.
#include "common.h"
#include "ensvs.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NTHR = 256;

template <typename T> struct Lds;
template <> struct Lds<__bf16> { static constexpr int K = 40; };  // 80 B rows
template <> struct Lds<float> { static constexpr int K = 36; };   // 144 B rows

enum {
  EPI_PLAIN = 0,     // Y = (accum ? Y : 0) + acc + bias, optional relu
  EPI_GATE = 1,      // DiffNet: gate/filter interleaved by 16 -> GF save + z = sig(g)*tanh(f)
  EPI_RESSKIP = 2,   // DiffNet: res/skip interleaved by 16 -> x' = (x + r)/sqrt2, skip (+)= s
  EPI_GATE_BWD = 3,  // DiffNet backward: dz -> d(gate), d(filter) pre-activation grads
  EPI_ADDSCALE = 4,  // Y = alpha * aux1 + acc + bias
  EPI_RELU_MASK = 5, // Y = (accum ? Y : 0) + (aux1 > 0 ? acc + bias : 0)   (ReLU backward)
  EPI_GATE_TS = 6,   // uSFGAN: xa/xb interleaved by 16 -> z = tanh(xa)*sigmoid(xb)
  EPI_NONE = 7,      // measurement only (tools/gate_probe.py): no output at all
  EPI_AUX0_BF16 = 256,  // flag: GATE writes its gate/filter save (aux0) in bf16
  EPI_AUX1_BF16 = 512,  // flag: GATE_BWD reads the gate/filter save (aux1) in bf16
};
// `relu` of EPI_PLAIN / EPI_ADDSCALE selects the output activation: 1 ReLU, 2 sigmoid.

struct SegDesc {
  const float* x;     // frame rows of this K-segment (already offset to its first channel)
  const float* radd;  // optional per-sequence vector added to in-range values (y = x + d[b])
  const float* pd;    // segment 0 only: per-row pitch-dependent dilation factor (uSFGAN)
  long long wofs;     // element offset of this segment's packed weights [taps][Npad][Kp]
  int ld, K, taps, dil, shift0, pad, radd_ld, Tin, Kp, vec, pd_dil;
};

struct GemmArgs {
  SegDesc seg[3];
  int nseg;
  int Tout, M, N, Npad;
  const void* W;
  const float* bias;
  float* Y;
  int ldy;
  int epi, relu, accum;
  float* aux0;
  const float* aux1;
  int ld0, ld1;
  float alpha;
  int C;
  // GATE saves its gate/filter pre-activations to aux0 in bf16, GATE_BWD reads them from
  // aux1 in bf16 (C ABI: bits EPI_AUX0_BF16 / EPI_AUX1_BF16 of `epi`)
  int aux0_bf, aux1_bf;
  int vec_out;  // Y / aux0 / aux1 rows 16-B aligned with ld % 4 == 0: 16-B epilogue stores
  // GATE / RESSKIP: every bf16 output (gate/filter save, ybf) 16-B aligned with ld % 8 == 0:
  // 8 channels per thread, 16-B bf16 stores (the 8-B ones made the epilogue store-issue
  // bound)
  int gate8;
  // optional bf16 copy of what is written to Y (LDS-staged epilogue only):
  // ybf[row*ybf_ld + col] = bf16(y + ybf_radd[(row / Tout)*ybf_radd_ld + col]) -- the next
  // GEMM's operand, rounded exactly as ensvs_cast_bf16 would, without the extra pass
  __bf16* ybf;
  const float* ybf_radd;
  int ybf_ld, ybf_radd_ld;
  // optional per-tile column sums, LDS-staged epilogue only, M % BM == 0: of the accumulator
  // (PLAIN / ADDSCALE / RELU_MASK, before bias) or of both outputs (GATE_BWD, in Y's column
  // space).  csum[(m0 / BM) * csum_ld + col] = sum over g = 0..7 (in order) of the sums of
  // rows g, g+8, .., g+120 (in order); ensvs_tile_colsum reproduces it for other paths
  float* csum;
  int csum_ld;
  // split-K (small M, bf16-operand 128 x 128 kernel): workgroup z takes K-steps
  // [nit * z / ksplit, nit * (z + 1) / ksplit) and stores its raw accumulator tile to
  // part[(z * M + row) * Npad + col]; splitk_epilogue_kernel sums the slices in z order and
  // runs the LDS-staged epilogue
  float* part;
  long long part_floats;
  int ksplit;
  // GATE_BWD in the production form (bf16 aux1 and ybf, no Y / bias / ybf_radd, C and M
  // multiples of 128, 16-B aligned rows): the 128 x 128 kernel's LDS-DMA epilogue
  int gbw_dma;
  // ADDSCALE with fp32 aux1 and Y, a bf16 copy, no relu / ybf_radd, M and N multiples of 128,
  // 16-B aligned rows: the LDS-DMA epilogue (addscale_epilogue_dma)
  int as_dma;
};

template <typename T>
__device__ __forceinline__ void store4(T* dst, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void store4<float>(float* dst, float a, float b, float c, float d) {
  *(f32x4*)dst = f32x4{a, b, c, d};
}
template <>
__device__ __forceinline__ void store4<__bf16>(__bf16* dst, float a, float b, float c, float d) {
  *(bf16x4*)dst = bf16x4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
}

// acc[mt][nt] += A_s[rows of wave][k] * B_s[cols of wave][k] over one BK tile.
template <typename T>
__device__ __forceinline__ void mma_tile(const T* As, const T* Bs, int wr, int wc, int lane,
                                         f32x4 (&acc)[4][4]) {
  constexpr int LK = Lds<T>::K;
  if constexpr (sizeof(T) == 2) {
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = *(const bf16x8*)(As + (wr * 64 + i * 16 + (lane & 15)) * LK + 8 * (lane >> 4));
      b[i] = *(const bf16x8*)(Bs + (wc * 64 + i * 16 + (lane & 15)) * LK + 8 * (lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = *(const f32x4*)(As + (wr * 64 + i * 16 + (lane & 15)) * LK + 16 * h + 4 * (lane >> 4));
        b[i] = *(const f32x4*)(Bs + (wc * 64 + i * 16 + (lane & 15)) * LK + 16 * h + 4 * (lane >> 4));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
    }
  }
}

// Output tile of this workgroup, XCD-aware (cdna_hip_programming.md T1): workgroups are
// dispatched round-robin over the 8 XCDs in flattened-id order; remap so that each XCD
// walks a contiguous range of tiles in N-fastest order -- the N tiles that re-read one
// 128-row A panel then run together on one XCD and share its L2.  Bijective for any grid.
__device__ __forceinline__ void xcd_tile(int& m0, int& n0) {
  const int nM = gridDim.x, nN = gridDim.y, total = nM * nN;
  const int orig = blockIdx.x + blockIdx.y * nM;
  const int xcd = orig & 7, q = total >> 3, r = total & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  m0 = (wg / nN) * BM;
  n0 = (wg % nN) * BN;
}

// ---------------------------------------------------------------- epilogue
// Shared by both forward kernels: acc holds the wave's 64x64 sub-tile (4x4 MFMA tiles).
// d(gate), d(filter) of z = sigmoid(g) * tanh(f); contraction off so the per-element and the
// LDS-staged epilogues round identically.
__device__ __forceinline__ void gate_bwd_(float dz, float g, float f, float& dg, float& df) {
#pragma clang fp contract(off)
  const float sg = fsigmoid_(g), th = ftanh_(f);
  dg = dz * th * sg * (1.f - sg);
  df = dz * sg * (1.f - th * th);
}

// one gate/filter pre-activation, fp32 or bf16 (GemmArgs::aux0_bf / aux1_bf)
__device__ __forceinline__ void st_aux0(const GemmArgs& a, long long i, float v) {
  if (a.aux0_bf) ((__bf16*)a.aux0)[i] = (__bf16)v;
  else a.aux0[i] = v;
}
__device__ __forceinline__ float ld_aux1(const GemmArgs& a, long long i) {
  return a.aux1_bf ? (float)((const __bf16*)a.aux1)[i] : a.aux1[i];
}
__device__ __forceinline__ void st4_aux0(const GemmArgs& a, long long i, f32x4 v) {
  if (a.aux0_bf)
    *(bf16x4*)((__bf16*)a.aux0 + i) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  else
    *(f32x4*)(a.aux0 + i) = v;
}
__device__ __forceinline__ f32x4 ld4_aux1(const GemmArgs& a, long long i) {
  if (a.aux1_bf) {
    const bf16x4 v = *(const bf16x4*)((const __bf16*)a.aux1 + i);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
  return *(const f32x4*)(a.aux1 + i);
}

__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, f32x4 (&acc)[4][4], int m0,
                                              int n0, int wr, int wc, int lane) {
  if (a.epi == EPI_NONE) {  // keep the accumulators live: one impossible store
    if (acc[0][0][0] == 12345.678f && m0 < 0) a.Y[0] = acc[3][3][3];
    return;
  }
  const int rbase = m0 + wr * 64 + (lane >> 4) * 4;
  if (a.epi == EPI_GATE || a.epi == EPI_RESSKIP || a.epi == EPI_GATE_TS) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int pc = n0 + wc * 64 + p * 32 + (lane & 15);
      const int c = (n0 + wc * 64) / 2 + p * 16 + (lane & 15);
      if (c >= a.C) continue;
      const float b0 = a.bias ? a.bias[pc] : 0.f;
      const float b1 = a.bias ? a.bias[pc + 16] : 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + mt * 16 + r;
          if (row >= a.M) continue;
          const float v0 = acc[mt][2 * p][r] + b0;
          const float v1 = acc[mt][2 * p + 1][r] + b1;
          if (a.epi == EPI_GATE) {
            st_aux0(a, (long long)row * a.ld0 + c, v0);
            st_aux0(a, (long long)row * a.ld0 + a.C + c, v1);
            a.Y[(long long)row * a.ldy + c] = fsigmoid_(v0) * ftanh_(v1);
          } else if (a.epi == EPI_GATE_TS) {
            a.Y[(long long)row * a.ldy + c] = ftanh_(v0) * fsigmoid_(v1);
          } else {
            const float xr = a.aux1[(long long)row * a.ld1 + c];
            a.Y[(long long)row * a.ldy + c] = (xr + v0) * 0.70710678118654752f;
            float* sk = a.aux0 + (long long)row * a.ld0 + c;
            *sk = a.accum ? fmaf(a.alpha, v1, *sk) : a.alpha * v1;
          }
        }
    }
    return;
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = n0 + wc * 64 + nt * 16 + (lane & 15);
    if (col >= a.N) continue;
    const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + mt * 16 + r;
        if (row >= a.M) continue;
        float v = acc[mt][nt][r] + bv;
        float* y = a.Y + (long long)row * a.ldy + col;
        if (a.epi == EPI_PLAIN) {
          if (a.accum) v += *y;
          if (a.relu == 1) v = fmaxf(v, 0.f);
          else if (a.relu == 2) v = sigmoidf_(v);
          *y = v;
        } else if (a.epi == EPI_ADDSCALE) {
          v = __builtin_fmaf(a.alpha, a.aux1[(long long)row * a.ld1 + col], v);
          *y = a.relu == 1 ? fmaxf(v, 0.f) : v;
        } else if (a.epi == EPI_RELU_MASK) {
          v = a.aux1[(long long)row * a.ld1 + col] > 0.f ? v : 0.f;
          *y = a.accum ? *y + v : v;
        } else if (a.epi == EPI_GATE_BWD) {
          const float g = ld_aux1(a, (long long)row * a.ld1 + col);
          const float f = ld_aux1(a, (long long)row * a.ld1 + a.C + col);
          float dg, df;
          gate_bwd_(v, g, f, dg, df);
          a.Y[(long long)row * a.ldy + col] = dg;
          a.Y[(long long)row * a.ldy + a.C + col] = df;
        }
      }
  }
}

// ---------------------------------------------------------- LDS-staged epilogue
// The fp32 output tile goes through LDS (row stride 132 floats: the fragment writes of a
// wave hit 64 distinct banks), then every thread handles 4 consecutive output columns of
// a row: one 16-B load / store per operand instead of four 4-B accesses (the per-element
// epilogue above is store-issue bound).  Same arithmetic per element as gemm_epilogue.
constexpr int EP = 132;
constexpr int CS_GROUPS = NTHR / 32;  // row groups of the column sums (32 lanes per row)
constexpr int EPI_LDS = BM * EP * 4 + CS_GROUPS * 2 * BN * 4;  // + column-sum exchange

__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *(f32x4*)p = v; }
// the same with the per-sequence add already loaded (rr)
__device__ __forceinline__ void shadow4r(const GemmArgs& a, int m, int col, f32x4 v, f32x4 rr) {
  if (!a.ybf) return;
  if (a.ybf_radd) v += rr;
  *(bf16x4*)(a.ybf + (long long)m * a.ybf_ld + col) =
      bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}
// bf16 shadow of 4 consecutive outputs (row m, columns col..col+3), see GemmArgs::ybf
__device__ __forceinline__ void shadow4(const GemmArgs& a, int m, int col, f32x4 v) {
  if (!a.ybf) return;
  if (a.ybf_radd) v += ld4(a.ybf_radd + (long long)(m / a.Tout) * a.ybf_radd_ld + col);
  *(bf16x4*)(a.ybf + (long long)m * a.ybf_ld + col) =
      bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

// NT threads share the element loops; only the waves with write_acc stage their
// accumulators (the 8-wave small-M kernel: the K-group that holds the reduced tile).
// 8 consecutive channels: bf16 copies as one 16-B store
__device__ __forceinline__ void st8_bf(__bf16* p, f32x4 lo, f32x4 hi) {
  *(bf16x8*)p = bf16x8{(__bf16)lo[0], (__bf16)lo[1], (__bf16)lo[2], (__bf16)lo[3],
                       (__bf16)hi[0], (__bf16)hi[1], (__bf16)hi[2], (__bf16)hi[3]};
}
__device__ __forceinline__ void shadow8(const GemmArgs& a, int m, int col, f32x4 lo, f32x4 hi) {
  if (!a.ybf) return;
  if (a.ybf_radd) {
    const float* r = a.ybf_radd + (long long)(m / a.Tout) * a.ybf_radd_ld + col;
    lo += ld4(r);
    hi += ld4(r + 4);
  }
  st8_bf(a.ybf + (long long)m * a.ybf_ld + col, lo, hi);
}
__device__ __forceinline__ void st8_aux0(const GemmArgs& a, long long i, f32x4 lo, f32x4 hi) {
  if (a.aux0_bf) {
    st8_bf((__bf16*)a.aux0 + i, lo, hi);
  } else {
    st4(a.aux0 + i, lo);
    st4(a.aux0 + i + 4, hi);
  }
}

// One row's 8 gate/filter channel pairs (GATE / GATE_TS epilogue): t points at the row's
// staged accumulator tile, gc the tile column of the first gate value (filter +16), c the
// first output channel, bb the 16 bias values of those columns (read once per thread, or
// null when the staged tile already holds acc + bias).  No global loads here: on gfx950
// vmcnt counts stores too, so a load issued after a row's stores (the bias, formerly
// re-read per row) waits for all of them -- one full store round trip per row.
__device__ __forceinline__ void gate_row8(const GemmArgs& a, const float* t, int gc, int m,
                                          int c, const f32x4* bb) {
  f32x4 g0 = ld4(t + gc), g1 = ld4(t + gc + 4), f0 = ld4(t + gc + 16), f1 = ld4(t + gc + 20);
  if (bb) {
    g0 += bb[0];
    g1 += bb[1];
    f0 += bb[2];
    f1 += bb[3];
  }
  f32x4 z0, z1;
  if (a.epi == EPI_GATE) {
    st8_aux0(a, (long long)m * a.ld0 + c, g0, g1);
    st8_aux0(a, (long long)m * a.ld0 + a.C + c, f0, f1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      z0[e] = fsigmoid_(g0[e]) * ftanh_(f0[e]);
      z1[e] = fsigmoid_(g1[e]) * ftanh_(f1[e]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      z0[e] = ftanh_(g0[e]) * fsigmoid_(f0[e]);
      z1[e] = ftanh_(g1[e]) * fsigmoid_(f1[e]);
    }
  }
  if (a.Y) {
    st4(a.Y + (long long)m * a.ldy + c, z0);
    st4(a.Y + (long long)m * a.ldy + c + 4, z1);
  }
  shadow8(a, m, c, z0, z1);
}

// 8-channel GATE / GATE_TS rows of a staged tile: NTT threads, tile rows [0, ROWS), T row
// stride ldT, ROWW 8-channel groups (threads) per row.  BIAS_IN_T: the staged tile already
// holds acc + bias (the 256 x 256 kernel adds it while staging).
template <int NTT, int ROWS, int ROWW, bool BIAS_IN_T = false>
__device__ __forceinline__ void gate_tile8(const GemmArgs& a, const float* T, int ldT, int mb,
                                           int n0, int tid) {
  constexpr int NI = ROWS * ROWW / NTT;
  static_assert(NTT % ROWW == 0 && NI >= 1, "gate8 geometry");
  const int q8 = tid % ROWW, q = q8 >> 1, j = (q8 & 1) * 8;
  const int c = n0 / 2 + q * 16 + j;
  const int gc = q * 32 + j;
  if (c >= a.C) return;
  f32x4 bb[4];
  const bool hb = !BIAS_IN_T && a.bias;
  if (hb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bb[i] = ld4(a.bias + n0 + gc + (i >> 1) * 16 + (i & 1) * 4);
  }
#pragma unroll 1
  for (int k = 0; k < NI; ++k) {
    const int row = tid / ROWW + k * (NTT / ROWW);
    const int m = mb + row;
    if (m >= a.M) continue;
    gate_row8(a, T + row * ldT, gc, m, c, hb ? bb : nullptr);
  }
}

// RESSKIP epilogue operands of one row (residual input x, running skip sum, the next
// block's per-sequence add for the bf16 copy), loaded a batch of rows AHEAD of the
// previous batch's stores: vmcnt counts loads and stores in issue order, so a load issued
// after stores can only be waited for together with them.
struct RsOps {
  f32x4 xr, s0, rr;
};
__device__ __forceinline__ void rs_load(const GemmArgs& a, int m, int c, RsOps& o) {
  if (m >= a.M) return;
  o.xr = ld4(a.aux1 + (long long)m * a.ld1 + c);
  if (a.accum) o.s0 = ld4(a.aux0 + (long long)m * a.ld0 + c);
  if (a.ybf && a.ybf_radd) o.rr = ld4(a.ybf_radd + (long long)(m / a.Tout) * a.ybf_radd_ld + c);
}
// x' = (x + r) / sqrt2 to Y (+ its bf16 copy with the next block's add), skip (+)= alpha * s
__device__ __forceinline__ void rs_store(const GemmArgs& a, int m, int c, f32x4 g, f32x4 f,
                                         const RsOps& o) {
  f32x4 y, sk;
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = (o.xr[e] + g[e]) * 0.70710678118654752f;
  st4(a.Y + (long long)m * a.ldy + c, y);
  if (a.ybf) {
    f32x4 v = y;
    if (a.ybf_radd) v += o.rr;
    *(bf16x4*)(a.ybf + (long long)m * a.ybf_ld + c) =
        bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  }
  if (a.accum) {
#pragma unroll
    for (int e = 0; e < 4; ++e) sk[e] = fmaf(a.alpha, f[e], o.s0[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) sk[e] = a.alpha * f[e];
  }
  st4(a.aux0 + (long long)m * a.ld0 + c, sk);
}

// operands of one row of the PLAIN (accum) / ADDSCALE / RELU_MASK / GATE_BWD epilogues
__device__ __forceinline__ void gen_load(const GemmArgs& a, int m, int col, bool want2, f32x4& p1,
                                         f32x4& p2) {
  if (m >= a.M) return;
  const float* y = a.Y + (long long)m * a.ldy + col;
  if (a.epi == EPI_PLAIN) {
    p1 = ld4(y);
  } else if (a.epi == EPI_GATE_BWD) {
    p1 = ld4_aux1(a, (long long)m * a.ld1 + col);
    p2 = ld4_aux1(a, (long long)m * a.ld1 + a.C + col);
  } else {
    p1 = ld4(a.aux1 + (long long)m * a.ld1 + col);
    if (want2) p2 = ld4(y);
  }
}

// MASK: the epilogues an instance may meet (bit e: a.epi == e), the others compiled out
template <int NT = NTHR, int EB = 1, unsigned MASK = ~0u>
__device__ __forceinline__ void gemm_epilogue_lds(const GemmArgs& a, f32x4 (&acc)[4][4], int m0,
                                                  int n0, int wr, int wc, int lane, int tid,
                                                  char* smem, bool write_acc = true) {
  auto ep = [&](int e) { return ((MASK >> e) & 1u) && a.epi == e; };
  if (ep(EPI_NONE)) {
    if (write_acc) gemm_epilogue(a, acc, m0, n0, wr, wc, lane);
    return;
  }
  float* T = (float*)smem;
  __syncthreads();  // every wave is done with the K-loop images
  if (write_acc) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(wr * 64 + mt * 16 + (lane >> 4) * 4 + r) * EP + wc * 64 + nt * 16 + (lane & 15)] =
              acc[mt][nt][r];
  }
  __syncthreads();
  const int M = a.M;
  // EB: rows per operand batch (one batch ahead in flight; 1 by register budget, more for
  // the GATE_BWD launches of the 128 x 128 kernel, whose epilogue is all operand traffic)
  // Every thread keeps one column group across its rows (NT is a multiple of 32), so the
  // bias is read once, and all of a thread's global operand loads (residual, skip, Y,
  // gate/filter save) are issued before its first store: with the loads after the stores
  // the compiler cannot reorder them (possible aliasing) and each row paid a full L2 / HBM
  // latency -- 12 of 18 us of a 2 000-row GEMM (tools/small_gemm_probe.py).
  if (a.gate8 && (ep(EPI_GATE) || ep(EPI_GATE_TS))) {
    gate_tile8<NT, BM, 8>(a, T, EP, m0, n0, tid);  // 64 channels per row: 8 threads
    return;
  }
  if (ep(EPI_GATE) || ep(EPI_RESSKIP) || ep(EPI_GATE_TS)) {
    // this tile holds 64 output channels (gate/filter interleaved by 16 in the packed columns)
    constexpr int NI = BM * 16 / NT;
    const int q4 = tid & 15, q = q4 >> 2, j = (q4 & 3) * 4;
    const int c = n0 / 2 + q * 16 + j;  // first of 4 output channels
    const int gc = q * 32 + j;          // tile column of the gate values; filter at +16
    if (c >= a.C) return;
    f32x4 bg = {0.f, 0.f, 0.f, 0.f}, bfl = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
      bg = ld4(a.bias + n0 + gc);
      bfl = ld4(a.bias + n0 + gc + 16);
    }
    static_assert(NI % EB == 0, "rows per thread in batches of EB");
    RsOps cur[EB], nxt[EB];
    if (ep(EPI_RESSKIP)) {
#pragma unroll
      for (int k = 0; k < EB; ++k) rs_load(a, m0 + (tid >> 4) + k * (NT / 16), c, cur[k]);
    }
#pragma unroll 1
    for (int kb = 0; kb < NI; kb += EB) {
    if (ep(EPI_RESSKIP) && kb + EB < NI) {
#pragma unroll
      for (int k = 0; k < EB; ++k)
        rs_load(a, m0 + (tid >> 4) + (kb + EB + k) * (NT / 16), c, nxt[k]);
    }
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      const int row = (tid >> 4) + (kb + k) * (NT / 16);
      const int m = m0 + row;
      if (m >= M) continue;
      f32x4 g = ld4(T + row * EP + gc), f = ld4(T + row * EP + gc + 16);
      if (a.bias) {
        g += bg;
        f += bfl;
      }
      if (ep(EPI_RESSKIP)) {
        rs_store(a, m, c, g, f, cur[k]);
      } else if (ep(EPI_GATE)) {
        st4_aux0(a, (long long)m * a.ld0 + c, g);
        st4_aux0(a, (long long)m * a.ld0 + a.C + c, f);
        f32x4 z;
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = fsigmoid_(g[e]) * ftanh_(f[e]);
        if (a.Y) st4(a.Y + (long long)m * a.ldy + c, z);
        shadow4(a, m, c, z);
      } else if (ep(EPI_GATE_TS)) {
        f32x4 z;
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = ftanh_(g[e]) * fsigmoid_(f[e]);
        if (a.Y) st4(a.Y + (long long)m * a.ldy + c, z);
        shadow4(a, m, c, z);
      }
    }
#pragma unroll
    for (int k = 0; k < EB; ++k) cur[k] = nxt[k];
    }
    return;
  }
  // column sums: this thread always has columns cq*4.. and rows (tid >> 5) + 8k
  f32x4 cs0 = {0.f, 0.f, 0.f, 0.f}, cs1 = {0.f, 0.f, 0.f, 0.f};
  {
    constexpr int NI = BM * 32 / NT;
    const int cq = tid & 31, col = n0 + cq * 4;
    const int ne = min(4, a.N - col);
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (a.bias && ne > 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < ne) bv[e] = a.bias[col + e];
    }
    const bool want1 = (ep(EPI_PLAIN) && a.accum) || ep(EPI_ADDSCALE) ||
                       ep(EPI_RELU_MASK) || ep(EPI_GATE_BWD);
    const bool want2 = (ep(EPI_RELU_MASK) && a.accum) || ep(EPI_GATE_BWD);
    static_assert(NI % EB == 0, "rows per thread in batches of EB");
    // operands of a batch of rows, loaded before the previous batch's stores
    const bool wl = ne == 4 && (want1 || want2);
    f32x4 p1[EB], p2[EB], q1[EB], q2[EB];
    if (wl) {
#pragma unroll
      for (int k = 0; k < EB; ++k)
        gen_load(a, m0 + (tid >> 5) + k * (NT / 32), col, want2, p1[k], p2[k]);
    }
#pragma unroll 1
    for (int kb = 0; kb < NI; kb += EB) {
    if (wl && kb + EB < NI) {
#pragma unroll
      for (int k = 0; k < EB; ++k)
        gen_load(a, m0 + (tid >> 5) + (kb + EB + k) * (NT / 32), col, want2, q1[k], q2[k]);
    }
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      const int row = (tid >> 5) + (kb + k) * (NT / 32);
      const int m = m0 + row;
      if (m >= M || ne <= 0) continue;
      f32x4 v = ld4(T + row * EP + cq * 4);
      if (a.csum && a.epi != EPI_GATE_BWD) cs0 += v;
      if (a.bias) v += bv;
      float* y = a.Y + (long long)m * a.ldy + col;
      if (ne == 4) {
        if (ep(EPI_PLAIN)) {
          if (a.accum) v += p1[k];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (a.relu == 1) v[e] = fmaxf(v[e], 0.f);
            else if (a.relu == 2) v[e] = sigmoidf_(v[e]);
          }
          st4(y, v);
          shadow4(a, m, col, v);
        } else if (ep(EPI_ADDSCALE)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = __builtin_fmaf(a.alpha, p1[k][e], v[e]);
            v[e] = a.relu == 1 ? fmaxf(v[e], 0.f) : v[e];
          }
          st4(y, v);
          shadow4(a, m, col, v);
        } else if (ep(EPI_RELU_MASK)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = p1[k][e] > 0.f ? v[e] : 0.f;
          if (a.accum) v += p2[k];
          st4(y, v);
          shadow4(a, m, col, v);
        } else if (ep(EPI_GATE_BWD)) {
          f32x4 dg, df;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float t0, t1;
            gate_bwd_(v[e], p1[k][e], p2[k][e], t0, t1);
            dg[e] = t0;
            df[e] = t1;
          }
          if (a.csum) {
            cs0 += dg;
            cs1 += df;
          }
          if (a.Y) {
            st4(y, dg);
            st4(y + a.C, df);
          }
          shadow4(a, m, col, dg);
          shadow4(a, m, a.C + col, df);
        }
      } else {
        for (int e = 0; e < ne; ++e) {
          float w = v[e];
          float* ye = y + e;
          if (ep(EPI_PLAIN)) {
            if (a.accum) w += *ye;
            if (a.relu == 1) w = fmaxf(w, 0.f);
            else if (a.relu == 2) w = sigmoidf_(w);
            *ye = w;
          } else if (ep(EPI_ADDSCALE)) {
            w = __builtin_fmaf(a.alpha, a.aux1[(long long)m * a.ld1 + col + e], w);
            *ye = a.relu == 1 ? fmaxf(w, 0.f) : w;
          } else if (ep(EPI_RELU_MASK)) {
            w = a.aux1[(long long)m * a.ld1 + col + e] > 0.f ? w : 0.f;
            *ye = a.accum ? *ye + w : w;
          } else if (ep(EPI_GATE_BWD)) {
            const float g = ld_aux1(a, (long long)m * a.ld1 + col + e);
            const float f = ld_aux1(a, (long long)m * a.ld1 + a.C + col + e);
            gate_bwd_(w, g, f, ye[0], ye[a.C]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      p1[k] = q1[k];
      p2[k] = q2[k];
    }
    }
  }
  if (NT == NTHR && a.csum) {  // uniform: every thread reaches the barrier
    float* X = T + BM * EP;  // [group][2*BN]
    const int g = tid >> 5, c4 = (tid & 31) * 4;
    *(f32x4*)(X + g * 2 * BN + c4) = cs0;
    *(f32x4*)(X + g * 2 * BN + BN + c4) = cs1;
    __syncthreads();
    const int j = tid;  // NTHR == 2 * BN: first BN the accumulator / d(gate), then d(filter)
    const bool bwd = ep(EPI_GATE_BWD);
    if (j < BN || bwd) {
      const int c = n0 + (j & (BN - 1));
      if (c < a.N) {
        float t = X[j];
#pragma unroll
        for (int q = 1; q < CS_GROUPS; ++q) t += X[q * 2 * BN + j];
        a.csum[(long long)(m0 / BM) * a.csum_ld + (j < BN ? c : a.C + c)] = t;
      }
    }
  }
}

// ------------------------------------------------------------------ forward
struct SegSel {  // the K-segment of one iteration, held in (wave-uniform) scalars
  const float* x;
  const float* radd;
  long long wofs;
  int ld, K, dil, shift0, pad, radd_ld, Tin, Kp, vec, j, kc, s;
};

// All staging loads are unconditional: an out-of-range row (padding, m >= M) or
// column quad points at g_zero, so no load is branched around or masked after it
// lands (a mask/add right after a load makes hipcc wait vmcnt(0) per row).  The
// per-sequence vector radd is loaded the same way (g_zero when absent) and added in
// the store phase, after the MFMAs.  VEC: every segment of the launch has K % 4 == 0,
// ld % 4 == 0 and 16-B aligned rows (one dwordx4 per quad); otherwise 4 scalar loads.
constexpr int ZERO_FLOATS = 64;
__device__ __attribute__((aligned(16))) float g_zero[ZERO_FLOATS];

// Pitch-dependent tap of an uSFGAN adaptive block (usfgan/utils/index.py:27-54), in the
// reference's float32 arithmetic: past = rint((t - L) - d*dil) + L, future = rint(t + d*dil)
// (round half to even); taps 0/1/2 = past/current/future, -1 = the zero padding.
__device__ __forceinline__ int pd_src(float d, float dil, int t, int L, int j) {
  const float dd = __fmul_rn(d, dil);
  const int past = (int)rintf(__fadd_rn(-dd, (float)(t - L))) + L;
  const int fut = (int)rintf(__fadd_rn(dd, (float)t));
  const int s = j == 0 ? past : (j == 1 ? t : fut);
  return (s >= 0 && s < L) ? s : -1;
}

template <bool VEC>
__device__ __forceinline__ void load_a_src(const SegSel& g, int k, int src, bool ok, int b,
                                           f32x4& v, f32x4& r) {
  const bool row_ok = ok && src >= 0;
  const float* xrow = g.x + (long long)(b * g.Tin + src) * g.ld;
  const float* rrow = g.radd + (long long)b * g.radd_ld;
  const bool has_r = g.radd != nullptr;
  if constexpr (VEC) {
    const bool q = row_ok && k < g.K;
    v = *(const f32x4*)(q ? xrow + k : g_zero);
    r = *(const f32x4*)((q && has_r) ? rrow + k : g_zero);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool q = row_ok && k + e < g.K;
      v[e] = *(q ? xrow + k + e : g_zero);
      r[e] = *((q && has_r) ? rrow + k + e : g_zero);
    }
  }
}

template <typename T, bool VEC, bool PD>
__global__ __launch_bounds__(NTHR) void conv_gemm_kernel(const GemmArgs a) {
  constexpr int LK = Lds<T>::K;
  constexpr int BCH = sizeof(T) == 2 ? 2 : 4;  // 16-B B chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* As = (T*)smem;
  T* Bs = As + 2 * BM * LK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  xcd_tile(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const char* const W = (const char*)a.W;

  // A staging: rows r_i = (tid>>3) + 32 i, 4 floats at column (tid&7)*4 of the k-chunk.
  const int ac4 = tid & 7, arow = tid >> 3;
  int b0, t0, b1, t1, b2, t2, b3, t3;
  bool ok0, ok1, ok2, ok3;
#define ROWINIT(i)                                     \
  {                                                    \
    const int m = m0 + arow + 32 * i;                  \
    ok##i = m < M;                                     \
    b##i = ok##i ? m / Tout : 0;                       \
    t##i = ok##i ? m - b##i * Tout : 0;                \
  }
  ROWINIT(0) ROWINIT(1) ROWINIT(2) ROWINIT(3)
#undef ROWINIT
  // PD: the dilation factor of each staged row (segment 0 is the pitch-dependent one)
  float pd0 = 0.f, pd1 = 0.f, pd2 = 0.f, pd3 = 0.f;
  if constexpr (PD) {
    const float* pdp = a.seg[0].pd;
    pd0 = ok0 ? pdp[m0 + arow] : 0.f;
    pd1 = ok1 ? pdp[m0 + arow + 32] : 0.f;
    pd2 = ok2 ? pdp[m0 + arow + 64] : 0.f;
    pd3 = ok3 ? pdp[m0 + arow + 96] : 0.f;
  }
  const float pdil = PD ? (float)a.seg[0].pd_dil : 0.f;

  // Flattened K iteration space (segment, tap, k-chunk); segment fields are picked with
  // wave-uniform selects on static indices.
  const int nseg = a.nseg;
  const int nk0 = __builtin_amdgcn_readfirstlane((a.seg[0].K + BK - 1) / BK);
  const int nk1 = __builtin_amdgcn_readfirstlane(nseg > 1 ? (a.seg[1].K + BK - 1) / BK : 0);
  const int nk2 = __builtin_amdgcn_readfirstlane(nseg > 2 ? (a.seg[2].K + BK - 1) / BK : 0);
  const int cum1 = nk0 * a.seg[0].taps;
  const int cum2 = cum1 + (nseg > 1 ? nk1 * a.seg[1].taps : 0);
  const int nit = cum2 + (nseg > 2 ? nk2 * a.seg[2].taps : 0);

  auto select = [&](int it) __attribute__((always_inline)) {
    const int s = __builtin_amdgcn_readfirstlane((it >= cum1) + (it >= cum2));
    const SegDesc& d = a.seg[s];  // uniform index into the kernarg segment: scalar loads
    SegSel g;
    const int base = s == 0 ? 0 : (s == 1 ? cum1 : cum2);
    const int nks = s == 0 ? nk0 : (s == 1 ? nk1 : nk2);
    g.j = __builtin_amdgcn_readfirstlane((it - base) / nks);
    g.kc = (it - base) - g.j * nks;
    g.x = d.x; g.radd = d.radd; g.wofs = d.wofs;
    g.ld = d.ld; g.K = d.K; g.dil = d.dil; g.shift0 = d.shift0;
    g.pad = d.pad; g.radd_ld = d.radd_ld; g.Tin = d.Tin; g.Kp = d.Kp;
    g.vec = d.vec;
    g.s = s;
    return g;
  };

  f32x4 ra0, ra1, ra2, ra3, rr0, rr1, rr2, rr3;
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t rw[BCH];
  auto load = [&](int it) __attribute__((always_inline)) {
    const SegSel g = select(it);
    const int k = g.kc * BK + ac4 * 4;
    int s0, s1, s2, s3;
    if (PD && g.s == 0) {
      s0 = pd_src(pd0, pdil, t0, g.Tin, g.j);
      s1 = pd_src(pd1, pdil, t1, g.Tin, g.j);
      s2 = pd_src(pd2, pdil, t2, g.Tin, g.j);
      s3 = pd_src(pd3, pdil, t3, g.Tin, g.j);
    } else {
      const int sh = g.shift0 + g.j * g.dil;
      s0 = pad_src(t0 + sh, g.Tin, g.pad);
      s1 = pad_src(t1 + sh, g.Tin, g.pad);
      s2 = pad_src(t2 + sh, g.Tin, g.pad);
      s3 = pad_src(t3 + sh, g.Tin, g.pad);
    }
    load_a_src<VEC>(g, k, s0, ok0, b0, ra0, rr0);
    load_a_src<VEC>(g, k, s1, ok1, b1, ra1, rr1);
    load_a_src<VEC>(g, k, s2, ok2, b2, ra2, rr2);
    load_a_src<VEC>(g, k, s3, ok3, b3, ra3, rr3);
    const char* wbase = W + ((g.wofs + ((long long)g.j * Npad + n0) * g.Kp + g.kc * BK) *
                             (long long)sizeof(T));
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int q = tid + NTHR * i;
      const int row = sizeof(T) == 2 ? (q >> 2) : (q >> 3);
      const int c = sizeof(T) == 2 ? (q & 3) : (q & 7);
      rw[i] = *(const u32x4_t*)(wbase + (long long)row * g.Kp * sizeof(T) + c * 16);
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    T* A = As + buf * BM * LK + arow * LK + ac4 * 4;
    ra0 += rr0;
    ra1 += rr1;
    ra2 += rr2;
    ra3 += rr3;
    store4<T>(A, ra0[0], ra0[1], ra0[2], ra0[3]);
    store4<T>(A + 32 * LK, ra1[0], ra1[1], ra1[2], ra1[3]);
    store4<T>(A + 64 * LK, ra2[0], ra2[1], ra2[2], ra2[3]);
    store4<T>(A + 96 * LK, ra3[0], ra3[1], ra3[2], ra3[3]);
    T* B = Bs + buf * BN * LK;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int q = tid + NTHR * i;
      const int row = sizeof(T) == 2 ? (q >> 2) : (q >> 3);
      const int c = sizeof(T) == 2 ? (q & 3) : (q & 7);
      *(u32x4_t*)((char*)(B + row * LK) + c * 16) = rw[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nit > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int buf = it & 1;
    if (it + 1 < nit) load(it + 1);
    mma_tile<T>(As + buf * BM * LK, Bs + buf * BN * LK, wr, wc, lane, acc);
    if (it + 1 < nit) store(buf ^ 1);
    __syncthreads();
  }

  gemm_epilogue(a, acc, m0, n0, wr, wc, lane);
}

// ------------------------------------------------- forward, bf16 activations
// Same contraction with every A segment already rounded to bf16 in HBM (ensvs_cast_bf16
// applies the rounding -- and the per-sequence radd -- that conv_gemm_kernel applies
// while staging; the MFMAs run over the same 32-deep k chunks in the same order, so both
// kernels return identical bits).  Both operands go HBM/L2 -> LDS by
// global_load_lds_dwordx4 (no staging VGPRs, no conversion VALU), K-steps of 64, STAGES
// deep with a counted vmcnt so younger tiles stay in flight across the raw s_barrier.
// LDS image per operand and stage: [128 rows][64 k] bf16, 128-B rows whose 16-B chunks
// are XOR-swizzled by (row >> 1) & 7, so a ds_read_b128 of 16 rows at one k-chunk hits 16
// distinct bank groups; glds writes lane-linearly (wave-instruction = 8 rows x 128 B), so
// the swizzle is applied to the source address (cdna_hip_programming.md §5.4 rule 21).
// The (segment, tap, k-step) cursor advances incrementally in scalars.
constexpr int BK2 = 64;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__device__ __forceinline__ int swz(int row, int c) { return c ^ ((row >> 1) & 7); }

// Workgroup barrier for LDS hand-offs only: __syncthreads() is a release/acquire, so hipcc
// waits vmcnt(0) before it -- in an epilogue that is every global store issued so far, once
// per staged chunk.  Here only the LDS accesses are drained (lgkmcnt(0)); global stores stay
// in flight across the barrier (nothing in the workgroup reads them back).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((glb_void*)g, (lds_void*)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

struct B16Cursor {  // wave-uniform position of the next tile to stage
  int s, j, kc;
};

// One segment's fields, wave-uniform.  Read once per kernel into SGPRs (readfirstlane),
// not re-loaded from the kernarg segment inside the K loop.
struct SegU {
  const __bf16* x;
  const char* w;  // packed weights of this segment (bytes)
  int ld, K, Tin, pad, Kp, shift0, dil, taps, nk;
};

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <typename P>
__device__ __forceinline__ P* unip(P* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = (unsigned)uni((int)(unsigned)u), hi = (unsigned)uni((int)(unsigned)(u >> 32));
  return (P*)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ SegU seg_u(const SegDesc& d, const void* W) {
  SegU u;
  u.x = unip((const __bf16*)d.x);
  u.w = unip((const char*)W + d.wofs * 2);
  u.ld = uni(d.ld);
  u.K = uni(d.K);
  u.Tin = uni(d.Tin);
  u.pad = uni(d.pad);
  u.Kp = uni(d.Kp);
  u.shift0 = uni(d.shift0);
  u.dil = uni(d.dil);
  u.taps = uni(d.taps);
  u.nk = uni((d.K + BK2 - 1) / BK2);
  return u;
}

// Stage one 64-deep K-step of both operand images (A at As, B at As + TILE).
// rb[i] = (b_i * Tin + t_i) * ld: this lane's A row i at tap shift 0 (segment-specific).
// Per-lane staging pointers of the current (segment, tap): A row i at k = 0 of this
// lane's chunk (or invalid: zero padding / rows past M), B row i likewise.  Rebuilt when
// the staging cursor enters a new tap; a K-step then only adds kb and checks the chunk
// against K (A) / Kp (B).  Passed by value (a reference or a capturing lambda would put
// these arrays in scratch).
struct TapPtrs {
  const char* pa[4];
  const char* pb[4];
  unsigned va;  // bit i: A row i reads data (else zeros)
  int K, Kp;    // wave-uniform
};

// pd: segment 0 of an uSFGAN adaptive block -- tap j of row i reads the pitch-dependent row
// pd_src(d_i, pdil, t_i, Tin, j) (d0..d3: the staged rows' dilation factors)
__device__ __forceinline__ TapPtrs tap_ptrs(const SegU S, int j, int Npad, int n0, int rl,
                                            int cq8a, int cq8b, const int b0, const int b1,
                                            const int b2, const int b3, const int t0,
                                            const int t1, const int t2, const int t3,
                                            unsigned okm, bool pd = false, float d0 = 0.f,
                                            float d1 = 0.f, float d2 = 0.f, float d3 = 0.f,
                                            float pdil = 0.f) {
  TapPtrs P;
  const int bt[4] = {b0, b1, b2, b3}, tt[4] = {t0, t1, t2, t3};
  const float dd[4] = {d0, d1, d2, d3};
  const int shj = S.shift0 + j * S.dil;
  P.va = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c8 = (i & 1) ? cq8b : cq8a;
    const int ts = tt[i] + shj;
    const int src = pd ? pd_src(dd[i], pdil, tt[i], S.Tin, j)
                       : S.pad == PAD_ZERO ? ((unsigned)ts < (unsigned)S.Tin ? ts : -1)
                                           : pad_src(ts, S.Tin, S.pad);
    const bool ok = ((okm >> i) & 1) && src >= 0;
    P.va |= ok ? (1u << i) : 0u;
    P.pa[i] = (const char*)(S.x + (unsigned)((bt[i] * S.Tin + (ok ? src : 0)) * S.ld + c8));
    P.pb[i] = S.w + ((unsigned)((j * Npad + n0 + rl + 8 * i) * S.Kp + c8)) * 2;
  }
  P.K = S.K;
  P.Kp = S.Kp;
  return P;
}

// FUSE (the uSFGAN residual block, usf_block_kernel): a is the block's gate GEMM (GATE_TS,
// all 128 gate/filter columns in this tile), a2 its output projection (ADDSCALE on the
// residual stream): z = tanh(gate) * sigmoid(filter) goes from the accumulators to a bf16
// LDS image (the rounding of z's bf16 copy), the 128 x 64 output GEMM reads it there and
// the weights from global memory, and a2's epilogue updates the residual stream -- no z
// round trip through HBM, one launch per block instead of two.
__device__ __forceinline__ void usf_block_tail(const GemmArgs& a, const GemmArgs& a2,
                                               f32x4 (&acc)[4][4], char* smem, int tid, int lane,
                                               int wr, int wc, int m0);

// GATE_BWD epilogue of the 128 x 128 bf16 kernel with its operands staged by LDS-DMA (the
// production form: bf16 gate/filter save in, bf16 d(pre) out, no fp32 Y, per-tile column
// sums).  The register form loads each thread's gate/filter values two rows ahead of its
// stores, ~2 x 8 B in flight per thread: 23.6 of the launch's 36.5 us (K loop alone 12.9 us,
// tools/dgrad_probe.py).  Here the accumulator rows go through LDS a 64-row half at a time
// and the half's gate / filter rows in 32-row quarters (2 x 8 KB), double-buffered and
// fetched by global_load_lds (no registers) one quarter ahead: a quarter's DMA is issued
// before the previous quarter's stores, so the counted wait for it never waits for stores
// (vmcnt counts both, in issue order).  A one-burst form (a half's operands, one wait) took
// 40.0 us: its wait covered the previous half's stores.  Rows and the column-sum order are the
// register form's (thread group g sums rows g, g + 8, .. in order): the same bits.
typedef __attribute__((address_space(3))) char lds_char;
constexpr int GBW_T = 64 * EP * 4, GBW_Q = 32 * 256;  // T half; one operand quarter (bf16)
static_assert(GBW_T + 4 * GBW_Q + CS_GROUPS * 2 * BN * 4 <= EPI_LDS, "GATE_BWD DMA LDS");
// The waits are counted by hand, so the LDS reads, the global stores and the barriers are
// issued as inline asm: the compiler drains every outstanding LDS-DMA (s_waitcnt vmcnt(0))
// in front of an LDS read it can see, and __syncthreads() drains the stores.
__device__ __forceinline__ void gbw_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void gbw_st8(__bf16* p, f32x4 v) {
  const bf16x4 h = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(__builtin_bit_cast(u32x2, h))
               : "memory");
}
__device__ __forceinline__ void gate_bwd_epilogue_dma(const GemmArgs& a, f32x4 (&acc)[4][4],
                                                      int m0, int n0, int wr, int wc, int lane,
                                                      int tid, char* smem) {
  float* T = (float*)smem;               // [64][EP] accumulator rows of the half
  char* GF = smem + GBW_T;               // [2 buffers][gate, filter][32][128] bf16
  float* X = (float*)(GF + 4 * GBW_Q);  // [group][2 * BN] column-sum exchange
  const int wid = tid >> 6, cq = tid & 31, grp = tid >> 5, col = n0 + cq * 4;
  const __bf16* aux = (const __bf16*)a.aux1;
  // quarter q's gate and filter rows into buffer q & 1: wave wid moves rows 8 wid .. 8 wid + 7,
  // 4 rows (1 KB) per instruction: 4 instructions per lane and quarter
  auto fetch = [&](int q) {
    char* G = GF + (q & 1) * 2 * GBW_Q;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 8 * wid + 4 * i;
      const __bf16* src =
          aux + (long long)(m0 + 32 * q + r + (lane >> 4)) * a.ld1 + n0 + (lane & 15) * 8;
      glds16(src, G + r * 256);
      glds16(src + a.C, G + GBW_Q + r * 256);
    }
  };
  auto stage = [&](int h) {  // the waves holding rows 64 h .. 64 h + 63 write them to T
    if (wr == h) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            T[(mt * 16 + (lane >> 4) * 4 + r) * EP + wc * 64 + nt * 16 + (lane & 15)] =
                acc[mt][nt][r];
    }
  };
  const unsigned tb = (unsigned)(size_t)(const lds_char*)(const char*)T;
  const unsigned gb = (unsigned)(size_t)(const lds_char*)(const char*)GF;
  f32x4 cs0 = {0.f, 0.f, 0.f, 0.f}, cs1 = {0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int q) {  // rows 32 q + grp + 8 k, k = 0..3: 8 stores per thread
    const unsigned g0 = gb + (q & 1) * 2 * GBW_Q + cq * 8;
    const unsigned t0 = tb + ((q & 1) * 32) * EP * 4 + cq * 16;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const int row = grp + 8 * k;
      const int m = m0 + 32 * q + row;
      f32x4 v;
      bf16x4 gv, fv;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(t0 + row * EP * 4) : "memory");
      asm volatile("ds_read_b64 %0, %1" : "=v"(gv) : "v"(g0 + row * 256) : "memory");
      asm volatile("ds_read_b64 %0, %1" : "=v"(fv) : "v"(g0 + GBW_Q + row * 256) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(gv), "+v"(fv));
      f32x4 dg, df;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float d0, d1;
        gate_bwd_(v[e], (float)gv[e], (float)fv[e], d0, d1);
        dg[e] = d0;
        df[e] = d1;
      }
      if (a.csum) {
        cs0 += dg;
        cs1 += df;
      }
      __bf16* yr = a.ybf + (long long)m * a.ybf_ld + col;
      gbw_st8(yr, dg);
      gbw_st8(yr + a.C, df);
    }
  };
  gbw_bar();  // every wave is done with the K loop's images (no loads outstanding)
  fetch(0);
  fetch(1);
  stage(0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // quarter 0 landed (quarter 1 may not)
  gbw_bar();
  compute(0);
  gbw_bar();  // buffer 0 free
  fetch(2);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // quarter 1 (then 8 stores, quarter 2)
  gbw_bar();
  compute(1);
  gbw_bar();  // buffer 1 and T free
  fetch(3);
  stage(1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // quarter 2 (then 8 stores, quarter 3)
  gbw_bar();
  compute(2);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // quarter 3 (then 8 stores)
  gbw_bar();
  compute(3);
  if (a.csum) {  // uniform
    const int c4 = cq * 4;
    *(f32x4*)(X + grp * 2 * BN + c4) = cs0;
    *(f32x4*)(X + grp * 2 * BN + BN + c4) = cs1;
    gbw_bar();
    const int j = tid;  // NTHR == 2 * BN: d(gate) columns, then d(filter)
    const int c = n0 + (j & (BN - 1));
    float t = X[j];
#pragma unroll
    for (int q = 1; q < CS_GROUPS; ++q) t += X[q * 2 * BN + j];
    a.csum[(long long)(m0 / BM) * a.csum_ld + (j < BN ? c : a.C + c)] = t;
  }
}

// The dilated-conv dgrad's ADDSCALE epilogue (Y = alpha aux1 + acc [+ bias], its bf16 copy,
// the accumulator's per-tile column sums) in the same form as gate_bwd_epilogue_dma: the fp32
// aux1 rows (512 B of the tile's columns per row) fetched by LDS-DMA in double-buffered
// 32-row quarters one quarter ahead, two stores per row (Y, bf16 copy), counted waits.  Same
// rows, arithmetic and column-sum order as the register form: the same bits.
// A store of more than 8 bytes reads its data VGPRs after issue: a VALU write to them in the
// next slot is a hazard the compiler's hazard recognizer cannot see inside inline asm (it put
// the bf16 packing of the same registers right behind the store, and lanes 12-15 of each
// 16 stored the packed bits), hence the s_nop.
__device__ __forceinline__ void gbw_st16(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void addscale_epilogue_dma(const GemmArgs& a, f32x4 (&acc)[4][4],
                                                      int m0, int n0, int wr, int wc, int lane,
                                                      int tid, char* smem) {
  float* T = (float*)smem;               // [64][EP] accumulator rows of the half
  char* AX = smem + GBW_T;               // [2 buffers][32][128] fp32 aux1 rows
  float* X = (float*)(AX + 4 * GBW_Q);  // [group][BN] column-sum exchange
  const int wid = tid >> 6, cq = tid & 31, grp = tid >> 5, col = n0 + cq * 4;
  auto fetch = [&](int q) {  // wave wid: rows 8 wid .. 8 wid + 7 of quarter q, 2 rows per DMA
    char* D = AX + (q & 1) * 2 * GBW_Q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 8 * wid + 2 * i;
      const float* src = a.aux1 + (long long)(m0 + 32 * q + r + (lane >> 5)) * a.ld1 + n0 +
                         (lane & 31) * 4;
      glds16(src, D + r * 512);
    }
  };
  auto stage = [&](int h) {
    if (wr == h) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            T[(mt * 16 + (lane >> 4) * 4 + r) * EP + wc * 64 + nt * 16 + (lane & 15)] =
                acc[mt][nt][r];
    }
  };
  const unsigned tb = (unsigned)(size_t)(const lds_char*)(const char*)T;
  const unsigned ab = (unsigned)(size_t)(const lds_char*)(const char*)AX;
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if (a.bias) bv = ld4(a.bias + col);
  f32x4 cs0 = {0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int q) {
    const unsigned a0 = ab + (q & 1) * 2 * GBW_Q + cq * 16;
    const unsigned t0 = tb + ((q & 1) * 32) * EP * 4 + cq * 16;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const int row = grp + 8 * k;
      const int m = m0 + 32 * q + row;
      f32x4 v, x;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(t0 + row * EP * 4) : "memory");
      asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"(a0 + row * 512) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(x));
      if (a.csum) cs0 += v;
      if (a.bias) v += bv;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf(a.alpha, x[e], v[e]);
      gbw_st16(a.Y + (long long)m * a.ldy + col, v);
      gbw_st8(a.ybf + (long long)m * a.ybf_ld + col, v);
    }
  };
  gbw_bar();
  fetch(0);
  fetch(1);
  stage(0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  gbw_bar();
  compute(0);
  gbw_bar();
  fetch(2);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  gbw_bar();
  compute(1);
  gbw_bar();
  fetch(3);
  stage(1);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  gbw_bar();
  compute(2);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  gbw_bar();
  compute(3);
  if (a.csum) {  // as gemm_epilogue_lds: group sums, then the 8 groups in order
    *(f32x4*)(X + grp * 2 * BN + cq * 4) = cs0;
    gbw_bar();
    if (tid < BN) {
      const int c = n0 + tid;
      float t = X[tid];
#pragma unroll
      for (int g = 1; g < CS_GROUPS; ++g) t += X[g * 2 * BN + tid];
      a.csum[(long long)(m0 / BM) * a.csum_ld + c] = t;
    }
  }
}

// GATE_BWD epilogue rows per operand batch in the 128 x 128 kernel: 2 builds without scratch
// (162 VGPRs; 4 spills 124 B) and takes the C = 256 gate-backward dgrad from 51.4 to 47.5 us
constexpr int GBW_EB = 2;

// EPK = EPI_RESSKIP / EPI_ADDSCALE: an instance compiled for that epilogue alone, its
// operands EB_* rows per batch (the DiffNet residual / skip update and the dilated-conv
// dgrad).  Batching 2 rows in the shared instance took it to 168 VGPRs and slowed its
// GATE_BWD launches (48.2 -> 50.5 us); one instance per epilogue keeps each one's registers
// to what it uses: res/skip 46.0 -> 38.9 us (2 rows; 144-151 VGPRs, no scratch), dilated
// dgrad 59.8 -> 48.9 us (4 rows) at M = 30 720, C = 256.  GATE_BWD stays in the shared
// instance: its own (2 rows, 166 VGPRs) measured 47.8 us and +0.08 ms/step, 4 rows spill.
constexpr int EB_RS = 2, EB_AS = 4;
template <int STAGES, bool FUSE, int EPK = -1>

__device__ __forceinline__ void b16_body(const GemmArgs& a, const GemmArgs& a2) {
  static_assert(STAGES >= 2 && STAGES <= 3, "stages");
  constexpr int TILE = BM * BK2 * 2;  // bytes of one operand image (16 KB)
  constexpr int GL = 8;               // glds per thread per tile (4 A rows + 4 B rows)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  xcd_tile(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);

  // Rows this lane stages (glds i of its wave: row wid*32 + 8i + lane/8) and the logical
  // 16-B chunk it fetches into its lane-linear slot: swz(rl + 8i, slot) = cq ^ 4(i & 1).
  const int rl = wid * 32 + (lane >> 3), slot = lane & 7;
  const int cq = swz(rl, slot), cq8a = cq * 8, cq8b = (cq ^ 4) * 8;
  int bt[4], tt[4];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rl + 8 * i;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  // uSFGAN adaptive block: segment 0 gathers pitch-dependent rows (the staged rows' factors)
  const bool hpd = a.seg[0].pd != nullptr;
  float pdv[4] = {0.f, 0.f, 0.f, 0.f};
  if (hpd) {
#pragma unroll
    for (int i = 0; i < 4; ++i) pdv[i] = ((okm >> i) & 1) ? a.seg[0].pd[m0 + rl + 8 * i] : 0.f;
  }
  const float pdil = (float)a.seg[0].pd_dil;
  // g_zero's address, opaque to the compiler: it would otherwise re-load it from the GOT
  // (s_load + lgkmcnt wait) at every use inside the K loop
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  const int c8[4] = {cq8a, cq8b, cq8a, cq8b};

  int qs = 0, qj = 0, qkc = 0;  // staging cursor (segment, tap, k-step)
  int nloc = nit;
  if (a.ksplit > 1) {  // this split's K-steps: advance the cursor to the first one
    const int z = blockIdx.z;
    const int i0 = (int)((long long)nit * z / a.ksplit);
    nloc = (int)((long long)nit * (z + 1) / a.ksplit) - i0;
    for (int i = 0; i < i0; ++i) {
      const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);
      const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);
      if (++qkc == nks_) {
        qkc = 0;
        if (++qj == taps_) {
          qj = 0;
          ++qs;
        }
      }
    }
  }
#define TAP_PTRS(S) \
  tap_ptrs(S, qj, Npad, n0, rl, cq8a, cq8b, bt[0], bt[1], bt[2], bt[3], tt[0], tt[1], tt[2], tt[3], okm, \
           &(S) == &S0 && hpd, pdv[0], pdv[1], pdv[2], pdv[3], pdil)
  TapPtrs P = qs == 0 ? TAP_PTRS(S0) : (qs == 1 ? TAP_PTRS(S1) : TAP_PTRS(S2));
#define ISSUE(it)                                                                        \
  do {                                                                                   \
    char* As_ = smem + ((it) % STAGES) * 2 * TILE + wid * 32 * 128;                      \
    const int kb_ = qkc * BK2;                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool oa = ((P.va >> i) & 1) && kb_ + c8[i] < P.K;                            \
      glds16(oa ? (const void*)(P.pa[i] + kb_ * 2) : (const void*)zp, As_ + i * 1024);   \
    }                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool ob = kb_ + c8[i] < P.Kp;                                                \
      glds16(ob ? (const void*)(P.pb[i] + kb_ * 2) : (const void*)zp,                    \
             As_ + TILE + i * 1024);                                                     \
    }                                                                                    \
    const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                        \
    const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
    if (++qkc == nks_) {                                                                 \
      qkc = 0;                                                                           \
      if (++qj == taps_) {                                                               \
        qj = 0;                                                                          \
        ++qs;                                                                            \
      }                                                                                  \
      if (qs < nseg) P = qs == 0 ? TAP_PTRS(S0) : (qs == 1 ? TAP_PTRS(S1) : TAP_PTRS(S2)); \
    }                                                                                    \
  } while (0)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nloc) ISSUE(p);
  const int arow = lane & 15, kq = lane >> 4;
  // fragment read offsets: rows ra + 16i share swz(ra, .), so i only adds 2048 B
  const int ra = wr * 64 + arow, rbr = wc * 64 + arow;
  const int oa0 = ra * 128 + swz(ra, kq) * 16, oa1 = ra * 128 + swz(ra, kq + 4) * 16;
  const int ob0 = TILE + rbr * 128 + swz(rbr, kq) * 16, ob1 = TILE + rbr * 128 + swz(rbr, kq + 4) * 16;
  for (int it = 0; it < nloc; ++it) {
    if constexpr (STAGES == 3) {
      if (it + 1 < nloc) wait_vm<GL>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // tile `it` visible; every wave is done with tile it-1
    if (it + STAGES - 1 < nloc) ISSUE(it + STAGES - 1);
    // (both 32-halves always: a zero half adds exact zeros, and a data-dependent skip
    // makes hipcc move the accumulators out of AGPRs every iteration)
    const char* St = smem + (it % STAGES) * 2 * TILE;
    // all 16 fragment reads of the K step first, then its 32 MFMAs: the scheduler would
    // otherwise sink each read next to its first MFMA behind an lgkmcnt(0) wait
    bf16x8 fa[2][4], fb[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[h][i] = *(const bf16x8*)(St + (h ? oa1 : oa0) + i * 2048);
        fb[h][i] = *(const bf16x8*)(St + (h ? ob1 : ob0) + i * 2048);
      }
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // DS reads
    __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);  // MFMAs
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[h][i], fb[h][j], acc[i][j], 0, 0, 0);
  }
#undef ISSUE
#undef TAP_PTRS
  if constexpr (FUSE) {
    usf_block_tail(a, a2, acc, smem, tid, lane, wr, wc, m0);
    return;
  }
  if (a.ksplit > 1) {  // raw partial tile of this K split
    float* pz = a.part + (long long)blockIdx.z * M * Npad;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pz[(long long)row * Npad + n0 + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    return;
  }
  if constexpr (EPK == EPI_GATE_BWD) {  // instance launched only with a.gbw_dma
    gate_bwd_epilogue_dma(a, acc, m0, n0, wr, wc, lane, tid, smem);
    return;
  }
  if constexpr (EPK == EPI_ADDSCALE + 16) {  // instance launched only with a.as_dma
    addscale_epilogue_dma(a, acc, m0, n0, wr, wc, lane, tid, smem);
    return;
  }
  if (a.vec_out) {
    if (EPK == EPI_RESSKIP)
      gemm_epilogue_lds<NTHR, EB_RS, 1u << EPI_RESSKIP>(a, acc, m0, n0, wr, wc, lane, tid, smem);
    else if (EPK == EPI_ADDSCALE)
      gemm_epilogue_lds<NTHR, EB_AS, 1u << EPI_ADDSCALE>(a, acc, m0, n0, wr, wc, lane, tid, smem);
    else if (GBW_EB > 1 && a.epi == EPI_GATE_BWD)
      gemm_epilogue_lds<NTHR, GBW_EB>(a, acc, m0, n0, wr, wc, lane, tid, smem);
    else
      gemm_epilogue_lds(a, acc, m0, n0, wr, wc, lane, tid, smem);
  }
  else gemm_epilogue(a, acc, m0, n0, wr, wc, lane);
}

template <int STAGES, int EPK = -1>
__global__ __launch_bounds__(NTHR, 3) void conv_gemm_b16_kernel(const GemmArgs a) {
  b16_body<STAGES, false, EPK>(a, a);
}

__global__ __launch_bounds__(NTHR, 2) void usf_block_kernel(const GemmArgs a, const GemmArgs a2) {
  b16_body<2, true>(a, a2);
}

// ------------------------------------------- 128 x 128, two K-groups of 4 waves (small M)
// Small-M launches (a 2 000-frame reverse-diffusion GEMM is 64 tiles: a quarter of the CUs)
// are bound by what ONE workgroup issues per K-step -- 8 LDS-DMA pieces and 32 MFMAs per
// wave (MI355X_MICROARCH.md: a DMA piece costs 60-185 issue cycles) -- not by load
// latency (three stages measured 3 % faster than two) or bytes.  Here 8 waves form two
// K-groups: group g stages and multiplies K-steps g, g+2, g+4, .. into its own 64 x 64
// sub-tile accumulators (its own half of each LDS stage), so a tile's K loop takes half the
// per-wave issue; the groups' tiles are added through LDS (acc0 + acc1: the sum differs from
// the one-group order only by fp32 rounding) and all 8 waves run the LDS-staged epilogue.
constexpr int NTHR2 = 2 * NTHR;

__global__ __launch_bounds__(NTHR2) void conv_gemm_b16_dual_kernel(const GemmArgs a) {
  constexpr int TILE = BM * BK2 * 2;      // bytes of one operand image (16 KB)
  constexpr int GSET = 2 * TILE;          // one K-group's A + B images
  constexpr int STAGE = 2 * GSET;         // both groups
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int kg = wid >> 2, w4 = wid & 3;  // K-group, wave within the group
  const int wr = w4 >> 1, wc = w4 & 1;
  int m0, n0;
  xcd_tile(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);
  const int nmine = (nit - kg + 1) / 2;  // K-steps kg, kg+2, ..
  const int npair = (nit + 1) / 2;

  const int rl = w4 * 32 + (lane >> 3), slot = lane & 7;
  const int cq = swz(rl, slot), cq8a = cq * 8, cq8b = (cq ^ 4) * 8;
  int bt[4], tt[4];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rl + 8 * i;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  const int c8[4] = {cq8a, cq8b, cq8a, cq8b};

  int qs = 0, qj = 0, qkc = 0;
#define ADV()                                                                      \
  do {                                                                             \
    const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                  \
    const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);           \
    if (++qkc == nks_) {                                                           \
      qkc = 0;                                                                     \
      if (++qj == taps_) {                                                         \
        qj = 0;                                                                    \
        ++qs;                                                                      \
      }                                                                            \
    }                                                                              \
  } while (0)
  if (kg == 1 && nit > 0) ADV();  // group 1 starts at K-step 1
#define TAP_PTRS(S) \
  tap_ptrs(S, qj, Npad, n0, rl, cq8a, cq8b, bt[0], bt[1], bt[2], bt[3], tt[0], tt[1], tt[2], tt[3], okm)
  TapPtrs P = qs == 0 ? TAP_PTRS(S0) : (qs == 1 ? TAP_PTRS(S1) : TAP_PTRS(S2));
  // issue this group's next K-step into stage `st`, then step the cursor over the other
  // group's K-step (pointers rebuilt when a tap / segment boundary is crossed)
#define ISSUE2(st)                                                                       \
  do {                                                                                   \
    char* As_ = smem + (st) * STAGE + kg * GSET + w4 * 32 * 128;                         \
    const int kb_ = qkc * BK2;                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool oa = ((P.va >> i) & 1) && kb_ + c8[i] < P.K;                            \
      glds16(oa ? (const void*)(P.pa[i] + kb_ * 2) : (const void*)zp, As_ + i * 1024);   \
    }                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool ob = kb_ + c8[i] < P.Kp;                                                \
      glds16(ob ? (const void*)(P.pb[i] + kb_ * 2) : (const void*)zp,                    \
             As_ + TILE + i * 1024);                                                     \
    }                                                                                    \
    const int qs0_ = qs, qj0_ = qj;                                                      \
    ADV();                                                                               \
    if (qs < nseg) ADV();                                                                \
    if (qs < nseg && (qs != qs0_ || qj != qj0_))                                         \
      P = qs == 0 ? TAP_PTRS(S0) : (qs == 1 ? TAP_PTRS(S1) : TAP_PTRS(S2));              \
  } while (0)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nmine > 0) ISSUE2(0);
  const int arow = lane & 15, kq = lane >> 4;
  const int ra = wr * 64 + arow, rbr = wc * 64 + arow;
  const int oa0 = ra * 128 + swz(ra, kq) * 16, oa1 = ra * 128 + swz(ra, kq + 4) * 16;
  const int ob0 = TILE + rbr * 128 + swz(rbr, kq) * 16, ob1 = TILE + rbr * 128 + swz(rbr, kq + 4) * 16;
  for (int p = 0; p < npair; ++p) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // pair p visible; every wave is done with pair p-1
    if (p + 1 < nmine) ISSUE2((p + 1) & 1);
    if (p < nmine) {
      const char* St = smem + (p & 1) * STAGE + kg * GSET;
      bf16x8 fa[2][4], fb[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          fa[h][i] = *(const bf16x8*)(St + (h ? oa1 : oa0) + i * 2048);
          fb[h][i] = *(const bf16x8*)(St + (h ? ob1 : ob0) + i * 2048);
        }
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[h][i], fb[h][j], acc[i][j], 0, 0, 0);
    }
  }
#undef ISSUE2
#undef TAP_PTRS
#undef ADV
  // group 1's tile through LDS into group 0's accumulators
  float* T = (float*)smem;
  __syncthreads();
  if (kg == 1) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(wr * 64 + mt * 16 + (lane >> 4) * 4 + r) * EP + wc * 64 + nt * 16 + (lane & 15)] =
              acc[mt][nt][r];
  }
  __syncthreads();
  if (kg == 0) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[mt][nt][r] +=
              T[(wr * 64 + mt * 16 + (lane >> 4) * 4 + r) * EP + wc * 64 + nt * 16 + (lane & 15)];
  }
  if (a.vec_out) {
    gemm_epilogue_lds<NTHR2>(a, acc, m0, n0, wr, wc, lane, tid, smem, kg == 0);
  } else if (kg == 0) {
    gemm_epilogue(a, acc, m0, n0, wr, wc, lane);
  }
}

// ------------------------------------------------------ 256 x 256 bf16-operand GEMM
// The large-M launches of the step (DiffNet gate / res-skip GEMMs at 30 k frames) are
// bound by what the CUs pull from L2 into LDS (~70 GB/s per CU, MI355X_MICROARCH.md
// "Indexed rows"): a 128 x 128 tile moves 32 KB per 64-deep K step for 2 MFLOP, a 256 x 256
// tile 64 KB for 8 MFLOP -- half the L2 -> LDS bytes per FLOP.  8 waves (2 x 4), each a
// 128 x 64 sub-tile of 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators; both operand images
// staged by global_load_lds with the same swizzle and per-tap staging pointers as the
// 128 x 128 kernel; two stages (128 KB of LDS, one workgroup per CU: a K step is 2 x 64
// MFMAs per SIMD, long enough to cover the L2 latency of the next step's loads).  The
// epilogue stages the fp32 tile through LDS in four 64-row chunks and runs the same
// per-element arithmetic as gemm_epilogue_lds (no column sums).
constexpr int BMB = 256, BNB = 256, NTHRB = 512, EPB = BNB + 4, CHR = 64;

__device__ __forceinline__ void xcd_tile_big(int& m0, int& n0) {
  const int nM = gridDim.x, nN = gridDim.y, total = nM * nN;
  const int orig = blockIdx.x + blockIdx.y * nM;
  const int xcd = orig & 7, q = total >> 3, r = total & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  m0 = (wg / nN) * BMB;
  n0 = (wg % nN) * BNB;
}

// Operands of one batch of EB epilogue rows, loaded ahead of the previous batch's stores
// (vmcnt counts loads and stores in issue order: a load issued after stores is waited for
// together with them).  RESSKIP: x = residual input, y = running skip sum, z = the next
// block's per-sequence add; other epilogues: x, y = their p1, p2 operands, z = the per-
// sequence add of the bf16 copy (PLAIN / ADDSCALE).
constexpr int EBB = 1;  // rows whose operands are in flight together (register budget: the
                        // waves of the second row half still hold 128 accumulators)
template <int EB>
struct EpiPreT {
  f32x4 x[EB], y[EB], z[EB];
};
using EpiPre = EpiPreT<EBB>;
__device__ __forceinline__ bool big_pairs(const GemmArgs& a) {
  return a.epi == EPI_GATE || a.epi == EPI_RESSKIP || a.epi == EPI_GATE_TS;
}
// loads batch kb (rows kb .. kb + EB - 1 of this thread) of the chunk at mb into p
template <int COLS, int NT, int EB = EBB>
__device__ __forceinline__ void epi_pre(const GemmArgs& a, int mb, int n0, int tid, int kb,
                                        EpiPreT<EB>& p) {
  if (a.epi == EPI_RESSKIP) {
    const int q4 = tid % (COLS / 8), c = n0 / 2 + (q4 >> 2) * 16 + (q4 & 3) * 4;
    if (c >= a.C) return;
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      RsOps o;
      rs_load(a, mb + tid / (COLS / 8) + (kb + k) * (NT / (COLS / 8)), c, o);
      p.x[k] = o.xr;
      p.y[k] = o.s0;
      p.z[k] = o.rr;
    }
    return;
  }
  if (big_pairs(a)) return;
  const bool want1 = (a.epi == EPI_PLAIN && a.accum) || a.epi == EPI_ADDSCALE ||
                     a.epi == EPI_RELU_MASK || a.epi == EPI_GATE_BWD;
  const bool want2 = (a.epi == EPI_RELU_MASK && a.accum) || a.epi == EPI_GATE_BWD;
  const bool wr = a.ybf && a.ybf_radd && (a.epi == EPI_PLAIN || a.epi == EPI_ADDSCALE);
  const int col = n0 + (tid % (COLS / 4)) * 4;
  if (!(want1 || want2 || wr) || a.N - col < 4) return;
#pragma unroll
  for (int k = 0; k < EB; ++k) {
    const int m = mb + tid / (COLS / 4) + (kb + k) * (NT / (COLS / 4));
    if (want1 || want2) gen_load(a, m, col, want2, p.x[k], p.y[k]);
    if (wr && m < a.M) p.z[k] = ld4(a.ybf_radd + (long long)(m / a.Tout) * a.ybf_radd_ld + col);
  }
}

// One staged tile (or chunk of one): rows [0, ROWS) of T (row stride LDT) are output rows
// mb.., columns [0, COLS) are n0.., NT threads.
// BIAS_IN_T: T already holds acc + bias.  pre holds this chunk's first batch of operands on
// entry; the last batch loads the next chunk's first batch (unless `last`) before its stores.
template <int ROWS, int COLS, int NT, int LDT, bool BIAS_IN_T, int EB = EBB>
__device__ __forceinline__ void epilogue_tile(const GemmArgs& a, const float* T, int mb, int n0,
                                              int tid, bool last, EpiPreT<EB>& pre) {
  const int M = a.M;
  if (a.epi == EPI_NONE) {
    if (T[tid] == 12345.678f && mb < 0) a.Y[0] = T[tid + 1];
    return;
  }
  const bool hb = !BIAS_IN_T && a.bias;
  if (a.gate8 && (a.epi == EPI_GATE || a.epi == EPI_GATE_TS)) {
    gate_tile8<NT, ROWS, COLS / 16, BIAS_IN_T>(a, T, LDT, mb, n0, tid);
    return;
  }
  if (big_pairs(a)) {
    // COLS / 2 output channels per row: gate/filter interleaved by 16 in the packed columns
    constexpr int NI = ROWS * (COLS / 8) / NT;
    const int q4 = tid % (COLS / 8), q = q4 >> 2, j = (q4 & 3) * 4;
    const int c = n0 / 2 + q * 16 + j;
    const int gc = q * 32 + j;
    if (c >= a.C) return;
    f32x4 bg = {0.f, 0.f, 0.f, 0.f}, bfl = {0.f, 0.f, 0.f, 0.f};
    if (hb) {
      bg = ld4(a.bias + n0 + gc);
      bfl = ld4(a.bias + n0 + gc + 16);
    }
#pragma unroll 1
    for (int kb = 0; kb < NI; kb += EB) {
    EpiPreT<EB> cur = pre;
    if (a.epi == EPI_RESSKIP) {
      if (kb + EB < NI) epi_pre<COLS, NT, EB>(a, mb, n0, tid, kb + EB, pre);
      else if (!last) epi_pre<COLS, NT, EB>(a, mb + ROWS, n0, tid, 0, pre);
    }
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      const int row = tid / (COLS / 8) + (kb + k) * (NT / (COLS / 8));
      const int m = mb + row;
      if (m >= M) continue;
      f32x4 g = ld4(T + row * LDT + gc), f = ld4(T + row * LDT + gc + 16);
      if (hb) {
        g += bg;
        f += bfl;
      }
      if (a.epi == EPI_RESSKIP) {
        rs_store(a, m, c, g, f, RsOps{cur.x[k], cur.y[k], cur.z[k]});
      } else if (a.epi == EPI_GATE) {
        st4_aux0(a, (long long)m * a.ld0 + c, g);
        st4_aux0(a, (long long)m * a.ld0 + a.C + c, f);
        f32x4 z;
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = fsigmoid_(g[e]) * ftanh_(f[e]);
        if (a.Y) st4(a.Y + (long long)m * a.ldy + c, z);
        shadow4(a, m, c, z);
      } else {
        f32x4 z;
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = ftanh_(g[e]) * fsigmoid_(f[e]);
        if (a.Y) st4(a.Y + (long long)m * a.ldy + c, z);
        shadow4(a, m, c, z);
      }
    }
    }
    return;
  }
  constexpr int NI = ROWS * (COLS / 4) / NT;
  const int cq = tid % (COLS / 4), col = n0 + cq * 4;
  const int ne = min(4, a.N - col);
  if (ne <= 0) return;
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if (hb) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < ne) bv[e] = a.bias[col + e];
  }
  static_assert(NI % EB == 0, "rows per thread in batches of EB");
#pragma unroll 1
  for (int kb = 0; kb < NI; kb += EB) {
  EpiPreT<EB> cur = pre;
  if (kb + EB < NI) epi_pre<COLS, NT, EB>(a, mb, n0, tid, kb + EB, pre);
  else if (!last) epi_pre<COLS, NT, EB>(a, mb + ROWS, n0, tid, 0, pre);
#pragma unroll
  for (int k = 0; k < EB; ++k) {
    const int row = tid / (COLS / 4) + (kb + k) * (NT / (COLS / 4));
    const int m = mb + row;
    if (m >= M) continue;
    f32x4 v = ld4(T + row * LDT + cq * 4);
    if (hb) v += bv;
    const f32x4 p1 = cur.x[k], p2 = cur.y[k];
    float* y = a.Y + (long long)m * a.ldy + col;
    if (ne == 4) {
      if (a.epi == EPI_PLAIN) {
        if (a.accum) v += p1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (a.relu == 1) v[e] = fmaxf(v[e], 0.f);
          else if (a.relu == 2) v[e] = sigmoidf_(v[e]);
        }
        st4(y, v);
        shadow4r(a, m, col, v, cur.z[k]);
      } else if (a.epi == EPI_ADDSCALE) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = __builtin_fmaf(a.alpha, p1[e], v[e]);
          v[e] = a.relu == 1 ? fmaxf(v[e], 0.f) : v[e];
        }
        st4(y, v);
        shadow4r(a, m, col, v, cur.z[k]);
      } else if (a.epi == EPI_RELU_MASK) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = p1[e] > 0.f ? v[e] : 0.f;
        if (a.accum) v += p2;
        st4(y, v);
        shadow4(a, m, col, v);
      } else if (a.epi == EPI_GATE_BWD) {
        f32x4 dg, df;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t0, t1;
          gate_bwd_(v[e], p1[e], p2[e], t0, t1);
          dg[e] = t0;
          df[e] = t1;
        }
        if (a.Y) {
          st4(y, dg);
          st4(y + a.C, df);
        }
        shadow4(a, m, col, dg);
        shadow4(a, m, a.C + col, df);
      }
    } else {
      for (int e = 0; e < ne; ++e) {
        float w = v[e];
        float* ye = y + e;
        if (a.epi == EPI_PLAIN) {
          if (a.accum) w += *ye;
          if (a.relu == 1) w = fmaxf(w, 0.f);
          else if (a.relu == 2) w = sigmoidf_(w);
          *ye = w;
        } else if (a.epi == EPI_ADDSCALE) {
          w = __builtin_fmaf(a.alpha, a.aux1[(long long)m * a.ld1 + col + e], w);
          *ye = a.relu == 1 ? fmaxf(w, 0.f) : w;
        } else if (a.epi == EPI_RELU_MASK) {
          w = a.aux1[(long long)m * a.ld1 + col + e] > 0.f ? w : 0.f;
          *ye = a.accum ? *ye + w : w;
        } else if (a.epi == EPI_GATE_BWD) {
          const float g = ld_aux1(a, (long long)m * a.ld1 + col + e);
          const float f = ld_aux1(a, (long long)m * a.ld1 + a.C + col + e);
          gate_bwd_(w, g, f, ye[0], ye[a.C]);
        }
      }
    }
  }
  }
}

// The fused uSFGAN block's second half (b16_body<.., true>): acc holds this wave's 64 x 64
// part of the 128 x 128 gate/filter tile (n0 = 0: packed column group q = 2 wc + p holds the
// gate of channels 16 q .. 16 q + 15, then their filter).
__device__ __forceinline__ void usf_block_tail(const GemmArgs& a, const GemmArgs& a2,
                                               f32x4 (&acc)[4][4], char* smem, int tid, int lane,
                                               int wr, int wc, int m0) {
  const int l16 = lane & 15, kq = lane >> 4;
  // output-projection weight fragments straight from global memory (8 KB, L2-resident):
  // rows n = wc*32 + 16 j + l16, k chunk h*4 + kq of the packed [Npad][Kp = 64] image
  const __bf16* W2 = (const __bf16*)a2.W + a2.seg[0].wofs;
  const int kp2 = a2.seg[0].Kp;
  bf16x8 fb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[h][j] = *(const bf16x8*)(W2 + (long long)(wc * 32 + 16 * j + l16) * kp2 + h * 32 + kq * 8);
  float bg[2] = {0.f, 0.f}, bfl[2] = {0.f, 0.f};
  if (a.bias) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      bg[p] = a.bias[wc * 64 + p * 32 + l16];
      bfl[p] = a.bias[wc * 64 + p * 32 + 16 + l16];
    }
  }
  EpiPreT<2> pre;
  epi_pre<64, NTHR, 2>(a2, m0, 0, tid, 0, pre);  // a2 has 64 output columns: its first batch
  // z = tanh(g) * sigmoid(f) in bf16 into the [128][64] swizzled A image of the second GEMM
  __syncthreads();  // every wave is done with the K loop's images
  char* A2 = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + i * 16 + kq * 4 + r, ch = wc * 32 + p * 16 + l16;
        const float g = acc[i][2 * p][r] + bg[p], f = acc[i][2 * p + 1][r] + bfl[p];
        const float z = ftanh_(g) * fsigmoid_(f);
        *(__bf16*)(A2 + row * 128 + swz(row, ch >> 3) * 16 + (ch & 7) * 2) = (__bf16)z;
      }
  __syncthreads();
  // out = z W_out^T: 128 x 64, waves 2 x 2 of 64 x 32 (4 x 2 MFMA tiles), K = 64
  f32x4 acc2[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ra = wr * 64 + l16;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bf16x8 fa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = *(const bf16x8*)(A2 + (ra + 16 * i) * 128 + swz(ra, kq + 4 * h) * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[h][j], acc2[i][j], 0, 0, 0);
  }
  // a2's epilogue (ADDSCALE on the residual stream + its bf16 copy) over an LDS-staged tile
  constexpr int LT = 64 + 4;
  float* T = (float*)(smem + 16384);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wr * 64 + i * 16 + kq * 4 + r) * LT + wc * 32 + j * 16 + l16] = acc2[i][j][r];
  __syncthreads();
  epilogue_tile<BM, 64, NTHR, LT, false, 2>(a2, T, m0, 0, tid, true, pre);
}

// per-lane bias of the wave's accumulator columns (nt = 0..3), added while staging
__device__ __forceinline__ void big_bias(const GemmArgs& a, int n0, int wc, int lane, float (&bs)[4]) {
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = n0 + wc * 64 + nt * 16 + (lane & 15);
    bs[nt] = a.bias && n < a.N ? a.bias[n] : 0.f;
  }
}

// GATE8: the launch runs the 16-B gate epilogue (the DiffNet gate GEMM), compiled without
// the other epilogues' operand registers.  (An activation image three slots deep, issued two
// K-steps ahead -- 96 KB in flight in all 160 KB of LDS -- measured slower: 47.9 vs 43.6 us.)
template <bool GATE8>
__global__ __launch_bounds__(NTHRB) void conv_gemm_b16_big_kernel(const GemmArgs a) {
  constexpr int TILE_A = BMB * BK2 * 2;  // 32 KB
  constexpr int STAGE = TILE_A + BNB * BK2 * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  xcd_tile_big(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);
  // staging: wave wid fills rows wid*32 .. +31 of both images, 4 glds (8 rows each) per image
  const int rl = wid * 32 + (lane >> 3), slot = lane & 7;
  const int cq = swz(rl, slot), cq8a = cq * 8, cq8b = (cq ^ 4) * 8;
  int bt[4], tt[4];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rl + 8 * i;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  const int c8[4] = {cq8a, cq8b, cq8a, cq8b};
  int qs = 0, qj = 0, qkc = 0;
#define TAP_PTRS(S) \
  tap_ptrs(S, qj, Npad, n0, rl, cq8a, cq8b, bt[0], bt[1], bt[2], bt[3], tt[0], tt[1], tt[2], tt[3], okm)
  TapPtrs P = TAP_PTRS(S0);
#define ISSUE_BIG(it)                                                                    \
  do {                                                                                   \
    char* As_ = smem + ((it) & 1) * STAGE + wid * 32 * 128;                              \
    const int kb_ = qkc * BK2;                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool oa = ((P.va >> i) & 1) && kb_ + c8[i] < P.K;                            \
      glds16(oa ? (const void*)(P.pa[i] + kb_ * 2) : (const void*)zp, As_ + i * 1024);   \
    }                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                      \
      const bool ob = kb_ + c8[i] < P.Kp;                                                \
      glds16(ob ? (const void*)(P.pb[i] + kb_ * 2) : (const void*)zp,                    \
             As_ + TILE_A + i * 1024);                                                   \
    }                                                                                    \
    const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                        \
    const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
    if (++qkc == nks_) {                                                                 \
      qkc = 0;                                                                           \
      if (++qj == taps_) {                                                               \
        qj = 0;                                                                          \
        ++qs;                                                                            \
      }                                                                                  \
      if (qs < nseg) P = qs == 0 ? TAP_PTRS(S0) : (qs == 1 ? TAP_PTRS(S1) : TAP_PTRS(S2)); \
    }                                                                                    \
  } while (0)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nit > 0) ISSUE_BIG(0);
  const int arow = lane & 15, kq = lane >> 4;
  const int ra = wr * 128 + arow, rbr = wc * 64 + arow;
  const int oa0 = ra * 128 + swz(ra, kq) * 16, oa1 = ra * 128 + swz(ra, kq + 4) * 16;
  const int ob0 = TILE_A + rbr * 128 + swz(rbr, kq) * 16;
  const int ob1 = TILE_A + rbr * 128 + swz(rbr, kq + 4) * 16;
  for (int it = 0; it < nit; ++it) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // tile `it` visible; every wave is done with tile it-1
    if (it + 1 < nit) ISSUE_BIG(it + 1);
    const char* St = smem + (it & 1) * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(St + (h ? ob1 : ob0) + j * 2048);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(St + (h ? oa1 : oa0) + i * 2048);
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // DS reads first
      __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);  // then the MFMAs
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
#undef ISSUE_BIG
#undef TAP_PTRS
  // epilogue: four 64-row chunks staged through LDS (row stride EPB floats) with the bias
  // added while staging; the first chunk's epilogue operands are loaded before any store
  float bs[4];
  const bool bias_st = a.bias != nullptr;
  if (bias_st) big_bias(a, n0, wc, lane, bs);
  EpiPre pre;
  if (!GATE8) epi_pre<BNB, NTHRB>(a, m0, n0, tid, 0, pre);
  float* T = (float*)smem;
  __syncthreads();
  // (the chunk loop is not unrolled -- its body is large -- so the accumulator half is
  // picked by a branch with static indices, never by a runtime index into acc)
#define STAGE_HALF(H)                                                                     \
  _Pragma("unroll") for (int mt2 = 0; mt2 < 4; ++mt2)                                     \
  _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                        \
  _Pragma("unroll") for (int r = 0; r < 4; ++r)                                           \
      T[(mt2 * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] =        \
          bias_st ? acc[(H) * 4 + mt2][nt][r] + bs[nt] : acc[(H) * 4 + mt2][nt][r]
#pragma unroll 1
  for (int c = 0; c < BMB / CHR; ++c) {
    if (wr == (c >> 1)) {
      if (c & 1) {
        STAGE_HALF(1);
      } else {
        STAGE_HALF(0);
      }
    }
    __syncthreads();
    if (GATE8) gate_tile8<NTHRB, CHR, BNB / 16, true>(a, T, EPB, m0 + c * CHR, n0, tid);
    else epilogue_tile<CHR, BNB, NTHRB, EPB, true>(a, T, m0 + c * CHR, n0, tid, c == BMB / CHR - 1, pre);
    __syncthreads();
  }
#undef STAGE_HALF
}

// Split-K reduction + epilogue: 64 rows x 256 columns per block, the ksplit partial slices
// summed in slice order into an LDS tile (columns past Npad read as zero), then the same
// per-element epilogue as the 256 x 256 kernel.
__global__ __launch_bounds__(NTHRB) void splitk_epilogue_kernel(const GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* T = (float*)smem;
  const int mb = blockIdx.x * CHR, n0 = blockIdx.y * BNB, tid = threadIdx.x;
  const int M = a.M, Npad = a.Npad;
  for (int e = tid; e < CHR * (BNB / 4); e += NTHRB) {
    const int row = e / (BNB / 4), c4 = e % (BNB / 4);
    const int m = mb + row, n = n0 + c4 * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m < M && n < Npad) {
      for (int z = 0; z < a.ksplit; ++z)
        v += *(const f32x4*)(a.part + ((long long)z * M + m) * Npad + n);
    }
    *(f32x4*)(T + row * EPB + c4 * 4) = v;
  }
  EpiPre pre;
  epi_pre<BNB, NTHRB>(a, mb, n0, tid, 0, pre);
  __syncthreads();
  epilogue_tile<CHR, BNB, NTHRB, EPB, false>(a, T, mb, n0, tid, true, pre);
}

// ---------------------------------------- 256 x 256, 32-deep K steps, S-stage ring
// Measured on the gate GEMM (tools/gate_probe.py, rocprofv3 PMC): the 64-deep two-stage
// kernels above wait on their LDS-DMA loads (SQ_WAIT_ANY 45 % of wave cycles, MFMA busy
// 21 %) at ~18 GB/s per CU -- the rate that 64 KB in flight per CU sustains at ~3.5 us
// of load latency under full-chip load, for both tile shapes.  Throughput follows bytes
// in flight, so this kernel keeps S - 1 32-deep stages of both operand images in flight
// (S = 5: 128 KB of 160 KB LDS) with the 256 x 256 tile's L2 -> LDS bytes per FLOP.
// 64-B LDS rows: the 16-B chunk c of row r sits in slot c ^ ((r >> 1) & 3), conflict-free
// for the MFMA fragment reads (ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS); the
// DMA writes stay lane-linear, each lane fetching the chunk its slot holds.
constexpr int BK3 = 32;

template <int N>
__device__ __forceinline__ void wait_vm_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

struct TapPtrs2 {
  const char* pa[2];
  const char* pb[2];
  unsigned va;
  int K, Kp;
};

__device__ __forceinline__ TapPtrs2 tap_ptrs2(const SegU S, int j, int Npad, int n0, int r0,
                                              int c8, const int b0, const int b1, const int t0,
                                              const int t1, unsigned okm) {
  TapPtrs2 P;
  const int bt[2] = {b0, b1}, tt[2] = {t0, t1};
  const int shj = S.shift0 + j * S.dil;
  P.va = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ts = tt[i] + shj;
    const int src = S.pad == PAD_ZERO ? ((unsigned)ts < (unsigned)S.Tin ? ts : -1)
                                      : pad_src(ts, S.Tin, S.pad);
    const bool ok = ((okm >> i) & 1) && src >= 0;
    P.va |= ok ? (1u << i) : 0u;
    P.pa[i] = (const char*)(S.x + (unsigned)((bt[i] * S.Tin + (ok ? src : 0)) * S.ld + c8));
    P.pb[i] = S.w + ((unsigned)((j * Npad + n0 + r0 + 16 * i) * S.Kp + c8)) * 2;
  }
  P.K = S.K;
  P.Kp = S.Kp;
  return P;
}

template <int STAGES>
__global__ __launch_bounds__(NTHRB) void conv_gemm_b16_ring_kernel(const GemmArgs a) {
  static_assert(STAGES >= 3 && STAGES <= 5, "stages");
  constexpr int IMG = BMB * BK3 * 2;   // 16 KB: one operand image of one stage
  constexpr int STAGE = 2 * IMG;
  constexpr int GL = 4;                // glds per thread per stage (2 A rows + 2 B rows)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  xcd_tile_big(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  auto nk3 = [](const SegU& S) { return (S.K + BK3 - 1) / BK3; };
  const int k0 = uni(nk3(S0)), k1 = uni(nk3(S1)), k2 = uni(nk3(S2));
  const int nit = k0 * S0.taps + (nseg > 1 ? k1 * S1.taps : 0) + (nseg > 2 ? k2 * S2.taps : 0);
  // staging: wave wid fills the 1-KB pieces 2*wid and 2*wid + 1 (16 rows each) of both
  // images: rows r0 = 32*wid + lane/4 and r0 + 16; lane slot lane & 3 holds chunk c
  const int r0 = wid * 32 + (lane >> 2);
  const int c = (lane & 3) ^ (((lane >> 2) >> 1) & 3), c8 = c * 8;
  int bt[2], tt[2];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + r0 + 16 * i;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  int qs = 0, qj = 0, qkc = 0;
#define TAP_PTRS2(S) tap_ptrs2(S, qj, Npad, n0, r0, c8, bt[0], bt[1], tt[0], tt[1], okm)
  TapPtrs2 P = TAP_PTRS2(S0);
#define ISSUE_RING(it)                                                                   \
  do {                                                                                   \
    char* As_ = smem + ((it) % STAGES) * STAGE + wid * 2048;                             \
    const int kb_ = qkc * BK3;                                                           \
    const bool in_ = kb_ + c8 < P.K, inb_ = kb_ + c8 < P.Kp;                             \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                      \
      const bool oa = ((P.va >> i) & 1) && in_;                                          \
      glds16(oa ? (const void*)(P.pa[i] + kb_ * 2) : (const void*)zp, As_ + i * 1024);   \
    }                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 2; ++i)                                        \
      glds16(inb_ ? (const void*)(P.pb[i] + kb_ * 2) : (const void*)zp,                  \
             As_ + IMG + i * 1024);                                                      \
    const int nks_ = qs == 0 ? k0 : (qs == 1 ? k1 : k2);                                 \
    const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
    if (++qkc == nks_) {                                                                 \
      qkc = 0;                                                                           \
      if (++qj == taps_) {                                                               \
        qj = 0;                                                                          \
        ++qs;                                                                            \
      }                                                                                  \
      if (qs < nseg) P = qs == 0 ? TAP_PTRS2(S0) : (qs == 1 ? TAP_PTRS2(S1) : TAP_PTRS2(S2)); \
    }                                                                                    \
  } while (0)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nit) ISSUE_RING(p);
  const int arow = lane & 15, kq = lane >> 4;
  const int sw = (kq ^ ((arow >> 1) & 3)) * 16;  // rows + 16 i keep the slot
  const int oa = (wr * 128 + arow) * 64 + sw, ob = IMG + (wc * 64 + arow) * 64 + sw;
  for (int it = 0; it < nit; ++it) {
    const int ahead = min(STAGES - 2, nit - 1 - it);  // stages issued after tile `it`
    if (ahead >= 3) wait_vm_n<3 * GL>();
    else if (ahead == 2) wait_vm_n<2 * GL>();
    else if (ahead == 1) wait_vm_n<GL>();
    else wait_vm_n<0>();
    __builtin_amdgcn_s_barrier();  // tile `it` visible; every wave is done with tile it-1
    if (it + STAGES - 1 < nit) ISSUE_RING(it + STAGES - 1);
    const char* St = smem + (it % STAGES) * STAGE;
    bf16x8 fa[8], fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(St + ob + j * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(St + oa + i * 1024);
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
#undef ISSUE_RING
#undef TAP_PTRS2
  EpiPre pre;
  epi_pre<BNB, NTHRB>(a, m0, n0, tid, 0, pre);
  float* T = (float*)smem;
  __syncthreads();
#define STAGE_HALF(H)                                                                     \
  _Pragma("unroll") for (int mt2 = 0; mt2 < 4; ++mt2)                                     \
  _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                        \
  _Pragma("unroll") for (int r = 0; r < 4; ++r)                                           \
      T[(mt2 * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] =        \
          acc[(H) * 4 + mt2][nt][r]
#pragma unroll 1
  for (int cch = 0; cch < BMB / CHR; ++cch) {
    if (wr == (cch >> 1)) {
      if (cch & 1) {
        STAGE_HALF(1);
      } else {
        STAGE_HALF(0);
      }
    }
    __syncthreads();
    epilogue_tile<CHR, BNB, NTHRB, EPB, false>(a, T, m0 + cch * CHR, n0, tid, cch == BMB / CHR - 1, pre);
    __syncthreads();
  }
#undef STAGE_HALF
}

// ------------------------------ 256 x 256, 8 waves, a 64-deep K-step in four phases
// The two-stage kernels above wait for the whole next K-step (vmcnt(0)) before every step's
// barrier, so each step starts with its loads' full latency exposed (MFMA busy ~26 % on the
// gate GEMM).  Here (the counted-wait schedule of cdna_hip_programming.md §5 "The 256² 8-phase
// template", laid out for this engine's implicit-conv staging) a K-step is four phases, each
// one output quadrant (64 x 32: 4 x 2 tiles x 2 k-chunks = 16 MFMAs) of every wave's 128 x 64
// sub-tile, and each operand image is four half-tiles whose LDS region is read in ONE phase:
//   j = 0  A0: A rows {0-63, 128-191} (the first 64 rows of each wave row)   read in phase 0
//   j = 1  B0: B rows 64 c + {0-31}, c = 0..3 (kept in registers for phase 3) read in phase 0
//   j = 2  B1: B rows 64 c + {32-63}                                          read in phase 1
//   j = 3  A1: A rows {64-127, 192-255}                                       read in phase 2
// Half-tile h = 4 t + j (K-step t, buffer t & 1) is issued in phase P = h - 6 (P = 4 t + p
// counts the phases of the K loop), two buffer_load ... lds per thread.  What it overwrites
// was last read in phase <= P - 2; what phase P + 1 reads is retired by the counted wait
// before phase P's barrier, so four half-tiles (8 DMA instructions per thread) stay in flight
// across every barrier and the loop never drains.  Per accumulator the K order is the other
// kernels' (k-chunks in order), so the bits are identical.  Operands through buffer
// resources: rows past M, zero padding and k past K / Kp read zeros (out-of-range offsets).
// Epilogue: the 256 x 256 kernel's (four 64-row chunks staged through LDS).
constexpr unsigned P8_OOB = 0x80000000u;  // a buffer offset past every resource (zeros)
constexpr int P8_IMG = BMB * BK2 * 2;      // 32 KB: one operand image of one K-step
constexpr int P8_BUF = 2 * P8_IMG;         // A + B images of one K-step

// this lane's 4 A row offsets (bytes from the segment's x; rows rA + {0, 128, 64, 192}) and
// its first B row's offset (rB; the others add a wave-uniform row delta) for tap j
struct P8Offs {
  unsigned oa[4];
  unsigned ob;
};

__device__ __forceinline__ P8Offs p8_offs(const SegU S, int j, int Npad, int n0, int rB, int ca8,
                                          int cb8, const int (&bt)[4], const int (&tt)[4],
                                          unsigned okm) {
  P8Offs o;
  const int shj = S.shift0 + j * S.dil;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ts = tt[i] + shj;
    const int src = S.pad == PAD_ZERO ? ((unsigned)ts < (unsigned)S.Tin ? ts : -1)
                                      : pad_src(ts, S.Tin, S.pad);
    const bool ok = ((okm >> i) & 1) && src >= 0;
    o.oa[i] = ok ? (unsigned)((bt[i] * S.Tin + src) * S.ld + ca8) * 2u : P8_OOB;
  }
  o.ob = (unsigned)((j * Npad + n0 + rB) * S.Kp + cb8) * 2u;
  return o;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t p8_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ void p8_dma(__amdgpu_buffer_rsrc_t r, unsigned off, char* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)l, 16, off, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void p8_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// BAR2: the template's second barrier after each phase's MFMAs (ONE barrier per phase is also
// valid: every region is rewritten >= 2 phases after its last read, so the writer has passed the
// barrier that the reader reaches only after its lgkmcnt wait of that read)
// EPK: EPI_GATE -- the 16-B gate epilogue (DiffNet gate GEMM); EPI_PLAIN -- the lean plain
// epilogue (fp32 Y = acc + bias, no accumulate / activation / copies, N % 4 == 0: the
// projections), the whole tile staged in two 128-row passes by all 8 waves; -1 -- every other
// epilogue (epilogue_tile, 64-row chunks).  Instances per epilogue keep the other epilogues'
// operand registers out of the K loop (the generic instance spills in its epilogue).
constexpr int P8_PROBE_NODMA = 100 + EPI_NONE, P8_PROBE_NOMMA = 200 + EPI_NONE;
template <int EPK, bool BAR2>
__global__ __launch_bounds__(NTHRB) void conv_gemm_b16_p8_kernel(const GemmArgs a) {
  constexpr bool GATE8 = EPK == EPI_GATE;
  constexpr bool NODMA = EPK == P8_PROBE_NODMA;  // measurement: the K loop without its loads
  constexpr bool NOMMA = EPK == P8_PROBE_NOMMA;  // measurement: the loads (and LDS reads) alone
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  xcd_tile_big(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);
  const int nh = 4 * nit;  // half-tiles
  // staged rows: A rA + {0, 128, 64, 192}, B rB + {0, 128, 32, 160}; every one of them keeps
  // the swizzle of rA / rB (bits 1..3 of the row), so one chunk per operand per lane
  const int rA = wid * 8 + (lane >> 3), rB = (wid & 3) * 8 + (wid >> 2) * 64 + (lane >> 3);
  const int ca8 = swz(rA, lane & 7) * 8, cb8 = swz(rB, lane & 7) * 8;
  int bt[4], tt[4];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rA + (i & 1) * 128 + (i >> 1) * 64;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  // wave-uniform LDS bases of this wave's pieces within an image
  const int la = wid * 8 * 128, lb = ((wid & 3) * 8 + (wid >> 2) * 64) * 128;
  // staging cursor: the K-step whose half-tiles are issued next (segment, tap, k-step)
  int qs = 0, qj = 0, qkc = 0;
#define P8_OFFS(S) p8_offs(S, qj, Npad, n0, rB, ca8, cb8, bt, tt, okm)
  P8Offs O = P8_OFFS(S0);
  __amdgpu_buffer_rsrc_t rxa = p8_rsrc(S0.x), rwb = p8_rsrc(S0.w);
  int qK = S0.K, qKp = S0.Kp;
  // half-tile h (its K-step's cursor is the current one)
#define P8_ISSUE(h)                                                                        \
  do {                                                                                     \
    const int j_ = (h) & 3;                                                                \
    char* L_ = smem + (((h) >> 2) & 1) * P8_BUF;                                           \
    const int kb_ = qkc * BK2;                                                             \
    const unsigned kb2_ = (unsigned)kb_ * 2u;                                              \
    if (j_ == 0 || j_ == 3) {                                                              \
      const bool in_ = kb_ + ca8 < qK;                                                     \
      const int i0_ = j_ == 0 ? 0 : 2;                                                     \
      char* La_ = L_ + la + (j_ == 0 ? 0 : 64 * 128);                                      \
      if (!NODMA) p8_dma(rxa, in_ ? O.oa[i0_] + kb2_ : P8_OOB, La_);                                   \
      if (!NODMA) p8_dma(rxa, in_ ? O.oa[i0_ + 1] + kb2_ : P8_OOB, La_ + 128 * 128);                   \
    } else {                                                                               \
      const bool in_ = kb_ + cb8 < qKp;                                                    \
      const int d_ = j_ == 1 ? 0 : 32;                                                     \
      char* Lb_ = L_ + P8_IMG + lb + d_ * 128;                                             \
      const unsigned ob_ = O.ob + (unsigned)(d_ * qKp) * 2u + kb2_;                        \
      if (!NODMA) p8_dma(rwb, in_ ? ob_ : P8_OOB, Lb_);                                                \
      if (!NODMA) p8_dma(rwb, in_ ? ob_ + (unsigned)(128 * qKp) * 2u : P8_OOB, Lb_ + 128 * 128);        \
    }                                                                                      \
    if (j_ == 3) { /* K-step done: advance the cursor */                                   \
      const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                        \
      const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
      if (++qkc == nks_) {                                                                 \
        qkc = 0;                                                                           \
        const int qs0_ = qs;                                                               \
        if (++qj == taps_) {                                                               \
          qj = 0;                                                                          \
          ++qs;                                                                            \
        }                                                                                  \
        if (qs < nseg) {                                                                   \
          if (qs != qs0_) {                                                                \
            rxa = p8_rsrc(qs == 1 ? S1.x : S2.x);                                          \
            rwb = p8_rsrc(qs == 1 ? S1.w : S2.w);                                          \
            qK = qs == 1 ? S1.K : S2.K;                                                    \
            qKp = qs == 1 ? S1.Kp : S2.Kp;                                                 \
          }                                                                                \
          O = qs == 0 ? P8_OFFS(S0) : (qs == 1 ? P8_OFFS(S1) : P8_OFFS(S2));               \
        }                                                                                  \
      }                                                                                    \
    }                                                                                      \
  } while (0)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: half-tiles 0..5, then wait for the two phase 0 reads (A0, B0 of K-step 0)
  const int npro = min(6, nh);
  for (int h = 0; h < npro; ++h) P8_ISSUE(h);
  if (npro - 2 >= 4) p8_wait<8>();
  else p8_wait<4>();  // nit == 1: half-tiles 0..3 issued, 2 may stay in flight
  __builtin_amdgcn_s_barrier();
  // BAR2: the two wave rows run half a phase apart (row 1 takes one extra barrier here, row 0
  // one after the loop), so on every SIMD one wave issues MFMAs while the other issues its LDS
  // reads and DMAs.  Phase P of row 0 is [barrier 2P-1, 2P] memory, [2P, 2P+1] MFMA; row 1 is
  // one barrier later.  WAR: a DMA of phase P (issued after barrier 2P-1 / 2P) overwrites data
  // last read at phase P-2, whose reads completed before the reader's MFMAs ended (barrier
  // 2P-3 / 2P-2).  RAW: each row's counted wait precedes its first barrier of the phase, which
  // the other row's reads of phase P+1 follow.
  if (BAR2 && wr == 1) __builtin_amdgcn_s_barrier();

  // fragment read offsets (rows + 16 i and the wave's quadrant rows keep the swizzle)
  const int arow = lane & 15, kq = lane >> 4;
  const int fa0 = (wr * 128 + arow) * 128 + swz(arow, kq) * 16;
  const int fa1 = (wr * 128 + arow) * 128 + swz(arow, kq + 4) * 16;
  const int fb0 = P8_IMG + (wc * 64 + arow) * 128 + swz(arow, kq) * 16;
  const int fb1 = P8_IMG + (wc * 64 + arow) * 128 + swz(arow, kq + 4) * 16;
  bf16x8 xa[2][4], xb0[2][2], xb1[2][2];
  // the counted wait of phase P (P = 4 t + p): the half-tiles phase P + 1 reads are retired;
  // `need` is the last of them, h = P + 6 the last issued (or nh - 1)
#define P8_WAIT(P, need)                                                                   \
  do {                                                                                     \
    const int al_ = min((P) + 7, nh) - 1 - (need);                                         \
    if (al_ >= 4) p8_wait<8>();                                                            \
    else if (al_ == 3) p8_wait<6>();                                                       \
    else if (al_ == 2) p8_wait<4>();                                                       \
    else if (al_ == 1) p8_wait<2>();                                                       \
    else p8_wait<0>();                                                                     \
  } while (0)
#define P8_MMA(I0, J0, B)                                                                  \
  do {                                                                                     \
    __builtin_amdgcn_s_setprio(1);                                                         \
    _Pragma("unroll") for (int h = 0; h < 2; ++h)                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                          \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                          \
      if (NOMMA) asm volatile("" ::"v"(xa[h][i]), "v"(B[h][j]));                           \
      else acc[(I0) + i][(J0) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(              \
          xa[h][i], B[h][j], acc[(I0) + i][(J0) + j], 0, 0, 0);                            \
    __builtin_amdgcn_s_setprio(0);                                                         \
    if (BAR2) __builtin_amdgcn_s_barrier();                                                \
  } while (0)

  for (int t = 0; t < nit; ++t) {
    const char* St = smem + (t & 1) * P8_BUF;
    const int P = 4 * t;
    // phase 0: quadrant (0, 0); reads A0, B0; issues half-tile P + 6 (B1 of K-step t + 1)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) xb0[h][j] = *(const bf16x8*)(St + (h ? fb1 : fb0) + j * 2048);
#pragma unroll
      for (int i = 0; i < 4; ++i) xa[h][i] = *(const bf16x8*)(St + (h ? fa1 : fa0) + i * 2048);
    }
    if (P + 6 < nh) P8_ISSUE(P + 6);
    P8_WAIT(P, P + 2);
    __builtin_amdgcn_s_barrier();
    P8_MMA(0, 0, xb0);
    // phase 1: quadrant (0, 1); reads B1; issues A1 of K-step t + 1
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        xb1[h][j] = *(const bf16x8*)(St + (h ? fb1 : fb0) + 32 * 128 + j * 2048);
    if (P + 7 < nh) P8_ISSUE(P + 7);
    P8_WAIT(P + 1, P + 3);
    __builtin_amdgcn_s_barrier();
    P8_MMA(0, 2, xb1);
    // phase 2: quadrant (1, 1); reads A1; issues A0 of K-step t + 2 (no wait: phase 3 reads
    // nothing)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        xa[h][i] = *(const bf16x8*)(St + (h ? fa1 : fa0) + 64 * 128 + i * 2048);
    if (P + 8 < nh) P8_ISSUE(P + 8);
    __builtin_amdgcn_s_barrier();
    P8_MMA(4, 2, xb1);
    // phase 3: quadrant (1, 0) from registers; issues B0 of K-step t + 2
    if (P + 9 < nh) P8_ISSUE(P + 9);
    if (t + 1 < nit) P8_WAIT(P + 3, P + 5);
    __builtin_amdgcn_s_barrier();
    P8_MMA(4, 0, xb0);
  }
  if (BAR2 && wr == 0) __builtin_amdgcn_s_barrier();  // pairs with row 1's last barrier
#undef P8_MMA
#undef P8_WAIT
#undef P8_ISSUE
#undef P8_OFFS
  // every DMA was waited for (the last K-step's phase 1 waits vmcnt(0))
  if constexpr (NOMMA) return;
  if constexpr (NODMA) {  // keep the MFMAs: the accumulators reach an (empty) use
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  float bs[4];
  const bool bias_st = a.bias != nullptr;
  if (bias_st) big_bias(a, n0, wc, lane, bs);
  float* T = (float*)smem;
  if constexpr (EPK == EPI_PLAIN) {
    // T rows [64 wr, 64 wr + 64) hold tile rows 128 wr + 64 pass + (0..63) of every wave's
    // half `pass`; a thread stores 4 consecutive columns of 16 rows (one 1-KB row per wave
    // instruction)
    lds_sync();
    const int cq = tid & 63, r0 = tid >> 6;
    const int col = n0 + cq * 4;
    const bool colok = col < a.N;
#define STAGE_P(H)                                                                        \
    _Pragma("unroll") for (int mt2 = 0; mt2 < 4; ++mt2)                                   \
    _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                      \
    _Pragma("unroll") for (int r = 0; r < 4; ++r)                                         \
        T[(wr * 64 + mt2 * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] = \
            bias_st ? acc[(H) * 4 + mt2][nt][r] + bs[nt] : acc[(H) * 4 + mt2][nt][r]
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (pass) {
        STAGE_P(1);
      } else {
        STAGE_P(0);
      }
#undef STAGE_P
      lds_sync();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int tr = r0 + 8 * i;  // T row
        const int m = m0 + (tr < 64 ? 0 : 64) + pass * 64 + tr;
        const f32x4 v = ld4(T + tr * EPB + cq * 4);
        if (colok && m < a.M) st4(a.Y + (long long)m * a.ldy + col, v);
      }
      lds_sync();
    }
    return;
  }
  EpiPre pre;
  if constexpr (EPK == -1) {
    // every other epilogue: the tile staged in two passes of both wave rows' halves (T rows
    // [64 wr, 64 wr + 64) = tile rows 128 wr + 64 pass + (0..63)), so at most half of the
    // accumulators stay live across an epilogue (staging one wave row's quarter per 64-row
    // chunk kept all 128 live in the other row's waves, and the instance spilled); each 64-row
    // block runs epilogue_tile with its own operand prefetch (epi_pre)
    lds_sync();
#define STAGE_P(H)                                                                        \
    _Pragma("unroll") for (int mt2 = 0; mt2 < 4; ++mt2)                                   \
    _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                      \
    _Pragma("unroll") for (int r = 0; r < 4; ++r)                                         \
        T[(wr * 64 + mt2 * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] = \
            bias_st ? acc[(H) * 4 + mt2][nt][r] + bs[nt] : acc[(H) * 4 + mt2][nt][r]
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (pass) {
        STAGE_P(1);
      } else {
        STAGE_P(0);
      }
      lds_sync();
#pragma unroll 1
      for (int blk = 0; blk < 2; ++blk) {
        const int mb = m0 + blk * 128 + pass * 64;
        epi_pre<BNB, NTHRB>(a, mb, n0, tid, 0, pre);
        epilogue_tile<CHR, BNB, NTHRB, EPB, true>(a, T + blk * 64 * EPB, mb, n0, tid, true, pre);
      }
      lds_sync();
    }
#undef STAGE_P
    return;
  }
  if (!GATE8) epi_pre<BNB, NTHRB>(a, m0, n0, tid, 0, pre);
  lds_sync();
#define STAGE_HALF(H)                                                                     \
  _Pragma("unroll") for (int mt2 = 0; mt2 < 4; ++mt2)                                     \
  _Pragma("unroll") for (int nt = 0; nt < 4; ++nt)                                        \
  _Pragma("unroll") for (int r = 0; r < 4; ++r)                                           \
      T[(mt2 * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] =        \
          bias_st ? acc[(H) * 4 + mt2][nt][r] + bs[nt] : acc[(H) * 4 + mt2][nt][r]
#pragma unroll 1
  for (int c = 0; c < BMB / CHR; ++c) {
    if (wr == (c >> 1)) {
      if (c & 1) {
        STAGE_HALF(1);
      } else {
        STAGE_HALF(0);
      }
    }
    lds_sync();
    if (GATE8) gate_tile8<NTHRB, CHR, BNB / 16, true>(a, T, EPB, m0 + c * CHR, n0, tid);
    else epilogue_tile<CHR, BNB, NTHRB, EPB, true>(a, T, m0 + c * CHR, n0, tid, c == BMB / CHR - 1, pre);
    lds_sync();
  }
#undef STAGE_HALF
}

// ------------------------------ 128 x 256, 8 waves, a 64-deep K-step in two phases
// For the N = 256 launches at 30 k frames (the DiffNet's dilated-conv input gradient, gate
// backward, residual and skip GEMMs): 256 x 256 tiles would be 120 workgroups, half the chip,
// and the 128 x 128 kernel keeps one K-step in flight.  Here the four-phase kernel's counted
// LDS-DMA pipeline on a 128 x 256 tile (240 workgroups): 8 waves in 2 x 4, each a 64 x 64
// sub-tile, a K-step in two phases of 16 MFMAs per wave (phase 0 reads the wave's A rows and
// its B columns 0-31, phase 1 its B columns 32-63 with A kept in registers).  A K-step's
// operands are six 8-KB pieces, one buffer_load ... lds per thread each:
//   part 0 / 1  A rows rA / rA + 64                          (read in phase 0)
//   part 2 / 3  B rows rB / rB + 128   (64 c + 0-31)         (read in phase 0)
//   part 4 / 5  B rows rB + 32 / + 160 (64 c + 32-63)        (read in phase 1)
// K-step t + 2 is issued in the two phases of K-step t (three pieces each) into buffer
// (t + 2) % 3 of three (3 x 48 KB): a region is rewritten >= 2 phases after its last read, and
// 8-9 pieces (64-72 KB per CU) stay in flight across every barrier.  Two barriers per phase
// with the wave rows staggered half a phase, as the four-phase kernel's default.  Per
// accumulator the K order is the other kernels' (k-chunks in order): the same bits.
// Epilogue: the tile staged through LDS; PLAIN lean (fp32 Y = acc + bias), or the non-pair
// epilogues of gemm_epilogue_lds (PLAIN with accumulate / activation / bf16 copy, ADDSCALE,
// RELU_MASK, GATE_BWD) with their column sums in the 128 x 128 kernel's row order.
constexpr int BMH = 128;
constexpr int P8H_AIMG = BMH * BK2 * 2;          // 16 KB
constexpr int P8H_BUF = P8H_AIMG + P8_IMG;       // 48 KB: A + B of one K-step
constexpr int P8H_LDS = 3 * P8H_BUF;             // 144 KB
constexpr int P8H_LDS_EPI = BMH * EPB * 4 + CS_GROUPS * 2 * BNB * 4;  // tile + column sums

__device__ __forceinline__ void xcd_tile_h(int& m0, int& n0) {
  const int nM = gridDim.x, nN = gridDim.y, total = nM * nN;
  const int orig = blockIdx.x + blockIdx.y * nM;
  const int xcd = orig & 7, q = total >> 3, r = total & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  m0 = (wg / nN) * BMH;
  n0 = (wg % nN) * BNB;
}

struct P8HOffs {
  unsigned oa[2];
  unsigned ob;
};

__device__ __forceinline__ P8HOffs p8h_offs(const SegU S, int j, int Npad, int n0, int rB,
                                            int ca8, int cb8, const int (&bt)[2],
                                            const int (&tt)[2], unsigned okm) {
  P8HOffs o;
  const int shj = S.shift0 + j * S.dil;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ts = tt[i] + shj;
    const int src = S.pad == PAD_ZERO ? ((unsigned)ts < (unsigned)S.Tin ? ts : -1)
                                      : pad_src(ts, S.Tin, S.pad);
    const bool ok = ((okm >> i) & 1) && src >= 0;
    o.oa[i] = ok ? (unsigned)((bt[i] * S.Tin + src) * S.ld + ca8) * 2u : P8_OOB;
  }
  o.ob = (unsigned)((j * Npad + n0 + rB) * S.Kp + cb8) * 2u;
  return o;
}

// The non-pair epilogues of a staged 128 x 256 tile T [128][EPB] (no bias in T): thread tid
// takes columns 4 (tid & 63) .. + 3 and rows (tid >> 6) + 8 k, k = 0..15, its next row's
// operands loaded before this row's stores.  Per column these are the rows and the order of
// the 128 x 128 kernel's column sums (row group g = 0..7 ascending, then the groups in order).
template <unsigned MASK>
__device__ __forceinline__ void p8h_epilogue(const GemmArgs& a, const float* T, float* X, int m0,
                                             int n0, int tid) {
  auto ep = [&](int e) { return ((MASK >> e) & 1u) && a.epi == e; };
  // rows whose operands are loaded together, one batch ahead (the all-epilogue instance: 2)
  constexpr int EBH = MASK == ~0u ? 2 : 8;
  const int cq = tid & 63, g = tid >> 6, col = n0 + cq * 4;
  const int ne = min(4, a.N - col);
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if (a.bias && ne > 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < ne) bv[e] = a.bias[col + e];
  }
  const bool want1 = (ep(EPI_PLAIN) && a.accum) || ep(EPI_ADDSCALE) || ep(EPI_RELU_MASK) ||
                     ep(EPI_GATE_BWD);
  const bool want2 = (ep(EPI_RELU_MASK) && a.accum) || ep(EPI_GATE_BWD);
  const bool wl = ne == 4 && (want1 || want2);
  // the bf16 copy's per-sequence add (PLAIN / ADDSCALE), loaded with the batch
  const bool wrr = ne == 4 && a.ybf && a.ybf_radd && (ep(EPI_PLAIN) || ep(EPI_ADDSCALE));
  f32x4 cs0 = {0.f, 0.f, 0.f, 0.f}, cs1 = {0.f, 0.f, 0.f, 0.f};
  f32x4 p1[EBH], p2[EBH], pr[EBH], q1[EBH], q2[EBH], qr[EBH];
  auto load_batch = [&](int kb, f32x4 (&x1)[EBH], f32x4 (&x2)[EBH], f32x4 (&xr)[EBH]) {
#pragma unroll
    for (int k = 0; k < EBH; ++k) {
      const int m = m0 + g + 8 * (kb + k);
      if (wl) gen_load(a, m, col, want2, x1[k], x2[k]);
      if (wrr && m < a.M) xr[k] = ld4(a.ybf_radd + (long long)(m / a.Tout) * a.ybf_radd_ld + col);
    }
  };
  load_batch(0, p1, p2, pr);
#pragma unroll 1
  for (int kb = 0; kb < BMH / 8; kb += EBH) {
    if (kb + EBH < BMH / 8) load_batch(kb + EBH, q1, q2, qr);
#pragma unroll
    for (int k = 0; k < EBH; ++k) {
      const int row = g + 8 * (kb + k);
      const int m = m0 + row;
      if (m >= a.M || ne <= 0) continue;
      f32x4 v = ld4(T + row * EPB + cq * 4);
      if (a.csum && a.epi != EPI_GATE_BWD) cs0 += v;
      if (a.bias) v += bv;
      float* y = a.Y + (long long)m * a.ldy + col;
      if (ne == 4) {
        if (ep(EPI_PLAIN)) {
          if (a.accum) v += p1[k];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (a.relu == 1) v[e] = fmaxf(v[e], 0.f);
            else if (a.relu == 2) v[e] = sigmoidf_(v[e]);
          }
          st4(y, v);
          shadow4r(a, m, col, v, pr[k]);
        } else if (ep(EPI_ADDSCALE)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = __builtin_fmaf(a.alpha, p1[k][e], v[e]);
            v[e] = a.relu == 1 ? fmaxf(v[e], 0.f) : v[e];
          }
          st4(y, v);
          shadow4r(a, m, col, v, pr[k]);
        } else if (ep(EPI_RELU_MASK)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = p1[k][e] > 0.f ? v[e] : 0.f;
          if (a.accum) v += p2[k];
          st4(y, v);
          shadow4(a, m, col, v);
        } else if (ep(EPI_GATE_BWD)) {
          f32x4 dg, df;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float t0, t1;
            gate_bwd_(v[e], p1[k][e], p2[k][e], t0, t1);
            dg[e] = t0;
            df[e] = t1;
          }
          if (a.csum) {
            cs0 += dg;
            cs1 += df;
          }
          if (a.Y) {
            st4(y, dg);
            st4(y + a.C, df);
          }
          shadow4(a, m, col, dg);
          shadow4(a, m, a.C + col, df);
        }
      } else {
        for (int e = 0; e < ne; ++e) {
          float w = v[e];
          float* ye = y + e;
          if (ep(EPI_PLAIN)) {
            if (a.accum) w += *ye;
            if (a.relu == 1) w = fmaxf(w, 0.f);
            else if (a.relu == 2) w = sigmoidf_(w);
            *ye = w;
          } else if (ep(EPI_ADDSCALE)) {
            w = __builtin_fmaf(a.alpha, a.aux1[(long long)m * a.ld1 + col + e], w);
            *ye = a.relu == 1 ? fmaxf(w, 0.f) : w;
          } else if (ep(EPI_RELU_MASK)) {
            w = a.aux1[(long long)m * a.ld1 + col + e] > 0.f ? w : 0.f;
            *ye = a.accum ? *ye + w : w;
          } else if (ep(EPI_GATE_BWD)) {
            const float gg = ld_aux1(a, (long long)m * a.ld1 + col + e);
            const float ff = ld_aux1(a, (long long)m * a.ld1 + a.C + col + e);
            gate_bwd_(w, gg, ff, ye[0], ye[a.C]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < EBH; ++k) {
      p1[k] = q1[k];
      p2[k] = q2[k];
      pr[k] = qr[k];
    }
  }
  if (a.csum) {  // uniform: every thread reaches the barrier
    *(f32x4*)(X + g * 2 * BNB + cq * 4) = cs0;
    *(f32x4*)(X + g * 2 * BNB + BNB + cq * 4) = cs1;
    lds_sync();
    const int j = tid;  // NTHRB == 2 * BNB: the accumulator / d(gate) columns, then d(filter)
    if (j < BNB || ep(EPI_GATE_BWD)) {
      const int c = n0 + (j & (BNB - 1));
      if (c < a.N) {
        float t = X[j];
#pragma unroll
        for (int q = 1; q < CS_GROUPS; ++q) t += X[q * 2 * BNB + j];
        a.csum[(long long)(m0 / BM) * a.csum_ld + (j < BNB ? c : a.C + c)] = t;
      }
    }
  }
}

// EPK: EPI_PLAIN -- the lean plain epilogue (as the four-phase kernel's); -1 -- p8h_epilogue
template <int EPK>
__global__ __launch_bounds__(NTHRB) void conv_gemm_b16_p8h_kernel(const GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  xcd_tile_h(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);
  const int np = 6 * nit;  // pieces
  const int rA = wid * 8 + (lane >> 3), rB = (wid & 3) * 8 + (wid >> 2) * 64 + (lane >> 3);
  const int ca8 = swz(rA, lane & 7) * 8, cb8 = swz(rB, lane & 7) * 8;
  int bt[2], tt[2];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + rA + i * 64;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  const int la = wid * 8 * 128, lb = ((wid & 3) * 8 + (wid >> 2) * 64) * 128;
  // staging cursor: the K-step whose pieces are issued next (segment, tap, k-step, buffer)
  int qs = 0, qj = 0, qkc = 0, qb = 0, nis = 0;
#define P8H_OFFS(S) p8h_offs(S, qj, Npad, n0, rB, ca8, cb8, bt, tt, okm)
  P8HOffs O = P8H_OFFS(S0);
  __amdgpu_buffer_rsrc_t rxa = p8_rsrc(S0.x), rwb = p8_rsrc(S0.w);
  int qK = S0.K, qKp = S0.Kp;
#define P8H_ISSUE(part)                                                                    \
  do {                                                                                     \
    char* L_ = smem + qb * P8H_BUF;                                                        \
    const int kb_ = qkc * BK2;                                                             \
    const unsigned kb2_ = (unsigned)kb_ * 2u;                                              \
    if ((part) < 2) {                                                                      \
      const bool in_ = kb_ + ca8 < qK;                                                     \
      p8_dma(rxa, in_ ? O.oa[(part) & 1] + kb2_ : P8_OOB, L_ + la + ((part) & 1) * 64 * 128);\
    } else {                                                                               \
      constexpr int d_ = (part) == 2 ? 0 : ((part) == 3 ? 128 : ((part) == 4 ? 32 : 160)); \
      const bool in_ = kb_ + cb8 < qKp;                                                    \
      p8_dma(rwb, in_ ? O.ob + (unsigned)(d_ * qKp) * 2u + kb2_ : P8_OOB,                   \
             L_ + P8H_AIMG + lb + d_ * 128);                                               \
    }                                                                                      \
    ++nis;                                                                                 \
    if ((part) == 5) { /* K-step done: advance the cursor */                               \
      qb = qb == 2 ? 0 : qb + 1;                                                           \
      const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                        \
      const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
      if (++qkc == nks_) {                                                                 \
        qkc = 0;                                                                           \
        const int qs0_ = qs;                                                               \
        if (++qj == taps_) {                                                               \
          qj = 0;                                                                          \
          ++qs;                                                                            \
        }                                                                                  \
        if (qs < nseg) {                                                                   \
          if (qs != qs0_) {                                                                \
            rxa = p8_rsrc(qs == 1 ? S1.x : S2.x);                                          \
            rwb = p8_rsrc(qs == 1 ? S1.w : S2.w);                                          \
            qK = qs == 1 ? S1.K : S2.K;                                                    \
            qKp = qs == 1 ? S1.Kp : S2.Kp;                                                 \
          }                                                                                \
          O = qs == 0 ? P8H_OFFS(S0) : (qs == 1 ? P8H_OFFS(S1) : P8H_OFFS(S2));            \
        }                                                                                  \
      }                                                                                    \
    }                                                                                      \
  } while (0)
#define P8H_KSTEP_LO() \
  do {                 \
    P8H_ISSUE(0);      \
    P8H_ISSUE(1);      \
    P8H_ISSUE(2);      \
  } while (0)
#define P8H_KSTEP_HI() \
  do {                 \
    P8H_ISSUE(3);      \
    P8H_ISSUE(4);      \
    P8H_ISSUE(5);      \
  } while (0)
  // the counted wait: at most nis - 1 - need pieces of this thread still in flight
#define P8H_WAIT(need)                            \
  do {                                            \
    const int al_ = nis - 1 - (need);             \
    if (al_ >= 9) p8_wait<9>();                   \
    else if (al_ == 8) p8_wait<8>();              \
    else if (al_ == 7) p8_wait<7>();              \
    else if (al_ == 6) p8_wait<6>();              \
    else if (al_ == 5) p8_wait<5>();              \
    else if (al_ == 4) p8_wait<4>();              \
    else if (al_ == 3) p8_wait<3>();              \
    else if (al_ == 2) p8_wait<2>();              \
    else if (al_ == 1) p8_wait<1>();              \
    else p8_wait<0>();                            \
  } while (0)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-steps 0 and 1, then wait for phase 0's pieces (0..3)
  for (int t = 0; t < min(2, nit); ++t) {
    P8H_KSTEP_LO();
    P8H_KSTEP_HI();
  }
  P8H_WAIT(3);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // rows staggered half a phase (see the p8 kernel)

  const int arow = lane & 15, kq = lane >> 4;
  const int fa0 = (wr * 64 + arow) * 128 + swz(arow, kq) * 16;
  const int fa1 = (wr * 64 + arow) * 128 + swz(arow, kq + 4) * 16;
  const int fb0 = P8H_AIMG + (wc * 64 + arow) * 128 + swz(arow, kq) * 16;
  const int fb1 = P8H_AIMG + (wc * 64 + arow) * 128 + swz(arow, kq + 4) * 16;
  bf16x8 xa[2][4], xb0[2][2], xb1[2][2];
#define P8H_MMA(J0, B)                                                                     \
  do {                                                                                     \
    __builtin_amdgcn_s_setprio(1);                                                         \
    _Pragma("unroll") for (int h = 0; h < 2; ++h)                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                          \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                          \
      acc[i][(J0) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[h][i], B[h][j],         \
                                                                acc[i][(J0) + j], 0, 0, 0); \
    __builtin_amdgcn_s_setprio(0);                                                         \
    __builtin_amdgcn_s_barrier();                                                          \
  } while (0)

  int rb = 0;  // buffer of K-step t
  for (int t = 0; t < nit; ++t) {
    const char* St = smem + rb * P8H_BUF;
    // phase 0: A rows and B columns 0-31 of the wave; issues K-step t + 2's pieces 0-2
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) xb0[h][j] = *(const bf16x8*)(St + (h ? fb1 : fb0) + j * 2048);
#pragma unroll
      for (int i = 0; i < 4; ++i) xa[h][i] = *(const bf16x8*)(St + (h ? fa1 : fa0) + i * 2048);
    }
    if (t + 2 < nit) P8H_KSTEP_LO();
    P8H_WAIT(6 * t + 5);
    __builtin_amdgcn_s_barrier();
    P8H_MMA(0, xb0);
    // phase 1: B columns 32-63; issues pieces 3-5
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        xb1[h][j] = *(const bf16x8*)(St + (h ? fb1 : fb0) + 32 * 128 + j * 2048);
    if (t + 2 < nit) P8H_KSTEP_HI();
    if (t + 1 < nit) P8H_WAIT(6 * t + 9);
    __builtin_amdgcn_s_barrier();
    P8H_MMA(2, xb1);
    rb = rb == 2 ? 0 : rb + 1;
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // pairs with row 1's last barrier
#undef P8H_MMA
#undef P8H_WAIT
#undef P8H_KSTEP_LO
#undef P8H_KSTEP_HI
#undef P8H_ISSUE
#undef P8H_OFFS
  // every DMA was waited for (the last K-step's phase 0 waits vmcnt(0))
  float* T = (float*)smem;
  if constexpr (EPK == EPI_PLAIN) {
    float bs[4];
    const bool bias_st = a.bias != nullptr;
    if (bias_st) big_bias(a, n0, wc, lane, bs);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(wr * 64 + mt * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] =
              bias_st ? acc[mt][nt][r] + bs[nt] : acc[mt][nt][r];
    lds_sync();
    const int cq = tid & 63, r0 = tid >> 6;
    const int col = n0 + cq * 4;
    if (col < a.N) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = m0 + r0 + 8 * i;
        const f32x4 v = ld4(T + (r0 + 8 * i) * EPB + cq * 4);
        if (m < a.M) st4(a.Y + (long long)m * a.ldy + col, v);
      }
    }
    return;
  } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T[(wr * 64 + mt * 16 + (lane >> 4) * 4 + r) * EPB + wc * 64 + nt * 16 + (lane & 15)] =
              acc[mt][nt][r];
    lds_sync();
    // EPK = 16 + e: epilogue e through p8h_epilogue (PLAIN with accumulate / activation /
    // copies); EPK = e (not PLAIN): that epilogue alone; -1: every epilogue
    constexpr unsigned MASK = EPK < 0 ? ~0u : (1u << (EPK >= 16 ? EPK - 16 : EPK));
    p8h_epilogue<MASK>(a, T, T + BMH * EPB, m0, n0, tid);
  }
}

// ------------------------------------------------- 64 x 64 bf16-operand GEMM (small M)
// The reverse diffusion's DiffNet GEMMs have M = 2 000 frame rows: 16 x 4 tiles of 128 x 128
// keep 64 CUs busy, each walking a 16-step K loop at one L2 round trip per step.  64 x 64
// tiles give 32 x 8 = 256 workgroups (the whole chip) whose operands sit in the XCD's L2
// (activations 1-2 MB bf16, weights 1 MB); each workgroup keeps SMS - 1 K-steps of both
// images in flight (an L2-resident LDS-DMA stream runs at ~70 GB/s per CU with 64-72 KiB in
// flight, MI355X_MICROARCH.md "Indexed rows"), so a 1 024-deep tile streams its 256 KB in
// ~4 us.  4 waves in 2 x 2, each a 32 x 32 sub-tile (2 x 2 v_mfma_f32_16x16x32_bf16) over the
// full K loop: every output element accumulates its K-steps in the same order as the 128 x
// 128 kernels, so the results are bit-identical to them.  Same LDS image / swizzle / staging
// pointers; the epilogue stages the fp32 tile through LDS (epilogue_tile).
constexpr int BMS = 64, BNS = 64, EPS = BNS + 4;

__device__ __forceinline__ void xcd_tile_small(int& m0, int& n0) {
  const int nM = gridDim.x, nN = gridDim.y, total = nM * nN;
  const int orig = blockIdx.x + blockIdx.y * nM;
  const int xcd = orig & 7, q = total >> 3, r = total & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  m0 = (wg / nN) * BMS;
  n0 = (wg % nN) * BNS;
}

// staging pointers of this lane's 2 A rows (rl, rl + 8) and 2 B rows of one (segment, tap)
struct TapPtrsS {
  const char* pa[2];
  const char* pb[2];
  unsigned va;
  int K, Kp;
};

__device__ __forceinline__ TapPtrsS tap_ptrs_s(const SegU S, int j, int Npad, int n0, int rl,
                                               int cq8a, int cq8b, const int b0, const int b1,
                                               const int t0, const int t1, unsigned okm) {
  TapPtrsS P;
  const int bt[2] = {b0, b1}, tt[2] = {t0, t1};
  const int shj = S.shift0 + j * S.dil;
  P.va = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c8 = i ? cq8b : cq8a;
    const int ts = tt[i] + shj;
    const int src = S.pad == PAD_ZERO ? ((unsigned)ts < (unsigned)S.Tin ? ts : -1)
                                      : pad_src(ts, S.Tin, S.pad);
    const bool ok = ((okm >> i) & 1) && src >= 0;
    P.va |= ok ? (1u << i) : 0u;
    P.pa[i] = (const char*)(S.x + (unsigned)((bt[i] * S.Tin + (ok ? src : 0)) * S.ld + c8));
    P.pb[i] = S.w + ((unsigned)((j * Npad + n0 + rl + 8 * i) * S.Kp + c8)) * 2;
  }
  P.K = S.K;
  P.Kp = S.Kp;
  return P;
}

template <int SMS>
__global__ __launch_bounds__(NTHR) void conv_gemm_b16_small_kernel(const GemmArgs a) {
  static_assert(SMS >= 2 && SMS <= 5, "stages (waits are counted up to 3 stages ahead)");
  constexpr int IMG = BMS * BK2 * 2;  // 8 KB: one operand image of one stage
  constexpr int STAGE = 2 * IMG;
  constexpr int GL = 4;               // glds per thread per stage (2 A rows + 2 B rows)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  xcd_tile_small(m0, n0);
  const int M = a.M, Tout = a.Tout, Npad = a.Npad;
  const int nseg = a.nseg;
  const SegU S0 = seg_u(a.seg[0], a.W);
  const SegU S1 = nseg > 1 ? seg_u(a.seg[1], a.W) : S0;
  const SegU S2 = nseg > 2 ? seg_u(a.seg[2], a.W) : S0;
  const int nit = S0.nk * S0.taps + (nseg > 1 ? S1.nk * S1.taps : 0) +
                  (nseg > 2 ? S2.nk * S2.taps : 0);
  // wave wid fills rows wid*16 + lane/8 + 8i (i = 0, 1) of both images
  const int rl = wid * 16 + (lane >> 3), slot = lane & 7;
  const int cq = swz(rl, slot), cq8a = cq * 8, cq8b = (cq ^ 4) * 8;
  int bt[2], tt[2];
  unsigned okm = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + rl + 8 * i;
    const bool ok = m < M;
    bt[i] = ok ? m / Tout : 0;
    tt[i] = ok ? m - bt[i] * Tout : 0;
    okm |= ok ? (1u << i) : 0u;
  }
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  int qs = 0, qj = 0, qkc = 0;
#define TAP_PTRS_S(S) tap_ptrs_s(S, qj, Npad, n0, rl, cq8a, cq8b, bt[0], bt[1], tt[0], tt[1], okm)
  TapPtrsS P = TAP_PTRS_S(S0);
#define ISSUE_S(it)                                                                      \
  do {                                                                                   \
    char* As_ = smem + ((it) % SMS) * STAGE + wid * 16 * 128;                            \
    const int kb_ = qkc * BK2;                                                           \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                      \
      const bool oa = ((P.va >> i) & 1) && kb_ + (i ? cq8b : cq8a) < P.K;                \
      glds16(oa ? (const void*)(P.pa[i] + kb_ * 2) : (const void*)zp, As_ + i * 1024);   \
    }                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                      \
      const bool ob = kb_ + (i ? cq8b : cq8a) < P.Kp;                                    \
      glds16(ob ? (const void*)(P.pb[i] + kb_ * 2) : (const void*)zp,                    \
             As_ + IMG + i * 1024);                                                      \
    }                                                                                    \
    const int nks_ = qs == 0 ? S0.nk : (qs == 1 ? S1.nk : S2.nk);                        \
    const int taps_ = qs == 0 ? S0.taps : (qs == 1 ? S1.taps : S2.taps);                 \
    if (++qkc == nks_) {                                                                 \
      qkc = 0;                                                                           \
      if (++qj == taps_) {                                                               \
        qj = 0;                                                                          \
        ++qs;                                                                            \
      }                                                                                  \
      if (qs < nseg) P = qs == 0 ? TAP_PTRS_S(S0) : (qs == 1 ? TAP_PTRS_S(S1) : TAP_PTRS_S(S2)); \
    }                                                                                    \
  } while (0)

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < SMS - 1; ++p)
    if (p < nit) ISSUE_S(p);
  // the epilogue's global operands (bias, residual / skip rows, per-sequence adds) are
  // loaded now, behind the K loop, instead of as a dependent round trip after it: at
  // M = 2 000 a launch is a few K-steps long and such round trips set its duration
  float bs[2] = {0.f, 0.f};
  const bool bias_st = a.bias != nullptr;
  if (bias_st) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 32 + j * 16 + (lane & 15);
      bs[j] = n < a.N ? a.bias[n] : 0.f;
    }
  }
  EpiPreT<2> pre;
  epi_pre<BNS, NTHR, 2>(a, m0, n0, tid, 0, pre);
  const int arow = lane & 15, kq = lane >> 4;
  const int ra = wr * 32 + arow, rbr = wc * 32 + arow;
  const int oa0 = ra * 128 + swz(ra, kq) * 16, oa1 = ra * 128 + swz(ra, kq + 4) * 16;
  const int ob0 = IMG + rbr * 128 + swz(rbr, kq) * 16;
  const int ob1 = IMG + rbr * 128 + swz(rbr, kq + 4) * 16;
  for (int it = 0; it < nit; ++it) {
    const int ahead = min(SMS - 2, nit - 1 - it);  // stages issued after tile `it`
    if (ahead >= 3) wait_vm_n<3 * GL>();
    else if (ahead == 2) wait_vm_n<2 * GL>();
    else if (ahead == 1) wait_vm_n<GL>();
    else wait_vm_n<0>();
    __builtin_amdgcn_s_barrier();  // tile `it` visible; every wave is done with tile it-1
    if (it + SMS - 1 < nit) ISSUE_S(it + SMS - 1);
    const char* St = smem + (it % SMS) * STAGE;
    bf16x8 fa[2][2], fb[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[h][i] = *(const bf16x8*)(St + (h ? oa1 : oa0) + i * 2048);
        fb[h][i] = *(const bf16x8*)(St + (h ? ob1 : ob0) + i * 2048);
      }
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // DS reads
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // MFMAs
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[h][i], fb[h][j], acc[i][j], 0, 0, 0);
  }
#undef ISSUE_S
#undef TAP_PTRS_S
  // epilogue: acc + bias staged through LDS as an fp32 tile
  float* T = (float*)smem;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wr * 32 + i * 16 + (lane >> 4) * 4 + r) * EPS + wc * 32 + j * 16 + (lane & 15)] =
            bias_st ? acc[i][j][r] + bs[j] : acc[i][j][r];
  __syncthreads();
  epilogue_tile<BMS, BNS, NTHR, EPS, true, 2>(a, T, m0, n0, tid, true, pre);
}

// y[m][k] = bf16(x[m][k] + radd[m / T][k]) for the bf16-activation GEMM (8 elements per thread).
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ radd,
                                                        int radd_ld, int T, long long M, int K,
                                                        __bf16* __restrict__ y, int ldy) {
  const int K8 = K / 8;
  const long long n = M * K8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / K8;
    const int k = (int)(i - m * K8) * 8;
    f32x4 v0 = *(const f32x4*)(x + m * ldx + k), v1 = *(const f32x4*)(x + m * ldx + k + 4);
    if (radd) {
      const float* r = radd + (m / T) * radd_ld + k;
      v0 += *(const f32x4*)r;
      v1 += *(const f32x4*)(r + 4);
    }
    *(bf16x8*)(y + m * ldy + k) = bf16x8{(__bf16)v0[0], (__bf16)v0[1], (__bf16)v0[2],
                                         (__bf16)v0[3], (__bf16)v1[0], (__bf16)v1[1],
                                         (__bf16)v1[2], (__bf16)v1[3]};
  }
}

// K % 8 != 0 (the uSFGAN auxiliary features, K = 65): y[m][k] = bf16(x[m][k]) for k < K and
// 0 up to the next multiple of 8 -- the zero K padding the 16-B operand chunks read.
__global__ __launch_bounds__(256) void cast_bf16_pad_kernel(const float* __restrict__ x, int ldx,
                                                            long long M, int K, int K8,
                                                            __bf16* __restrict__ y, int ldy) {
  const long long n = M * K8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long m = i / K8;
    const int k = (int)(i - m * K8) * 8;
    // loads at clamped (valid) columns, then the select: a predicated load per element
    // compiles to a branch and a wait each (eight serial round trips)
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = x[m * ldx + min(k + e, K - 1)];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (__bf16)(k + e < K ? v[e] : 0.f);
    *(bf16x8*)(y + m * ldy + k) = o;
  }
}

// ------------------------------------------------------------ weight grads
struct WgradArgs {
  const float* dy;
  const float* x;
  const float* radd;
  float* part;  // [splits][taps][N][K]
  float* dst;   // splits == 1: written directly, dst[n*sn + k*sk + j*sj]
  long long sn, sk, sj;
  float scale;
  int accum;
  int ldy, ldx, K, taps, dil, shift0, pad, Tin, radd_ld;
  int Tout, M, N, splits, rows_per_split, vecy, vecx;
};

// bf16 staging image of one operand: [BK frames][128 channels], 256-B rows whose 16-B
// chunks are XOR-swizzled so the transposed MFMA-operand reads (ds_read_b64_tr_b16)
// and the row writes are bank-conflict free (cdna_hip_programming.md T10, image (b)).
__device__ __forceinline__ int wg_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Operand fragment for rows [c0, c0+16) of the image's channel axis: lane l gets
// channel c0 + (l&15), frames 8(l>>4) .. +7 (the 16x16x32 A/B lane map).
__device__ __forceinline__ bf16x8 wg_frag(const char* img, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (c0 >> 3) + (p >> 1);
  const int o0 = wg_off(8 * g + q, ch) + 8 * (p & 1);
  const int o1 = wg_off(8 * g + 4 + q, ch) + 8 * (p & 1);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + o0));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + o1));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// XCD-aware workgroup -> (tile, tap, row split) map of the weight-gradient kernels.  Every
// (N tile, K tile, tap) workgroup of one row split reads that split's dy and x rows; the
// dispatcher deals consecutive workgroups round-robin over the 8 XCDs (8 L2s), so the raw
// blockIdx order sent each split's workgroups to different XCDs and every one of them fetched
// the shared rows through the fabric (rocprofv3 FETCH_SIZE: 15 GB per training step across
// the wgrad kernels, profiles/r3_step_pmc.json).  When the split count is a multiple of 8,
// split s runs all its workgroups on XCD s % 8: hardware id b -> xcd = b % 8, then the
// workgroup index w inside the split and s = 8 (b / 8 / W) + xcd.  Bijective; the partial of
// split s covers the same rows as before, so the results are bitwise unchanged.  (Grouping by
// (split, tap) instead measured 17.50 vs 17.40 ms/step; the raw order 17.72.)
// Any split count: XCD x receives the hardware ids b = x (mod 8), count_x = q + (x < r) of
// them for total = 8 q + r workgroups; it runs the contiguous range [x q + min(x, r), + count_x)
// of the split-major (split, tap, K tile, N tile) order, so a split's workgroups share one XCD
// (a split straddles two XCDs at most at a range boundary).  The first version required
// splits % 8 == 0 and left the DiffNet dilated conv's 21 splits in raw order (2.8x its operand
// bytes fetched, profiles/r3_step_pmc.json).
__device__ __forceinline__ void wgrad_tile(const WgradArgs& a, int& n0, int& k0, int& j, int& s) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int total = gx * gy * gridDim.z;
  const int q = total >> 3, r = total & 7, x = b & 7;
  const int idx = x * q + min(x, r) + (b >> 3);
  const int W = gx * gy * a.taps;  // workgroups per split
  s = idx / W;
  const int w = idx - s * W;
  j = w / (gx * gy);
  const int t = w - j * gx * gy;
  k0 = (t / gx) * BN;
  n0 = (t % gx) * BM;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(NTHR) void wgrad_kernel(const WgradArgs a) {
  constexpr int LK = Lds<T>::K;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int n0, k0, j, s;
  wgrad_tile(a, n0, k0, j, s);
  const int mbeg = s * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int nch = mbeg < mend ? (mend - mbeg + BK - 1) / BK : 0;

  // bf16: lanes walk channels (coalesced rows), images kept [frame][channel].
  // fp32 (parity mode): lanes walk frames, images transposed [channel][frame].
  // Loads are unconditional (g_zero for rows/quads out of range, and for radd when
  // absent); radd is added in the store phase.  Each thread tracks the (b, t) of
  // its 4 frame rows incrementally (no per-chunk division).
  int fb[4], ft[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + NTHR * i;
    const int f = sizeof(T) == 2 ? (q >> 5) : (q & 31);
    const int m = mbeg + f;
    fb[i] = m / a.Tout;
    ft[i] = m - fb[i] * a.Tout;
  }
  f32x4 ra[4], rx[4], rr[4];
  auto load = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + NTHR * i;
      const int f = sizeof(T) == 2 ? (q >> 5) : (q & 31);
      const int c4 = sizeof(T) == 2 ? (q & 31) : (q >> 5);
      const int m = mbeg + ch * BK + f;
      const bool mv = m < mend;
      const int b = fb[i], t = ft[i];
      const int n = n0 + c4 * 4, k = k0 + c4 * 4;
      const float* dyrow = a.dy + (long long)m * a.ldy;
      const int src = pad_src(t + a.shift0 + j * a.dil, a.Tin, a.pad);
      const bool xrow_ok = mv && src >= 0;
      const float* xrow = a.x + (long long)(b * a.Tin + src) * a.ldx;
      const float* rrow = a.radd + (long long)b * a.radd_ld;
      const bool has_r = a.radd != nullptr;
      if constexpr (VEC) {
        ra[i] = *(const f32x4*)((mv && n < a.N) ? dyrow + n : g_zero);
        const bool kq = xrow_ok && k < a.K;
        rx[i] = *(const f32x4*)(kq ? xrow + k : g_zero);
        rr[i] = *(const f32x4*)((kq && has_r) ? rrow + k : g_zero);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ra[i][e] = *((mv && n + e < a.N) ? dyrow + n + e : g_zero);
          const bool kq = xrow_ok && k + e < a.K;
          rx[i][e] = *(kq ? xrow + k + e : g_zero);
          rr[i][e] = *((kq && has_r) ? rrow + k + e : g_zero);
        }
      }
      // advance this row slot to the next chunk's frame
      int nt = t + BK, nb = b;
      while (nt >= a.Tout) {
        nt -= a.Tout;
        ++nb;
      }
      fb[i] = nb;
      ft[i] = nt;
    }
  };
  constexpr int IMG = sizeof(T) == 2 ? BK * 256 : BM * LK * (int)sizeof(T);  // bytes / image
  auto store = [&](int buf) __attribute__((always_inline)) {
    char* A = smem + buf * 2 * IMG;
    char* B = A + IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + NTHR * i;
      rx[i] += rr[i];
      if constexpr (sizeof(T) == 2) {
        const int f = q >> 5, c4 = q & 31;
        const int o = wg_off(f, c4 >> 1) + 8 * (c4 & 1);
        *(bf16x4*)(A + o) = bf16x4{(__bf16)ra[i][0], (__bf16)ra[i][1], (__bf16)ra[i][2],
                                   (__bf16)ra[i][3]};
        *(bf16x4*)(B + o) = bf16x4{(__bf16)rx[i][0], (__bf16)rx[i][1], (__bf16)rx[i][2],
                                   (__bf16)rx[i][3]};
      } else {
        const int f = q & 31, c4 = q >> 5;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ((T*)A)[(c4 * 4 + e) * LK + f] = (T)ra[i][e];
          ((T*)B)[(c4 * 4 + e) * LK + f] = (T)rx[i][e];
        }
      }
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* A = smem + buf * 2 * IMG;
    const char* B = A + IMG;
    if constexpr (sizeof(T) == 2) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i] = wg_frag(A, wr * 64 + i * 16, lane);
        fb[i] = wg_frag(B, wc * 64 + i * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[jj], acc[i][jj], 0, 0, 0);
    } else {
      mma_tile<T>((const T*)A, (const T*)B, wr, wc, lane, acc);
    }
  };
  if (nch > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load(ch + 1);
    compute(buf);
    if (ch + 1 < nch) store(buf ^ 1);
    __syncthreads();
  }
  if (a.splits == 1) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
      if (k >= a.K) continue;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
          if (n < a.N) {
            float* d = a.dst + n * a.sn + k * a.sk + j * a.sj;
            const float v = acc[mt][nt][r] * a.scale;
            *d = a.accum ? *d + v : v;
          }
        }
    }
    return;
  }
  float* out = a.part + ((long long)(s * a.taps + j) * a.N) * a.K;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
    if (k >= a.K) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
        if (n < a.N) out[(long long)n * a.K + k] = acc[mt][nt][r];
      }
  }
}

// ------------------------------------ weight grads, fp32 operands, deep register prefetch
// wgrad_kernel<bf16, VEC> with WR chunks of fp32 rows in flight per thread instead of one.
// A 32-frame chunk is 16 MFMAs per wave: with one chunk loading behind one computing, every
// chunk's HBM/L2 latency was exposed (N = 256, K = 64: 31.6 us for 39 MB, ~1.2 TB/s).  Here
// chunk c lives in register slot c % WR from its load until it is rounded into the LDS image,
// so WR - 1 chunks stay in flight while one is multiplied.  Same staging rounding, the same
// LDS images and the same MFMA order as wgrad_kernel<bf16>: identical bits.
constexpr int WR = 3;

template <bool HAS_R>
__global__ __launch_bounds__(NTHR, 2) void wgrad_f32r_kernel(const WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int IMG = BK * 256;  // bytes per bf16 operand image (32 frames x 128 channels)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int n0, k0, j, s;
  wgrad_tile(a, n0, k0, j, s);
  const int mbeg = s * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int nch = mbeg < mend ? (mend - mbeg + BK - 1) / BK : 0;
  int fb[4], ft[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mbeg + ((tid + NTHR * i) >> 5);
    fb[i] = m / a.Tout;
    ft[i] = m - fb[i] * a.Tout;
  }
  f32x4 ra[WR][4], rx[WR][4], rr[WR][HAS_R ? 4 : 1];
  // chunk ch's rows into ring slot S (S is a compile-time constant at every call site)
  auto load = [&](int ch, f32x4 (&A)[4], f32x4 (&X)[4], f32x4 (&RR)[HAS_R ? 4 : 1])
      __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + NTHR * i, f = q >> 5, c4 = q & 31;
      const int m = mbeg + ch * BK + f;
      const bool mv = m < mend;
      const int b = fb[i], t = ft[i];
      const int n = n0 + c4 * 4, k = k0 + c4 * 4;
      const int src = pad_src(t + a.shift0 + j * a.dil, a.Tin, a.pad);
      const bool kq = mv && src >= 0 && k < a.K;
      A[i] = *(const f32x4*)((mv && n < a.N) ? a.dy + (long long)m * a.ldy + n : g_zero);
      X[i] = *(const f32x4*)(kq ? a.x + (long long)(b * a.Tin + src) * a.ldx + k : g_zero);
      if constexpr (HAS_R) RR[i] = *(const f32x4*)(kq ? a.radd + (long long)b * a.radd_ld + k
                                                      : g_zero);
      int nt = t + BK, nb = b;
      while (nt >= a.Tout) {
        nt -= a.Tout;
        ++nb;
      }
      fb[i] = nb;
      ft[i] = nt;
    }
  };
  auto store = [&](int buf, const f32x4 (&A)[4], const f32x4 (&X)[4],
                   const f32x4 (&RR)[HAS_R ? 4 : 1]) __attribute__((always_inline)) {
    char* As = smem + buf * 2 * IMG;
    char* Bs = As + IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + NTHR * i, f = q >> 5, c4 = q & 31;
      f32x4 xv = X[i];
      if constexpr (HAS_R) xv += RR[i];
      const int o = wg_off(f, c4 >> 1) + 8 * (c4 & 1);
      *(bf16x4*)(As + o) = bf16x4{(__bf16)A[i][0], (__bf16)A[i][1], (__bf16)A[i][2],
                                  (__bf16)A[i][3]};
      *(bf16x4*)(Bs + o) = bf16x4{(__bf16)xv[0], (__bf16)xv[1], (__bf16)xv[2], (__bf16)xv[3]};
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* As = smem + buf * 2 * IMG;
    const char* Bs = As + IMG;
    bf16x8 fa[4], fbv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i] = wg_frag(As, wr * 64 + i * 16, lane);
      fbv[i] = wg_frag(Bs, wc * 64 + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fbv[jj], acc[i][jj], 0, 0, 0);
  };
  // Loads and stores are unconditional (chunks past the split read zeros through g_zero):
  // a conditional load makes the waitcnt pass assume it may be missing and drain the ring
  // (vmcnt(0) before every store) instead of waiting for one chunk (vmcnt(16)).
#pragma unroll
  for (int p = 0; p < WR; ++p) load(p, ra[p], rx[p], rr[p]);
  store(0, ra[0], rx[0], rr[0]);
  load(WR, ra[0], rx[0], rr[0]);
  __syncthreads();
  for (int c0 = 0; c0 < nch; c0 += WR) {
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      const int ch = c0 + r;
      if (ch >= nch) break;
      const int ns = (r + 1) % WR;  // ring slot of chunk ch + 1 (constant after unrolling)
      // buffer (ch + 1) & 1 was last read by chunk ch - 1, before the previous barrier
      store((ch + 1) & 1, ra[ns], rx[ns], rr[ns]);
      load(ch + 1 + WR, ra[ns], rx[ns], rr[ns]);
      compute(ch & 1);
      __syncthreads();
    }
  }
  if (a.splits == 1) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
      if (k >= a.K) continue;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
          if (n < a.N) {
            float* d = a.dst + n * a.sn + k * a.sk + j * a.sj;
            const float v = acc[mt][nt][r] * a.scale;
            *d = a.accum ? *d + v : v;
          }
        }
    }
    return;
  }
  float* out = a.part + ((long long)(s * a.taps + j) * a.N) * a.K;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
    if (k >= a.K) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
        if (n < a.N) out[(long long)n * a.K + k] = acc[mt][nt][r];
      }
  }
}

// ------------------------------------------------- weight grads, bf16 operands
// wgrad_kernel<bf16> with dy and x already rounded to bf16 in HBM (the staging rounding of
// wgrad_kernel, so the result is bit-identical): both [32 frames][128 channels] images
// are filled by global_load_lds_dwordx4 into a WNS-slot ring (64 KB of LDS; WNS - 1 chunks,
// 48 KB, in flight per workgroup, 96 KB per CU at two workgroups: a 32-frame chunk is only 16 MFMAs
// per wave, so one chunk in flight left every chunk's L2 latency exposed), with a counted
// vmcnt and raw barriers.  The images keep wg_off's XOR swizzle (conflict-free ds_read_b64_tr_b16
// operand reads); the DMA writes lane-linearly, so each lane fetches the chunk that the
// swizzle maps to its slot.  a.dy / a.x point at bf16 rows here (ldy / ldx in elements).
__device__ __forceinline__ int wg_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// wg_frag's two transposed reads issued by inline asm.  The builtin's LDS read makes the
// compiler drain every outstanding global_load_lds first (s_waitcnt vmcnt(0) in front of
// it: it cannot tell the read from the ring slots being filled), which serialised each
// chunk's DMA with the MFMAs.  The caller waits with a counted lgkmcnt that takes the
// destination registers as operands, so nothing reads them earlier.
__device__ __forceinline__ void wg_frag_issue(const char* img, int c0, int lane, bf16x4& lo,
                                              bf16x4& hi) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (c0 >> 3) + (p >> 1);
  const unsigned base = (unsigned)(size_t)(const lds_char*)img;
  const unsigned o0 = base + wg_off(8 * g + q, ch) + 8 * (p & 1);
  const unsigned o1 = base + wg_off(8 * g + 4 + q, ch) + 8 * (p & 1);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(o0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(o1) : "memory");
}
constexpr int WNS = 4;  // wgrad_b16 / wgrad_b16_big ring slots
// (an 8-slot ring, 7 chunks in flight at one workgroup per CU, measured no faster: 74 vs 77 us
// for N = K = 128 at 8 splits -- a split's chunks stream at the per-CU rate, ~26 GB/s, not at a
// latency limit; tools/wgrad_split_sweep.py, profiles/r4_wgrad_split_sweep.txt)
// s_waitcnt vmcnt(N) for a compile-time N (the ring waits below count 4 DMAs per chunk)
template <int N>
__device__ __forceinline__ void wait_vm_c() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most `ahead` chunks (4 DMAs each) are outstanding, ahead in [0, MAXA]
template <int MAXA>
__device__ __forceinline__ void wait_chunks(int ahead) {
  if constexpr (MAXA > 0) {
    if (ahead >= MAXA) {
      wait_vm_c<4 * MAXA>();
      return;
    }
    wait_chunks<MAXA - 1>(ahead);
  } else {
    wait_vm_c<0>();
  }
}

__global__ __launch_bounds__(NTHR) void wgrad_b16_kernel(const WgradArgs a) {
  constexpr int IMG = BK * 256;  // bytes per operand image (32 frames x 128 channels bf16)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int n0, k0, j, s;
  wgrad_tile(a, n0, k0, j, s);
  const int mbeg = s * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int nch = mbeg < mend ? (mend - mbeg + BK - 1) / BK : 0;
  const __bf16* dy = (const __bf16*)a.dy;
  const __bf16* x = (const __bf16*)a.x;
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;

  // this lane's two frame rows (glds i: row wid*8 + 4i + lane/16) and their 16-B chunks
  int fr[2], cc[2], fb[2], ft[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    fr[i] = wid * 8 + 4 * i + (lane >> 4);
    cc[i] = (lane & 15) ^ wg_swz(fr[i]);
    const int m = mbeg + fr[i];
    fb[i] = m / a.Tout;
    ft[i] = m - fb[i] * a.Tout;
  }
  auto issue = [&](int ch) __attribute__((always_inline)) {
    char* A = smem + (ch % WNS) * 2 * IMG;
    char* Bm = A + IMG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mbeg + ch * BK + fr[i];
      const bool mv = m < mend;
      const int n = n0 + cc[i] * 8, k = k0 + cc[i] * 8;
      const void* ga = (mv && n < a.N) ? (const void*)(dy + (long long)m * a.ldy + n)
                                       : (const void*)zp;
      const int src = pad_src(ft[i] + a.shift0 + j * a.dil, a.Tin, a.pad);
      const void* gb = (mv && src >= 0 && k < a.K)
                           ? (const void*)(x + (long long)(fb[i] * a.Tin + src) * a.ldx + k)
                           : (const void*)zp;
      glds16(ga, A + (wid * 8 + 4 * i) * 256);
      glds16(gb, Bm + (wid * 8 + 4 * i) * 256);
      int nt = ft[i] + BK, nb = fb[i];  // this row slot's frame in the next chunk
      while (nt >= a.Tout) {
        nt -= a.Tout;
        ++nb;
      }
      fb[i] = nb;
      ft[i] = nt;
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 4 DMA instructions per lane and chunk: chunk ch has landed once at most 4 * (chunks
  // issued after it) remain outstanding
#pragma unroll
  for (int c = 0; c < WNS - 1; ++c)
    if (c < nch) issue(c);
  for (int ch = 0; ch < nch; ++ch) {
    wait_chunks<WNS - 2>(min(WNS - 2, nch - 1 - ch));
    // chunk ch visible to every wave; every wave is done with chunk ch-1, whose slot the
    // next issue refills
    __builtin_amdgcn_s_barrier();
    if (ch + WNS - 1 < nch) issue(ch + WNS - 1);
    const char* A = smem + (ch % WNS) * 2 * IMG;
    const char* Bm = A + IMG;
    // B fragments, then A fragment rows; row i's MFMAs start once its reads have returned
    bf16x4 blo[4], bhi[4], alo[4], ahi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) wg_frag_issue(Bm, wc * 64 + i * 16, lane, blo[i], bhi[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) wg_frag_issue(A, wr * 64 + i * 16, lane, alo[i], ahi[i]);
    asm volatile("s_waitcnt lgkmcnt(6)"
                 : "+v"(blo[0]), "+v"(bhi[0]), "+v"(blo[1]), "+v"(bhi[1]), "+v"(blo[2]),
                   "+v"(bhi[2]), "+v"(blo[3]), "+v"(bhi[3]), "+v"(alo[0]), "+v"(ahi[0]));
    bf16x8 fbv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      fbv[jj] = __builtin_shufflevector(blo[jj], bhi[jj], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i == 1) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(alo[1]), "+v"(ahi[1]));
      if (i == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(alo[2]), "+v"(ahi[2]));
      if (i == 3) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(alo[3]), "+v"(ahi[3]));
      const bf16x8 fa = __builtin_shufflevector(alo[i], ahi[i], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fbv[jj], acc[i][jj], 0, 0, 0);
    }
  }
  if (a.splits == 1) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
      if (k >= a.K) continue;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
          if (n < a.N) {
            float* d = a.dst + n * a.sn + k * a.sk + j * a.sj;
            const float v = acc[mt][nt][r] * a.scale;
            *d = a.accum ? *d + v : v;
          }
        }
    }
    return;
  }
  float* out = a.part + ((long long)(s * a.taps + j) * a.N) * a.K;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int k = k0 + wc * 64 + nt * 16 + (lane & 15);
    if (k >= a.K) continue;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * 64 + mt * 16 + (lane >> 4) * 4 + r;
        if (n < a.N) out[(long long)n * a.K + k] = acc[mt][nt][r];
      }
  }
}

// ------------------------------------------------- weight grads, 256 x 256 tiles
// wgrad_b16_kernel with a 256 (dy channels) x 256 (x channels) output tile per workgroup of 8
// waves (2 x 4 of 128 x 64: 8 x 4 MFMA tiles), one workgroup per CU (a 4-slot ring of 32 KB
// chunks).  Per frame of a row split it stages 2 x 256 channels where the 128 x 128 kernel's
// four workgroups stage 4 x 256: half the L2 -> LDS bytes, the bound of the 128 x 128 form
// (the DiffNet dilated conv: 380 MB per launch, 42 us).  Each output element takes the same
// chunk sequence and MFMA order as in wgrad_b16_kernel for the same split count: the same bits.
// Staging: the chunk's four [32 frames][128 channels] sub-images (dy lo / hi, x lo / hi, with
// wg_off's swizzle); wave w moves rows 4w .. 4w + 3 of each (one 1-KB DMA per sub-image).
constexpr int WGB = 256, NTHRW = 512;
__device__ __forceinline__ void wgrad_tile_big(const WgradArgs& a, int& n0, int& k0, int& j,
                                               int& s) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int total = gx * gy * gridDim.z;
  const int q = total >> 3, r = total & 7, x = b & 7;
  const int idx = x * q + min(x, r) + (b >> 3);  // XCD-contiguous, as wgrad_tile
  const int W = gx * gy * a.taps;
  s = idx / W;
  const int w = idx - s * W;
  j = w / (gx * gy);
  const int t = w - j * gx * gy;
  k0 = (t / gx) * WGB;
  n0 = (t % gx) * WGB;
}

__global__ __launch_bounds__(NTHRW) void wgrad_b16_big_kernel(const WgradArgs a) {
  constexpr int IMG = BK * 256;  // one sub-image: 32 frames x 128 channels bf16
  constexpr int STG = 4 * IMG;   // dy lo, dy hi, x lo, x hi
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int n0, k0, j, s;
  wgrad_tile_big(a, n0, k0, j, s);
  const int mbeg = s * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int nch = mbeg < mend ? (mend - mbeg + BK - 1) / BK : 0;
  const __bf16* dy = (const __bf16*)a.dy;
  const __bf16* x = (const __bf16*)a.x;
  unsigned long long zpu = (unsigned long long)(const void*)g_zero;
  asm volatile("" : "+s"(zpu));
  const char* zp = (const char*)zpu;
  const int fr = wid * 4 + (lane >> 4);            // this lane's frame row of the chunk
  const int cc = (lane & 15) ^ wg_swz(fr);         // the logical 16-B chunk it fetches
  int fb = (mbeg + fr) / a.Tout, ft = mbeg + fr - fb * a.Tout;
  auto issue = [&](int ch) __attribute__((always_inline)) {
    char* base = smem + (ch % WNS) * STG + (wid * 4) * 256;
    const int m = mbeg + ch * BK + fr;
    const bool mv = m < mend;
    const int src = pad_src(ft + a.shift0 + j * a.dil, a.Tin, a.pad);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = n0 + h * 128 + cc * 8, k = k0 + h * 128 + cc * 8;
      glds16((mv && n < a.N) ? (const void*)(dy + (long long)m * a.ldy + n) : (const void*)zp,
             base + h * IMG);
      glds16((mv && src >= 0 && k < a.K)
                 ? (const void*)(x + (long long)(fb * a.Tin + src) * a.ldx + k)
                 : (const void*)zp,
             base + (2 + h) * IMG);
    }
    ft += BK;
    while (ft >= a.Tout) {
      ft -= a.Tout;
      ++fb;
    }
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  // 4 DMA instructions per lane and chunk, as wgrad_b16_kernel
#pragma unroll
  for (int c = 0; c < WNS - 1; ++c)
    if (c < nch) issue(c);
  for (int ch = 0; ch < nch; ++ch) {
    const int ahead = min(WNS - 2, nch - 1 - ch);
    if (ahead >= 2) wait_vm_n<8>();
    else if (ahead == 1) wait_vm_n<4>();
    else wait_vm_n<0>();
    __builtin_amdgcn_s_barrier();  // chunk ch visible; chunk ch-1's slot free for the refill
    if (ch + WNS - 1 < nch) issue(ch + WNS - 1);
    const char* St = smem + (ch % WNS) * STG;
    const char* Ad = St + wr * IMG;                  // this wave's 128 dy channels
    const char* Bx = St + (2 + (wc >> 1)) * IMG;     // the x sub-image of its 64 channels
    const int cb = (wc & 1) * 64;
    bf16x4 blo[4], bhi[4], alo[8], ahi[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) wg_frag_issue(Bx, cb + 16 * q, lane, blo[q], bhi[q]);
    wg_frag_issue(Ad, 0, lane, alo[0], ahi[0]);
    wg_frag_issue(Ad, 16, lane, alo[1], ahi[1]);
    asm volatile("s_waitcnt lgkmcnt(4)"
                 : "+v"(blo[0]), "+v"(bhi[0]), "+v"(blo[1]), "+v"(bhi[1]), "+v"(blo[2]),
                   "+v"(bhi[2]), "+v"(blo[3]), "+v"(bhi[3]));
    bf16x8 fbv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      fbv[q] = __builtin_shufflevector(blo[q], bhi[q], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i + 2 < 8) {
        wg_frag_issue(Ad, 16 * (i + 2), lane, alo[i + 2], ahi[i + 2]);
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(alo[i]), "+v"(ahi[i]));
      } else if (i == 6) {
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(alo[i]), "+v"(ahi[i]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(alo[i]), "+v"(ahi[i]));
      }
      const bf16x8 fa = __builtin_shufflevector(alo[i], ahi[i], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fbv[q], acc[i][q], 0, 0, 0);
    }
  }
  float* out = a.splits == 1 ? nullptr : a.part + ((long long)(s * a.taps + j) * a.N) * a.K;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = k0 + wc * 64 + q * 16 + (lane & 15);
    if (k >= a.K) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * 128 + i * 16 + (lane >> 4) * 4 + r;
        if (n >= a.N) continue;
        if (out) {
          out[(long long)n * a.K + k] = acc[i][q][r];
        } else {
          float* d = a.dst + n * a.sn + k * a.sk + j * a.sj;
          const float v = acc[i][q][r] * a.scale;
          *d = a.accum ? *d + v : v;
        }
      }
  }
}

// dst[n*sn + k*sk + j*sj] (+)= scale * sum_s part[s][j][n][k]   (fixed summation order: split
// 0, 1, 2, ..). One thread per (j, n, k) element, 16 split loads in flight per thread (4
// measured as a latency-bound 7 us average launch: 4 waves per CU x 4 loads).
constexpr int WRED_ILP = 16;
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                           float* __restrict__ dst, int splits,
                                                           int taps, int N, int K, long long sn,
                                                           long long sk, long long sj, int accum,
                                                           float scale) {
  const long long stride = (long long)N * K * taps;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // (j * N + n) * K + k
  if (e >= stride) return;
  const int row = (int)(e / K), k = (int)(e - (long long)row * K);
  const int j = row / N, n = row - j * N;
  const float* p = part + e;
  float v = 0.f;
  int sp = 0;
  for (; sp + WRED_ILP <= splits; sp += WRED_ILP) {
    float t[WRED_ILP];
#pragma unroll
    for (int i = 0; i < WRED_ILP; ++i) t[i] = p[(sp + i) * stride];
#pragma unroll
    for (int i = 0; i < WRED_ILP; ++i) v += t[i];
  }
  for (; sp < splits; ++sp) v += p[sp * stride];
  v *= scale;
  float* d = dst + n * sn + k * sk + j * sj;
  *d = accum ? (*d + v) : v;
}

// Deferred reductions of several weight gradients in one launch (ensvs_wgrad_reduce_batch):
// blockIdx.y picks the descriptor, each thread one destination element -- the per-element sum
// of wgrad_reduce_kernel, so the bits are the same.
constexpr int WRED_BATCH = 48;
struct WredBatch {
  ensvs_wred_desc d[WRED_BATCH];
};
static_assert(sizeof(WredBatch) <= 3584, "kernel argument size");

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(const WredBatch b) {
  const ensvs_wred_desc& d = b.d[blockIdx.y];
  const long long stride = (long long)d.N * d.K * d.taps;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // (j * N + n) * K + k
  if (e >= stride) return;
  const int row = (int)(e / d.K), k = (int)(e - (long long)row * d.K);
  const int j = row / d.N, n = row - j * d.N;
  const float* p = d.part + e;
  const int splits = d.splits;
  float v = 0.f;
  int sp = 0;
  for (; sp + WRED_ILP <= splits; sp += WRED_ILP) {
    float t[WRED_ILP];
#pragma unroll
    for (int i = 0; i < WRED_ILP; ++i) t[i] = p[(sp + i) * stride];
#pragma unroll
    for (int i = 0; i < WRED_ILP; ++i) v += t[i];
  }
  for (; sp < splits; ++sp) v += p[sp * stride];
  v *= d.scale;
  float* o = d.dst + n * d.sn + k * d.sk + j * d.sj;
  *o = (d.accum & 1) ? (*o + v) : v;
}

// ---------------------------------------------------------- weight packing
struct PackDesc {
  const float* src;
  const float* src2;  // optional second source added element-wise (fused biases)
  void* dst;
  long long sn, sk, sj;
  int N, K, taps, Npad, Kp, perm_c, flip, transpose, dtype;
  float scale;
  int ldk;    // dst row stride (elements); 0 -> Kp
  int tile0;  // pack_tile_kernel: the descriptor's first tile in the launch
};

__global__ void pack_kernel(const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  const long long total = (long long)d.taps * d.Npad * d.Kp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % d.Kp);
    const int n = (int)((i / d.Kp) % d.Npad);
    const int j = (int)(i / ((long long)d.Kp * d.Npad));
    // logical (packed) n -> source output row
    int nn = n;
    if (d.perm_c > 0) {  // 16-interleave of two halves of width perm_c
      const int q = n >> 5, w = n & 31;
      nn = (w < 16) ? q * 16 + w : d.perm_c + q * 16 + (w - 16);
    }
    const int jj = d.flip ? (d.taps - 1 - j) : j;
    const int nlim = d.transpose ? d.K : d.N;
    const int klim = d.transpose ? d.N : d.K;
    float v = 0.f;
    if (nn < nlim && k < klim && n < (d.perm_c > 0 ? 2 * d.perm_c : nlim)) {
      long long off = d.transpose ? (k * d.sn + (long long)nn * d.sk + jj * d.sj)
                                  : ((long long)nn * d.sn + k * d.sk + jj * d.sj);
      v = d.src[off];
      if (d.src2) v += d.src2[off];
      v *= d.scale;
    }
    const long long o = d.ldk > 0 ? ((long long)j * d.Npad + n) * d.ldk + k : i;
    if (d.dtype == DT_BF16) ((__bf16*)d.dst)[o] = (__bf16)v;
    else ((float*)d.dst)[o] = v;
  }
}

// Tiled repack: one workgroup per 64 x 64 (n, k) tile of one tap of one descriptor, the
// descriptors' tiles numbered consecutively (tile0: prefix sums of taps * cdiv(Npad, 64) *
// cdiv(Kp, 64)).  The tile is read along the source's unit-stride axis into LDS and written
// along the packed rows, so both sides are coalesced -- the transposed (input-gradient)
// operands read a column per wavefront in pack_kernel -- with 32-bit index arithmetic, and the
// grid is exactly the tiles (pack_kernel launches max-size x n workgroups, most of them idle).
// Each element is the same value as in pack_kernel (same source element, same adds and
// scaling, same rounding).
constexpr int PACK_T = 64;

__global__ __launch_bounds__(256) void pack_tile_kernel(const PackDesc* __restrict__ descs,
                                                        int n) {
  __shared__ float tile[PACK_T][PACK_T + 1];
  const int b = blockIdx.x;
  // the last descriptor with tile0 <= b (tile0 ascending): a count, one load round per 256
  int cnt = 0;
  for (int base = 0; base < n; base += 256) {
    const int i = base + (int)threadIdx.x;
    cnt += __syncthreads_count(i < n && descs[i].tile0 <= b);
  }
  if (cnt < 1) return;
  const PackDesc d = descs[cnt - 1];
  const int nt = (d.Npad + PACK_T - 1) / PACK_T, kt = (d.Kp + PACK_T - 1) / PACK_T;
  int t = b - d.tile0;
  const int kb = t % kt;
  t /= kt;
  const int nb = t % nt, j = t / nt;
  if (t < 0 || j >= d.taps) return;  // (a tile count that does not match the descriptors)
  const int n0 = nb * PACK_T, k0 = kb * PACK_T;
  const int jj = d.flip ? (d.taps - 1 - j) : j;
  const int nlim = d.transpose ? d.K : d.N;
  const int klim = d.transpose ? d.N : d.K;
  const int nmax = d.perm_c > 0 ? 2 * d.perm_c : nlim;
  const long long s_n = d.transpose ? d.sk : d.sn;  // source stride along packed n
  const long long s_k = d.transpose ? d.sn : d.sk;  // ... along packed k
  const float* src = d.src + jj * d.sj;
  const float* src2 = d.src2 ? d.src2 + jj * d.sj : nullptr;
  const bool kfast = s_k <= s_n;
  // all 16 loads of a lane in flight before the first use (then the adds, scaling and LDS
  // stores), so a tile costs about one memory latency
  constexpr int PER = PACK_T * PACK_T / 256;
  float v[PER], v2[PER];
  bool in[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 256;
    const int a = e & (PACK_T - 1), c = e / PACK_T;
    const int pn = n0 + (kfast ? c : a), k = k0 + (kfast ? a : c);
    int nn = pn;
    if (d.perm_c > 0) {  // 16-interleave of two halves of width perm_c
      const int q = pn >> 5, w = pn & 31;
      nn = (w < 16) ? q * 16 + w : d.perm_c + q * 16 + (w - 16);
    }
    in[i] = nn < nlim && k < klim && pn < nmax;
    const long long off = in[i] ? (long long)nn * s_n + (long long)k * s_k : 0;
    v[i] = in[i] ? src[off] : 0.f;
    v2[i] = (in[i] && src2) ? src2[off] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 256;
    const int a = e & (PACK_T - 1), c = e / PACK_T;
    float x = v[i];
    if (in[i]) {
      if (src2) x += v2[i];
      x *= d.scale;
    }
    tile[kfast ? c : a][kfast ? a : c] = x;
  }
  __syncthreads();
  const int ld = d.ldk > 0 ? d.ldk : d.Kp;
  for (int e = threadIdx.x; e < PACK_T * PACK_T; e += 256) {
    const int tk = e & (PACK_T - 1), tn = e / PACK_T;
    const int pn = n0 + tn, k = k0 + tk;
    if (pn >= d.Npad || k >= d.Kp) continue;
    const long long o = ((long long)j * d.Npad + pn) * ld + k;
    const float v = tile[tn][tk];
    if (d.dtype == DT_BF16) ((__bf16*)d.dst)[o] = (__bf16)v;
    else ((float*)d.dst)[o] = v;
  }
}

// --------------------------------------------------------- column reductions
// part[s][n] = sum over rows [s*rps, (s+1)*rps) of f(Y[row, n]); mode 0: y, 1: (y-mean)^2
// Column sums over frame rows (bias gradients, BatchNorm statistics, per-sequence
// sums).  Memory-bound: 64 columns x 16 row lanes per block, float4 loads with 4
// rows in flight per lane; partials [group][split][N] are reduced by colsum_final
// in a fixed order (deterministic).
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ y, int ld,
                                                             int M, int N, int rps,
                                                             const float* __restrict__ mean,
                                                             float* __restrict__ part) {
  __shared__ f32x4 red[16][17];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  const int s = blockIdx.y;
  y += (long long)blockIdx.z * M * ld;
  part += (long long)blockIdx.z * gridDim.y * N;
  const int r0 = s * rps, r1 = min(M, r0 + rps);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 mu = {0.f, 0.f, 0.f, 0.f};
  if (mean) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (col + e < N) mu[e] = mean[(long long)blockIdx.z * N + col + e];
  }
  auto ld4 = [&](int r) -> f32x4 {
    const float* q = y + (long long)r * ld + col;
    f32x4 v;
    if (VEC && col + 3 < N) {
      v = *(const f32x4*)q;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = col + e < N ? q[e] : 0.f;
    }
    if (mean) {
      v -= mu;
      v *= v;
#pragma unroll
      for (int e = 0; e < 4; ++e) if (col + e >= N) v[e] = 0.f;
    }
    return v;
  };
  if (col < N) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      const f32x4 v0 = ld4(r), v1 = ld4(r + 16), v2 = ld4(r + 32), v3 = ld4(r + 48);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; r < r1; r += 16) acc += ld4(r);
  }
  red[rl][cq] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;  // column within the block
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c >> 2][c & 3];
    const int gc = blockIdx.x * 64 + c;
    if (gc < N) part[(long long)s * N + gc] = t;
  }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int S,
                                                           int N, float scale,
                                                           float* __restrict__ out, int ldo,
                                                           int accum) {
  // 16 columns x 16 split lanes per block, 4 partial loads in flight per lane.
  __shared__ double red[16][17];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c;
  part += (long long)blockIdx.y * S * N;
  out += (long long)blockIdx.y * ldo;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (col < N) {
    int s = sl;
    for (; s + 48 < S; s += 64) {
      a0 += part[(long long)s * N + col];
      a1 += part[(long long)(s + 16) * N + col];
      a2 += part[(long long)(s + 32) * N + col];
      a3 += part[(long long)(s + 48) * N + col];
    }
    for (; s < S; s += 16) a0 += part[(long long)s * N + col];
  }
  red[sl][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && col < N) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    const float v = (float)(t * scale);
    out[col] = accum ? out[col] + v : v;
  }
}

// Deferred column sums of several parameter gradients (ensvs_colsum_batch): blockIdx.z /
// blockIdx.y picks the descriptor; each block runs colsum_partial_kernel's / colsum_final_kernel's
// body on its columns (the same split count, rows per split and summation order: the same bits).
struct CsDesc {
  const float* y;
  float* out;
  int ld, M, N, rps, S, vec;
  long long part_off;
  float scale;
  int accum;
};
constexpr int CS_BATCH = 48;
struct CsBatch {
  CsDesc d[CS_BATCH];
};
static_assert(sizeof(CsBatch) <= 3584, "kernel argument size");

__global__ __launch_bounds__(256) void colsum_partial_batch_kernel(const CsBatch b,
                                                                   float* __restrict__ part) {
  const CsDesc& d = b.d[blockIdx.z];
  if ((int)blockIdx.x * 64 >= d.N || (int)blockIdx.y >= d.S) return;
  __shared__ f32x4 red[16][17];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int N = d.N, col = blockIdx.x * 64 + cq * 4;
  const int s = blockIdx.y;
  const int r0 = s * d.rps, r1 = min(d.M, r0 + d.rps);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto ld4 = [&](int r) -> f32x4 {
    const float* q = d.y + (long long)r * d.ld + col;
    f32x4 v;
    if (d.vec && col + 3 < N) {
      v = *(const f32x4*)q;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = col + e < N ? q[e] : 0.f;
    }
    return v;
  };
  if (col < N) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      const f32x4 v0 = ld4(r), v1 = ld4(r + 16), v2 = ld4(r + 32), v3 = ld4(r + 48);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; r < r1; r += 16) acc += ld4(r);
  }
  red[rl][cq] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c >> 2][c & 3];
    const int gc = blockIdx.x * 64 + c;
    if (gc < N) part[d.part_off + (long long)s * N + gc] = t;
  }
}

__global__ __launch_bounds__(256) void colsum_final_batch_kernel(const CsBatch b,
                                                                 const float* __restrict__ part) {
  const CsDesc& d = b.d[blockIdx.y];
  if ((int)blockIdx.x * 16 >= d.N) return;
  __shared__ double red[16][17];
  const int N = d.N, S = d.S;
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c;
  const float* p = part + d.part_off;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (col < N) {
    int s = sl;
    for (; s + 48 < S; s += 64) {
      a0 += p[(long long)s * N + col];
      a1 += p[(long long)(s + 16) * N + col];
      a2 += p[(long long)(s + 32) * N + col];
      a3 += p[(long long)(s + 48) * N + col];
    }
    for (; s < S; s += 16) a0 += p[(long long)s * N + col];
  }
  red[sl][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && col < N) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    const float v = (float)(t * d.scale);
    d.out[col] = d.accum ? d.out[col] + v : v;
  }
}

// colsum_partial_kernel + colsum_final_kernel in one launch: each block writes its split's
// partial row as the partial kernel does, then takes a ticket on its (column block, group)
// counter; the block that draws the last ticket runs the final kernel's sums for its 64
// columns (four 16-column passes of the same 16 split lanes, the same double-precision order:
// the same bits) and resets the counter.  Publish / acquire: the guide's in-launch split
// reduction in its write-through form (cdna_hip_programming.md, "Projection GEMM at M = 256"
// item 2): sc1 partial stores -> vmcnt(0) -> barrier -> relaxed agent ticket; the last block
// reads every partial with sc1 loads.  (The release / acquire-fence form wrote the L2 back in
// every one of the ~1 000 blocks of a step's column sums: 23.6 us per launch against 10.3 for
// the two launches, profiles/r5_colsum_once_fence.txt.)
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_once_kernel(const float* __restrict__ y, int ld,
                                                          int M, int N, int rps,
                                                          const float* __restrict__ mean,
                                                          float* __restrict__ part,
                                                          unsigned* __restrict__ cnt, float scale,
                                                          float* __restrict__ out, int ldo,
                                                          int accum) {
  __shared__ f32x4 red[16][17];
  __shared__ double dred[16][17];
  __shared__ int last;
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  const int s = blockIdx.y, S = gridDim.y;
  y += (long long)blockIdx.z * M * ld;
  float* gpart = part + (long long)blockIdx.z * S * N;
  const int r0 = s * rps, r1 = min(M, r0 + rps);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 mu = {0.f, 0.f, 0.f, 0.f};
  if (mean) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (col + e < N) mu[e] = mean[(long long)blockIdx.z * N + col + e];
  }
  auto ld4 = [&](int r) -> f32x4 {
    const float* q = y + (long long)r * ld + col;
    f32x4 v;
    if (VEC && col + 3 < N) {
      v = *(const f32x4*)q;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = col + e < N ? q[e] : 0.f;
    }
    if (mean) {
      v -= mu;
      v *= v;
#pragma unroll
      for (int e = 0; e < 4; ++e) if (col + e >= N) v[e] = 0.f;
    }
    return v;
  };
  if (col < N) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      const f32x4 v0 = ld4(r), v1 = ld4(r + 16), v2 = ld4(r + 32), v3 = ld4(r + 48);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; r < r1; r += 16) acc += ld4(r);
  }
  red[rl][cq] = acc;
  __syncthreads();
  // this group's partials [S][N] through a buffer resource: sc1 stores and loads
  const __amdgpu_buffer_rsrc_t pr =
      __builtin_amdgcn_make_buffer_rsrc(gpart, 0, (int)((long long)S * N * 4), 0x00020000);
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c >> 2][c & 3];
    const int gc = blockIdx.x * 64 + c;
    if (gc < N)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, t), pr,
                                            (s * N + gc) * 4, 0, 16 /* sc1 */);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* c = cnt + blockIdx.z * gridDim.x + blockIdx.x;
    const unsigned tk = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == (unsigned)(S - 1);
    if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // colsum_final_kernel's body for columns blockIdx.x * 64 + 16 q + c
  float* o = out + (long long)blockIdx.z * ldo;
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  for (int q = 0; q < 4; ++q) {
    const int cc = blockIdx.x * 64 + q * 16 + c;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (cc < N) {
      int sp = sl;
      auto ldp = [&](int i) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(pr, (i * N + cc) * 4,
                                                                              0, 16 /* sc1 */));
      };
      for (; sp + 48 < S; sp += 64) {
        a0 += ldp(sp);
        a1 += ldp(sp + 16);
        a2 += ldp(sp + 32);
        a3 += ldp(sp + 48);
      }
      for (; sp < S; sp += 16) a0 += ldp(sp);
    }
    dred[sl][c] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (sl == 0 && cc < N) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += dred[i][c];
      const float v = (float)(t * scale);
      o[cc] = accum ? o[cc] + v : v;
    }
    __syncthreads();
  }
}

}  // namespace

// =================================================================== C ABI

static inline long long cdiv_ll(long long a, long long b) { return (a + b - 1) / b; }


static int fill_gemm_args(GemmArgs& a, const ensvs_conv_seg* segs, int nseg, int B, int Tout,
                          int N, int Npad, const void* W, const float* bias, float* Y, int ldy,
                          int epi, int relu, int accum, float* aux0, int ld0, const float* aux1,
                          int ld1, float alpha, int C) {
  if (nseg < 1 || nseg > 3 || B <= 0 || Tout <= 0 || N <= 0 || Npad % BN != 0 || Npad < N)
    return ENSVS_E_SHAPE;
  for (int s = 0; s < nseg; ++s) {
    const ensvs_conv_seg& g = segs[s];
    if (g.Kp % BK != 0 || g.Kp < g.K || g.taps < 1) return ENSVS_E_SHAPE;
    a.seg[s].x = g.x;
    a.seg[s].radd = g.radd;
    a.seg[s].pd = g.pd;
    a.seg[s].pd_dil = g.pd_dil;
    // a pitch-dependent segment: the first one, 3 taps (past/current/future), Tin == Tout
    if (g.pd && (s != 0 || g.taps != 3 || g.Tin != Tout)) return ENSVS_E_SHAPE;
    a.seg[s].wofs = g.wofs;
    a.seg[s].ld = g.ld;
    a.seg[s].K = g.K;
    a.seg[s].taps = g.taps;
    a.seg[s].dil = g.dil;
    a.seg[s].shift0 = g.shift0;
    a.seg[s].pad = g.pad;
    a.seg[s].radd_ld = g.radd_ld;
    a.seg[s].Tin = g.Tin;
    a.seg[s].Kp = g.Kp;
    a.seg[s].vec = (g.K % 4 == 0) && (g.ld % 4 == 0) && (((uintptr_t)g.x & 15) == 0) &&
                   (!g.radd || ((g.radd_ld % 4 == 0) && (((uintptr_t)g.radd & 15) == 0)));
  }
  // epi bits 8 / 9: aux0 / aux1 hold bf16 (only the gate save and its backward read)
  a.aux0_bf = (epi & EPI_AUX0_BF16) ? 1 : 0;
  a.aux1_bf = (epi & EPI_AUX1_BF16) ? 1 : 0;
  epi &= 0xff;
  if ((a.aux0_bf && epi != EPI_GATE) || (a.aux1_bf && epi != EPI_GATE_BWD)) return ENSVS_E_ARG;
  // each epilogue's output / operand widths: an inconsistent set would index past the
  // caller's rows (the kernels trust these)
  switch (epi) {
    case EPI_PLAIN:
      if (Y && ldy < N) return ENSVS_E_SHAPE;
      break;
    case EPI_GATE:
    case EPI_GATE_TS:
    case EPI_RESSKIP:  // N = 2C interleaved pairs -> C output channels
      if (C <= 0 || N != 2 * C || (Y && ldy < C)) return ENSVS_E_SHAPE;
      if (epi == EPI_GATE && aux0 && ld0 < 2 * C) return ENSVS_E_SHAPE;
      if (epi == EPI_RESSKIP && (!Y || !aux0 || !aux1 || ld0 < C || ld1 < C)) return ENSVS_E_ARG;
      break;
    case EPI_GATE_BWD:  // N = C channels of dz -> 2C pre-activation gradients
      if (C <= 0 || N != C || !aux1 || ld1 < 2 * C || (Y && ldy < 2 * C)) return ENSVS_E_SHAPE;
      break;
    case EPI_ADDSCALE:
    case EPI_RELU_MASK:
      if (!Y || !aux1 || ldy < N || ld1 < N) return ENSVS_E_ARG;
      break;
    case EPI_NONE:
      break;
    default:
      return ENSVS_E_ARG;
  }
  a.nseg = nseg;
  a.Tout = Tout;
  a.M = B * Tout;
  a.N = N;
  a.Npad = Npad;
  a.W = W;
  a.bias = bias;
  a.Y = Y;
  a.ldy = ldy;
  a.epi = epi;
  a.relu = relu;
  a.accum = accum;
  a.aux0 = aux0;
  a.aux1 = aux1;
  a.ld0 = ld0;
  a.ld1 = ld1;
  a.alpha = alpha;
  a.C = C;
  auto al = [](const void* p, int ld) { return !p || ((((uintptr_t)p) & 15) == 0 && ld % 4 == 0); };
  auto al8 = [](const void* p, int ld) { return !p || ((((uintptr_t)p) & 7) == 0 && ld % 4 == 0); };
  a.vec_out = al(Y, ldy) && (a.aux0_bf ? al8(aux0, ld0) : al(aux0, ld0)) &&
              (a.aux1_bf ? al8(aux1, ld1) : al(aux1, ld1)) && (C % 4 == 0);
  a.gate8 = a.vec_out && C % 8 == 0 &&
            (!a.aux0_bf || (((uintptr_t)aux0 & 15) == 0 && ld0 % 8 == 0));
  return ENSVS_OK;
}

ENSVS_API int ensvs_conv_gemm(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N,
                              int Npad, const void* W, int wdtype, const float* bias, float* Y,
                              int ldy, int epi, int relu, int accum, float* aux0, int ld0,
                              const float* aux1, int ld1, float alpha, int C, void* stream) {
  GemmArgs a{};
  const int rc = fill_gemm_args(a, segs, nseg, B, Tout, N, Npad, W, bias, Y, ldy, epi, relu,
                                accum, aux0, ld0, aux1, ld1, alpha, C);
  if (rc != ENSVS_OK) return rc;
  bool vec = true;
  for (int s = 0; s < nseg; ++s) vec = vec && a.seg[s].vec;
  dim3 grid(cdiv(a.M, BM), Npad / BN);
  hipStream_t st = (hipStream_t)stream;
  const bool pd = a.seg[0].pd != nullptr;
#define LAUNCH_GEMM(T, V, P)                                                            \
  hipLaunchKernelGGL((conv_gemm_kernel<T, V, P>), grid, dim3(NTHR),                    \
                     2 * (BM + BN) * Lds<T>::K * sizeof(T), st, a)
  if (wdtype == DT_BF16) {
    if (pd) {
      if (vec) LAUNCH_GEMM(__bf16, true, true); else LAUNCH_GEMM(__bf16, false, true);
    } else {
      if (vec) LAUNCH_GEMM(__bf16, true, false); else LAUNCH_GEMM(__bf16, false, false);
    }
  } else if (wdtype == DT_F32) {
    if (pd) {
      if (vec) LAUNCH_GEMM(float, true, true); else LAUNCH_GEMM(float, false, true);
    } else {
      if (vec) LAUNCH_GEMM(float, true, false); else LAUNCH_GEMM(float, false, false);
    }
  } else {
    return ENSVS_E_DTYPE;
  }
#undef LAUNCH_GEMM
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// The 256 x 256 kernel takes a bf16-operand launch when it fills the chip with whole
// tiles (>= 192 workgroups of 256 x 256), its LDS epilogue applies (16-B rows, no column
// sums) and the padded N is a multiple of 256.  Mode (ensvs_set_big_tile): 0 off, 1 the
// 32-deep ring kernel with g_big_stages stages, 2 (default) the 64-deep two-stage kernel,
// 3 as 2 for every eligible epilogue (the bitwise tests).  Gate GEMM (tools/gate_probe.py):
// 2 -> 44.8 us, 1 (5 / 4 / 3 stages) -> 53.3 / 53.0 / 50.2 us, 0 (128 x 128) -> 51.0 us:
// more LDS stages in flight did not pay.
static int g_big_tile = 2, g_big_stages = 5, g_big_all = 0;
// GATE_BWD LDS-DMA epilogue (gate_bwd_epilogue_dma); off: the register form, same bits
static int g_gbw_dma = 1;
// bf16 weight gradients with N, K >= 256 on the 256 x 256-tile kernel (same bits for the same
// split count); off: the 128 x 128 one
static int g_wgrad_big = 1;
// Only where there are many output tiles (>= 16 of 256 x 256): the 256 x 256 form was slower
// wherever a few tiles take many row splits (tools/wgrad_bench.py: DiffNet dilated conv 48.2
// -> 52.5 us, residual 1x1 24.5 -> 35.0, LSTM W_ih 33.5 -> 42.9) and faster on the block-shared
// conditioner (N = 10 240: 296 -> 231 us) and skip projection (K = 5 120: 131 -> 118 us):
// with one workgroup per CU its chunks ran 1.8 us apart, twice the 128 x 128 kernel's per-CU
// byte rate lost to the barrier of one 8-wave workgroup (profiles/r4_wgrad_big_bench.txt).
static bool wgrad_big_shape(int N, int K, int taps) {
  return g_wgrad_big && N >= WGB && K >= WGB && (long long)cdiv(N, WGB) * cdiv(K, WGB) * taps >= 16;
}
// split-K fills about this many workgroups (only when the caller passes a workspace)
static const int SPLITK_TARGET = 256;
// launches of fewer than 128 tiles of 128 x 128 that the 64 x 64 kernel does not take (no
// 16-B epilogue rows) run the two-K-group kernel when on (ensvs_set_dual_small; off: the
// one-group kernel keeps the register-staged bits, e.g. the DiffNet output projection's
// 5-column rows)
static int g_dual_small = 0;
// launches of fewer than 128 tiles of 128 x 128 run the 64 x 64-tile kernel (ensvs_set_small,
// default on); it takes precedence over split-K and dual
static int g_small = 1;
// the 64 x 64 kernel's LDS-DMA ring depth (3..5 measured on the 2 000-frame reverse process)
static const int SMALL_STAGES = 5;
// at least this many 256 x 256 tiles (the chip's 256 CUs less a margin) for the big kernel
static const int BIG_MIN_TILES = 192;

// The four-phase 256 x 256 kernel (conv_gemm_b16_p8_kernel): 0 off, 1 in place of the
// two-stage 256 x 256 kernel (the gate GEMMs), 2 (default) also for every other launch the
// 256 x 256 epilogue serves with at least P8_MIN_TILES tiles -- the recurrences' input
// projections and input gradients, the 1 x 1 and conv-stack GEMMs: with the lean plain epilogue
// at or below hipBLASLt on those shapes (tools/p8_bench.py, profiles/r6_p8_bench.txt), main line
// 13.47 / 13.47 ms vs 13.44 / 13.38 with hipBLASLt for the plain GEMMs and 13.61 / 13.63 with
// them on the 128 x 128 kernel; SeparateF0 43.0 / 42.5 vs 42.9 / 42.9 and 43.9 / 43.9
// (profiles/r6_blas_ab.txt, r6_blas_ab_sf0.txt).
// 2 (default): every launch of >= 128 tiles its epilogues serve.  The generic instance stages
// the tile in two passes (no spills): relu + bf16-copy and ReLU-mask launches 77 / 86 / 127 us
// vs the 128 x 128 kernel's 87 / 107 / 170, main line 13.33 / 13.33 vs 13.41 / 13.38 ms with
// them on the 128 x 128 kernel (mode 3), Transformer leg 3.74 vs 3.78 (profiles/
// r6_p8_generic_bench.txt, r6_p8_generic_ab.txt; with the spilling one-pass instance mode 3 was
// the faster: r6_tf_p8_ab.txt, r6_p8_mode7_ab.txt).  3: the gate GEMMs and the lean plain
// launches only.
static int g_p8 = 2;
// 1: two barriers per phase with the wave rows staggered half a phase (default: 1-5 % faster
// than one barrier per phase on every shape, bit-identical output; tools/p8_bench.py,
// profiles/r6_p8_stagger.txt); 0: one barrier per phase, rows in lockstep
static int g_p8_bar2 = 1;
static int g_p8_nodma = 0;  // measurement (EPI_NONE launches only): skip the K loop's loads
static const int P8_MIN_TILES = 128;
// the four-phase kernel's smallest launch (tiles of 256 x 256) for its non-gate epilogues
// (ensvs_set_p8_min_tiles; A/B)
static int g_p8_min_tiles = P8_MIN_TILES;

// the lean plain epilogue's launches: fp32 Y = acc (+ bias), nothing else, 16-B aligned rows
static bool p8_plain(const GemmArgs& a) {
  return a.epi == EPI_PLAIN && !a.accum && !a.relu && !a.ybf && !a.csum && a.Y &&
         a.N % 4 == 0 && a.ldy % 4 == 0 && ((uintptr_t)a.Y & 15) == 0 &&
         (!a.bias || ((uintptr_t)a.bias & 3) == 0);
}

static bool use_p8(const GemmArgs& a, const ensvs_conv_seg* segs, int nseg, int B) {
  if (!g_p8 || a.csum || !a.vec_out || a.Npad % BNB || a.gbw_dma || a.as_dma) return false;
  for (int s = 0; s < nseg; ++s)  // 31-bit byte offsets into the operand resources
    if ((long long)B * segs[s].Tin * segs[s].ld >= (1ll << 30)) return false;
  const long long tiles = (long long)cdiv(a.M, BMB) * (a.Npad / BNB);
  if (a.epi == EPI_GATE) return g_big_tile && tiles >= BIG_MIN_TILES;
  if (tiles < g_p8_min_tiles || g_p8 < 2) return false;
  // mode 3: the lean plain launches only (the generic epilogue's launches on the 128 x 128
  // kernel); EPI_NONE: the K loop alone, measurement
  return g_p8 == 2 || p8_plain(a) || a.epi == EPI_NONE;
}

// The 128 x 256 kernel (conv_gemm_b16_p8h_kernel) for the launches the 256 x 256 one leaves
// with too few tiles -- the N = 256 GEMMs at 30 k frames (240 workgroups of 128 x 256 vs 120 of
// 256 x 256).  Its K loop streams ~33 GB/s of operands per CU, as the four-phase kernel's
// does (the bytes in flight per CU over the L2 / fabric latency bound both), which at 48 KB
// per 4.2-MFLOP K-step is 0.29 of the MFMA peak, and its one workgroup per CU runs an
// operand-heavy epilogue at one row of loads in flight per thread: on the DiffNet's dilated
// dgrad, gate-backward and residual launches it measured 49 / 38 / 25 us against the 128 x 128
// kernel's 38.7 / 24.9 / 21.7 (two workgroups per CU, LDS-DMA epilogues), the step +1.2 ms
// (tools/p8h_bench.py, profiles/r6_p8h_bench.txt, r6_p8h_ab.txt).  It runs where it wins: the
// lean plain epilogue over a long K (>= 32 K-steps: the skip sum K = 5 120, 111.7 vs
// 123.6 us; the conditioner input gradient K = 10 240).  Every epilogue stays available
// (ensvs_set_p8h(2), bitwise tests).  0: off; 1: long-K plain launches; 2: every launch.
static int g_p8h = 1;
// the lean plain launches it takes: >= this many K-steps.  1 (default): the short-K ones win
// too -- the DiffNet's d(skip) GEMM (K = 256) 14.4 vs 20.6 us on the 128 x 128 kernel (16.8 on
// the 256 x 256 kernel at 120 tiles; r6_p8_n256_bench.txt); 32 was round 6's first rule
static int g_p8h_min_ksteps = 1;

static bool use_p8h(const GemmArgs& a, const ensvs_conv_seg* segs, int nseg, int B) {
  if (!g_p8h || !a.vec_out || a.Npad % BNB) return false;
  if (a.epi == EPI_GATE || a.epi == EPI_RESSKIP || a.epi == EPI_GATE_TS) return false;
  for (int s = 0; s < nseg; ++s)  // 31-bit byte offsets into the operand resources
    if ((long long)B * segs[s].Tin * segs[s].ld >= (1ll << 30)) return false;
  if ((long long)cdiv(a.M, BMH) * (a.Npad / BNB) < P8_MIN_TILES) return false;
  if (g_p8h == 2) return true;
  int nit = 0;
  for (int s = 0; s < nseg; ++s) nit += cdiv(segs[s].K, BK2) * segs[s].taps;
  if (nit < g_p8h_min_ksteps) return false;
  const bool lean = a.epi == EPI_PLAIN && !a.accum && !a.relu && !a.ybf && !a.csum;
  if (g_p8h == 3) return lean;
  // mode 1: also the PLAIN epilogues with operands / copies / column sums and ADDSCALE without
  // column sums, whose operands the epilogue prefetches 8 rows ahead (skip ReLU + bf16 copy
  // 20.0 vs 23.1 us, first dilated dgrad with tile sums 45.8 vs 47.3, residual ADDSCALE 21.1
  // vs 21.7) and RELU_MASK without column sums (19.0 vs 24.0 us,
  // profiles/r6_p8h_relumask_bench.txt); the gate backward and the ADDSCALE dgrad with tile
  // sums stay on the 128 x 128 kernel's LDS-DMA epilogues (38.7 vs 25.6, 46.6 vs 39.2 us;
  // profiles/r6_p8h_epi_bench.txt)
  return a.epi == EPI_PLAIN || ((a.epi == EPI_ADDSCALE || a.epi == EPI_RELU_MASK) && !a.csum);
}

static bool use_big_tile(const GemmArgs& a) {
  if (!g_big_tile || a.csum || !a.vec_out || a.Npad % BNB) return false;
  // Only the gate GEMMs (K = 1 024) take the 256 x 256 kernel: the DiffNet res/skip GEMM
  // (K = 256, an epilogue reading the residual and skip rows) runs 47 vs 55 us per launch on
  // 128 x 128 tiles, the other wide launches (N = 512 plain / ReLU-mask, K = 256-512) 39 vs
  // 46 and 62 vs 71 us; step 20.1 vs 20.75 ms (profiles/r2_schedule_ab.txt).
  if (!g_big_all && a.epi != EPI_GATE) return false;
  return (long long)cdiv(a.M, BMB) * (a.Npad / BNB) >= BIG_MIN_TILES;
}

static int launch_b16(GemmArgs& a, const ensvs_conv_seg* segs, int nseg, int B, int Npad,
                      const void* W, int stages, hipStream_t st) {
  for (int s = 0; s < nseg; ++s) {
    const ensvs_conv_seg& g = segs[s];
    // K % 8 != 0: the caller zero-pads the operand rows to a multiple of 8 within ld (the
    // last 16-B chunk reads the padding; the packed weights are zero there anyway)
    // (pd: segment 0 only, checked by fill_gemm_args; the 128 x 128 kernel gathers it)
    if (g.radd || g.ld % 8 || g.ld < ((g.K + 7) & ~7) || ((uintptr_t)g.x & 15))
      return ENSVS_E_ARG;
  }
  if (((uintptr_t)W & 15)) return ENSVS_E_ARG;
  dim3 grid(cdiv(a.M, BM), Npad / BN);
  const bool has_pd = segs[0].pd != nullptr;
  for (int s = 0; s < nseg; ++s) {  // 32-bit element offsets inside the kernel
    const ensvs_conv_seg& g = segs[s];
    if ((long long)B * g.Tin * g.ld >= (1ll << 31) ||
        (long long)g.taps * Npad * g.Kp >= (1ll << 30))
      return ENSVS_E_SHAPE;
  }
  if (!has_pd && use_p8(a, segs, nseg, B)) {
    const dim3 grid_b(cdiv(a.M, BMB), Npad / BNB);
    const bool gate = a.gate8 && (a.epi == EPI_GATE || a.epi == EPI_GATE_TS);
    const size_t lb = (size_t)2 * P8_BUF;  // two K-steps of both images (128 KB)
    const bool plain = p8_plain(a);
    const size_t lbp = std::max<size_t>(lb, (size_t)128 * EPB * 4);  // two 128-row passes
#define P8(E, B2, L)                                                                      \
  do {                                                                                    \
    static const hipError_t ep = hipFuncSetAttribute(                                     \
        (const void*)conv_gemm_b16_p8_kernel<E, B2>,                                      \
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(L));                            \
    if (ep != hipSuccess) return ENSVS_E_HIP;                                             \
    hipLaunchKernelGGL((conv_gemm_b16_p8_kernel<E, B2>), grid_b, dim3(NTHRB), (L), st, a); \
  } while (0)
    if (a.epi == EPI_NONE && g_p8_nodma == 2) {
      P8(P8_PROBE_NOMMA, true, lb);
    } else if (a.epi == EPI_NONE && g_p8_nodma) {
      P8(P8_PROBE_NODMA, true, lb);
    } else if (g_p8_bar2) {
      if (gate) P8(EPI_GATE, true, lb);
      else if (plain) P8(EPI_PLAIN, true, lbp);
      else P8(-1, true, lbp);
    } else {
      if (gate) P8(EPI_GATE, false, lb);
      else if (plain) P8(EPI_PLAIN, false, lbp);
      else P8(-1, false, lbp);
    }
#undef P8
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  if (!has_pd && use_p8h(a, segs, nseg, B)) {
    const dim3 grid_h(cdiv(a.M, BMH), Npad / BNB);
    const bool plain = a.epi == EPI_PLAIN && !a.accum && !a.relu && !a.ybf && !a.csum && a.Y &&
                       a.N % 4 == 0 && a.ldy % 4 == 0 && ((uintptr_t)a.Y & 15) == 0 &&
                       (!a.bias || ((uintptr_t)a.bias & 3) == 0);
    const size_t lh = std::max<size_t>(P8H_LDS, plain ? (size_t)BMH * EPB * 4 : P8H_LDS_EPI);
#define P8H(E)                                                                            \
  do {                                                                                    \
    static const hipError_t eh = hipFuncSetAttribute(                                     \
        (const void*)conv_gemm_b16_p8h_kernel<E>,                                         \
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lh);                             \
    if (eh != hipSuccess) return ENSVS_E_HIP;                                             \
    hipLaunchKernelGGL((conv_gemm_b16_p8h_kernel<E>), grid_h, dim3(NTHRB), lh, st, a);    \
  } while (0)
    if (plain) P8H(EPI_PLAIN);
    else if (a.epi == EPI_PLAIN) P8H(16 + EPI_PLAIN);
    else if (a.epi == EPI_ADDSCALE) P8H(EPI_ADDSCALE);
    else if (a.epi == EPI_GATE_BWD) P8H(EPI_GATE_BWD);
    else if (a.epi == EPI_RELU_MASK) P8H(EPI_RELU_MASK);
    else P8H(-1);
#undef P8H
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  if (!has_pd && use_big_tile(a)) {
    const dim3 grid_b(cdiv(a.M, BMB), Npad / BNB);
    if (g_big_tile == 2) {
      const bool gate = a.gate8 && (a.epi == EPI_GATE || a.epi == EPI_GATE_TS);
#define BIG(G)                                                                            \
  do {                                                                                    \
    const size_t lb = (size_t)2 * (BMB + BNB) * BK2 * 2;  /* two stages of both images */ \
    static const hipError_t eb = hipFuncSetAttribute(                                     \
        (const void*)conv_gemm_b16_big_kernel<G>, hipFuncAttributeMaxDynamicSharedMemorySize, \
        (int)lb);                                                                         \
    if (eb != hipSuccess) return ENSVS_E_HIP;                                             \
    hipLaunchKernelGGL(conv_gemm_b16_big_kernel<G>, grid_b, dim3(NTHRB), lb, st, a);      \
  } while (0)
      if (gate) BIG(true);
      else BIG(false);
#undef BIG
    } else {
#define RING(S)                                                                           \
  do {                                                                                    \
    const size_t lr = std::max<size_t>((size_t)(S) * 2 * BMB * BK3 * 2,                   \
                                       (size_t)CHR * EPB * 4);                            \
    static const hipError_t er = hipFuncSetAttribute(                                     \
        (const void*)conv_gemm_b16_ring_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize, \
        (int)lr);                                                                         \
    if (er != hipSuccess) return ENSVS_E_HIP;                                             \
    hipLaunchKernelGGL(conv_gemm_b16_ring_kernel<S>, grid_b, dim3(NTHRB), lr, st, a);     \
  } while (0)
      if (g_big_stages == 3) RING(3);
      else if (g_big_stages == 4) RING(4);
      else RING(5);
#undef RING
    }
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  // small M (fewer than 128 tiles of 128 x 128): the 64 x 64-tile kernel fills the chip; it
  // also takes N <= 64 at any M (a 128-wide tile would leave half its columns and half the
  // epilogue threads idle: the uSFGAN block output GEMMs, 480 000 x 64)
  if (g_small && !has_pd && !a.csum && a.vec_out && Npad % BNS == 0 &&
      ((long long)grid.x * grid.y < 128 || a.N <= BNS ||
       (g_small == 2 && Npad <= 2 * BNS && (long long)grid.x * grid.y < 256))) {
    constexpr int sms = SMALL_STAGES;
    const dim3 gs(cdiv(a.M, BMS), a.N <= BNS ? 1 : Npad / BNS);
#define SMALL(S)                                                                          \
  do {                                                                                    \
    const size_t ls = std::max<size_t>((size_t)(S) * 2 * BMS * BK2 * 2, (size_t)BMS * EPS * 4); \
    static const hipError_t es = hipFuncSetAttribute(                                     \
        (const void*)conv_gemm_b16_small_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize, \
        (int)ls);                                                                         \
    if (es != hipSuccess) return ENSVS_E_HIP;                                             \
    hipLaunchKernelGGL(conv_gemm_b16_small_kernel<S>, gs, dim3(NTHR), ls, st, a);         \
  } while (0)
    if (sms == 3) SMALL(3);
    else if (sms == 4) SMALL(4);
    else SMALL(5);
#undef SMALL
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  // small M: split K over up to 8 workgroups per output tile so the launch fills the chip
  // (a 2 000-frame DiffNet GEMM is 64 tiles of 128 x 128; each tile's 16 K-steps would run
  // serially on one CU).  Needs a caller workspace for ksplit x M x Npad fp32 partials.
  if (!has_pd && a.part && !a.csum && a.vec_out && a.epi != EPI_NONE) {
    const long long tiles = (long long)grid.x * grid.y;
    int nit = 0;
    for (int s = 0; s < nseg; ++s) nit += cdiv(segs[s].K, BK2) * segs[s].taps;
    int S = (int)std::min<long long>(8, (SPLITK_TARGET + tiles - 1) / tiles);
    S = std::min(S, nit / 2);
    while (S > 1 && (long long)S * a.M * Npad > a.part_floats) --S;
    if (S > 1 && tiles < SPLITK_TARGET / 2) a.ksplit = S;
  }
  const size_t lds = (size_t)2 * BM * BK2 * 2;  // one stage (A + B images)
  // the LDS-staged epilogue reuses the stage buffers for the fp32 output tile
  const size_t l2 = std::max<size_t>(2 * lds, EPI_LDS), l3 = std::max<size_t>(3 * lds, EPI_LDS);
  if (a.ksplit > 1) grid.z = a.ksplit;
  if (g_dual_small && !has_pd && a.ksplit <= 1 && !a.csum &&
      (long long)grid.x * grid.y < 128) {
    const size_t ld2 = std::max<size_t>(4 * lds, EPI_LDS);  // 2 stages x 2 K-groups
    static const hipError_t ed = hipFuncSetAttribute(
        (const void*)conv_gemm_b16_dual_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)ld2);
    if (ed != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL(conv_gemm_b16_dual_kernel, grid, dim3(NTHR2), ld2, st, a);
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  const bool spec = stages == 2 && a.ksplit <= 1 && a.vec_out;
#define SPEC(E)                                                                                \
  do {                                                                                         \
    static const hipError_t es = hipFuncSetAttribute((const void*)conv_gemm_b16_kernel<2, E>, \
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                     (int)l2);                                 \
    if (es != hipSuccess) return ENSVS_E_HIP;                                                  \
    hipLaunchKernelGGL((conv_gemm_b16_kernel<2, E>), grid, dim3(NTHR), l2, st, a);             \
  } while (0)
  if (spec && a.gbw_dma) {
    SPEC(EPI_GATE_BWD);
  } else if (spec && a.as_dma) {
    SPEC(EPI_ADDSCALE + 16);
  } else if (spec && a.epi == EPI_RESSKIP) {
    SPEC(EPI_RESSKIP);
  } else if (spec && a.epi == EPI_ADDSCALE) {
    SPEC(EPI_ADDSCALE);
  } else if (stages == 2) {
    static const hipError_t e2 = hipFuncSetAttribute((const void*)conv_gemm_b16_kernel<2>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)l2);
    if (e2 != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL(conv_gemm_b16_kernel<2>, grid, dim3(NTHR), l2, st, a);
  } else if (stages == 3) {
    static const hipError_t e3 = hipFuncSetAttribute((const void*)conv_gemm_b16_kernel<3>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)l3);
    if (e3 != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL(conv_gemm_b16_kernel<3>, grid, dim3(NTHR), l3, st, a);
  } else {
    return ENSVS_E_ARG;
  }
#undef SPEC
  ENSVS_CHECK_LAUNCH();
  if (a.ksplit > 1) {
    const size_t le = (size_t)CHR * EPB * 4;
    static const hipError_t ee = hipFuncSetAttribute(
        (const void*)splitk_epilogue_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)le);
    if (ee != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(cdiv(a.M, CHR), cdiv(Npad, BNB)),
                       dim3(NTHRB), le, st, a);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_small(int on) {
  g_small = on == 2 ? 2 : on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_dual_small(int on) {
  g_dual_small = on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_wgrad_big(int on) {
  g_wgrad_big = on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_gbw_dma(int on) {
  g_gbw_dma = on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_p8(int mode) {
  if (mode < 0 || mode > 31) return ENSVS_E_ARG;
  g_p8 = mode & 3;
  g_p8_bar2 = (mode & 4) ? 1 : 0;  // bit 2: two barriers per phase, rows staggered
  // bit 3: EPI_NONE probes without the K loop's loads; bit 4: without its MFMAs
  g_p8_nodma = (mode & 16) ? 2 : ((mode & 8) ? 1 : 0);
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_p8_min_tiles(int n) {
  if (n < 1) return ENSVS_E_ARG;
  g_p8_min_tiles = n;
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_p8h(int mode) {
  if (mode < 0 || mode > 3 + 4 * 64) return ENSVS_E_ARG;
  g_p8h = mode & 3;
  if (mode >> 2) g_p8h_min_ksteps = mode >> 2;  // + 4 k: lean plain launches of >= k K-steps
  return ENSVS_OK;
}

ENSVS_API int ensvs_set_big_tile(int mode, int stages) {
  if (mode < 0 || mode > 3 || (stages != 0 && (stages < 3 || stages > 5))) return ENSVS_E_ARG;
  g_big_all = mode == 3;
  if (mode == 3) mode = 2;
  g_big_tile = mode;
  if (stages) g_big_stages = stages;
  return ENSVS_OK;
}

ENSVS_API int ensvs_conv_gemm_bf16a(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N,
                                    int Npad, const void* W, const float* bias, float* Y, int ldy,
                                    int epi, int relu, int accum, float* aux0, int ld0,
                                    const float* aux1, int ld1, float alpha, int C, int stages,
                                    float* part, long long part_floats, void* stream) {
  GemmArgs a{};
  const int rc = fill_gemm_args(a, segs, nseg, B, Tout, N, Npad, W, bias, Y, ldy, epi, relu,
                                accum, aux0, ld0, aux1, ld1, alpha, C);
  if (rc != ENSVS_OK) return rc;
  a.part = part;
  a.part_floats = part ? part_floats : 0;
  return launch_b16(a, segs, nseg, B, Npad, W, stages, (hipStream_t)stream);
}

// ensvs_conv_gemm_bf16a plus a bf16 copy of the output for the next GEMM (see GemmArgs::ybf).
// Only the 16-B LDS-staged epilogue writes it: output rows must be 16-B aligned with
// ld % 4 == 0 (and N % 4 == 0, C % 4 == 0), ybf rows 8-B aligned with ybf_ld % 4 == 0.
ENSVS_API int ensvs_conv_gemm_bf16a_out(const ensvs_conv_seg* segs, int nseg, int B, int Tout,
                                        int N, int Npad, const void* W, const float* bias,
                                        float* Y, int ldy, int epi, int relu, int accum,
                                        float* aux0, int ld0, const float* aux1, int ld1,
                                        float alpha, int C, void* ybf, int ybf_ld,
                                        const float* ybf_radd, int ybf_radd_ld, float* csum,
                                        int csum_ld, int stages, float* part,
                                        long long part_floats, void* stream) {
  GemmArgs a{};
  const int rc = fill_gemm_args(a, segs, nseg, B, Tout, N, Npad, W, bias, Y, ldy, epi, relu,
                                accum, aux0, ld0, aux1, ld1, alpha, C);
  if (rc != ENSVS_OK) return rc;
  a.part = part;
  a.part_floats = part ? part_floats : 0;
  if (csum) {
    if (!a.vec_out || a.M % BM || N % 4 || csum_ld < (a.epi == EPI_GATE_BWD ? 2 * C : N) ||
        (a.epi != EPI_PLAIN && a.epi != EPI_ADDSCALE && a.epi != EPI_RELU_MASK &&
         a.epi != EPI_GATE_BWD))
      return ENSVS_E_ARG;
    a.csum = csum;
    a.csum_ld = csum_ld;
  }
  // Y may be dropped where the epilogue's other outputs are all the caller needs
  if (!Y && !(((a.epi == EPI_GATE || a.epi == EPI_GATE_TS) && ybf) ||
              (a.epi == EPI_GATE_BWD && (ybf || csum))))
    return ENSVS_E_ARG;
  if (ybf) {
    if (!a.vec_out || N % 4 || ybf_ld % 4 || ((uintptr_t)ybf & 7) ||
        (ybf_radd && (ybf_radd_ld % 4 || ((uintptr_t)ybf_radd & 15))))
      return ENSVS_E_ARG;
    a.ybf = (__bf16*)ybf;
    a.ybf_ld = ybf_ld;
    a.ybf_radd = ybf_radd;
    a.ybf_radd_ld = ybf_radd_ld;
    a.gate8 = a.gate8 && ((uintptr_t)ybf & 15) == 0 && ybf_ld % 8 == 0;
  }
  a.gbw_dma = g_gbw_dma && a.epi == EPI_GATE_BWD && a.aux1_bf && a.ybf && !a.Y && !a.bias &&
              !a.ybf_radd && C % BN == 0 && a.M % BM == 0 && ((uintptr_t)aux1 & 15) == 0 &&
              ld1 % 8 == 0 && ((uintptr_t)ybf & 15) == 0 && ybf_ld % 8 == 0;
  a.as_dma = g_gbw_dma && a.epi == EPI_ADDSCALE && !a.aux1_bf && a.Y && a.ybf && !a.ybf_radd &&
             !a.relu && N % BN == 0 && a.M % BM == 0 && ((uintptr_t)aux1 & 15) == 0 &&
             ld1 % 4 == 0 && ((uintptr_t)Y & 15) == 0 && ldy % 4 == 0 &&
             ((uintptr_t)ybf & 7) == 0 && ybf_ld % 4 == 0 && (!a.bias || ((uintptr_t)a.bias & 15) == 0);
  return launch_b16(a, segs, nseg, B, Npad, W, stages, (hipStream_t)stream);
}

// One uSFGAN residual block (usfgan/layers/residual_block.py: gated dilated / pitch-dependent
// conv + aux conv, tanh * sigmoid, 1x1 output conv, (x + out) / sqrt 2) as one launch of
// usf_block_kernel: segs = the gate GEMM's bf16 segments (x's copy, taps 3, optional pd; the
// aux features' copy), W packed bf16 ([2C = 128 gate/filter columns interleaved by 16] and
// the output conv at wofs2 as [Npad >= 64][Kp2 = 64]); x [M][ldx] fp32 updated in place,
// xb its bf16 copy (optional).  Same bits as the two-GEMM path with a bf16 z copy.
ENSVS_API int ensvs_usf_block(const ensvs_conv_seg* segs, int nseg, int B, int Tout,
                              const void* W, const float* bias1, int C, long long wofs2, int Kp2,
                              const float* bias2, float* x, int ldx, float alpha, int relu,
                              void* xb, int xb_ld, void* stream) {
  if (C != 64 || Kp2 != 64 || nseg < 1) return ENSVS_E_SHAPE;
  GemmArgs a{}, a2{};
  int rc = fill_gemm_args(a, segs, nseg, B, Tout, 2 * C, BN, W, bias1, nullptr, 0, EPI_GATE_TS, 0,
                          0, nullptr, 0, nullptr, 0, 0.f, C);
  if (rc != ENSVS_OK) return rc;
  ensvs_conv_seg z{};
  z.x = x;
  z.ld = C;
  z.K = C;
  z.taps = 1;
  z.dil = 1;
  z.pad = PAD_ZERO;
  z.Tin = Tout;
  z.Kp = Kp2;
  z.wofs = wofs2;
  rc = fill_gemm_args(a2, &z, 1, B, Tout, 64, BN, W, bias2, x, ldx, EPI_ADDSCALE, relu, 0, nullptr,
                      0, x, ldx, alpha, C);
  if (rc != ENSVS_OK) return rc;
  if (!a2.vec_out || ((uintptr_t)W & 15)) return ENSVS_E_ARG;
  if (xb) {
    if (xb_ld % 4 || ((uintptr_t)xb & 7)) return ENSVS_E_ARG;
    a2.ybf = (__bf16*)xb;
    a2.ybf_ld = xb_ld;
  }
  for (int s = 0; s < nseg; ++s) {  // the bf16 operand contract of launch_b16
    const ensvs_conv_seg& g = segs[s];
    if (g.radd || g.ld % 8 || g.ld < ((g.K + 7) & ~7) || ((uintptr_t)g.x & 15))
      return ENSVS_E_ARG;
    if ((long long)B * g.Tin * g.ld >= (1ll << 31) || (long long)g.taps * BN * g.Kp >= (1ll << 30))
      return ENSVS_E_SHAPE;
  }
  const size_t lds = (size_t)2 * 2 * BM * BK2 * 2;  // two stages of both images (64 KB)
  static const hipError_t e = hipFuncSetAttribute(
      (const void*)usf_block_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(usf_block_kernel, dim3(cdiv(a.M, BM), 1), dim3(NTHR), lds,
                     (hipStream_t)stream, a, a2);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// The column sums of GemmArgs::csum for a Y written by any other path, in the same order:
// per BM-row tile and column, the 8 row groups g (rows g, g+8, ..) each summed in row order,
// then the group sums added in order.
__global__ __launch_bounds__(BN) void tile_colsum_kernel(const float* __restrict__ y, int ldy,
                                                         int N, float* __restrict__ out,
                                                         int ldo) {
  const int m0 = blockIdx.x * BM, n = blockIdx.y * BN + threadIdx.x;
  if (n >= N) return;
  float t = 0.f;
  for (int g = 0; g < CS_GROUPS; ++g) {
    float s = 0.f;
    for (int r = g; r < BM; r += CS_GROUPS) s += y[(long long)(m0 + r) * ldy + n];
    t = g ? t + s : s;
  }
  out[(long long)blockIdx.x * ldo + n] = t;
}

ENSVS_API int ensvs_tile_colsum(const float* y, int ldy, int M, int N, float* out, int ldo,
                                void* stream) {
  if (M <= 0 || N <= 0) return ENSVS_OK;
  if (M % BM || ldo < N) return ENSVS_E_ARG;
  hipLaunchKernelGGL(tile_colsum_kernel, dim3(M / BM, cdiv(N, BN)), dim3(BN), 0,
                     (hipStream_t)stream, y, ldy, N, out, ldo);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_cast_bf16(const float* x, int ldx, const float* radd, int radd_ld, int T,
                              long long M, int K, void* y, int ldy, void* stream) {
  if (M <= 0 || K <= 0) return ENSVS_OK;
  if (K % 8 && !radd) {  // zero-padded copy (a K % 8 != 0 operand of the bf16 kernels)
    const int K8 = (K + 7) / 8;
    if (ldy % 8 || ldy < 8 * K8 || ldx < K || ((uintptr_t)y & 15)) return ENSVS_E_ARG;
    const long long n = M * K8;
    const int blocks = (int)std::min<long long>(8192, (n + 255) / 256);
    hipLaunchKernelGGL(cast_bf16_pad_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x,
                       ldx, M, K, K8, (__bf16*)y, ldy);
    ENSVS_CHECK_LAUNCH();
    return ENSVS_OK;
  }
  if (K % 8 || ldx % 4 || ldy % 8 || (radd && (radd_ld % 4 || T <= 0)) ||
      (((uintptr_t)x | (uintptr_t)y | (uintptr_t)radd) & 15))
    return ENSVS_E_ARG;
  const long long n = M * (K / 8);
  const int blocks = (int)std::min<long long>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     radd, radd_ld, T, M, K, (__bf16*)y, ldy);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// Weight gradient of a conv/linear: dst[n*sn + k*sk + j*sj] (+)= sum_m dY[m,n] X[src(m,j),k].
// `part` must hold splits*taps*N*K floats.
ENSVS_API int ensvs_conv_wgrad(const float* dy, int ldy, const float* x, int ldx, const float* radd,
                               int radd_ld, int B, int Tout, int Tin, int N, int K, int taps, int dil,
                               int shift0, int pad, int splits, float* part, float* dst,
                               long long sn, long long sk, long long sj, int accum, float scale,
                               int dtype, void* stream) {
  const int defer = accum;  // ENSVS_WGRAD_DEFER: partials only
  accum &= 1;
  if (B <= 0 || Tout <= 0 || N <= 0 || K <= 0 || taps <= 0 || splits <= 0) return ENSVS_E_SHAPE;
  WgradArgs a{};
  a.dy = dy;
  a.x = x;
  a.radd = radd;
  a.part = part;
  a.ldy = ldy;
  a.ldx = ldx;
  a.K = K;
  a.taps = taps;
  a.dil = dil;
  a.shift0 = shift0;
  a.pad = pad;
  a.Tin = Tin;
  a.radd_ld = radd_ld;
  a.Tout = Tout;
  a.M = B * Tout;
  a.N = N;
  a.splits = splits;
  a.rows_per_split = (cdiv(a.M, splits) + BK - 1) / BK * BK;
  a.vecy = (N % 4 == 0) && (ldy % 4 == 0) && (((uintptr_t)dy & 15) == 0);
  a.vecx = (K % 4 == 0) && (ldx % 4 == 0) && (((uintptr_t)x & 15) == 0) &&
           (!radd || ((radd_ld % 4 == 0) && (((uintptr_t)radd & 15) == 0)));
  const bool vec = a.vecy && a.vecx;
  a.dst = dst;
  a.sn = sn;
  a.sk = sk;
  a.sj = sj;
  a.scale = scale;
  a.accum = accum;
  dim3 grid(cdiv(N, BM), cdiv(K, BN), taps * splits);
  if (N * taps > 65535) return ENSVS_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DT_BF16) {
    size_t lds = 2 * 2 * BK * 256;
    // (with radd the ring's extra registers spill: that rare case keeps one chunk in flight)
    if (vec && !radd)
      hipLaunchKernelGGL((wgrad_f32r_kernel<false>), grid, dim3(NTHR), lds, st, a);
    else if (vec)
      hipLaunchKernelGGL((wgrad_kernel<__bf16, true>), grid, dim3(NTHR), lds, st, a);
    else
      hipLaunchKernelGGL((wgrad_kernel<__bf16, false>), grid, dim3(NTHR), lds, st, a);
  } else {
    size_t lds = 2 * (BM + BN) * Lds<float>::K * sizeof(float);
    if (vec)
      hipLaunchKernelGGL((wgrad_kernel<float, true>), grid, dim3(NTHR), lds, st, a);
    else
      hipLaunchKernelGGL((wgrad_kernel<float, false>), grid, dim3(NTHR), lds, st, a);
  }
  ENSVS_CHECK_LAUNCH();
  if (splits > 1 && !(defer & ENSVS_WGRAD_DEFER)) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv_ll((long long)N * taps * K, 256)),
                       dim3(256), 0, st, part, dst, splits, taps, N, K, sn, sk, sj, accum, scale);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}


// Weight gradient with bf16 operands (dy, x rounded to bf16 in HBM; radd folded into x).
ENSVS_API int ensvs_conv_wgrad_bf16(const void* dy, int ldy, const void* x, int ldx, int B,
                                    int Tout, int Tin, int N, int K, int taps, int dil, int shift0,
                                    int pad, int splits, float* part, float* dst, long long sn,
                                    long long sk, long long sj, int accum, float scale,
                                    void* stream) {
  const int defer = accum;  // ENSVS_WGRAD_DEFER: partials only
  accum &= 1;
  if (B <= 0 || Tout <= 0 || N <= 0 || K <= 0 || taps <= 0 || splits <= 0) return ENSVS_E_SHAPE;
  // K (N) % 8 != 0: the last 16-B chunk of an x (dy) row reads up to K (N) rounded to 8, the
  // caller's zero padding (stores check k < K, n < N)
  if (ldy % 8 || ldy < (N + 7) / 8 * 8 || ldx % 8 || ldx < (K + 7) / 8 * 8 ||
      (((uintptr_t)dy | (uintptr_t)x) & 15))
    return ENSVS_E_ARG;
  WgradArgs a{};
  a.dy = (const float*)dy;
  a.x = (const float*)x;
  a.part = part;
  a.ldy = ldy;
  a.ldx = ldx;
  a.K = K;
  a.taps = taps;
  a.dil = dil;
  a.shift0 = shift0;
  a.pad = pad;
  a.Tin = Tin;
  a.Tout = Tout;
  a.M = B * Tout;
  a.N = N;
  a.splits = splits;
  a.rows_per_split = (cdiv(a.M, splits) + BK - 1) / BK * BK;
  a.dst = dst;
  a.sn = sn;
  a.sk = sk;
  a.sj = sj;
  a.scale = scale;
  a.accum = accum;
  if (N * taps > 65535) return ENSVS_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (wgrad_big_shape(N, K, taps)) {
    const size_t lds = WNS * 4 * BK * 256;
    static const hipError_t e = hipFuncSetAttribute(
        (const void*)wgrad_b16_big_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL(wgrad_b16_big_kernel, dim3(cdiv(N, WGB), cdiv(K, WGB), taps * splits),
                       dim3(NTHRW), lds, st, a);
  } else {
    dim3 grid(cdiv(N, BM), cdiv(K, BN), taps * splits);
    hipLaunchKernelGGL(wgrad_b16_kernel, grid, dim3(NTHR), WNS * 2 * BK * 256, st, a);
  }
  ENSVS_CHECK_LAUNCH();
  if (splits > 1 && !(defer & ENSVS_WGRAD_DEFER)) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv_ll((long long)N * taps * K, 256)),
                       dim3(256), 0, st, part, dst, splits, taps, N, K, sn, sk, sj, accum, scale);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

ENSVS_API int ensvs_wgrad_reduce_batch(const ensvs_wred_desc* descs, int n, void* stream) {
  if (n < 0 || (n > 0 && !descs)) return ENSVS_E_ARG;
  for (int i0 = 0; i0 < n; i0 += WRED_BATCH) {
    const int m = std::min(WRED_BATCH, n - i0);
    WredBatch b{};
    long long most = 0;
    for (int i = 0; i < m; ++i) {
      const ensvs_wred_desc& d = descs[i0 + i];
      if (!d.part || !d.dst || d.splits < 1 || d.taps < 1 || d.N < 1 || d.K < 1)
        return ENSVS_E_ARG;
      b.d[i] = d;
      most = std::max(most, (long long)d.N * d.K * d.taps);
    }
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((unsigned)cdiv_ll(most, 256), m),
                       dim3(256), 0, (hipStream_t)stream, b);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

// the split count ensvs_colsum picks for one group (>= ~2048 blocks, >= 128 rows per split)
static int colsum_splits(int M, int N, int groups, int max_splits) {
  return std::max(1, std::min({max_splits, M / 128, cdiv(2048, cdiv(N, 64) * groups)}));
}

ENSVS_API long long ensvs_colsum_batch_part_floats(const ensvs_colsum_desc* descs, int n) {
  long long t = 0;
  for (int i = 0; i < n; ++i)
    t += (long long)colsum_splits(descs[i].M, descs[i].N, 1, descs[i].max_splits) * descs[i].N;
  return t;
}

ENSVS_API int ensvs_colsum_batch(const ensvs_colsum_desc* descs, int n, float* part,
                                 long long part_floats, void* stream) {
  if (n < 0 || (n > 0 && (!descs || !part))) return ENSVS_E_ARG;
  if (part_floats < ensvs_colsum_batch_part_floats(descs, n)) return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  long long off = 0;
  for (int i0 = 0; i0 < n; i0 += CS_BATCH) {
    const int m = std::min(CS_BATCH, n - i0);
    CsBatch b{};
    int most_cb = 1, most_s = 1, most_c16 = 1;
    for (int i = 0; i < m; ++i) {
      const ensvs_colsum_desc& e = descs[i0 + i];
      if (!e.y || !e.out || e.M <= 0 || e.N <= 0 || e.ld < e.N || e.max_splits < 1)
        return ENSVS_E_ARG;
      CsDesc& d = b.d[i];
      d.y = e.y;
      d.out = e.out;
      d.ld = e.ld;
      d.M = e.M;
      d.N = e.N;
      d.S = colsum_splits(e.M, e.N, 1, e.max_splits);
      d.rps = cdiv(e.M, d.S);
      d.vec = (e.ld % 4 == 0) && (((uintptr_t)e.y & 15) == 0);
      d.part_off = off;
      d.scale = e.scale;
      d.accum = e.accum;
      off += (long long)d.S * e.N;
      most_cb = std::max(most_cb, cdiv(e.N, 64));
      most_s = std::max(most_s, d.S);
      most_c16 = std::max(most_c16, cdiv(e.N, 16));
    }
    hipLaunchKernelGGL(colsum_partial_batch_kernel, dim3(most_cb, most_s, m), dim3(256), 0, st,
                       b, part);
    ENSVS_CHECK_LAUNCH();
    hipLaunchKernelGGL(colsum_final_batch_kernel, dim3(most_c16, m), dim3(256), 0, st, b, part);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

// Batched weight repack: `descs` is a DEVICE array of `n` descriptors.
ENSVS_API int ensvs_pack_weights(const ensvs_pack_desc* descs, int n, int max_elems, void* stream) {
  static_assert(sizeof(ensvs_pack_desc) == sizeof(PackDesc), "desc layout");
  if (n <= 0) return ENSVS_OK;
  int bx = std::min(1024, std::max(1, (max_elems + 255) / 256));
  hipLaunchKernelGGL(pack_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream,
                     (const PackDesc*)descs);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_pack_weights_tiled(const ensvs_pack_desc* descs, int n, int tiles,
                                       void* stream) {
  if (n <= 0 || tiles <= 0) return ENSVS_OK;
  if (!descs) return ENSVS_E_ARG;
  hipLaunchKernelGGL(pack_tile_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream,
                     (const PackDesc*)descs, n);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

// out[g][n] (+)= scale * sum_{m < M} f(Y[g*M + m, n]) for g < groups;
// f = identity, or (y - mean[g][n])^2 when mean != null.  `part` holds groups*max_splits*N floats.
ENSVS_API int ensvs_colsum_once(const float* y, int ld, int M, int groups, int N,
                                const float* mean, float scale, float* part, int max_splits,
                                unsigned* counters, float* out, int ldo, int accum, void* stream) {
  if (M <= 0 || N <= 0 || groups <= 0) return ENSVS_E_SHAPE;
  if (!counters || !part || !out) return ENSVS_E_ARG;
  const int cb = cdiv(N, 64);  // the split count ensvs_colsum picks
  int S = std::max(1, std::min({max_splits, M / 128, cdiv(2048, cb * groups)}));
  int rps = cdiv(M, S);
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (ld % 4 == 0) && (((uintptr_t)y & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(colsum_once_kernel<true>, dim3(cb, S, groups), dim3(256), 0, st, y, ld, M,
                       N, rps, mean, part, counters, scale, out, ldo > 0 ? ldo : N, accum);
  else
    hipLaunchKernelGGL(colsum_once_kernel<false>, dim3(cb, S, groups), dim3(256), 0, st, y, ld, M,
                       N, rps, mean, part, counters, scale, out, ldo > 0 ? ldo : N, accum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_colsum(const float* y, int ld, int M, int groups, int N, const float* mean,
                           float scale, float* part, int max_splits, float* out, int ldo, int accum,
                           void* stream) {
  if (M <= 0 || N <= 0 || groups <= 0) return ENSVS_E_SHAPE;
  // aim for >= ~2048 blocks (8 XCDs x 32 CUs x several waves), >= 128 rows per split
  const int cb = cdiv(N, 64);
  int S = std::max(1, std::min({max_splits, M / 128, cdiv(2048, cb * groups)}));
  int rps = cdiv(M, S);
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (ld % 4 == 0) && (((uintptr_t)y & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3(cb, S, groups), dim3(256), 0, st, y, ld,
                       M, N, rps, mean, part);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3(cb, S, groups), dim3(256), 0, st, y, ld,
                       M, N, rps, mean, part);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(N, 16), groups), dim3(256), 0, st, part, S, N,
                     scale, out, ldo > 0 ? ldo : N, accum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
