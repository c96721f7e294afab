// Batched MFMA bidirectional LSTM recurrence for H = 64 / 128 (the FFConvLSTM encoders of the
// lf0 / mgc / bap / vuv streams, nnsvs/model.py:862-869, 914-916, and the multi-track lf0
// encoder, acoustic_models/tacotron_f0.py:876-883) in production (bf16 GEMM) precision.
//
// Same contract as lstm.hip's ensvs_lstm_fwd / ensvs_lstm_bwd (packed sequences, zero state,
// zero outputs past each length, saved [B*T][2][5H] = i f g o c).  lstm.hip runs one
// workgroup per (sequence, direction) and spends the step on fp32 VALU dot products: 60
// workgroups for the bench's 30 sequences, 0.5 / 0.6 us per step at H = 64, 0.76 / 1.19 at
// H = 128.  Here one workgroup per (group of S sequences, direction) holds the direction's
// whole W_hh as MFMA fragments in VGPRs (fp16 forward: h in [-1, 1]; bf16 backward: dG spans
// many decades -- as the reference recipe's fp16 autocast runs its cuDNN LSTM,
// myconfig_notuseIL.yaml:6), the S sequences are the MFMA N columns, and h (fp16) / dG (bf16)
// is exchanged through a double-buffered LDS image: one workgroup barrier per step, nothing
// between workgroups.  Gates, cell state, saved values and the outputs stay fp32; the fp32
// parity mode keeps lstm.hip's exact kernels.
//
// S = 16 / KS.  With KS = 2 (8 sequences) the 16 MFMA columns are 8 sequences x 2 halves of
// the K chunks (column n reads sequence n % 8 and only chunks kk with kk % 2 == n / 8; the
// other half reads a zero row), the halves are added across lanes n and n + 8 (DPP row_ror 8)
// and each lane applies the cell to half of the values: the same MFMA count, half the cell
// work and half the global traffic per workgroup, twice the workgroups.
//
// Forward: wave v owns units [v H/4, (v+1) H/4) = NMT = H/16 tiles of 16 gate rows; row m of
// tile mt is gate m % 4 of unit v H/4 + (m / 4) NMT + mt, so the four C values a lane holds
// (rows 4 (lane / 16) + r) are the four gates of one unit and lane (lg, n) applies the cell
// to the contiguous units v H/4 + lg NMT + sp NC + i (sp = n / S, NC = NMT / KS cells).
// Backward: dh = W_hh^T dG with the units as M (H/64 tiles per wave) and K = 4H in the dG
// image's order n' = 4 unit + gate; lane (lg, n) handles units v H/4 + lg 4 TPW + sp NCB + i.
// Both packs are independent of KS.
//
// Inputs of step t + D are loaded into registers at step t (D-step register pipeline); every
// load and store of a step is a 16-B (NC >= 4) vector access of contiguous units.
#include "coop.h"
#include "ensvs.h"

#ifndef LB_DBG
#define LB_DBG 0
#endif
namespace {

using coop::sigm;
using coop::tanh_fast;

constexpr int NT = 256;

template <int H, int KS> struct BGeo {
  static constexpr int S = 16 / KS;         // sequences per workgroup
  static constexpr int UPW = H / 4;         // units per wave
  static constexpr int NMT = H / 16;        // forward M tiles per wave (4 gate rows per unit)
  static constexpr int KCF = H == 64 ? 16 : 32;  // forward K per MFMA (16x16x16 at H = 64, so
                                                 // that a 4-way K split has a chunk per part)
  static constexpr int NKC = H / KCF;       // forward K chunks (K = H)
  static constexpr int NC = NMT / KS;       // forward cells (units) per lane
  static constexpr int TPW = H / 64;        // backward M tiles per wave (units)
  static constexpr int NKB = H / 8;         // backward K chunks (K = 4H)
  static constexpr int NCB = TPW * 4 / KS;  // backward cells per lane
  static constexpr int HP = H + 8;          // fp16 h row in LDS (halves; bank padding)
  static constexpr int GP = 4 * H + 8;      // bf16 dG row in LDS
  static_assert(NC >= 1 && NCB >= 1 && NKC % KS == 0 && NMT % KS == 0, "cells");
};

template <int N>
__device__ __forceinline__ void vld(float (&d)[N], const float* p) {
  if constexpr (N == 2) {
    const f32x2 v = *(const f32x2*)p;
    d[0] = v.x;
    d[1] = v.y;
  } else {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      const f32x4 v = *(const f32x4*)(p + k);
      d[k] = v[0]; d[k + 1] = v[1]; d[k + 2] = v[2]; d[k + 3] = v[3];
    }
  }
}
// Stores go through a buffer resource over the whole output: a lane whose sequence has ended
// passes an offset past the end and the hardware drops its store.  No branch around the
// stores, so the waitcnt pass keeps exact counts for the register pipeline of the loads
// (with an exec-masked store block it falls back to vmcnt(0) every step).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// 2^31 (an offset past every output: sizes are checked below 2^31 bytes) when step t is past
// the sequence end, else 0 -- arithmetic, not a select, which the compiler turns back into an
// exec-masked branch around the store
__device__ __forceinline__ unsigned oob(int t, int L) {
  return ((unsigned)(L - 1 - t) >> 31) << 31;
}
template <int N>
__device__ __forceinline__ void vst(__amdgpu_buffer_rsrc_t r, unsigned off, const float (&s)[N]) {
  if constexpr (N == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s[0]), r, off, 0, 0);
  } else if constexpr (N == 2) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f32x2{s[0], s[1]}), r, off, 0, 0);
  } else {
#pragma unroll
    for (int k = 0; k < N; k += 4)
      __builtin_amdgcn_raw_buffer_store_b128(f32x4{s[k], s[k + 1], s[k + 2], s[k + 3]}, r,
                                             off + 4 * k, 0, 0);
  }
}

// N dropped stores, one per vst<NC> instruction, issued by inline asm against a zero-size
// buffer descriptor (every offset out of range): the compiler can neither merge these stores
// nor drop them as overwritten (it did both to builtin stores at one out-of-range offset,
// which made the counted waits of the first steps too short)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <int NC, int N>
__device__ __forceinline__ void pad_stores(__amdgpu_buffer_rsrc_t) {
  const u32x4 none = {0u, 0u, 0u, 0x00020000u};
  const unsigned off = 0u;
  constexpr int K = N * (NC >= 4 ? NC / 4 : 1);
#pragma unroll
  for (int k = 0; k < K; ++k)
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(0.f), "v"(off), "s"(none) : "memory");
}
// keeps the compiler from moving memory operations across (the pipeline's issue order)
__device__ __forceinline__ void fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ float ror8(float v) {  // lane n <- lane n ^ 8 of its 16-lane row
  // bound_ctrl set (no lane of a row rotation is out of range): lets the compiler fold the
  // move into the add as one v_add_f32_dpp
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128,
                                                            0xF, 0xF, true));
}
__device__ __forceinline__ float ror4(float v) {  // lane n <- lane (n - 4) mod 16 of its row
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124,
                                                            0xF, 0xF, true));
}
__device__ __forceinline__ f32x4 add_ror8(f32x4 a) {
  return f32x4{a[0] + ror8(a[0]), a[1] + ror8(a[1]), a[2] + ror8(a[2]), a[3] + ror8(a[3])};
}
__device__ __forceinline__ f32x4 add_ror4(f32x4 a) {
  return f32x4{a[0] + ror4(a[0]), a[1] + ror4(a[1]), a[2] + ror4(a[2]), a[3] + ror4(a[3])};
}
// sum of the KS K-parts of a tile: columns n, n + S, ... of a 16-lane row (S = 16 / KS)
template <int KS>
__device__ __forceinline__ f32x4 ksum(f32x4 a) {
  if constexpr (KS >= 2) a = add_ror8(a);
  if constexpr (KS == 4) a = add_ror4(a);
  return a;
}
// b where the mask is set, else a: bit selects, so the compiler does not turn a lane-dependent
// choice between two accumulator registers into a scratch-indexed load
__device__ __forceinline__ float bsel(unsigned m, float a, float b) {
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, a) & ~m) |
                                       (__builtin_bit_cast(unsigned, b) & m));
}
// v[sp] for the lane's K part sp (m0 / m1: all-ones when bit 0 / 1 of sp is set)
template <int KS>
__device__ __forceinline__ float kpick(unsigned m0, unsigned m1, const float (&v)[KS]) {
  if constexpr (KS == 1) return v[0];
  else if constexpr (KS == 2) return bsel(m0, v[0], v[1]);
  else return bsel(m1, bsel(m0, v[0], v[1]), bsel(m0, v[2], v[3]));
}

// ---------------------------------------------------------------------------------- packs
// forward fragments [dir][v][mt][kk][lane][KCF/4] fp16: A[m][k] = W_hh[g H + unit][k],
// m = lane & 15, unit = v H/4 + (m / 4) NMT + mt, g = m % 4, k = KCF kk + KCF/4 (lane / 16) + e
template <int H>
__global__ void batch_pack_fwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                      _Float16* __restrict__ out) {
  using G = BGeo<H, 1>;
  constexpr int E = G::KCF / 4;
  const int n = 2 * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int e = i % E, lane = (i / E) & 63;
    int r = i / (E * 64);
    const int kk = r % G::NKC; r /= G::NKC;
    const int mt = r % G::NMT; r /= G::NMT;
    const int v = r % 4, d = r / 4;
    const int m = lane & 15;
    const int unit = v * G::UPW + (m >> 2) * G::NMT + mt, g = m & 3;
    const int k = kk * G::KCF + E * (lane >> 4) + e;
    out[i] = (_Float16)(d ? w1 : w0)[(long long)(g * H + unit) * H + k];
  }
}

// backward fragments of W_hh^T [dir][v][mt][kk][lane][8] bf16: row m = lane & 15 -> f = 4 mt +
// m % 4 ... unit = v H/4 + (m / 4) 4 TPW + 4 mt + m % 4; k = n' = 32 kk + 8 (lane / 16) + e in
// the dG image's order n' = 4 unit' + g (gate row g H + unit')
template <int H>
__global__ void batch_pack_bwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                      __bf16* __restrict__ out) {
  using G = BGeo<H, 1>;
  const int n = 2 * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int e = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int kk = r % G::NKB; r /= G::NKB;
    const int mt = r % G::TPW; r /= G::TPW;
    const int v = r % 4, d = r / 4;
    const int m = lane & 15;
    const int unit = v * G::UPW + (m >> 2) * 4 * G::TPW + 4 * mt + (m & 3);
    const int np = kk * 32 + 8 * (lane >> 4) + e;
    const int row = (np & 3) * H + (np >> 2);
    out[i] = (__bf16)(d ? w1 : w0)[(long long)row * H + unit];
  }
}

// ---------------------------------------------------------------------------------- pipeline
// The inputs of step t are loaded into registers at step t - D by inline-asm loads, so the
// compiler's waitcnt pass (which merges the loop-entry and back-edge states conservatively and
// then waits for loads -- and every store behind them -- one step after issue) knows nothing
// of them; each step waits with an exact counted vmcnt instead: the loads of a step and the
// buffer stores of its outputs are issued in a fixed order (fence()), and the prologue issues
// the same pattern with dropped out-of-range stores, so the count of memory operations behind
// step t's inputs is the same constant at every step.  The wait takes the input registers as
// in/out operands: no use of them can be scheduled above it.
template <int N> struct Vec { using T = f32x4; static constexpr int n = N / 4; };
template <> struct Vec<2> { using T = f32x2; static constexpr int n = 1; };
template <> struct Vec<1> { using T = float; static constexpr int n = 1; };

__device__ __forceinline__ void ald(f32x4& v, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
__device__ __forceinline__ void ald(f32x2& v, const float* p) {
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
__device__ __forceinline__ void ald(float& v, const float* p) {
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
template <int NC>
__device__ __forceinline__ void aldv(typename Vec<NC>::T (&v)[Vec<NC>::n], const float* p) {
#pragma unroll
  for (int k = 0; k < Vec<NC>::n; ++k) ald(v[k], p + 4 * k);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <typename V>
__device__ __forceinline__ void after_wait(V& v) { asm volatile("" : "+v"(v)); }
template <int NC>
__device__ __forceinline__ float el(const typename Vec<NC>::T (&v)[Vec<NC>::n], int i) {
  if constexpr (NC == 1) return v[0];
  else return v[i / 4][i % 4];
}

// ---------------------------------------------------------------------------------- forward
template <int H, int KS, int D>
__global__ __launch_bounds__(NT) void lstm_batch_fwd_kernel(
    const float* __restrict__ gx, int ldg,     // [B*T][ldg], dir d gate g unit u at d 4H + g H + u
    const void* __restrict__ wpv,              // packed forward fragments
    const long long* __restrict__ lengths, int B, int T,
    float* __restrict__ y, int ldy,            // [B*T][ldy], dir d at d H + u
    float* __restrict__ sv) {                  // [B*T][2][5H]
  using G = BGeo<H, KS>;
  constexpr int S = G::S, NMT = G::NMT, NKC = G::NKC, NC = G::NC, HP = G::HP, KCF = G::KCF;
  typedef _Float16 FT __attribute__((ext_vector_type(KCF / 4)));  // A / B fragment
  const FT* wp = (const FT*)wpv;
  using VT = typename Vec<NC>::T;
  constexpr int NV = Vec<NC>::n, LD = 4 * NV, ST = 6 * NV;
  constexpr int WAIT = ST + (D - 1) * (LD + ST);  // operations issued after step t's inputs
  __shared__ __attribute__((aligned(16))) _Float16 hs[2][S + 1][HP];  // row S: zeros
  __shared__ int sL[S];
  const int d = blockIdx.y, b0 = blockIdx.x * S;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6;
  const int lg = lane >> 4, n = lane & 15, sp = n / S, sq = n % S;
  const unsigned m0 = (sp & 1) ? ~0u : 0u, m1 = (sp & 2) ? ~0u : 0u;
  if (tid < S) sL[tid] = b0 + tid < B ? (int)lengths[b0 + tid] : 0;
  for (int i = tid; i < 2 * (S + 1) * HP; i += NT) (&hs[0][0][0])[i] = (_Float16)0.f;

  FT wf[NMT][NKC];
  {
    const FT* src = wp + ((long long)(d * 4 + v) * NMT * NKC) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) wf[mt][kk] = src[(mt * NKC + kk) * 64];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) asm volatile("" ::"v"(wf[mt][kk]));
  }
  __syncthreads();
  int maxL = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) maxL = max(maxL, sL[s]);
  // pad_packed_sequence: outputs past each sequence's end are zero
  for (int s = 0; s < S && b0 + s < B; ++s) {
    const int L = sL[s];
    for (int i = tid; i < (T - L) * H; i += NT)
      y[((long long)(b0 + s) * T + L + i / H) * ldy + d * H + i % H] = 0.f;
  }

  const int b = min(b0 + sq, B - 1), L = sL[sq];
  const int u0 = v * G::UPW + lg * NMT + sp * NC;  // this lane's first unit
  // B-operand source of chunk kk: the sequence's h row, or the zero row for the other half
  int boff[NKC];
#pragma unroll
  for (int kk = 0; kk < NKC; ++kk)
    boff[kk] = ((kk % KS) == sp ? sq : S) * HP + kk * KCF + (KCF / 4) * lg;
  const long long rb = (long long)b * T;
  auto row_of = [L, rb, d](int t) -> long long {  // clamped: always a readable row
    const int tt = max(min(t, L - 1), 0);
    return rb + (d ? max(L - 1 - tt, 0) : tt);
  };
  const float* gbase = gx + d * 4 * H + u0;
  const unsigned ybytes = (unsigned)B * T * ldy * 4u, svbytes = (unsigned)B * T * 10 * H * 4u;
  const __amdgpu_buffer_rsrc_t yr = rsrc(y, ybytes), svr = rsrc(sv, svbytes);

  VT gin[D][4][NV];
#pragma unroll
  for (int u = 0; u < D; ++u) {
    const long long r = row_of(u);
#pragma unroll
    for (int g = 0; g < 4; ++g) aldv<NC>(gin[u][g], gbase + r * ldg + g * H);
    fence();
    pad_stores<NC, 6>(yr);
    fence();
  }
  float cst[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) cst[i] = 0.f;

  for (int t0 = 0; t0 < maxL; t0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int t = t0 + u;
      if (t >= maxL) break;
      const _Float16* hb = &hs[(t + 1) & 1][0][0];
      FT bf[NKC];
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) bf[kk] = *(const FT*)(hb + boff[kk]);
      // tiles in the order the cells consume them (cell i: tiles i and NC + i), K inner, so
      // the cell math of the first tiles can issue between the later tiles' MFMAs
      f32x4 acc[NMT];
#pragma unroll
      for (int i = 0; i < NC; ++i)
#pragma unroll
        for (int hh = 0; hh < KS; ++hh) {
          const int mt = hh * NC + i;
          acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < NKC; ++kk) {
            if constexpr (KCF == 32)
              acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[mt][kk], bf[kk], acc[mt], 0, 0, 0);
            else
              acc[mt] = __builtin_amdgcn_mfma_f32_16x16x16f16(wf[mt][kk], bf[kk], acc[mt], 0, 0, 0);
          }
        }
      wait_vm<WAIT>();
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int k = 0; k < NV; ++k) after_wait(gin[u][g][k]);
      float h[NC], o[5][NC];
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        f32x4 a;
        {
          f32x4 part[KS];
#pragma unroll
          for (int hh = 0; hh < KS; ++hh) part[hh] = ksum<KS>(acc[hh * NC + i]);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float c[KS];
#pragma unroll
            for (int hh = 0; hh < KS; ++hh) c[hh] = part[hh][k];
            a[k] = kpick<KS>(m0, m1, c);
          }
        }
        const float ig = sigm(a[0] + el<NC>(gin[u][0], i)), fg = sigm(a[1] + el<NC>(gin[u][1], i));
        const float gg = tanh_fast(a[2] + el<NC>(gin[u][2], i));
        const float og = sigm(a[3] + el<NC>(gin[u][3], i));
        const float cn = fg * cst[i] + ig * gg;
        cst[i] = cn;
        h[i] = og * tanh_fast(cn);
        o[0][i] = ig; o[1][i] = fg; o[2][i] = gg; o[3][i] = og; o[4][i] = cn;
      }
      {  // publish h_t (fp16) for the next step's B operand: one NC x 2-byte LDS store
        if constexpr (NC == 1) {
          hs[t & 1][sq][u0] = (_Float16)h[0];
        } else {
          typedef _Float16 hvec __attribute__((ext_vector_type(NC)));
          hvec hv;
#pragma unroll
          for (int i = 0; i < NC; ++i) hv[i] = (_Float16)h[i];
          *(hvec*)&hs[t & 1][sq][u0] = hv;
        }
      }
      fence();
      if (!(LB_DBG & 2)) {  // inputs of step t + D (a clamped, always readable row past the end)
        const long long r = row_of(t + D);
#pragma unroll
        for (int g = 0; g < 4; ++g) aldv<NC>(gin[u][g], gbase + r * ldg + g * H);
      }
      fence();
      if (!(LB_DBG & 1)) {
        const unsigned r = (unsigned)row_of(t), past = oob(t, L);
        vst<NC>(yr, ((r * ldy + d * H + u0) * 4u) | past, h);
        const unsigned so = (((r * 2 + d) * 5 * H + u0) * 4u) | past;
#pragma unroll
        for (int g = 0; g < 5; ++g) vst<NC>(svr, so + g * H * 4, o[g]);
      }
      fence();
      __syncthreads();
    }
  }
  wait_vm<0>();  // no load still landing in a register when the wave ends
}

// ---------------------------------------------------------------------------------- backward
template <int H, int KS, int D>
__global__ __launch_bounds__(NT) void lstm_batch_bwd_kernel(
    const float* __restrict__ dy, int lddy,    // [B*T][lddy], grad of outputs
    const bf16x8* __restrict__ wp,             // packed backward fragments
    const long long* __restrict__ lengths, int B, int T,
    const float* __restrict__ sv,              // saved [B*T][2][5H]
    float* __restrict__ dg, int lddg) {        // [B*T][lddg], dir d gate g unit u at d 4H + g H + u
  using G = BGeo<H, KS>;
  constexpr int S = G::S, TPW = G::TPW, NKB = G::NKB, NCB = G::NCB, GP = G::GP, G4 = 4 * H;
  using VT = typename Vec<NCB>::T;
  constexpr int NV = Vec<NCB>::n, LD = 7 * NV, ST = 4 * NV;
  constexpr int WAIT = (D - 1) * (LD + ST);  // each step stores, then loads
  __shared__ __attribute__((aligned(16))) __bf16 gs[2][S + 1][GP];  // row S: zeros
  __shared__ int sL[S];
  const int d = blockIdx.y, b0 = blockIdx.x * S;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6;
  const int lg = lane >> 4, n = lane & 15, sp = n / S, sq = n % S;
  const unsigned m0 = (sp & 1) ? ~0u : 0u, m1 = (sp & 2) ? ~0u : 0u;
  if (tid < S) sL[tid] = b0 + tid < B ? (int)lengths[b0 + tid] : 0;
  for (int i = tid; i < 2 * (S + 1) * GP; i += NT) (&gs[0][0][0])[i] = (__bf16)0.f;

  bf16x8 wb[TPW][NKB];
  {
    const bf16x8* src = wp + ((long long)(d * 4 + v) * TPW * NKB) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < TPW; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) wb[mt][kk] = src[(mt * NKB + kk) * 64];
#pragma unroll
    for (int mt = 0; mt < TPW; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) asm volatile("" ::"v"(wb[mt][kk]));
  }
  __syncthreads();
  int maxL = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) maxL = max(maxL, sL[s]);
  for (int s = 0; s < S && b0 + s < B; ++s) {  // zero the gate gradients past the end
    const int L = sL[s];
    for (int i = tid; i < (T - L) * G4; i += NT)
      dg[((long long)(b0 + s) * T + L + i / G4) * lddg + d * G4 + i % G4] = 0.f;
  }

  const int b = min(b0 + sq, B - 1), L = sL[sq];
  const int u0 = v * G::UPW + lg * 4 * TPW + sp * NCB;
  int boff[NKB];
#pragma unroll
  for (int kk = 0; kk < NKB; ++kk)
    boff[kk] = ((kk % KS) == sp ? sq : S) * GP + kk * 32 + 8 * lg;
  const long long rb = (long long)b * T;
  // processing index q of the sequence is its forward step L - 1 - q: row L-1-q (dir 0) or q
  auto row_of = [L, rb, d](int q) -> long long {
    const int qq = max(min(q, L - 1), 0);
    return rb + (d ? qq : max(L - 1 - qq, 0));
  };
  auto prow_of = [L, rb, d](int q) -> long long {  // c of the previous forward step (or own row)
    const int qq = max(min(q, L - 1), 0);
    return qq < L - 1 ? rb + (d ? qq + 1 : L - 2 - qq) : rb + (d ? qq : max(L - 1 - qq, 0));
  };
  const float* svb = sv + d * 5 * H + u0;
  const float* dyb = dy + d * H + u0;
  const unsigned dgbytes = (unsigned)B * T * lddg * 4u;
  const __amdgpu_buffer_rsrc_t dgr = rsrc(dg, dgbytes);

  VT in[D][7][NV];  // i f g o c (row), c (previous step), dy
#define LB_LOAD(dst, q)                                                   \
  {                                                                       \
    const long long r_ = row_of(q), pr_ = prow_of(q);                     \
    _Pragma("unroll") for (int g = 0; g < 5; ++g)                         \
        aldv<NCB>(dst[g], svb + r_ * 10 * H + g * H);                     \
    aldv<NCB>(dst[5], svb + pr_ * 10 * H + 4 * H);                        \
    aldv<NCB>(dst[6], dyb + r_ * lddy);                                   \
  }
#pragma unroll
  for (int u = 0; u < D; ++u) {
    pad_stores<NCB, 4>(dgr);
    fence();
    LB_LOAD(in[u], u);
    fence();
  }
  float dcs[NCB];
#pragma unroll
  for (int i = 0; i < NCB; ++i) dcs[i] = 0.f;

  for (int q0 = 0; q0 < maxL; q0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int q = q0 + u;
      if (q >= maxL) break;
      const __bf16* gb = &gs[(q + 1) & 1][0][0];
      bf16x8 bf[NKB];
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) bf[kk] = *(const bf16x8*)(gb + boff[kk]);
      f32x4 acc[TPW];
#pragma unroll
      for (int mt = 0; mt < TPW; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKB; ++kk)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[mt][kk], bf[kk], acc[mt], 0, 0, 0);
      }
      wait_vm<WAIT>();
#pragma unroll
      for (int g = 0; g < 7; ++g)
#pragma unroll
        for (int k = 0; k < NV; ++k) after_wait(in[u][g][k]);
      float dhr[NCB];
      if constexpr (KS == 1) {
#pragma unroll
        for (int i = 0; i < NCB; ++i) dhr[i] = acc[i >> 2][i & 3];
      } else {
#pragma unroll
        for (int mt = 0; mt < TPW; ++mt) acc[mt] = ksum<KS>(acc[mt]);
#pragma unroll
        for (int i = 0; i < NCB; ++i) {  // cell f = sp NCB + i of the flat [TPW][4] sums
          float c[KS];
#pragma unroll
          for (int hh = 0; hh < KS; ++hh) c[hh] = acc[(hh * NCB + i) >> 2][(hh * NCB + i) & 3];
          dhr[i] = kpick<KS>(m0, m1, c);
        }
      }
      const bool val = q < L;
      float o[4][NCB];
#pragma unroll
      for (int i = 0; i < NCB; ++i) {
        const float ig = el<NCB>(in[u][0], i), fg = el<NCB>(in[u][1], i);
        const float gg = el<NCB>(in[u][2], i), og = el<NCB>(in[u][3], i);
        const float cp = q < L - 1 ? el<NCB>(in[u][5], i) : 0.f;
        const float dh = el<NCB>(in[u][6], i) + dhr[i];
        const float tc = tanh_fast(el<NCB>(in[u][4], i));
        const float dcc = dcs[i] + dh * og * (1.f - tc * tc);
        o[0][i] = dcc * gg * ig * (1.f - ig);
        o[1][i] = dcc * cp * fg * (1.f - fg);
        o[2][i] = dcc * ig * (1.f - gg * gg);
        o[3][i] = dh * tc * og * (1.f - og);
        dcs[i] = dcc * fg;
      }
      {  // publish dG_q (bf16) in the order n' = 4 unit + g
        __bf16* gw = &gs[q & 1][sq][4 * u0];
        if constexpr (NCB == 1) {
          bf16x4 nb;
#pragma unroll
          for (int g = 0; g < 4; ++g) nb[g] = (__bf16)(val ? o[g][0] : 0.f);
          *(bf16x4*)gw = nb;
        } else {
#pragma unroll
          for (int i = 0; i < NCB; i += 2) {
            bf16x8 nb;
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int g = 0; g < 4; ++g) nb[4 * k + g] = (__bf16)(val ? o[g][i + k] : 0.f);
            *(bf16x8*)(gw + 4 * i) = nb;
          }
        }
      }
      fence();
      if (!(LB_DBG & 1)) {
        const unsigned off = (((unsigned)row_of(q) * lddg + d * G4 + u0) * 4u) | oob(q, L);
#pragma unroll
        for (int g = 0; g < 4; ++g) vst<NCB>(dgr, off + g * H * 4, o[g]);
      }
      fence();
      if (!(LB_DBG & 2)) LB_LOAD(in[u], q + D);  // a clamped, always readable row past the end
      fence();
      __syncthreads();
    }
  }
#undef LB_LOAD
  wait_vm<0>();
}

// ---------------------------------------------------------------------------------- launch
int g_ks = 4, g_depth = 2;  // 4 sequences per workgroup, 2 steps ahead (profiles/r3_lstm_batch_bench.txt)

size_t excl(size_t need) {
  return ensvs_rec_exclusive() ? std::max<size_t>(need, 160 * 1024) : need;
}

template <typename K>
int set_dyn(K kern, size_t st_lds, size_t& dyn) {
  dyn = excl(st_lds) - st_lds;
  return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)dyn) == hipSuccess ? ENSVS_OK : ENSVS_E_HIP;
}

template <int H, int KS, int D>
int launch_fwd(const float* gx, int ldg, const void* wp, const long long* lengths, int B, int T,
               float* y, int ldy, float* sv, hipStream_t st) {
  using G = BGeo<H, KS>;
  size_t dyn;
  if (set_dyn(lstm_batch_fwd_kernel<H, KS, D>, 2 * (2 * (G::S + 1) * G::HP) + 4 * G::S, dyn))
    return ENSVS_E_HIP;
  hipLaunchKernelGGL((lstm_batch_fwd_kernel<H, KS, D>), dim3(cdiv(B, G::S), 2), dim3(NT), dyn, st,
                     gx, ldg, wp, lengths, B, T, y, ldy, sv);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H, int KS, int D>
int launch_bwd(const float* dy, int lddy, const void* wp, const long long* lengths, int B, int T,
               const float* sv, float* dg, int lddg, hipStream_t st) {
  using G = BGeo<H, KS>;
  size_t dyn;
  if (set_dyn(lstm_batch_bwd_kernel<H, KS, D>, 2 * (2 * (G::S + 1) * G::GP) + 4 * G::S, dyn))
    return ENSVS_E_HIP;
  hipLaunchKernelGGL((lstm_batch_bwd_kernel<H, KS, D>), dim3(cdiv(B, G::S), 2), dim3(NT), dyn, st,
                     dy, lddy, (const bf16x8*)wp, lengths, B, T, sv, dg, lddg);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H>
int fwd_h(const float* gx, int ldg, const void* wp, const long long* lengths, int B, int T,
          float* y, int ldy, float* sv, hipStream_t st) {
#define LB_F(KS, D) \
  if (g_ks == KS && g_depth == D) return launch_fwd<H, KS, D>(gx, ldg, wp, lengths, B, T, y, ldy, sv, st);
  LB_F(1, 2) LB_F(1, 3) LB_F(2, 2) LB_F(2, 3) LB_F(4, 2) LB_F(4, 3)
#undef LB_F
  return ENSVS_E_ARG;
}

template <int H>
int bwd_h(const float* dy, int lddy, const void* wp, const long long* lengths, int B, int T,
          const float* sv, float* dg, int lddg, hipStream_t st) {
#define LB_B(KS, D) \
  if (g_ks == KS && g_depth == D) return launch_bwd<H, KS, D>(dy, lddy, wp, lengths, B, T, sv, dg, lddg, st);
  LB_B(1, 2) LB_B(1, 3) LB_B(2, 2) LB_B(2, 3) LB_B(4, 2) LB_B(4, 3)
#undef LB_B
  return ENSVS_E_ARG;
}

bool aligned16(const void* p) { return (uintptr_t)p % 16 == 0; }
// the outputs are addressed through 32-bit buffer offsets
bool fits(long long rows, long long ld) { return rows * ld * 4 < (1LL << 31); }

}  // namespace

ENSVS_API int ensvs_lstm_batch_supported(int B, int H) {
  return B >= 1 && (H == 64 || H == 128) ? 1 : 0;
}

ENSVS_API int ensvs_lstm_batch_set_cfg(int seqs_per_wg, int depth) {
  if ((seqs_per_wg != 4 && seqs_per_wg != 8 && seqs_per_wg != 16) || (depth != 2 && depth != 3))
    return ENSVS_E_ARG;
  g_ks = 16 / seqs_per_wg;
  g_depth = depth;
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_batch_pack(const float* whh_f, const float* whh_r, int H, int bwd,
                                    void* out, void* stream) {
  if (H != 64 && H != 128) return ENSVS_E_SHAPE;
  if (!out || !aligned16(out) || !whh_f || !whh_r) return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(cdiv(2LL * 4 * H * H, 256)), block(256);
  if (H == 64) {
    if (bwd) hipLaunchKernelGGL(batch_pack_bwd_kernel<64>, grid, block, 0, st, whh_f, whh_r, (__bf16*)out);
    else hipLaunchKernelGGL(batch_pack_fwd_kernel<64>, grid, block, 0, st, whh_f, whh_r, (_Float16*)out);
  } else {
    if (bwd) hipLaunchKernelGGL(batch_pack_bwd_kernel<128>, grid, block, 0, st, whh_f, whh_r, (__bf16*)out);
    else hipLaunchKernelGGL(batch_pack_fwd_kernel<128>, grid, block, 0, st, whh_f, whh_r, (_Float16*)out);
  }
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_batch_fwd(const float* gx, int ldg, const void* wpack,
                                   const long long* lengths, int B, int T, int H, float* y, int ldy,
                                   float* saved, void* stream) {
  if (!ensvs_lstm_batch_supported(B, H) || T <= 0 || ldg < 8 * H || ldy < 2 * H ||
      !fits((long long)B * T, ldy) || !fits((long long)B * T, 10 * H))
    return ENSVS_E_SHAPE;
  if (ldg % 4 || ldy % 4 || !aligned16(gx) || !aligned16(y) || !aligned16(saved) ||
      !aligned16(wpack) || !lengths)
    return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  return H == 64 ? fwd_h<64>(gx, ldg, wpack, lengths, B, T, y, ldy, saved, st)
                 : fwd_h<128>(gx, ldg, wpack, lengths, B, T, y, ldy, saved, st);
}

ENSVS_API int ensvs_lstm_batch_bwd(const float* dy, int lddy, const void* wpack,
                                   const long long* lengths, int B, int T, int H,
                                   const float* saved, float* dg, int lddg, void* stream) {
  if (!ensvs_lstm_batch_supported(B, H) || T <= 0 || lddy < 2 * H || lddg < 8 * H ||
      !fits((long long)B * T, lddg))
    return ENSVS_E_SHAPE;
  if (lddy % 4 || lddg % 4 || !aligned16(dy) || !aligned16(dg) || !aligned16(saved) ||
      !aligned16(wpack) || !lengths)
    return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  return H == 64 ? bwd_h<64>(dy, lddy, wpack, lengths, B, T, saved, dg, lddg, st)
                 : bwd_h<128>(dy, lddy, wpack, lengths, B, T, saved, dg, lddg, st);
}
