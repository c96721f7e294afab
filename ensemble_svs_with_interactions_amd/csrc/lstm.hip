// Packed bidirectional LSTM recurrence (forward + backward through time).
//
// Replaces the time recurrence of nn.LSTM(bidirectional=True, batch_first=True)
// over pack_padded_sequence input as used by FFConvLSTM (nnsvs/model.py:862-869,
// 914-916) and the multi-track lf0 encoder (acoustic_models/tacotron_f0.py:876-883,
// 981-983).  The input projections x_t W_ih^T + b_ih + b_hh for all t are one
// MFMA GEMM beforehand (gemm.hip); only h_{t-1} W_hh^T stays in the loop.
//
// One workgroup per (sequence, direction) runs every step of its sequence
// (persistent), holding its W_hh slice in VGPRs:
//   thread (u, q), u = unit (16 per wave, lane & 15), q = lane >> 4 (K quarter)
//   fwd: w[g][k] = W_hh[g*H + u][q*H/4 + k], g in {i,f,g,o}
//   bwd: w[g][k] = W_hh[q*H + ?]... (transposed: column u of gate block q)
// The four K-quarter partial sums are combined with cross-lane xor shuffles,
// h (fwd) / dG (bwd) is exchanged through a double-buffered LDS vector: one
// __syncthreads per time step.
//
// Packed semantics: sequence b has length L_b; the forward direction runs
// t = 0..L_b-1, the reverse direction t = L_b-1..0 from a zero state, and
// outputs at t >= L_b are zero (pad_packed_sequence).
#include "common.h"
#include "ensvs.h"

namespace {

// 16 units per wave (lane & 15), 4 K-parts (lane >> 4); H < 16 pads idle units.
template <int H> struct Geo {
  static constexpr int WAVES = H >= 16 ? H / 16 : 1;
  static constexpr int THREADS = 64 * WAVES;
};

template <int N>
__device__ __forceinline__ void load_row(float (&dst)[N], const float* src) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      f32x4 v = *(const f32x4*)(src + k);
      dst[k] = v[0]; dst[k + 1] = v[1]; dst[k + 2] = v[2]; dst[k + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) dst[k] = src[k];
  }
}

template <int H>
__global__ __launch_bounds__(Geo<H>::THREADS) void lstm_fwd_kernel(
    const float* __restrict__ gx, int ldg,        // [B*T][ldg], dir d gates at cols d*4H + g*H + u
    const float* __restrict__ whh0, const float* __restrict__ whh1,  // [4H][H] per direction
    const long long* __restrict__ lengths, int T,
    float* __restrict__ y, int ldy,               // [B*T][ldy], dir d at cols d*H + u
    float* __restrict__ sv) {                     // saved [B*T][2][5H]: i,f,g,o,c
  constexpr int Q = H / 4;
  __shared__ __attribute__((aligned(16))) float hbuf[2][H];
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int u = wave * 16 + (lane & 15), q = lane >> 4;
  const bool act = u < H;
  const int L = (int)lengths[b];
  const float* W = dir ? whh1 : whh0;

  float w[4][Q];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    if (act) load_row<Q>(w[g], W + (long long)(g * H + u) * H + q * Q);
    else
#pragma unroll
      for (int k = 0; k < Q; ++k) w[g][k] = 0.f;
  }
  if (tid < H) hbuf[0][tid] = 0.f;
  float c = 0.f;
  __syncthreads();

  const long long rowb = (long long)b * T;
  for (int i = tid; i < (T - L) * H; i += Geo<H>::THREADS)
    y[(rowb + L + i / H) * ldy + dir * H + (i % H)] = 0.f;

  float gnext[4] = {0.f, 0.f, 0.f, 0.f};
  if (L > 0 && act) {
    const int t0 = dir ? L - 1 : 0;
    const float* gp = gx + (rowb + t0) * ldg + dir * 4 * H + u;
#pragma unroll
    for (int g = 0; g < 4; ++g) gnext[g] = gp[g * H];
  }
  for (int s = 0; s < L; ++s) {
    const int t = dir ? L - 1 - s : s;
    const float* hc = hbuf[s & 1] + q * Q;
    float acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = gnext[g];
    if (s + 1 < L && act) {
      const int tn = dir ? t - 1 : t + 1;
      const float* gp = gx + (rowb + tn) * ldg + dir * 4 * H + u;
#pragma unroll
      for (int g = 0; g < 4; ++g) gnext[g] = gp[g * H];
    }
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      const float hv = hc[k];
#pragma unroll
      for (int g = 0; g < 4; ++g) p[g] = fmaf(w[g][k], hv, p[g]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      p[g] += __shfl_xor(p[g], 16);
      p[g] += __shfl_xor(p[g], 32);
      acc[g] += p[g];
    }
    const float ig = sigmoidf_(acc[0]);
    const float fg = sigmoidf_(acc[1]);
    const float gg = tanhf(acc[2]);
    const float og = sigmoidf_(acc[3]);
    c = fg * c + ig * gg;
    const float h = og * tanhf(c);
    if (act) {
      const long long row = rowb + t;
      if (q == 0) {
        hbuf[(s + 1) & 1][u] = h;
        y[row * ldy + dir * H + u] = h;
      }
      float* svp = sv + (row * 2 + dir) * 5 * H + u;
      const float mine = q == 0 ? ig : q == 1 ? fg : q == 2 ? gg : og;
      svp[q * H] = mine;
      if (q == 0) svp[4 * H] = c;
    }
    __syncthreads();
  }
}

template <int H>
__global__ __launch_bounds__(Geo<H>::THREADS) void lstm_bwd_kernel(
    const float* __restrict__ dy, int lddy,       // [B*T][lddy], grad of outputs
    const float* __restrict__ whh0, const float* __restrict__ whh1,  // [4H][H] per direction
    const long long* __restrict__ lengths, int T,
    const float* __restrict__ sv,                 // saved [B*T][2][5H]
    float* __restrict__ dg, int lddg) {           // [B*T][lddg], dir d pre-act grads at d*4H + g*H + u
  __shared__ __attribute__((aligned(16))) float gbuf[2][4 * H];
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int u = wave * 16 + (lane & 15), q = lane >> 4;
  const bool act = u < H;
  const int L = (int)lengths[b];
  const float* W = dir ? whh1 : whh0;

  // column u of gate block q: w[j] = W_hh[q*H + j][u]
  float w[H];
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] = act ? W[(long long)(q * H + j) * H + u] : 0.f;

  const long long rowb = (long long)b * T;
  for (int i = tid; i < (T - L) * 4 * H; i += Geo<H>::THREADS)
    dg[(rowb + L + i / (4 * H)) * lddg + dir * 4 * H + (i % (4 * H))] = 0.f;

  float dhr = 0.f, dc = 0.f;
  for (int s = L - 1; s >= 0; --s) {
    const int t = dir ? L - 1 - s : s;
    const long long row = rowb + t;
    float* gb = gbuf[s & 1];
    if (act) {
      const float* svp = sv + (row * 2 + dir) * 5 * H + u;
      const float ig = svp[0], fg = svp[H], gg = svp[2 * H], og = svp[3 * H], ct = svp[4 * H];
      float cp = 0.f;
      if (s > 0) {
        const int tp = dir ? t + 1 : t - 1;
        cp = sv[((rowb + tp) * 2 + dir) * 5 * H + 4 * H + u];
      }
      const float dh = dy[row * lddy + dir * H + u] + dhr;
      const float tc = tanhf(ct);
      const float dcc = dc + dh * og * (1.f - tc * tc);
      const float d_i = dcc * gg * ig * (1.f - ig);
      const float d_f = dcc * cp * fg * (1.f - fg);
      const float d_g = dcc * ig * (1.f - gg * gg);
      const float d_o = dh * tc * og * (1.f - og);
      dc = dcc * fg;
      const float mine = q == 0 ? d_i : q == 1 ? d_f : q == 2 ? d_g : d_o;
      gb[q * H + u] = mine;
      dg[row * lddg + dir * 4 * H + q * H + u] = mine;
    }
    __syncthreads();
    float p = 0.f;
    const float* gq = gb + q * H;
#pragma unroll
    for (int j = 0; j < H; ++j) p = fmaf(w[j], gq[j], p);
    p += __shfl_xor(p, 16);
    p += __shfl_xor(p, 32);
    dhr = p;
  }
}

template <int H>
int launch_fwd(const float* gx, int ldg, const float* w0, const float* w1,
               const long long* lengths, int B, int T, float* y, int ldy, float* sv,
               hipStream_t st) {
  hipLaunchKernelGGL(lstm_fwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::THREADS), 0, st, gx, ldg, w0, w1,
                     lengths, T, y, ldy, sv);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H>
int launch_bwd(const float* dy, int lddy, const float* w0, const float* w1,
               const long long* lengths, int B, int T, const float* sv, float* dg, int lddg,
               hipStream_t st) {
  hipLaunchKernelGGL(lstm_bwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::THREADS), 0, st, dy, lddy, w0, w1,
                     lengths, T, sv, dg, lddg);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

}  // namespace

ENSVS_API int ensvs_lstm_fwd(const float* gx, int ldg, const float* whh_f, const float* whh_r,
                             const long long* lengths, int B, int T, int H, float* y, int ldy,
                             float* saved, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (H) {
    case 8: return launch_fwd<8>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 16: return launch_fwd<16>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 32: return launch_fwd<32>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 64: return launch_fwd<64>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 128: return launch_fwd<128>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    default: return ENSVS_E_SHAPE;
  }
}

ENSVS_API int ensvs_lstm_bwd(const float* dy, int lddy, const float* whh_f, const float* whh_r,
                             const long long* lengths, int B, int T, int H, const float* saved,
                             float* dg, int lddg, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (H) {
    case 8: return launch_bwd<8>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 16: return launch_bwd<16>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 32: return launch_bwd<32>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 64: return launch_bwd<64>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 128: return launch_bwd<128>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    default: return ENSVS_E_SHAPE;
  }
}
