// Packed bidirectional LSTM recurrence (forward + backward through time).
//
// Replaces the time recurrence of nn.LSTM(bidirectional=True, batch_first=True)
// over pack_padded_sequence input as used by FFConvLSTM (nnsvs/model.py:862-869,
// 914-916) and the multi-track lf0 encoder (acoustic_models/tacotron_f0.py:876-883,
// 981-983).  The input projections x_t W_ih^T + b_ih + b_hh for all t are one
// MFMA GEMM beforehand (gemm.hip); only h_{t-1} W_hh^T stays in the loop.
//
// One workgroup per (sequence, direction) runs every step of its sequence
// (persistent), holding its W_hh slice in VGPRs.  KP lanes (4 or 8, adjacent lanes of
// one quad / half-row) share a unit u and split its dot products:
//   fwd: lane q holds w[g][k] = W_hh[g*H + u][q*H/KP + k] (the 4 gates, K-part q);
//   bwd: lane q holds w[j]    = W_hh[q*4H/KP + j][u]     (column u, part q of 4H).
// Partial sums are combined with DPP (row_half_mirror, quad_perm xor 1 / xor 2) in
// registers, so every lane of the unit ends with the same bits.  In the forward step
// lane q evaluates only gate q&3 (tanh(x) = 2 sigmoid(2x) - 1 for g) and the four
// activations are exchanged by quad broadcasts.
//
// Global memory stays off the per-step critical path: inputs are staged through LDS in
// chunks of CH steps (loaded to registers one chunk ahead), outputs are collected in
// LDS and written back at the chunk boundary.  (vmcnt counts loads and stores in issue
// order, so a per-step prefetch would wait on the previous step's stores.)  h (fwd) /
// dG (bwd) is exchanged through a double-buffered LDS vector: one barrier per step.
//
// Packed semantics: sequence b has length L_b; the forward direction runs
// t = 0..L_b-1, the reverse direction t = L_b-1..0 from a zero state, and
// outputs at t >= L_b are zero (pad_packed_sequence).
#include "common.h"
#include "ensvs.h"

namespace {

// Lanes per unit (KPF forward, KPB backward; measured on MI355X at 30 x 1024 frames):
// the forward H=128 step is FMA-issue bound and prefers 512 threads, the backward one
// is bound by its dependent dot-product chain and prefers 1024.
template <int H> struct Geo {
  static constexpr int KPF = H == 64 ? 8 : 4, KPB = H >= 64 ? 8 : 4;
  // bwd units per lane group: at H=128 one group of KPB lanes serves two units, so each
  // dG value read from LDS feeds two dot products (the step is bound by LDS data return:
  // lanes x 4H/KPB floats per step, halved with the lane count)
  static constexpr int UPB = H >= 128 ? 2 : 1;
  static constexpr int TF = H * KPF, TB = H * KPB / UPB;  // threads
  static constexpr int Q = H / KPF;                 // fwd: h elements per lane
  static constexpr int QB = 4 * H / KPB;            // bwd: dG elements per lane
  // steps per staged chunk (bwd H=128: 4, keeping its prefetch next to 2 x 64 weights)
  static constexpr int CHF = 16, CHB = H >= 128 ? 4 : 16;
  // The exchanged vectors (h: KPF parts of Q, dG: KPB parts of QB) are stored with a
  // 16-B pad after each part, so the distinct addresses one wave reads per
  // ds_read_b128 fall in distinct banks.
  static constexpr int HP = Q + 4, GP = QB + 4;
  static constexpr int HBUF = KPF * HP, GBUF = KPB * GP;
  // LDS bytes: fwd h[2] + in[CH][4H] + out[CH][6H]; bwd dG[2] + in[CH][7H] + out[CH][4H]
  static constexpr int FWD_LDS = (2 * HBUF + CHF * 4 * H + CHF * 6 * H) * 4;
  static constexpr int BWD_LDS = (2 * GBUF + CHB * 7 * H + CHB * 4 * H) * 4;
};

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                            0xF, 0xF, false));
}
// sum over the KP lanes of a unit; identical bits in all of them
template <int KP>
__device__ __forceinline__ float unit_sum(float v) {
  if constexpr (KP == 8) v += dpp<0x141>(v);  // row_half_mirror: lane i + lane 7-i
  v += dpp<0xB1>(v);                          // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);                          // quad_perm [2,3,0,1]
  return v;
}

// Recurrence nonlinearities on v_exp / v_rcp (absolute error ~1e-7; the IEEE division
// and the branchy libm tanhf would sit on the per-step dependency chain).
__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)), 1.f);
}
// one of four values by a lane index, with bit selects (no exec-mask branches)
__device__ __forceinline__ float pick4(const float (&v)[4], int i) {
  const unsigned m0 = i == 0 ? ~0u : 0u, m1 = i == 1 ? ~0u : 0u, m2 = i == 2 ? ~0u : 0u,
                 m3 = i == 3 ? ~0u : 0u;
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, v[0]) & m0) |
                                       (__builtin_bit_cast(unsigned, v[1]) & m1) |
                                       (__builtin_bit_cast(unsigned, v[2]) & m2) |
                                       (__builtin_bit_cast(unsigned, v[3]) & m3));
}
// Make the waitcnt pass retire a register's load here (before the step loop) instead
// of with a conservative vmcnt(0) inside it, which would also drain the chunk prefetch.
template <int N>
__device__ __forceinline__ void settle(const float (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" ::"v"(v[k]));
}

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
__global__ __launch_bounds__(Geo<H>::TF) void lstm_fwd_kernel(
    const float* __restrict__ gx, int ldg,        // [B*T][ldg], dir d gates at cols d*4H + g*H + u
    const float* __restrict__ whh0, const float* __restrict__ whh1,  // [4H][H] per direction
    const long long* __restrict__ lengths, int T,
    float* __restrict__ y, int ldy,               // [B*T][ldy], dir d at cols d*H + u
    float* __restrict__ sv) {                     // saved [B*T][2][5H]: i,f,g,o,c
  using G = Geo<H>;
  constexpr int KP = G::KPF, Q = G::Q, NT = G::TF, GW = 4 * H, OW = 6 * H, CH = G::CHF;
  constexpr int PF = CH * GW / 4 / NT;  // float4 of one input chunk per thread (= CH / KP)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* hbuf = lds;              // [2][KP][Q + 4]
  float* gin = hbuf + 2 * G::HBUF;  // [CH][4H] gate pre-activations x W_ih^T + b
  float* out = gin + CH * GW;     // [CH][6H]: h, then i f g o c
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, u = tid / KP, q = tid % KP, gq = q & 3;
  const int L = (int)lengths[b];
  const float* W = dir ? whh1 : whh0;

  float w[4][Q];
#pragma unroll
  for (int g = 0; g < 4; ++g) load_row<Q>(w[g], W + (long long)(g * H + u) * H + q * Q);
#pragma unroll
  for (int g = 0; g < 4; ++g) settle(w[g]);
  for (int i = tid; i < G::HBUF; i += NT) hbuf[i] = 0.f;
  const int hslot = (u / Q) * G::HP + u % Q;  // where unit u's h goes
  float c = 0.f;

  const long long rowb = (long long)b * T;
  for (int i = tid; i < (T - L) * H; i += NT)
    y[(rowb + L + i / H) * ldy + dir * H + (i % H)] = 0.f;

  const int nch = (L + CH - 1) / CH;
  f32x4 rin[PF];
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT, st = e / (GW / 4), c4 = e % (GW / 4);
      const int s = ch * CH + st;
      const int row = dir ? L - 1 - s : s;
      rin[i] = s < L ? *(const f32x4*)(gx + (rowb + row) * ldg + dir * GW + c4 * 4)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_in = [&]() {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT;
      *(f32x4*)(gin + (e / (GW / 4)) * GW + (e % (GW / 4)) * 4) = rin[i];
    }
  };
  auto flush = [&](int ch) {
    const int n = min(CH, L - ch * CH);
    for (int e = tid; e < n * (OW / 4); e += NT) {
      const int st = e / (OW / 4), c4 = e % (OW / 4);
      const int s = ch * CH + st;
      const long long row = rowb + (dir ? L - 1 - s : s);
      const f32x4 v = *(const f32x4*)(out + st * OW + c4 * 4);
      if (c4 < H / 4) *(f32x4*)(y + row * ldy + dir * H + c4 * 4) = v;
      else *(f32x4*)(sv + (row * 2 + dir) * 5 * H + (c4 - H / 4) * 4) = v;
    }
  };

  if (nch > 0) {
    load_chunk(0);
    store_in();
  }
  if (nch > 1) load_chunk(1);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int n = min(CH, L - ch * CH);
    for (int st = 0; st < n; ++st) {
      const int s = ch * CH + st;
      const float* hc = hbuf + (s & 1) * G::HBUF + q * G::HP;
      float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        const float hv = hc[k];
#pragma unroll
        for (int g = 0; g < 4; ++g) p[g] = fmaf(w[g][k], hv, p[g]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) p[g] = unit_sum<KP>(p[g]);
      const float x = gin[st * GW + gq * H + u] + pick4(p, gq);
      const float sg = sigm(gq == 2 ? 2.f * x : x);
      const float act = gq == 2 ? fmaf(2.f, sg, -1.f) : sg;
      const float ig = dpp<0x00>(act), fg = dpp<0x55>(act), gg = dpp<0xAA>(act),
                  og = dpp<0xFF>(act);
      c = fg * c + ig * gg;
      const float h = og * tanh_fast(c);
      float* o = out + st * OW;
      if (q == 0) {
        hbuf[((s + 1) & 1) * G::HBUF + hslot] = h;
        o[u] = h;
        o[5 * H + u] = c;
      }
      if (q < 4) o[H + q * H + u] = act;
      __syncthreads();
    }
    if (ch + 1 < nch) store_in();
    flush(ch);
    if (ch + 2 < nch) load_chunk(ch + 2);
    __syncthreads();
  }
}

template <int H>
__global__ __launch_bounds__(Geo<H>::TB) void lstm_bwd_kernel(
    const float* __restrict__ dy, int lddy,       // [B*T][lddy], grad of outputs
    const float* __restrict__ whh0, const float* __restrict__ whh1,  // [4H][H] per direction
    const long long* __restrict__ lengths, int T,
    const float* __restrict__ sv,                 // saved [B*T][2][5H]
    float* __restrict__ dg, int lddg) {           // [B*T][lddg], dir d pre-act grads at d*4H + g*H + u
  using G = Geo<H>;
  constexpr int KP = G::KPB, QB = G::QB, NT = G::TB, IW = 7 * H, GW = 4 * H, CH = G::CHB;
  constexpr int UP = G::UPB, HU = H / UP;  // units per lane group, group count
  constexpr int NIN = CH * IW / 4;                 // float4 per input chunk
  constexpr int PF = (NIN + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gbuf = lds;              // [2][KP][QB + 4] dG exchange
  float* gin = gbuf + 2 * G::GBUF;  // [CH][7H]: i f g o c (row t), dy (row t), c (previous step)
  float* out = gin + CH * IW;     // [CH][4H]
  const int b = blockIdx.x, dir = blockIdx.y;
  // lane group grp serves units grp + k*HU (k < UP); lane q evaluates gate q&3 of unit
  // uq (UP = 2: lanes 0-3 the first unit, 4-7 the second) and holds, for every unit of
  // its group, column u of part q of W_hh (QB rows)
  const int tid = threadIdx.x, grp = tid / KP, q = tid % KP, gq = q & 3;
  const int uk = UP == 1 ? 0 : q / (KP / UP), u = grp + uk * HU;
  const int L = (int)lengths[b];
  const float* W = dir ? whh1 : whh0;

  float w[UP][QB];
#pragma unroll
  for (int k = 0; k < UP; ++k) {
#pragma unroll
    for (int j = 0; j < QB; ++j) w[k][j] = W[(long long)(q * QB + j) * H + grp + k * HU];
    settle(w[k]);
  }
  const int f = gq * H + u;                      // this lane's gate gradient
  const int gslot = (f / QB) * G::GP + f % QB;

  const long long rowb = (long long)b * T;
  for (int i = tid; i < (T - L) * GW; i += NT)
    dg[(rowb + L + i / GW) * lddg + dir * GW + (i % GW)] = 0.f;

  // chunk ch holds processing steps s = L-1-ch*CH-st, st = 0..CH-1 (descending s)
  const int nch = (L + CH - 1) / CH;
  f32x4 rin[PF];
  auto svrow = [&](int s) { return sv + ((rowb + (dir ? L - 1 - s : s)) * 2 + dir) * 5 * H; };
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT, st = e / (IW / 4), c4 = e % (IW / 4);
      const int s = L - 1 - ch * CH - st;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < NIN && s >= 0) {
        if (c4 < 5 * H / 4) v = *(const f32x4*)(svrow(s) + c4 * 4);
        else if (c4 < 6 * H / 4)
          v = *(const f32x4*)(dy + (rowb + (dir ? L - 1 - s : s)) * lddy + dir * H +
                              (c4 - 5 * H / 4) * 4);
        else if (s > 0) v = *(const f32x4*)(svrow(s - 1) + 4 * H + (c4 - 6 * H / 4) * 4);
      }
      rin[i] = v;
    }
  };
  auto store_in = [&]() {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT;
      if (e < NIN) *(f32x4*)(gin + (e / (IW / 4)) * IW + (e % (IW / 4)) * 4) = rin[i];
    }
  };
  auto flush = [&](int ch) {
    const int n = min(CH, L - ch * CH);
    for (int e = tid; e < n * (GW / 4); e += NT) {
      const int st = e / (GW / 4), c4 = e % (GW / 4);
      const int s = L - 1 - ch * CH - st;
      const long long row = rowb + (dir ? L - 1 - s : s);
      *(f32x4*)(dg + row * lddg + dir * GW + c4 * 4) = *(const f32x4*)(out + st * GW + c4 * 4);
    }
  };

  if (nch > 0) {
    load_chunk(0);
    store_in();
  }
  if (nch > 1) load_chunk(1);
  __syncthreads();
  float dhr = 0.f, dc = 0.f;
  for (int ch = 0; ch < nch; ++ch) {
    const int n = min(CH, L - ch * CH);
    for (int st = 0; st < n; ++st) {
      const int s = L - 1 - ch * CH - st;
      const float* in = gin + st * IW;
      const float ig = in[u], fg = in[H + u], gg = in[2 * H + u], og = in[3 * H + u];
      const float ct = in[4 * H + u], dyv = in[5 * H + u], cp = in[6 * H + u];
      const float dh = dyv + dhr;
      const float tc = tanh_fast(ct);
      const float dcc = dc + dh * og * (1.f - tc * tc);
      const float d_i = dcc * gg * ig * (1.f - ig);
      const float d_f = dcc * cp * fg * (1.f - fg);
      const float d_g = dcc * ig * (1.f - gg * gg);
      const float d_o = dh * tc * og * (1.f - og);
      dc = dcc * fg;
      const float dgs[4] = {d_i, d_f, d_g, d_o};
      const float mine = pick4(dgs, gq);
      float* gb = gbuf + (s & 1) * G::GBUF;
      if (UP == 2 || q < 4) {
        gb[gslot] = mine;
        out[st * GW + f] = mine;
      }
      __syncthreads();
      const float* gp = gb + q * G::GP;
      // 4 chains per unit: the FMA latency, not issue, bounds one
      float p[UP][4];
#pragma unroll
      for (int k = 0; k < UP; ++k) p[k][0] = p[k][1] = p[k][2] = p[k][3] = 0.f;
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const float gv = gp[j];
#pragma unroll
        for (int k = 0; k < UP; ++k) p[k][j & 3] = fmaf(w[k][j], gv, p[k][j & 3]);
      }
      float dsum[UP];
#pragma unroll
      for (int k = 0; k < UP; ++k) dsum[k] = unit_sum<KP>((p[k][0] + p[k][1]) + (p[k][2] + p[k][3]));
      dhr = UP == 1 ? dsum[0] : (uk == 0 ? dsum[0] : dsum[UP - 1]);
    }
    __syncthreads();
    if (ch + 1 < nch) store_in();
    flush(ch);
    if (ch + 2 < nch) load_chunk(ch + 2);
    __syncthreads();
  }
}

template <int H>
int launch_fwd(const float* gx, int ldg, const float* w0, const float* w1,
               const long long* lengths, int B, int T, float* y, int ldy, float* sv,
               hipStream_t st) {
  if (ldg % 4 || ldy % 4 || ((uintptr_t)gx | (uintptr_t)y | (uintptr_t)sv) % 16)
    return ENSVS_E_ARG;
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_fwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, Geo<H>::FWD_LDS);
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_fwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::TF), Geo<H>::FWD_LDS, st,
                     gx, ldg, w0, w1, lengths, T, y, ldy, sv);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H>
int launch_bwd(const float* dy, int lddy, const float* w0, const float* w1,
               const long long* lengths, int B, int T, const float* sv, float* dg, int lddg,
               hipStream_t st) {
  if (lddy % 4 || lddg % 4 || ((uintptr_t)dy | (uintptr_t)sv | (uintptr_t)dg) % 16)
    return ENSVS_E_ARG;
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, Geo<H>::BWD_LDS);
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_bwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::TB), Geo<H>::BWD_LDS, st,
                     dy, lddy, w0, w1, lengths, T, sv, dg, lddg);
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
