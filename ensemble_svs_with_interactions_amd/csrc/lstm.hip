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

static int g_rec_excl = 1;
int ensvs_rec_exclusive() { return g_rec_excl; }  // (common.h)

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

  static_assert(QB % 4 == 0, "bwd K-part in quads");
  float w[UP][QB];
#pragma unroll
  for (int k = 0; k < UP; ++k) {
#pragma unroll
    for (int j = 0; j < QB; ++j) w[k][j] = W[(long long)(q * QB + j) * H + grp + k * HU];
    settle(w[k]);
  }
  // UP = 1: weight rows (j, j + 1) as v_pk_fma_f32 operand pairs
  f32x2 w2[UP == 1 ? QB / 2 : 1];
  if constexpr (UP == 1) {
#pragma unroll
    for (int j = 0; j < QB; j += 2) w2[j / 2] = f32x2{w[0][j], w[0][j + 1]};
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
      // UP = 1: chains (0, 1) and (2, 3) as v_pk_fma_f32 pairs (the same fmaf sequence per
      // chain, half the VALU issue: H = 64 548 vs 629 ns/step); UP = 2 stays scalar (its
      // 128 weight registers leave no room for the pairs: 1 224 vs 1 180 ns/step packed)
      float p[UP][4];
      if constexpr (UP == 2) {
#pragma unroll
        for (int k = 0; k < UP; ++k) p[k][0] = p[k][1] = p[k][2] = p[k][3] = 0.f;
#pragma unroll
        for (int j = 0; j < QB; ++j) {
          const float gv = gp[j];
#pragma unroll
          for (int k = 0; k < UP; ++k) p[k][j & 3] = fmaf(w[k][j], gv, p[k][j & 3]);
        }
      } else {
        f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < QB; j += 4) {
          a01 = __builtin_elementwise_fma(w2[j / 2], f32x2{gp[j], gp[j + 1]}, a01);
          a23 = __builtin_elementwise_fma(w2[j / 2 + 1], f32x2{gp[j + 2], gp[j + 3]}, a23);
        }
        p[0][0] = a01.x;
        p[0][1] = a01.y;
        p[0][2] = a23.x;
        p[0][3] = a23.y;
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

// Each persistent recurrence workgroup reserves its CU's whole LDS, so no GEMM workgroup
// of a concurrent branch stream lands beside it (a co-resident GEMM stretches the
// latency-bound step): 20.8 vs 21.3 ms per training step (profiles/r2_schedule_ab.txt).
// ensvs_set_recurrence_exclusive switches it per launch (the caller's branch schedule; read
// at launch, so a captured graph keeps it).
static size_t excl_lds(size_t need) {
  return ensvs_rec_exclusive() ? std::max<size_t>(need, 160 * 1024) : need;
}

template <int H>
int launch_fwd(const float* gx, int ldg, const float* w0, const float* w1,
               const long long* lengths, int B, int T, float* y, int ldy, float* sv,
               hipStream_t st) {
  if (ldg % 4 || ldy % 4 || ((uintptr_t)gx | (uintptr_t)y | (uintptr_t)sv) % 16)
    return ENSVS_E_ARG;
  const size_t lds = excl_lds(Geo<H>::FWD_LDS);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_fwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)std::max<size_t>(lds, 160 * 1024));  // the exclusive size, whatever this launch asks
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_fwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::TF), lds, st,
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
  const size_t lds = excl_lds(Geo<H>::BWD_LDS);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)std::max<size_t>(lds, 160 * 1024));  // the exclusive size, whatever this launch asks
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_bwd_kernel<H>, dim3(B, 2), dim3(Geo<H>::TB), lds, st,
                     dy, lddy, w0, w1, lengths, T, sv, dg, lddg);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}


// ---------------------------------------------------------------------------------------
// Any hidden size (the encoders' H = 256 / 512, the bap decoder's H = 62): one launch per
// time step over all sequences and both directions.  W_hh (1-4 MB per direction in fp32)
// does not fit one CU's registers or LDS, so the step's dot products are spread over
// ceil(H/U) x 2 workgroups, each owning U hidden units (their 4 gate rows of W_hh, read
// from L2) for every sequence; the kernel boundary is the step's grid-wide barrier, and the
// previous step's h / c (forward) and dG (backward) are read back from the outputs.  A
// thread owns 4 sequences x (4 gates x U units) accumulators over one K slice (K = H
// forward, 4H backward); slices are summed through LDS, then one thread per (sequence,
// unit) applies the cell.  Sequence b's step s is its forward step s (row s forward, row
// L_b-1-s reverse); backward launch p is step s = L_b-1-p.
constexpr int SNT = 256;

__device__ __forceinline__ long long step_row(int b, int T, int L, int dir, int s) {
  return (long long)b * T + (dir ? L - 1 - s : s);
}
__device__ __forceinline__ void step_geo(int B, int& RB, int& KS) {
  RB = (B + 3) / 4;
  KS = 1;
  while (RB * KS * 2 <= SNT) KS *= 2;
}

template <int U, bool VEC>
__global__ __launch_bounds__(SNT) void lstm_step_fwd_kernel(
    const float* __restrict__ gx, int ldg, const float* __restrict__ whh0,
    const float* __restrict__ whh1, const long long* __restrict__ lengths, int B, int T, int H,
    float* __restrict__ y, int ldy, float* __restrict__ sv, int s) {
  __shared__ float part[SNT * 16 * U];  // [KS][4 RB][4][U]
  const int dir = blockIdx.y, j0 = blockIdx.x * U, tid = threadIdx.x;
  const float* W = dir ? whh1 : whh0;
  int RB, KS;
  step_geo(B, RB, KS);
  const int kc = ((H + KS - 1) / KS + 3) & ~3;
  const int BR = RB * 4;
  for (int it = tid; it < RB * KS; it += SNT) {
    const int rb = it / KS, ks = it % KS;
    const int k0 = ks * kc, k1 = min(H, k0 + kc);
    float acc[4][4][U];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[r][g][u] = 0.f;
    const float* hp[4];
    bool any = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = rb * 4 + r;
      const int L = b < B ? (int)lengths[b] : 0;
      const bool on = s > 0 && s < L;
      hp[r] = on ? y + step_row(b, T, L, dir, s - 1) * ldy + dir * H : nullptr;
      any |= on;
    }
    if (any) {
      const float* wr[4][U];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int u = 0; u < U; ++u) wr[g][u] = W + (long long)(g * H + min(j0 + u, H - 1)) * H;
      if constexpr (VEC) {
        for (int k = k0; k < k1; k += 4) {
          f32x4 hv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            hv[r] = hp[r] ? *(const f32x4*)(hp[r] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const f32x4 wv = *(const f32x4*)(wr[g][u] + k);
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[r][g][u] = fmaf(hv[r][e], wv[e], acc[r][g][u]);
            }
        }
      } else {
        for (int k = k0; k < k1; ++k) {
          float hv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) hv[r] = hp[r] ? hp[r][k] : 0.f;
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const float wv = wr[g][u][k];
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[r][g][u] = fmaf(hv[r], wv, acc[r][g][u]);
            }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int u = 0; u < U; ++u) part[((ks * BR + rb * 4 + r) * 4 + g) * U + u] = acc[r][g][u];
  }
  __syncthreads();
  const int G4 = 4 * H;
  for (int it = tid; it < B * U; it += SNT) {
    const int b = it / U, u = it % U, j = j0 + u;
    if (j >= H) continue;
    const int L = (int)lengths[b];
    if (s == 0)  // pad_packed_sequence: zero outputs past the sequence end
      for (int t = L; t < T; ++t) y[((long long)b * T + t) * ldy + dir * H + j] = 0.f;
    if (s >= L) continue;
    const long long row = step_row(b, T, L, dir, s);
    float pre[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float a = 0.f;
      for (int ks = 0; ks < KS; ++ks) a += part[((ks * BR + b) * 4 + g) * U + u];
      pre[g] = gx[row * ldg + dir * G4 + g * H + j] + a;
    }
    const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanh_fast(pre[2]), og = sigm(pre[3]);
    const float cp = s > 0 ? sv[(step_row(b, T, L, dir, s - 1) * 2 + dir) * 5 * H + 4 * H + j] : 0.f;
    const float c = fg * cp + ig * gg;
    const float h = og * tanh_fast(c);
    y[row * ldy + dir * H + j] = h;
    float* o = sv + (row * 2 + dir) * 5 * H + j;
    o[0] = ig;
    o[H] = fg;
    o[2 * H] = gg;
    o[3 * H] = og;
    o[4 * H] = c;
  }
}

template <int U, bool VEC>
__global__ __launch_bounds__(SNT) void lstm_step_bwd_kernel(
    const float* __restrict__ dy, int lddy, const float* __restrict__ whh0,
    const float* __restrict__ whh1, const long long* __restrict__ lengths, int B, int T, int H,
    const float* __restrict__ sv, float* __restrict__ dg, int lddg, float* __restrict__ dcs,
    int p) {
  __shared__ float part[SNT * 4 * U];  // [KS][4 RB][U]
  const int dir = blockIdx.y, j0 = blockIdx.x * U, tid = threadIdx.x;
  const float* W = dir ? whh1 : whh0;
  const int G4 = 4 * H;
  int RB, KS;
  step_geo(B, RB, KS);
  const int kc = ((G4 + KS - 1) / KS + 3) & ~3;
  const int BR = RB * 4;
  if (p > 0) {
    for (int it = tid; it < RB * KS; it += SNT) {
      const int rb = it / KS, ks = it % KS;
      const int k0 = ks * kc, k1 = min(G4, k0 + kc);
      float acc[4][U];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[r][u] = 0.f;
      const float* gp[4];
      bool any = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rb * 4 + r;
        const int L = b < B ? (int)lengths[b] : 0;
        const int sb = L - 1 - p;  // this launch's step; dG of step sb + 1 was the last one
        gp[r] = sb >= 0 ? dg + step_row(b, T, L, dir, sb + 1) * lddg + dir * G4 : nullptr;
        any |= sb >= 0;
      }
      if (any) {
        int jc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) jc[u] = min(j0 + u, H - 1);
        if constexpr (VEC) {
          for (int k = k0; k < k1; k += 4) {
            f32x4 gv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
              gv[r] = gp[r] ? *(const f32x4*)(gp[r] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float* wrow = W + (long long)(k + e) * H;
#pragma unroll
              for (int u = 0; u < U; ++u) {
                const float wv = wrow[jc[u]];
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[r][u] = fmaf(gv[r][e], wv, acc[r][u]);
              }
            }
          }
        } else {
          for (int k = k0; k < k1; ++k) {
            const float* wrow = W + (long long)k * H;
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const float wv = wrow[jc[u]];
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[r][u] = fmaf(gp[r] ? gp[r][k] : 0.f, wv, acc[r][u]);
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) part[(ks * BR + rb * 4 + r) * U + u] = acc[r][u];
    }
    __syncthreads();
  }
  for (int it = tid; it < B * U; it += SNT) {
    const int b = it / U, u = it % U, j = j0 + u;
    if (j >= H) continue;
    const int L = (int)lengths[b];
    if (p == 0)  // zero gate gradients past the sequence end
      for (int t = L; t < T; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) dg[((long long)b * T + t) * lddg + dir * G4 + g * H + j] = 0.f;
    const int s = L - 1 - p;
    if (s < 0) continue;
    const long long row = step_row(b, T, L, dir, s);
    float dhr = 0.f;
    if (p > 0)
      for (int ks = 0; ks < KS; ++ks) dhr += part[(ks * BR + b) * U + u];
    const float* in = sv + (row * 2 + dir) * 5 * H + j;
    const float ig = in[0], fg = in[H], gg = in[2 * H], og = in[3 * H], ct = in[4 * H];
    const float cp = s > 0 ? sv[(step_row(b, T, L, dir, s - 1) * 2 + dir) * 5 * H + 4 * H + j] : 0.f;
    float* dcp = dcs + ((long long)dir * B + b) * H + j;
    const float dc = p > 0 ? *dcp : 0.f;
    const float dh = dy[row * lddy + dir * H + j] + dhr;
    const float tc = tanh_fast(ct);
    const float dcc = dc + dh * og * (1.f - tc * tc);
    float* o = dg + row * lddg + dir * G4 + j;
    o[0] = dcc * gg * ig * (1.f - ig);
    o[H] = dcc * cp * fg * (1.f - fg);
    o[2 * H] = dcc * ig * (1.f - gg * gg);
    o[3 * H] = dh * tc * og * (1.f - og);
    *dcp = dcc * fg;
  }
}

template <int U, bool VEC>
int launch_step_fwd(const float* gx, int ldg, const float* w0, const float* w1,
                    const long long* lengths, int B, int T, int H, float* y, int ldy, float* sv,
                    hipStream_t st) {
  const dim3 grid((H + U - 1) / U, 2);
  for (int s = 0; s < T; ++s) {
    hipLaunchKernelGGL((lstm_step_fwd_kernel<U, VEC>), grid, dim3(SNT), 0, st, gx, ldg, w0, w1,
                       lengths, B, T, H, y, ldy, sv, s);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

template <int U, bool VEC>
int launch_step_bwd(const float* dy, int lddy, const float* w0, const float* w1,
                    const long long* lengths, int B, int T, int H, const float* sv, float* dg,
                    int lddg, float* dcs, hipStream_t st) {
  const dim3 grid((H + U - 1) / U, 2);
  for (int p = 0; p < T; ++p) {
    hipLaunchKernelGGL((lstm_step_bwd_kernel<U, VEC>), grid, dim3(SNT), 0, st, dy, lddy, w0, w1,
                       lengths, B, T, H, sv, dg, lddg, dcs, p);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

int g_force_step = 0;  // ensvs_lstm_set_step(1): the per-step kernels at every H (tests)
bool use_step(int H) {
  return g_force_step || !(H == 8 || H == 16 || H == 32 || H == 64 || H == 128);
}

int step_fwd(const float* gx, int ldg, const float* w0, const float* w1, const long long* lengths,
             int B, int T, int H, float* y, int ldy, float* sv, hipStream_t st) {
  if (H <= 0 || B <= 0 || T <= 0 || B > 4 * SNT) return ENSVS_E_SHAPE;
  const bool vec = H % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)y | (uintptr_t)w0 | (uintptr_t)w1) % 16 == 0;
  if (H >= 512)
    return vec ? launch_step_fwd<4, true>(gx, ldg, w0, w1, lengths, B, T, H, y, ldy, sv, st)
               : launch_step_fwd<4, false>(gx, ldg, w0, w1, lengths, B, T, H, y, ldy, sv, st);
  return vec ? launch_step_fwd<2, true>(gx, ldg, w0, w1, lengths, B, T, H, y, ldy, sv, st)
             : launch_step_fwd<2, false>(gx, ldg, w0, w1, lengths, B, T, H, y, ldy, sv, st);
}

int step_bwd(const float* dy, int lddy, const float* w0, const float* w1, const long long* lengths,
             int B, int T, int H, const float* sv, float* dg, int lddg, float* work,
             long long work_floats, hipStream_t st) {
  if (H <= 0 || B <= 0 || T <= 0 || B > 4 * SNT) return ENSVS_E_SHAPE;
  if (!work || work_floats < 2LL * B * H) return ENSVS_E_ARG;
  const bool vec = lddg % 4 == 0 && ((uintptr_t)dg % 16) == 0;
  if (H >= 512)
    return vec ? launch_step_bwd<4, true>(dy, lddy, w0, w1, lengths, B, T, H, sv, dg, lddg, work, st)
               : launch_step_bwd<4, false>(dy, lddy, w0, w1, lengths, B, T, H, sv, dg, lddg, work, st);
  return vec ? launch_step_bwd<2, true>(dy, lddy, w0, w1, lengths, B, T, H, sv, dg, lddg, work, st)
             : launch_step_bwd<2, false>(dy, lddy, w0, w1, lengths, B, T, H, sv, dg, lddg, work, st);
}

}  // namespace

ENSVS_API int ensvs_set_recurrence_exclusive(int on) {
  g_rec_excl = on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_fwd(const float* gx, int ldg, const float* whh_f, const float* whh_r,
                             const long long* lengths, int B, int T, int H, float* y, int ldy,
                             float* saved, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (use_step(H)) return step_fwd(gx, ldg, whh_f, whh_r, lengths, B, T, H, y, ldy, saved, st);
  switch (H) {
    case 8: return launch_fwd<8>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 16: return launch_fwd<16>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 32: return launch_fwd<32>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 64: return launch_fwd<64>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    case 128: return launch_fwd<128>(gx, ldg, whh_f, whh_r, lengths, B, T, y, ldy, saved, st);
    default: return ENSVS_E_SHAPE;
  }
}

ENSVS_API int ensvs_lstm_set_step(int force) {
  g_force_step = force;
  return ENSVS_OK;
}

ENSVS_API long long ensvs_lstm_bwd_work_floats(int B, int H) {
  return use_step(H) ? 2LL * B * H : 0;
}

ENSVS_API int ensvs_lstm_bwd(const float* dy, int lddy, const float* whh_f, const float* whh_r,
                             const long long* lengths, int B, int T, int H, const float* saved,
                             float* dg, int lddg, float* work, long long work_floats,
                             void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (use_step(H))
    return step_bwd(dy, lddy, whh_f, whh_r, lengths, B, T, H, saved, dg, lddg, work, work_floats, st);
  switch (H) {
    case 8: return launch_bwd<8>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 16: return launch_bwd<16>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 32: return launch_bwd<32>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 64: return launch_bwd<64>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    case 128: return launch_bwd<128>(dy, lddy, whh_f, whh_r, lengths, B, T, saved, dg, lddg, st);
    default: return ENSVS_E_SHAPE;
  }
}
