// Cooperative bidirectional LSTM recurrence for the large hidden sizes (H = 256, 512: the
// MultiTrackLSTMEncoder and the decoders of the recipe-default SeparateF0 model,
// nnsvs/model.py:1435-1537, 862-869) in production (bf16 GEMM) precision.
//
// Same contract as lstm.hip's ensvs_lstm_fwd / ensvs_lstm_bwd (packed sequences, zero state,
// zero outputs past each length, saved [B*T][2][5H] = i f g o c).  W_hh (4 MB fp32 per
// direction at H = 512) does not fit one CU, and the per-step kernels of lstm.hip re-launch
// and re-read it from L2 every step (17.5 / 52 us per step forward / backward at H = 512).
// Here one launch runs every step:
//   * each direction is split over NW = H / 16 workgroups; workgroup w owns hidden units
//     [16 w, 16 w + 16) and holds their 64 gate rows of W_hh (forward) or their 16 columns
//     (backward: dh = W_hh^T dG) as MFMA A fragments in VGPRs for the whole sequence;
//   * the sequences of a tile (16 or 32) are the MFMA N dimension (one or two 16-column
//     tiles), the K dimension is split over the four waves and their partial sums are added
//     through LDS;
//   * the recurrent products run in fp16 (forward: h in [-1, 1]) / bf16 (backward: dG spans
//     many decades) with fp32 accumulation -- as the reference recipe's fp16 autocast runs its
//     cuDNN LSTM (myconfig_notuseIL.yaml:6) -- while gates, cell state and every saved value
//     stay fp32; the fp32 parity mode keeps lstm.hip's exact kernels;
//   * h_t (fp16) / dG_t (bf16) is handed to every workgroup of the direction through a
//     double-buffered slab in the caller's workspace: 16-B sc1 stores, s_waitcnt vmcnt(0) of
//     every storing wave, then one agent-scope counter add per workgroup; readers poll the
//     counter with sc1 loads and read the slab with sc1 loads only (the hand-off form of
//     MI355X_MICROARCH.md, "Hand-offs measured with sc1 loads", first row).
// Every workgroup of a tile must be resident at once (2 NW <= 64 workgroups, one per CU);
// the polls are bounded, so a grid that cannot become resident ends (flagging the error word
// of the workspace) instead of hanging.
#include <atomic>

#include "coop.h"
#include "ensvs.h"

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_;

namespace {

using namespace coop;

constexpr int PSF = 68;     // forward partial-sum row per sequence: 64 gate rows + 4 (banks)
constexpr int PSB = 20;     // backward: 16 units + 4

// S = sequences per tile: 32 (two MFMA N tiles, two cells per thread) or 16 (one N tile, one
// cell per thread).  A 16-sequence tile halves what every workgroup reads from the slab each
// step -- the backward's whole dG_t, 64 KB instead of 128 KB at H = 512, which the per-CU
// read rate from the Infinity Cache (~65 GB/s, MI355X_MICROARCH.md handoff-payload) turns
// into ~1 us per step -- at twice the workgroups; tile_seqs() picks it for small batches.
template <int H, int S> struct CGeo {
  static constexpr int NW = H / UW;       // workgroups per direction
  static constexpr int KCW = H / 128;     // forward: 32-deep K chunks per wave (K = H)
  static constexpr int KCBW = H / 32;     // backward: per wave (K = 4H)
  static constexpr int NTN = S / 16;      // MFMA N tiles
  static constexpr int NC = S * UW / NT;  // cells per compute thread
  static constexpr int FX = 2 * 2 * S * H * 2;      // forward slab bytes: [dir][buf][s][H] f16
  static constexpr int BX = 2 * 2 * S * 4 * H * 2;  // backward: [dir][buf][s][4H] bf16
  static_assert(H % 128 == 0 && (S == 16 || S == 32), "H, S");
};

// W_hh [4H][H] fp32 (both directions) -> forward A fragments
// [dir][w][wave][mt][kk][lane][8] fp16: row m = lane & 15 of tile mt is unit 16 w + 4 mt + m / 4,
// gate m % 4; k = (wave KCW + kk) 32 + 8 (lane >> 4) + j.
template <int H>
__global__ void coop_pack_fwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                     int ndir, _Float16* __restrict__ out) {
  using G = CGeo<H, 32>;
  const int n = ndir * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int kk = r % G::KCW; r /= G::KCW;
    const int mt = r % 4; r /= 4;
    const int wv = r % 4; r /= 4;
    const int w = r % G::NW, d = r / G::NW;
    const int m = lane & 15, u = w * UW + 4 * mt + m / 4, g = m % 4;
    const int k = (wv * G::KCW + kk) * 32 + 8 * (lane >> 4) + j;
    out[i] = (_Float16)(d ? w1 : w0)[(long long)(g * H + u) * H + k];
  }
}

// backward A fragments of W_hh^T [dir][w][wave][kk][lane][8] bf16: row m = lane & 15 is unit
// 16 w + m; k = n' = (wave KCBW + kk) 32 + 8 (lane >> 4) + j in the dG slab's order
// n' = 64 w' + 4 u' + g (workgroup-major, unit-major inside), i.e. gate row g H + 16 w' + u'.
template <int H>
__global__ void coop_pack_bwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                     int ndir, __bf16* __restrict__ out) {
  using G = CGeo<H, 32>;
  const int n = ndir * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int kk = r % G::KCBW; r /= G::KCBW;
    const int wv = r % 4; r /= 4;
    const int w = r % G::NW, d = r / G::NW;
    const int u = w * UW + (lane & 15);
    const int np = (wv * G::KCBW + kk) * 32 + 8 * (lane >> 4) + j;
    const int row = (np % 4) * H + (np / 64) * UW + (np % 64) / 4;
    out[i] = (__bf16)(d ? w1 : w0)[(long long)row * H + u];
  }
}

// Round 5: a fifth "service" wave per workgroup writes every step's outputs (y and the saved
// i f g o c, staged in LDS by the compute waves) with 16-B stores after the step's barriers,
// so no compute wave carries a global store in its vmcnt (ardec.hip's forward does the same;
// tools/ardec_phase_probe.py measured the stores at ~0.44 us of a 4.6 us step there).
constexpr int NTS = NT + 64;

template <int H, int S>
__global__ __launch_bounds__(NTS) void lstm_coop_fwd_kernel(
    const float* __restrict__ gx, int ldg,     // [B*T][ldg], dir d gate g unit u at d 4H + g H + u
    const f16x8* __restrict__ wp,              // packed forward fragments
    const long long* __restrict__ lengths, int B, int T,
    float* __restrict__ y, int ldy,            // [B*T][ldy], dir d at d H + u
    __bf16* __restrict__ y16, int ldy16,       // optional bf16 copy of y (the next GEMMs' operand)
    float* __restrict__ sv,                    // [B*T][2][5H]
    unsigned* __restrict__ work, Ctl c) {
  using G = CGeo<H, S>;
  constexpr int KCW = G::KCW, NW = G::NW, NTN = G::NTN, NC = G::NC;
  __shared__ __attribute__((aligned(16))) float part[4 * S * PSF];
  __shared__ __attribute__((aligned(16))) _Float16 hs[S * UW];
  __shared__ int sL[S];
  __shared__ __attribute__((aligned(16))) float st6[S * 6 * UW];  // [s][h i f g o c][u]
  const int d = blockIdx.y, w = blockIdx.x, u0 = w * UW;
  {  // this workgroup's sequence tile: sequences [S z, S z + S)
    const int s0 = blockIdx.z * S;
    B = min(S, B - s0);
    lengths += s0;
    gx += (long long)s0 * T * ldg;
    y += (long long)s0 * T * ldy;
    if (y16) y16 += (long long)s0 * T * ldy16;
    sv += (long long)s0 * T * 10 * H;
  }
  unsigned* hdr = tile_hdr(work, blockIdx.z);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < S) sL[tid] = tid < B ? (int)lengths[tid] : 0;
  __syncthreads();
  int maxL = 0;
  for (int s = 0; s < B; ++s) maxL = max(maxL, sL[s]);
  // pad_packed_sequence: this workgroup's output columns past each sequence's end are zero
  for (int s = 0; s < B; ++s) {
    const int L = sL[s];
    for (int i = tid; i < (T - L) * UW; i += NTS) {
      const long long row = (long long)s * T + L + i / UW;
      y[row * ldy + d * H + u0 + i % UW] = 0.f;
      if (y16) y16[row * ldy16 + d * H + u0 + i % UW] = (__bf16)0.f;
    }
  }
  const __amdgpu_buffer_rsrc_t xr = slab(work, gridDim.z, blockIdx.z, G::BX);

  if (wv == 4) {
    // ---------------------------------------------------------------- the service wave
    for (int t = 0; t < maxL; ++t) {
      if (t > 0) wait_count(hdr, d, (unsigned)(NW * t), c);
      lds_barrier();  // (1)
      lds_barrier();  // (2) step t's outputs staged in st6
      // S sequences x 6 rows (h i f g o c) of 16 units, 16 B per store
#pragma unroll
      for (int k4 = 0; k4 < S * 6 * UW / 4 / 64; ++k4) {
        const int gi = lane + 64 * k4, sq = gi / (6 * UW / 4), rem = gi % (6 * UW / 4);
        const int q = rem / (UW / 4), c4 = (rem % (UW / 4)) * 4;
        const f32x4 v = *(const f32x4*)&st6[(sq * 6 + q) * UW + c4];
        const int L = sq < B ? sL[sq] : 0;
        if (t < L) {
          const long long row = (long long)sq * T + (d ? L - 1 - t : t);
          float* dst = q == 0 ? y + row * ldy + d * H : sv + (row * 2 + d) * 5 * H + (q - 1) * H;
          *(f32x4*)(dst + u0 + c4) = v;
          if (q == 0 && y16) {
            bf16x4_ b;
#pragma unroll
            for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[e];
            *(bf16x4_*)(y16 + row * ldy16 + d * H + u0 + c4) = b;
          }
        }
      }
    }
    return;
  }

  f16x8 wf[4][KCW];
  {
    const f16x8* src = wp + (((long long)(d * NW + w) * 4 + wv) * 4 * KCW) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk) wf[mt][kk] = src[(mt * KCW + kk) * 64];
  }

  // cells (unit u = p & 15, sequence s = p >> 4), p = tid + 256 i
  int cs[NC], cu[NC];
  long long grow[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int p = tid + NT * i;
    cu[i] = p & 15;
    cs[i] = p >> 4;
  }
  auto in_row = [&](int i, int t) -> long long {  // clamped: always a readable row
    const int sc = min(cs[i], B - 1), L = sL[sc];
    const int tt = max(min(t, L - 1), 0);
    return (long long)sc * T + (d ? max(L - 1 - tt, 0) : tt);
  };
  float gin[NC][4], cst[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) cst[i] = 0.f;
  auto load_in = [&](int t) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      grow[i] = in_row(i, t);
      const float* src = gx + grow[i] * ldg + d * 4 * H + u0 + cu[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) gin[i][g] = src[g * H];
    }
  };
  load_in(0);

  for (int t = 0; t < maxL; ++t) {
    f32x4 acc[4][NTN];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t > 0) {
      wait_count(hdr, d, (unsigned)(NW * t), c);
      f16x8 bf[KCW][NTN];
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) {
          const int off = (((d * 2 + ((t - 1) & 1)) * S + nt * 16 + (lane & 15)) * H +
                           (wv * KCW + kk) * 32 + 8 * (lane >> 4)) * 2;
          bf[kk][nt] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, CP_SC1));
        }
      // all slab loads in flight together (one L2 round trip), then the MFMAs
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) asm volatile("" ::"v"(bf[kk][nt]));
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < NTN; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[mt][kk], bf[kk][nt], acc[mt][nt], 0, 0, 0);
    }
    // partial sums: lane holds gate rows 16 mt + 4 (lane >> 4) + r of sequence 16 nt + (lane & 15)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt)
        *(f32x4*)&part[(wv * S + nt * 16 + (lane & 15)) * PSF + 16 * mt + 4 * (lane >> 4)] = acc[mt][nt];
    lds_barrier();
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int s = cs[i], u = cu[i];
      f32x4 a = *(const f32x4*)&part[s * PSF + 4 * u];
#pragma unroll
      for (int q = 1; q < 4; ++q) a += *(const f32x4*)&part[(q * S + s) * PSF + 4 * u];
      const float ig = sigm(a[0] + gin[i][0]), fg = sigm(a[1] + gin[i][1]);
      const float gg = tanh_fast(a[2] + gin[i][2]), og = sigm(a[3] + gin[i][3]);
      const float cn = fg * cst[i] + ig * gg;
      const float h = og * tanh_fast(cn);
      const bool val = t < sL[s];
      cst[i] = cn;
      hs[s * UW + u] = (_Float16)(val ? h : 0.f);
      float* o6 = st6 + s * 6 * UW + u;
      o6[0] = h;
      o6[UW] = ig;
      o6[2 * UW] = fg;
      o6[3 * UW] = gg;
      o6[4 * UW] = og;
      o6[5 * UW] = cn;
    }
    lds_barrier();
    if (wv == 0) {  // publish h_t: S sequences x 16 units, one 16-B sc1 store per lane < 2 S
      if (lane < 2 * S) {
        const f32x4 v = *(const f32x4*)&hs[(lane >> 1) * UW + (lane & 1) * 8];
        const int off = (((d * 2 + (t & 1)) * S + (lane >> 1)) * H + u0 + (lane & 1) * 8) * 2;
        __builtin_amdgcn_raw_buffer_store_b128(v, xr, off, 0, CP_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(hdr, d, t, c);
    }
    if (t + 1 < maxL) load_in(t + 1);
  }
}

// The backward keeps its gate-gradient stores in the compute waves: with the service wave
// (round 5) it measured slower, H = 256 4.39 -> 4.73 and H = 512 6.16 -> 6.57 us per step
// (tools/lstm_coop_bench.py, profiles/r5_coop_service_wave.txt) -- its dG payload (32 KB per
// wave per step at H = 512) shares SIMD 0 with the fifth wave.
template <int H, int S>
__global__ __launch_bounds__(NT) void lstm_coop_bwd_kernel(
    const float* __restrict__ dy, int lddy,    // [B*T][lddy], grad of outputs
    const bf16x8* __restrict__ wp,             // packed backward fragments
    const long long* __restrict__ lengths, int B, int T,
    const float* __restrict__ sv,              // saved [B*T][2][5H]
    float* __restrict__ dg, int lddg,          // [B*T][lddg], dir d gate g unit u at d 4H + g H + u
    __bf16* __restrict__ dgb, int lddgb,       // optional bf16 copy of dg (either may be null)
    float* __restrict__ bpart,                 // optional [B][8H]: dg summed over each sequence
    unsigned* __restrict__ work, Ctl c) {
  using G = CGeo<H, S>;
  constexpr int KCBW = G::KCBW, NW = G::NW, G4 = 4 * H, NTN = G::NTN, NC = G::NC;
  __shared__ __attribute__((aligned(16))) float part[4 * S * PSB];
  __shared__ __attribute__((aligned(16))) __bf16 gs[S * 64];  // [s][4 u + g]
  __shared__ int sL[S];
  const int d = blockIdx.y, w = blockIdx.x, u0 = w * UW;
  {  // this workgroup's sequence tile
    const int s0 = blockIdx.z * S;
    B = min(S, B - s0);
    lengths += s0;
    dy += (long long)s0 * T * lddy;
    sv += (long long)s0 * T * 10 * H;
    if (dg) dg += (long long)s0 * T * lddg;
    if (dgb) dgb += (long long)s0 * T * lddgb;
    if (bpart) bpart += (long long)s0 * 8 * H;
  }
  unsigned* hdr = tile_hdr(work, blockIdx.z);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < S) sL[tid] = tid < B ? (int)lengths[tid] : 0;

  bf16x8 wb[KCBW];
  {
    const bf16x8* src = wp + (((long long)(d * NW + w) * 4 + wv) * KCBW) * 64 + lane;
#pragma unroll
    for (int kk = 0; kk < KCBW; ++kk) wb[kk] = src[kk * 64];
  }
  __syncthreads();
  int maxL = 0;
  for (int s = 0; s < B; ++s) maxL = max(maxL, sL[s]);
  for (int s = 0; s < B; ++s) {  // zero this workgroup's gate-gradient columns past the end
    const int L = sL[s];
    for (int i = tid; i < (T - L) * 64; i += NT) {
      const int c = i % 64;
      const long long row = (long long)s * T + L + i / 64;
      const int col = d * G4 + (c / 16) * H + u0 + c % 16;
      if (dg) dg[row * lddg + col] = 0.f;
      if (dgb) dgb[row * lddgb + col] = (__bf16)0.f;
    }
  }
  const __amdgpu_buffer_rsrc_t xr = slab(work, gridDim.z, blockIdx.z, G::BX);

  int cs[NC], cu[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int p = tid + NT * i;
    cu[i] = p & 15;
    cs[i] = p >> 4;
  }
  // processing index q of sequence s is its forward step L - 1 - q: row L-1-q (dir 0) or q
  float in[NC][7], dcs[NC], bs[NC][4];
  long long grow[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    dcs[i] = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) bs[i][g] = 0.f;
  }
  auto load_in = [&](int q) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int sc = min(cs[i], B - 1), L = sL[sc];
      const int qq = max(min(q, L - 1), 0);
      const long long rb = (long long)sc * T;
      grow[i] = rb + (d ? qq : max(L - 1 - qq, 0));
      const bool hasp = qq < L - 1;  // c at forward step L - 2 - q exists
      const long long prow = hasp ? rb + (d ? qq + 1 : L - 2 - qq) : grow[i];
      const int j = u0 + cu[i];
      const float* s5 = sv + (grow[i] * 2 + d) * 5 * H + j;
#pragma unroll
      for (int g = 0; g < 5; ++g) in[i][g] = s5[g * H];
      const float cp = sv[(prow * 2 + d) * 5 * H + 4 * H + j];
      in[i][5] = hasp ? cp : 0.f;
      in[i][6] = dy[grow[i] * lddy + d * H + j];
    }
  };
  load_in(0);

  for (int q = 0; q < maxL; ++q) {
    f32x4 acc[NTN];
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q > 0) {
      wait_count(hdr, d, (unsigned)(NW * q), c);
      bf16x8 bf[KCBW][NTN];
#pragma unroll
      for (int kk = 0; kk < KCBW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) {
          const int off = (((d * 2 + ((q - 1) & 1)) * S + nt * 16 + (lane & 15)) * G4 +
                           (wv * KCBW + kk) * 32 + 8 * (lane >> 4)) * 2;
          bf[kk][nt] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, CP_SC1));
        }
#pragma unroll
      for (int kk = 0; kk < KCBW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) asm volatile("" ::"v"(bf[kk][nt]));
#pragma unroll
      for (int kk = 0; kk < KCBW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[kk], bf[kk][nt], acc[nt], 0, 0, 0);
    }
    // lane holds dh of units 4 (lane >> 4) + r for sequence 16 nt + (lane & 15)
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
      *(f32x4*)&part[(wv * S + nt * 16 + (lane & 15)) * PSB + 4 * (lane >> 4)] = acc[nt];
    lds_barrier();
    float o[NC][4];
    bf16x4_ ob[NC];
    bool val[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int s = cs[i], u = cu[i];
      float dhr = part[s * PSB + u];
#pragma unroll
      for (int k = 1; k < 4; ++k) dhr += part[(k * S + s) * PSB + u];
      const float ig = in[i][0], fg = in[i][1], gg = in[i][2], og = in[i][3];
      const float dh = in[i][6] + dhr;
      const float tc = tanh_fast(in[i][4]);
      const float dcc = dcs[i] + dh * og * (1.f - tc * tc);
      o[i][0] = dcc * gg * ig * (1.f - ig);
      o[i][1] = dcc * in[i][5] * fg * (1.f - fg);
      o[i][2] = dcc * ig * (1.f - gg * gg);
      o[i][3] = dh * tc * og * (1.f - og);
      dcs[i] = dcc * fg;
      val[i] = q < sL[s];
      bf16x4_ nb;
#pragma unroll
      for (int g = 0; g < 4; ++g) nb[g] = (__bf16)(val[i] ? o[i][g] : 0.f);
      *(bf16x4_*)&gs[s * 64 + 4 * u] = nb;
      ob[i] = nb;
    }
    lds_barrier();
    // publish dG (S sequences x 64 values, 8 S 16-B sc1 stores) from wave 0 alone, as the
    // forward publishes h: only wave 0's memory operations gate the signal, and the other
    // waves go on to their gate-gradient stores and next inputs without a second barrier
    // (the earlier form stored from waves 0 and 1, waited vmcnt(0) in every wave -- their
    // previous step's dg stores and next inputs included -- and signalled after a barrier)
    if (wv == 0) {
#pragma unroll
      for (int k = lane; k < 8 * S; k += 64) {
        const f32x4 v = *(const f32x4*)&gs[(k >> 3) * 64 + (k & 7) * 8];
        const int off = (((d * 2 + (q & 1)) * S + (k >> 3)) * G4 + w * 64 + (k & 7) * 8) * 2;
        __builtin_amdgcn_raw_buffer_store_b128(v, xr, off, 0, CP_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(hdr, d, q, c);
    }
#pragma unroll
    for (int i = 0; i < NC; ++i)
      if (val[i]) {
        if (dg) {
          float* dst = dg + grow[i] * lddg + d * G4 + u0 + cu[i];
#pragma unroll
          for (int g = 0; g < 4; ++g) dst[g * H] = o[i][g];
        }
        if (dgb) {
          __bf16* dst = dgb + grow[i] * lddgb + d * G4 + u0 + cu[i];
#pragma unroll
          for (int g = 0; g < 4; ++g) dst[g * H] = ob[i][g];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) bs[i][g] += o[i][g];
      }
    if (q + 1 < maxL) load_in(q + 1);
  }
  if (bpart) {  // the bias gradient's per-sequence sums (b_ih and b_hh share them)
#pragma unroll
    for (int i = 0; i < NC; ++i)
      if (cs[i] < B) {
        float* dst = bpart + (long long)cs[i] * 8 * H + d * G4 + u0 + cu[i];
#pragma unroll
        for (int g = 0; g < 4; ++g) dst[g * H] = bs[i][g];
      }
  }
}

// any B: tiles of S sequences (coop.h), launched in waves of up to MAX_TILES tiles (at H = 512
// and S = 32 a wave is 8 x 64 workgroups).  Wave k owns the workspace region of its tiles --
// their headers, then their slabs -- so every launch sees the layout coop.h describes; a wave's
// tiles need only be co-resident one at a time (tiles never wait on each other), and
// consecutive waves on the stream run one after the other.
constexpr int MAX_TILES = 8;

// sequences per tile: 16 while the launch stays within 128 workgroups (H = 512: B <= 32, H = 256:
// B <= 64), else 32; ensvs_lstm_coop_set_tile_seqs forces one (A/B runs, tests)
int g_tile_seqs = 0;
int tile_seqs(int B, int H) {
  if (g_tile_seqs) return g_tile_seqs;
  return 2 * (H / UW) * ((B + 15) / 16) <= 128 ? 16 : 32;
}
inline int ntiles_s(int B, int S) { return (B + S - 1) / S; }

template <int H, int S>
long long wave_bytes() { return (long long)MAX_TILES * (HDR + CGeo<H, S>::BX); }

template <int H, int S>
int launch_fwd(const float* gx, int ldg, const void* wp, const long long* lengths, int B, int T,
               float* y, int ldy, __bf16* y16, int ldy16, float* sv, unsigned* work,
               hipStream_t st) {
  using G = CGeo<H, S>;
  const size_t st_lds = sizeof(float) * (4 * S * PSF + S * 6 * UW) + 2 * S * UW + 4 * S;
  static const bool attr = set_max_lds((const void*)lstm_coop_fwd_kernel<H, S>, st_lds);
  if (!attr) return ENSVS_E_HIP;
  const Ctl ctl = host_ctl();
  const int ntt = ntiles_s(B, S);
  for (int t0 = 0; t0 < ntt; t0 += MAX_TILES) {
    const int nt = std::min(MAX_TILES, ntt - t0);
    const long long b0 = (long long)t0 * S;
    unsigned* wk = (unsigned*)((char*)work + (t0 / MAX_TILES) * wave_bytes<H, S>());
    if (hipMemsetAsync(wk, 0, (size_t)nt * HDR, st) != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL((lstm_coop_fwd_kernel<H, S>), dim3(G::NW, 2, nt), dim3(NTS), dyn_lds(st_lds),
                       st, gx + b0 * T * ldg, ldg, (const f16x8*)wp, lengths + b0, (int)(B - b0),
                       T, y + b0 * T * ldy, ldy, y16 ? y16 + b0 * T * ldy16 : nullptr, ldy16,
                       sv + b0 * T * 10 * H, wk, ctl);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

template <int H, int S>
int launch_bwd(const float* dy, int lddy, const void* wp, const long long* lengths, int B, int T,
               const float* sv, float* dg, int lddg, __bf16* dgb, int lddgb, float* bpart,
               unsigned* work, hipStream_t st) {
  using G = CGeo<H, S>;
  const size_t st_lds = sizeof(float) * 4 * S * PSB + 2 * S * 64 + 4 * S;
  static const bool attr = set_max_lds((const void*)lstm_coop_bwd_kernel<H, S>, st_lds);
  if (!attr) return ENSVS_E_HIP;
  const Ctl ctl = host_ctl();
  const int ntt = ntiles_s(B, S);
  for (int t0 = 0; t0 < ntt; t0 += MAX_TILES) {
    const int nt = std::min(MAX_TILES, ntt - t0);
    const long long b0 = (long long)t0 * S;
    unsigned* wk = (unsigned*)((char*)work + (t0 / MAX_TILES) * wave_bytes<H, S>());
    if (hipMemsetAsync(wk, 0, (size_t)nt * HDR, st) != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL((lstm_coop_bwd_kernel<H, S>), dim3(G::NW, 2, nt), dim3(NT), dyn_lds(st_lds),
                       st, dy + b0 * T * lddy, lddy, (const bf16x8*)wp, lengths + b0,
                       (int)(B - b0), T, sv + b0 * T * 10 * H, dg ? dg + b0 * T * lddg : nullptr,
                       lddg, dgb ? dgb + b0 * T * lddgb : nullptr, lddgb,
                       bpart ? bpart + b0 * 8 * H : nullptr, wk, ctl);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

bool coop_shape(int B, int H) { return B >= 1 && (H == 256 || H == 512); }

// full waves of MAX_TILES tiles, then the last wave's tiles
long long work_bytes(int H, int B) {
  const int S = tile_seqs(B, H);
  const long long slab = H == 256 ? (S == 16 ? CGeo<256, 16>::BX : CGeo<256, 32>::BX)
                                  : (S == 16 ? CGeo<512, 16>::BX : CGeo<512, 32>::BX);
  return (long long)ntiles_s(B, S) * (HDR + slab);
}

int check_work(const void* work, long long nbytes, int H, int B) {
  if (!work || (uintptr_t)work % 256 || nbytes < work_bytes(H, B)) return ENSVS_E_ARG;
  return ENSVS_OK;
}

// failure controls of every cooperative launch (coop.h Ctl): one error word and one wall-clock
// rate per device, picked by the launching thread's current device (hipGetDevice), so a
// process driving several GPUs never points a kernel at another device's word
constexpr int MAX_DEV = 64;
std::atomic<unsigned*> g_err[MAX_DEV];
std::atomic<int> g_rate_khz[MAX_DEV];
long long g_timeout_us = 1000000;
int g_fault = 0;

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) dev = 0;
  return dev;
}

}  // namespace

coop::Ctl coop::host_ctl() {
  const int dev = current_device();
  int rate_khz = g_rate_khz[dev].load(std::memory_order_relaxed);
  if (rate_khz <= 0) {
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        rate_khz <= 0)
      rate_khz = 100000;  // 100 MHz
    g_rate_khz[dev].store(rate_khz, std::memory_order_relaxed);
  }
  return Ctl{g_err[dev].load(std::memory_order_acquire), g_timeout_us * rate_khz / 1000, g_fault};
}

ENSVS_API int ensvs_coop_set_error_word_dev(int device, unsigned* word) {
  if (device < 0 || device >= MAX_DEV || (uintptr_t)word % 4) return ENSVS_E_ARG;
  g_err[device].store(word, std::memory_order_release);
  return ENSVS_OK;
}

ENSVS_API unsigned* ensvs_coop_error_word(int device) {
  return device < 0 || device >= MAX_DEV ? nullptr : g_err[device].load(std::memory_order_acquire);
}

ENSVS_API int ensvs_coop_set_error_word(unsigned* word) {
  return ensvs_coop_set_error_word_dev(current_device(), word);
}

ENSVS_API int ensvs_coop_set_timeout_us(long long us) {
  if (us <= 0) return ENSVS_E_ARG;
  g_timeout_us = us;
  return ENSVS_OK;
}

ENSVS_API int ensvs_coop_inject_fault(int on) {
  g_fault = on ? 1 : 0;
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_coop_supported(int B, int H) { return coop_shape(B, H) ? 1 : 0; }

ENSVS_API int ensvs_lstm_coop_set_tile_seqs(int s) {
  if (s != 0 && s != 16 && s != 32) return ENSVS_E_ARG;
  g_tile_seqs = s;
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_coop_tile_seqs(int B, int H) { return coop_shape(B, H) ? tile_seqs(B, H) : 0; }

ENSVS_API long long ensvs_lstm_coop_work_bytes(int H, int B) {
  return coop_shape(B, H) ? work_bytes(H, B) : 0;
}

int coop::pack(const float* w0, const float* w1, int ndir, int H, int bwd, void* out,
               hipStream_t st) {
  if (H != 128 && H != 256 && H != 512) return ENSVS_E_SHAPE;
  if (!out || (uintptr_t)out % 16) return ENSVS_E_ARG;
  const dim3 grid(cdiv((long long)ndir * 4 * H * H, 256)), block(256);
#define COOP_PACK(HH)                                                                            \
  if (H == HH) {                                                                                 \
    if (bwd) hipLaunchKernelGGL(coop_pack_bwd_kernel<HH>, grid, block, 0, st, w0, w1, ndir, (__bf16*)out); \
    else hipLaunchKernelGGL(coop_pack_fwd_kernel<HH>, grid, block, 0, st, w0, w1, ndir, (_Float16*)out); \
  }
  COOP_PACK(128)
  COOP_PACK(256)
  COOP_PACK(512)
#undef COOP_PACK
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_coop_pack(const float* whh_f, const float* whh_r, int H, int bwd,
                                   void* out, void* stream) {
  if (H != 256 && H != 512) return ENSVS_E_SHAPE;
  return coop::pack(whh_f, whh_r, 2, H, bwd, out, (hipStream_t)stream);
}

ENSVS_API int ensvs_lstm_coop_fwd_ex(const float* gx, int ldg, const void* wpack,
                                     const long long* lengths, int B, int T, int H, float* y,
                                     int ldy, float* saved, void* y16, int ldy16, void* work,
                                     long long work_bytes, void* stream) {
  if (!coop_shape(B, H) || T <= 0 || ldg < 8 * H || ldy < 2 * H) return ENSVS_E_SHAPE;
  if (check_work(work, work_bytes, H, B) || !wpack || (uintptr_t)wpack % 16) return ENSVS_E_ARG;
  if ((uintptr_t)y % 16 || ldy % 4 || (uintptr_t)saved % 16) return ENSVS_E_ARG;  // 16-B stores
  if (y16 && ((uintptr_t)y16 % 8 || ldy16 % 4 || ldy16 < 2 * H)) return ENSVS_E_ARG;  // 8-B stores
  hipStream_t st = (hipStream_t)stream;
  unsigned* wk = (unsigned*)work;
  __bf16* yb = (__bf16*)y16;
  const bool s16 = tile_seqs(B, H) == 16;
  if (H == 256)
    return s16 ? launch_fwd<256, 16>(gx, ldg, wpack, lengths, B, T, y, ldy, yb, ldy16, saved, wk, st)
               : launch_fwd<256, 32>(gx, ldg, wpack, lengths, B, T, y, ldy, yb, ldy16, saved, wk, st);
  return s16 ? launch_fwd<512, 16>(gx, ldg, wpack, lengths, B, T, y, ldy, yb, ldy16, saved, wk, st)
             : launch_fwd<512, 32>(gx, ldg, wpack, lengths, B, T, y, ldy, yb, ldy16, saved, wk, st);
}

ENSVS_API int ensvs_lstm_coop_fwd(const float* gx, int ldg, const void* wpack,
                                  const long long* lengths, int B, int T, int H, float* y, int ldy,
                                  float* saved, void* work, long long work_bytes, void* stream) {
  return ensvs_lstm_coop_fwd_ex(gx, ldg, wpack, lengths, B, T, H, y, ldy, saved, nullptr, 0, work,
                                work_bytes, stream);
}

ENSVS_API int ensvs_lstm_coop_bwd_ex(const float* dy, int lddy, const void* wpack,
                                     const long long* lengths, int B, int T, int H,
                                     const float* saved, float* dg, int lddg, void* dgb, int lddgb,
                                     float* bpart, void* work, long long work_bytes, void* stream) {
  if (!coop_shape(B, H) || T <= 0 || lddy < 2 * H) return ENSVS_E_SHAPE;
  if ((dg && lddg < 8 * H) || (dgb && lddgb < 8 * H)) return ENSVS_E_SHAPE;
  if (!dg && !dgb) return ENSVS_E_ARG;
  if (check_work(work, work_bytes, H, B) || !wpack || (uintptr_t)wpack % 16) return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  unsigned* wk = (unsigned*)work;
  __bf16* gb = (__bf16*)dgb;
  const bool s16 = tile_seqs(B, H) == 16;
#define COOP_BWD(HH, SS) \
  launch_bwd<HH, SS>(dy, lddy, wpack, lengths, B, T, saved, dg, lddg, gb, lddgb, bpart, wk, st)
  if (H == 256) return s16 ? COOP_BWD(256, 16) : COOP_BWD(256, 32);
  return s16 ? COOP_BWD(512, 16) : COOP_BWD(512, 32);
#undef COOP_BWD
}

ENSVS_API int ensvs_lstm_coop_bwd(const float* dy, int lddy, const void* wpack,
                                  const long long* lengths, int B, int T, int H,
                                  const float* saved, float* dg, int lddg, void* work,
                                  long long work_bytes, void* stream) {
  if (!dg) return ENSVS_E_ARG;
  return ensvs_lstm_coop_bwd_ex(dy, lddy, wpack, lengths, B, T, H, saved, dg, lddg, nullptr, 0,
                                nullptr, work, work_bytes, stream);
}
