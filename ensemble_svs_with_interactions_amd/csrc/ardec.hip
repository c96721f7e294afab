// Autoregressive residual-F0 decoder of the multi-track lf0 model, forward and
// backward through the free-running chain, plus its strided depthwise
// down-sampling convolution.
//
// Replaces ResF0NonAttentiveDecoder.forward (nnsvs/acoustic_models/tacotron_f0.py:126-237)
// as configured by the recipe (prenet_layers 0, one ZoneOutCell(LSTMCell) with
// zoneout 0, out_dim 1, reduction factor 4, scaled tanh, downsample_by_conv),
// which the diffusion model runs WITHOUT teacher forcing in training
// (multistream.py:1646-1651).  Per step t of T/4:
//   p    = prev * mask_t                       (F.dropout(prev, .5, training=True), :191)
//   g    = Gx_t + w_p * p + W_hh h             (Gx_t = W_ih[:, :C] e_t + b_ih + b_hh: one GEMM)
//   c, h = LSTMCell update
//   o    = Ofx_t + W_fo[:, :H] h               (Ofx_t = W_fo[:, H:] e_t: one GEMM)
//   res  = 0.34657 tanh(o);  lf0 = (score_denorm + res - mean) / scale;  prev = lf0[r-1]
//
// One workgroup (H/16 waves) per sequence runs all T/4 steps.  Thread (u, q):
// unit u = 16*wave + (lane & 15), K-quarter q = lane >> 4.  W_hh is streamed
// from L2 each step in a lane-contiguous packed layout (1 KiB per wave
// instruction); h / dG are exchanged through double-buffered LDS.  The
// feat_out reduction maps output row r onto K-quarter lane q, so one
// __syncthreads per step suffices in both directions.
#include "coop.h"
#include "ensvs.h"

namespace {

constexpr float MAX_LF0_RATIO = 0.34657359027997264f;  // 600 * ln 2 / 1200

// WpF[w][g][i4][q][u16][e] = W[g*H + 16w + u16][q*H/4 + 4 i4 + e]
// WpB[w][i4][q][k16][e]    = W[q*H + 4 i4 + e][16w + k16]
__global__ void ardec_pack_kernel(const float* __restrict__ w, int H, float* __restrict__ wf,
                                  float* __restrict__ wb) {
  const int n = 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    {  // forward layout
      int e = i & 3, u16 = (i >> 2) & 15, q = (i >> 6) & 3;
      int rest = i >> 8;
      int i4 = rest % (H / 16);
      rest /= (H / 16);
      int g = rest & 3, wv = rest >> 2;
      wf[i] = w[(long long)(g * H + 16 * wv + u16) * H + q * (H / 4) + 4 * i4 + e];
    }
    {  // backward (transposed) layout
      int e = i & 3, k16 = (i >> 2) & 15, q = (i >> 6) & 3;
      int rest = i >> 8;
      int i4 = rest % (H / 4);
      int wv = rest / (H / 4);
      wb[i] = w[(long long)(q * H + 4 * i4 + e) * H + 16 * wv + k16];
    }
  }
}

struct ArConsts {
  float in_min, in_max, mean, scale;
};

template <int H>
__global__ __launch_bounds__(4 * H) void ardec_fwd_kernel(
    const float* __restrict__ gx, int ldgx,     // [B*Tr][ldgx]
    const float* __restrict__ ofx, int ldo,     // [B*Tr][ldo] (4 used)
    const float* __restrict__ wpf,              // packed W_hh
    const float* __restrict__ wih_p,            // [4H] prenet column of W_ih
    const float* __restrict__ wfo, int ldwfo,   // W_fo [4][ldwfo], cols [0, H)
    const float* __restrict__ score, int lds,   // raw score lf0 at score[(b*T + f)*lds]
    const float* __restrict__ mask,             // [B][Tr] scaled keep mask
    const float* __restrict__ teach, int ldt,   // teacher forcing: targets[(b*T + f)*ldt]
    int T, ArConsts k,
    float* __restrict__ lf0, float* __restrict__ res,   // [B*T]
    float* __restrict__ sg, float* __restrict__ sc, float* __restrict__ sh,  // [B*Tr][4H|H|H]
    float* __restrict__ so, float* __restrict__ sp) {   // [B*Tr][4], [B*Tr]
  constexpr int NW = H / 16, Q = H / 4;
  __shared__ __attribute__((aligned(16))) float hbuf[2][H];
  __shared__ float red[2][NW][4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int u = 16 * wv + (lane & 15), q = lane >> 4;
  const int Tr = T / 4;
  float wp[4], wo;
#pragma unroll
  for (int g = 0; g < 4; ++g) wp[g] = wih_p[g * H + u];
  wo = wfo[(long long)q * ldwfo + u];
  if (tid < H) hbuf[0][tid] = 0.f;
  float c = 0.f, prev = 0.f;
  const float den = k.in_max - k.in_min;
  const float* wbase = wpf + (long long)wv * 4 * (H / 16) * 256 + lane * 4;
  __syncthreads();
  for (int t = 0; t < Tr; ++t) {
    const long long row = (long long)b * Tr + t;
    const float p = prev * mask[row];
    const float* hc = hbuf[t & 1] + q * Q;
    float acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = gx[row * ldgx + g * H + u] + wp[g] * p;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float* wg = wbase + (long long)g * (H / 16) * 256;
#pragma unroll 4
      for (int i4 = 0; i4 < H / 16; ++i4) {
        const f32x4 w4 = *(const f32x4*)(wg + i4 * 256);
        const f32x4 h4 = *(const f32x4*)(hc + 4 * i4);
        s[g] = fmaf(w4[0], h4[0], s[g]);
        s[g] = fmaf(w4[1], h4[1], s[g]);
        s[g] = fmaf(w4[2], h4[2], s[g]);
        s[g] = fmaf(w4[3], h4[3], s[g]);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      s[g] += __shfl_xor(s[g], 16);
      s[g] += __shfl_xor(s[g], 32);
      acc[g] += s[g];
    }
    const float ig = sigmoidf_(acc[0]), fg = sigmoidf_(acc[1]);
    const float gg = tanhf(acc[2]), og = sigmoidf_(acc[3]);
    c = fg * c + ig * gg;
    const float h = og * tanhf(c);
    const float mine = q == 0 ? ig : q == 1 ? fg : q == 2 ? gg : og;
    sg[row * 4 * H + q * H + u] = mine;
    if (q == 0) {
      hbuf[(t + 1) & 1][u] = h;
      sc[row * H + u] = c;
      sh[row * H + u] = h;
    }
    // feat_out partial: lane q handles output row r = q
    float o = wo * h;
    o += __shfl_xor(o, 1);
    o += __shfl_xor(o, 2);
    o += __shfl_xor(o, 4);
    o += __shfl_xor(o, 8);
    if ((lane & 15) == 0) red[t & 1][wv][q] = o;
    __syncthreads();
    // every thread needs lf0[r = 3] for the next step; threads 0..3 emit outputs
    const int r = tid < 4 ? tid : 3;
    float ov = ofx[row * ldo + r];
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) ov += red[t & 1][w2][r];
    const float rs = MAX_LF0_RATIO * tanhf(ov);
    const long long f = (long long)b * T + 4 * t + r;
    const float sd = score[f * lds] * den + k.in_min;
    const float l = (sd + rs - k.mean) / k.scale;
    if (tid < 4) {
      lf0[f] = l;
      res[f] = rs;
      so[row * 4 + r] = ov;
    }
    if (tid == 0) sp[row] = p;
    if (teach) {
      // teacher forcing (tacotron_f0.py:156-159, 226-228): the next input is the target
      // of this step's last frame, decoder_targets[:, t] = targets[:, 4t + 3]
      prev = teach[((long long)b * T + 4 * t + 3) * ldt];
    } else {
      prev = l;  // r == 3 for tid >= 3
      prev = __shfl(prev, 3);
    }
  }
}

template <int H>
__global__ __launch_bounds__(4 * H) void ardec_bwd_kernel(
    const float* __restrict__ glf0, const float* __restrict__ gres,  // [B*T] (gres may be null)
    const float* __restrict__ wpb,              // packed transposed W_hh
    const float* __restrict__ wih_p,            // [4H]
    const float* __restrict__ wfo, int ldwfo,   // W_fo [4][ldwfo]
    const float* __restrict__ mask, int teacher, int T, ArConsts k,
    const float* __restrict__ sg, const float* __restrict__ sc, const float* __restrict__ so,
    float* __restrict__ dg,                     // [B*Tr][4H]
    float* __restrict__ do4) {                  // [B*Tr][4]
  constexpr int NW = H / 16;
  __shared__ __attribute__((aligned(16))) float gbuf[2][4 * H];
  __shared__ float red[2][NW];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int u = 16 * wv + (lane & 15), q = lane >> 4;
  const int Tr = T / 4;
  float wo[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) wo[r] = wfo[(long long)r * ldwfo + u];
  const float wpq = wih_p[q * H + u];
  const float* wbase = wpb + (long long)wv * (H / 4) * 256 + lane * 4;
  float dhr = 0.f, dc = 0.f, dprev = 0.f;
  for (int t = Tr - 1; t >= 0; --t) {
    const long long row = (long long)b * Tr + t;
    float dh = dhr;
    float d4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long f = (long long)b * T + 4 * t + r;
      float dl = glf0[f] + (r == 3 ? dprev : 0.f);
      float dr = (gres ? gres[f] : 0.f) + dl / k.scale;
      const float th = tanhf(so[row * 4 + r]);
      d4[r] = dr * MAX_LF0_RATIO * (1.f - th * th);
      dh = fmaf(wo[r], d4[r], dh);
    }
    if (tid < 4) do4[row * 4 + tid] = tid == 0 ? d4[0] : tid == 1 ? d4[1] : tid == 2 ? d4[2] : d4[3];
    const float* gp = sg + row * 4 * H + u;
    const float ig = gp[0], fg = gp[H], gg = gp[2 * H], og = gp[3 * H];
    const float ct = sc[row * H + u];
    const float cp = t > 0 ? sc[(row - 1) * H + u] : 0.f;
    const float tc = tanhf(ct);
    const float dcc = dc + dh * og * (1.f - tc * tc);
    const float d_i = dcc * gg * ig * (1.f - ig);
    const float d_f = dcc * cp * fg * (1.f - fg);
    const float d_g = dcc * ig * (1.f - gg * gg);
    const float d_o = dh * tc * og * (1.f - og);
    dc = dcc * fg;
    const float mine = q == 0 ? d_i : q == 1 ? d_f : q == 2 ? d_g : d_o;
    float* gb = gbuf[t & 1];
    gb[q * H + u] = mine;
    dg[row * 4 * H + q * H + u] = mine;
    float dpp = wpq * mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) dpp += __shfl_xor(dpp, o);
    if (lane == 0) red[t & 1][wv] = dpp;
    __syncthreads();
    float s = 0.f;
    const float* gq = gb + q * H;
#pragma unroll 4
    for (int i4 = 0; i4 < H / 4; ++i4) {
      const f32x4 w4 = *(const f32x4*)(wbase + i4 * 256);
      const f32x4 g4 = *(const f32x4*)(gq + 4 * i4);
      s = fmaf(w4[0], g4[0], s);
      s = fmaf(w4[1], g4[1], s);
      s = fmaf(w4[2], g4[2], s);
      s = fmaf(w4[3], g4[3], s);
    }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    dhr = s;
    float dp = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) dp += red[t & 1][w2];
    // teacher forcing: the step input is a target, not the previous output
    dprev = teacher ? 0.f : dp * mask[row];
  }
}

// e[b][t'][c] = bias[c] + sum_r w[c][r] * x_c[b][4t'+r]; input channels come from
// up to 3 segments (ptr, ld, nch) concatenated.
struct DsSeg {
  const float* p;
  int ld, nch;
};
struct DsArgs {
  DsSeg seg[3];
  int nseg, C, T, B;
};

__device__ __forceinline__ float ds_src(const DsArgs& a, int b, int f, int c) {
  int cc = c;
  for (int s = 0; s < a.nseg; ++s) {
    if (cc < a.seg[s].nch) return a.seg[s].p[((long long)b * a.T + f) * a.seg[s].ld + cc];
    cc -= a.seg[s].nch;
  }
  return 0.f;
}

__global__ void downsample_fwd_kernel(DsArgs a, const float* __restrict__ w,
                                      const float* __restrict__ bias, float* __restrict__ e,
                                      int lde) {
  const int Tr = a.T / 4;
  const long long n = (long long)a.B * Tr * a.C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % a.C);
    const long long bt = i / a.C;
    const int b = (int)(bt / Tr), t = (int)(bt % Tr);
    float v = bias[c];
#pragma unroll
    for (int r = 0; r < 4; ++r) v = fmaf(w[c * 4 + r], ds_src(a, b, 4 * t + r, c), v);
    e[bt * lde + c] = v;
  }
}

// d x[b][4t'+r][c] = w[c][r] * de[b][t'][c] for the first `nout` channels.
__global__ void downsample_dgrad_kernel(const float* __restrict__ de, int lde,
                                        const float* __restrict__ w, int B, int T, int nout,
                                        float* __restrict__ dx, int lddx) {
  const long long n = (long long)B * T * nout;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % nout);
    const long long bf = i / nout;
    const int f = (int)(bf % T);
    const long long b = bf / T;
    const long long row = b * (T / 4) + f / 4;
    dx[bf * lddx + c] = w[c * 4 + (f & 3)] * de[row * lde + c];
  }
}

// dw[c][r] (+)= sum de[.][c] x_c[4t'+r], dbias[c] (+)= sum de[.][c]; one block per channel.
__global__ void downsample_wgrad_kernel(DsArgs a, const float* __restrict__ de, int lde,
                                        float* __restrict__ dw, float* __restrict__ db) {
  const int c = blockIdx.x;
  const int Tr = a.T / 4;
  const long long n = (long long)a.B * Tr;
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    const int b = (int)(i / Tr), t = (int)(i % Tr);
    const float g = de[i * lde + c];
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] = fmaf(g, ds_src(a, b, 4 * t + r, c), s[r]);
    s[4] += g;
  }
  __shared__ float red[5][256];
#pragma unroll
  for (int j = 0; j < 5; ++j) red[j][threadIdx.x] = s[j];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
#pragma unroll
      for (int j = 0; j < 5; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x < 4) dw[c * 4 + threadIdx.x] += red[threadIdx.x][0];
  if (threadIdx.x == 4) db[c] += red[4][0];
}

// The decoder workgroup reserves its CU's LDS (lstm.hip ensvs_rec_exclusive,
// ensvs_set_recurrence_exclusive)
static size_t ar_excl_lds() {
  return ensvs_rec_exclusive() ? 96 * 1024 : 0;  // + the static LDS: no 64 KB GEMM workgroup fits beside it
}

template <int H>
int fwd_launch(const float* gx, int ldgx, const float* ofx, int ldo, const float* wpf,
               const float* wih_p, const float* wfo, int ldwfo, const float* score, int lds,
               const float* mask, const float* teach, int ldt, int B, int T, ArConsts k,
               float* lf0, float* res, float* sg, float* sc, float* sh, float* so, float* sp,
               hipStream_t st) {
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)ardec_fwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(ardec_fwd_kernel<H>, dim3(B), dim3(4 * H), ar_excl_lds(), st, gx, ldgx, ofx, ldo, wpf,
                     wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, T, k, lf0, res, sg, sc, sh,
                     so, sp);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H>
int bwd_launch(const float* glf0, const float* gres, const float* wpb, const float* wih_p,
               const float* wfo, int ldwfo, const float* mask, int teacher, int B, int T,
               ArConsts k, const float* sg, const float* sc, const float* so, float* dg,
               float* do4, hipStream_t st) {
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)ardec_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(ardec_bwd_kernel<H>, dim3(B), dim3(4 * H), ar_excl_lds(), st, glf0, gres, wpb, wih_p, wfo,
                     ldwfo, mask, teacher, T, k, sg, sc, so, dg, do4);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}


// ------------------------------------------------------------------ cooperative decoder
// Production (bf16 GEMM) precision at H in {128, 256}, any B: the per-sequence kernels above
// stream the 1 MB fp32 W_hh from L2 every step (8.7 us per step at H = 256).  All sequences
// step in lockstep on the same W_hh, so here the recurrence is one MFMA product per step,
// W_hh . [h_1 .. h_B] (N = the sequences), split over NW = H/16 workgroups that keep their 64
// gate rows (forward, fp16) or 16 columns of W_hh^T (backward, bf16) in VGPRs for the whole
// launch -- the lstm_coop.hip scheme with one direction.  The AR feedback needs no extra hop:
//   forward:  each workgroup publishes, with its 16 units of h_t (fp16), its fp32 partial sums
//             of feat_out W_fo[r, :H] h_t (r = 0..3); every workgroup then forms o_t, lf0_t and
//             the next prenet input p_{t+1} = lf0_t[3] * mask itself from the 16 partials;
//   backward: with its 64 gate gradients (bf16) each workgroup publishes its fp32 partial of
//             w_p . dG_t, from which every workgroup forms d prev and the feat_out gradients.
// Gates, cell state and every saved value stay fp32 (the recurrent products in fp16 / bf16 as
// the recipe's fp16 autocast runs the LSTMCell, myconfig_notuseIL.yaml:6); the fp32 parity
// mode keeps the exact kernels above.
// S = sequences per tile: 32 (two MFMA N tiles, two cells per compute thread) or 16 (one N
// tile, one cell per thread: half the slab bytes every workgroup reads per step, at twice the
// workgroups); ar_tile_seqs() picks it per batch.
template <int H, int S> struct ArGeo {
  static constexpr int NW = H / coop::UW, KCW = H / 128, KCBW = H / 32;
  static constexpr int NTN = S / 16, NC = S * coop::UW / coop::NT;
  static constexpr int FH = S * H * 2;           // forward slab per buffer: h [s][H] fp16
  static constexpr int FBUF = FH + S * NW * 16;  // + feat_out partials [w][s][4] fp32
  static constexpr int BG = S * 4 * H * 2;       // backward per buffer: dG [s][4H] bf16
  static constexpr int BBUF = BG + S * NW * 4;   // + prenet partials [s][w] fp32
  static constexpr int SLAB = 2 * (FBUF > BBUF ? FBUF : BBUF);  // one tile's double buffer
  static_assert(H % 128 == 0 && NW % 4 == 0 && (S == 16 || S == 32), "H, S");
};

constexpr int AR_PSF = 68;  // forward partial-sum row per sequence: 64 gate rows + 4 (banks)
constexpr int AR_PSB = 20;  // backward: 16 units + 4

// Forward, with a fifth "service" wave per workgroup (round 5, tools/ardec_phase_probe.py):
// the four compute waves run the recurrent product and the cell update and issue no global
// store; the service wave forms step t-1's outputs from the published feat_out partials (its
// reducer lanes, one per sequence: lf0, residual, o, and the next input p, which the compute
// waves read from LDS) and writes every saved value of step t (i f g o c h, staged in LDS by
// the compute waves) with 16-B stores after the step's second barrier.  Its stores never sit
// in a compute wave's vmcnt, and the reduction no longer lengthens compute wave 0's step
// (probe: 4.57 us per AR step with both in the compute waves, 4.13 without the stores, 3.71
// without the reduction).
constexpr int AR_NTS = coop::NT + 64;

template <int H, int S>
__global__ __launch_bounds__(AR_NTS) void ardec_coop_fwd_kernel(
    const float* __restrict__ gx, int ldgx, const float* __restrict__ ofx, int ldo,
    const f16x8* __restrict__ wp, const float* __restrict__ wih_p,
    const float* __restrict__ wfo, int ldwfo, const float* __restrict__ score, int lds,
    const float* __restrict__ mask, const float* __restrict__ teach, int ldt, int B, int T,
    ArConsts k, float* __restrict__ lf0, float* __restrict__ res, float* __restrict__ sg,
    float* __restrict__ sc, float* __restrict__ sh, float* __restrict__ so,
    float* __restrict__ sp, unsigned* __restrict__ work, coop::Ctl c) {
  using namespace coop;
  using G = ArGeo<H, S>;
  constexpr int KCW = G::KCW, NW = G::NW, NTN = G::NTN, NC = G::NC;
  __shared__ __attribute__((aligned(16))) float part[4 * S * AR_PSF];
  __shared__ __attribute__((aligned(16))) _Float16 hs[S * UW];
  __shared__ __attribute__((aligned(16))) float ops[S * 4];
  __shared__ float pv[S];
  __shared__ __attribute__((aligned(16))) float sv6[S * 6 * UW];  // [s][i f g o c h][u]
  const int w = blockIdx.x, u0 = w * UW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool service = wv == 4;
  const int Tr = T / 4;
  {  // this workgroup's sequence tile (blockIdx.y): sequences [32 y, 32 y + 32)
    const int s0 = blockIdx.y * S;
    B = min(S, B - s0);
    const long long r = (long long)s0 * Tr, f = (long long)s0 * T;
    gx += r * ldgx;
    ofx += r * ldo;
    score += f * lds;
    mask += r;
    if (teach) teach += f * ldt;
    lf0 += f;
    res += f;
    sg += r * 4 * H;
    sc += r * H;
    sh += r * H;
    so += r * 4;
    sp += r;
  }
  unsigned* hdr = tile_hdr(work, blockIdx.y);
  const float den = k.in_max - k.in_min;
  const __amdgpu_buffer_rsrc_t xr = slab(work, gridDim.y, blockIdx.y, G::SLAB);

  if (service) {
    // ---------------------------------------------------------------- the service wave
    // reducer lane `lane` < S owns sequence `lane`: the inputs of step t-1's outputs and p_t
    const int rsq = min(lane, B - 1);
    const bool red = lane < S;
    const bool rw = red && lane < B && w == 0;  // writes the per-sequence outputs
    float rofx[4], rsd[4], rmask = 0.f, rteach = 0.f;
    auto load_red = [&](int t) {  // ofx / score of step t - 1, mask of step t
      if (red) {
        const long long row = (long long)rsq * Tr + max(t - 1, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          rofx[r] = ofx[row * ldo + r];
          rsd[r] = score[((long long)rsq * T + 4 * max(t - 1, 0) + r) * lds];
        }
        if (t < Tr) rmask = mask[(long long)rsq * Tr + t];
        if (teach) rteach = teach[((long long)rsq * T + 4 * max(t - 1, 0) + 3) * ldt];
      }
    };
    // step t-1's outputs from the published feat_out partials (slab layout [w][s][4]); lf0[3]
    auto reduce_out = [&](int t, int base) -> float {
      f32x4 op[NW];
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) op[w2] = ld16(xr, base + G::FH + (w2 * S + lane) * 16);
      float l3 = 0.f;
      const long long row = (long long)rsq * Tr + t - 1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float ov = rofx[r];
#pragma unroll
        for (int w2 = 0; w2 < NW; ++w2) ov += op[w2][r];
        // the exp-based tanh of the cell update (on the step's critical path; libm tanhf
        // added ~0.1 us per AR step): |error| ~1e-7, the exact kernel keeps tanhf
        const float rs = MAX_LF0_RATIO * tanh_fast(ov);
        const float sd = rsd[r] * den + k.in_min;
        const float l = (sd + rs - k.mean) / k.scale;
        if (rw) {
          const long long f = (long long)rsq * T + 4 * (t - 1) + r;
          lf0[f] = l;
          res[f] = rs;
          so[row * 4 + r] = ov;
        }
        l3 = l;
      }
      return l3;
    };
    load_red(0);
    for (int t = 0; t < Tr; ++t) {
      float l3 = 0.f;
      if (t > 0) {
        wait_count(hdr, 0, (unsigned)(NW * t), c);
        if (red) l3 = reduce_out(t, ((t - 1) & 1) * G::FBUF);
      }
      if (red) {
        // the next input: the last frame of step t-1, or the target there (teacher forcing);
        // prev = 0 before the first step
        const float p = (t == 0 ? 0.f : (teach ? rteach : l3)) * rmask;
        pv[lane] = p;
        if (rw) sp[(long long)rsq * Tr + t] = p;
      }
      lds_barrier();  // (1) p of every sequence in LDS
      lds_barrier();  // (2) step t's saved values in sv6
      // step t's saved values: 32 sequences x 6 rows of 16 units, 16 B per store
#pragma unroll
      for (int k4 = 0; k4 < S * 6 * UW / 4 / 64; ++k4) {
        const int gi = lane + 64 * k4, sq = gi / (6 * UW / 4), rem = gi % (6 * UW / 4);
        const int q = rem / (UW / 4), c4 = (rem % (UW / 4)) * 4;
        const f32x4 v = *(const f32x4*)&sv6[(sq * 6 + q) * UW + c4];
        if (sq < B) {
          const long long row = (long long)sq * Tr + t;
          float* dst = q < 4 ? sg + row * 4 * H + q * H : (q == 4 ? sc : sh) + row * H;
          *(f32x4*)(dst + u0 + c4) = v;
        }
      }
      load_red(t + 1);
    }
    if (w == 0) {  // the last step's outputs
      wait_count(hdr, 0, (unsigned)(NW * Tr), c);
      if (red) reduce_out(Tr, ((Tr - 1) & 1) * G::FBUF);
    }
    return;
  }

  // ------------------------------------------------------------------ the compute waves
  f16x8 wf[4][KCW];
  {
    const f16x8* src = wp + (((long long)w * 4 + wv) * 4 * KCW) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk) wf[mt][kk] = src[(mt * KCW + kk) * 64];
  }
  // cells (unit u = p & 15, sequence s = p >> 4), p = tid + 256 i: 16 lanes per sequence
  int cs[NC], cu[NC];
  float wpc[NC][4], woc[NC][4];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int p = tid + NT * i;
    cu[i] = p & 15;
    cs[i] = p >> 4;
#pragma unroll
    for (int g = 0; g < 4; ++g) wpc[i][g] = wih_p[g * H + u0 + cu[i]];
#pragma unroll
    for (int r = 0; r < 4; ++r) woc[i][r] = wfo[(long long)r * ldwfo + u0 + cu[i]];
  }
  float gin[NC][4], cst[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) cst[i] = 0.f;
  auto load_in = [&](int t) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const float* src = gx + ((long long)min(cs[i], B - 1) * Tr + t) * ldgx + u0 + cu[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) gin[i][g] = src[g * H];
    }
  };
  load_in(0);

  for (int t = 0; t < Tr; ++t) {
    f32x4 acc[4][NTN];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t > 0) {
      wait_count(hdr, 0, (unsigned)(NW * t), c);
      const int base = ((t - 1) & 1) * G::FBUF;
      f16x8 bf[KCW][NTN];
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
          bf[kk][nt] = __builtin_bit_cast(
              f16x8, ld16(xr, ((nt * 16 + (lane & 15)) * H + (wv * KCW + kk) * 32 + 8 * (lane >> 4)) * 2 + base));
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
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt)
        *(f32x4*)&part[(wv * S + nt * 16 + (lane & 15)) * AR_PSF + 16 * mt + 4 * (lane >> 4)] = acc[mt][nt];
    lds_barrier();  // (1)
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int s = cs[i], u = cu[i];
      f32x4 a = *(const f32x4*)&part[s * AR_PSF + 4 * u];
#pragma unroll
      for (int q = 1; q < 4; ++q) a += *(const f32x4*)&part[(q * S + s) * AR_PSF + 4 * u];
      const float p = pv[s];
      float pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) pre[g] = fmaf(wpc[i][g], p, gin[i][g]) + a[g];
      const float ig = sigm(pre[0]), fg = sigm(pre[1]);
      const float gg = tanh_fast(pre[2]), og = sigm(pre[3]);
      const float cn = fg * cst[i] + ig * gg;
      const float h = og * tanh_fast(cn);
      cst[i] = cn;
      const bool val = s < B;
      hs[s * UW + u] = (_Float16)(val ? h : 0.f);
      f32x4 ov;
#pragma unroll
      for (int r = 0; r < 4; ++r) ov[r] = sum16(woc[i][r] * (val ? h : 0.f));
      if (u == 0) *(f32x4*)&ops[s * 4] = ov;
      float* o6 = sv6 + s * 6 * UW + u;
      o6[0] = ig;
      o6[UW] = fg;
      o6[2 * UW] = gg;
      o6[3 * UW] = og;
      o6[4 * UW] = cn;
      o6[5 * UW] = h;
    }
    lds_barrier();  // (2)
    if (wv == 0) {  // publish h_t (32 sequences x 16 units) and the feat_out partials
      const int base = (t & 1) * G::FBUF;
      if (lane < 2 * S)
        st16(xr, base + ((lane >> 1) * H + u0 + (lane & 1) * 8) * 2,
             *(const f32x4*)&hs[(lane >> 1) * UW + (lane & 1) * 8]);
      if (lane < S) st16(xr, base + G::FH + (w * S + lane) * 16, *(const f32x4*)&ops[lane * 4]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(hdr, 0, t, c);
    }
    if (t + 1 < Tr) load_in(t + 1);
  }
  if (w == 0) wait_count(hdr, 0, (unsigned)(NW * Tr), c);  // (the service wave's last outputs)
}

// Backward, with the forward's service wave: it forms d o_t (the feat_out output gradient,
// tanhf of the saved o) and d prev from the published prenet partials (reducer lanes, one
// per sequence) and writes the gate gradients dG_t (staged in LDS by the compute waves) and
// d o_t with 16-B stores after the step's barriers; the compute waves run W_hh^T dG, the cell
// backward and the dG hand-off, and issue no other global store.
template <int H, int S>
__global__ __launch_bounds__(AR_NTS) void ardec_coop_bwd_kernel(
    const float* __restrict__ glf0, const float* __restrict__ gres,
    const bf16x8* __restrict__ wp, const float* __restrict__ wih_p,
    const float* __restrict__ wfo, int ldwfo, const float* __restrict__ mask, int teacher, int B,
    int T, ArConsts k, const float* __restrict__ sg, const float* __restrict__ sc,
    const float* __restrict__ so, float* __restrict__ dg, float* __restrict__ do4,
    unsigned* __restrict__ work, coop::Ctl c) {
  using namespace coop;
  using G = ArGeo<H, S>;
  constexpr int KCBW = G::KCBW, NW = G::NW, NTN = G::NTN, NC = G::NC;
  __shared__ __attribute__((aligned(16))) float part[4 * S * AR_PSB];
  __shared__ __attribute__((aligned(16))) __bf16 gs[S * 64];  // [s][4 u + g]
  __shared__ float d4s[S * 4];
  __shared__ float dps[S];
  __shared__ __attribute__((aligned(16))) float dg4[S * 4 * UW];  // [s][g][u]
  const int w = blockIdx.x, u0 = w * UW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Tr = T / 4;
  {  // this workgroup's sequence tile (blockIdx.y)
    const int s0 = blockIdx.y * S;
    B = min(S, B - s0);
    const long long r = (long long)s0 * Tr, f = (long long)s0 * T;
    glf0 += f;
    if (gres) gres += f;
    mask += r;
    sg += r * 4 * H;
    sc += r * H;
    so += r * 4;
    dg += r * 4 * H;
    do4 += r * 4;
  }
  unsigned* hdr = tile_hdr(work, blockIdx.y);
  const __amdgpu_buffer_rsrc_t xr = slab(work, gridDim.y, blockIdx.y, G::SLAB);

  if (wv == 4) {
    // ---------------------------------------------------------------- the service wave
    const int rsq = min(lane, B - 1);
    const bool red = lane < S;
    const bool rw = red && lane < B && w == 0;
    // Step inputs two steps ahead (steps run t = Tr-1 .. 0): at the end of step t, behind its
    // dG stores, the inputs of step t-1 -- loaded (n*) at the end of step t+1 -- are taken,
    // with 1 - tanh^2 of the saved o (c1), and the loads of step t-2 are issued.  That load has
    // landed by then, and the wait for it (vmcnt counts loads and stores in issue order) does
    // not cover the stores.  tanhf after the hand-off wait lengthened every step; formed right
    // after a load issued behind the stores, it stalled the service wave until they drained.
    float ngl[4], ngr[4], nso[4], nmask = 0.f;
    float rgl[4], rgr[4], c1[4], rmask = 0.f;
    auto load_red = [&](int t) {  // output grads / saved o of step t, mask of step t + 1
      if (red) {
        const long long row = (long long)rsq * Tr + t;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long f = (long long)rsq * T + 4 * t + r;
          ngl[r] = glf0[f];
          ngr[r] = gres ? gres[f] : 0.f;
          nso[r] = so[row * 4 + r];
        }
        nmask = t + 1 < Tr ? mask[row + 1] : 0.f;
      }
    };
    auto take = [&]() {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rgl[r] = ngl[r];
        rgr[r] = ngr[r];
        const float th = tanhf(nso[r]);
        c1[r] = 1.f - th * th;
      }
      rmask = nmask;
    };
    load_red(Tr - 1);
    take();
    if (Tr > 1) load_red(Tr - 2);
    for (int q = 0; q < Tr; ++q) {
      const int t = Tr - 1 - q;
      float dprev = 0.f;
      if (q > 0) {
        wait_count(hdr, 0, (unsigned)(NW * q), c);
        if (red && !teacher) {
          const int base = ((q - 1) & 1) * G::BBUF;
          f32x4 pp[NW / 4];
#pragma unroll
          for (int j = 0; j < NW / 4; ++j) pp[j] = ld16(xr, base + G::BG + (lane * NW + 4 * j) * 4);
          float dp = 0.f;
#pragma unroll
          for (int j = 0; j < NW / 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) dp += pp[j][e];
          dprev = dp * rmask;  // p_{t+1} = lf0_t[3] * mask_{t+1}
        }
      }
      float d4[4];
      if (red) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dl = rgl[r] + (r == 3 ? dprev : 0.f);
          const float dr = rgr[r] + dl / k.scale;
          d4[r] = dr * MAX_LF0_RATIO * c1[r];
          d4s[lane * 4 + r] = d4[r];
        }
        if (rw) *(f32x4*)(do4 + ((long long)rsq * Tr + t) * 4) = f32x4{d4[0], d4[1], d4[2], d4[3]};
      }
      lds_barrier();  // (1) d o_t in LDS
      lds_barrier();  // (2) dG_t staged
      lds_barrier();  // (3) dG_t published
      // dG_t: 32 sequences x 4 gates x 16 units, 16 B per store
#pragma unroll
      for (int k4 = 0; k4 < S * 4 * UW / 4 / 64; ++k4) {
        const int gi = lane + 64 * k4, sq = gi / UW, g = (gi / (UW / 4)) % 4, c4 = (gi % (UW / 4)) * 4;
        const f32x4 v = *(const f32x4*)&dg4[(sq * 4 + g) * UW + c4];
        if (sq < B) *(f32x4*)(dg + ((long long)sq * Tr + t) * 4 * H + g * H + u0 + c4) = v;
      }
      if (t > 0) {
        take();
        if (t > 1) load_red(t - 2);
      }
    }
    return;
  }

  // ------------------------------------------------------------------ the compute waves
  bf16x8 wb[KCBW];
  {
    const bf16x8* src = wp + (((long long)w * 4 + wv) * KCBW) * 64 + lane;
#pragma unroll
    for (int kk = 0; kk < KCBW; ++kk) wb[kk] = src[kk * 64];
  }
  int cs[NC], cu[NC];
  float wo[NC][4], wpg[NC][4];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int p = tid + NT * i;
    cu[i] = p & 15;
    cs[i] = p >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) wo[i][r] = wfo[(long long)r * ldwfo + u0 + cu[i]];
#pragma unroll
    for (int g = 0; g < 4; ++g) wpg[i][g] = wih_p[g * H + u0 + cu[i]];
  }
  float in[NC][6], dcs[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) dcs[i] = 0.f;
  auto load_in = [&](int t) {  // saved i f g o, c_t, c_{t-1} of step t
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long long row = (long long)min(cs[i], B - 1) * Tr + t;
      const int j = u0 + cu[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) in[i][g] = sg[row * 4 * H + g * H + j];
      in[i][4] = sc[row * H + j];
      in[i][5] = t > 0 ? sc[(row - 1) * H + j] : 0.f;
    }
  };
  load_in(Tr - 1);

  for (int q = 0; q < Tr; ++q) {
    const int t = Tr - 1 - q;
    f32x4 acc[NTN];
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q > 0) {
      wait_count(hdr, 0, (unsigned)(NW * q), c);
      const int base = ((q - 1) & 1) * G::BBUF;
      bf16x8 bf[KCBW][NTN];
#pragma unroll
      for (int kk = 0; kk < KCBW; ++kk)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
          bf[kk][nt] = __builtin_bit_cast(
              bf16x8, ld16(xr, ((nt * 16 + (lane & 15)) * 4 * H + (wv * KCBW + kk) * 32 + 8 * (lane >> 4)) * 2 + base));
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
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
      *(f32x4*)&part[(wv * S + nt * 16 + (lane & 15)) * AR_PSB + 4 * (lane >> 4)] = acc[nt];
    lds_barrier();  // (1)
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int s = cs[i], u = cu[i];
      float dh = part[s * AR_PSB + u];
#pragma unroll
      for (int kq = 1; kq < 4; ++kq) dh += part[(kq * S + s) * AR_PSB + u];
#pragma unroll
      for (int r = 0; r < 4; ++r) dh = fmaf(wo[i][r], d4s[s * 4 + r], dh);
      const float ig = in[i][0], fg = in[i][1], gg = in[i][2], og = in[i][3];
      const float tc = tanh_fast(in[i][4]);
      const float dcc = dcs[i] + dh * og * (1.f - tc * tc);
      float o[4];
      o[0] = dcc * gg * ig * (1.f - ig);
      o[1] = dcc * in[i][5] * fg * (1.f - fg);
      o[2] = dcc * ig * (1.f - gg * gg);
      o[3] = dh * tc * og * (1.f - og);
      dcs[i] = dcc * fg;
      const bool val = s < B;
      bf16x4 nb;
      float pp = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        nb[g] = (__bf16)(val ? o[g] : 0.f);
        pp = fmaf(wpg[i][g], o[g], pp);
        dg4[(s * 4 + g) * UW + u] = o[g];
      }
      *(bf16x4*)&gs[s * 64 + 4 * u] = nb;
      pp = sum16(val ? pp : 0.f);
      if (u == 0) dps[s] = pp;
    }
    lds_barrier();  // (2)
    {  // publish dG_t (32 sequences x 64 values) and the prenet partials
      const int base = (q & 1) * G::BBUF;
      if (tid < 8 * S)
        st16(xr, base + ((tid >> 3) * 4 * H + w * 64 + (tid & 7) * 8) * 2,
             *(const f32x4*)&gs[(tid >> 3) * 64 + (tid & 7) * 8]);
      if (tid < S) st4(xr, base + G::BG + (tid * NW + w) * 4, dps[tid]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();  // (3)
      if (tid == 0) signal(hdr, 0, q, c);
    }
    if (t > 0) load_in(t - 1);
  }
}

// any B: tiles of S sequences in waves of up to AR_MAX_TILES tiles per launch (at H = 256 and
// S = 32 a wave is 16 x 8 workgroups); wave k owns its tiles' workspace region (headers, then
// slabs), as lstm_coop.hip's waves do
constexpr int AR_MAX_TILES = 8;

// sequences per tile: 16 when that takes no more workgroups than tiles of 32 (B <= 16), else 32.
// At the bench's 30 pairs x 1024 frames 16-sequence tiles run the AR step in 2.79 / 3.24 us
// instead of 3.43 / 4.41 (forward / backward) but hold 32 CUs instead of 16 for the decoder's
// ~2 ms, and the training step measured 14.24 vs 13.97 ms (profiles/r5_ar_tile_ab.txt): there
// the decoder is off the critical path, and its CUs are worth more to the concurrent DiffNet
// GEMMs.  ensvs_ardec_coop_set_tile_seqs forces one (A/B runs, tests).
int g_ar_tile_seqs = 0;
int ar_tile_seqs(int B, int H) {
  (void)H;
  if (g_ar_tile_seqs) return g_ar_tile_seqs;
  return B <= 16 ? 16 : 32;
}

template <int H, int S>
long long ar_wave_bytes() { return (long long)AR_MAX_TILES * (coop::HDR + ArGeo<H, S>::SLAB); }

template <int H, int S>
int coop_fwd_launch(const float* gx, int ldgx, const float* ofx, int ldo, const void* wp,
                    const float* wih_p, const float* wfo, int ldwfo, const float* score, int lds,
                    const float* mask, const float* teach, int ldt, int B, int T, ArConsts k,
                    float* lf0, float* res, float* sg, float* sc, float* sh, float* so, float* sp,
                    unsigned* work, hipStream_t st) {
  const size_t st_lds = sizeof(float) * (4 * S * AR_PSF + S * 5 + S * 6 * coop::UW) +
                        2 * S * coop::UW;
  static const bool attr = coop::set_max_lds((const void*)ardec_coop_fwd_kernel<H, S>, st_lds);
  if (!attr) return ENSVS_E_HIP;
  const coop::Ctl ctl = coop::host_ctl();
  const int ntt = (B + S - 1) / S, Tr = T / 4;
  for (int t0 = 0; t0 < ntt; t0 += AR_MAX_TILES) {
    const int nt = std::min(AR_MAX_TILES, ntt - t0);
    const long long b0 = (long long)t0 * S, r = b0 * Tr, f = b0 * T;
    unsigned* wk = (unsigned*)((char*)work + (t0 / AR_MAX_TILES) * ar_wave_bytes<H, S>());
    if (hipMemsetAsync(wk, 0, (size_t)nt * coop::HDR, st) != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL((ardec_coop_fwd_kernel<H, S>), dim3(ArGeo<H, S>::NW, nt), dim3(AR_NTS),
                       coop::dyn_lds(st_lds), st, gx + r * ldgx, ldgx, ofx + r * ldo, ldo,
                       (const f16x8*)wp, wih_p, wfo, ldwfo, score + f * lds, lds, mask + r,
                       teach ? teach + f * ldt : teach, ldt, (int)(B - b0), T, k, lf0 + f, res + f,
                       sg + r * 4 * H, sc + r * H, sh + r * H, so + r * 4, sp + r, wk, ctl);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

template <int H, int S>
int coop_bwd_launch(const float* glf0, const float* gres, const void* wp, const float* wih_p,
                    const float* wfo, int ldwfo, const float* mask, int teacher, int B, int T,
                    ArConsts k, const float* sg, const float* sc, const float* so, float* dg,
                    float* do4, unsigned* work, hipStream_t st) {
  const size_t st_lds = sizeof(float) * (4 * S * AR_PSB + S * 5 + S * 4 * coop::UW) + 2 * S * 64;
  static const bool attr = coop::set_max_lds((const void*)ardec_coop_bwd_kernel<H, S>, st_lds);
  if (!attr) return ENSVS_E_HIP;
  const coop::Ctl ctl = coop::host_ctl();
  const int ntt = (B + S - 1) / S, Tr = T / 4;
  for (int t0 = 0; t0 < ntt; t0 += AR_MAX_TILES) {
    const int nt = std::min(AR_MAX_TILES, ntt - t0);
    const long long b0 = (long long)t0 * S, r = b0 * Tr, f = b0 * T;
    unsigned* wk = (unsigned*)((char*)work + (t0 / AR_MAX_TILES) * ar_wave_bytes<H, S>());
    if (hipMemsetAsync(wk, 0, (size_t)nt * coop::HDR, st) != hipSuccess) return ENSVS_E_HIP;
    hipLaunchKernelGGL((ardec_coop_bwd_kernel<H, S>), dim3(ArGeo<H, S>::NW, nt), dim3(AR_NTS),
                       coop::dyn_lds(st_lds), st, glf0 + f, gres ? gres + f : gres,
                       (const bf16x8*)wp, wih_p, wfo, ldwfo, mask + r, teacher, (int)(B - b0), T,
                       k, sg + r * 4 * H, sc + r * H, so + r * 4, dg + r * 4 * H, do4 + r * 4, wk,
                       ctl);
    ENSVS_CHECK_LAUNCH();
  }
  return ENSVS_OK;
}

bool ar_coop_shape(int B, int H) { return B >= 1 && (H == 128 || H == 256); }

long long ar_coop_work(int H, int B) {
  const int S = ar_tile_seqs(B, H);
  const long long slab = H == 128 ? (S == 16 ? ArGeo<128, 16>::SLAB : ArGeo<128, 32>::SLAB)
                                  : (S == 16 ? ArGeo<256, 16>::SLAB : ArGeo<256, 32>::SLAB);
  return (long long)((B + S - 1) / S) * (coop::HDR + slab);
}

int ar_coop_check(int B, int T, int H, const void* wp, const void* work, long long work_bytes) {
  if (!ar_coop_shape(B, H) || T <= 0 || T % 4) return ENSVS_E_SHAPE;
  if (!wp || (uintptr_t)wp % 16 || !work || (uintptr_t)work % 256 ||
      work_bytes < ar_coop_work(H, B))
    return ENSVS_E_ARG;
  return ENSVS_OK;
}

}  // namespace

ENSVS_API int ensvs_ardec_pack(const float* whh, int H, float* wpf, float* wpb, void* stream) {
  if (H % 16 != 0 || H > 256) return ENSVS_E_SHAPE;
  int n = 4 * H * H;
  hipLaunchKernelGGL(ardec_pack_kernel, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, whh, H, wpf, wpb);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_ardec_fwd(const float* gx, int ldgx, const float* ofx, int ldo,
                              const float* wpf, const float* wih_p, const float* wfo, int ldwfo,
                              const float* score, int lds, const float* mask,
                              const float* teach, int ldt, int B, int T, int H,
                              float in_min, float in_max, float mean, float scale, float* lf0,
                              float* res, float* sg, float* sc, float* sh, float* so, float* sp,
                              void* stream) {
  if (T % 4 != 0) return ENSVS_E_SHAPE;
  ArConsts k{in_min, in_max, mean, scale};
  hipStream_t st = (hipStream_t)stream;
  switch (H) {
    case 16: return fwd_launch<16>(gx, ldgx, ofx, ldo, wpf, wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, so, sp, st);
    case 32: return fwd_launch<32>(gx, ldgx, ofx, ldo, wpf, wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, so, sp, st);
    case 64: return fwd_launch<64>(gx, ldgx, ofx, ldo, wpf, wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, so, sp, st);
    case 128: return fwd_launch<128>(gx, ldgx, ofx, ldo, wpf, wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, so, sp, st);
    case 256: return fwd_launch<256>(gx, ldgx, ofx, ldo, wpf, wih_p, wfo, ldwfo, score, lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, so, sp, st);
    default: return ENSVS_E_SHAPE;
  }
}

ENSVS_API int ensvs_ardec_bwd(const float* glf0, const float* gres, const float* wpb,
                              const float* wih_p, const float* wfo, int ldwfo, const float* mask,
                              int teacher, int B, int T, int H, float in_min, float in_max,
                              float mean,
                              float scale, const float* sg, const float* sc, const float* so,
                              float* dg, float* do4, void* stream) {
  if (T % 4 != 0) return ENSVS_E_SHAPE;
  ArConsts k{in_min, in_max, mean, scale};
  hipStream_t st = (hipStream_t)stream;
  switch (H) {
    case 16: return bwd_launch<16>(glf0, gres, wpb, wih_p, wfo, ldwfo, mask, teacher, B, T, k, sg, sc, so, dg, do4, st);
    case 32: return bwd_launch<32>(glf0, gres, wpb, wih_p, wfo, ldwfo, mask, teacher, B, T, k, sg, sc, so, dg, do4, st);
    case 64: return bwd_launch<64>(glf0, gres, wpb, wih_p, wfo, ldwfo, mask, teacher, B, T, k, sg, sc, so, dg, do4, st);
    case 128: return bwd_launch<128>(glf0, gres, wpb, wih_p, wfo, ldwfo, mask, teacher, B, T, k, sg, sc, so, dg, do4, st);
    case 256: return bwd_launch<256>(glf0, gres, wpb, wih_p, wfo, ldwfo, mask, teacher, B, T, k, sg, sc, so, dg, do4, st);
    default: return ENSVS_E_SHAPE;
  }
}

ENSVS_API int ensvs_ardec_coop_supported(int B, int H) { return ar_coop_shape(B, H) ? 1 : 0; }

ENSVS_API int ensvs_ardec_coop_set_tile_seqs(int s) {
  if (s != 0 && s != 16 && s != 32) return ENSVS_E_ARG;
  g_ar_tile_seqs = s;
  return ENSVS_OK;
}

ENSVS_API int ensvs_ardec_coop_tile_seqs(int B, int H) {
  return ar_coop_shape(B, H) ? ar_tile_seqs(B, H) : 0;
}

ENSVS_API long long ensvs_ardec_coop_work_bytes(int H, int B) {
  return ar_coop_shape(B, H) ? ar_coop_work(H, B) : 0;
}

ENSVS_API int ensvs_ardec_coop_pack(const float* whh, int H, int bwd, void* out, void* stream) {
  if (H != 128 && H != 256) return ENSVS_E_SHAPE;
  return coop::pack(whh, whh, 1, H, bwd, out, (hipStream_t)stream);
}

ENSVS_API int ensvs_ardec_coop_fwd(const float* gx, int ldgx, const float* ofx, int ldo,
                                   const void* wpack, const float* wih_p, const float* wfo,
                                   int ldwfo, const float* score, int lds, const float* mask,
                                   const float* teach, int ldt, int B, int T, int H,
                                   float in_min, float in_max, float mean, float scale,
                                   float* lf0, float* res, float* sg, float* sc, float* sh,
                                   float* so, float* sp, void* work, long long work_bytes,
                                   void* stream) {
  if (int e = ar_coop_check(B, T, H, wpack, work, work_bytes)) return e;
  if (ldgx < 4 * H || ldo < 4) return ENSVS_E_SHAPE;
  if (((uintptr_t)sg | (uintptr_t)sc | (uintptr_t)sh) & 15) return ENSVS_E_ARG;  // 16-B stores
  ArConsts k{in_min, in_max, mean, scale};
  hipStream_t st = (hipStream_t)stream;
  unsigned* wk = (unsigned*)work;
#define AR_FWD(HH, SS) coop_fwd_launch<HH, SS>(gx, ldgx, ofx, ldo, wpack, wih_p, wfo, ldwfo, score, \
                                             lds, mask, teach, ldt, B, T, k, lf0, res, sg, sc, sh, \
                                             so, sp, wk, st)
  const bool s16 = ar_tile_seqs(B, H) == 16;
  if (H == 128) return s16 ? AR_FWD(128, 16) : AR_FWD(128, 32);
  return s16 ? AR_FWD(256, 16) : AR_FWD(256, 32);
#undef AR_FWD
}

ENSVS_API int ensvs_ardec_coop_bwd(const float* glf0, const float* gres, const void* wpack,
                                   const float* wih_p, const float* wfo, int ldwfo,
                                   const float* mask, int teacher, int B, int T, int H,
                                   float in_min, float in_max, float mean, float scale,
                                   const float* sg, const float* sc, const float* so, float* dg,
                                   float* do4, void* work, long long work_bytes, void* stream) {
  if (int e = ar_coop_check(B, T, H, wpack, work, work_bytes)) return e;
  if (((uintptr_t)dg | (uintptr_t)do4) & 15) return ENSVS_E_ARG;  // 16-B stores
  ArConsts k{in_min, in_max, mean, scale};
  hipStream_t st = (hipStream_t)stream;
  unsigned* wk = (unsigned*)work;
#define AR_BWD(HH, SS) coop_bwd_launch<HH, SS>(glf0, gres, wpack, wih_p, wfo, ldwfo, mask, teacher, \
                                             B, T, k, sg, sc, so, dg, do4, wk, st)
  const bool s16 = ar_tile_seqs(B, H) == 16;
  if (H == 128) return s16 ? AR_BWD(128, 16) : AR_BWD(128, 32);
  return s16 ? AR_BWD(256, 16) : AR_BWD(256, 32);
#undef AR_BWD
}

ENSVS_API int ensvs_downsample_fwd(const float* p0, int ld0, int n0, const float* p1, int ld1,
                                   int n1, const float* p2, int ld2, int n2, const float* w,
                                   const float* bias, int B, int T, float* e, int lde,
                                   void* stream) {
  DsArgs a{};
  a.seg[0] = {p0, ld0, n0};
  a.seg[1] = {p1, ld1, n1};
  a.seg[2] = {p2, ld2, n2};
  a.nseg = p2 ? 3 : (p1 ? 2 : 1);
  a.C = n0 + (p1 ? n1 : 0) + (p2 ? n2 : 0);
  a.T = T;
  a.B = B;
  long long n = (long long)B * (T / 4) * a.C;
  hipLaunchKernelGGL(downsample_fwd_kernel, dim3((int)std::min<long long>(4096, (n + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, a, w, bias, e, lde);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_downsample_bwd(const float* de, int lde, const float* p0, int ld0, int n0,
                                   const float* p1, int ld1, int n1, const float* p2, int ld2,
                                   int n2, const float* w, int B, int T, float* dx, int lddx,
                                   float* dw, float* db, void* stream) {
  DsArgs a{};
  a.seg[0] = {p0, ld0, n0};
  a.seg[1] = {p1, ld1, n1};
  a.seg[2] = {p2, ld2, n2};
  a.nseg = p2 ? 3 : (p1 ? 2 : 1);
  a.C = n0 + (p1 ? n1 : 0) + (p2 ? n2 : 0);
  a.T = T;
  a.B = B;
  hipStream_t st = (hipStream_t)stream;
  long long n = (long long)B * T * n0;
  hipLaunchKernelGGL(downsample_dgrad_kernel, dim3((int)std::min<long long>(4096, (n + 255) / 256)),
                     dim3(256), 0, st, de, lde, w, B, T, n0, dx, lddx);
  ENSVS_CHECK_LAUNCH();
  hipLaunchKernelGGL(downsample_wgrad_kernel, dim3(a.C), dim3(256), 0, st, a, de, lde, dw, db);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}
