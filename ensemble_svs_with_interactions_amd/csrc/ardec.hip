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
#include "common.h"
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

// The decoder workgroup reserves its CU's LDS (lstm.hip ensvs_rec_exclusive: ENSVS_LSTM_EXCLUSIVE,
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
