// Phase sensitivity of the cooperative AR-decoder forward step (dev tool, not part of the
// product): a copy of ensemble_svs_with_interactions_amd/csrc/ardec.hip's
// ardec_coop_fwd_kernel<256> (free-running, one 32-sequence tile) with one phase removed per
// MODE, so tools/ardec_phase_probe.py can time what each phase adds to an AR step.  Results
// of modes > 0 are wrong by construction.
//   0 full step                      4 no slab h loads (registers)
//   1 no global stores (saved state) 5 no feat_out reduction (partials, tanhf)
//   2 no global input loads          6 publish without its vmcnt(0) drain
//   3 no MFMA                        7 hand-off only (wait, publish, barriers)
#include "coop.h"

namespace {
using namespace coop;
constexpr int H = 256, NW = H / UW, KCW = H / 128;
constexpr int FH = SB * H * 2, FBUF = FH + SB * NW * 16, SLAB = 2 * (SB * 4 * H * 2 + SB * NW * 4 > FBUF ? SB * 4 * H * 2 + SB * NW * 4 : FBUF);
constexpr int PSF = 68;

template <int MODE>
__global__ __launch_bounds__(NT) void probe_kernel(
    const float* __restrict__ gx, const float* __restrict__ ofx, const f16x8* __restrict__ wp,
    const float* __restrict__ wih_p, const float* __restrict__ wfo, const float* __restrict__ mask,
    int B, int T, float* __restrict__ lf0, float* __restrict__ sg, float* __restrict__ sc,
    float* __restrict__ sh, float* __restrict__ so, unsigned* __restrict__ work, Ctl c) {
  __shared__ __attribute__((aligned(16))) float part[4 * SB * PSF];
  __shared__ __attribute__((aligned(16))) _Float16 hs[SB * UW];
  __shared__ __attribute__((aligned(16))) float ops[SB * 4];
  __shared__ float pv[SB];
  const int w = blockIdx.x, u0 = w * UW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Tr = T / 4;
  unsigned* hdr = tile_hdr(work, 0);
  f16x8 wf[4][KCW];
  {
    const f16x8* src = wp + (((long long)w * 4 + wv) * 4 * KCW) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int kk = 0; kk < KCW; ++kk) wf[mt][kk] = src[(mt * KCW + kk) * 64];
  }
  const __amdgpu_buffer_rsrc_t xr = slab(work, 1, 0, SLAB);
  int cs[2], cu[2];
  float wpc[2][4], woc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + NT * i;
    cu[i] = p & 15;
    cs[i] = p >> 4;
#pragma unroll
    for (int g = 0; g < 4; ++g) wpc[i][g] = wih_p[g * H + u0 + cu[i]];
#pragma unroll
    for (int r = 0; r < 4; ++r) woc[i][r] = wfo[r * (H + 130) + u0 + cu[i]];
  }
  float gin[2][4], cst[2] = {0.f, 0.f};
  auto load_in = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* src = gx + ((long long)min(cs[i], B - 1) * Tr + t) * 4 * H + u0 + cu[i];
#pragma unroll
      for (int g = 0; g < 4; ++g) gin[i][g] = MODE == 2 ? 0.1f * g : src[g * H];
    }
  };
  const int rsq = min(tid, B - 1);
  float rofx[4], rmask = 1.f;
  auto load_red = [&](int t) {
    if (MODE == 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) rofx[r] = 0.f;
      return;
    }
    if (tid < SB) {
      const long long row = (long long)rsq * Tr + max(t - 1, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) rofx[r] = ofx[row * 4 + r];
      if (t < Tr) rmask = mask[(long long)rsq * Tr + t];
    }
  };
  load_in(0);
  load_red(0);
  for (int t = 0; t < Tr; ++t) {
    f32x4 acc[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t > 0) {
      wait_count(hdr, 0, (unsigned)(NW * t), c);
      const int base = ((t - 1) & 1) * FBUF;
      if (MODE != 7) {
        f16x8 bf[KCW][2];
#pragma unroll
        for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            bf[kk][nt] = MODE == 4 ? f16x8{} : __builtin_bit_cast(
                f16x8, ld16(xr, ((nt * 16 + (lane & 15)) * H + (wv * KCW + kk) * 32 + 8 * (lane >> 4)) * 2 + base));
        f32x4 op[NW];
        if (tid < SB && MODE != 5)
#pragma unroll
          for (int w2 = 0; w2 < NW; ++w2) op[w2] = ld16(xr, base + FH + (w2 * SB + tid) * 16);
#pragma unroll
        for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) asm volatile("" ::"v"(bf[kk][nt]));
        if (MODE != 3) {
#pragma unroll
          for (int kk = 0; kk < KCW; ++kk)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
              for (int nt = 0; nt < 2; ++nt)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[mt][kk], bf[kk][nt], acc[mt][nt], 0, 0, 0);
        }
        if (tid < SB) {
          float l3 = 0.f;
          if (MODE != 5) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float ov = rofx[r];
#pragma unroll
              for (int w2 = 0; w2 < NW; ++w2) ov += op[w2][r];
              const float rs = 0.6f * tanhf(ov);
              l3 = (rs + 5.5f) / 0.35f;
              if (MODE != 1 && w == 0) {
                lf0[(long long)rsq * T + 4 * (t - 1) + r] = l3;
                so[((long long)rsq * Tr + t - 1) * 4 + r] = ov;
              }
            }
          }
          pv[tid] = l3 * rmask;
        }
      }
    } else if (tid < SB) {
      pv[tid] = 0.f;
    }
    if (MODE != 7) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          *(f32x4*)&part[(wv * SB + nt * 16 + (lane & 15)) * PSF + 16 * mt + 4 * (lane >> 4)] = acc[mt][nt];
    }
    lds_barrier();
    float out[2][6];
    if (MODE != 7) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int s = cs[i], u = cu[i];
        f32x4 a = *(const f32x4*)&part[s * PSF + 4 * u];
#pragma unroll
        for (int q = 1; q < 4; ++q) a += *(const f32x4*)&part[(q * SB + s) * PSF + 4 * u];
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
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = sum16(woc[i][r] * (val ? h : 0.f));
          if (u == 0) ops[s * 4 + r] = v;
        }
        out[i][0] = ig; out[i][1] = fg; out[i][2] = gg; out[i][3] = og; out[i][4] = cn; out[i][5] = h;
      }
    }
    lds_barrier();
    if (wv == 0) {
      const int base = (t & 1) * FBUF;
      st16(xr, base + ((lane >> 1) * H + u0 + (lane & 1) * 8) * 2,
           *(const f32x4*)&hs[(lane >> 1) * UW + (lane & 1) * 8]);
      if (lane < SB) st16(xr, base + FH + (w * SB + lane) * 16, *(const f32x4*)&ops[lane * 4]);
      if (MODE != 6) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(hdr, 0, t, c);
    }
    if (MODE != 1 && MODE != 7) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (cs[i] < B) {
          const long long row = (long long)cs[i] * Tr + t;
          const int j = u0 + cu[i];
#pragma unroll
          for (int g = 0; g < 4; ++g) sg[row * 4 * H + g * H + j] = out[i][g];
          sc[row * H + j] = out[i][4];
          sh[row * H + j] = out[i][5];
        }
    }
    if (MODE != 7) {
      if (t + 1 < Tr) load_in(t + 1);
      load_red(t + 1);
    }
  }
}

}  // namespace

extern "C" int probe_launch(int mode, const float* gx, const float* ofx, const void* wp,
                            const float* wih_p, const float* wfo, const float* mask, int B, int T,
                            float* lf0, float* sg, float* sc, float* sh, float* so, void* work,
                            void* stream) {
  if (B > SB || T % 4) return 1;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(work, 0, HDR, st) != hipSuccess) return 3;
  int rate = 100000;
  hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
  const Ctl c{nullptr, 1000000LL * rate / 1000, 0};
#define L(M)                                                                                    \
  if (mode == M)                                                                                \
    hipLaunchKernelGGL(probe_kernel<M>, dim3(NW), dim3(NT), 0, st, gx, ofx, \
                       (const f16x8*)wp, wih_p, wfo, mask, B, T, lf0, sg, sc, sh, so,           \
                       (unsigned*)work, c);
  L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7)
#undef L
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" long long probe_work_bytes() { return HDR + SLAB; }
