// Per-phase sensitivity probe of the MFMA LSTM recurrence (dev tool, not product code).
//
// Copies of lstm_mfma.hip's forward / backward step loops with a MODE template parameter that
// removes one phase at a time; the step time of each mode (tools/lstm_phase_probe.py) shows
// what the production step pays for that phase:
//   0 full step (the production kernel's work)
//   1 no recurrent product (no MFMA; the h / dG reads from LDS stay)
//   2 no activation math (sigmoid / tanh replaced by one FMA each)
//   3 no global traffic (no chunk loads or flushes: LDS staging buffers reused)
//   4 no LDS read of h / dG (constant MFMA operand; the MFMAs stay)
//   5 barrier + loop only (nothing above)
//   6 chunk flush only (no chunk loads)      7 chunk loads only (no flush)
//   8 flush reads LDS and computes addresses but stores nothing
// Outputs are garbage for modes > 0.  Built by tools/lstm_phase_probe.py into
// tools/liblstm_probe.so (hipcc --offload-arch=gfx950).
#include <hip/hip_runtime.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)), 1.f);
}
__device__ __forceinline__ float bsel(unsigned m, float a, float b) {
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, a) & ~m) |
                                       (__builtin_bit_cast(unsigned, b) & m));
}

template <int H> struct MGeo {
  static constexpr int UPW = H / 4, NMT = H / 16, NKC = H / 32, TPW = H / 64, NKB = H / 8;
  static constexpr int HP = H + 8, GP = 4 * H + 8, CH = 16;
  static constexpr int FWD_LDS = CH * 10 * H * 4 + 2 * HP * 2;
  static constexpr int BWD_LDS = CH * 11 * H * 4 + 2 * GP * 2;
};

template <int H, int MODE>
__global__ __launch_bounds__(NT) void probe_fwd(const float* __restrict__ gx, int ldg,
                                                const f16x8* __restrict__ wp, int L, int T,
                                                float* __restrict__ y, int ldy,
                                                float* __restrict__ sv) {
  using G = MGeo<H>;
  constexpr int NMT = G::NMT, NKC = G::NKC, HP = G::HP, CH = G::CH, GW = 4 * H, OW = 6 * H;
  constexpr int PF = CH * GW / 4 / NT;
  constexpr bool MF = MODE != 1 && MODE != 5, ACT = MODE != 2 && MODE != 5;
  constexpr bool GIO = MODE != 3 && MODE != 5, HRD = MODE != 4 && MODE != 5;
  constexpr bool LDC = MODE != 6, FLS = MODE != 7, STO = MODE != 8;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gin = lds;
  float* out = gin + CH * GW;
  _Float16* hb = (_Float16*)(out + CH * OW);
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6, lg = lane >> 4, n = lane & 15;
  f16x8 wf[NMT][NKC];
  {
    const f16x8* src = wp + ((long long)(dir * 4 + v) * NMT * NKC) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) wf[mt][kk] = src[(mt * NKC + kk) * 64];
  }
  for (int i = tid; i < 2 * HP; i += NT) hb[i] = (_Float16)0.f;
  for (int i = tid; i < CH * GW; i += NT) gin[i] = 0.f;
  constexpr int NUG = H / 64;
  const int ug = NUG == 2 ? (lg >> 1) : 0;
  const bool act = NUG == 2 ? (lg & 1) == 0 : lg == 0;
  const unsigned mug = ug ? ~0u : 0u;
  const int u = v * G::UPW + 16 * ug + n;
  float c = 0.f;
  const long long rowb = (long long)b * T;
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
    const int cnt = min(CH, L - ch * CH);
    for (int e = tid; e < cnt * (OW / 4); e += NT) {
      const int st = e / (OW / 4), c4 = e % (OW / 4);
      const int s = ch * CH + st;
      const long long row = rowb + (dir ? L - 1 - s : s);
      const f32x4 val = *(const f32x4*)(out + st * OW + c4 * 4);
      if (!STO) {
        asm volatile("" ::"v"(val), "v"(row));
        continue;
      }
      if (c4 < H / 4) *(f32x4*)(y + row * ldy + dir * H + c4 * 4) = val;
      else *(f32x4*)(sv + (row * 2 + dir) * 5 * H + (c4 - H / 4) * 4) = val;
    }
  };
  if (GIO) {
    if (nch > 0) {
      load_chunk(0);
      store_in();
    }
    if (nch > 1) load_chunk(1);
  }
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cnt = min(CH, L - ch * CH);
    for (int st = 0; st < cnt; ++st) {
      const int s = ch * CH + st;
      float gv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) gv[g] = gin[st * GW + g * H + u];
      f16x8 bf[NKC];
      if (HRD) {
        const _Float16* hc = hb + ((s + 1) & 1) * HP + 8 * lg;
#pragma unroll
        for (int kk = 0; kk < NKC; ++kk) bf[kk] = *(const f16x8*)(hc + 32 * kk);
      } else {
#pragma unroll
        for (int kk = 0; kk < NKC; ++kk)
#pragma unroll
          for (int e = 0; e < 8; ++e) bf[kk][e] = (_Float16)(0.001f * s);
      }
      f32x4 acc[NMT];
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (MF) {
#pragma unroll
          for (int kk = 0; kk < NKC; ++kk)
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kk], wf[mt][kk], acc[mt], 0, 0, 0);
        } else {
          acc[mt][0] = (float)bf[mt % NKC][0];
        }
      }
      float a[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        a[g] = (NUG == 2 ? bsel(mug, acc[g][0], acc[4 + g][0]) : acc[g][0]) + gv[g];
      float ig, fg, gg, og, h;
      if (ACT) {
        ig = sigm(a[0]), fg = sigm(a[1]), gg = tanh_fast(a[2]), og = sigm(a[3]);
        c = fg * c + ig * gg;
        h = og * tanh_fast(c);
      } else {
        ig = fmaf(0.25f, a[0], 0.5f), fg = fmaf(0.25f, a[1], 0.5f), gg = a[2] * 0.5f;
        og = fmaf(0.25f, a[3], 0.5f);
        c = fg * c + ig * gg;
        h = og * c;
      }
      if (act) {
        hb[(s & 1) * HP + u] = (_Float16)h;
        float* o = out + st * OW;
        o[u] = h;
        o[H + u] = ig;
        o[2 * H + u] = fg;
        o[3 * H + u] = gg;
        o[4 * H + u] = og;
        o[5 * H + u] = c;
      }
      __syncthreads();
    }
    if (GIO) {
      if (LDC && ch + 1 < nch) store_in();
      if (LDC && ch + 2 < nch) load_chunk(ch + 2);  // loads before the stores (lstm_mfma.hip)
      if (FLS) flush(ch);
    }
    __syncthreads();
  }
}

template <int H, int MODE>
__global__ __launch_bounds__(NT) void probe_bwd(const float* __restrict__ dy, int lddy,
                                                const bf16x8* __restrict__ wp, int L, int T,
                                                const float* __restrict__ sv,
                                                float* __restrict__ dg, int lddg) {
  using G = MGeo<H>;
  constexpr int TPW = G::TPW, NKB = G::NKB, GP = G::GP, CH = G::CH, IW = 7 * H, GW = 4 * H;
  constexpr int NIN = CH * IW / 4;
  constexpr int PF = (NIN + NT - 1) / NT;
  constexpr bool MF = MODE != 1 && MODE != 5, ACT = MODE != 2 && MODE != 5;
  constexpr bool GIO = MODE != 3 && MODE != 5, HRD = MODE != 4 && MODE != 5;
  constexpr bool LDC = MODE != 6, FLS = MODE != 7, STO = MODE != 8;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gin = lds;
  float* out = gin + CH * IW;
  __bf16* gb = (__bf16*)(out + CH * GW);
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6, lg = lane >> 4, n = lane & 15;
  bf16x8 wb[TPW][NKB];
  {
    const bf16x8* src = wp + ((long long)(dir * 4 + v) * TPW * NKB) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < TPW; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) wb[mt][kk] = src[(mt * NKB + kk) * 64];
  }
  for (int i = tid; i < 2 * GP; i += NT) gb[i] = (__bf16)0.f;
  for (int i = tid; i < CH * IW; i += NT) gin[i] = 0.5f;
  const int tb = TPW == 2 ? (lg >> 1) : 0;
  const bool act = TPW == 2 ? (lg & 1) == 0 : lg == 0;
  const unsigned mtb = tb ? ~0u : 0u;
  const int u = v * G::UPW + 16 * tb + n;
  const long long rowb = (long long)b * T;
  const int nch = (L + CH - 1) / CH;
  f32x4 rin[PF];
  auto svrow = [&](int s) { return sv + ((rowb + (dir ? L - 1 - s : s)) * 2 + dir) * 5 * H; };
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * NT, st = e / (IW / 4), c4 = e % (IW / 4);
      const int s = L - 1 - ch * CH - st;
      f32x4 val = {0.f, 0.f, 0.f, 0.f};
      if (e < NIN && s >= 0) {
        if (c4 < 5 * H / 4) val = *(const f32x4*)(svrow(s) + c4 * 4);
        else if (c4 < 6 * H / 4)
          val = *(const f32x4*)(dy + (rowb + (dir ? L - 1 - s : s)) * lddy + dir * H +
                                (c4 - 5 * H / 4) * 4);
        else if (s > 0) val = *(const f32x4*)(svrow(s - 1) + 4 * H + (c4 - 6 * H / 4) * 4);
      }
      rin[i] = val;
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
    const int cnt = min(CH, L - ch * CH);
    for (int e = tid; e < cnt * (GW / 4); e += NT) {
      const int st = e / (GW / 4), c4 = e % (GW / 4);
      const int s = L - 1 - ch * CH - st;
      const long long row = rowb + (dir ? L - 1 - s : s);
      const f32x4 val = *(const f32x4*)(out + st * GW + c4 * 4);
      if (!STO) {
        asm volatile("" ::"v"(val), "v"(row));
        continue;
      }
      *(f32x4*)(dg + row * lddg + dir * GW + c4 * 4) = val;
    }
  };
  if (GIO) {
    if (nch > 0) {
      load_chunk(0);
      store_in();
    }
    if (nch > 1) load_chunk(1);
  }
  __syncthreads();
  float dc = 0.f;
  for (int ch = 0; ch < nch; ++ch) {
    const int cnt = min(CH, L - ch * CH);
    for (int st = 0; st < cnt; ++st) {
      const int p = ch * CH + st;
      const float* in = gin + st * IW;
      float iv[7];
#pragma unroll
      for (int g = 0; g < 7; ++g) iv[g] = in[g * H + u];
#pragma unroll
      for (int g = 0; g < 7; ++g) asm volatile("" : "+v"(iv[g]));
      bf16x8 bf[NKB];
      if (HRD) {
        const __bf16* gc = gb + ((p + 1) & 1) * GP + 8 * lg;
#pragma unroll
        for (int kk = 0; kk < NKB; ++kk) bf[kk] = *(const bf16x8*)(gc + 32 * kk);
      } else {
#pragma unroll
        for (int kk = 0; kk < NKB; ++kk)
#pragma unroll
          for (int e = 0; e < 8; ++e) bf[kk][e] = (__bf16)(0.001f * p);
      }
      f32x4 acc[TPW];
#pragma unroll
      for (int mt = 0; mt < TPW; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (MF) {
#pragma unroll
          for (int kk = 0; kk < NKB; ++kk)
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kk], wb[mt][kk], acc[mt], 0, 0, 0);
        } else {
          acc[mt][0] = (float)bf[mt][0];
        }
      }
      const float dhr = TPW == 2 ? bsel(mtb, acc[0][0], acc[TPW - 1][0]) : acc[0][0];
      const float ig = iv[0], fg = iv[1], gg = iv[2], og = iv[3];
      const float ct = iv[4], dyv = iv[5], cp = iv[6];
      const float dh = dyv + dhr;
      const float tc = ACT ? tanh_fast(ct) : ct * 0.5f;
      const float dcc = dc + dh * og * (1.f - tc * tc);
      const float d_i = dcc * gg * ig * (1.f - ig);
      const float d_f = dcc * cp * fg * (1.f - fg);
      const float d_g = dcc * ig * (1.f - gg * gg);
      const float d_o = dh * tc * og * (1.f - og);
      dc = dcc * fg;
      if (act) {
        bf16x4 nb;
        nb[0] = (__bf16)d_i;
        nb[1] = (__bf16)d_f;
        nb[2] = (__bf16)d_g;
        nb[3] = (__bf16)d_o;
        *(bf16x4*)(gb + (p & 1) * GP + 4 * u) = nb;
        float* o = out + st * GW;
        o[u] = d_i;
        o[H + u] = d_f;
        o[2 * H + u] = d_g;
        o[3 * H + u] = d_o;
      }
      __syncthreads();
    }
    if (GIO) {
      if (LDC && ch + 1 < nch) store_in();
      if (LDC && ch + 2 < nch) load_chunk(ch + 2);  // loads before the stores (lstm_mfma.hip)
      if (FLS) flush(ch);
    }
    __syncthreads();
  }
}

template <int H, int MODE>
void launch(int bwd, const void* in, const void* wp, int B, int T, void* o1, void* o2,
            hipStream_t st) {
  const int lds = bwd ? MGeo<H>::BWD_LDS : MGeo<H>::FWD_LDS;
  const int excl = 160 * 1024;
  if (bwd) {
    (void)hipFuncSetAttribute((const void*)probe_bwd<H, MODE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, excl);
    hipLaunchKernelGGL((probe_bwd<H, MODE>), dim3(B, 2), dim3(NT), excl > lds ? excl : lds, st,
                       (const float*)in, 2 * H, (const bf16x8*)wp, T, T, (const float*)o1,
                       (float*)o2, 8 * H);
  } else {
    (void)hipFuncSetAttribute((const void*)probe_fwd<H, MODE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, excl);
    hipLaunchKernelGGL((probe_fwd<H, MODE>), dim3(B, 2), dim3(NT), excl > lds ? excl : lds, st,
                       (const float*)in, 8 * H, (const f16x8*)wp, T, T, (float*)o1, 2 * H,
                       (float*)o2);
  }
}

template <int H>
void launch_mode(int mode, int bwd, const void* in, const void* wp, int B, int T, void* o1,
                 void* o2, hipStream_t st) {
  switch (mode) {
    case 0: launch<H, 0>(bwd, in, wp, B, T, o1, o2, st); break;
    case 1: launch<H, 1>(bwd, in, wp, B, T, o1, o2, st); break;
    case 2: launch<H, 2>(bwd, in, wp, B, T, o1, o2, st); break;
    case 3: launch<H, 3>(bwd, in, wp, B, T, o1, o2, st); break;
    case 4: launch<H, 4>(bwd, in, wp, B, T, o1, o2, st); break;
    case 5: launch<H, 5>(bwd, in, wp, B, T, o1, o2, st); break;
    case 6: launch<H, 6>(bwd, in, wp, B, T, o1, o2, st); break;
    case 7: launch<H, 7>(bwd, in, wp, B, T, o1, o2, st); break;
    default: launch<H, 8>(bwd, in, wp, B, T, o1, o2, st); break;
  }
}

}  // namespace

// fwd (bwd = 0): in = gx [B*T][8H], o1 = y [B*T][2H], o2 = saved [B*T][10H]
// bwd (bwd = 1): in = dy [B*T][2H], o1 = saved, o2 = dg [B*T][8H]; every sequence of length T
extern "C" int probe_launch(int H, int mode, int bwd, const void* in, const void* wp, int B, int T,
                            void* o1, void* o2, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (H == 64) launch_mode<64>(mode, bwd, in, wp, B, T, o1, o2, st);
  else if (H == 128) launch_mode<128>(mode, bwd, in, wp, B, T, o1, o2, st);
  else return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
