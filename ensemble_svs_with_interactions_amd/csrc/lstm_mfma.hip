// Bidirectional LSTM recurrence with MFMA recurrent products for H = 64 / 128 (the FFConvLSTM
// encoders of the lf0 / mgc / bap / vuv streams, nnsvs/model.py:862-869, 914-916, the
// multi-track lf0 encoder, acoustic_models/tacotron_f0.py:876-883, and the SeparateF0 bap
// decoder's H = 62 on zero-padded gates) in production (bf16 GEMM) precision.
//
// Same contract and structure as lstm.hip's persistent kernels -- one workgroup per (sequence,
// direction) runs every step, inputs staged through LDS in chunks of CH steps loaded one chunk
// ahead, outputs collected in LDS and written at chunk boundaries, h / dG exchanged through a
// double-buffered LDS vector, one barrier per step -- with the step's recurrent product on the
// matrix cores instead of fp32 VALU FMAs.  lstm.hip's steps are bound by that VALU work and its
// LDS operand traffic (H = 128: 0.76 / 1.19 us forward / backward, 128 FMAs and 64 LDS floats
// per lane per step).  Here the workgroup's 4 waves hold the direction's W_hh as fp16 (forward:
// h in [-1, 1]) / bf16 (backward, W_hh^T: dG spans many decades) MFMA B-operand fragments in
// VGPRs -- as the reference recipe's fp16 autocast runs its cuDNN LSTM (myconfig_notuseIL.yaml:6)
// -- and the A operand is the h / dG vector in every row (an LDS broadcast), so the 16 rows of
// each 16 x 16 result are identical and result column n, which lane n of every 16-lane row
// holds, is one gate row's product: the lane owns a cell's values straight from the MFMA, no
// cross-lane reduction and no selection among tiles (the transposed layout, with W as A and h
// in every column, left each lane choosing its cell among H/16 tiles: H = 128 forward 768 ->
// see DESIGN.md §3 for the per-step times).  Gates, cell state, saved values and outputs stay fp32;
// the fp32 parity mode keeps lstm.hip's exact kernels.  One sequence per workgroup keeps each
// CU's global traffic at lstm.hip's (a batched layout with 4-16 sequences per workgroup was
// bound by the per-CU store/load issue rate: profiles/r3_lstm_batch_bench.txt).
//
// Forward: wave v owns units [v H/4, (v+1) H/4) in NUG = H/64 groups of 16; N tile t = 4 ug + g
// holds gate g of unit group ug (column n: unit v H/4 + 16 ug + n), so lane (lg = lane / 16, n)
// of unit group ug = lg / 2 (H = 128; 0 for H = 64) reads its four gates from tiles 4 ug + g.
// Backward: dh = W_hh^T dG with the units as N (TPW = H/64 tiles of 16 per wave) and K = 4H in
// the exchange order n' = 4 unit + gate; lane (lg, n) of tile lg / 2 (H = 128) applies the cell
// of unit v H/4 + 16 (lg / 2) + n.  Lanes of the other row groups hold copies and do not write.
#include "coop.h"
#include "ensvs.h"

namespace {

using coop::sigm;
using coop::tanh_fast;

constexpr int NT = 256;        // the four compute waves
constexpr int NTW = NT + 64;   // + the I/O wave
constexpr unsigned OOB = 0x7ffffff0u;  // buffer offset past every resource: the op is dropped

template <int H> struct MGeo {
  static constexpr int UPW = H / 4;     // units per wave
  static constexpr int NMT = H / 16;    // forward M tiles per wave
  static constexpr int NKC = H / 32;    // forward K chunks (K = H)
  static constexpr int TPW = H / 64;    // backward M tiles per wave
  static constexpr int NKB = H / 8;     // backward K chunks (K = 4H)
  static constexpr int HP = H + 8;      // fp16 h vector (halves)
  static constexpr int GP = 4 * H + 8;  // bf16 dG vector
  static constexpr int CH = 1024 / H;   // steps per staged chunk (16 KB of fp32 gates)
  // LDS bytes, chunk buffers doubled (the I/O wave fills / drains one while the compute waves
  // use the other): fwd in[2][CH][4H] + out[2][CH][6H] fp32 + h[2][HP] fp16; bwd
  // in[2][CH][7H] + out[2][CH][4H] fp32 + dG[2][GP] bf16
  static constexpr int FWD_LDS = 2 * CH * 10 * H * 4 + 2 * HP * 2;
  static constexpr int BWD_LDS = 2 * CH * 11 * H * 4 + 2 * GP * 2;
  // I/O wave per step of a full chunk: vector-memory instructions issued after a chunk's
  // loads (the counted wait before the chunk's last step)
  static constexpr int FWD_ST = 2 + (5 * H / 4 + 63) / 64;  // y, ybf, saved
  static constexpr int BWD_ST = 2 * (H / 64);               // dg, dgbf
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// 16 B per lane, global -> LDS without registers (the wave writes 1 KB at `l`, lane-linear)
__device__ __forceinline__ void dma16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((glb_void*)g, (lds_void*)l, 16, 0, 0);
}
// 16 B per lane through a buffer resource into LDS (lane-linear 1 KB at `l`): offsets at or
// past the resource's size (or "negative", wrapped) read zeros
__device__ __forceinline__ void dma16b(__amdgpu_buffer_rsrc_t r, unsigned off, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)l, 16, off, 0, 0, 0);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)min(bytes, 0x7fffffffLL),
                                           0x00020000);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v), r, off, 0, 0);
}
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
  const bf16x4 h = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), r, off, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the I/O wave's side of a step barrier: its LDS reads done, its stores and DMA NOT waited for
// (__syncthreads() would drain them: a release fence, s_waitcnt vmcnt(0), before every barrier)
__device__ __forceinline__ void io_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// ---------------------------------------------------------------------------------- packs
// forward B fragments [dir][v][t][kk][lane][8] fp16: B[k][n] = W_hh[g H + unit][k], n = lane & 15,
// unit = v H/4 + 16 (t / 4) + n, g = t % 4, k = 32 kk + 8 (lane / 16) + e
template <int H>
__global__ void mfma_pack_fwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                     _Float16* __restrict__ out) {
  using G = MGeo<H>;
  const int n = 2 * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int e = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int kk = r % G::NKC; r /= G::NKC;
    const int t = r % G::NMT; r /= G::NMT;
    const int v = r % 4, d = r / 4;
    const int unit = v * G::UPW + 16 * (t >> 2) + (lane & 15), g = t & 3;
    const int k = kk * 32 + 8 * (lane >> 4) + e;
    out[i] = (_Float16)(d ? w1 : w0)[(long long)(g * H + unit) * H + k];
  }
}

// backward B fragments [dir][v][t][kk][lane][8] bf16: B[k][n] = W_hh[gate row of k][unit], column
// n = lane & 15 is unit v H/4 + 16 t + n; k = n' = 32 kk + 8 (lane / 16) + e in the exchange
// order n' = 4 unit' + g (gate row g H + unit')
template <int H>
__global__ void mfma_pack_bwd_kernel(const float* __restrict__ w0, const float* __restrict__ w1,
                                     __bf16* __restrict__ out) {
  using G = MGeo<H>;
  const int n = 2 * 4 * H * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int e = i & 7, lane = (i >> 3) & 63;
    int r = i >> 9;
    const int kk = r % G::NKB; r /= G::NKB;
    const int t = r % G::TPW; r /= G::TPW;
    const int v = r % 4, d = r / 4;
    const int unit = v * G::UPW + 16 * t + (lane & 15);
    const int np = kk * 32 + 8 * (lane >> 4) + e;
    const int row = (np & 3) * H + (np >> 2);
    out[i] = (__bf16)(d ? w1 : w0)[(long long)row * H + unit];
  }
}

// ---------------------------------------------------------------------------------- helpers
// b where the mask is set, else a: a bit select (v_bfi), so the compiler does not turn a
// lane-dependent choice between registers into a scratch-indexed load
__device__ __forceinline__ float bsel(unsigned m, float a, float b) {
  return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, a) & ~m) |
                                       (__builtin_bit_cast(unsigned, b) & m));
}

// ---------------------------------------------------------------------------------- forward
// Chunks of CH steps: the compute waves (0-3) run chunk ch out of LDS buffer ch & 1 while the
// I/O wave (4) fills buffer (ch + 1) & 1 with the next chunk's gate inputs by LDS-DMA and writes
// the previous chunk's outputs from the other output buffer, one step row per step.  The compute
// waves issue no global memory instruction inside the recurrence (the earlier layout staged and
// flushed each chunk itself at the chunk boundary: 40-140 ns per step, profiles/r4_lstm_phase*).
// The I/O wave joins every step barrier; its stores are always issued (masked lanes write past
// the buffer resource), so its wait for the DMA before a chunk's last step is a counted vmcnt.
template <int H>
__global__ __launch_bounds__(NTW) void lstm_mfma_fwd_kernel(
    const float* __restrict__ gx, int ldg,        // [B*T][ldg], dir d gates at cols d*4H + g*H + u
    const f16x8* __restrict__ wp,                 // packed forward fragments
    const long long* __restrict__ lengths, int T,
    float* __restrict__ y, int ldy,               // [B*T][ldy], dir d at cols d*H + u
    float* __restrict__ sv,                       // saved [B*T][2][5H]: i,f,g,o,c
    __bf16* __restrict__ yb, int ldyb) {          // optional bf16 copy of y (as y)
  using G = MGeo<H>;
  constexpr int NMT = G::NMT, NKC = G::NKC, HP = G::HP, CH = G::CH, GW = 4 * H, OW = 6 * H;
  constexpr int KST = G::FWD_ST, NSV = KST - 2;
  constexpr int NLD = CH * GW / 256, KP = (NLD + CH / 2 - 1) / (CH / 2), NLS = (NLD + KP - 1) / KP;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gin = lds;                              // [2][CH][4H] gate pre-activations x W_ih^T + b
  float* out = gin + 2 * CH * GW;                // [2][CH][6H]: h, then i f g o c
  _Float16* hb = (_Float16*)(out + 2 * CH * OW);  // [2][HP] h_{t-1} (fp16)
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6, lg = lane >> 4, n = lane & 15;
  const int L = (int)lengths[b];
  const long long rowb = (long long)b * T;
  const int nch = (L + CH - 1) / CH;

  for (int i = tid; i < 2 * HP; i += NTW) hb[i] = (_Float16)0.f;
  for (int i = tid; i < (T - L) * H; i += NTW) {
    y[(rowb + L + i / H) * ldy + dir * H + (i % H)] = 0.f;
    if (yb) yb[(rowb + L + i / H) * ldyb + dir * H + (i % H)] = (__bf16)0.f;
  }

  if (v == 4) {
    // ------------------------------------------------------------------ the I/O wave
    // Offsets are precomputed per lane; per chunk and per row only scalar work remains (a
    // buffer resource per output row; one add per DMA), so the wave's VALU use -- shared with
    // compute wave 0 on its SIMD -- stays small.  Row r of this sequence (0 <= r < T).
    const int sgn = dir ? -1 : 1, r0 = dir ? L - 1 : 0;  // row of forward step s: r0 + sgn s
    const __amdgpu_buffer_rsrc_t rg = rsrc(gx + rowb * ldg, (long long)L * ldg * 4);
    // DMA k of a chunk covers row st_k = k / (H / 64) of it, columns c4 = (k % (H / 64)) 64 + lane
    int vk[NLD];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int st = k / (H / 64), c4 = (k % (H / 64)) * 64 + lane;
      vk[k] = ((r0 + sgn * st) * ldg + dir * GW + 4 * c4) * 4;
    }
    auto load_part = [&](int c, int p) {  // KP DMA of chunk c into buffer c & 1
      char* dst = (char*)(gin + (c & 1) * CH * GW);
      const int dlt = sgn * c * CH * ldg * 4;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const int k = p * KP + j;
        if (k < NLD) dma16b(rg, (unsigned)(vk[k] + dlt), dst + k * 1024);
      }
    };
    const unsigned voy = lane < H / 4 ? (unsigned)((dir * H + 4 * lane) * 4) : OOB;
    const unsigned vob = lane < H / 4 ? (unsigned)((dir * H + 4 * lane) * 2) : OOB;
    auto flush_row = [&](int c, int st) {  // step row st of chunk c from buffer c & 1
      const int s = c * CH + st;
      const bool ok = st < CH && s < L;
      const long long row = rowb + (ok ? r0 + sgn * s : 0);
      const __amdgpu_buffer_rsrc_t ry = rsrc(y + row * ldy, ok ? ldy * 4 : 0);
      const __amdgpu_buffer_rsrc_t rb = rsrc(yb ? (const void*)(yb + row * ldyb) : (const void*)y,
                                             ok && yb ? ldyb * 2 : 0);
      const __amdgpu_buffer_rsrc_t rs = rsrc(sv + row * 10 * H, ok ? 10 * H * 4 : 0);
      const float* o = out + (c & 1) * CH * OW + (ok ? st : 0) * OW;
      const f32x4 val = *(const f32x4*)(o + 4 * (lane & (H / 4 - 1)));
      st16(ry, voy, val);
      st8(rb, vob, val);
#pragma unroll
      for (int k = 0; k < NSV; ++k) {
        const int j = k * 64 + lane;
        const bool on = j < 5 * H / 4;
        const f32x4 w = *(const f32x4*)(o + H + 4 * (on ? j : 0));
        st16(rs, on ? (unsigned)((dir * 5 * H + 4 * j) * 4) : OOB, w);
      }
    };
    if (nch > 0)
      for (int p = 0; p < NLS; ++p) load_part(0, p);
    wait_vm<0>();
    io_barrier();
    for (int ch = 0; ch < nch; ++ch) {
      const int cnt = min(CH, L - ch * CH);
      for (int st = 0; st < cnt; ++st) {
        if (st < NLS && ch + 1 < nch) load_part(ch + 1, st);
        // the next chunk's rows have landed before the last step's barrier (issued after
        // them: KST row stores per step from step NLS - 1 on, none in chunk 0)
        if (st == CH - 1 && ch + 1 < nch) {
          if (ch > 0) wait_vm<KST * (CH - NLS)>();
          else wait_vm<0>();
        }
        if (ch > 0) flush_row(ch - 1, st);
        io_barrier();
      }
    }
    io_barrier();
    if (nch > 1) {
      const int cnt = min(CH, L - (nch - 1) * CH);
      for (int st = cnt; st < CH; ++st) flush_row(nch - 2, st);
    }
    if (nch > 0)
      for (int st = 0; st < CH; ++st) flush_row(nch - 1, st);
    return;
  }

  // -------------------------------------------------------------------- the compute waves
  f16x8 wf[NMT][NKC];
  {
    const f16x8* src = wp + ((long long)(dir * 4 + v) * NMT * NKC) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) wf[mt][kk] = src[(mt * NKC + kk) * 64];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) asm volatile("" ::"v"(wf[mt][kk]));
  }
  // lane (lg, n) takes unit 16 ug + n of its wave, ug = lg / 2 for two unit groups (H = 128);
  // the row groups with the same unit hold copies and do not write
  constexpr int NUG = H / 64;
  const int ug = NUG == 2 ? (lg >> 1) : 0;
  const bool act = NUG == 2 ? (lg & 1) == 0 : lg == 0;
  const unsigned mug = ug ? ~0u : 0u;
  const int u = v * G::UPW + 16 * ug + n;
  float c = 0.f;
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cnt = min(CH, L - ch * CH);
    const float* gc = gin + (ch & 1) * CH * GW;
    float* oc = out + (ch & 1) * CH * OW;
    for (int st = 0; st < cnt; ++st) {
      const int s = ch * CH + st;
      float gv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) gv[g] = gc[st * GW + g * H + u];
      const _Float16* hc = hb + ((s + 1) & 1) * HP + 8 * lg;
      f16x8 bf[NKC];
#pragma unroll
      for (int kk = 0; kk < NKC; ++kk) bf[kk] = *(const f16x8*)(hc + 32 * kk);
      f32x4 acc[NMT];
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKC; ++kk)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[kk], wf[mt][kk], acc[mt], 0, 0, 0);
      }
      float a[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        a[g] = (NUG == 2 ? bsel(mug, acc[g][0], acc[4 + g][0]) : acc[g][0]) + gv[g];
      const float ig = sigm(a[0]), fg = sigm(a[1]), gg = tanh_fast(a[2]), og = sigm(a[3]);
      c = fg * c + ig * gg;
      const float h = og * tanh_fast(c);
      // h on every lane before the branch: otherwise the compiler sinks the o gate (its gin
      // read and activation) into the writing lanes' branch, a second LDS round trip after
      // the MFMAs on every step
      asm volatile("" ::"v"(h));
      if (act) {
        hb[(s & 1) * HP + u] = (_Float16)h;
        float* o = oc + st * OW;
        o[u] = h;
        o[H + u] = ig;
        o[2 * H + u] = fg;
        o[3 * H + u] = gg;
        o[4 * H + u] = og;
        o[5 * H + u] = c;
      }
      __syncthreads();
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------- backward
// Same chunk / I/O-wave structure as the forward: chunk ch's input rows (i f g o c of the step,
// its output gradient, the previous step's c: 7H floats) are staged by the I/O wave one chunk
// ahead, the gate gradients written back one chunk behind.
template <int H>
__global__ __launch_bounds__(NTW) void lstm_mfma_bwd_kernel(
    const float* __restrict__ dy, int lddy,       // [B*T][lddy], grad of outputs
    const bf16x8* __restrict__ wp,                // packed backward fragments
    const long long* __restrict__ lengths, int T,
    const float* __restrict__ sv,                 // saved [B*T][2][5H]
    float* __restrict__ dg, int lddg,             // [B*T][lddg], dir d pre-act grads at d*4H + g*H + u
    __bf16* __restrict__ dgb, int lddgb,          // optional bf16 copy of dg (either may be null)
    float* __restrict__ bsum) {                   // optional [B][8H]: sum over t of dg row (b, t)
  using G = MGeo<H>;
  constexpr int TPW = G::TPW, NKB = G::NKB, GP = G::GP, CH = G::CH, IW = 7 * H, GW = 4 * H;
  constexpr int KST = G::BWD_ST;
  // input DMA per chunk: saved rows (CH x 5H floats), dy rows (CH x H), previous c (CH x H)
  constexpr int NSVL = CH * 5 * H / 256, NDYL = CH * H / 256, NLD = NSVL + 2 * NDYL;
  constexpr int KP = (NLD + CH / 2 - 1) / (CH / 2), NLS = (NLD + KP - 1) / KP;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gin = lds;                        // [2] x {[CH][5H] i f g o c (row t), [CH][H] dy (row
                                           // t), [CH][H] c (t-1)}
  float* out = gin + 2 * CH * IW;          // [2][CH][4H]
  __bf16* gb = (__bf16*)(out + 2 * CH * GW);  // [2][GP] dG of the previous processing step
  const int b = blockIdx.x, dir = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, v = tid >> 6, lg = lane >> 4, n = lane & 15;
  const int L = (int)lengths[b];
  const long long rowb = (long long)b * T;
  // chunk ch holds processing steps p = ch*CH + st: forward step s = L-1-p (descending s)
  const int nch = (L + CH - 1) / CH;

  for (int i = tid; i < 2 * GP; i += NTW) gb[i] = (__bf16)0.f;
  for (int i = tid; i < (T - L) * GW; i += NTW) {
    if (dg) dg[(rowb + L + i / GW) * lddg + dir * GW + (i % GW)] = 0.f;
    if (dgb) dgb[(rowb + L + i / GW) * lddgb + dir * GW + (i % GW)] = (__bf16)0.f;
  }

  if (v == 4) {
    // ------------------------------------------------------------------ the I/O wave
    // As the forward's.  Processing index p = c CH + rel is forward step L-1-p, at row
    // r0 + sgn p of this sequence (dir 0: L-1-p, dir 1: p); the previous step's cell state
    // sits one row further, r0 + sgn (p + 1), which for p = L-1 (the first forward step)
    // is row -1 or L: outside the resource, so it reads as zero (c_{-1} = 0).
    const int sgn = dir ? 1 : -1, r0 = dir ? 0 : L - 1;
    const __amdgpu_buffer_rsrc_t rsv = rsrc(sv + rowb * 10 * H, (long long)L * 10 * H * 4);
    const __amdgpu_buffer_rsrc_t rdy = rsrc(dy + rowb * lddy, (long long)L * lddy * 4);
    int vk[NLD];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      if (k < NSVL) {  // saved rows: 5H/4 float4 per row, i f g o c of the step
        const int q = k * 64 + lane, st = q / (5 * H / 4), c4 = q - st * (5 * H / 4);
        vk[k] = ((r0 + sgn * st) * 10 * H + dir * 5 * H + 4 * c4) * 4;
      } else {
        const int kk = (k - NSVL) % NDYL, q = kk * 64 + lane, st = q / (H / 4), c4 = q % (H / 4);
        vk[k] = k < NSVL + NDYL ? ((r0 + sgn * st) * lddy + dir * H + 4 * c4) * 4
                                : ((r0 + sgn * st + sgn) * 10 * H + dir * 5 * H + 4 * H + 4 * c4) * 4;
      }
    }
    auto load_part = [&](int c, int p) {  // KP DMA of chunk c's inputs into buffer c & 1
      char* base = (char*)(gin + (c & 1) * CH * IW);
      const int dsv = sgn * c * CH * 10 * H * 4, ddy = sgn * c * CH * lddy * 4;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const int k = p * KP + j;
        if (k >= NLD) break;
        if (k < NSVL) dma16b(rsv, (unsigned)(vk[k] + dsv), base + k * 1024);
        else if (k < NSVL + NDYL)
          dma16b(rdy, (unsigned)(vk[k] + ddy), base + CH * 5 * H * 4 + (k - NSVL) * 1024);
        else dma16b(rsv, (unsigned)(vk[k] + dsv), base + CH * 5 * H * 4 + (k - NSVL) * 1024);
      }
    };
    const unsigned vo = (unsigned)(dir * GW * 4);
    auto flush_row = [&](int c, int st) {  // processing row st of chunk c from buffer c & 1
      const int pp = c * CH + st;
      const bool ok = st < CH && pp < L;
      const long long row = rowb + (ok ? r0 + sgn * pp : 0);
      const __amdgpu_buffer_rsrc_t rg = rsrc(dg ? (const void*)(dg + row * lddg) : (const void*)sv,
                                             ok && dg ? lddg * 4 : 0);
      const __amdgpu_buffer_rsrc_t rb = rsrc(dgb ? (const void*)(dgb + row * lddgb) : (const void*)sv,
                                             ok && dgb ? lddgb * 2 : 0);
      const float* o = out + (c & 1) * CH * GW + (ok ? st : 0) * GW;
#pragma unroll
      for (int k = 0; k < H / 64; ++k) {
        const int j = k * 64 + lane;
        const f32x4 val = *(const f32x4*)(o + 4 * j);
        st16(rg, vo + 16 * j, val);
        st8(rb, vo / 2 + 8 * j, val);
      }
    };
    if (nch > 0)
      for (int p = 0; p < NLS; ++p) load_part(0, p);
    wait_vm<0>();
    io_barrier();
    for (int ch = 0; ch < nch; ++ch) {
      const int cnt = min(CH, L - ch * CH);
      for (int st = 0; st < cnt; ++st) {
        if (st < NLS && ch + 1 < nch) load_part(ch + 1, st);
        if (st == CH - 1 && ch + 1 < nch) {  // as the forward
          if (ch > 0) wait_vm<KST * (CH - NLS)>();
          else wait_vm<0>();
        }
        if (ch > 0) flush_row(ch - 1, st);
        io_barrier();
      }
    }
    io_barrier();
    if (nch > 1) {
      const int cnt = min(CH, L - (nch - 1) * CH);
      for (int st = cnt; st < CH; ++st) flush_row(nch - 2, st);
    }
    if (nch > 0)
      for (int st = 0; st < CH; ++st) flush_row(nch - 1, st);
    return;
  }

  // -------------------------------------------------------------------- the compute waves
  bf16x8 wb[TPW][NKB];
  {
    const bf16x8* src = wp + ((long long)(dir * 4 + v) * TPW * NKB) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < TPW; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) wb[mt][kk] = src[(mt * NKB + kk) * 64];
#pragma unroll
    for (int mt = 0; mt < TPW; ++mt)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) asm volatile("" ::"v"(wb[mt][kk]));
  }
  // lane (lg, n) takes unit 16 tb + n of its wave, tb = lg / 2 for two tiles (H = 128); the
  // row groups with the same unit hold copies and do not write
  const int tb = TPW == 2 ? (lg >> 1) : 0;
  const bool act = TPW == 2 ? (lg & 1) == 0 : lg == 0;
  const unsigned mtb = tb ? ~0u : 0u;
  const int u = v * G::UPW + 16 * tb + n;
  float dc = 0.f;
  float ds[4] = {0.f, 0.f, 0.f, 0.f};  // this cell's dg summed over its steps (bias gradient)
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cnt = min(CH, L - ch * CH);
    const float* gc = gin + (ch & 1) * CH * IW;
    float* oc = out + (ch & 1) * CH * GW;
    for (int st = 0; st < cnt; ++st) {
      const int p = ch * CH + st;  // processing index
      const float* in = gc + st * 5 * H;
      float iv[7];
#pragma unroll
      for (int g = 0; g < 5; ++g) iv[g] = in[g * H + u];
      iv[5] = gc[CH * 5 * H + st * H + u];
      iv[6] = gc[CH * 6 * H + st * H + u];
      // read before the product: their LDS latency hides under the dG reads and the MFMAs
      // (H = 128: 711 -> 672 ns per step)
#pragma unroll
      for (int g = 0; g < 7; ++g) asm volatile("" : "+v"(iv[g]));
      const __bf16* gcur = gb + ((p + 1) & 1) * GP + 8 * lg;
      bf16x8 bf[NKB];
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) bf[kk] = *(const bf16x8*)(gcur + 32 * kk);
      // every dG read in flight before the first MFMA (with the I/O wave's two waves on one
      // SIMD the compiler otherwise reuses one register quad: a read and its full LDS latency
      // per MFMA pair, H = 128 645 -> 753 ns per step)
#pragma unroll
      for (int kk = 0; kk < NKB; ++kk) asm volatile("" : "+v"(bf[kk]));
      f32x4 acc[TPW];
#pragma unroll
      for (int mt = 0; mt < TPW; ++mt) {
        acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKB; ++kk)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kk], wb[mt][kk], acc[mt], 0, 0, 0);
      }
      const float dhr = TPW == 2 ? bsel(mtb, acc[0][0], acc[TPW - 1][0]) : acc[0][0];
      const float ig = iv[0], fg = iv[1], gg = iv[2], og = iv[3];
      const float ct = iv[4], dyv = iv[5], cp = iv[6];
      const float dh = dyv + dhr;
      const float tc = tanh_fast(ct);
      const float dcc = dc + dh * og * (1.f - tc * tc);
      const float d_i = dcc * gg * ig * (1.f - ig);
      const float d_f = dcc * cp * fg * (1.f - fg);
      const float d_g = dcc * ig * (1.f - gg * gg);
      const float d_o = dh * tc * og * (1.f - og);
      dc = dcc * fg;
      ds[0] += d_i;
      ds[1] += d_f;
      ds[2] += d_g;
      ds[3] += d_o;
      if (act) {
        bf16x4 nb;
        nb[0] = (__bf16)d_i;
        nb[1] = (__bf16)d_f;
        nb[2] = (__bf16)d_g;
        nb[3] = (__bf16)d_o;
        *(bf16x4*)(gb + (p & 1) * GP + 4 * u) = nb;
        float* o = oc + st * GW;
        o[u] = d_i;
        o[H + u] = d_f;
        o[2 * H + u] = d_g;
        o[3 * H + u] = d_o;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (bsum && act) {
#pragma unroll
    for (int g = 0; g < 4; ++g) bsum[(long long)b * 2 * GW + dir * GW + g * H + u] = ds[g];
  }
}

// ---------------------------------------------------------------------------------- launch
size_t excl(size_t need) {
  return ensvs_rec_exclusive() ? std::max<size_t>(need, 160 * 1024) : need;
}

template <int H>
int launch_fwd(const float* gx, int ldg, const void* wp, const long long* lengths, int B, int T,
               float* y, int ldy, float* sv, __bf16* yb, int ldyb, hipStream_t st) {
  const size_t lds = excl(MGeo<H>::FWD_LDS);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_mfma_fwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)std::max<size_t>(lds, 160 * 1024));  // the exclusive size, whatever this launch asks
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_mfma_fwd_kernel<H>, dim3(B, 2), dim3(NTW), lds, st, gx, ldg,
                     (const f16x8*)wp, lengths, T, y, ldy, sv, yb, ldyb);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

template <int H>
int launch_bwd(const float* dy, int lddy, const void* wp, const long long* lengths, int B, int T,
               const float* sv, float* dg, int lddg, __bf16* dgb, int lddgb, float* bsum,
               hipStream_t st) {
  const size_t lds = excl(MGeo<H>::BWD_LDS);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)lstm_mfma_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)std::max<size_t>(lds, 160 * 1024));  // the exclusive size, whatever this launch asks
  if (attr != hipSuccess) return ENSVS_E_HIP;
  hipLaunchKernelGGL(lstm_mfma_bwd_kernel<H>, dim3(B, 2), dim3(NTW), lds, st, dy, lddy,
                     (const bf16x8*)wp, lengths, T, sv, dg, lddg, dgb, lddgb, bsum);
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

bool aligned16(const void* p) { return (uintptr_t)p % 16 == 0; }

}  // namespace

ENSVS_API int ensvs_lstm_mfma_supported(int H) { return H == 64 || H == 128 ? 1 : 0; }

ENSVS_API int ensvs_lstm_mfma_pack(const float* whh_f, const float* whh_r, int H, int bwd,
                                   void* out, void* stream) {
  if (!ensvs_lstm_mfma_supported(H)) return ENSVS_E_SHAPE;
  if (!out || !aligned16(out) || !whh_f || !whh_r) return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(cdiv(2LL * 4 * H * H, 256)), block(256);
  if (H == 64) {
    if (bwd) hipLaunchKernelGGL(mfma_pack_bwd_kernel<64>, grid, block, 0, st, whh_f, whh_r, (__bf16*)out);
    else hipLaunchKernelGGL(mfma_pack_fwd_kernel<64>, grid, block, 0, st, whh_f, whh_r, (_Float16*)out);
  } else {
    if (bwd) hipLaunchKernelGGL(mfma_pack_bwd_kernel<128>, grid, block, 0, st, whh_f, whh_r, (__bf16*)out);
    else hipLaunchKernelGGL(mfma_pack_fwd_kernel<128>, grid, block, 0, st, whh_f, whh_r, (_Float16*)out);
  }
  ENSVS_CHECK_LAUNCH();
  return ENSVS_OK;
}

ENSVS_API int ensvs_lstm_mfma_fwd(const float* gx, int ldg, const void* wpack,
                                  const long long* lengths, int B, int T, int H, float* y, int ldy,
                                  float* saved, void* ybf, int ldyb, void* stream) {
  if (!ensvs_lstm_mfma_supported(H) || B <= 0 || T <= 0 || ldg < 8 * H || ldy < 2 * H ||
      (ybf && ldyb < 2 * H))
    return ENSVS_E_SHAPE;
  if (ldg % 4 || ldy % 4 || !aligned16(gx) || !aligned16(y) || !aligned16(saved) ||
      !aligned16(wpack) || !lengths || (ybf && (ldyb % 4 || (uintptr_t)ybf % 8)))
    return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  __bf16* yb = (__bf16*)ybf;
  return H == 64 ? launch_fwd<64>(gx, ldg, wpack, lengths, B, T, y, ldy, saved, yb, ldyb, st)
                 : launch_fwd<128>(gx, ldg, wpack, lengths, B, T, y, ldy, saved, yb, ldyb, st);
}

ENSVS_API int ensvs_lstm_mfma_bwd(const float* dy, int lddy, const void* wpack,
                                  const long long* lengths, int B, int T, int H,
                                  const float* saved, float* dg, int lddg, void* dgbf,
                                  int lddgb, float* bsum, void* stream) {
  if (!ensvs_lstm_mfma_supported(H) || B <= 0 || T <= 0 || lddy < 2 * H ||
      (dg && lddg < 8 * H) || (dgbf && lddgb < 8 * H))
    return ENSVS_E_SHAPE;
  if (lddy % 4 || !aligned16(dy) || !aligned16(saved) || !aligned16(wpack) || !lengths ||
      (!dg && !dgbf) || (dg && (lddg % 4 || !aligned16(dg))) ||
      (dgbf && (lddgb % 4 || (uintptr_t)dgbf % 8)))
    return ENSVS_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  __bf16* dgb = (__bf16*)dgbf;
  return H == 64 ? launch_bwd<64>(dy, lddy, wpack, lengths, B, T, saved, dg, lddg, dgb, lddgb,
                                  bsum, st)
                 : launch_bwd<128>(dy, lddy, wpack, lengths, B, T, saved, dg, lddg, dgb, lddgb,
                                   bsum, st);
}
