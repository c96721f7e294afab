// Cross-workgroup hand-off primitives of the cooperative recurrences (lstm_coop.hip: the large
// bidirectional LSTMs; ardec.hip: the AR residual-F0 decoder).
//
// A recurrence is split over the workgroups of one launch; every step each workgroup publishes
// its slice of the state into a double-buffered slab of the caller's workspace and bumps a
// per-direction counter, and every workgroup waits for the counter before reading the slab.
// The hand-off form is MI355X_MICROARCH.md "Hand-offs measured with sc1 loads", first row:
// 16-B (or 4-B) sc1 stores, s_waitcnt vmcnt(0) of every storing wave (behind a workgroup
// barrier when one lane signals for several waves), one agent-scope counter add per workgroup;
// readers poll the counter from one lane and read the slab with sc1 loads only.
//
// Workspace: HDR bytes of header (one 64-B counter line per direction at word 16 d, the error
// word at byte 128), then the slab.  The polls are bounded: a grid that cannot become resident
// flags the error word and runs on instead of hanging.
#pragma once
#include "common.h"

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace coop {

constexpr int NT = 256;     // 4 waves per workgroup
constexpr int UW = 16;      // hidden units per workgroup
constexpr int SB = 32;      // sequence columns: two MFMA N tiles
constexpr int CP_SC1 = 16;  // buffer-op cache policy: sc1 (L1 bypass on both sides)
constexpr int HDR = 256;    // workspace header
constexpr unsigned SPIN_MAX = 1u << 24;

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)), 1.f);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab(unsigned* work, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((char*)work + HDR, 0, bytes, 0x00020000);
}

// wait until direction d's counter reaches `target` (one lane), then release the workgroup
__device__ __forceinline__ void wait_count(unsigned* work, int d, unsigned target) {
  if (threadIdx.x == 0) {
    unsigned* cnt = work + d * 16;
    unsigned it = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++it == SPIN_MAX) {  // a workgroup never arrived: flag it and go on
        __hip_atomic_store(work + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void signal(unsigned* work, int d) {
  __hip_atomic_fetch_add(work + d * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ f32x4 ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, CP_SC1));
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, CP_SC1);
}
__device__ __forceinline__ void st4(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, CP_SC1);
}

// sum over the 16 lanes of a unit group (lanes 16 j .. 16 j + 15), every lane gets the sum
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// W_hh [4H][H] fp32 of ndir (1 or 2) directions -> MFMA A fragments in registers' order
// (lstm_coop.hip): bwd = 0 fp16 fragments of W_hh (gate rows of 16 units per workgroup),
// bwd = 1 bf16 fragments of W_hh^T (16 unit columns per workgroup, K in the dG slab order
// n' = 64 w' + 4 u' + g).  H in {128, 256, 512}; out holds ndir*4*H*H 2-byte elements.
int pack(const float* w0, const float* w1, int ndir, int H, int bwd, void* out, hipStream_t st);

}  // namespace coop
