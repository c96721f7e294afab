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
// Sequence tiles.  The MFMA N dimension holds SB = 32 sequences; a batch of B > 32 sequences is
// split into ceil(B / 32) independent tiles, one per blockIdx.z (lstm_coop) / blockIdx.y
// (ardec), each with its own counters and slabs.  Tiles never wait on each other, so a tile
// needs only its own workgroups co-resident: workgroups are dispatched in block order, every
// tile's workgroups come before the next tile's, and a resident tile runs to the end and frees
// its CUs for the next.  The tiles run concurrently when the chip holds them (P = 60 pairs of
// 512 frames: two tiles side by side, the same step count as 30 x 1024).
//
// Workspace of ntiles tiles: ntiles headers of HDR bytes (the tile's error word at byte 128;
// from byte 256 the step counters, SHARDS per direction, each on a 64-B line of its own), then
// ntiles slabs of the kernel's slab size.
//
// Sharded counters (round 5): workgroup w adds to shard w % SHARDS of its direction, and a
// waiter's first wave polls every shard with one load per lane and sums them (DPP adds).  One
// counter took all NW agent-scope adds of a step serially at the memory side (~12 ns each,
// MI355X_MICROARCH.md fanin: 32 arrivals ~0.4 us) under the pollers' loads of the same line; the
// guide's fanin row: "for many arrivers shard the counter", and a sharded counter is polled
// "every shard" (Valid forms, first row).
//
// Failure handling (a grid that cannot become resident, e.g. CUs held by another stream's
// long-running kernel): the polls are bounded in time (Ctl::timeout ticks of the 100 MHz
// steady counter, 1 s by default).  The workgroup that times out sets the ABORT bit of the
// direction's counter -- every later poll of any workgroup of the tile then passes at once, so
// the launch ends within one timeout instead of one per step -- and ORs 1 into the tile's
// header word and into Ctl::err, a caller-registered persistent device word
// (ensvs_coop_set_error_word) that the launch's header memset does not clear.  The product
// folds that word into the step's gradient-norm check (ensvs_l2norm_chk: the update is
// skipped) and raises on the host (engine.check_coop_errors).
#pragma once
#include "common.h"

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace coop {

constexpr int NT = 256;     // 4 waves per workgroup
constexpr int UW = 16;      // hidden units per workgroup
constexpr int SB = 32;      // sequence columns of one tile: two MFMA N tiles
constexpr int CP_SC1 = 16;  // buffer-op cache policy: sc1 (L1 bypass on both sides)
constexpr int HDR = 2048;   // workspace header per tile
constexpr int SHARDS = 8;   // step-counter shards per direction (one 64-B line each)
constexpr int CNT0 = 64;    // first counter word (byte 256)
constexpr unsigned ABORT = 0x80000000u;  // counter bit: a workgroup of the tile timed out

// per-launch failure controls (by value in the kernel arguments)
struct Ctl {
  unsigned* err;            // persistent error word (the tile header's word when none is set)
  long long timeout;        // poll bound in steady-counter ticks
  int fault;                // test only: workgroup (0, 0) of tile 0 skips its step-1 signal
};

// host side (lstm_coop.hip): the registered error word, timeout and fault switch
Ctl host_ctl();

inline int ntiles(int B) { return (B + SB - 1) / SB; }

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)), 1.f);
}

// tile z's header and slab resource in a workspace of nt tiles with slab_bytes per slab
__device__ __forceinline__ unsigned* tile_hdr(unsigned* work, int z) {
  return work + z * (HDR / 4);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab(unsigned* work, int nt, int z,
                                                       int slab_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((char*)work + (long long)nt * HDR +
                                               (long long)z * slab_bytes, 0, slab_bytes, 0x00020000);
}

// A workgroup barrier for LDS exchange only: the wave's LDS operations done, then s_barrier.
// __syncthreads() is a workgroup release / acquire, and hipcc drains every outstanding global
// load AND store (s_waitcnt vmcnt(0)) before its s_barrier: in the step loops that made every
// barrier wait for the previous step's saved-state stores (tools/ardec_phase_probe.py: the AR
// step without those stores 4.85 -> 4.39 us).  Global data is never exchanged between the
// waves of a workgroup through these barriers (the hand-off slabs have their own vmcnt(0) and
// counters), and the compiler still waits for each global load before its first use.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned* shard(unsigned* hdr, int d, int s) {
  return hdr + CNT0 + (d * SHARDS + s) * 16;
}

// direction d's step count: lanes 0..SHARDS-1 of the calling wave each load one shard (the
// others contribute 0), summed over each 8-lane group by three DPP adds (the xor 1, xor 2 and
// half-row-mirror pairs of coop::sum16's first three levels); the wave's first lane's total,
// as a uniform value
__device__ __forceinline__ unsigned shard_total(unsigned* hdr, int d, int lane) {
  unsigned v = lane < SHARDS
                   ? __hip_atomic_load(shard(hdr, d, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // xor 1
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // xor 2
  v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // 7 - i
  return __builtin_amdgcn_readfirstlane(v);
}

// wait until direction d's count of the tile reaches `target` (the workgroup's first wave
// polls every shard), then release the workgroup.  The first poll costs what the unbounded
// loop did; the clock is read only once the count is behind, and then every 8th poll.
__device__ __forceinline__ void wait_count(unsigned* hdr, int d, unsigned target, const Ctl& c) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (shard_total(hdr, d, lane) < target) {
      const long long t0 = wall_clock64();
      for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (shard_total(hdr, d, lane) >= target) break;
        if ((it & 7) == 0 && wall_clock64() - t0 > c.timeout) {
          // a workgroup never arrived: release every waiter of this direction (the ABORT bit
          // in one shard makes every total pass), flag the failure
          if (lane == 0) {
            __hip_atomic_fetch_or(shard(hdr, d, 0), ABORT, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_or(hdr + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_or(c.err ? c.err : hdr + 32, 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
          }
          break;
        }
      }
    }
  }
  lds_barrier();
}

// publish step `step`'s slice: one agent-scope add to this workgroup's shard (blockIdx.x is
// the workgroup's unit block in every cooperative kernel; skipped by the test fault)
__device__ __forceinline__ void signal(unsigned* hdr, int d, int step, const Ctl& c) {
  if (c.fault && step == 1 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) return;
  __hip_atomic_fetch_add(shard(hdr, d, blockIdx.x % SHARDS), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
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

// lane i reads lane perm(i) of its DPP row (ctrl: quad_perm 0x00-0xFF, row_mirror 0x140,
// row_half_mirror 0x141); every lane of every row is enabled
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of a unit group (lanes 16 j .. 16 j + 15), every lane gets the sum.
// Four DPP adds within the row: xor 1, xor 2 (quad_perm), then the half-row and row mirrors,
// which pair each lane with a lane of the other quad / other half as xor 4 / xor 8 would
// (the same operand pairs, so the bits of the xor butterfly).  __shfl_xor compiles to
// ds_bpermute_b32, an LDS round trip per level: 32 dependent ones per AR forward step.
__device__ __forceinline__ float sum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm(1, 0, 3, 2)
  v += dpp<0x4E>(v);   // quad_perm(2, 3, 0, 1)
  v += dpp<0x141>(v);  // row_half_mirror: lane 7 - i of the 8
  v += dpp<0x140>(v);  // row_mirror: lane 15 - i of the 16
  return v;
}

// W_hh [4H][H] fp32 of ndir (1 or 2) directions -> MFMA A fragments in registers' order
// (lstm_coop.hip): bwd = 0 fp16 fragments of W_hh (gate rows of 16 units per workgroup),
// bwd = 1 bf16 fragments of W_hh^T (16 unit columns per workgroup, K in the dG slab order
// n' = 64 w' + 4 u' + g).  H in {128, 256, 512}; out holds ndir*4*H*H 2-byte elements.
int pack(const float* w0, const float* w1, int ndir, int H, int bwd, void* out, hipStream_t st);

// dynamic LDS of a launch: the rest of the CU's 160 KB when the recurrence reserves its CU
// (ensvs_rec_exclusive, read per launch), else none.  The kernel attribute is set once to the
// exclusive size, whatever the first launch's setting.
inline size_t dyn_lds(size_t static_lds) {
  return ensvs_rec_exclusive() ? 160 * 1024 - static_lds : 0;
}
inline bool set_max_lds(const void* kernel, size_t static_lds) {
  return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)(160 * 1024 - static_lds)) == hipSuccess;
}

}  // namespace coop
