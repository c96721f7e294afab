// Lane mapping of v_permlane16_swap / v_permlane32_swap on gfx950 (dev probe).  Row q (16 lanes)
// feeds 10 q + (lane & 15) / 100; prints the gather of the four rows' values into every lane
// (p16 of the value with itself, then p32 of each result with itself), as lstm_mfma.hip uses it.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* o) {
  const float v = 10.f * (threadIdx.x >> 4) + (threadIdx.x & 15) / 100.f;
  const unsigned u = __builtin_bit_cast(unsigned, v);
  // inline asm: the builtins' second result is not trustworthy when both operands hold the
  // same value (hipcc ROCm 7.2 stores the first result for both); s_nop 1 = the 2 wait states
  // after a VALU write of either operand (MI355X: VALU write -> v_permlane read hazard)
  unsigned a0 = u, a1 = u;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a0), "+v"(a1));
  unsigned b0 = a0, b1 = a0, c0 = a1, c1 = a1;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(b0), "+v"(b1));
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c0), "+v"(c1));
  const unsigned s1[2] = {a0, a1}, s2[2] = {b0, b1}, s3[2] = {c0, c1};
  o[threadIdx.x * 6 + 0] = __builtin_bit_cast(float, s1[0]);
  o[threadIdx.x * 6 + 1] = __builtin_bit_cast(float, s1[1]);
  o[threadIdx.x * 6 + 2] = __builtin_bit_cast(float, s2[0]);
  o[threadIdx.x * 6 + 3] = __builtin_bit_cast(float, s2[1]);
  o[threadIdx.x * 6 + 4] = __builtin_bit_cast(float, s3[0]);
  o[threadIdx.x * 6 + 5] = __builtin_bit_cast(float, s3[1]);
}
int main() {
  float* d;
  float h[384];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l = 0; l < 64; l += 5)
    printf("lane %2d: s1 (%6.2f %6.2f)  s2 (%6.2f %6.2f)  s3 (%6.2f %6.2f)\n", l, h[6 * l],
           h[6 * l + 1], h[6 * l + 2], h[6 * l + 3], h[6 * l + 4], h[6 * l + 5]);
  return 0;
}
