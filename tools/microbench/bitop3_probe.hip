// Which operand of v_bitop3_b32 indexes the truth table's most significant bit (gfx950)? Evaluates
// bitop3(0xF0.., 0xCC.., 0xAA.., t) for t = 0xCA and 0xD8 (e ? f : g under the two orders) and
// prints the results: with S0 as the MSB the first returns 0xCA, with S0 as the LSB the second does.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(uint32_t* o, uint32_t a, uint32_t b, uint32_t c) {
  o[0] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xCA);
  o[1] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xD8);
  o[2] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xF0);
  o[3] = __builtin_amdgcn_bitop3_b32(a, b, c, 0xAA);
}
int main() {
  uint32_t* d;
  uint32_t h[4];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d, 0xF0F0F0F0u, 0xCCCCCCCCu, 0xAAAAAAAAu);
  if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("{\"t_CA\": \"0x%08x\", \"t_D8\": \"0x%08x\", \"t_F0\": \"0x%08x\", \"t_AA\": \"0x%08x\"}\n", h[0], h[1], h[2], h[3]);
  return 0;
}
