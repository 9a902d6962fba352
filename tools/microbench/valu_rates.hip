// Issue-rate microbenchmark for the VALU opcodes the field arithmetic is made of (gfx950).
// Each lane runs 8 independent chains of one opcode (inline asm, so the compiler cannot
// fold them); rate = lane-ops / s over a full-chip grid. Used to price instructions
// (DESIGN.md §5), not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 2048
#define CH 8

#define K32(NAME, ASM)                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                              \
    uint32_t a[CH];                                                                 \
    const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;                      \
    for (int k = 0; k < CH; ++k) a[k] = threadIdx.x * 7u + k;                       \
    for (int it = 0; it < ITERS; ++it) {                                            \
      _Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(ASM : "+v"(a[k]) : "v"(b), "v"(c) : "vcc", "s0", "s1"); \
    }                                                                               \
    uint32_t s = 0;                                                                 \
    for (int k = 0; k < CH; ++k) s ^= a[k];                                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                 \
  }

#define K64(NAME, ASM)                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                              \
    uint64_t a[CH];                                                                 \
    const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;                      \
    for (int k = 0; k < CH; ++k) a[k] = threadIdx.x * 7ull + k;                     \
    for (int it = 0; it < ITERS; ++it) {                                            \
      _Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(ASM : "+v"(a[k]) : "v"(b), "v"(c) : "vcc", "s0", "s1"); \
    }                                                                               \
    uint64_t s = 0;                                                                 \
    for (int k = 0; k < CH; ++k) s ^= a[k];                                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32); \
  }

K32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K32(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 4, %1")
K32(k_add_u32, "v_add_u32 %0, %0, %1")
K32(k_and_b32, "v_and_b32 %0, %0, %1")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
K32(k_cndmask, "v_cmp_gt_u32 vcc, %1, %2\n v_cndmask_b32 %0, %0, %1, vcc")
K64(k_mad_u64_u32, "v_mad_u64_u32 %0, s[0:1], %1, %2, %0")
K64(k_lshrrev_b64, "v_lshrrev_b64 %0, 3, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %0")

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  const int blocks = 256 * 8 * 4, threads = 256;
  uint32_t* out;
  if (hipMalloc(&out, (size_t)blocks * threads * 4) != hipSuccess) return 1;
  struct {
    const char* name;
    kfn f;
    int insts;  // VALU instructions per asm statement
  } ks[] = {{"v_mul_lo_u32", k_mul_lo_u32, 1},     {"v_mul_hi_u32", k_mul_hi_u32, 1},
            {"v_mad_u32_u24", k_mad_u32_u24, 1},   {"v_lshl_add_u32", k_lshl_add_u32, 1},
            {"v_add_u32", k_add_u32, 1},           {"v_and_b32", k_and_b32, 1},
            {"v_alignbit_b32", k_alignbit, 1},     {"v_cmp+v_cndmask", k_cndmask, 2},
            {"v_mad_u64_u32", k_mad_u64_u32, 1},   {"v_lshrrev_b64", k_lshrrev_b64, 1},
            {"v_lshl_add_u64", k_lshl_add_u64, 1}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u);  // warm
    hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u + r);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = 5.0 * blocks * threads * (double)ITERS * CH;
    printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"insts_per_stmt\": %d}\n", k.name, ops / (ms * 1e-3), k.insts);
  }
  hipFree(out);
  return 0;
}
