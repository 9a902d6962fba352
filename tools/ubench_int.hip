// Integer-VALU throughput microbenchmark for gfx950 (MI355X).
// Measures wave64 issue throughput of the instructions a 256-bit field multiply can be
// built from, to fix the roofline peak and to choose the radix.
// Each thread runs 8 independent dependency chains of the instruction under test.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 4096

#define CHAIN8(body)                                                                          \
  body(0) body(1) body(2) body(3) body(4) body(5) body(6) body(7)

__global__ void k_mad_u64_u32(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s, b = blockIdx.x * 40503u + 7;
#define I(j) acc[j] = (uint64_t)(a + j) << 7;
  CHAIN8(I)
#undef I
  for (int it = 0; it < ITERS; ++it) {
#define M(j) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : "vcc");
    CHAIN8(M)
#undef M
  }
  uint64_t r = 0;
#define R(j) r ^= acc[j];
  CHAIN8(R)
#undef R
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

#define SIMPLE_KERNEL(name, asmstr)                                                            \
  __global__ void name(uint32_t* out, uint32_t s) {                                            \
    uint32_t acc[8];                                                                           \
    uint32_t a = threadIdx.x * 2654435761u + s, b = blockIdx.x * 40503u + 7;                   \
    for (int j = 0; j < 8; ++j) acc[j] = a + j;                                                \
    for (int it = 0; it < ITERS; ++it) {                                                       \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(asmstr : "+v"(acc[j]) : "v"(b)); \
    }                                                                                          \
    uint32_t r = 0;                                                                            \
    for (int j = 0; j < 8; ++j) r ^= acc[j];                                                   \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                            \
  }

SIMPLE_KERNEL(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
SIMPLE_KERNEL(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
SIMPLE_KERNEL(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
SIMPLE_KERNEL(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
SIMPLE_KERNEL(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0")
SIMPLE_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
SIMPLE_KERNEL(k_add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
SIMPLE_KERNEL(k_addc_co_u32, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
SIMPLE_KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 3, %1")
SIMPLE_KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")

__global__ void k_fma_f64(uint32_t* out, uint32_t s) {
  double acc[8];
  double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999 + s * 1e-12;
  for (int j = 0; j < 8; ++j) acc[j] = a + j;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(b), "v"(a));
  }
  double r = 0;
  for (int j = 0; j < 8; ++j) r += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r);
}

__global__ void k_lshlrev_b64(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t b = (blockIdx.x & 3) + 1;
  for (int j = 0; j < 8; ++j) acc[j] = ((uint64_t)threadIdx.x << 20) + j + s;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(acc[j]) : "v"(b));
  }
  uint64_t r = 0;
  for (int j = 0; j < 8; ++j) r ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  int cus = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, cus, prop.clockRate);
  const int block = 256, grid = cus * 8;
  uint32_t* out;
  hipMalloc(&out, sizeof(uint32_t) * block * grid);
  struct { const char* n; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mul_lo_u32", k_mul_lo_u32},   {"v_mul_hi_u32", k_mul_hi_u32},
      {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
      {"v_mad_u32_u24", k_mad_u32_u24}, {"v_add_u32", k_add_u32},         {"v_add_co_u32", k_add_co_u32},
      {"v_addc_co_u32", k_addc_co_u32}, {"v_lshl_add_u32", k_lshl_add_u32}, {"v_alignbit_b32", k_alignbit},
      {"v_fma_f64", k_fma_f64},         {"v_lshlrev_b64", k_lshlrev_b64},
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 1);  // warm
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, rep);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    double ops = (double)grid * block * ITERS * 8;  // lane-ops
    double rate = ops / (best * 1e-3);
    // cycles per wave64 instruction per SIMD at the observed rate, assuming 2.4 GHz
    double per_simd = rate / (cus * 4.0) / 2.4e9;  // lanes per clock per SIMD
    printf("{\"instr\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"lanes_per_clk_per_simd_at_2.4GHz\": %.2f}\n",
           k.n, best, rate, per_simd);
  }
  hipFree(out);
  return 0;
}
