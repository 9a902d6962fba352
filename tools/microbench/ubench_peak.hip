// Integer-VALU peak, re-measured: is 2.79e13 MAC32/s (profiles/r01/ubench_int.json)
// the chip's v_mad_u64_u32 rate, or the rate of a latency-limited harness?
//
// Differences from tools/ubench_int.hip: 16 independent chains per lane (not 8); the grid is sized
// for W resident waves per SIMD (W = 1, 2, 4, 8; every wave resident at once: no tail); each launch
// runs ~5-20 ms (launch overhead < 0.2%); the shader clock is measured inside the kernel (every
// wave's s_memtime and s_memrealtime deltas, the latter at the 100 MHz wall-clock rate) so rates are
// reported per clock as well as per second. The per-clock figure is compared with the 2-cycle wave64
// issue of a SIMD-32 (32 lanes/clk/SIMD, MI355X_MICROARCH.md "Wave scheduling").
//
// Mixes: MAC + k independent v_add_u32 per MAC show whether adds issue in the MAC's shadow.
//
// Not part of the product. Build: hipcc -O3 --offload-arch=gfx950 tools/microbench/ubench_peak.hip -o ...
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CH 16

struct Clk {
  unsigned long long t0, t1, r0, r1;
};

__device__ __forceinline__ void clk_begin(Clk& c) {
  c.t0 = __builtin_readcyclecounter();
  c.r0 = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void clk_end(Clk& c, unsigned long long* clk) {
  c.t1 = __builtin_readcyclecounter();
  c.r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[2 * w] = c.t1 - c.t0;
    clk[2 * w + 1] = c.r1 - c.r0;
  }
}

// Each kernel's loop body is ONE asm statement of CH independent instructions (the compiler
// puts s_nop hazards between separate asm statements that write an SGPR).

__global__ void __launch_bounds__(256) k_add_u32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add_u32 %8, %8, %16\nv_add_u32 %9, %9, %16\nv_add_u32 %10, %10, %16\nv_add_u32 %11, %11, %16\nv_add_u32 %12, %12, %16\nv_add_u32 %13, %13, %16\nv_add_u32 %14, %14, %16\nv_add_u32 %15, %15, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_and_b32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_and_b32 %0, %0, %16\nv_and_b32 %1, %1, %16\nv_and_b32 %2, %2, %16\nv_and_b32 %3, %3, %16\nv_and_b32 %4, %4, %16\nv_and_b32 %5, %5, %16\nv_and_b32 %6, %6, %16\nv_and_b32 %7, %7, %16\nv_and_b32 %8, %8, %16\nv_and_b32 %9, %9, %16\nv_and_b32 %10, %10, %16\nv_and_b32 %11, %11, %16\nv_and_b32 %12, %12, %16\nv_and_b32 %13, %13, %16\nv_and_b32 %14, %14, %16\nv_and_b32 %15, %15, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_add_co_u32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %16\nv_add_co_u32 %1, vcc, %1, %16\nv_add_co_u32 %2, vcc, %2, %16\nv_add_co_u32 %3, vcc, %3, %16\nv_add_co_u32 %4, vcc, %4, %16\nv_add_co_u32 %5, vcc, %5, %16\nv_add_co_u32 %6, vcc, %6, %16\nv_add_co_u32 %7, vcc, %7, %16\nv_add_co_u32 %8, vcc, %8, %16\nv_add_co_u32 %9, vcc, %9, %16\nv_add_co_u32 %10, vcc, %10, %16\nv_add_co_u32 %11, vcc, %11, %16\nv_add_co_u32 %12, vcc, %12, %16\nv_add_co_u32 %13, vcc, %13, %16\nv_add_co_u32 %14, vcc, %14, %16\nv_add_co_u32 %15, vcc, %15, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_alignbit(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %16, 7\nv_alignbit_b32 %1, %1, %16, 7\nv_alignbit_b32 %2, %2, %16, 7\nv_alignbit_b32 %3, %3, %16, 7\nv_alignbit_b32 %4, %4, %16, 7\nv_alignbit_b32 %5, %5, %16, 7\nv_alignbit_b32 %6, %6, %16, 7\nv_alignbit_b32 %7, %7, %16, 7\nv_alignbit_b32 %8, %8, %16, 7\nv_alignbit_b32 %9, %9, %16, 7\nv_alignbit_b32 %10, %10, %16, 7\nv_alignbit_b32 %11, %11, %16, 7\nv_alignbit_b32 %12, %12, %16, 7\nv_alignbit_b32 %13, %13, %16, 7\nv_alignbit_b32 %14, %14, %16, 7\nv_alignbit_b32 %15, %15, %16, 7" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_lshl_add_u32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_lshl_add_u32 %0, %0, 4, %16\nv_lshl_add_u32 %1, %1, 4, %16\nv_lshl_add_u32 %2, %2, 4, %16\nv_lshl_add_u32 %3, %3, 4, %16\nv_lshl_add_u32 %4, %4, 4, %16\nv_lshl_add_u32 %5, %5, 4, %16\nv_lshl_add_u32 %6, %6, 4, %16\nv_lshl_add_u32 %7, %7, 4, %16\nv_lshl_add_u32 %8, %8, 4, %16\nv_lshl_add_u32 %9, %9, 4, %16\nv_lshl_add_u32 %10, %10, 4, %16\nv_lshl_add_u32 %11, %11, 4, %16\nv_lshl_add_u32 %12, %12, 4, %16\nv_lshl_add_u32 %13, %13, 4, %16\nv_lshl_add_u32 %14, %14, 4, %16\nv_lshl_add_u32 %15, %15, 4, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mul_lo_u32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mul_lo_u32 %0, %0, %16\nv_mul_lo_u32 %1, %1, %16\nv_mul_lo_u32 %2, %2, %16\nv_mul_lo_u32 %3, %3, %16\nv_mul_lo_u32 %4, %4, %16\nv_mul_lo_u32 %5, %5, %16\nv_mul_lo_u32 %6, %6, %16\nv_mul_lo_u32 %7, %7, %16\nv_mul_lo_u32 %8, %8, %16\nv_mul_lo_u32 %9, %9, %16\nv_mul_lo_u32 %10, %10, %16\nv_mul_lo_u32 %11, %11, %16\nv_mul_lo_u32 %12, %12, %16\nv_mul_lo_u32 %13, %13, %16\nv_mul_lo_u32 %14, %14, %16\nv_mul_lo_u32 %15, %15, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mul_u32_u24(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint32_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mul_u32_u24 %0, %0, %16\nv_mul_u32_u24 %1, %1, %16\nv_mul_u32_u24 %2, %2, %16\nv_mul_u32_u24 %3, %3, %16\nv_mul_u32_u24 %4, %4, %16\nv_mul_u32_u24 %5, %5, %16\nv_mul_u32_u24 %6, %6, %16\nv_mul_u32_u24 %7, %7, %16\nv_mul_u32_u24 %8, %8, %16\nv_mul_u32_u24 %9, %9, %16\nv_mul_u32_u24 %10, %10, %16\nv_mul_u32_u24 %11, %11, %16\nv_mul_u32_u24 %12, %12, %16\nv_mul_u32_u24 %13, %13, %16\nv_mul_u32_u24 %14, %14, %16\nv_mul_u32_u24 %15, %15, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mad_u64_u32(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint64_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[8:9], %16, %17, %0\nv_mad_u64_u32 %1, s[8:9], %16, %17, %1\nv_mad_u64_u32 %2, s[8:9], %16, %17, %2\nv_mad_u64_u32 %3, s[8:9], %16, %17, %3\nv_mad_u64_u32 %4, s[8:9], %16, %17, %4\nv_mad_u64_u32 %5, s[8:9], %16, %17, %5\nv_mad_u64_u32 %6, s[8:9], %16, %17, %6\nv_mad_u64_u32 %7, s[8:9], %16, %17, %7\nv_mad_u64_u32 %8, s[8:9], %16, %17, %8\nv_mad_u64_u32 %9, s[8:9], %16, %17, %9\nv_mad_u64_u32 %10, s[8:9], %16, %17, %10\nv_mad_u64_u32 %11, s[8:9], %16, %17, %11\nv_mad_u64_u32 %12, s[8:9], %16, %17, %12\nv_mad_u64_u32 %13, s[8:9], %16, %17, %13\nv_mad_u64_u32 %14, s[8:9], %16, %17, %14\nv_mad_u64_u32 %15, s[8:9], %16, %17, %15" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_lshrrev_b64(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint64_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_lshrrev_b64 %0, 3, %0\nv_lshrrev_b64 %1, 3, %1\nv_lshrrev_b64 %2, 3, %2\nv_lshrrev_b64 %3, 3, %3\nv_lshrrev_b64 %4, 3, %4\nv_lshrrev_b64 %5, 3, %5\nv_lshrrev_b64 %6, 3, %6\nv_lshrrev_b64 %7, 3, %7\nv_lshrrev_b64 %8, 3, %8\nv_lshrrev_b64 %9, 3, %9\nv_lshrrev_b64 %10, 3, %10\nv_lshrrev_b64 %11, 3, %11\nv_lshrrev_b64 %12, 3, %12\nv_lshrrev_b64 %13, 3, %13\nv_lshrrev_b64 %14, 3, %14\nv_lshrrev_b64 %15, 3, %15" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_fma_f64(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  double a[CH];
  uint32_t d[CH];
  const double b = 1.0 + seed * 1e-9, c = 0.5;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = 1.0 + k * 1e-3; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_fma_f64 %0, %0, %16, %17\nv_fma_f64 %1, %1, %16, %17\nv_fma_f64 %2, %2, %16, %17\nv_fma_f64 %3, %3, %16, %17\nv_fma_f64 %4, %4, %16, %17\nv_fma_f64 %5, %5, %16, %17\nv_fma_f64 %6, %6, %16, %17\nv_fma_f64 %7, %7, %16, %17\nv_fma_f64 %8, %8, %16, %17\nv_fma_f64 %9, %9, %16, %17\nv_fma_f64 %10, %10, %16, %17\nv_fma_f64 %11, %11, %16, %17\nv_fma_f64 %12, %12, %16, %17\nv_fma_f64 %13, %13, %16, %17\nv_fma_f64 %14, %14, %16, %17\nv_fma_f64 %15, %15, %16, %17" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s += (uint64_t)(a[k] * 1e6); }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mix_mac_add1(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint64_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[8:9], %32, %33, %0\nv_add_u32 %16, %16, %32\nv_mad_u64_u32 %1, s[8:9], %32, %33, %1\nv_add_u32 %17, %17, %32\nv_mad_u64_u32 %2, s[8:9], %32, %33, %2\nv_add_u32 %18, %18, %32\nv_mad_u64_u32 %3, s[8:9], %32, %33, %3\nv_add_u32 %19, %19, %32\nv_mad_u64_u32 %4, s[8:9], %32, %33, %4\nv_add_u32 %20, %20, %32\nv_mad_u64_u32 %5, s[8:9], %32, %33, %5\nv_add_u32 %21, %21, %32\nv_mad_u64_u32 %6, s[8:9], %32, %33, %6\nv_add_u32 %22, %22, %32\nv_mad_u64_u32 %7, s[8:9], %32, %33, %7\nv_add_u32 %23, %23, %32\nv_mad_u64_u32 %8, s[8:9], %32, %33, %8\nv_add_u32 %24, %24, %32\nv_mad_u64_u32 %9, s[8:9], %32, %33, %9\nv_add_u32 %25, %25, %32\nv_mad_u64_u32 %10, s[8:9], %32, %33, %10\nv_add_u32 %26, %26, %32\nv_mad_u64_u32 %11, s[8:9], %32, %33, %11\nv_add_u32 %27, %27, %32\nv_mad_u64_u32 %12, s[8:9], %32, %33, %12\nv_add_u32 %28, %28, %32\nv_mad_u64_u32 %13, s[8:9], %32, %33, %13\nv_add_u32 %29, %29, %32\nv_mad_u64_u32 %14, s[8:9], %32, %33, %14\nv_add_u32 %30, %30, %32\nv_mad_u64_u32 %15, s[8:9], %32, %33, %15\nv_add_u32 %31, %31, %32" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]), "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]), "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; s ^= d[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mix_mac_add2(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint64_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[8:9], %32, %33, %0\nv_add_u32 %16, %16, %32\nv_add_u32 %17, %17, %32\nv_mad_u64_u32 %1, s[8:9], %32, %33, %1\nv_add_u32 %17, %17, %32\nv_add_u32 %18, %18, %32\nv_mad_u64_u32 %2, s[8:9], %32, %33, %2\nv_add_u32 %18, %18, %32\nv_add_u32 %19, %19, %32\nv_mad_u64_u32 %3, s[8:9], %32, %33, %3\nv_add_u32 %19, %19, %32\nv_add_u32 %20, %20, %32\nv_mad_u64_u32 %4, s[8:9], %32, %33, %4\nv_add_u32 %20, %20, %32\nv_add_u32 %21, %21, %32\nv_mad_u64_u32 %5, s[8:9], %32, %33, %5\nv_add_u32 %21, %21, %32\nv_add_u32 %22, %22, %32\nv_mad_u64_u32 %6, s[8:9], %32, %33, %6\nv_add_u32 %22, %22, %32\nv_add_u32 %23, %23, %32\nv_mad_u64_u32 %7, s[8:9], %32, %33, %7\nv_add_u32 %23, %23, %32\nv_add_u32 %24, %24, %32\nv_mad_u64_u32 %8, s[8:9], %32, %33, %8\nv_add_u32 %24, %24, %32\nv_add_u32 %25, %25, %32\nv_mad_u64_u32 %9, s[8:9], %32, %33, %9\nv_add_u32 %25, %25, %32\nv_add_u32 %26, %26, %32\nv_mad_u64_u32 %10, s[8:9], %32, %33, %10\nv_add_u32 %26, %26, %32\nv_add_u32 %27, %27, %32\nv_mad_u64_u32 %11, s[8:9], %32, %33, %11\nv_add_u32 %27, %27, %32\nv_add_u32 %28, %28, %32\nv_mad_u64_u32 %12, s[8:9], %32, %33, %12\nv_add_u32 %28, %28, %32\nv_add_u32 %29, %29, %32\nv_mad_u64_u32 %13, s[8:9], %32, %33, %13\nv_add_u32 %29, %29, %32\nv_add_u32 %30, %30, %32\nv_mad_u64_u32 %14, s[8:9], %32, %33, %14\nv_add_u32 %30, %30, %32\nv_add_u32 %31, %31, %32\nv_mad_u64_u32 %15, s[8:9], %32, %33, %15\nv_add_u32 %31, %31, %32\nv_add_u32 %16, %16, %32" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]), "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]), "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; s ^= d[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void __launch_bounds__(256) k_mix_mac_add3(uint32_t* out, unsigned long long* clk, uint32_t seed, int iters) {
  uint64_t a[CH];
  uint32_t d[CH];
  const uint32_t b = seed ^ threadIdx.x, c = seed * 3u + 1u;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = threadIdx.x * 7u + k; d[k] = k; }
  Clk t;
  clk_begin(t);
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_mad_u64_u32 %0, s[8:9], %32, %33, %0\nv_add_u32 %16, %16, %32\nv_add_u32 %17, %17, %32\nv_add_u32 %18, %18, %32\nv_mad_u64_u32 %1, s[8:9], %32, %33, %1\nv_add_u32 %17, %17, %32\nv_add_u32 %18, %18, %32\nv_add_u32 %19, %19, %32\nv_mad_u64_u32 %2, s[8:9], %32, %33, %2\nv_add_u32 %18, %18, %32\nv_add_u32 %19, %19, %32\nv_add_u32 %20, %20, %32\nv_mad_u64_u32 %3, s[8:9], %32, %33, %3\nv_add_u32 %19, %19, %32\nv_add_u32 %20, %20, %32\nv_add_u32 %21, %21, %32\nv_mad_u64_u32 %4, s[8:9], %32, %33, %4\nv_add_u32 %20, %20, %32\nv_add_u32 %21, %21, %32\nv_add_u32 %22, %22, %32\nv_mad_u64_u32 %5, s[8:9], %32, %33, %5\nv_add_u32 %21, %21, %32\nv_add_u32 %22, %22, %32\nv_add_u32 %23, %23, %32\nv_mad_u64_u32 %6, s[8:9], %32, %33, %6\nv_add_u32 %22, %22, %32\nv_add_u32 %23, %23, %32\nv_add_u32 %24, %24, %32\nv_mad_u64_u32 %7, s[8:9], %32, %33, %7\nv_add_u32 %23, %23, %32\nv_add_u32 %24, %24, %32\nv_add_u32 %25, %25, %32\nv_mad_u64_u32 %8, s[8:9], %32, %33, %8\nv_add_u32 %24, %24, %32\nv_add_u32 %25, %25, %32\nv_add_u32 %26, %26, %32\nv_mad_u64_u32 %9, s[8:9], %32, %33, %9\nv_add_u32 %25, %25, %32\nv_add_u32 %26, %26, %32\nv_add_u32 %27, %27, %32\nv_mad_u64_u32 %10, s[8:9], %32, %33, %10\nv_add_u32 %26, %26, %32\nv_add_u32 %27, %27, %32\nv_add_u32 %28, %28, %32\nv_mad_u64_u32 %11, s[8:9], %32, %33, %11\nv_add_u32 %27, %27, %32\nv_add_u32 %28, %28, %32\nv_add_u32 %29, %29, %32\nv_mad_u64_u32 %12, s[8:9], %32, %33, %12\nv_add_u32 %28, %28, %32\nv_add_u32 %29, %29, %32\nv_add_u32 %30, %30, %32\nv_mad_u64_u32 %13, s[8:9], %32, %33, %13\nv_add_u32 %29, %29, %32\nv_add_u32 %30, %30, %32\nv_add_u32 %31, %31, %32\nv_mad_u64_u32 %14, s[8:9], %32, %33, %14\nv_add_u32 %30, %30, %32\nv_add_u32 %31, %31, %32\nv_add_u32 %16, %16, %32\nv_mad_u64_u32 %15, s[8:9], %32, %33, %15\nv_add_u32 %31, %31, %32\nv_add_u32 %16, %16, %32\nv_add_u32 %17, %17, %32" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15]), "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]), "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13]), "+v"(d[14]), "+v"(d[15]) : "v"(b), "v"(c) : "s8", "s9", "vcc");
  }
  clk_end(t, clk);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) { s ^= (uint64_t)a[k]; s ^= d[k]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t, int);

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount, simds = cus * 4;
  int wall_khz = 0;
  hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz_max\": %d, \"wall_clock_khz\": %d, \"chains\": %d}\n",
         prop.gcnArchName, cus, prop.clockRate, wall_khz, CH);
  const int threads = 256;
  const int max_blocks = simds * 8 / 4;  // 8 waves per SIMD, 4 waves per block
  uint32_t* out;
  unsigned long long* clk;
  hipMalloc(&out, sizeof(uint32_t) * max_blocks * threads);
  hipMalloc(&clk, sizeof(unsigned long long) * 2 * max_blocks * 4);
  std::vector<unsigned long long> hclk(2 * max_blocks * 4);
  struct K {
    const char* n;
    kfn f;
    int per;       // VALU instructions per chain step
    int lane_ops;  // counted lane-ops per chain step (MACs for the mixes)
  } ks[] = {
      {"v_add_u32", k_add_u32, 1, 1},         {"v_and_b32", k_and_b32, 1, 1},
      {"v_add_co_u32", k_add_co_u32, 1, 1},   {"v_alignbit_b32", k_alignbit, 1, 1},
      {"v_lshl_add_u32", k_lshl_add_u32, 1, 1}, {"v_mul_lo_u32", k_mul_lo_u32, 1, 1},
      {"v_mul_u32_u24", k_mul_u32_u24, 1, 1}, {"v_mad_u64_u32", k_mad_u64_u32, 1, 1},
      {"v_lshrrev_b64", k_lshrrev_b64, 1, 1}, {"v_fma_f64", k_fma_f64, 1, 1},
      {"mac+1add", k_mix_mac_add1, 2, 1},     {"mac+2add", k_mix_mac_add2, 3, 1},
      {"mac+3add", k_mix_mac_add3, 4, 1},
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int waves_list[] = {1, 2, 4, 8};
  for (auto& k : ks) {
    for (int wps : waves_list) {
      const int blocks = simds * wps / 4;
      const int iters = 65536 / wps * 2;  // ~ constant work per SIMD across wave counts
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, clk, 1u, 64);  // warm
      hipDeviceSynchronize();
      float best = 1e30f;
      double clk_ratio = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, clk, (uint32_t)rep, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) {
          best = ms;
          const int nw = blocks * 4;
          hipMemcpy(hclk.data(), clk, sizeof(unsigned long long) * 2 * nw, hipMemcpyDeviceToHost);
          double cyc = 0, rt = 0;
          for (int w = 0; w < nw; ++w) {
            cyc += (double)hclk[2 * w];
            rt += (double)hclk[2 * w + 1];
          }
          clk_ratio = cyc / rt;  // memtime ticks per wall-clock tick
        }
      }
      const double lane_ops = (double)blocks * threads * iters * CH * k.lane_ops;
      const double instrs = (double)blocks * threads * iters * CH * k.per;
      const double rate = lane_ops / (best * 1e-3);
      const double memtime_mhz = clk_ratio * wall_khz / 1e3;
      printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"lane_ops_per_s\": %.4e, "
             "\"valu_lane_instr_per_s\": %.4e, \"memtime_mhz\": %.1f, \"lanes_per_clk_per_simd_at_2.4GHz\": %.2f, "
             "\"instr_lanes_per_clk_per_simd_at_memtime\": %.2f}\n",
             k.n, wps, best, rate, instrs / (best * 1e-3), memtime_mhz, rate / simds / 2.4e9,
             instrs / (best * 1e-3) / simds / (memtime_mhz * 1e6));
      fflush(stdout);
    }
  }
  hipFree(out);
  hipFree(clk);
  return 0;
}
