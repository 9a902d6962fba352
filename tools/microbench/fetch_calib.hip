// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns the bench's
// roofline.traffic prices (`hbm = 2 FETCH_SIZE + WRITE_SIZE` was an unvalidated
// "upper estimate for table gathers"). Each kernel moves a known number of bytes from / to HBM
// (tables far larger than the 256 MB Infinity Cache, every line touched once per launch):
//   stream  : 16 B per lane, coalesced, over N bytes; writes the same N bytes elsewhere
//   gather7 : the wide ladders' pattern: per lane 7 x 16-B global_load_lds of one 112-B entry at a
//             random 16-B-aligned offset (the entry is contiguous, lanes are scattered), K per lane
//   gather1 : one 16-B load per lane at a random 16-B-aligned offset
// Printed per kernel: launches, the bytes a lane requested, and the HBM bytes they touch in whole
// 128-B lines (the minimum the memory side can move). Run each PMC pass separately:
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -- ./fetch_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -d <dir> -- ./fetch_calib
// and compare FETCH_SIZE (kB) per dispatch with the printed line bytes (tools/pmc_traffic.py uses
// the measured ratio). Build: hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// one 112-B entry per lane and round into the wave's LDS slot (global_load_lds_dwordx4, as
// ed_glds_niels9 does), then one VGPR read so the loads are not dead
__global__ void __launch_bounds__(256) k_gather7(const uint8_t* __restrict__ tab, uint64_t entries, int rounds,
                                                 uint32_t* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4 * 7 * 1024];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint8_t* wl = stage + wave * 7 * 1024;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  typedef __attribute__((address_space(1))) void* gbl_ptr;
  const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr)wl);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    const uint64_t e = ((uint64_t)mix(t * 0x9E3779B9u + (uint32_t)r * 0x85EBCA6Bu) * 4096u + mix(t + 77u * r)) % entries;
    const uint8_t* p = tab + e * 112;
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      __builtin_amdgcn_global_load_lds((gbl_ptr)(p + 16 * c), (lds_ptr)(uintptr_t)(base + c * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += ((const uint32_t*)(wl + lane * 16))[0];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) sink[t] = acc;
}

__global__ void __launch_bounds__(256) k_gather1(const uint4* __restrict__ tab, uint64_t n16, int rounds,
                                                 uint32_t* __restrict__ sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    const uint64_t e = ((uint64_t)mix(t * 0x9E3779B9u + (uint32_t)r * 0x85EBCA6Bu) * 4096u + mix(t + 77u * r)) % n16;
    acc += tab[e].x;
  }
  if (acc == 0x12345678u) sink[t] = acc;
}

int main() {
  const uint64_t tab_bytes = 8ull << 30;  // 8 GB: far past the Infinity Cache
  uint8_t *tab = nullptr, *dst = nullptr;
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(&tab, tab_bytes));
  CHECK(hipMalloc(&dst, 2ull << 30));
  CHECK(hipMalloc(&sink, 64u << 20));
  CHECK(hipMemset(tab, 1, tab_bytes));
  CHECK(hipDeviceSynchronize());
  // stream: 2 GB read + 2 GB written
  const uint64_t sbytes = 2ull << 30;
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)tab, (uint4*)dst, sbytes / 16);
  CHECK(hipDeviceSynchronize());
  printf("{\"kernel\": \"k_stream\", \"read_bytes\": %llu, \"write_bytes\": %llu, \"line_bytes\": %llu}\n",
         (unsigned long long)sbytes, (unsigned long long)sbytes, (unsigned long long)sbytes);
  // gather7: 256k lanes x 8 rounds of one 112-B entry (random over 8 GB: essentially no line reuse)
  const uint32_t lanes = 1u << 18;
  const int rounds = 8;
  const uint64_t entries = tab_bytes / 112;
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_gather7, dim3(lanes / 256), dim3(256), 0, 0, tab, entries, rounds, sink);
  CHECK(hipDeviceSynchronize());
  // a 112-B entry at 112 k starts at 16 (7 k mod 8) within its 128-B line: it fits one line for
  // offsets 0 and 16 (2 of 8), else spans two -> 1.75 lines = 224 B per entry on average
  const double lines7 = 1.75;
  printf("{\"kernel\": \"k_gather7\", \"read_bytes\": %llu, \"line_bytes\": %llu}\n",
         (unsigned long long)((uint64_t)lanes * rounds * 112), (unsigned long long)((double)lanes * rounds * lines7 * 128));
  // gather1: 256k lanes x 32 rounds of 16 B
  const int r1 = 32;
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_gather1, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)tab, tab_bytes / 16, r1, sink);
  CHECK(hipDeviceSynchronize());
  printf("{\"kernel\": \"k_gather1\", \"read_bytes\": %llu, \"line_bytes\": %llu}\n",
         (unsigned long long)((uint64_t)lanes * r1 * 16), (unsigned long long)((uint64_t)lanes * r1 * 128));
  CHECK(hipFree(tab));
  CHECK(hipFree(dst));
  CHECK(hipFree(sink));
  return 0;
}
