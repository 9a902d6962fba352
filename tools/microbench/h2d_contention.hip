// Does an H2D stream slow device kernels? Times an HBM-bound copy kernel and a small fill kernel
// (the plan's shapes) alone, beside a pageable hipMemcpyAsync, beside a pinned one, and beside a
// pinned one fed by a 16-thread host memcpy (the CG_STAGED_H2D design). Run on the GPU box.
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 h2d_contention.hip -o h2d_contention -lpthread
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void k_fill(uint32_t* __restrict__ p, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

int main() {
  const size_t NB = 256u << 20, NH = 1024u << 20, NF = 2u << 20;
  uint4 *a, *b;
  uint32_t* f;
  uint8_t *dh, *pg, *pin;
  CK(hipMalloc(&a, NB));
  CK(hipMalloc(&b, NB));
  CK(hipMalloc(&f, NF * 4));
  CK(hipMalloc(&dh, NH));
  pg = (uint8_t*)aligned_alloc(4096, NH);
  memset(pg, 1, NH);
  CK(hipHostMalloc(&pin, NH, hipHostMallocDefault));
  memset(pin, 2, NH);
  hipStream_t sk, sc;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  auto kernels = [&](const char* tag) {
    // 20 copy launches then 200 fills, each group timed by events
    const int nc = 20, nf = 200;
    CK(hipEventRecord(e0, sk));
    for (int r = 0; r < nc; ++r) hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, sk, a, b, NB / 16);
    CK(hipEventRecord(e1, sk));
    for (int r = 0; r < nf; ++r) hipLaunchKernelGGL(k_fill, dim3((unsigned)(NF / 256)), dim3(256), 0, sk, f, NF);
    CK(hipEventRecord(e2, sk));
    CK(hipEventSynchronize(e2));
    float c = 0, d = 0;
    CK(hipEventElapsedTime(&c, e0, e1));
    CK(hipEventElapsedTime(&d, e1, e2));
    printf("{\"case\": \"%s\", \"copy_us\": %.1f, \"copy_GBps\": %.0f, \"fill_us\": %.2f}\n", tag, c * 1e3 / nc,
           2.0 * NB * nc / (c * 1e-3) / 1e9, d * 1e3 / nf);
  };
  kernels("warm");
  kernels("alone");
  // beside a long pageable copy: the host thread is blocked in the call, so launch kernels first
  // from a helper thread
  auto beside = [&](const char* tag, auto copy) {
    std::atomic<bool> go{false};
    std::thread t([&] {
      CK(hipSetDevice(0));
      while (!go.load()) {
      }
      copy();
    });
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    kernels(tag);
    t.join();
    CK(hipStreamSynchronize(sc));
  };
  auto pageable = [&] {
    for (int r = 0; r < 4; ++r) CK(hipMemcpyAsync(dh, pg, NH, hipMemcpyHostToDevice, sc));
  };
  auto pinned = [&] {
    for (int r = 0; r < 4; ++r) CK(hipMemcpyAsync(dh, pin, NH, hipMemcpyHostToDevice, sc));
  };
  auto staged = [&] {
    // 16 host threads refill 32 MB slots while the DMA drains them
    const size_t piece = 32u << 20;
    hipEvent_t ev[4];
    bool used[4] = {};
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int r = 0; r < 4; ++r)
      for (size_t off = 0, k = 0; off < NH; off += piece, ++k) {
        const int s = (int)(k & 3);
        if (used[s]) CK(hipEventSynchronize(ev[s]));
        std::vector<std::thread> th;
        for (int t = 0; t < 16; ++t)
          th.emplace_back([=] { memcpy(pin + s * piece + piece * t / 16, pg + off + piece * t / 16, piece / 16); });
        for (auto& x : th) x.join();
        CK(hipMemcpyAsync(dh + off, pin + s * piece, piece, hipMemcpyHostToDevice, sc));
        CK(hipEventRecord(ev[s], sc));
        used[s] = true;
      }
  };
  beside("pageable_h2d", pageable);
  beside("pinned_h2d", pinned);
  beside("staged_h2d", staged);
  kernels("alone_after");
  // copy rates alone
  for (int m = 0; m < 3; ++m) {
    auto t0 = std::chrono::steady_clock::now();
    if (m == 0) pageable();
    if (m == 1) pinned();
    if (m == 2) staged();
    CK(hipStreamSynchronize(sc));
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"copy\": \"%s\", \"GBps\": %.1f}\n", m == 0 ? "pageable" : m == 1 ? "pinned" : "staged", 4.0 * NH / s / 1e9);
  }
  return 0;
}
