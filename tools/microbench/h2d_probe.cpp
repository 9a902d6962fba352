// H2D transfer probe for the host-buffer entry points' staging design (run on the GPU box):
// pageable vs pinned hipMemcpyAsync, a threaded memcpy into pinned staging, hipHostRegister cost.
// Build: hipcc -O2 -std=c++17 h2d_probe.cpp -o h2d_probe -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_memcpy(uint8_t* d, const uint8_t* s, size_t n, int nt) {
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    size_t a = n * t / nt, b = n * (t + 1) / nt;
    th.emplace_back([=] { memcpy(d + a, s + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const size_t N = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024) << 20;
  const int reps = 3;
  uint8_t* pg = (uint8_t*)aligned_alloc(4096, N);
  for (size_t i = 0; i < N; i += 4096) pg[i] = (uint8_t)i;
  memset(pg, 1, N);
  uint8_t *pin, *dev;
  CK(hipHostMalloc(&pin, N, hipHostMallocDefault));
  memset(pin, 2, N);
  CK(hipMalloc(&dev, N));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto bw = [&](const char* name, auto fn) {
    fn();
    CK(hipStreamSynchronize(s));
    double t = now_ms();
    for (int r = 0; r < reps; ++r) fn();
    CK(hipStreamSynchronize(s));
    double ms = (now_ms() - t) / reps;
    printf("{\"probe\": \"%s\", \"MB\": %zu, \"ms\": %.3f, \"GBps\": %.2f}\n", name, N >> 20, ms, N / ms / 1e6);
  };
  bw("pageable_async", [&] { CK(hipMemcpyAsync(dev, pg, N, hipMemcpyHostToDevice, s)); });
  // host-side blocking time of one pageable async call
  {
    double t = now_ms();
    CK(hipMemcpyAsync(dev, pg, N, hipMemcpyHostToDevice, s));
    double ret = now_ms() - t;
    CK(hipStreamSynchronize(s));
    printf("{\"probe\": \"pageable_async_return\", \"ms_to_return\": %.3f, \"ms_total\": %.3f}\n", ret, now_ms() - t);
  }
  bw("pinned_async", [&] { CK(hipMemcpyAsync(dev, pin, N, hipMemcpyHostToDevice, s)); });
  for (int nt : {1, 4, 8, 16}) {
    char name[64];
    snprintf(name, sizeof name, "memcpy_to_pinned_%dt", nt);
    bw(name, [&] { par_memcpy(pin, pg, N, nt); });
  }
  // staged: threaded memcpy of 64 MB pieces into two pinned halves, each followed by its DMA
  for (int nt : {8, 16}) {
    const size_t piece = 64u << 20;
    hipEvent_t ev[2];
    CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    bool rec[2] = {false, false};
    char name[64];
    snprintf(name, sizeof name, "staged_64MB_x2_%dt", nt);
    bw(name, [&] {
      for (size_t off = 0, k = 0; off < N; off += piece, ++k) {
        const size_t n = N - off < piece ? N - off : piece;
        uint8_t* st = pin + (k & 1) * piece;
        if (rec[k & 1]) CK(hipEventSynchronize(ev[k & 1]));
        par_memcpy(st, pg + off, n, nt);
        CK(hipMemcpyAsync(dev + off, st, n, hipMemcpyHostToDevice, s));
        CK(hipEventRecord(ev[k & 1], s));
        rec[k & 1] = true;
      }
    });
  }
  {
    double t = now_ms();
    CK(hipHostRegister(pg, N, hipHostRegisterDefault));
    double reg = now_ms() - t;
    bw("registered_async", [&] { CK(hipMemcpyAsync(dev, pg, N, hipMemcpyHostToDevice, s)); });
    t = now_ms();
    CK(hipHostUnregister(pg));
    printf("{\"probe\": \"host_register\", \"ms_register\": %.3f, \"ms_unregister\": %.3f}\n", reg, now_ms() - t);
  }
  bw("d2h_pinned", [&] { CK(hipMemcpyAsync(pin, dev, N, hipMemcpyDeviceToHost, s)); });
  bw("d2h_pageable", [&] { CK(hipMemcpyAsync(pg, dev, N, hipMemcpyDeviceToHost, s)); });
  return 0;
}
