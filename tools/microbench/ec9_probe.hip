// Static instruction counts of one ec9 product / one wide-ladder addition (ec9.h), compiled alone
// so that an edit to the field code can be priced in seconds instead of verify_ec.hip's minutes:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -Icorda_amd/csrc -Iinclude \
//         tools/microbench/ec9_probe.hip -o /tmp/ec9.s && python3 tools/isa_mix.py /tmp/ec9.s <symbol>
// Each kernel's loop body is one operation on loop-carried values (nothing is hoisted).
#define EC9_NO_EXACT 1
#include <hip/hip_runtime.h>

#include "ec9.h"

namespace cgp {
template <int C, int Form>
__global__ void __launch_bounds__(256) k_mul(uint32_t* __restrict__ io, int n) {
  f29 a, b, c, d;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < 9; ++i) {
    a.v[i] = io[i * 4096 + t];
    b.v[i] = io[(9 + i) * 4096 + t];
    c.v[i] = io[(18 + i) * 4096 + t];
    d.v[i] = io[(27 + i) * 4096 + t];
  }
  for (int k = 0; k < n; ++k) {
    f29 r;
    if (Form == 0) ec9_mul<C>(r, a, b);
    else if (Form == 1) ec9_mul_add<C>(r, a, b, c);
    else ec9_mul2<C>(r, a, b, c, d);
    a = b;
    b = r;
  }
  for (int i = 0; i < 9; ++i) io[i * 4096 + t] = b.v[i];
}

template <int C>
__global__ void __launch_bounds__(256) k_madd(uint32_t* __restrict__ io, const uint32_t* __restrict__ tab, int n) {
  Jac r;
  f29 x2, y2;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < 9; ++i) {
    r.X.v[i] = io[i * 4096 + t];
    r.Y.v[i] = io[(9 + i) * 4096 + t];
    r.Z.v[i] = io[(18 + i) * 4096 + t];
  }
  EcConsts K;
  bool inf = false;
  for (int k = 0; k < n; ++k) {
    for (int i = 0; i < 9; ++i) {
      x2.v[i] = tab[(k & 1023) * 18 + i];
      y2.v[i] = tab[(k & 1023) * 18 + 9 + i];
    }
    jac_madd9<C>(r, inf, x2, y2, (k & 1) != 0, K);
  }
  for (int i = 0; i < 9; ++i) io[i * 4096 + t] = r.X.v[i] + r.Y.v[i] + r.Z.v[i] + inf;
}

template __global__ void k_mul<CG_CURVE_R1, 0>(uint32_t*, int);
template __global__ void k_mul<CG_CURVE_R1, 1>(uint32_t*, int);
template __global__ void k_mul<CG_CURVE_R1, 2>(uint32_t*, int);
template __global__ void k_mul<CG_CURVE_K1, 0>(uint32_t*, int);
template __global__ void k_mul<CG_CURVE_K1, 1>(uint32_t*, int);
template __global__ void k_mul<CG_CURVE_K1, 2>(uint32_t*, int);
template __global__ void k_madd<CG_CURVE_R1>(uint32_t*, const uint32_t*, int);
template __global__ void k_madd<CG_CURVE_K1>(uint32_t*, const uint32_t*, int);
}  // namespace cgp
