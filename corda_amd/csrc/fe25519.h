// GF(2^255 - 19) arithmetic for gfx950, one field element per lane in VGPRs.
//
// Representation: 10 unsigned 32-bit limbs, radix 2^25.5 (limb i at bit offset
// ceil(25.5 i): 0,26,51,77,102,128,153,179,204,230; even limbs 26 bits, odd limbs 25 bits).
// Chosen from the gfx950 integer microbenchmark (profiles/r01/ubench_int.json): a
// 32x32->64 multiply-accumulate (v_mad_u64_u32) costs about one carry-producing add,
// while plain 32-bit adds (VOP2, no VCC write) issue at twice that rate. With 25.5-bit
// limbs every limb product is ONE v_mad_u64_u32 into a 64-bit column accumulator with no
// per-product carry, and field add/sub are carry-free 32-bit VOP2 ops.
//
// Bound discipline (checked on the host by tests/test_fe_host.py through the
// FE_BOUNDS_CHECK build of this header):
//   "tight"  = output of fe_mul / fe_sq / fe_carry / fe_frombytes:
//              even limbs < 2^26, odd limbs < 2^25 + 2^18 (limb 1 may carry a little).
//   fe_add(T,T)            -> <= 2 tight
//   fe_sub(a, b)           a + 2p - b, requires b tight;      -> <= 3 tight
//   fe_sub4(a, b)          a + 4p - b, requires b <= 2 tight;  -> <= 5 tight (use fe_carry)
//   fe_mul(f, g)           f <= 5 tight, g <= 3 tight  (19*g_j must fit 32 bits)
//   fe_sq(f)               f <= 2 tight
// The point formulas in ge25519.h are written against these rules.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CG_HD __host__ __device__ __forceinline__
#define CG_HDS __host__ __device__ static __forceinline__  // static member functions
#define CG_HDM __host__ __device__ __forceinline__         // non-static member functions
#else
#define CG_HD static inline
#define CG_HDS static inline
#define CG_HDM inline
#endif

#ifdef FE_BOUNDS_CHECK
#include <assert.h>
typedef unsigned __int128 fe_acc_t;
#define FE_ASSERT(x) assert(x)
#else
typedef uint64_t fe_acc_t;
#define FE_ASSERT(x) ((void)0)
#endif

struct fe {
  uint32_t v[10];
};

// Host-build op counters (tests/native/host_kernels.cpp): define the executed-work figure
// bench.py prices the kernels with. Compiled out of the device build.
#ifdef FE_OP_COUNT
extern uint64_t g_fe_nmul, g_fe_nsq;
#define FE_COUNT(c) (++(c))
#else
#define FE_COUNT(c) ((void)0)
#endif

#define FE_M26 0x3ffffffu
#define FE_M25 0x1ffffffu

CG_HD void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
CG_HD void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
// 1/2 = (p + 1) / 2 = 2^254 - 9 (tight)
CG_HD void fe_half(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = (i & 1) ? 0x1ffffffu : 0x3ffffffu;
  h.v[0] = 0x3fffff7u;
  h.v[9] = 0xffffffu;
}
CG_HD void fe_copy(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i];
}

CG_HD void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// h = f + 2p - g ; requires g tight (each limb of g <= limb of 2p)
CG_HD void fe_sub(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t b = (i == 0) ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu);
    FE_ASSERT(g.v[i] <= b);
    h.v[i] = (f.v[i] + b) - g.v[i];
  }
}

// h = f + 4p - g ; requires g <= 2 tight
CG_HD void fe_sub4(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t b = (i == 0) ? 0xfffffb4u : ((i & 1) ? 0x7fffffcu : 0xffffffcu);
    FE_ASSERT(g.v[i] <= b);
    h.v[i] = (f.v[i] + b) - g.v[i];
  }
}

// h = -f = 2p - f (f tight)
CG_HD void fe_neg(fe& h, const fe& f) {
  fe z;
  fe_0(z);
  fe_sub(h, z, f);
}

// One carry pass on 32-bit limbs (cheap VOP2 ops): output tight.
CG_HD void fe_carry(fe& h) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    c = h.v[i] >> sh;
    h.v[i] &= (i & 1) ? FE_M25 : FE_M26;
    h.v[i + 1] += c;
  }
  c = h.v[9] >> 25;
  h.v[9] &= FE_M25;
  h.v[0] += 19u * c;
  c = h.v[0] >> 26;
  h.v[0] &= FE_M26;
  h.v[1] += c;
}

// 64-bit column accumulators -> tight 32-bit limbs (ref10 carry order, unsigned truncation).
CG_HD void fe_reduce_cols(fe& out, fe_acc_t* h) {
#define FE_CARRY(i, sh)                       \
  {                                           \
    fe_acc_t c = h[i] >> (sh);                \
    h[(i) + 1] += c;                          \
    h[i] &= ((fe_acc_t)1 << (sh)) - 1;        \
  }
#ifdef FE_SINGLE_CARRY_CHAIN  // one chain 0 -> 9 (11 carries): 2% fewer ladder instructions, a longer dependency chain
  FE_CARRY(0, 26);
  FE_CARRY(1, 25);
  FE_CARRY(2, 26);
  FE_CARRY(3, 25);
  FE_CARRY(4, 26);
  FE_CARRY(5, 25);
  FE_CARRY(6, 26);
  FE_CARRY(7, 25);
  FE_CARRY(8, 26);
#else  // two interleaved chains (ref10 order, 12 carries)
  FE_CARRY(0, 26);
  FE_CARRY(4, 26);
  FE_CARRY(1, 25);
  FE_CARRY(5, 25);
  FE_CARRY(2, 26);
  FE_CARRY(6, 26);
  FE_CARRY(3, 25);
  FE_CARRY(7, 25);
  FE_CARRY(4, 26);
  FE_CARRY(8, 26);
#endif
  {
    fe_acc_t c = h[9] >> 25;
    h[9] &= FE_M25;
    h[0] += c * 19u;
  }
  FE_CARRY(0, 26);
#undef FE_CARRY
#ifdef FE_BOUNDS_CHECK
  for (int i = 0; i < 10; ++i) FE_ASSERT(h[i] < ((fe_acc_t)1 << 32));
#endif
#pragma unroll
  for (int i = 0; i < 10; ++i) out.v[i] = (uint32_t)h[i];
}

// h = f * g
CG_HD void fe_mul(fe& out, const fe& f, const fe& g) {
  FE_COUNT(g_fe_nmul);
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    FE_ASSERT((uint64_t)g.v[i] * 19u < (1ull << 32));
    g19[i] = g.v[i] * 19u;
    f2[i] = (i & 1) ? (f.v[i] << 1) : f.v[i];
  }
  fe_acc_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int k = i + j;
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      const uint32_t b = (k >= 10) ? g19[j] : g.v[j];
      h[k >= 10 ? k - 10 : k] += (fe_acc_t)((uint64_t)a * b);
#ifdef FE_BOUNDS_CHECK
      FE_ASSERT(h[k >= 10 ? k - 10 : k] < ((fe_acc_t)1 << 64));
#endif
    }
  }
  fe_reduce_cols(out, h);
}

// h = f^2
CG_HD void fe_sq(fe& out, const fe& f) {
  // term (i<j): 2 f_i f_j, times 2 if both odd, times 19 if i+j >= 10
  // term (i=i): f_i^2, times 2 if i odd, times 19 if 2i >= 10
  FE_COUNT(g_fe_nsq);
  uint32_t f2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    FE_ASSERT((uint64_t)f.v[i] * 19u < (1ull << 32));
    f2[i] = f.v[i] << 1;
    f19[i] = f.v[i] * 19u;
  }
  fe_acc_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      const int k = i + j;
      const bool odd2 = (i & 1) && (j & 1);
      const bool wrap = k >= 10;
      // multiplier = (i<j ? 2 : 1) * (odd2 ? 2 : 1) * (wrap ? 19 : 1)
      uint32_t a, b;
      if (i < j) {
        a = odd2 ? (f2[i] << 1) : f2[i];      // 2 or 4 times f_i  (f_i odd when odd2: <= 2^27.x)
        b = wrap ? f19[j] : f.v[j];
      } else {
        a = odd2 ? f2[i] : f.v[i];
        b = wrap ? f19[j] : f.v[j];
      }
      FE_ASSERT(i < j ? ((uint64_t)f.v[i] * (odd2 ? 4u : 2u) < (1ull << 32)) : true);
      h[wrap ? k - 10 : k] += (fe_acc_t)((uint64_t)a * b);
#ifdef FE_BOUNDS_CHECK
      FE_ASSERT(h[wrap ? k - 10 : k] < ((fe_acc_t)1 << 64));
#endif
    }
  }
  fe_reduce_cols(out, h);
}

// h = 2 f^2
CG_HD void fe_sq2(fe& out, const fe& f) {
  fe t;
  fe_sq(t, f);
  fe_add(t, t, t);
  fe_carry(t);
  fe_copy(out, t);
}

CG_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// z^(p-2) (addition chain of ref10 fe_invert: 254 squarings, 11 multiplies)
CG_HD void fe_invert(fe& out, const fe& z) {
  fe t0, t1, t2, t3;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(t0, t0, t1);
  fe_sq(t2, t0);
  fe_mul(t1, t1, t2);
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 5);
  fe_mul(out, t1, t0);
}

// z^((p-5)/8) = z^(2^252 - 3)
CG_HD void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq(t0, z);
  fe_sqn(t1, t0, 2);
  fe_mul(t1, z, t1);
  fe_mul(t0, t0, t1);
  fe_sq(t0, t0);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);
  fe_sqn(t0, t0, 2);
  fe_mul(out, t0, z);
}

// Little-endian 32 bytes (bit 255 ignored) -> limbs. Accepts y >= p (i2p fromByteArray).
CG_HD void fe_frombytes_words(fe& h, const uint32_t w[8]) {
  // bit offsets 0,26,51,77,102,128,153,179,204,230
  auto bits = [&](int off, int n) -> uint32_t {
    const int wi = off >> 5, sh = off & 31;
    uint64_t x = (uint64_t)w[wi] >> sh;
    if (sh + n > 32 && wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    return (uint32_t)x & ((1u << n) - 1);
  };
  h.v[0] = bits(0, 26);
  h.v[1] = bits(26, 25);
  h.v[2] = bits(51, 26);
  h.v[3] = bits(77, 25);
  h.v[4] = bits(102, 26);
  h.v[5] = bits(128, 25);
  h.v[6] = bits(153, 26);
  h.v[7] = bits(179, 25);
  h.v[8] = bits(204, 26);
  h.v[9] = bits(230, 25);
}

// Canonical encoding (fully reduced mod p) as 8 little-endian words. Input: any limbs that
// fe_carry accepts (<= 5 tight).
CG_HD void fe_tobytes_words(uint32_t w[8], const fe& f) {
  fe h;
  fe_copy(h, f);
  fe_carry(h);
  fe_carry(h);  // now tight with limb1 < 2^25 + tiny; value < 2^255 + small
  // q = floor((h + 19) / 2^255) in {0,1}
  uint32_t q = (h.v[0] + 19u) >> 26;
  q = (h.v[1] + q) >> 25;
  q = (h.v[2] + q) >> 26;
  q = (h.v[3] + q) >> 25;
  q = (h.v[4] + q) >> 26;
  q = (h.v[5] + q) >> 25;
  q = (h.v[6] + q) >> 26;
  q = (h.v[7] + q) >> 25;
  q = (h.v[8] + q) >> 26;
  q = (h.v[9] + q) >> 25;
  h.v[0] += 19u * q;
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int sh = (i & 1) ? 25 : 26;
    c = h.v[i] >> sh;
    h.v[i] &= (i & 1) ? FE_M25 : FE_M26;
    h.v[i + 1] += c;
  }
  h.v[9] &= FE_M25;  // drop 2^255 * q
  w[0] = h.v[0] | (h.v[1] << 26);
  w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
  w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
  w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
  w[4] = h.v[5];
  w[4] |= h.v[6] << 25;
  w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
  w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
  w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

CG_HD int fe_isnegative(const fe& f) {
  uint32_t w[8];
  fe_tobytes_words(w, f);
  return (int)(w[0] & 1);
}

CG_HD int fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes_words(w, f);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= w[i];
  return o == 0;
}

// constant-index select helpers
CG_HD void fe_cmov(fe& h, const fe& f, uint32_t b) {
  const uint32_t m = 0u - b;
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] ^= (h.v[i] ^ f.v[i]) & m;
}
