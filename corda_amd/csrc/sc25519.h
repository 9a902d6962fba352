// Scalars modulo L = 2^252 + 27742317777372353535851937790883648493 (the Ed25519 group
// order), one scalar per lane as 8 little-endian 32-bit words. Barrett reduction
// (HAC 14.42, b = 2^32, k = 8) on v_mad_u64_u32 products; everything fully unrolled so the
// words stay in VGPRs.
#pragma once
#include "fe25519.h"

#define SC_L0 0x5cf5d3edu
#define SC_L1 0x5812631au
#define SC_L2 0xa2f79cd6u
#define SC_L3 0x14def9deu
#define SC_L4 0u
#define SC_L5 0u
#define SC_L6 0u
#define SC_L7 0x10000000u

CG_HD uint32_t sc_Lw(int i) {
  return i == 0 ? SC_L0 : i == 1 ? SC_L1 : i == 2 ? SC_L2 : i == 3 ? SC_L3 : i == 7 ? SC_L7 : 0u;
}
// mu = floor(2^512 / L), 9 words (top word 0xf)
CG_HD uint32_t sc_MUw(int i) {
  const uint32_t MU[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du,
                          0xffffffebu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  return MU[i];
}

// r (8 words) = x mod L, x given as 16 words (512-bit little-endian)
CG_HD void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  // q1 = x >> 224 (9 words: x[7..15])
  // q3 = (q1 * mu) >> 288 ; we need words 9..17 of the 18-word product
  uint32_t q3[9];
  {
    uint64_t acc_lo = 0;  // column accumulator as 96-bit: (hi32:acc_lo)
    uint32_t acc_hi = 0;
    uint32_t prod[18];
#pragma unroll
    for (int k = 0; k < 18; ++k) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int j = k - i;
        if (j < 0 || j > 8) continue;
        const uint64_t p = (uint64_t)x[7 + i] * sc_MUw(j);
        const uint64_t s = acc_lo + p;
        acc_hi += (s < p);
        acc_lo = s;
      }
      prod[k] = (uint32_t)acc_lo;
      acc_lo = (acc_lo >> 32) | ((uint64_t)acc_hi << 32);
      acc_hi = 0;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) q3[i] = prod[9 + i];
  }
  // r2 = (q3 * L) mod 2^288 (9 words)
  uint32_t r2[9];
  {
    uint64_t acc_lo = 0;
    uint32_t acc_hi = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int j = k - i;
        if (j < 0 || j > 7) continue;
        const uint32_t lw = sc_Lw(j);
        if (lw == 0) continue;
        const uint64_t p = (uint64_t)q3[i] * lw;
        const uint64_t s = acc_lo + p;
        acc_hi += (s < p);
        acc_lo = s;
      }
      r2[k] = (uint32_t)acc_lo;
      acc_lo = (acc_lo >> 32) | ((uint64_t)acc_hi << 32);
      acc_hi = 0;
    }
  }
  // r = x mod 2^288 - r2 (mod 2^288)
  uint32_t t[9];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - br;
    t[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  // at most two subtractions of L
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    uint32_t u[9];
    uint64_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const uint64_t d = (uint64_t)t[i] - (i < 8 ? sc_Lw(i) : 0u) - b2;
      u[i] = (uint32_t)d;
      b2 = (d >> 63) & 1;
    }
    const uint32_t keep = (uint32_t)b2;  // borrow => t < L => keep t
    const uint32_t m = keep - 1u;        // all ones when we take u
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = (t[i] & ~m) | (u[i] & m);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = t[i];
}

CG_HD void sc_reduce256(uint32_t r[8], const uint32_t x[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = x[i];
    w[8 + i] = 0;
  }
  sc_reduce512(r, w);
}

// r = a - b mod L, a, b < L
CG_HD void sc_sub(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[8];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - br;
    t[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  const uint32_t m = 0u - (uint32_t)br;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t s = (uint64_t)t[i] + (sc_Lw(i) & m) + c;
    r[i] = (uint32_t)s;
    c = s >> 32;
  }
}

// 2^256 mod L
CG_HD uint32_t sc_R1w(int i) {
  const uint32_t R1[8] = {0x8d98951du, 0xd6ec3174u, 0x737dcf70u, 0xc6ef5bf4u,
                          0xfffffffeu, 0xffffffffu, 0xffffffffu, 0x0fffffffu};
  return R1[i];
}

// i2p GroupElement.slide(S) drops a carry that runs past bit 255. slide() is the width-5
// signed sliding window (digits odd in [-15,15]); emulate its carries on W = S and report
// whether one escaped. Only possible when bit 255 of S is set, so the
// caller runs this only for those lanes.
CG_HD uint32_t sc_slide_escapes(const uint32_t s[8]) {
  uint32_t w[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = s[i];
  w[8] = 0;
  for (int i = 0; i < 252; ++i) {
    if (w[0] & 1) {
      const uint32_t v = w[0] & 31u;
      if (v >= 16) {
        // W += 32 - v
        uint64_t c = (uint64_t)w[0] + (32u - v);
        w[0] = (uint32_t)c;
        c >>= 32;
#pragma unroll
        for (int k = 1; k < 9; ++k) {
          c += w[k];
          w[k] = (uint32_t)c;
          c >>= 32;
        }
      } else {
        w[0] -= v;  // low 5 bits become 0, no borrow
      }
    }
    // W >>= 1
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = (w[k] >> 1) | (w[k + 1] << 31);
    w[8] >>= 1;
  }
  // W = U >> 252 ; bit 256 of U is bit 4 of W
  return (w[0] >> 4) & 1u;
}

// Signed radix-16 digits e[0..63] in [-8, 8] of a < 2^255 (ref10 ge_scalarmult_base recoding),
// packed 8 per word as 4-bit two's complement... stored as (e + 8) in 4 bits does not fit 17
// values, so keep e in [-8,7] via carry: digits in [-8,7], carry into the top digit (<= 8).
// Returned as 64 signed bytes packed in 16 words.
CG_HD void sc_recode16(uint32_t packed[16], const uint32_t a[8]) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) packed[w] = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    int e = (int)((a[i >> 3] >> ((i & 7) * 4)) & 15u) + carry;
    carry = (e + 8) >> 4;
    e -= carry << 4;
    packed[i >> 2] |= ((uint32_t)(e & 0xff)) << ((i & 3) * 8);
  }
  // a < 2^253 -> top nibble <= 1, so the final carry is 0 and e[63] in [-8, 8]
}

CG_HD int sc_digit(const uint32_t packed[16], int i) {
  return (int)(int8_t)(uint8_t)(packed[i >> 2] >> ((i & 3) * 8));
}
