// FIPS 180-4 SHA-256 / SHA-512 for one message per lane (host + device).
//
// Messages are read straight out of the caller's arena with 4-byte loads
// (unaligned offsets handled by a funnel shift), so nothing is staged per item.
// SHA-512 runs on 64-bit words (two VGPRs each); a 64-bit rotate is written as two
// v_alignbit_b32 (the compiler otherwise emits two 64-bit shifts + two ORs), Ch and Maj as one
// v_bfi_b32 per half, a 64-bit add is one v_lshl_add_u64.
#pragma once
#include "fe25519.h"

#if defined(__HIPCC__)
#define CG_BSWAP32(x) __builtin_bswap32(x)
#else
#define CG_BSWAP32(x) __builtin_bswap32(x)
#endif

CG_HD uint32_t cg_ld32(const uint8_t* p) { return *(const uint32_t*)p; }

// 4 little-endian bytes at arena[off..off+4); bytes at or past `len_rounded` (the arena
// length rounded up to 4) read as 0. The arena base must be 4-byte aligned.
CG_HD uint32_t cg_ld_bytes4(const uint8_t* arena, uint64_t len_rounded, uint64_t off) {
  const uint64_t a0 = off & ~(uint64_t)3;
  const uint32_t sh = (uint32_t)(off & 3) * 8u;
  const uint32_t w0 = a0 < len_rounded ? cg_ld32(arena + a0) : 0u;
  if (sh == 0) return w0;
  const uint32_t w1 = (a0 + 4) < len_rounded ? cg_ld32(arena + a0 + 4) : 0u;
  return (w0 >> sh) | (w1 << (32u - sh));
}

// Big-endian 32-bit word at message byte position `pos` (multiple of 4) of msg||0x80||0..
// with only the message part loaded; `len` = message length.
CG_HD uint32_t cg_msg_word_be(const uint8_t* arena, uint64_t len_rounded, uint64_t msg_off, uint64_t len,
                              uint64_t pos) {
  uint32_t raw = 0;
  if (pos < len) raw = cg_ld_bytes4(arena, len_rounded, msg_off + pos);
  const uint64_t rem = len > pos ? len - pos : 0;  // valid bytes in this word (capped below)
  uint32_t w;
  if (rem >= 4) {
    w = raw;
  } else {
    const uint32_t keep = rem ? (0xffffffffu >> (32u - 8u * (uint32_t)rem)) : 0u;
    w = raw & keep;
    if (pos <= len) w |= 0x80u << (8u * (uint32_t)rem);  // pad byte lives in this word
  }
  return CG_BSWAP32(w);
}

// ----------------------------------------------------------------- SHA-512
CG_HD uint64_t cg_rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  // n is a compile-time constant at every call site
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t a = n < 32 ? hi : lo, b = n < 32 ? lo : hi;
  const uint32_t r = (uint32_t)n & 31u;
  return ((uint64_t)__builtin_amdgcn_alignbit(b, a, r) << 32) | __builtin_amdgcn_alignbit(a, b, r);
#else
  return (x >> n) | (x << (64 - n));
#endif
}

// Three-input XOR and Maj(a, b, c): one v_bitop3_b32 per 32-bit word (truth tables 0x96 and 0xE8,
// symmetric in the operands). The compiler forms bitop3 from some 32-bit expressions but not from
// the halves of the 64-bit SHA-512 words.
CG_HD uint32_t cg_xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
CG_HD uint32_t cg_maj32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) | (c & (a | b));
#endif
}
CG_HD uint64_t cg_xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return ((uint64_t)cg_xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
         cg_xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
#ifndef CG_SHA512_BITOP3
// 2: Maj as bitop3 (priced 3% better, round 2); 4: Ch as bitop3 (round 5: k_ed_hash 5.5 -> 5.35 ms
// per headline step, profiles/r05/hash); the 64-bit xor3 form (1) costs more moves than it saves
#define CG_SHA512_BITOP3 6
#endif
// (e & f) ^ (~e & g): one bitfield select per 32-bit half. With CG_SHA512_BITOP3 & 4 an opaque
// bitop3 (truth table 0xCA: e ? f : g) per half: the compiler otherwise splits the disjoint OR into
// two terms it adds into T1 separately (v_and + v_bfi + two 64-bit adds per round)
CG_HD uint64_t cg_ch64(uint64_t e, uint64_t f, uint64_t g) {
#if (CG_SHA512_BITOP3 & 4) && defined(__HIP_DEVICE_COMPILE__)
  // (the builtin returns a signed int: each half goes through uint32_t before widening)
  const uint32_t hi = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(e >> 32), (uint32_t)(f >> 32),
                                                            (uint32_t)(g >> 32), 0xCA);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)e, (uint32_t)f, (uint32_t)g, 0xCA);
  return ((uint64_t)hi << 32) | lo;
#else
  return (e & f) | (~e & g);
#endif
}
CG_HD uint64_t cg_maj64(uint64_t a, uint64_t b, uint64_t c) {
#if CG_SHA512_BITOP3 & 2
  return ((uint64_t)cg_maj32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
         cg_maj32((uint32_t)a, (uint32_t)b, (uint32_t)c);
#else
  const uint64_t m = a ^ b;
  return (m & c) | (~m & b);
#endif
}
CG_HD uint64_t cg_x3_64(uint64_t a, uint64_t b, uint64_t c) {
#if CG_SHA512_BITOP3 & 1
  return cg_xor3_64(a, b, c);
#else
  return a ^ b ^ c;
#endif
}

// Round constants in constant memory: the rounds run in a rolled loop of 16 unrolled rounds
// (sha512_compress), so the constant of round r + j is a scalar load at a uniform index.
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ const uint64_t CG_K512[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
#else
static const uint64_t CG_K512[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
#endif
CG_HD uint64_t cg_k512(int i) { return CG_K512[i]; }

CG_HD void sha512_init(uint64_t s[8]) {
  s[0] = 0x6a09e667f3bcc908ULL;
  s[1] = 0xbb67ae8584caa73bULL;
  s[2] = 0x3c6ef372fe94f82bULL;
  s[3] = 0xa54ff53a5f1d36f1ULL;
  s[4] = 0x510e527fade682d1ULL;
  s[5] = 0x9b05688c2b3e6c1fULL;
  s[6] = 0x1f83d9abfb41bd6bULL;
  s[7] = 0x5be0cd19137e2179ULL;
}

// One SHA-512 round on the working variables named in rotated order (a..h of round i are
// v[(8 - i) & 7] .. : the caller passes them rotated, so no register moves are needed).
#define CG_SHA512_ROUND(a, b, c, d, e, f, g, h, k, wi)                                                   \
  {                                                                                                   \
    const uint64_t t1 = h + cg_x3_64(cg_rotr64(e, 14), cg_rotr64(e, 18), cg_rotr64(e, 41)) +            \
                        cg_ch64(e, f, g) + (k) + (wi);                                                \
    const uint64_t t2 = cg_x3_64(cg_rotr64(a, 28), cg_rotr64(a, 34), cg_rotr64(a, 39)) + cg_maj64(a, b, c); \
    d += t1;                                                                                          \
    h = t1 + t2;                                                                                      \
  }

// 8 rounds: after them the variables are back in their own roles
#define CG_SHA512_8ROUNDS(i0, W)                                   \
  CG_SHA512_ROUND(a, b, c, d, e, f, g, h, cg_k512((i0) + 0), W(0)) \
  CG_SHA512_ROUND(h, a, b, c, d, e, f, g, cg_k512((i0) + 1), W(1)) \
  CG_SHA512_ROUND(g, h, a, b, c, d, e, f, cg_k512((i0) + 2), W(2)) \
  CG_SHA512_ROUND(f, g, h, a, b, c, d, e, cg_k512((i0) + 3), W(3)) \
  CG_SHA512_ROUND(e, f, g, h, a, b, c, d, cg_k512((i0) + 4), W(4)) \
  CG_SHA512_ROUND(d, e, f, g, h, a, b, c, cg_k512((i0) + 5), W(5)) \
  CG_SHA512_ROUND(c, d, e, f, g, h, a, b, cg_k512((i0) + 6), W(6)) \
  CG_SHA512_ROUND(b, c, d, e, f, g, h, a, cg_k512((i0) + 7), W(7))

// message schedule word i = r + j (r a multiple of 16, j < 16) into the circular buffer slot j
CG_HD uint64_t sha512_sched(uint64_t w[16], int j) {
  const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
  const uint64_t s0 = cg_x3_64(cg_rotr64(w15, 1), cg_rotr64(w15, 8), w15 >> 7);
  const uint64_t s1 = cg_x3_64(cg_rotr64(w2, 19), cg_rotr64(w2, 61), w2 >> 6);
  w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
  return w[j];
}

// Rounds 0..15 straight, then 16..79 as a rolled loop of 16 unrolled rounds: the working
// variables rotate by renaming inside the body and come back to their roles every 8 rounds, the
// schedule's circular buffer is indexed statically, the constants are scalar loads. (Fully
// unrolled, 80 rounds per block spilled and thrashed the instruction cache; rolled round by round,
// every round paid 8 register moves.)
CG_HD void sha512_compress(uint64_t s[8], uint64_t w[16]) {
  uint64_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#define CG_W0(j) w[(j)]
#define CG_W1(j) w[8 + (j)]
  CG_SHA512_8ROUNDS(0, CG_W0)
  CG_SHA512_8ROUNDS(8, CG_W1)
#undef CG_W0
#undef CG_W1
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#define CG_S0(j) sha512_sched(w, (j))
#define CG_S1(j) sha512_sched(w, 8 + (j))
    CG_SHA512_8ROUNDS(r, CG_S0)
    CG_SHA512_8ROUNDS(r + 8, CG_S1)
#undef CG_S0
#undef CG_S1
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

// The same 80 rounds over a precomputed schedule with the round constants folded in
// (wk[t] = W[t] + K[t]: a block every lane of the wave shares, keyws.h TmplW512). The caller passes
// a wave-uniform pointer, so the words are scalar loads, as the round constants are.
CG_HD void sha512_compress_wk(uint64_t s[8], const uint64_t* __restrict__ wk) {
  uint64_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll 1
  for (int r = 0; r < 80; r += 8) {
    CG_SHA512_ROUND(a, b, c, d, e, f, g, h, wk[r + 0], 0)
    CG_SHA512_ROUND(h, a, b, c, d, e, f, g, wk[r + 1], 0)
    CG_SHA512_ROUND(g, h, a, b, c, d, e, f, wk[r + 2], 0)
    CG_SHA512_ROUND(f, g, h, a, b, c, d, e, wk[r + 3], 0)
    CG_SHA512_ROUND(e, f, g, h, a, b, c, d, wk[r + 4], 0)
    CG_SHA512_ROUND(d, e, f, g, h, a, b, c, wk[r + 5], 0)
    CG_SHA512_ROUND(c, d, e, f, g, h, a, b, wk[r + 6], 0)
    CG_SHA512_ROUND(b, c, d, e, f, g, h, a, wk[r + 7], 0)
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

// Four aligned little-endian dwords at arena[addr, addr + 16) (addr a multiple of 4), zero past
// `len_rounded`: one 16-byte load when the whole span is inside (gfx950 loads need only dword
// alignment), else dword by dword.
CG_HD void cg_ld_dwords4(uint32_t out[4], const uint8_t* arena, uint64_t len_rounded, uint64_t addr) {
  if (addr + 16 <= len_rounded) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4_a4 v = *(const u32x4_a4*)(arena + addr);
    out[0] = v.x;
    out[1] = v.y;
    out[2] = v.z;
    out[3] = v.w;
#else
    for (int q = 0; q < 4; ++q) out[q] = cg_ld32(arena + addr + 4 * q);
#endif
  } else {
    for (int q = 0; q < 4; ++q) out[q] = addr + 4 * q < len_rounded ? cg_ld32(arena + addr + 4 * q) : 0u;
  }
}

// ---- message sources. A message is read as aligned little-endian dwords at byte offsets relative
// to its 4-aligned base: ArenaLd over a contiguous arena span, or SpliceLd over a SignableData
// splice (cg_verify_tx_signatures): the template image prefix || 0^32 || suffix with the 32-byte tx
// id ORed in at byte `at` (two aligned id dwords and a funnel shift per overlapping word), so the
// spliced bytes are never written to memory.
struct ArenaLd {
  const uint8_t* arena;
  uint64_t len_rounded;
  CG_HDM void dwords4(uint32_t out[4], uint64_t addr) const { cg_ld_dwords4(out, arena, len_rounded, addr); }
  CG_HDM uint32_t bytes4(uint64_t off) const { return cg_ld_bytes4(arena, len_rounded, off); }
};
// The id's bytes x .. x + 3 (x may start before or run past the 32 id bytes: those read 0).
CG_HD uint32_t splice_id_word(const uint32_t* id, int64_t x) {
  if (x <= -4 || x >= 32) return 0u;
  const int64_t a = x >= 0 ? x >> 2 : -1;
  const uint32_t r = (uint32_t)(x - 4 * a);
  const uint32_t lo = a >= 0 ? id[a] : 0u;
  const uint32_t hi = a + 1 < 8 ? id[a + 1] : 0u;
  return r ? (lo >> (8 * r)) | (hi << (32 - 8 * r)) : lo;
}
struct SpliceLd {
  const uint8_t* img;   // template image, 16-aligned
  uint64_t img_len;     // image bytes (loads past them read 0)
  const uint32_t* id;   // 8 aligned dwords
  uint32_t at;          // id position (the prefix length)
  CG_HDM void dwords4(uint32_t out[4], uint64_t addr) const {
    cg_ld_dwords4(out, img, img_len, addr);
    const int64_t x0 = (int64_t)addr - (int64_t)at;
    if (x0 > -16 && x0 < 32) {
#pragma unroll
      for (int q = 0; q < 4; ++q) out[q] |= splice_id_word(id, x0 + 4 * q);
    }
  }
  CG_HDM uint32_t bytes4(uint64_t off) const {  // off is 4-aligned for a splice (base 0)
    return cg_ld_bytes4(img, img_len, off) | splice_id_word(id, (int64_t)off - (int64_t)at);
  }
};

// SHA-512(prefix64 || msg) where prefix64 is 16 little-endian words (e.g. R || Abyte).
// Output: the 64 digest bytes as 16 little-endian words (ready for sc_reduce512).
// The message is read as aligned 16-byte chunks (33 dwords per 128-byte block) and realigned with
// one funnel shift per word, instead of two dword loads per word (round 1: 136 loads per
// 270-byte message, the challenge kernel's memory-wait share was ~0.3).
template <class Ld>
CG_HD void sha512_prefix64_ld(uint32_t out[16], const uint32_t prefix[16], const Ld& ld, uint64_t msg_off,
                              uint64_t msg_len) {
  uint64_t s[8];
  sha512_init(s);
  const uint64_t n = 64 + msg_len;
  const uint64_t nblocks = (n + 17 + 127) >> 7;
  const uint64_t base = msg_off & ~(uint64_t)3;
  const uint32_t sh8 = (uint32_t)(msg_off & 3) * 8u;
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    // message words k0 .. k0 + 31 of this block (k0 = 32 blk - 16; block 0 starts with the prefix)
    const int64_t k0 = (int64_t)blk * 32 - 16;
    uint32_t W[36];  // aligned dwords k0 .. k0 + 35
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (blk == 0 && t < 4) {
        W[4 * t] = W[4 * t + 1] = W[4 * t + 2] = W[4 * t + 3] = 0u;
      } else {
        ld.dwords4(&W[4 * t], base + (uint64_t)(k0 + 4 * t) * 4);
      }
    }
    const bool last = blk + 1 == nblocks;
    uint32_t be[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int64_t k = k0 + j;  // message word (negative: prefix)
      uint32_t w;
      if (k < 0) {
        w = prefix[j];
      } else {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t raw = __builtin_amdgcn_alignbit(W[j + 1], W[j], sh8);
#else
        const uint32_t raw = (uint32_t)((((uint64_t)W[j + 1] << 32) | W[j]) >> sh8);
#endif
        const int64_t rem = (int64_t)msg_len - 4 * k;  // message bytes in this word
        if (rem >= 4) {
          w = raw;
        } else if (rem > 0) {
          w = (raw & (0xffffffffu >> (32u - 8u * (uint32_t)rem))) | (0x80u << (8u * (uint32_t)rem));
        } else {
          w = rem == 0 ? 0x80u : 0u;
        }
      }
      be[j] = CG_BSWAP32(w);
    }
    if (last) {  // the 128-bit big-endian bit length ends the last block
      be[28] = 0;
      be[29] = 0;
      be[30] = (uint32_t)((n * 8) >> 32);
      be[31] = (uint32_t)(n * 8);
    }
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = ((uint64_t)be[2 * j] << 32) | be[2 * j + 1];
    sha512_compress(s, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    out[2 * k] = CG_BSWAP32((uint32_t)(s[k] >> 32));
    out[2 * k + 1] = CG_BSWAP32((uint32_t)s[k]);
  }
}

// SHA-512(prefix64 || M) for M a SignableData splice (SpliceLd: base 0, zero past the message):
// the padding byte is ORed into its word, so no word tests the length, and with wk1 != nullptr
// (a wave-uniform TmplW512 record, the template's prefix covering M[64, 192)) block 1 runs from
// its precomputed schedule (sha512_compress_wk).
template <class Ld>
CG_HD void sha512_prefix64_splice(uint32_t out[16], const uint32_t prefix[16], const Ld& ld, uint32_t msg_len,
                                  const uint64_t* wk1) {
  uint64_t s[8];
  sha512_init(s);
  const uint64_t n = 64ull + msg_len;
  const uint32_t nblocks = (uint32_t)((n + 17u + 127u) >> 7);
  const int mw = (int)(msg_len >> 2);
  const uint32_t mk = 0x80u << (8u * (msg_len & 3u));
  for (uint32_t blk = 0; blk < nblocks; ++blk) {
    if (blk == 1 && wk1 != nullptr) {
      sha512_compress_wk(s, wk1);
      continue;
    }
    const int k0 = (int)blk * 32 - 16;  // message word of the block's first word (block 0: prefix first)
    uint32_t W[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (blk == 0 && q < 4) {
        W[4 * q] = W[4 * q + 1] = W[4 * q + 2] = W[4 * q + 3] = 0u;
      } else {
        ld.dwords4(&W[4 * q], (uint64_t)(k0 + 4 * q) * 4u);
      }
    }
    const int km = mw - k0;  // the padding byte's word in this block (may lie outside it)
    uint32_t be[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint32_t w = (blk == 0 && j < 16) ? prefix[j] : (W[j] | (j == km ? mk : 0u));
      be[j] = CG_BSWAP32(w);
    }
    if (blk + 1 == nblocks) {
      be[28] = 0;
      be[29] = 0;
      be[30] = (uint32_t)((n * 8u) >> 32);
      be[31] = (uint32_t)(n * 8u);
    }
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = ((uint64_t)be[2 * j] << 32) | be[2 * j + 1];
    sha512_compress(s, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    out[2 * k] = CG_BSWAP32((uint32_t)(s[k] >> 32));
    out[2 * k + 1] = CG_BSWAP32((uint32_t)s[k]);
  }
}

CG_HD void sha512_prefix64_msg(uint32_t out[16], const uint32_t prefix[16], const uint8_t* arena,
                               uint64_t len_rounded, uint64_t msg_off, uint64_t msg_len) {
  sha512_prefix64_ld(out, prefix, ArenaLd{arena, len_rounded}, msg_off, msg_len);
}

// Plain SHA-512 of arena[off, off+len)
CG_HD void sha512_arena(uint64_t s_out[8], const uint8_t* arena, uint64_t len_rounded, uint64_t off, uint64_t len) {
  uint64_t s[8];
  sha512_init(s);
  const uint64_t nblocks = (len + 17 + 127) >> 7;
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t pos = blk * 128 + (uint64_t)j * 8;
      uint32_t hi = cg_msg_word_be(arena, len_rounded, off, len, pos);
      uint32_t lo = cg_msg_word_be(arena, len_rounded, off, len, pos + 4);
      if (blk == nblocks - 1 && j == 15) {
        hi = (uint32_t)((len * 8) >> 32);
        lo = (uint32_t)(len * 8);
      } else if (blk == nblocks - 1 && j == 14) {
        hi = 0;
        lo = 0;
      }
      w[j] = ((uint64_t)hi << 32) | lo;
    }
    sha512_compress(s, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) s_out[k] = s[k];
}

// ----------------------------------------------------------------- SHA-256
CG_HD uint32_t cg_rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ const uint32_t CG_K256[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#else
static const uint32_t CG_K256[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#endif
CG_HD uint32_t cg_k256(int i) { return CG_K256[i]; }

CG_HD void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667;
  s[1] = 0xbb67ae85;
  s[2] = 0x3c6ef372;
  s[3] = 0xa54ff53a;
  s[4] = 0x510e527f;
  s[5] = 0x9b05688c;
  s[6] = 0x1f83d9ab;
  s[7] = 0x5be0cd19;
}

#define CG_SHA256_ROUND(a, b, c, d, e, f, g, h, k, wi)                                                    \
  {                                                                                                    \
    const uint32_t t1 =                                                                                \
        h + cg_xor3_32(cg_rotr32(e, 6), cg_rotr32(e, 11), cg_rotr32(e, 25)) + ((e & f) ^ (~e & g)) + (k) + (wi); \
    const uint32_t t2 = cg_xor3_32(cg_rotr32(a, 2), cg_rotr32(a, 13), cg_rotr32(a, 22)) + cg_maj32(a, b, c); \
    d += t1;                                                                                           \
    h = t1 + t2;                                                                                       \
  }
#define CG_SHA256_8ROUNDS(i0, W)                                   \
  CG_SHA256_ROUND(a, b, c, d, e, f, g, h, cg_k256((i0) + 0), W(0)) \
  CG_SHA256_ROUND(h, a, b, c, d, e, f, g, cg_k256((i0) + 1), W(1)) \
  CG_SHA256_ROUND(g, h, a, b, c, d, e, f, cg_k256((i0) + 2), W(2)) \
  CG_SHA256_ROUND(f, g, h, a, b, c, d, e, cg_k256((i0) + 3), W(3)) \
  CG_SHA256_ROUND(e, f, g, h, a, b, c, d, cg_k256((i0) + 4), W(4)) \
  CG_SHA256_ROUND(d, e, f, g, h, a, b, c, cg_k256((i0) + 5), W(5)) \
  CG_SHA256_ROUND(c, d, e, f, g, h, a, b, cg_k256((i0) + 6), W(6)) \
  CG_SHA256_ROUND(b, c, d, e, f, g, h, a, cg_k256((i0) + 7), W(7))

CG_HD uint32_t sha256_sched(uint32_t w[16], int j) {
  const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
  const uint32_t s0 = cg_xor3_32(cg_rotr32(w15, 7), cg_rotr32(w15, 18), w15 >> 3);
  const uint32_t s1 = cg_xor3_32(cg_rotr32(w2, 17), cg_rotr32(w2, 19), w2 >> 10);
  w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
  return w[j];
}

// Same structure as sha512_compress: rounds 0..15 straight, 16..63 as a rolled loop of 16.
CG_HD void sha256_compress(uint32_t s[8], uint32_t w[16]) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#define CG_W0(j) w[(j)]
#define CG_W1(j) w[8 + (j)]
  CG_SHA256_8ROUNDS(0, CG_W0)
  CG_SHA256_8ROUNDS(8, CG_W1)
#undef CG_W0
#undef CG_W1
#pragma unroll 1
  for (int r = 16; r < 64; r += 16) {
#define CG_S0(j) sha256_sched(w, (j))
#define CG_S1(j) sha256_sched(w, 8 + (j))
    CG_SHA256_8ROUNDS(r, CG_S0)
    CG_SHA256_8ROUNDS(r + 8, CG_S1)
#undef CG_S0
#undef CG_S1
  }
  s[0] += a;
  s[1] += b;
  s[2] += c;
  s[3] += d;
  s[4] += e;
  s[5] += f;
  s[6] += g;
  s[7] += h;
}

// SHA-256 of arena[off, off+len) || suffix (0 or 32 bytes given as 8 big-endian words;
// used for serialised-component || nonce, MerkleTransaction.kt:23). Output: the state as
// 8 big-endian words (the digest).
// mid (optional): the state after the message's first `mid_blocks` 64-byte blocks (a SignableData
// template's constant prefix, cg_verify_tx_signatures); hashing resumes at that block.
template <class Ld>
CG_HD void sha256_ld_suffix(uint32_t out[8], const Ld& ld, uint64_t off, uint64_t len,
                            const uint32_t* suffix_be /* 8 words or null */, const uint32_t* mid = nullptr,
                            uint32_t mid_blocks = 0) {
  uint32_t s[8];
  if (mid) {
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = mid[k];
  } else {
    sha256_init(s);
    mid_blocks = 0;
  }
  const uint64_t sfx = suffix_be ? 32 : 0;
  const uint64_t n = len + sfx;
  const uint64_t nblocks = (n + 9 + 63) >> 6;
  // blocks made of message bytes only: straight loads, no per-word position logic
  const uint64_t nfull = len >> 6;
  const uint64_t base = off & ~(uint64_t)3;
  const uint32_t sh8 = (uint32_t)(off & 3) * 8u;
  for (uint64_t blk = mid_blocks; blk < nfull; ++blk) {
    uint32_t W[20], w[16];  // aligned dwords of the block (+1 for the realignment), 16-byte loads
#pragma unroll
    for (int t = 0; t < 5; ++t) ld.dwords4(&W[4 * t], base + blk * 64 + 16 * t);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
      w[j] = CG_BSWAP32(__builtin_amdgcn_alignbit(W[j + 1], W[j], sh8));
#else
      w[j] = CG_BSWAP32((uint32_t)((((uint64_t)W[j + 1] << 32) | W[j]) >> sh8));
#endif
    }
    sha256_compress(s, w);
  }
  for (uint64_t blk = nfull > mid_blocks ? nfull : mid_blocks; blk < nblocks; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t pos = blk * 64 + (uint64_t)j * 4;
      uint32_t v;
      if (pos + 4 <= len) {
        v = CG_BSWAP32(ld.bytes4(off + pos));
      } else if (sfx && (len & 3) == 0 && pos >= len && pos + 4 <= n) {
        v = suffix_be[(pos - len) >> 2];
      } else if (pos > n) {
        v = 0;
      } else {
        uint32_t acc = 0;
        for (int bb = 0; bb < 4; ++bb) {
          const uint64_t p = pos + (uint64_t)bb;
          uint32_t byte;
          if (p < len) {
            byte = ld.bytes4(off + p) & 0xffu;
          } else if (p < n) {
            const uint64_t q = p - len;
            byte = (suffix_be[q >> 2] >> (24 - 8 * (q & 3))) & 0xffu;
          } else {
            byte = (p == n) ? 0x80u : 0u;
          }
          acc = (acc << 8) | byte;
        }
        v = acc;
      }
      w[j] = v;
    }
    if (blk == nblocks - 1) {
      w[14] = (uint32_t)((n * 8) >> 32);
      w[15] = (uint32_t)(n * 8);
    }
    sha256_compress(s, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = s[k];
}

CG_HD void sha256_arena_suffix(uint32_t out[8], const uint8_t* arena, uint64_t len_rounded, uint64_t off,
                               uint64_t len, const uint32_t* suffix_be /* 8 words or null */,
                               const uint32_t* mid = nullptr, uint32_t mid_blocks = 0) {
  sha256_ld_suffix(out, ArenaLd{arena, len_rounded}, off, len, suffix_be, mid, mid_blocks);
}
