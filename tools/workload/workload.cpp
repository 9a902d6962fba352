// Synthetic workload generator for bench.py and the GPU parity tests (not product code,
// not the oracle). Produces seeded Ed25519 key pairs, RFC 8032 signatures over
// SignableData-sized messages and the corruption classes of SURVEY.md Appendix A, laid out
// in the cg_key / cg_item / arena format of include/cordagpu.h.
//
// Signing reuses the host build of the lane arithmetic (corda_amd/csrc/*.h); every
// signature it makes is independently checked by the C oracle in the parity tests, so a
// fault here cannot hide a fault in the kernels.
#include <stdint.h>
#include <string.h>

#include <thread>
#include <vector>

#include "../../corda_amd/csrc/ed25519.h"
#include "../../include/cordagpu.h"

namespace {

Ed25519Consts g_C;
bool g_init = false;
void comb_init();
void init() {
  if (!g_init) {
    ed_consts_init(g_C);
    comb_init();
    g_init = true;
  }
}

inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

void sha512_bytes(uint8_t out[64], const uint8_t* a, size_t na, const uint8_t* b, size_t nb, const uint8_t* c,
                  size_t nc) {
  std::vector<uint8_t> buf(na + nb + nc + 8, 0);
  if (na) memcpy(buf.data(), a, na);
  if (nb) memcpy(buf.data() + na, b, nb);
  if (nc) memcpy(buf.data() + na + nb, c, nc);
  uint64_t s[8];
  const uint64_t n = na + nb + nc;
  sha512_arena(s, buf.data(), (n + 3) & ~3ull, 0, n);
  for (int k = 0; k < 8; ++k)
    for (int j = 0; j < 8; ++j) out[8 * k + j] = (uint8_t)(s[k] >> (56 - 8 * j));
}

// [k]B for k < L (8 words): comb over 64 radix-16 digits with a 64 x 8 table of
// d * 16^i * B (built once), 64 mixed additions and no doublings.
ge_niels g_comb[64][9];
void comb_init() {
  ge_p3 P;  // 16^i * B
  uint32_t yw[8];
  (void)yw;
  ge_p3_0(P);
  // start from B: decode via consts table entry 1 is affine niels; rebuild B as p3
  {
    fe x, y, two_inv, t;
    fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);  // 2x
    fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);  // 2y
    fe_0(t);
    t.v[0] = 2;
    fe_invert(two_inv, t);
    fe_mul(P.X, x, two_inv);
    fe_mul(P.Y, y, two_inv);
    fe_1(P.Z);
    fe_mul(P.T, P.X, P.Y);
  }
  for (int i = 0; i < 64; ++i) {
    ge_niels_identity(g_comb[i][0]);
    ge_cached c;
    ge_p3_to_cached(c, P, g_C.d2);
    ge_p3 Q = P;
    ge_p1p1 t;
    for (int d = 1; d <= 8; ++d) {
      if (d > 1) {
        ge_add_cached(t, Q, c);
        ge_p1p1_to_p3(Q, t);
      }
      fe zi, x, y, xy;
      fe_invert(zi, Q.Z);
      fe_mul(x, Q.X, zi);
      fe_mul(y, Q.Y, zi);
      fe_add(g_comb[i][d].ypx, y, x);
      fe_carry(g_comb[i][d].ypx);
      fe_sub(g_comb[i][d].ymx, y, x);
      fe_carry(g_comb[i][d].ymx);
      fe_mul(xy, x, y);
      fe_mul(g_comb[i][d].xy2d, xy, g_C.d2);
    }
    // P = 16 P
    ge_p2 q;
    ge_p3_to_p2(q, P);
    for (int k = 0; k < 3; ++k) {
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
    }
    ge_p2_dbl(t, q);
    ge_p1p1_to_p3(P, t);
  }
}

void scalarmult_base(uint32_t enc[8], const uint32_t k[8]) {
  uint32_t e[16];
  sc_recode16(e, k);
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  for (int i = 0; i < 64; ++i) {
    const int db = sc_digit(e, i);
    ge_niels nb = g_comb[i][db < 0 ? -db : db];
    ge_niels_cneg(nb, db < 0);
    ge_madd(t, R, nb);
    ge_p1p1_to_p3(R, t);
  }
  ed_encode_affine(enc, R.X, R.Y, R.Z);
}

void expand(const uint8_t seed[32], uint32_t a[8], uint8_t prefix[32], uint8_t pub[32]) {
  uint8_t h[64];
  sha512_bytes(h, seed, 32, nullptr, 0, nullptr, 0);
  h[0] &= 248;
  h[31] &= 63;
  h[31] |= 64;
  uint32_t aw[16];
  memcpy(aw, h, 32);
  memset(aw + 8, 0, 32);
  sc_reduce512(a, aw);  // a < 2^255; reduce mod L (same group element)
  memcpy(prefix, h + 32, 32);
  uint32_t enc[8];
  scalarmult_base(enc, a);
  memcpy(pub, enc, 32);
}

void expand_scalar(const uint8_t seed[32], uint32_t a[8], uint8_t prefix[32]) {
  uint8_t h[64];
  sha512_bytes(h, seed, 32, nullptr, 0, nullptr, 0);
  h[0] &= 248;
  h[31] &= 63;
  h[31] |= 64;
  uint32_t aw[16];
  memcpy(aw, h, 32);
  memset(aw + 8, 0, 32);
  sc_reduce512(a, aw);
  memcpy(prefix, h + 32, 32);
}

void sign(uint8_t sig[64], const uint8_t seed[32], const uint8_t pub[32], const uint8_t* msg, size_t len) {
  uint32_t a[8];
  uint8_t prefix[32];
  expand_scalar(seed, a, prefix);
  const uint8_t* pubc = pub;
  uint8_t rh[64];
  sha512_bytes(rh, prefix, 32, msg, len, nullptr, 0);
  uint32_t r[8], rw[16];
  memcpy(rw, rh, 64);
  sc_reduce512(r, rw);
  uint32_t R[8];
  scalarmult_base(R, r);
  uint8_t kh[64];
  sha512_bytes(kh, (const uint8_t*)R, 32, pubc, 32, msg + 0, len);
  uint32_t k[8], kw[16];
  memcpy(kw, kh, 64);
  sc_reduce512(k, kw);
  // S = r + k a mod L  (schoolbook 8x8 words then Barrett)
  uint32_t prod[16];
  memset(prod, 0, sizeof prod);
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 8; ++j) {
      c += (uint64_t)k[i] * a[j] + prod[i + j];
      prod[i + j] = (uint32_t)c;
      c >>= 32;
    }
    prod[i + 8] = (uint32_t)c;
  }
  uint64_t c = 0;
  for (int i = 0; i < 16; ++i) {
    c += (uint64_t)prod[i] + (i < 8 ? r[i] : 0);
    prod[i] = (uint32_t)c;
    c >>= 32;
  }
  uint32_t S[8];
  sc_reduce512(S, prod);
  memcpy(sig, R, 32);
  memcpy(sig + 32, S, 32);
}

void add_L(uint8_t s[32], int k) {
  uint64_t c = 0;
  for (int w = 0; w < 8; ++w) {
    uint32_t v;
    memcpy(&v, s + 4 * w, 4);
    c += (uint64_t)v + (uint64_t)sc_Lw(w) * (uint64_t)k;
    v = (uint32_t)c;
    memcpy(s + 4 * w, &v, 4);
    c >>= 32;
  }
}

}  // namespace

extern "C" {

// n_keys seeds -> public keys (32 B each). Key i's seed is derived from (seed, i).
// `bad_every` > 0 replaces every bad_every-th key with an undecodable 32-byte string
// (class A8). Returns the number of undecodable keys.
int wl_ed25519_keys(uint32_t n_keys, uint64_t seed, uint32_t bad_every, uint8_t* seeds_out, uint8_t* pubs_out,
                    int nthreads) {
  init();
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=]() {
      for (uint32_t i = (uint32_t)t; i < n_keys; i += (uint32_t)nthreads) {
        uint64_t s = seed * 0x100000001b3ULL + i;
        uint8_t* sd = seeds_out + 32 * (size_t)i;
        for (int w = 0; w < 4; ++w) {
          uint64_t v = splitmix(s);
          memcpy(sd + 8 * w, &v, 8);
        }
        uint32_t a[8];
        uint8_t prefix[32];
        expand(sd, a, prefix, pubs_out + 32 * (size_t)i);
        if (bad_every && (i % bad_every) == bad_every - 1) {
          // undecodable: search y values with no square root
          for (uint64_t tries = 0;; ++tries) {
            uint32_t yw[8];
            for (int w = 0; w < 8; ++w) yw[w] = (uint32_t)splitmix(s);
            ge_p3 P;
            if (ed_decode_point(P, yw, g_C) != ED_ST_VALID) {
              memcpy(pubs_out + 32 * (size_t)i, yw, 32);
              break;
            }
          }
        }
      }
    });
  }
  for (auto& x : th) x.join();
  int bad = 0;
  if (bad_every)
    for (uint32_t i = 0; i < n_keys; ++i) bad += (i % bad_every) == bad_every - 1;
  return bad;
}

// Fill n_items Ed25519 items. Layout written into `arena` (caller-sized):
//   [keys: 32 * n_keys][item 0: sig 64 | msg msg_len | pad to 4] ...
// keys_out (cg_key[n_keys]) and items_out (cg_item[n_items]) describe it. labels_out[i]
// is the corruption class (0 = valid, 1..9 = A1..A9 as in SURVEY Appendix A; 4 = S+L).
// corrupt_permille of items are corrupted, spread evenly over classes A1-A7.
void wl_ed25519_items(uint64_t n_items, uint32_t n_keys, const uint8_t* seeds, const uint8_t* pubs, uint32_t msg_len,
                      uint32_t corrupt_permille, uint64_t seed, uint8_t* arena, cg_key* keys_out, cg_item* items_out,
                      uint8_t* labels_out, int nthreads) {
  init();
  for (uint32_t i = 0; i < n_keys; ++i) {
    memcpy(arena + 32 * (size_t)i, pubs + 32 * (size_t)i, 32);
    keys_out[i].off = 32ull * i;
    keys_out[i].len = 32;
    keys_out[i].scheme = CG_EDDSA_ED25519_SHA512;
    keys_out[i].fmt = CG_KEY_RAW;
    keys_out[i].reserved = 0;
  }
  const uint64_t base = 32ull * n_keys;
  const uint64_t stride = (64 + msg_len + 3 + 4) & ~3ull;  // room for a 65-byte signature variant
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=]() {
      for (uint64_t i = (uint64_t)t; i < n_items; i += (uint64_t)nthreads) {
        uint64_t s = seed ^ (i * 0x9e3779b97f4a7c15ULL);
        const uint32_t k = (uint32_t)(splitmix(s) % n_keys);
        uint8_t* p = arena + base + stride * i;
        uint8_t* sig = p;
        uint8_t* msg = p + 64;
        for (uint32_t b = 0; b < msg_len; b += 8) {
          uint64_t v = splitmix(s);
          memcpy(msg + b, &v, (msg_len - b) < 8 ? (msg_len - b) : 8);
        }
        sign(sig, seeds + 32 * (size_t)k, pubs + 32 * (size_t)k, msg, msg_len);
        uint8_t label = 0;
        uint16_t sig_len = 64;
        const uint32_t r = (uint32_t)(splitmix(s) % 1000);
        if (r < corrupt_permille) {
          const uint32_t cls = 1 + (uint32_t)(splitmix(s) % 7);  // A1..A7
          label = (uint8_t)cls;
          const uint64_t rb = splitmix(s);
          switch (cls) {
            case 1: msg[(rb >> 8) % msg_len] ^= (uint8_t)(1u << (rb & 7)); break;    // A1 message bit
            case 2: sig[(rb >> 8) % 31] ^= (uint8_t)(1u << (rb & 7)); break;         // A2 R bit (not sign)
            case 3: sig[32 + (rb >> 8) % 31] ^= (uint8_t)(1u << (rb & 7)); break;    // A3 S bit (< 2^248)
            case 4: add_L(sig + 32, 1); break;                                       // A4 S + L (valid)
            case 5: add_L(sig + 32, 2 + (int)(rb % 13)); sig[63] |= 0x80; break;     // A5 high S
            case 6: sig[31] ^= 0x80; break;                                          // A6 R sign bit
            case 7: sig_len = (rb & 1) ? 63 : 65; break;                             // A7 length
          }
        }
        items_out[i].sig_off = base + stride * i;
        items_out[i].msg_off = base + stride * i + 64;
        items_out[i].msg_len = msg_len;
        items_out[i].key_idx = k;
        items_out[i].sig_len = sig_len;
        items_out[i].reserved0 = 0;
        items_out[i].reserved1 = 0;
        labels_out[i] = label;
        if (sig_len == 65) {
          // a 65-byte signature overlaps the message start; keep the message intact by
          // pointing the message one byte later in a copy is unnecessary: length 65 fails
          // the length check before any byte is read.
        }
      }
    });
  }
  for (auto& x : th) x.join();
}

uint64_t wl_ed25519_arena_bytes(uint64_t n_items, uint32_t n_keys, uint32_t msg_len) {
  return 32ull * n_keys + ((64 + msg_len + 3 + 4) & ~3ull) * n_items + 64;
}
}
