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

// Signable mode (wl_set_signable): item i's clear data is SignableData(id, metadata) =
// pre || id(i / group) || suf instead of random bytes, so the same items can be handed to
// cg_verify_tx_signatures as (id, template) pairs. A message-corruption item (A1 / E1) then signs
// a flipped copy and keeps the true SignableData bytes (same verdict: INVALID).
struct Signable {
  bool on = false;
  std::vector<uint8_t> pre, suf;
  uint32_t group = 1;
  uint64_t seed = 0;
};
Signable g_signable;
// wl_set_key_choice: item i of the next generator call signs with key g_key_choice[i] (key-
// distribution workloads: every item its own key, Zipf draws) instead of a uniform draw.
std::vector<uint32_t> g_key_choice;

void signable_msg(uint8_t* msg, uint64_t i) {
  const Signable& S = g_signable;
  memcpy(msg, S.pre.data(), S.pre.size());
  uint64_t s = S.seed ^ ((i / S.group) * 0xa0761d6478bd642fULL);
  for (int w = 0; w < 4; ++w) {
    const uint64_t v = splitmix(s);
    memcpy(msg + S.pre.size() + 8 * w, &v, 8);
  }
  memcpy(msg + S.pre.size() + 32, S.suf.data(), S.suf.size());
}

}  // namespace

extern "C" {

// pre == NULL: back to random messages. Otherwise the item generators write pre || id || suf
// (msg_len must be pre_len + 32 + suf_len), `group` consecutive items sharing one id.
void wl_set_signable(const uint8_t* pre, uint32_t pre_len, const uint8_t* suf, uint32_t suf_len, uint32_t group,
                     uint64_t id_seed) {
  g_signable.on = pre != nullptr;
  g_signable.pre.assign(pre, pre ? pre + pre_len : pre);
  g_signable.suf.assign(suf, suf ? suf + suf_len : suf);
  g_signable.group = group ? group : 1;
  g_signable.seed = id_seed;
}

// k == NULL: uniform key draws again. Otherwise item i uses key k[i] (k[i] < n_keys of the call).
void wl_set_key_choice(const uint32_t* k, uint64_t n) { g_key_choice.assign(k, k ? k + n : k); }

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
        uint32_t k = (uint32_t)(splitmix(s) % n_keys);
        if (i < g_key_choice.size()) k = g_key_choice[i] % n_keys;
        uint8_t* p = arena + base + stride * i;
        uint8_t* sig = p;
        uint8_t* msg = p + 64;
        if (g_signable.on) {
          signable_msg(msg, i);
        } else {
          for (uint32_t b = 0; b < msg_len; b += 8) {
            uint64_t v = splitmix(s);
            memcpy(msg + b, &v, (msg_len - b) < 8 ? (msg_len - b) : 8);
          }
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
            case 1:                                                                  // A1 message bit
              msg[(rb >> 8) % msg_len] ^= (uint8_t)(1u << (rb & 7));
              if (g_signable.on) {  // sign the flipped copy, keep the true SignableData
                sign(sig, seeds + 32 * (size_t)k, pubs + 32 * (size_t)k, msg, msg_len);
                msg[(rb >> 8) % msg_len] ^= (uint8_t)(1u << (rb & 7));
              }
              break;
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

// ---------------------------------------------------------------- ECDSA (secp256r1 / k1)
#include "../../corda_amd/csrc/ecdsa.h"

#include "../../corda_amd/csrc/ecdsa_rows.h"

namespace {
EcConsts g_K[2];
EcRowTab g_GT[2];  // G rows built with the verify path's row construction (ec_row_bases / ec_row_build)
bool g_ec_init = false;

template <int C>
void ec_g_rows_init(EcRowTab& T, EcRowScratch& s, const EcConsts& K) {
  Jac bases[EC_ROWS];
  ec_row_bases<C>(bases, K.gx, K.gy, K);
  for (int j = 0; j < EC_ROWS; ++j) ec_row_build<C>(T.t[j], bases[j], s, K);
}

void ec_init() {
  if (!g_ec_init) {
    static EcRowScratch scr;
    ec_consts_init<CG_CURVE_K1>(g_K[0]);
    ec_consts_init<CG_CURVE_R1>(g_K[1]);
    ec_g_rows_init<CG_CURVE_K1>(g_GT[0], scr, g_K[0]);
    ec_g_rows_init<CG_CURVE_R1>(g_GT[1], scr, g_K[1]);
    g_ec_init = true;
  }
}

// affine plain (x, y) of k*G (0 < k < n) over the G rows
template <int C>
void ec_mul_base(u256w& x, u256w& y, const u256w& k) {
  const EcConsts& K = g_K[C];
  uint32_t d[EC_PACKED];
  ec_recode_w6(d, k);
  Jac R;
  jac_set_inf<C>(R, K);
  for (int i = EC_WINDOWS - 1; i >= 0; --i) {
    if (i != EC_WINDOWS - 1)
      for (int t = 0; t < EC_W; ++t) jac_dbl<C>(R, R);
    for (int j = 0; j < EC_ROWS; ++j) {
      const int t = EC_WINDOWS * j + i;
      if (t >= EC_DIGITS) continue;
      const int a = ec_digit6(d, t);
      if (!a) continue;
      f29 xx = g_GT[C].t[j][(a < 0 ? -a : a) - 1].x, yy = g_GT[C].t[j][(a < 0 ? -a : a) - 1].y;
      if (a < 0) m29_neg<C, 0>(yy, yy);
      jac_madd<C>(R, R, xx, yy, K);
    }
  }
  f29 xm, ym;
  jac_to_affine<C>(xm, ym, R, K);
  m29_to_plain<C, 0>(x, xm);
  m29_to_plain<C, 0>(y, ym);
}

void put_be32(uint8_t* out, const u256w& v) {
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = v.w[7 - i];
    out[4 * i] = (uint8_t)(w >> 24);
    out[4 * i + 1] = (uint8_t)(w >> 16);
    out[4 * i + 2] = (uint8_t)(w >> 8);
    out[4 * i + 3] = (uint8_t)w;
  }
}

// DER INTEGER of a non-negative 256-bit value (minimal), returns bytes written
int der_int_enc(uint8_t* out, const u256w& v, bool extra_pad) {
  uint8_t be[32];
  put_be32(be, v);
  int s = 0;
  while (s < 31 && be[s] == 0) ++s;
  const bool pad = (be[s] & 0x80) != 0 || extra_pad;
  const int len = 32 - s + (pad ? 1 : 0);
  out[0] = 0x02;
  out[1] = (uint8_t)len;
  int o = 2;
  if (pad) out[o++] = 0;
  memcpy(out + o, be + s, 32 - s);
  return 2 + len;
}

template <int C>
void rand_scalar(u256w& k, uint64_t& s) {
  for (;;) {
    for (int i = 0; i < 8; ++i) k.w[i] = (uint32_t)splitmix(s);
    if (!u256_iszero(k) && u256_lt_mod<C, 1>(k)) return;
  }
}

// sign: returns DER length; r_out/s_out plain
template <int C>
int ec_sign(uint8_t* der, const u256w& d, const uint8_t* msg, size_t len, uint64_t& rng, int cls, u256w& r,
            u256w& s) {
  const EcConsts& K = g_K[C];
  uint32_t h[8];
  sha256_arena_suffix(h, msg, (len + 3) & ~3ull, 0, len, nullptr);
  u256w e;
  for (int i = 0; i < 8; ++i) e.w[i] = h[7 - i];
  if (!u256_lt_mod<C, 1>(e)) {
    uint32_t br = 0;
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = (uint64_t)e.w[i] - Mod<C, 1>::w(i) - br;
      e.w[i] = (uint32_t)x;
      br = (uint32_t)(x >> 63);
    }
  }
  for (;;) {
    u256w k, x, y;
    rand_scalar<C>(k, rng);
    ec_mul_base<C>(x, y, k);
    r = x;
    if (!u256_lt_mod<C, 1>(r)) {
      uint32_t br = 0;
      for (int i = 0; i < 8; ++i) {
        const uint64_t t = (uint64_t)r.w[i] - Mod<C, 1>::w(i) - br;
        r.w[i] = (uint32_t)t;
        br = (uint32_t)(t >> 63);
      }
    }
    if (u256_iszero(r)) continue;
    // s = k^-1 (e + r d) mod n  (Montgomery mod n, mont29.h)
    f29 km, kinv, rf, df, rd, ef, t, sm;
    m29_from_plain<C, 1>(km, k, K.r2_n);  // k R
    m29_inv<C, 1>(kinv, km, K.one_n);     // k^-1 R
    f29_from_words(rf, r.w);
    f29_from_words(df, d.w);
    m29_mul<C, 1>(rd, rf, df);            // r d R^-1
    m29_mul<C, 1>(rd, rd, K.r2_n);        // r d
    f29_from_words(ef, e.w);
    m29_add<C, 1>(t, ef, rd);             // e + r d
    m29_mul<C, 1>(sm, t, kinv);           // (e + r d) k^-1 (plain)
    m29_to_words_canon<C, 1>(s.w, sm);
    if (u256_iszero(s)) continue;
    break;
  }
  if (cls == 2) {  // E2 high-S: s' = n - s (still valid)
    uint32_t br = 0;
    for (int i = 0; i < 8; ++i) {
      const uint64_t t = (uint64_t)Mod<C, 1>::w(i) - s.w[i] - br;
      s.w[i] = (uint32_t)t;
      br = (uint32_t)(t >> 63);
    }
  }
  uint8_t body[96];
  int o = 0;
  u256w rr = r, ss = s;
  if (cls == 3) u256_zero(rr);  // E3 r = 0
  o += der_int_enc(body + o, rr, cls == 5);  // E5 non-minimal INTEGER (extra 00)
  o += der_int_enc(body + o, ss, false);
  if (cls == 7) {  // E7 three elements: append INTEGER 1
    body[o++] = 0x02;
    body[o++] = 0x01;
    body[o++] = 0x01;
  }
  der[0] = 0x30;
  der[1] = (uint8_t)o;
  memcpy(der + 2, body, o);
  int n = 2 + o;
  if (cls == 6) der[n++] = 0;  // E6 trailing byte
  return n;
}
}  // namespace

extern "C" {
// curve: 0 = secp256k1 (scheme 2), 1 = secp256r1 (scheme 3). d_out 32 B (LE words), pub_out 64 B X||Y BE.
void wl_ecdsa_keys(int curve, uint32_t n_keys, uint64_t seed, uint8_t* d_out, uint8_t* pub_out, int nthreads) {
  init();
  ec_init();
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=]() {
      for (uint32_t i = (uint32_t)t; i < n_keys; i += (uint32_t)nthreads) {
        uint64_t s = seed * 0x9e3779b97f4a7c15ULL + i + 1;
        u256w d, x, y;
        if (curve == 1) {
          rand_scalar<CG_CURVE_R1>(d, s);
          ec_mul_base<CG_CURVE_R1>(x, y, d);
        } else {
          rand_scalar<CG_CURVE_K1>(d, s);
          ec_mul_base<CG_CURVE_K1>(x, y, d);
        }
        memcpy(d_out + 32 * (size_t)i, d.w, 32);
        put_be32(pub_out + 64 * (size_t)i, x);
        put_be32(pub_out + 64 * (size_t)i + 32, y);
      }
    });
  }
  for (auto& x : th) x.join();
}

uint64_t wl_ecdsa_arena_bytes(uint64_t n_items, uint32_t n_keys, uint32_t msg_len) {
  return 64ull * n_keys + ((80 + msg_len + 3) & ~3ull) * n_items + 64;
}

// labels: 0 valid, 1 E1 msg flip, 2 E2 high-S (valid), 3 E3 r = 0, 5 E5 non-minimal,
// 6 E6 trailing byte, 7 E7 three elements
void wl_ecdsa_items(int curve, uint64_t n_items, uint32_t n_keys, const uint8_t* ds, const uint8_t* pubs,
                    uint32_t msg_len, uint32_t corrupt_permille, uint64_t seed, uint8_t* arena, cg_key* keys_out,
                    cg_item* items_out, uint8_t* labels_out, int nthreads) {
  init();
  ec_init();
  const uint8_t scheme = curve == 1 ? CG_ECDSA_SECP256R1_SHA256 : CG_ECDSA_SECP256K1_SHA256;
  for (uint32_t i = 0; i < n_keys; ++i) {
    memcpy(arena + 64 * (size_t)i, pubs + 64 * (size_t)i, 64);
    keys_out[i].off = 64ull * i;
    keys_out[i].len = 64;
    keys_out[i].scheme = scheme;
    keys_out[i].fmt = CG_KEY_RAW;
    keys_out[i].reserved = 0;
  }
  const uint64_t base = 64ull * n_keys;
  const uint64_t stride = (80 + msg_len + 3) & ~3ull;
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([=]() {
      for (uint64_t i = (uint64_t)t; i < n_items; i += (uint64_t)nthreads) {
        uint64_t s = seed ^ (i * 0xd6e8feb86659fd93ULL);
        uint32_t k = (uint32_t)(splitmix(s) % n_keys);
        if (i < g_key_choice.size()) k = g_key_choice[i] % n_keys;
        uint8_t* p = arena + base + stride * i;
        uint8_t* msg = p + 80;
        if (g_signable.on) {
          signable_msg(msg, i);
        } else {
          for (uint32_t b = 0; b < msg_len; b += 8) {
            uint64_t v = splitmix(s);
            memcpy(msg + b, &v, (msg_len - b) < 8 ? (msg_len - b) : 8);
          }
        }
        int cls = 0;
        if (splitmix(s) % 1000 < corrupt_permille) {
          const int choices[6] = {1, 2, 3, 5, 6, 7};
          cls = choices[splitmix(s) % 6];
        }
        u256w d, r, sv;
        memcpy(d.w, ds + 32 * (size_t)k, 32);
        int n;
        // E1: the signature is over a message differing in one bit from the stored one (signable
        // mode flips before signing and restores the true SignableData; else flips after)
        uint64_t flip_at = 0;
        uint8_t flip_bit = 0;
        if (cls == 1) {
          flip_at = splitmix(s) % msg_len;
          flip_bit = (uint8_t)(1u << (splitmix(s) & 7));
          if (g_signable.on) msg[flip_at] ^= flip_bit;
        }
        if (curve == 1) n = ec_sign<CG_CURVE_R1>(p, d, msg, msg_len, s, cls, r, sv);
        else n = ec_sign<CG_CURVE_K1>(p, d, msg, msg_len, s, cls, r, sv);
        if (cls == 1) msg[flip_at] ^= flip_bit;
        items_out[i].sig_off = base + stride * i;
        items_out[i].msg_off = base + stride * i + 80;
        items_out[i].msg_len = msg_len;
        items_out[i].key_idx = k;
        items_out[i].sig_len = (uint16_t)n;
        items_out[i].reserved0 = 0;
        items_out[i].reserved1 = 0;
        labels_out[i] = (uint8_t)cls;
      }
    });
  }
  for (auto& x : th) x.join();
}
}

extern "C" {
// dst[dst_off[i] ..) = src[src_off[i] .. + len[i]) for every i (packing a message-form batch's
// signature / key bytes into a compact arena, bench.py)
void wl_gather(const uint8_t* src, const uint64_t* src_off, const uint16_t* len, uint64_t n, uint8_t* dst,
               const uint64_t* dst_off, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([=]() {
      const uint64_t a = n * t / nthreads, b = n * (t + 1) / nthreads;
      for (uint64_t i = a; i < b; ++i) memcpy(dst + dst_off[i], src + src_off[i], len[i]);
    });
  for (auto& x : th) x.join();
}
}

// ---------------------------------------------------------------- transaction pipeline (config 4)
namespace {
void sha256_bytes_suffix(uint8_t out[32], const uint8_t* arena, uint64_t arena_len, uint64_t off, uint64_t len,
                         const uint32_t* suffix_be) {
  uint32_t h[8];
  sha256_arena_suffix(h, arena, (arena_len + 3) & ~3ull, off, len, suffix_be);
  for (int k = 0; k < 8; ++k)
    for (int j = 0; j < 4; ++j) out[4 * k + j] = (uint8_t)(h[k] >> (24 - 8 * j));
}

void sha256_64(uint8_t out[32], const uint8_t l[32], const uint8_t r[32]) {
  uint8_t buf[64 + 8];
  memcpy(buf, l, 32);
  memcpy(buf + 32, r, 32);
  sha256_bytes_suffix(out, buf, 64, 0, 64, nullptr);
}

// WireTransaction.id (MerkleTransaction.kt:16-33,74-93; MerkleTree.kt:27-66), host side
void tx_id(uint8_t id[32], const cg_tx& tx, const cg_component* comps, const uint8_t* arena, uint64_t arena_len) {
  std::vector<uint8_t> lv(32 * (size_t)tx.n);
  for (uint32_t i = 0; i < tx.n; ++i) {
    const cg_component& c = comps[tx.first + i];
    if (c.flags & 1u) {
      sha256_bytes_suffix(&lv[32 * i], arena, arena_len, c.off, c.len, nullptr);
    } else {
      uint8_t nb[40];
      memcpy(nb, arena + tx.salt_off, 32);
      nb[32] = (uint8_t)(i >> 24);
      nb[33] = (uint8_t)(i >> 16);
      nb[34] = (uint8_t)(i >> 8);
      nb[35] = (uint8_t)i;
      uint8_t nonce[32];
      sha256_bytes_suffix(nonce, nb, 36, 0, 36, nullptr);
      uint32_t nbe[8];
      for (int k = 0; k < 8; ++k)
        nbe[k] = ((uint32_t)nonce[4 * k] << 24) | ((uint32_t)nonce[4 * k + 1] << 16) |
                 ((uint32_t)nonce[4 * k + 2] << 8) | nonce[4 * k + 3];
      sha256_bytes_suffix(&lv[32 * i], arena, arena_len, c.off, c.len, nbe);
    }
  }
  uint32_t m = 1;
  while (m < tx.n) m <<= 1;
  lv.resize(32 * (size_t)m, 0);
  while (m > 1) {
    for (uint32_t j = 0; j < m / 2; ++j) sha256_64(&lv[32 * j], &lv[64 * j], &lv[64 * j + 32]);
    m /= 2;
  }
  memcpy(id, lv.data(), 32);
}
}  // namespace

extern "C" {
// Config 4 generator: given packed transactions (cg_tx / cg_component / arena,
// laid out by tools/workload/wl.py), computes every id on the host and writes, for every
// signature row, an Ed25519 signature over prefix || id || suffix (the SignableData template,
// corda_amd/signable.py) into arena[sig_off..+64). corrupt_permille of the signatures get one
// flipped bit of R (labels_out[j] = 1).
void wl_tx_sign(uint64_t n_tx, const cg_tx* txs, const cg_component* comps, uint8_t* arena, uint64_t arena_len,
                uint64_t n_sigs, const cg_txsig* sigs, const uint8_t* seeds, const uint8_t* pubs,
                const uint8_t* prefix, uint32_t pre_len, const uint8_t* suffix, uint32_t suf_len,
                uint32_t corrupt_permille, uint64_t seed, uint8_t* ids_out, uint8_t* labels_out, int nthreads) {
  init();
  if (nthreads <= 0) nthreads = 1;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([=]() {
        for (uint64_t i = (uint64_t)t; i < n_tx; i += (uint64_t)nthreads)
          tx_id(ids_out + 32 * i, txs[i], comps, arena, arena_len);
      });
    for (auto& x : th) x.join();
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([=]() {
      std::vector<uint8_t> msg(pre_len + 32 + suf_len);
      memcpy(msg.data(), prefix, pre_len);
      memcpy(msg.data() + pre_len + 32, suffix, suf_len);
      for (uint64_t j = (uint64_t)t; j < n_sigs; j += (uint64_t)nthreads) {
        const cg_txsig& sg = sigs[j];
        memcpy(msg.data() + pre_len, ids_out + 32 * (uint64_t)sg.tx_idx, 32);
        uint8_t* sig = arena + sg.sig_off;
        sign(sig, seeds + 32 * (size_t)sg.key_idx, pubs + 32 * (size_t)sg.key_idx, msg.data(), msg.size());
        uint64_t s = seed ^ (j * 0x9e3779b97f4a7c15ULL);
        uint8_t label = 0;
        if ((uint32_t)(splitmix(s) % 1000) < corrupt_permille) {
          const uint64_t rb = splitmix(s);
          sig[(rb >> 8) % 31] ^= (uint8_t)(1u << (rb & 7));
          label = 1;
        }
        labels_out[j] = label;
      }
    });
  for (auto& x : th) x.join();
}
}
