#include <type_traits>
#include <vector>
// Host build of the device lane code (corda_amd/csrc/*.h) with FE_BOUNDS_CHECK on, so the
// exact arithmetic the HIP kernels run is checked on the CPU against the oracle and every
// limb bound assumed by fe25519.h is asserted. Test infrastructure only.
#include <stdint.h>
#include <string.h>

#include "../../corda_amd/csrc/ed25519.h"
#include "../../corda_amd/csrc/fe9.h"
#ifdef FE_OP_COUNT
uint64_t g_fe_nmul = 0, g_fe_nsq = 0;
uint64_t g_fe9_nmul = 0;
uint64_t g_m29_nmul[2][2] = {{0, 0}, {0, 0}};
uint64_t g_m29_nsqr[2] = {0, 0};
#endif

static Ed25519Consts g_C;
static int g_init = 0;
static void init() {
  if (!g_init) {
    ed_consts_init(g_C);
    g_init = 1;
  }
}

extern "C" {
void t_fe_mul(const uint32_t* f, const uint32_t* g, uint32_t* out) {
  fe a, b, c;
  memcpy(a.v, f, 40);
  memcpy(b.v, g, 40);
  fe_mul(c, a, b);
  memcpy(out, c.v, 40);
}
void t_fe_sq(const uint32_t* f, uint32_t* out) {
  fe a, c;
  memcpy(a.v, f, 40);
  fe_sq(c, a);
  memcpy(out, c.v, 40);
}
// radix-2^29 products (fe9.h): sgn selects fe9_mul<true> (signed limbs)
void t_fe9_mul(int sgn, const uint32_t* f, const uint32_t* g, uint32_t* out) {
  fe9 a, b, c;
  memcpy(a.v, f, 36);
  memcpy(b.v, g, 36);
  if (sgn) fe9_mul<true>(c, a, b);
  else fe9_mul<false>(c, a, b);
  memcpy(out, c.v, 36);
}
void t_fe9_to_words(const uint32_t* f, uint32_t* out) {
  fe9 a;
  memcpy(a.v, f, 36);
  fe9_to_words255(out, a);
}
void t_fe9_from_fe(const uint32_t* f, uint32_t* out) {
  fe a;
  fe9 b;
  memcpy(a.v, f, 40);
  fe9_from_fe(b, a);
  memcpy(out, b.v, 36);
}
void t_fe_tobytes(const uint32_t* f, uint32_t* out) {
  fe a;
  memcpy(a.v, f, 40);
  fe_tobytes_words(out, a);
}
void t_fe_frombytes(const uint32_t* w, uint32_t* out) {
  fe a;
  fe_frombytes_words(a, w);
  memcpy(out, a.v, 40);
}
void t_fe_invert(const uint32_t* f, uint32_t* out) {
  fe a, c;
  memcpy(a.v, f, 40);
  fe_invert(c, a);
  memcpy(out, c.v, 40);
}
void t_sc_reduce512(const uint32_t* x, uint32_t* out) { sc_reduce512(out, x); }
uint32_t t_slide_escapes(const uint32_t* s) { return sc_slide_escapes(s); }
void t_recode16(const uint32_t* a, int32_t* digits) {
  uint32_t p[16];
  sc_recode16(p, a);
  for (int i = 0; i < 64; ++i) digits[i] = sc_digit(p, i);
}
int t_ed_keyprep(const uint32_t* aw, uint32_t* abyte_out) {
  init();
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  memcpy(abyte_out, kp.abyte, 32);
  return (int)kp.status;
}
void t_ed_abyte_fast(const uint32_t* aw, uint32_t* abyte_out) { ed_abyte_fast(abyte_out, aw); }
int t_ed_verify(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len) {
  init();
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  if (kp.status) return (int)kp.status;
  // message buffer must be 4-aligned with a rounded length
  static uint8_t buf[1 << 20];
  memcpy(buf, msg, msg_len);
  memset(buf + msg_len, 0xEE, 8);  // garbage past the end must not matter
  return ed_verify_core(kp, kp.tab, sw, buf, (msg_len + 3) & ~3ull, 0, msg_len, g_C, g_C.Btab);
}
void t_sha512_prefix(const uint32_t* pre, const uint8_t* msg, uint64_t off, uint64_t len, uint32_t* out) {
  sha512_prefix64_msg(out, pre, msg, (off + len + 3) & ~3ull, off, len);
}
void t_sha256_suffix(const uint8_t* arena, uint64_t off, uint64_t len, const uint32_t* sfx, uint32_t* out) {
  sha256_arena_suffix(out, arena, (off + len + 3) & ~3ull, off, len, sfx);
}
}

// ---------------------------------------------------------------- ECDSA
#include "../../corda_amd/csrc/ecdsa.h"
static EcConsts g_K[2];
static int g_kinit = 0;
static void kinit() {
  if (!g_kinit) {
    ec_consts_init<CG_CURVE_K1>(g_K[0]);
    ec_consts_init<CG_CURVE_R1>(g_K[1]);
    g_kinit = 1;
  }
}
// ---------------------------------------------------------------- Ed25519 v2 (row tables)
static EdRowTab g_TB;
static int g_rinit = 0;
extern "C" int t_ed_verify_v2(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len) {
  init();
  if (!g_rinit) {
    ge_p3 B;
    fe x, y, two_inv, t;
    fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_0(t);
    t.v[0] = 2;
    fe_invert(two_inv, t);
    fe_mul(B.X, x, two_inv);
    fe_mul(B.Y, y, two_inv);
    fe_1(B.Z);
    fe_mul(B.T, B.X, B.Y);
    ed_rows_init(g_TB, B, g_C.d2);
    g_rinit = 1;
  }
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  if (kp.status) return (int)kp.status;
  ge_p3 A, N;
  ed_decode_point(A, aw, g_C);
  ed_neg_point(N, A);
  static EdRowTab TA;
  ed_rows_init(TA, N, g_C.d2);
  static uint8_t buf[1 << 20];
  memcpy(buf, msg, msg_len);
  uint32_t eh[16], es[16];
  ed_scalars(eh, es, kp.abyte, sw, buf, (msg_len + 3) & ~3ull, 0, msg_len);
  ge_p2 R;
  ed_double_scalar_rows(R, eh, es, TA, g_TB);
  fe zi;
  fe_invert(zi, R.Z);
  return ed_encode_cmp(R, zi, sw);
}

// ---------------------------------------------------------------- Ed25519 rows, generic W/K
#include "../../corda_amd/csrc/ed25519_rows.h"
template <int W, int K>
static int verify_w(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len) {
  init();
  typedef EdRowTabW<W, K> Tab;
  static Tab* TB = nullptr;
  static Tab* TA = nullptr;
  if (!TB) {
    TB = new Tab;
    TA = new Tab;
    ge_p3 B;
    fe x, y, two_inv, t;
    fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_0(t);
    t.v[0] = 2;
    fe_invert(two_inv, t);
    fe_mul(B.X, x, two_inv);
    fe_mul(B.Y, y, two_inv);
    fe_1(B.Z);
    fe_mul(B.T, B.X, B.Y);
    ed_rows_w_init<W, K>(*TB, B, g_C.d2);
  }
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  if (kp.status) return (int)kp.status;
  ge_p3 A, N;
  ed_decode_point(A, aw, g_C);
  ed_neg_point(N, A);
  ed_rows_w_init<W, K>(*TA, N, g_C.d2);
  static uint8_t buf[1 << 20];
  memcpy(buf, msg, msg_len);
  // scalars
  uint32_t pre[16], hw[16], h[8];
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];
    pre[8 + i] = kp.abyte[i];
  }
  sha512_prefix64_msg(hw, pre, buf, (msg_len + 3) & ~3ull, 0, msg_len);
  sc_reduce512(h, hw);
  uint32_t s[8], sr[8];
  for (int i = 0; i < 8; ++i) s[i] = sw[8 + i];
  sc_reduce256(sr, s);
  if ((s[7] >> 31) && sc_slide_escapes(s)) {
    uint32_t r1[8];
    for (int i = 0; i < 8; ++i) r1[i] = sc_R1w(i);
    sc_sub(sr, sr, r1);
  }
  const int NW = EdRowsCfg<W, K>::kPackedWords;
  uint32_t eh[NW], es[NW];
  sc_recode_w<W>(eh, NW, h);
  sc_recode_w<W>(es, NW, sr);
  ge_p2 R;
  ed_double_scalar_w<W, K>(R, eh, es, *TA, *TB);
  fe zi;
  fe_invert(zi, R.Z);
  return ed_encode_cmp(R, zi, sw);
}
extern "C" int t_ed_verify_w(int w, const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len) {
  if (w == 4) return verify_w<4, 8>(aw, sw, msg, msg_len);
  if (w == 5) return verify_w<5, 4>(aw, sw, msg, msg_len);
  return verify_w<6, 4>(aw, sw, msg, msg_len);
}

// ---------------------------------------------------------------- executed-work counters
// Field multiplies / squarings the GPU path executes (same code, host build):
//   out[0..1] per item in k_ed_verify (double-scalar over the W=6, K=4 rows)
//   out[2..3] per item in k_ed_finish excluding the shared inversion (prefix product,
//             unwinding, encode)
//   out[4..5] one fe_invert (shared by ED_FINISH_K items)
//   out[6..7] per key: k_ed_keyprep_rows + k_ed_keyprep_tab (decode, Abyte, 11 bases, 352
//             affine multiples)
extern "C" int t_ed_count_w6(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len,
                             uint64_t* out) {
#ifdef FE_OP_COUNT
  init();
  (void)verify_w<6, 4>(aw, sw, msg, msg_len);  // builds static tables once
  typedef EdRowsCfg<6, 4> C;
  static EdRowTabW<6, 4> TA;
  static EdRowTabW<ED_W, ED_K> TP;
  ge_p3 A, N;
  // per key
  g_fe_nmul = g_fe_nsq = 0;
  {
    static EdKeyPrep kp;
    fe x, y, z;
    (void)x; (void)y; (void)z;
    ed_decode_point(A, aw, g_C);
    uint32_t ab[8];
    ed_encode_affine(ab, A.X, A.Y, A.Z);
    ed_neg_point(N, A);
    ed_rows_w_init<ED_W, ED_K>(TP, N, g_C.d2);
  }
  out[6] = g_fe_nmul;
  out[7] = g_fe_nsq;
  // per item: double-scalar with fixed digits (the schedule is data-independent)
  uint32_t h[8], sr[8];
  for (int i = 0; i < 8; ++i) {
    h[i] = 0x9e3779b9u * (i + 1);
    sr[i] = 0x7f4a7c15u * (i + 3);
  }
  h[7] &= 0x0fffffffu;
  sr[7] &= 0x0fffffffu;
  uint32_t eh[C::kPackedWords], es[C::kPackedWords];
  sc_recode_w<6>(eh, C::kPackedWords, h);
  sc_recode_w<6>(es, C::kPackedWords, sr);
  ge_p2 R;
  ed_rows_w_init<6, 4>(TA, N, g_C.d2);
  g_fe_nmul = g_fe_nsq = 0;
  ed_double_scalar_w<6, 4>(R, eh, es, TA, TA);
  out[0] = g_fe_nmul;
  out[1] = g_fe_nsq;
  // finish per item: prefix product (1 mul), unwinding (2 mul), encode (2 mul)
  g_fe_nmul = g_fe_nsq = 0;
  fe run, zi, t;
  fe_1(run);
  fe_mul(run, run, R.Z);
  fe_mul(zi, run, R.Z);
  fe_mul(t, zi, R.Z);
  (void)ed_encode_cmp(R, zi, sw);
  out[2] = g_fe_nmul;
  out[3] = g_fe_nsq;
  g_fe_nmul = g_fe_nsq = 0;
  fe_invert(t, R.Z);
  out[4] = g_fe_nmul;
  out[5] = g_fe_nsq;
  return 0;
#else
  (void)aw; (void)sw; (void)msg; (void)msg_len; (void)out;
  return -1;
#endif
}

// ---------------------------------------------------------------- ECDSA rows (v2 pipeline)
#include "../../corda_amd/csrc/ecdsa_rows.h"
// The constant radix-2^22 G table (1.8 GB per curve): the host builds, with the device lane's code
// (ec_gwide_group_from), only the groups of 32 multiples the u1 digits touch.
template <int C>
static EcGWideTab* ec_gwide_host() {
  static EcGWideTab* TG = nullptr;
  if (!TG) TG = new EcGWideTab;
  return TG;
}
template <int C>
static void ec_gwide_touch(const u256w& u1) {
  constexpr int GG = EC_WIDE_GMULT / EC_MULT;
  static std::vector<bool> built;
  static Jac base[EC_WIDE_GDIGITS];  // 2^{22u} G
  static EcRowScratch* S = new EcRowScratch;
  const EcConsts& K = g_K[C];
  if (built.empty()) {
    built.assign(EC_WIDE_GDIGITS * GG, false);
    Jac P = {K.gx, K.gy, K.one_p};
    for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
      if (u > 0) jac_dbl_n<C>(P, P, EC_WIDE_GW);
      base[u] = P;
    }
  }
  EcGWideTab* TG = ec_gwide_host<C>();
  uint32_t dg[EC_WIDE_GPACKED];
  ec_recode_wide<EC_WIDE_GW, EC_WIDE_GDIGITS, false, EC_WIDE_GBITS>(dg, u1);
  for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
    const int d = ec_digit_at<EC_WIDE_GBITS>(dg, u), a = d < 0 ? -d : d;
    if (a == 0 || built[u * GG + (a - 1) / EC_MULT]) continue;
    const int g = (a - 1) / EC_MULT;
#ifdef FE_OP_COUNT
    const uint64_t m0 = g_m29_nmul[C][0], m1 = g_m29_nmul[C][1];  // table build: not item work
#endif
    ec_gwide_group_from<C>(&TG->t[u][g * EC_MULT], base[u], g, *S, K);
#ifdef FE_OP_COUNT
    g_m29_nmul[C][0] = m0;
    g_m29_nmul[C][1] = m1;
#endif
    built[u * GG + g] = true;
  }
}

template <int C>
static int ecdsa_rows_verify(const uint8_t* arena, uint64_t lr, uint64_t key_off, uint32_t key_len, uint32_t fmt,
                             uint64_t sig_off, uint32_t sig_len, uint64_t msg_off, uint64_t msg_len) {
  kinit();
  const EcConsts& K = g_K[C];
  static EcGTab* TG[2] = {nullptr, nullptr};
  static EcRowTab* TQ = new EcRowTab;
  static EcRowScratch* S = new EcRowScratch;
  if (!TG[C]) {  // the device table build, lane by lane
    TG[C] = new EcGTab;
    for (int l = 0; l < EC_G_DIGITS * (EC_G_MULT / EC_MULT); ++l)
      ec_gtab_group<C>(&TG[C]->t[l / (EC_G_MULT / EC_MULT)][(l % (EC_G_MULT / EC_MULT)) * EC_MULT],
                       l / (EC_G_MULT / EC_MULT), l % (EC_G_MULT / EC_MULT), *S, K);
  }
  f29 xm, ym;
  uint32_t st = ec_key_decode_bytes<C>(xm, ym, arena, lr, key_off, key_len, fmt, K);
  if (st) return (int)st;
  Jac bases[EC_ROWS];
  ec_row_bases<C>(bases, xm, ym, K);
  for (int j = 0; j < EC_ROWS; ++j) ec_row_build<C>(TQ->t[j], bases[j], *S, K);
  EcItemWs ws;
  st = ecdsa_prep<C>(ws, arena, lr, sig_off, sig_len, arena, lr, msg_off, msg_len);
  if (st) return (int)st;
  ecdsa_batch_inv<C, 1>(&ws, 1, 1u, K);
  kinit();
  ec_gwide_touch<C>(ws.a);
  return (int)ecdsa_ladder_check<C>(ws.a, ws.b, ws.r, *ec_gwide_host<C>(), *TQ, K);
}
// Executed Montgomery products per ECDSA item and stage (the GPU path's own lane code, host build):
// out[0..1] k_ec_prep (mod p, mod n), out[2..3] k_ec_inv per item (one shared inversion over 16
// items, EC_INV_K), out[4..5] k_ec_ladder with full tables. Returns the verdict.
template <int C>
static int ecdsa_count(const uint8_t* arena, uint64_t lr, uint64_t key_off, uint32_t key_len, uint32_t fmt,
                       uint64_t sig_off, uint32_t sig_len, uint64_t msg_off, uint64_t msg_len, uint64_t* out) {
#ifdef FE_OP_COUNT
  (void)ecdsa_rows_verify<C>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len);  // tables
  kinit();
  const EcConsts& K = g_K[C];
  static EcGTab* TG = nullptr;
  static EcRowTab* TQ = new EcRowTab;
  static EcRowScratch* S = new EcRowScratch;
  if (!TG) {
    TG = new EcGTab;
    for (int l = 0; l < EC_G_DIGITS * (EC_G_MULT / EC_MULT); ++l)
      ec_gtab_group<C>(&TG->t[l / (EC_G_MULT / EC_MULT)][(l % (EC_G_MULT / EC_MULT)) * EC_MULT],
                       l / (EC_G_MULT / EC_MULT), l % (EC_G_MULT / EC_MULT), *S, K);
  }
  f29 xm, ym;
  uint32_t st = ec_key_decode_bytes<C>(xm, ym, arena, lr, key_off, key_len, fmt, K);
  if (st) return (int)st;
  Jac bases[EC_ROWS];
  ec_row_bases<C>(bases, xm, ym, K);
  for (int j = 0; j < EC_ROWS; ++j) ec_row_build<C>(TQ->t[j], bases[j], *S, K);
  auto snap = [&](uint64_t* o) {
    o[0] = g_m29_nmul[C][0];
    o[1] = g_m29_nmul[C][1];
    g_m29_nmul[C][0] = g_m29_nmul[C][1] = 0;
  };
  g_m29_nmul[C][0] = g_m29_nmul[C][1] = 0;
  EcItemWs ws[EC_INV_K];
  st = ecdsa_prep<C>(ws[0], arena, lr, sig_off, sig_len, arena, lr, msg_off, msg_len);
  snap(out);
  if (st) return (int)st;
  for (int k = 1; k < EC_INV_K; ++k) ws[k] = ws[0];
  ecdsa_batch_inv<C, EC_INV_K>(ws, EC_INV_K, (1u << EC_INV_K) - 1u, K);
  snap(out + 2);
  ec_gwide_touch<C>(ws[0].a);
  st = ecdsa_ladder_check<C>(ws[0].a, ws[0].b, ws[0].r, *ec_gwide_host<C>(), *TQ, K);
  snap(out + 4);
  return (int)st;
#else
  return -1;
#endif
}
extern "C" int t_ecdsa_count(int scheme, const uint8_t* arena, uint64_t arena_len, uint64_t key_off, uint32_t key_len,
                             uint32_t fmt, uint64_t sig_off, uint32_t sig_len, uint64_t msg_off, uint64_t msg_len,
                             uint64_t* out) {
  const uint64_t lr = (arena_len + 3) & ~3ull;
  if (scheme == 3)
    return ecdsa_count<CG_CURVE_R1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len, out);
  return ecdsa_count<CG_CURVE_K1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len, out);
}

extern "C" int t_ecdsa_verify_rows(int scheme, const uint8_t* arena, uint64_t arena_len, uint64_t key_off,
                                   uint32_t key_len, uint32_t fmt, uint64_t sig_off, uint32_t sig_len,
                                   uint64_t msg_off, uint64_t msg_len) {
  const uint64_t lr = (arena_len + 3) & ~3ull;
  if (scheme == 3)
    return ecdsa_rows_verify<CG_CURVE_R1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len);
  return ecdsa_rows_verify<CG_CURVE_K1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len);
}

// ---------------------------------------------------------------- 29-bit Montgomery
#include "../../corda_amd/csrc/mont29.h"
template <int C, int N>
static void m29_mul_words(const uint32_t* a, const uint32_t* b, uint32_t* out, int lazy) {
  f29 x, y, r;
  f29_from_words(x, a);
  f29_from_words(y, b);
  if (lazy) {  // feed x + x and y + y (limbs < 2^30, value < 4m) as the operands
    m29_add_lazy(x, x, x);
    m29_add_lazy(y, y, y);
  }
  m29_mul<C, N>(r, x, y);
  m29_to_words_canon<C, N>(out, r);
}
// 1 if (curve, n) elements are kept in plain form (R = 1, mont29.h m29_plain), else 0 (R = 2^261)
extern "C" int t_m29_plain(int curve, int n) {
  return curve == 0 && n == 0 ? m29_plain(0, 0) : curve == 0 ? m29_plain(0, 1) : n == 0 ? m29_plain(1, 0) : m29_plain(1, 1);
}

extern "C" void t_m29_op(int curve, int n, int op, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  // op 0: a b R^-1; 1: (2a)(2b) R^-1 via lazy sums; 2: a + b; 3: a - b (inputs reduced < 2m)
  if (op <= 1) {
    if (curve == 1 && n == 0) m29_mul_words<1, 0>(a, b, out, op);
    else if (curve == 1) m29_mul_words<1, 1>(a, b, out, op);
    else if (n == 0) m29_mul_words<0, 0>(a, b, out, op);
    else m29_mul_words<0, 1>(a, b, out, op);
    return;
  }
  f29 x, y, r;
  f29_from_words(x, a);
  f29_from_words(y, b);
#define M29_BIN(CC, NN)                                    \
  if (op == 2) m29_add<CC, NN>(r, x, y);                   \
  else m29_sub<CC, NN>(r, x, y);                           \
  m29_to_words_canon<CC, NN>(out, r);
  if (curve == 1 && n == 0) { M29_BIN(1, 0) }
  else if (curve == 1) { M29_BIN(1, 1) }
  else if (n == 0) { M29_BIN(0, 0) }
  else { M29_BIN(0, 1) }
#undef M29_BIN
}

// ---------------------------------------------------------------- Ed25519 rows + radix-2^10 B
struct EdBWideTab;
static void tbw_init();
static void tbw_touch(const uint32_t* es);
static EdBWideTab* g_TBW = nullptr;
static EdBTabW<ED_W, ED_K, ED_WB>* g_TB10 = nullptr;
static void tb10_init() {
  if (g_TB10) return;
  g_TB10 = new EdBTabW<ED_W, ED_K, ED_WB>;
  ge_p3 B;
  fe x, y, two_inv, t;
  fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
  fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
  fe_0(t);
  t.v[0] = 2;
  fe_invert(two_inv, t);
  fe_mul(B.X, x, two_inv);
  fe_mul(B.Y, y, two_inv);
  fe_1(B.Z);
  fe_mul(B.T, B.X, B.Y);
  for (int u = 0; u < EdBCfg<ED_W, ED_K, ED_WB>::kDigits; ++u) ed_btab_wb_row<ED_W, ED_K, ED_WB>(g_TB10->t[u], B, u, g_C.d2);
}
static void host_pick(ge_niels& out, const ge_niels* row, int d) { ed_pick_w(out, row, d); }

template <bool Signed>
static int ed_verify_wb(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len,
                        uint64_t* counts) {
  init();
  tb10_init();
  typedef EdRowsCfg<ED_W, ED_K> C;
  typedef EdBCfg<ED_W, ED_K, ED_WB> CB;
  static EdRowTabW<ED_W, ED_K> TA;
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  if (kp.status) return (int)kp.status;
  ge_p3 A, N;
  ed_decode_point(A, aw, g_C);
  ed_neg_point(N, A);
  ed_rows_w_init<ED_W, ED_K>(TA, N, g_C.d2);
  static uint8_t buf[1 << 20];
  memcpy(buf, msg, msg_len);
  uint32_t pre[16], hw[16], h[8];
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];
    pre[8 + i] = kp.abyte[i];
  }
  sha512_prefix64_msg(hw, pre, buf, (msg_len + 3) & ~3ull, 0, msg_len);
  sc_reduce512(h, hw);
  uint32_t s[8], sr[8];
  for (int i = 0; i < 8; ++i) s[i] = sw[8 + i];
  sc_reduce256(sr, s);
  if ((s[7] >> 31) && sc_slide_escapes(s)) {
    uint32_t r1[8];
    for (int i = 0; i < 8; ++i) r1[i] = sc_R1w(i);
    sc_sub(sr, sr, r1);
  }
  uint32_t eh[C::kPackedWords], es[EdWideCfg::kBPackedWords];
  sc_recode_w<ED_W>(eh, C::kPackedWords, h);
  sc_recode_wb<ED_WIDE_BW, EdWideCfg::kBBits>(es, EdWideCfg::kBPackedWords, sr);
  tbw_init();
  tbw_touch(es);
  ge_p2 R;
#ifdef FE_OP_COUNT
  g_fe_nmul = g_fe_nsq = g_fe9_nmul = 0;
#endif
  ed_double_scalar_fw<ED_W, ED_K, Signed>(R, eh, es, TA, *g_TBW, host_pick, host_pick);
#ifdef FE_OP_COUNT
  if (counts) {  // [0..1] radix-2^25.5 products and squarings (A part), [2] radix-2^29 products (B part)
    counts[0] = g_fe_nmul;
    counts[1] = g_fe_nsq;
    counts[2] = g_fe9_nmul;
  }
#endif
  fe zi;
  fe_invert(zi, R.Z);
  return ed_encode_cmp(R, zi, sw);
}

extern "C" int t_ed_verify_wb(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len,
                              uint64_t* counts) {
  return ed_verify_wb<false>(aw, sw, msg, msg_len, counts);
}

// the signed-addition form of k_ed_ladder_pf (ge_madd_signed), bounds-checked
extern "C" int t_ed_verify_wb_signed(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len,
                                     uint64_t* counts) {
  return ed_verify_wb<true>(aw, sw, msg, msg_len, counts);
}

// ---------------------------------------------------------------- wide tables (hot keys)
// k_ed_wide_chain / k_ed_wide_tab / k_ed_bwide_init / k_ed_ladder_wide's arithmetic, bounds-checked.
// The constant B table is 62.9 MB (radix 2^16): the host builds, with the device lane's code
// (ed_bwide_group), only the groups of 8 multiples an item's digits touch.
static std::vector<bool> g_TBW_built;
static ge_p3 g_TBW_base[EdWideCfg::kBDigits];  // 2^{16u} B
static void tbw_init() {
  if (g_TBW) return;
  g_TBW = new EdBWideTab;
  ge9_niels_identity_half(g_TBW->ident);
  g_TBW_built.assign(EdWideCfg::kBDigits * (EdWideCfg::kBMult / 8), false);
  ge_p3 B;
  fe x, y, two_inv, t;
  fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
  fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
  fe_0(t);
  t.v[0] = 2;
  fe_invert(two_inv, t);
  fe_mul(B.X, x, two_inv);
  fe_mul(B.Y, y, two_inv);
  fe_1(B.Z);
  fe_mul(B.T, B.X, B.Y);
  ge_p3 P = B;
  for (int u = 0; u < EdWideCfg::kBDigits; ++u) {
    if (u > 0) ed_dbl_n(P, P, ED_WIDE_BW);
    g_TBW_base[u] = P;
  }
}
static void tbw_touch(const uint32_t* es) {
  for (int u = 0; u < EdWideCfg::kBDigits; ++u) {
    const int d = sc_digit_at<EdWideCfg::kBBits>(es, u), a = d < 0 ? -d : d;
    if (a == 0) continue;
    const int grp = (a - 1) / 8;
    const size_t k = (size_t)u * (EdWideCfg::kBMult / 8) + grp;
    if (g_TBW_built[k]) continue;
    ed_bwide_group(&g_TBW->t[u][8 * grp], g_TBW_base[u], 0, grp, g_C.d2);
    g_TBW_built[k] = true;
  }
}

// counts (optional): [0..1] ladder fe_mul / fe_sq per item, [2..3] table build per key (chain + rows)
// k_ed_wide_rows (one lane per row) against the three-pass build (k_ed_wide_fwd / _inv / _bwd)
// for the row base P = m B (m >= 1): the number of entries whose canonical encodings differ.
extern "C" int t_ed_wide_row_cmp(uint32_t m) {
  init();
  ge_p3 B, P;
  {  // B from the constant niels entry 1 B (as t_ed_verify_v2)
    fe x, y, two_inv, t;
    fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_0(t);
    t.v[0] = 2;
    fe_invert(two_inv, t);
    fe_mul(B.X, x, two_inv);
    fe_mul(B.Y, y, two_inv);
    fe_1(B.Z);
    fe_mul(B.T, B.X, B.Y);
  }
  ed_small_mul(P, B, m, g_C.d2);
  static ge_niels a[EdWideCfg::kMult], b[EdWideCfg::kMult];
  static fe pre[EdWideCfg::kMult], zc[EdWideCfg::kMult], px[EdWideCfg::kMult], py[EdWideCfg::kMult],
      pz[EdWideCfg::kMult];
  for (int g = 0; g < 4; ++g)  // any split; parked in plain arrays (the host policy) ...
    ed_wide_row_build(a, EdParkRow{px + 32 * g, py + 32 * g, pz + 32 * g, pre + 32 * g}, P, 32 * g, 32 * g + 32,
                      g_C.d2);
  {  // ... or lane-interleaved (the device policy): the same entries
    static ge_niels a2[EdWideCfg::kMult];
    static uint32_t park[EdWideCfg::kMult * ED_PARK_DWORDS];
    for (int g = 0; g < 4; ++g)
      ed_wide_row_build(a2, EdParkLanes{park, (uint32_t)g, 4u}, P, 32 * g, 32 * g + 32, g_C.d2);
    if (memcmp(a, a2, sizeof a) != 0) return -1;
  }
  {  // k_ed_wide_rows' radix-2^29 walk (ed_wide_row_build9, split in 2 lanes): equal mod p
    static ge9_niels a9[EdWideCfg::kMult];
    static uint32_t park9[EdWideCfg::kMult * ED_PARK9_DWORDS];
    for (int g = 0; g < 2; ++g)
      ed_wide_row_build9(a9, EdPark9Lanes{park9, (uint32_t)g, 2u}, P, 64 * g, 64 * g + 64, g_C.d2);
    for (int k = 0; k < EdWideCfg::kMult; ++k) {
      const fe* fa[3] = {&a[k].ypx, &a[k].ymx, &a[k].xy2d};
      const fe9* f9[3] = {&a9[k].ypx, &a9[k].ymx, &a9[k].xy2d};
      for (int q = 0; q < 3; ++q) {
        uint32_t u[8], v[8];
        fe t;
        fe_from_fe9(t, *f9[q]);
        fe_tobytes_words(u, *fa[q]);
        fe_tobytes_words(v, t);
        if (memcmp(u, v, 32) != 0) return -2;
        for (int i = 0; i < 9; ++i)  // tight limbs (class T): the ladder's operand bound
          if (f9[q]->v[i] >= (i == 1 ? (1u << 29) + (1u << 17) : (1u << 29))) return -3;
      }
    }
  }
  constexpr int CPG = ED_WIDE_GROUP / ED_WIDE_CHUNK;
  for (int g = 0; g < ED_WIDE_GROUPS; ++g) ed_wide_group_pass<false>((ge_niels*)nullptr, &zc[CPG * g], P, g, g_C.d2);
  fe_invert_run<ED_WIDE_CHUNKS>(zc, zc + ED_WIDE_CHUNKS);
  for (int g = 0; g < ED_WIDE_GROUPS; ++g) ed_wide_group_pass<true>(&b[ED_WIDE_GROUP * g], &zc[CPG * g], P, g, g_C.d2);
  int bad = 0;
  for (int k = 0; k < EdWideCfg::kMult; ++k) {
    uint32_t u[8], v[8];
    const fe* fa[3] = {&a[k].ypx, &a[k].ymx, &a[k].xy2d};
    const fe* fb[3] = {&b[k].ypx, &b[k].ymx, &b[k].xy2d};
    for (int q = 0; q < 3; ++q) {
      fe_tobytes_words(u, *fa[q]);
      fe_tobytes_words(v, *fb[q]);
      if (memcmp(u, v, 32) != 0) {
        ++bad;
        break;
      }
    }
  }
  return bad;
}

extern "C" int t_ed_verify_wide(const uint32_t* aw, const uint32_t* sw, const uint8_t* msg, uint64_t msg_len,
                                uint64_t* counts) {
  init();
  tbw_init();
  static EdWideTab* TA = new EdWideTab;
  static fe (*zpre)[EdWideCfg::kMult] = new fe[EdWideCfg::kRows][EdWideCfg::kMult];
  static EdKeyPrep kp;
  ed_key_prep(kp, aw, g_C);
  if (kp.status) return (int)kp.status;
  ge_p3 A, P;
  ed_decode_point(A, aw, g_C);
  ed_neg_point(P, A);
  static uint32_t last_key[8];
  static bool have = false;
  static uint64_t build_mul = 0, build_sq = 0;
  if (!have || memcmp(last_key, aw, 32) != 0) {  // the fixtures reuse keys: rebuild on change
#ifdef FE_OP_COUNT
    g_fe_nmul = g_fe_nsq = 0;
#endif
    for (int j = 0; j < EdWideCfg::kRows; ++j) {  // k_ed_wide_chain, then the k_ed_wide_rows lanes
      if (j > 0) ed_dbl_n(P, P, ED_WIDE_W);
      for (int g = 0; g < ED_WIDE_ROW_LANES; ++g)
      {
        const int e0 = g * (EdWideCfg::kMult / ED_WIDE_ROW_LANES), e1 = e0 + EdWideCfg::kMult / ED_WIDE_ROW_LANES;
        static fe px[EdWideCfg::kMult], py[EdWideCfg::kMult], pz[EdWideCfg::kMult];
        ed_wide_row_build(TA->t[j], EdParkRow{px, py, pz, zpre[j] + e0}, P, e0, e1, g_C.d2);
      }
    }
#ifdef FE_OP_COUNT
    build_mul = g_fe_nmul;
    build_sq = g_fe_nsq;
#endif
    memcpy(last_key, aw, 32);
    have = true;
  }
  if (counts) {
    counts[2] = build_mul;
    counts[3] = build_sq;
  }
  static uint8_t buf[1 << 20];
  memcpy(buf, msg, msg_len);
  uint32_t pre[16], hw[16], h[8];
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];
    pre[8 + i] = kp.abyte[i];
  }
  sha512_prefix64_msg(hw, pre, buf, (msg_len + 3) & ~3ull, 0, msg_len);
  sc_reduce512(h, hw);
  uint32_t s[8], sr[8];
  for (int i = 0; i < 8; ++i) s[i] = sw[8 + i];
  sc_reduce256(sr, s);
  if ((s[7] >> 31) && sc_slide_escapes(s)) {
    uint32_t r1[8];
    for (int i = 0; i < 8; ++i) r1[i] = sc_R1w(i);
    sc_sub(sr, sr, r1);
  }
  uint32_t eh[EdWideCfg::kPackedWords], es[EdWideCfg::kBPackedWords];
  sc_recode_w<ED_WIDE_W>(eh, EdWideCfg::kPackedWords, h);
  sc_recode_wb<ED_WIDE_BW, EdWideCfg::kBBits>(es, EdWideCfg::kBPackedWords, sr);
  tbw_touch(es);
  ge_p2 R;
#ifdef FE_OP_COUNT
  g_fe_nmul = g_fe_nsq = 0;
#endif
  g_fe9_nmul = 0;
  ed_double_scalar_wide(R, eh, es, *TA, *g_TBW);
#ifdef FE_OP_COUNT
  if (counts) {
    counts[0] = g_fe9_nmul;  // radix-2^29 products (fe9.h): the wide ladder has no fe products
    counts[1] = g_fe_nsq;
  }
#endif
  fe zi;
  fe_invert(zi, R.Z);
  return ed_encode_cmp(R, zi, sw);
}

// k_ec_gwide_init / k_ec_wide_chain / k_ec_wide_tab / k_ec_ladder_wide. counts (optional):
// [0] ladder Montgomery products mod p per item, [1] table build per key (chain + rows).
template <int C>
static int ecdsa_wide_verify(const uint8_t* arena, uint64_t lr, uint64_t key_off, uint32_t key_len, uint32_t fmt,
                             uint64_t sig_off, uint32_t sig_len, uint64_t msg_off, uint64_t msg_len, uint64_t* counts) {
  kinit();
  const EcConsts& K = g_K[C];
  static EcGWideTab* TG[2] = {nullptr, nullptr};
  static std::vector<bool> tg_built[2];
  static Jac tg_base[2][EC_WIDE_GDIGITS];  // 2^{16u} G
  static EcWideTab* TQ = new EcWideTab;
  static EcWideScratch* WS = new EcWideScratch;
  static EcRowScratch* S = new EcRowScratch;
  constexpr int GG = EC_WIDE_GMULT / EC_MULT;
  if (!TG[C]) {  // the device lane's code (ec_gwide_group_from), for the groups the digits touch
    TG[C] = new EcGWideTab;
    tg_built[C].assign(EC_WIDE_GDIGITS * GG, false);
    Jac P = {K.gx, K.gy, K.one_p};
    for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
      if (u > 0) jac_dbl_n<C>(P, P, EC_WIDE_GW);
      tg_base[C][u] = P;
    }
  }
  f29 xm, ym;
  uint32_t st = ec_key_decode_bytes<C>(xm, ym, arena, lr, key_off, key_len, fmt, K);
  if (st) return (int)st;
  static f29 last_x, last_y;
  static int last_c = -1;
  static uint64_t build_count = 0;
  if (last_c != C || !f29_eq_raw(last_x, xm) || !f29_eq_raw(last_y, ym)) {  // rebuild on key change
#ifdef FE_OP_COUNT
    g_m29_nmul[C][0] = g_m29_nmul[C][1] = 0;
#endif
    static Jac jb[EC_WIDE_DIGITS];  // k_ec_wide_chain: Jacobian chain, then affine bases
    static EcAff ab[EC_WIDE_DIGITS];
    Jac P = {xm, ym, K.one_p};
    for (int j = 0; j < EC_WIDE_DIGITS; ++j) {
      if (j > 0) jac_dbl_n<C>(P, P, EC_WIDE_W);
      jb[j] = P;
    }
    jac_batch_to_affine<C>(ab, jb, EC_WIDE_DIGITS, WS->pre, K);
    for (int j = 0; j < EC_WIDE_ROWS; ++j) {  // k_ec_wide_rows lanes
      const EcAff& base = ab[j < EC_WIDE_DIGITS ? j : EC_WIDE_DIGITS - 1];
      for (int g = 0; g < EC_WIDE_ROW_LANES; ++g) {
        const int e0 = g * (EC_WIDE_MULT / EC_WIDE_ROW_LANES), e1 = e0 + EC_WIDE_MULT / EC_WIDE_ROW_LANES;
        ec_wide_row_build<C>(TQ->t[j], EcParkRow{TQ->t[j] + e0, WS->z + e0}, base, j == EC_WIDE_DIGITS, e0, e1, K);
      }
    }
#ifdef FE_OP_COUNT
    build_count = g_m29_nmul[C][0];
#endif
    last_x = xm;
    last_y = ym;
    last_c = C;
  }
  if (counts) counts[1] = build_count;
  EcItemWs ws;
  st = ecdsa_prep<C>(ws, arena, lr, sig_off, sig_len, arena, lr, msg_off, msg_len);
  if (st) return (int)st;
  ecdsa_batch_inv<C, 1>(&ws, 1, 1u, K);
  {
    uint32_t dg[EC_WIDE_GPACKED];
    ec_recode_wide<EC_WIDE_GW, EC_WIDE_GDIGITS, false, EC_WIDE_GBITS>(dg, ws.a);
    for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
      const int d = ec_digit_at<EC_WIDE_GBITS>(dg, u), a = d < 0 ? -d : d;
      if (a == 0 || tg_built[C][u * GG + (a - 1) / EC_MULT]) continue;
      const int g = (a - 1) / EC_MULT;
      ec_gwide_group_from<C>(&TG[C]->t[u][g * EC_MULT], tg_base[C][u], g, *S, K);
      tg_built[C][u * GG + g] = true;
    }
  }
#ifdef FE_OP_COUNT
  g_m29_nmul[C][0] = g_m29_nmul[C][1] = 0;
  g_m29_nsqr[C] = 0;
#endif
  st = ecdsa_ladder_check_wide<C>(ws.a, ws.b, ws.r, *TG[C], *TQ, K);
#ifdef FE_OP_COUNT
  if (counts) {
    counts[0] = g_m29_nmul[C][0];
    counts[2] = g_m29_nsqr[C];  // of counts[0], the squares
  }
#endif
  return (int)st;
}

// k_ec_wide_rows (co-Z, one lane per row) against the three-pass build (k_ec_wide_fwd / _inv /
// _bwd) for row base m * G (m >= 1): every entry of rows 0, 1 and 32-style (top) equal after
// canonicalisation. Returns the number of differing entries.
template <int C>
static int ec_wide_row_cmp(uint32_t m) {
  kinit();
  const EcConsts& K = g_K[C];
  Jac P;
  jac_small_mul_aff<C>(P, K.gx, K.gy, m, K);
  EcAff base;
  jac_to_affine<C>(base.x, base.y, P, K);
  static EcAff a[EC_WIDE_MULT], b[EC_WIDE_MULT];
  static f29 lam[EC_WIDE_MULT];
  static EcWideScratch ws;
  int bad = 0;
  for (int top = 0; top < 2; ++top) {
    const int j = top ? EC_WIDE_DIGITS : 0;
    for (int g = 0; g < 4; ++g)  // split in 4 lanes (the same entries as one lane, or any split)
      ec_wide_row_build<C>(a, EcParkRow{a + 32 * g, lam + 32 * g}, base, top != 0, 32 * g, 32 * g + 32, K);
    {  // lane-interleaved parking (the device policy): the same entries
      static EcAff a2[EC_WIDE_MULT];
      static uint32_t park[EC_WIDE_MULT * EC_PARK_DWORDS];
      for (int g = 0; g < 4; ++g)
        ec_wide_row_build<C>(a2, EcParkLanes{park, (uint32_t)g, 4u}, base, top != 0, 32 * g, 32 * g + 32, K);
      if (memcmp(a, a2, sizeof a) != 0) ++bad;
    }
    constexpr int CPG = 32 / EC_WIDE_CHUNK;
    for (int g = 0; g < EC_WIDE_MULT / 32; ++g) ec_wide_group_pass<C, false>(nullptr, &ws.z[CPG * g], base, j, g, K);
    m29_invert_run<C, EC_WIDE_CHUNKS>(ws.z, ws.pre, K);
    for (int g = 0; g < EC_WIDE_MULT / 32; ++g) ec_wide_group_pass<C, true>(&b[32 * g], &ws.z[CPG * g], base, j, g, K);
    for (int e = 0; e < EC_WIDE_MULT; ++e)
      if (!m29_eq<C, 0>(a[e].x, b[e].x) || !m29_eq<C, 0>(a[e].y, b[e].y)) ++bad;
  }
  return bad;
}
extern "C" int t_ec_wide_row_cmp(int curve, uint32_t m) {
  return curve == CG_CURVE_R1 ? ec_wide_row_cmp<CG_CURVE_R1>(m) : ec_wide_row_cmp<CG_CURVE_K1>(m);
}

extern "C" int t_ecdsa_verify_wide(int scheme, const uint8_t* arena, uint64_t arena_len, uint64_t key_off,
                                   uint32_t key_len, uint32_t fmt, uint64_t sig_off, uint32_t sig_len,
                                   uint64_t msg_off, uint64_t msg_len, uint64_t* counts) {
  const uint64_t lr = (arena_len + 3) & ~3ull;
  if (scheme == 3)
    return ecdsa_wide_verify<CG_CURVE_R1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len, counts);
  return ecdsa_wide_verify<CG_CURVE_K1>(arena, lr, key_off, key_len, fmt, sig_off, sig_len, msg_off, msg_len, counts);
}

// jac_madd_w (the wide ladder's mixed addition: lazy sums, inf flag, Z3 = Z1 * 2H) against
// jac_madd on chains of random additions of multiples of G with random signs, plus the exceptional
// cases: acc + acc (doubling), acc + (-acc) (infinity), infinity + Q. Returns mismatches.
template <int C>
static int madd_w_cmp(uint64_t seed, int n) {
  EcConsts K;
  ec_consts_init<C>(K);
  int bad = 0;
  uint64_t s = seed;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  auto same = [&](const Jac& a, bool ainf, const Jac& b) {
    const bool binf = m29_iszero<C, 0>(b.Z);
    if (ainf || binf) return ainf == binf;
    f29 x1, y1, x2, y2;
    jac_to_affine<C>(x1, y1, a, K);
    jac_to_affine<C>(x2, y2, b, K);
    return m29_eq<C, 0>(x1, x2) && m29_eq<C, 0>(y1, y2);
  };
  for (int t = 0; t < n; ++t) {
    // acc = k G (Jacobian, Z != 1 after the multiplication), q = m G affine
    Jac acc, q;
    jac_small_mul_aff<C>(acc, K.gx, K.gy, 2 + (uint32_t)(rnd() % 5000), K);
    const int kind = t % 4;
    f29 qx, qy;
    if (kind == 0) {
      jac_small_mul_aff<C>(q, K.gx, K.gy, 2 + (uint32_t)(rnd() % 5000), K);
      jac_to_affine<C>(qx, qy, q, K);
    } else {  // kinds 1, 2: Q = +-acc (doubling / infinity); kind 3: acc = infinity
      jac_to_affine<C>(qx, qy, acc, K);
    }
    const bool neg = kind == 2 ? true : (kind == 1 ? false : (rnd() & 1));
    Jac ref = acc, got = acc;
    bool inf = kind == 3;
    if (kind == 3) jac_set_inf<C>(ref, K);
    f29 y = qy;
    if (neg) m29_neg<C, 0>(y, qy);
    jac_madd<C>(ref, ref, qx, y, K);
    jac_madd_w<C>(got, inf, qx, qy, neg, K);
    // and a second addition on top (the flag and the outputs' bounds carry over)
    f29 y2 = K.gy;
    jac_madd<C>(ref, ref, K.gx, y2, K);
    jac_madd_w<C>(got, inf, K.gx, K.gy, false, K);
    if (!same(got, inf, ref)) ++bad;
    // doublings: jac_dbl_w against jac_dbl, twice (the second on a semi-lazy-built input)
    if (!inf) {
      Jac d1 = got, d2 = got;
      jac_dbl<C>(d1, d1);
      jac_dbl<C>(d1, d1);
      jac_dbl_w<C>(d2, d2);
      jac_dbl_w<C>(d2, d2);
      if (!same(d2, false, d1)) ++bad;
    }
  }
  return bad;
}
// jac_madd9 (ec9.h, signed limbs) against the exception-complete jac_madd over chains of n additions
// of random multiples of G (a wide ladder's 44 and more), with Q = +-acc cases (the exact path);
// every product's columns are asserted below 2^63 (FE_BOUNDS_CHECK). Returns mismatching chains.
template <int C>
static int madd9_cmp(uint64_t seed, int chains, int len) {
  EcConsts K;
  ec_consts_init<C>(K);
  uint64_t s = seed;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  int bad = 0;
  for (int t = 0; t < chains; ++t) {
    Jac ref, got;
    jac_set_inf<C>(ref, K);
    got = ref;
    bool inf = true;
    for (int o = 0; o < len; ++o) {
      f29 qx, qy;
      const int kind = (int)(rnd() % 64);
      bool neg = rnd() & 1;
      if (o > 0 && kind == 0) {  // Q = +-R (doubling or infinity through the exact path)
        f29 ax, ay;
        jac_to_affine<C>(ax, ay, ref, K);
        if (m29_iszero<C, 0>(ref.Z)) continue;
        qx = ax;
        qy = ay;
      } else {
        Jac q;
        jac_small_mul_aff<C>(q, K.gx, K.gy, 1 + (uint32_t)(rnd() % 100000), K);
        jac_to_affine<C>(qx, qy, q, K);
      }
      f29 y = qy;
      if (neg) m29_neg<C, 0>(y, qy);
      if (m29_iszero<C, 0>(ref.Z)) {  // jac_madd's infinity input: R = Q
        ref.X = qx;
        ref.Y = y;
        ref.Z = K.one_p;
      } else {
        jac_madd<C>(ref, ref, qx, y, K);
      }
      jac_madd9<C>(got, inf, qx, qy, neg, K);
    }
    Jac g;
    ec9_to_m29<C>(g.X, got.X);
    ec9_to_m29<C>(g.Y, got.Y);
    ec9_to_m29<C>(g.Z, got.Z);
    const bool rinf = m29_iszero<C, 0>(ref.Z), ginf = inf || m29_iszero<C, 0>(g.Z);
    if (rinf || ginf) {
      bad += rinf != ginf;
      continue;
    }
    f29 x1, y1, x2, y2;
    jac_to_affine<C>(x1, y1, ref, K);
    jac_to_affine<C>(x2, y2, g, K);
    if (!(m29_eq<C, 0>(x1, x2) && m29_eq<C, 0>(y1, y2))) ++bad;
  }
  return bad;
}
extern "C" void t_ec9_to_m29(int curve, const uint32_t* in, uint32_t* out) {
  f29 a, r;
  memcpy(a.v, in, 36);
  if (curve == 1) ec9_to_m29<CG_CURVE_R1>(r, a);
  else ec9_to_m29<CG_CURVE_K1>(r, a);
  memcpy(out, r.v, 36);
}
extern "C" void t_ec9_mul(int curve, int form, const uint32_t* a, const uint32_t* b, const uint32_t* c,
                          const uint32_t* d, uint32_t* out) {
  f29 A, B, Cc, D, R;
  memcpy(A.v, a, 36);
  memcpy(B.v, b, 36);
  memcpy(Cc.v, c, 36);
  memcpy(D.v, d, 36);
  if (curve == 1) {
    if (form == 0) ec9_mul<CG_CURVE_R1>(R, A, B);
    else if (form == 1) ec9_mul_add<CG_CURVE_R1>(R, A, B, Cc);
    else if (form == 2) ec9_mul2<CG_CURVE_R1>(R, A, B, Cc, D);
    else if (form == 3) ec9_sqr<CG_CURVE_R1>(R, A);
    else ec9_sqr_add<CG_CURVE_R1>(R, A, Cc);
  } else {
    if (form == 0) ec9_mul<CG_CURVE_K1>(R, A, B);
    else if (form == 1) ec9_mul_add<CG_CURVE_K1>(R, A, B, Cc);
    else if (form == 2) ec9_mul2<CG_CURVE_K1>(R, A, B, Cc, D);
    else if (form == 3) ec9_sqr<CG_CURVE_K1>(R, A);
    else ec9_sqr_add<CG_CURVE_K1>(R, A, Cc);
  }
  memcpy(out, R.v, 36);
}
extern "C" int t_ec_madd9_cmp(int curve, uint64_t seed, int chains, int len) {
  return curve == 1 ? madd9_cmp<CG_CURVE_R1>(seed, chains, len) : madd9_cmp<CG_CURVE_K1>(seed, chains, len);
}
extern "C" int t_ec_madd_w_cmp(int curve, uint64_t seed, int n) {
  return curve == 1 ? madd_w_cmp<CG_CURVE_R1>(seed, n) : madd_w_cmp<CG_CURVE_K1>(seed, n);
}

// SpliceLd (sha2.h: the hash kernels' view of prefix || id || suffix) against the same bytes
// materialised: SHA-512 with a 64-byte prefix (the Ed25519 challenge) and SHA-256 from a midstate
// (ECDSA's e), for prefixes of 0..299 and suffixes of 0..17 bytes. Returns mismatches.
extern "C" int t_sha_splice_cmp(uint64_t seed, int n) {
  uint64_t s = seed | 1;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  int bad = 0;
  for (int t = 0; t < n; ++t) {
    const uint32_t pl = (uint32_t)(rnd() % 300), sl = (uint32_t)(rnd() % 18), len = pl + 32 + sl;
    const uint32_t slot = (len + 15) & ~15u;
    std::vector<uint8_t> img(slot + 64, 0), msg(((len + 3) & ~3u) + 64, 0);
    uint32_t id[8];
    for (int k = 0; k < 8; ++k) id[k] = (uint32_t)rnd();
    for (uint32_t k = 0; k < len; ++k) {
      uint8_t b = (uint8_t)rnd();
      if (k >= pl && k < pl + 32) b = ((const uint8_t*)id)[k - pl];
      else img[k] = b;
      msg[k] = b;
    }
    SpliceLd ld{img.data(), slot, id, pl};
    uint32_t pre[16], a[16], b[16];
    for (int k = 0; k < 16; ++k) pre[k] = (uint32_t)rnd();
    sha512_prefix64_ld(a, pre, ld, 0, len);
    sha512_prefix64_msg(b, pre, msg.data(), (len + 3) & ~3u, 0, len);
    if (memcmp(a, b, sizeof a)) ++bad;
    // the Ed25519 challenge's splice form, with and without block 1's template schedule (k_tmpl_prep)
    uint32_t c[16];
    sha512_prefix64_splice(c, pre, ld, len, nullptr);
    if (memcmp(c, b, sizeof c)) ++bad;
    if (pl >= 192) {  // keyws.h TMPL_ED_MID_MIN_PREFIX: block 1 is all template prefix
      uint64_t wk[80], w8[16];
      for (int j = 0; j < 16; ++j) {
        uint64_t v = 0;
        for (int q = 0; q < 8; ++q) v = (v << 8) | img[64 + 8 * j + q];
        w8[j] = v;
        wk[j] = v + cg_k512(j);
      }
      for (int r = 16; r < 80; r += 16)
        for (int j = 0; j < 16; ++j) wk[r + j] = sha512_sched(w8, j) + cg_k512(r + j);
      sha512_prefix64_splice(c, pre, ld, len, wk);
      if (memcmp(c, b, sizeof c)) ++bad;
    }
    // SHA-256 from the midstate after the prefix's full blocks
    uint32_t st[8], w[16];
    sha256_init(st);
    const uint32_t blocks = pl / 64;
    for (uint32_t bl = 0; bl < blocks; ++bl) {
      for (int j = 0; j < 16; ++j)
        w[j] = ((uint32_t)msg[64 * bl + 4 * j] << 24) | ((uint32_t)msg[64 * bl + 4 * j + 1] << 16) |
               ((uint32_t)msg[64 * bl + 4 * j + 2] << 8) | msg[64 * bl + 4 * j + 3];
      sha256_compress(st, w);
    }
    uint32_t h1[8], h2[8];
    sha256_ld_suffix(h1, ld, 0, len, nullptr, st, blocks);
    sha256_arena_suffix(h2, msg.data(), (len + 3) & ~3u, 0, len, nullptr);
    if (memcmp(h1, h2, sizeof h1)) ++bad;
  }
  return bad;
}

// k_ed_keyprep_tab / k_ec_keyprep_tab (ed_row_build_parked / ec_row_build_parked, lane-interleaved
// park of 3 lanes, this lane = 1) against ed_row_build / ec_row_build for the row base m B / m G:
// the number of entries that differ (byte-identical: the same field operations in the same order).
extern "C" int t_row_parked_cmp(int family, uint32_t m) {
  if (family == 2) {
    init();
    ge_p3 B, P;
    fe x, y, two_inv, t;
    fe_sub(x, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_add(y, g_C.Btab[1].ypx, g_C.Btab[1].ymx);
    fe_0(t);
    t.v[0] = 2;
    fe_invert(two_inv, t);
    fe_mul(B.X, x, two_inv);
    fe_mul(B.Y, y, two_inv);
    fe_1(B.Z);
    fe_mul(B.T, B.X, B.Y);
    ed_small_mul(P, B, m, g_C.d2);
    static ge_niels a[(EdRowsCfg<ED_W, ED_K>::kMult)], b[(EdRowsCfg<ED_W, ED_K>::kMult)];
    static fe zpre[(EdRowsCfg<ED_W, ED_K>::kMult)];
    static uint32_t park[3 * (EdRowsCfg<ED_W, ED_K>::kMult) * ED_PARK_DWORDS];
    ed_row_build<(EdRowsCfg<ED_W, ED_K>::kMult)>(a, P, g_C.d2, zpre);
    ed_row_build_parked<(EdRowsCfg<ED_W, ED_K>::kMult)>(b, P, g_C.d2, EdParkLanes{park, 1u, 3u});
    int bad = 0;
    for (int k = 0; k < (EdRowsCfg<ED_W, ED_K>::kMult); ++k) bad += memcmp(&a[k], &b[k], sizeof a[k]) != 0;
    return bad;
  }
  auto cmp = [&](auto tag) {
    constexpr int C = decltype(tag)::value;
    kinit();
    const EcConsts& K = g_K[C];
    Jac P;
    jac_small_mul_aff<C>(P, K.gx, K.gy, m, K);
    static EcAff a[EC_MULT], b[EC_MULT];
    static EcRowScratch s;
    static uint32_t park[3 * EC_MULT * EC_ROW_PARK];
    ec_row_build<C>(a, P, s, K);
    ec_row_build_parked<C>(b, P, EcRowParkLanes{park, 1u, 3u}, K);
    int bad = 0;
    for (int k = 0; k < EC_MULT; ++k) bad += memcmp(&a[k], &b[k], sizeof a[k]) != 0;
    return bad;
  };
  return family == CG_CURVE_R1 ? cmp(std::integral_constant<int, CG_CURVE_R1>())
                               : cmp(std::integral_constant<int, CG_CURVE_K1>());
}
