// Host build of the device lane code (corda_amd/csrc/*.h) with FE_BOUNDS_CHECK on, so the
// exact arithmetic the HIP kernels run is checked on the CPU against the oracle and every
// limb bound assumed by fe25519.h is asserted. Test infrastructure only.
#include <stdint.h>
#include <string.h>

#include "../../corda_amd/csrc/ed25519.h"

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
