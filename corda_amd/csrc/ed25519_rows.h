// Ed25519 double-scalar multiplication over per-key "row" tables, generic in the signed
// window width W and the number of windows K per row.
//
// A 253-bit scalar k is recoded into D = ceil(253 / W) + 1 signed radix-2^W digits
// e_t in [-2^(W-1), 2^(W-1)]. Digit t = K j + i belongs to row j and window i, so
//     [k] P = sum_{i<K} 2^{W i} sum_{j<R} e_{K j + i} P_j,   P_j = 2^{W K j} P.
// Each row stores the affine multiples 1..2^(W-1) of P_j (niels form, 120 B each). The loop
// runs K windows, (K-1) W doublings in total, and one mixed addition per digit. With W = 6,
// K = 4: 43 digits in 11 rows, 18 doublings, 86 mixed additions for h(-A) + S'B (the 4-bit
// 8-row layout needed 28 doublings and 128 additions). Every lane runs the same sequence:
// no data-dependent control flow, so the 64 lanes of a wave never diverge.
#pragma once
#include "ed25519.h"
#include "fe9.h"

// Product configuration (k_ed_keyprep_* / k_ed_ladder): -A rows of signed radix-2^6 digits in
// 2 windows (22 rows x 32 multiples per key, 6 doublings per item), B in signed radix 2^10
// over a constant table (26 rows x 512).
#define ED_W 6
#ifndef ED_K  // windows per row (A/B builds: 11 gives 4 rows and 60 doublings per item)
#define ED_K 2
#endif
#ifndef ED_WB
#define ED_WB 10
#endif

template <int W, int K>
struct EdRowsCfg {
  // the top digit keeps >= 1 bit of headroom for the recoding carry unless W divides 253
  static constexpr int kDigits = (253 + W - 1) / W + (253 % W == 0 ? 1 : 0);
  static constexpr int kRows = (kDigits + K - 1) / K;
  static constexpr int kMult = 1 << (W - 1);  // entries per row: 1 .. 2^(W-1)
  static constexpr int kPackedWords = (kDigits + 3) / 4;
};

template <int W, int K>
struct EdRowTabW {
  ge_niels t[EdRowsCfg<W, K>::kRows][EdRowsCfg<W, K>::kMult];
};

// signed radix-2^W digits of a < 2^253, packed 4 per word as signed bytes
template <int W>
CG_HD void sc_recode_w(uint32_t* packed, int nwords, const uint32_t a[8]) {
  constexpr int D = (253 + W - 1) / W + (253 % W == 0 ? 1 : 0);
  for (int w = 0; w < nwords; ++w) packed[w] = 0;
  int carry = 0;
#pragma unroll
  for (int t = 0; t < D; ++t) {
    const int bit = t * W;
    uint32_t v = 0;
    if (bit < 256) {
      const int wi = bit >> 5, sh = bit & 31;
      uint64_t x = (uint64_t)a[wi] >> sh;
      if (sh + W > 32 && wi + 1 < 8) x |= (uint64_t)a[wi + 1] << (32 - sh);
      v = (uint32_t)x & ((1u << W) - 1);
    }
    int e = (int)v + carry;
    carry = (e + (1 << (W - 1))) >> W;
    e -= carry << W;
    packed[t >> 2] |= ((uint32_t)(e & 0xff)) << ((t & 3) * 8);
  }
}

CG_HD int sc_digit_b(const uint32_t* packed, int t) {
  return (int)(int8_t)(uint8_t)(packed[t >> 2] >> ((t & 3) * 8));
}

// 2^n * P
CG_HD void ed_dbl_n(ge_p3& R, const ge_p3& P, int n) {
  ge_p2 q;
  ge_p1p1 t;
  ge_p3_to_p2(q, P);
  for (int i = 0; i < n - 1; ++i) {
    ge_p2_dbl(t, q);
    ge_p1p1_to_p2(q, t);
  }
  ge_p2_dbl(t, q);
  ge_p1p1_to_p3(R, t);
}

// Affine niels multiples 1..M of P (M a multiple of 8), normalised in groups of 8.
template <int M>
CG_HD void ed_row_multiples(ge_niels* row, const ge_p3& P, const fe& d2) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p3 cur = P;
  ge_p1p1 t;
  for (int g = 0; g < M / 8; ++g) {
    ge_p3 pts[8];
    for (int k = 0; k < 8; ++k) {
      if (g == 0 && k == 0) {
        pts[0] = P;
      } else {
        ge_add_cached(t, cur, c);
        ge_p1p1_to_p3(pts[k], t);
      }
      cur = pts[k];
    }
    ed_niels_batch8(row + 8 * g, pts, d2);
  }
}

// Affine niels multiples 1..M of P with ONE field inversion per row (Montgomery's trick over
// the whole row): the forward pass leaves each multiple's projective X, Y, Z in its own niels
// slot (the row is its own scratch) and the running Z prefix products in zpre[0..M-1]; the
// backward pass turns 1 / (Z_0 ... Z_{M-1}) into every 1/Z_k. ~23 field ops per entry
// instead of ~52 for batches of 8.
template <int M>
CG_HD void ed_multiples_from(ge_niels* row, const ge_p3& first, const ge_p3& P, const fe& d2, fe* zpre);
template <int M>
CG_HD void ed_row_build(ge_niels* row, const ge_p3& P, const fe& d2, fe* zpre) {
  ed_multiples_from<M>(row, P, P, d2, zpre);
}

// The affine niels points first + k P, k = 0..M-1, one inversion (ed_row_build's passes).
// Forward pass: projective X, Y, Z of each point wait in its niels slot, the running Z products in
// zpre[0..M-1] (zpre[M-1] = the product of all M). Backward pass: from inv = 1 / zpre[M-1], every
// 1 / Z_k, then the niels form. The wide-table build runs the passes as separate kernels with
// one shared inversion per row between them (verify_ed.hip).
template <int M>
CG_HD void ed_multiples_fwd(ge_niels* row, const ge_p3& first, const ge_p3& P, const fe& d2, fe* zpre) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p3 cur = first;
  ge_p1p1 t;
  fe run;
  for (int k = 0; k < M; ++k) {
    if (k != 0) {
      ge_add_cached(t, cur, c);
      ge_p1p1_to_p3(cur, t);
    }
    ge_niels& s = row[k];
    fe_copy(s.ypx, cur.X);
    fe_copy(s.ymx, cur.Y);
    fe_copy(s.xy2d, cur.Z);
    if (k == 0) {
      fe_copy(run, cur.Z);
    } else {
      fe_mul(run, run, cur.Z);
    }
    fe_copy(zpre[k], run);
  }
}

template <int M>
CG_HD void ed_multiples_bwd(ge_niels* row, const fe& inv_all, const fe* zpre, const fe& d2) {
  fe inv;
  fe_copy(inv, inv_all);
  for (int k = M - 1; k >= 0; --k) {
    ge_niels& s = row[k];
    fe zi;
    if (k > 0) {
      fe_mul(zi, inv, zpre[k - 1]);
      fe_mul(inv, inv, s.xy2d);
    } else {
      fe_copy(zi, inv);
    }
    fe x, y, xy;
    fe_mul(x, s.ypx, zi);
    fe_mul(y, s.ymx, zi);
    fe_add(s.ypx, y, x);
    fe_carry(s.ypx);
    fe_sub(s.ymx, y, x);
    fe_carry(s.ymx);
    fe_mul(xy, x, y);
    fe_mul(s.xy2d, xy, d2);
  }
}

template <int M>
CG_HD void ed_multiples_from(ge_niels* row, const ge_p3& first, const ge_p3& P, const fe& d2, fe* zpre) {
  ed_multiples_fwd<M>(row, first, P, d2, zpre);
  fe inv;
  fe_invert(inv, zpre[M - 1]);
  ed_multiples_bwd<M>(row, inv, zpre, d2);
}

// Inverses of G group products t_g (one inversion, Montgomery's trick): out[g] = 1 / t_g.
template <int G>
CG_HD void fe_batch_invert_small(fe* out, const fe* t) {
  fe pre[G];
  fe_copy(pre[0], t[0]);
  for (int g = 1; g < G; ++g) fe_mul(pre[g], pre[g - 1], t[g]);
  fe inv;
  fe_invert(inv, pre[G - 1]);
  for (int g = G - 1; g > 0; --g) {
    fe_mul(out[g], inv, pre[g - 1]);
    fe_mul(inv, inv, t[g]);
  }
  fe_copy(out[0], inv);
}

template <int W, int K>
CG_HD void ed_rows_w_init(EdRowTabW<W, K>& T, const ge_p3& P, const fe& d2) {
  typedef EdRowsCfg<W, K> C;
  ge_p3 Pj = P;
  for (int j = 0; j < C::kRows; ++j) {
    fe zpre[C::kMult];
    ed_row_build<C::kMult>(T.t[j], Pj, d2, zpre);
    if (j + 1 < C::kRows) ed_dbl_n(Pj, Pj, W * K);
  }
}

// entry |d| of a row (d in [-M, M]) with sign; 0 gives the identity
CG_HD void ed_pick_w(ge_niels& out, const ge_niels* row, int d) {
  const int a = d < 0 ? -d : d;
  out = row[a > 0 ? a - 1 : 0];
  if (a == 0) ge_niels_identity(out);
  ge_niels_cneg(out, d < 0);
}

// R' = h*(-A) + S'*B (digits already recoded), left projective.
template <int W, int K, class RowA, class RowB>
CG_HD void ed_double_scalar_w(ge_p2& out, const uint32_t* eh, const uint32_t* es, const RowA& TA, const RowB& TB) {
  typedef EdRowsCfg<W, K> C;
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  bool have_q = false;
  for (int i = K - 1; i >= 0; --i) {
    if (i != K - 1) {
      ge_p3_to_p2(q, R);
      for (int d = 0; d < W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    for (int j = 0; j < C::kRows; ++j) {
      const int tdig = K * j + i;
      if (tdig >= C::kDigits) continue;
      ge_niels n;
      ed_pick_w(n, TA.t[j], sc_digit_b(eh, tdig));
      ge_madd(t, R, n);
      ge_p1p1_to_p3(R, t);
      ed_pick_w(n, TB.t[j], sc_digit_b(es, tdig));
      ge_madd(t, R, n);
      const bool last = (i == 0) && (j + 1 == C::kRows);
      if (last) {
        ge_p1p1_to_p2(q, t);
        have_q = true;
      } else {
        ge_p1p1_to_p3(R, t);
      }
    }
  }
  if (!have_q) ge_p3_to_p2(q, R);
  out = q;
}

// ---------------------------------------------------------------- wide-radix B table
// S' B with signed radix-2^WB digits (WB > W): the B table is shared by every key, so it can
// be larger than the per-key tables (it lives in global memory, L2-resident; WB = 10 is
// 26 rows x 512 niels = 1.6 MB). B digit u is added in window i_u = floor(u K / NB), where it
// still gets doubled 6 i_u more times, so row u holds d * 2^(WB u - W i_u) * B.
// With W = 6, K = 4, WB = 10: 43 + 26 = 69 mixed additions instead of 86.
template <int W, int K, int WB>
struct EdBCfg {
  static constexpr int kDigits = (253 + WB - 1) / WB + (253 % WB == 0 ? 1 : 0);
  static constexpr int kMult = 1 << (WB - 1);
  static constexpr int kPackedWords = (kDigits + 1) / 2;  // int16 digits, 2 per word
  static constexpr int window(int u) { return (u * K) / kDigits; }
  static constexpr int shift(int u) { return WB * u - W * window(u); }  // row scale 2^shift
};

template <int W, int K, int WB>
struct EdBTabW {
  ge_niels t[EdBCfg<W, K, WB>::kDigits][EdBCfg<W, K, WB>::kMult];
};

// signed radix-2^WB digits of a < 2^253, packed 2 per word as int16
template <int WB>
CG_HD void sc_recode_w16(uint32_t* packed, int nwords, const uint32_t a[8]) {
  constexpr int D = (253 + WB - 1) / WB + (253 % WB == 0 ? 1 : 0);
  for (int w = 0; w < nwords; ++w) packed[w] = 0;
  int carry = 0;
#pragma unroll
  for (int t = 0; t < D; ++t) {
    const int bit = t * WB;
    uint32_t v = 0;
    if (bit < 256) {
      const int wi = bit >> 5, sh = bit & 31;
      uint64_t x = (uint64_t)a[wi] >> sh;
      if (sh + WB > 32 && wi + 1 < 8) x |= (uint64_t)a[wi + 1] << (32 - sh);
      v = (uint32_t)x & ((1u << WB) - 1);
    }
    int e = (int)v + carry;
    carry = (e + (1 << (WB - 1))) >> WB;
    e -= carry << WB;
    packed[t >> 1] |= ((uint32_t)(e & 0xffff)) << ((t & 1) * 16);
  }
}

CG_HD int sc_digit_h(const uint32_t* packed, int t) {
  return (int)(int16_t)(uint16_t)(packed[t >> 1] >> ((t & 1) * 16));
}

// signed radix-2^WB digits packed in Bits-bit slots (16: two per word, 32: one per word)
template <int WB, int Bits>
CG_HD void sc_recode_wb(uint32_t* packed, int nwords, const uint32_t a[8]) {
  if (Bits == 16) {
    sc_recode_w16<WB>(packed, nwords, a);
    return;
  }
  constexpr int D = (253 + WB - 1) / WB + (253 % WB == 0 ? 1 : 0);
  int carry = 0;
#pragma unroll
  for (int t = 0; t < D; ++t) {
    const int bit = t * WB;
    uint32_t v = 0;
    if (bit < 256) {
      const int wi = bit >> 5, sh = bit & 31;
      uint64_t x = (uint64_t)a[wi] >> sh;
      if (sh + WB > 32 && wi + 1 < 8) x |= (uint64_t)a[wi + 1] << (32 - sh);
      v = (uint32_t)x & ((1u << WB) - 1);
    }
    int e = (int)v + carry;
    carry = (e + (1 << (WB - 1))) >> WB;
    e -= carry << WB;
    packed[t] = (uint32_t)e;
  }
  for (int w = D; w < nwords; ++w) packed[w] = 0;
}
template <int Bits>
CG_HD int sc_digit_at(const uint32_t* packed, int t) {
  return Bits == 16 ? sc_digit_h(packed, t) : (int)packed[t];
}

// R' = h (-A) + S' B: A over the per-key W/K rows, B over the WB table; left projective.
// `Pick(out, row, digit)` loads a signed niels entry (identity for 0) from either table.
// Signed = true: entries are picked by |digit| and the sign goes through ge_madd_signed (the
// form k_ed_ladder_pf runs; the host tests run it with bounds checks).
template <int W, int K, int WB, bool Signed = false, class RowA, class TabB, class PickA, class PickB>
CG_HD void ed_double_scalar_wb(ge_p2& out, const uint32_t* eh, const uint32_t* esb, const RowA& TA, const TabB& TB,
                               PickA pick_a, PickB pick_b) {
  typedef EdRowsCfg<W, K> C;
  typedef EdBCfg<W, K, WB> CB;
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int i = K - 1; i >= 0; --i) {
    if (i != K - 1) {  // R arrives as p2 (q) from the previous window's last addition
      for (int d = 0; d < W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    const int u_lo = (i * CB::kDigits + K - 1) / K, u_hi = ((i + 1) * CB::kDigits + K - 1) / K;
    const int n_a = (C::kDigits - i + K - 1) / K;  // rows with a digit in this window
    const int n_ops = n_a + (u_hi - u_lo);
    for (int k = 0; k < n_ops; ++k) {
      ge_niels n;
      const int dg = k < n_a ? sc_digit_b(eh, K * k + i) : sc_digit_h(esb, u_lo + k - n_a);
      const int dp = Signed && dg < 0 ? -dg : dg;
      if (k < n_a) {
        pick_a(n, TA.t[k], dp);
      } else {
        pick_b(n, TB.t[u_lo + k - n_a], dp);
      }
      if (Signed) {
        ge_madd_signed(t, R, n, dg < 0);
      } else {
        ge_madd(t, R, n);
      }
      if (k + 1 == n_ops) {
        ge_p1p1_to_p2(q, t);  // next: doublings (or the end), which need no T
      } else {
        ge_p1p1_to_p3(R, t);
      }
    }
  }
  out = q;
}

// R' = h (-A) + S' B for a key that has only row 0 of its table (a key with few items in the
// batch, keyws.h): Horner over h's signed radix-2^W digits, W doublings between digits (252 in
// all), each B row added at the digit position whose remaining doublings its row scale
// expects (digit position i_u = EdBCfg::window(u) < K is followed by W i_u doublings, as in
// ed_double_scalar_wb). Same digits, same B table, same result.
template <int W, int K, int WB, class TabB, class PickA, class PickB>
CG_HD void ed_double_scalar_row0(ge_p2& out, const uint32_t* eh, const uint32_t* esb, const ge_niels* row0,
                                 const TabB& TB, PickA pick_a, PickB pick_b) {
  typedef EdRowsCfg<W, K> C;
  typedef EdBCfg<W, K, WB> CB;
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int td = C::kDigits - 1; td >= 0; --td) {
    if (td != C::kDigits - 1) {
      for (int d = 0; d < W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    const int u_lo = td < K ? (td * CB::kDigits + K - 1) / K : 0;
    const int u_hi = td < K ? ((td + 1) * CB::kDigits + K - 1) / K : 0;
    const int n_ops = 1 + (u_hi - u_lo);
    for (int k = 0; k < n_ops; ++k) {
      ge_niels n;
      if (k == 0) {
        pick_a(n, row0, sc_digit_b(eh, td));
      } else {
        pick_b(n, TB.t[u_lo + k - 1], sc_digit_h(esb, u_lo + k - 1));
      }
      ge_madd(t, R, n);
      if (k + 1 == n_ops) {
        ge_p1p1_to_p2(q, t);
      } else {
        ge_p1p1_to_p3(R, t);
      }
    }
  }
  out = q;
}

// Table rows: row u holds the affine multiples 1..kMult of 2^shift(u) B.
template <int W, int K, int WB>
CG_HD void ed_btab_wb_row(ge_niels* row, const ge_p3& B, int u, const fe& d2) {
  typedef EdBCfg<W, K, WB> CB;
  ge_p3 P = B;
  if (CB::shift(u) > 0) ed_dbl_n(P, P, CB::shift(u));
  ed_row_multiples<CB::kMult>(row, P, d2);
}

// ---------------------------------------------------------------- wide tables (hot keys)
// A key with many items in the call (keyws.h KEY_WIDE_MIN_USES) gets one row per signed
// radix-2^8 digit of h: row j holds the affine multiples 1..128 of 2^{8j} (-A) (32 rows,
// 491 520 B). B gets one row per signed radix-2^22 digit of S' over a constant table built once
// per context (row u holds 1..2^21 times 2^{22u} B: 12 rows, 3.0 GB in HBM). R' = sum of one entry
// per row: 32 + 12 = 44 mixed additions and no doublings, against 69 additions + 6 doublings over
// the full tables. (B radix 2^12 / 2^16 / 2^20 took 22 / 16 / 13 additions; the per-op LDS
// prefetch hides the HBM gathers of the 3 GB table: ecdsa_rows.h has the A/B.)
#define ED_WIDE_W 8
#ifndef ED_WIDE_BW
#define ED_WIDE_BW 26
#endif
struct EdWideCfg {
  static constexpr int kDigits = (253 + ED_WIDE_W - 1) / ED_WIDE_W;  // 32: h < 2^253 leaves the carry room
  static constexpr int kRows = kDigits;
  static constexpr int kMult = 1 << (ED_WIDE_W - 1);                 // 128
  static constexpr int kPackedWords = (kDigits + 3) / 4;             // int8 digits
  static constexpr int kBDigits = (253 + ED_WIDE_BW - 1) / ED_WIDE_BW;  // 12 at radix 2^22
  static constexpr int kBMult = 1 << (ED_WIDE_BW - 1);                // |digit| <= 2^(BW-1)
  static constexpr int kBBits = ED_WIDE_BW <= 16 ? 16 : 32;           // B digit slot: int16 or int32
  static constexpr int kBPackedWords = (kBDigits * kBBits + 31) / 32;
  static constexpr int kOps = kRows + kBDigits;                       // 44 at radix 2^22
};
static_assert(253 % ED_WIDE_W != 0 && 253 % ED_WIDE_BW != 0, "the top digit keeps headroom for the carry");

// Both wide tables hold half-scaled niels entries ((y+x)/2, (y-x)/2, x y d), added with
// ge_madd_half_signed (no doubling of Z and no carry pass per addition); digit 0 adds the
// half-scaled identity (ge_niels_identity_half).
// Entries in the radix-2^29 form (fe9.h: the wide ladders run in it), 112 B each.
struct EdWideTab {
  ge9_niels t[EdWideCfg::kRows][EdWideCfg::kMult];  // t[j][k-1] = k 2^{8j} (-A), half-scaled
};
struct EdBWideTab {
  ge9_niels t[EdWideCfg::kBDigits][EdWideCfg::kBMult];  // t[u][k-1] = k 2^{ED_WIDE_BW u} B, half-scaled
  // the half-scaled identity, gathered for a zero digit of either table: a select of constants in
  // the ladder let the compiler specialise the products on it (64 x 32-bit multiplies, ~+40% VALU)
  ge9_niels ident;
};

// R' = h (-A) + S' B over the wide tables, digits already recoded (eh: radix 2^8, esb: radix
// 2^ED_WIDE_BW): 44 signed mixed additions in the radix-2^29 arithmetic (fe9.h), entries by |digit|
// (digit 0 adds the half-scaled identity), the sign through ge9_madd_half: the form k_ed_ladder_wide
// runs.
CG_HD void ed_double_scalar_wide(ge_p2& out, const uint32_t* eh, const uint32_t* esb, const EdWideTab& TA,
                                 const EdBWideTab& TB) {
  auto entry = [&](int o, bool& neg) -> ge9_niels {
    const bool is_b = o >= EdWideCfg::kRows;
    const int dg = is_b ? sc_digit_at<EdWideCfg::kBBits>(esb, o - EdWideCfg::kRows) : sc_digit_b(eh, o);
    const int dp = dg < 0 ? -dg : dg;
    neg = dg < 0;
    return dp == 0 ? TB.ident : is_b ? TB.t[o - EdWideCfg::kRows][dp - 1] : TA.t[o][dp - 1];
  };
  ge9_p3 R;
  bool n0;
  const ge9_niels q0 = entry(0, n0);
#if ED_SIGN_FOLD
  // the running point is s_o R (fe9.h ge9_madd_half_flip): op o adds the stored entry of |digit|
  // and flips its output by s_o s_{o+1}; the last op by s_{N-1} alone
  bool n1;
  ge9_niels q = entry(1, n1);
  ge9_from_niels_half(R, q0, n0 != n1);
  for (int o = 1; o < EdWideCfg::kOps; ++o) {
    bool nn = false;
    const ge9_niels qn = o + 1 < EdWideCfg::kOps ? entry(o + 1, nn) : q;
    if (o + 1 < EdWideCfg::kOps) ge9_madd_half_flip<true>(R, R, q, n1 != nn);
    else ge9_madd_half_flip<false>(R, R, q, n1);
    q = qn;
    n1 = nn;
  }
#else
  ge9_from_niels_half(R, q0, n0);  // identity + q0: one product, not seven
  for (int o = 1; o < EdWideCfg::kOps; ++o) {
    bool neg;
    const ge9_niels n = entry(o, neg);
    if (o + 1 < EdWideCfg::kOps) ge9_madd_half<true>(R, R, n, neg);
    else ge9_madd_half<false>(R, R, n, neg);
  }
#endif
  ge9_to_p2(out, R);
}

// m * P for a small m >= 1 (double-and-add, MSB first)
CG_HD void ed_small_mul(ge_p3& R, const ge_p3& P, uint32_t m, const fe& d2) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  R = P;
  ge_p1p1 t;
  int top = 31 - __builtin_clz(m);
  for (int b = top - 1; b >= 0; --b) {
    ge_p3_dbl(t, R);
    ge_p1p1_to_p3(R, t);
    if ((m >> b) & 1u) {
      ge_add_cached(t, R, c);
      ge_p1p1_to_p3(R, t);
    }
  }
}

// Wide B row u, multiples 8 grp + 1 .. 8 grp + 8 of 2^{ED_WIDE_BW u} B (one lane of the
// per-context build k_ed_bwide_init; the host tests build the groups their digits touch).
template <class Out>
CG_HD void ed_bwide_group(Out* out8, const ge_p3& B, int u, int grp, const fe& d2) {
  ge_p3 P = B;
  if (u > 0) ed_dbl_n(P, P, ED_WIDE_BW * u);
  ge_p3 pts[8];
  ed_small_mul(pts[0], P, 8u * (uint32_t)grp + 1u, d2);
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p1p1 t;
  for (int k = 1; k < 8; ++k) {
    ge_add_cached(t, pts[k - 1], c);
    ge_p1p1_to_p3(pts[k], t);
  }
  ge_niels n8[8];
  ed_niels_batch8<true>(n8, pts, d2);
  for (int k = 0; k < 8; ++k) ed_niels_store(out8 + k, n8[k]);
}

// ---------------------------------------------------------------- wide-table build
// One lane per (wide key, row j, group g of ED_WIDE_GROUP = 32 consecutive multiples of the row base
// P), in chunks of ED_WIDE_CHUNK = 2: pass 1 walks the group by additions and stores only each
// chunk's Z product (16 per lane); pass 2 batch-inverts a row's 64 chunk products (one lane per row);
// pass 3 walks the group again, keeping a chunk's points in VGPRs, and writes its normalised niels
// entries (240 contiguous bytes; chunks of 4 spilled at 256 VGPRs). The three-pass form that stored every multiple's projective X, Y, Z
// and running product in memory between passes moved ~1 KB of uncoalesced traffic per entry (12.6 +
// 4.2 GB per headline call, profiles/r02/p3/pmc_traffic.json) and stalled the challenge hashes and
// ECDSA fronts sharing the chip with it; this form moves ~130 B per entry.
#define ED_WIDE_GROUP 32
#define ED_WIDE_GROUPS (EdWideCfg::kMult / ED_WIDE_GROUP)  // 4 group lanes per row
#define ED_WIDE_CHUNK 2
#define ED_WIDE_CHUNKS (EdWideCfg::kMult / ED_WIDE_CHUNK)  // 64 chunk products per row

// the chunk's niels entries from zinv = 1 / (Z_0 Z_1) (straight-line: a loop here was left rolled
// and put the points in scratch)
static_assert(ED_WIDE_CHUNK == 2, "ed_wide_chunk_out is written for chunks of 2");
// zi = 1 / (2 Z) and d4 = 4d give the half-scaled entry
CG_HD void ed_niels_from(ge_niels& n, const ge_p2& p, const fe& zi, const fe& d4) {
  fe x, y, xy;
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(n.ypx, y, x);
  fe_carry(n.ypx);
  fe_sub(n.ymx, y, x);
  fe_carry(n.ymx);
  fe_mul(xy, x, y);
  fe_mul(n.xy2d, xy, d4);
}
// zinv = 1 / (2 Z_0 Z_1) (fe_invert_run's 1/2 included)
template <class Out>
CG_HD void ed_wide_chunk_out(Out* out, const ge_p2 pts[ED_WIDE_CHUNK], const fe& zinv, const fe& d2) {
  fe z1i, z0i, d4;
  fe_add(d4, d2, d2);
  fe_carry(d4);
  fe_mul(z1i, zinv, pts[0].Z);  // 1 / Z_1
  fe_mul(z0i, zinv, pts[1].Z);  // 1 / Z_0
  ge_niels n0, n1;
  ed_niels_from(n0, pts[0], z0i, d4);
  ed_niels_from(n1, pts[1], z1i, d4);
  ed_niels_store(out, n0);
  ed_niels_store(out + 1, n1);
}

// Pass 1 (Out = false): zc[c] = chunk c's Z product. Pass 3 (Out = true): the group's 32 entries
// into out[0..31] from the inverted chunk products zc[c].
template <bool Out, class OutT = ge_niels>
CG_HD void ed_wide_group_pass(OutT* out, fe* zc, const ge_p3& P, int g, const fe& d2) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p3 R;
  ed_small_mul(R, P, (uint32_t)(ED_WIDE_GROUP * g + 1), d2);
  ge_p1p1 t;
#pragma unroll 1
  for (int ch = 0; ch < ED_WIDE_GROUP / ED_WIDE_CHUNK; ++ch) {
    ge_p2 pts[ED_WIDE_CHUNK];
    fe zp;
    if (ch > 0) {  // the chunk's first point: one addition past the previous chunk's last
      ge_add_cached(t, R, c);
      ge_p1p1_to_p3(R, t);
    }
    if (Out) ge_p3_to_p2(pts[0], R);
    else fe_copy(zp, R.Z);
#pragma unroll
    for (int k = 1; k < ED_WIDE_CHUNK; ++k) {
      ge_add_cached(t, R, c);
      ge_p1p1_to_p3(R, t);
      if (Out) ge_p3_to_p2(pts[k], R);
      else fe_mul(zp, zp, R.Z);
    }
    if (Out) ed_wide_chunk_out(out + ED_WIDE_CHUNK * ch, pts, zc[ch], d2);
    else fe_copy(zc[ch], zp);
  }
}

// in place: z[g] <- 1 / (2 z[g]) for the NG products of one row (prefix products in pre[]); the 1/2
// rides on the single inversion and reaches every z[g] once (half-scaled entries)
template <int NG>
CG_HD void fe_invert_run(fe* z, fe* pre) {
  fe run;
  fe_copy(run, z[0]);
  fe_copy(pre[0], run);
  for (int g = 1; g < NG; ++g) {
    fe_mul(run, run, z[g]);
    fe_copy(pre[g], run);
  }
  fe inv, h;
  fe_invert(inv, run);
  fe_half(h);
  fe_mul(inv, inv, h);
  for (int g = NG - 1; g > 0; --g) {
    fe zg, t;
    fe_copy(zg, z[g]);
    fe_mul(t, inv, pre[g - 1]);
    fe_copy(z[g], t);
    fe_mul(inv, inv, zg);
  }
  fe_copy(z[0], inv);
}

// Wide-table row in one lane (round 3): R walks the row's 128 multiples k P by cached additions,
// each multiple's X, Y, Z parked in its output entry and the running Z product in pre[k]; one
// inversion (with the 1/2 of the half-scaled entries), then the walk back writes the normalised
// entries (zi = inv pre[k-1], inv <- inv Z_k, four products per entry). ~15 products per entry
// against the three-pass form's ~30 (no group-start scalar multiplications, nothing walked
// twice), and one launch instead of three.
// Where a row lane parks its multiples between the walks (k = entry index relative to the lane's
// first): EdParkRow in the row's own entries + pre[] (host build), EdParkLanes lane-interleaved
// (the device build, keyws.h EdWideSlot::park).
#define ED_PARK_DWORDS 40  // X, Y, Z and the running product: 4 x 10 limbs
struct EdParkRow {  // host build: X, Y, Z and the running product in four arrays of fe
  fe *x, *y, *z, *pre;
  CG_HDM void put(int k, const fe& X, const fe& Y, const fe& Z, const fe& run) const {
    x[k] = X;
    y[k] = Y;
    z[k] = Z;
    pre[k] = run;
  }
  CG_HDM void get(int k, fe& X, fe& Y, fe& Z) const {
    X = x[k];
    Y = y[k];
    Z = z[k];
  }
  CG_HDM void get_run(int k, fe& run) const { run = pre[k]; }
};
struct EdParkLanes {
  uint32_t* base;
  uint32_t lane, lanes;
  CG_HDM void st(int k, int q, const fe& f) const {
    uint32_t* p = base + (size_t)(k * ED_PARK_DWORDS + q * 10) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 10; ++d) p[(size_t)d * lanes] = f.v[d];
  }
  CG_HDM void ld(int k, int q, fe& f) const {
    const uint32_t* p = base + (size_t)(k * ED_PARK_DWORDS + q * 10) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 10; ++d) f.v[d] = p[(size_t)d * lanes];
  }
  CG_HDM void put(int k, const fe& X, const fe& Y, const fe& Z, const fe& run) const {
    st(k, 0, X);
    st(k, 1, Y);
    st(k, 2, Z);
    st(k, 3, run);
  }
  CG_HDM void get(int k, fe& X, fe& Y, fe& Z) const {
    ld(k, 0, X);
    ld(k, 1, Y);
    ld(k, 2, Z);
  }
  CG_HDM void get_run(int k, fe& run) const { ld(k, 3, run); }
};

// Entries [e0, e1) (entry k = (k + 1) P); a lane not starting at 0 starts by a scalar multiplication.
template <class Park, class Out>
CG_HD void ed_wide_row_build(Out* out, const Park& pk, const ge_p3& P, int e0, int e1, const fe& d2) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p3 R;
  if (e0 == 0) R = P;
  else ed_small_mul(R, P, (uint32_t)e0 + 1u, d2);
  fe run;
#pragma unroll 1
  for (int k = e0; k < e1; ++k) {
    if (k > e0) {
      ge_p1p1 t;
      ge_add_cached(t, R, c);
      ge_p1p1_to_p3(R, t);
      fe_mul(run, run, R.Z);
    } else {
      fe_copy(run, R.Z);
    }
    pk.put(k - e0, R.X, R.Y, R.Z, run);  // un-normalised until the walk back
  }
  fe inv, h, d4;
  fe_invert(inv, run);
  fe_half(h);
  fe_mul(inv, inv, h);  // 1 / (2 Z_e0 .. Z_e1-1): the half-scaled entries' 1/2
  fe_add(d4, d2, d2);
  fe_carry(d4);
#ifndef ED_ROWS_PREFETCH  // 1: the walk back loads each entry's parked values one entry ahead
#define ED_ROWS_PREFETCH 1
#endif
#if ED_ROWS_PREFETCH
  fe X, Y, Z, pr;
  pk.get(e1 - 1 - e0, X, Y, Z);
  if (e1 - 1 > e0) pk.get_run(e1 - 2 - e0, pr);
#pragma unroll 1
  for (int k = e1 - 1; k >= e0; --k) {
    fe Xn = X, Yn = Y, Zn = Z, prn = pr;
    if (k > e0) {
      pk.get(k - 1 - e0, Xn, Yn, Zn);
      if (k - 1 > e0) pk.get_run(k - 2 - e0, prn);
    }
#else  // parked lane-interleaved, the loads are coalesced: no prefetch registers (occupancy)
#pragma unroll 1
  for (int k = e1 - 1; k >= e0; --k) {
    fe X, Y, Z, pr;
    pk.get(k - e0, X, Y, Z);
    if (k > e0) pk.get_run(k - 1 - e0, pr);
#endif
    ge_p2 p;
    p.X = X;
    p.Y = Y;
    fe zi;
    if (k > e0) {
      fe_mul(zi, inv, pr);
      fe_mul(inv, inv, Z);
    } else {
      fe_copy(zi, inv);
    }
    ge_niels n;
    ed_niels_from(n, p, zi, d4);
    ed_niels_store(out + k, n);
#if ED_ROWS_PREFETCH
    X = Xn;
    Y = Yn;
    Z = Zn;
    pr = prn;
#endif
  }
}

// ed_wide_row_build in the radix-2^29 arithmetic (fe9.h), the form k_ed_wide_rows runs (round 4):
// the walk R += P by the cached addition in fe9 (every product's operand classes: A = (Y1+X1)(y+x)
// uu A2 x T, B = (Y1-X1)(y-x) ss S x T, C = T1 2dT uu T x T, D = Z1 2Z uu T x T; E = A - B (S),
// H = A + B (A2), G = D + C (A2), F = D + 128p - C (V); X3 = E F ss S x V, Y3 = G H uu A2 x A2,
// Z3 = G F uu A2 x V, T3 = E H ss S x A2), the cached P, 1/(2 Z) and 4d made tight once per lane
// in radix 2^25.5, the entries' sums carried to tight limbs (fe9_carry). The same entries as
// ed_wide_row_build, equal mod p (test_ed_wide_row_build9_matches).
#define ED_PARK9_DWORDS 36  // X, Y, Z and the running product: 4 x 9 limbs
struct EdPark9Lanes {
  uint32_t* base;
  uint32_t lane, lanes;
  CG_HDM void st(int k, int q, const fe9& f) const {
    uint32_t* p = base + (size_t)(k * ED_PARK9_DWORDS + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) p[(size_t)d * lanes] = f.v[d];
  }
  CG_HDM void ld(int k, int q, fe9& f) const {
    const uint32_t* p = base + (size_t)(k * ED_PARK9_DWORDS + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) f.v[d] = p[(size_t)d * lanes];
  }
};
// FE9_ROWS_ILP (round 6, A/B): the row walk's products without the ladders' opaque column chains
// (fe9_mul Pin = false): one lane per row, 2 waves per SIMD, every entry dependent on the previous
// one -- latency-bound, so the products' own instruction-level parallelism is what hides latency
#ifndef FE9_ROWS_ILP
#define FE9_ROWS_ILP 0
#endif
#define FE9_ROWS_PIN (!FE9_ROWS_ILP)
template <class Park>
CG_HD void ed_wide_row_build9(ge9_niels* out, const Park& pk, const ge_p3& P, int e0, int e1, const fe& d2) {
  fe9 cYpX, cYmX, cZ2, cT2d, d4;
  {  // the cached P and 4d, tight
    fe t;
    fe_add(t, P.Y, P.X);
    fe_carry(t);
    fe9_from_fe(cYpX, t);
    fe_sub(t, P.Y, P.X);
    fe_carry(t);
    fe9_from_fe(cYmX, t);
    fe_add(t, P.Z, P.Z);
    fe_carry(t);
    fe9_from_fe(cZ2, t);
    fe_mul(t, P.T, d2);
    fe9_from_fe(cT2d, t);
    fe_add(t, d2, d2);
    fe_carry(t);
    fe9_from_fe(d4, t);
  }
  ge9_p3 R;
  {
    ge_p3 R0;
    if (e0 == 0) R0 = P;
    else ed_small_mul(R0, P, (uint32_t)e0 + 1u, d2);
    ge9_from_p3(R, R0);
  }
  fe9 run = R.Z;
#pragma unroll 1
  for (int k = e0; k < e1; ++k) {
    if (k > e0) {
      fe9 a, b, A, B, C, D, E, H, G, F;
      fe9_add(a, R.Y, R.X);
      fe9_sub(b, R.Y, R.X);
      fe9_mul<false, FE9_ROWS_PIN>(A, a, cYpX);
      fe9_mul<true, FE9_ROWS_PIN>(B, b, cYmX);
      fe9_mul<false, FE9_ROWS_PIN>(C, R.T, cT2d);
      fe9_mul<false, FE9_ROWS_PIN>(D, R.Z, cZ2);
      fe9_sub(E, A, B);
      fe9_add(H, A, B);
      fe9_add(G, D, C);
      fe9_subk(F, D, C);
      fe9_mul<true, FE9_ROWS_PIN>(R.X, E, F);
      fe9_mul<false, FE9_ROWS_PIN>(R.Y, G, H);
      fe9_mul<false, FE9_ROWS_PIN>(R.Z, G, F);
      fe9_mul<true, FE9_ROWS_PIN>(R.T, E, H);
      fe9_mul<false, FE9_ROWS_PIN>(run, run, R.Z);
    }
    const int i = k - e0;
    pk.st(i, 0, R.X);
    pk.st(i, 1, R.Y);
    pk.st(i, 2, R.Z);
    pk.st(i, 3, run);
  }
  fe9 inv;
  {  // 1 / (2 Z_e0 .. Z_e1-1): the half-scaled entries' 1/2, one inversion in radix 2^25.5
    fe r, h, t;
    fe_from_fe9(r, run);
    fe_invert(t, r);
    fe_half(h);
    fe_mul(r, t, h);
    fe9_from_fe(inv, r);
  }
#pragma unroll 1
  for (int k = e1 - 1; k >= e0; --k) {
    const int i = k - e0;
    fe9 X, Y, zi;
    pk.ld(i, 0, X);
    pk.ld(i, 1, Y);
    if (k > e0) {
      fe9 pr, Z;
      pk.ld(i - 1, 3, pr);
      pk.ld(i, 2, Z);
      fe9_mul<false, FE9_ROWS_PIN>(zi, inv, pr);
      fe9_mul<false, FE9_ROWS_PIN>(inv, inv, Z);
    } else {
      zi = inv;
    }
    fe9 x, y, s, xy;
    fe9_mul<false, FE9_ROWS_PIN>(x, X, zi);
    fe9_mul<false, FE9_ROWS_PIN>(y, Y, zi);
    ge9_niels n;
    fe9_add(s, y, x);
    fe9_carry(n.ypx, s);
    fe9_subk(s, y, x);
    fe9_carry(n.ymx, s);
    fe9_mul<false, FE9_ROWS_PIN>(xy, x, y);
    fe9_mul<false, FE9_ROWS_PIN>(n.xy2d, xy, d4);
    for (uint32_t& w : n.pad) w = 0;
    out[k] = n;
  }
}

// Full / row-0 row of plain niels multiples 1..M of P (ed_row_build's entries) with the walk parked
// in `pk` (EdParkLanes: lane-interleaved, so a wave's stores are coalesced; ed_row_build parks in
// the row's own entries, 64 cache lines per store of a wave: the 2^20-distinct-key leg's row-0
// builds took 108 ms per call, profiles/r04/kd). k_ed_keyprep_tab's form.
template <int M, class Park>
CG_HD void ed_row_build_parked(ge_niels* row, const ge_p3& P, const fe& d2, const Park& pk) {
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p3 R = P;
  fe run;
  fe_copy(run, R.Z);
  pk.put(0, R.X, R.Y, R.Z, run);
#pragma unroll 1
  for (int k = 1; k < M; ++k) {
    ge_p1p1 t;
    ge_add_cached(t, R, c);
    ge_p1p1_to_p3(R, t);
    fe_mul(run, run, R.Z);
    pk.put(k, R.X, R.Y, R.Z, run);
  }
  fe inv;
  fe_invert(inv, run);
#pragma unroll 1
  for (int k = M - 1; k >= 0; --k) {
    fe X, Y, Z, zi;
    pk.get(k, X, Y, Z);
    if (k > 0) {
      fe pr;
      pk.get_run(k - 1, pr);
      fe_mul(zi, inv, pr);
      fe_mul(inv, inv, Z);
    } else {
      fe_copy(zi, inv);
    }
    fe x, y, xy;
    ge_niels n;
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_add(n.ypx, y, x);
    fe_carry(n.ypx);
    fe_sub(n.ymx, y, x);
    fe_carry(n.ymx);
    fe_mul(xy, x, y);
    fe_mul(n.xy2d, xy, d2);
    row[k] = n;
  }
}

#ifndef ED_WIDE_ROW_LANES  // lanes per row (as EC_WIDE_ROW_LANES): 1 / 2 / 4 lanes, headline A/B in 3
#define ED_WIDE_ROW_LANES 1  // rounds: 314.2 / 311.5 / 311.1 M sigs/s (profiles/r04/erl; one inversion per row,
#endif                       // one round of 2 waves per SIMD for the 4 096 keys' 32 rows)
static_assert(EdWideCfg::kMult % ED_WIDE_ROW_LANES == 0, "row split");

// ---------------------------------------------------------------- full / row-0 tables + wide B
// R' = h (-A) + S' B for keys with full tables (W/K rows of -A, K windows, (K-1) W doublings) or
// row 0 only (Horner, 252 doublings), with S' B from the constant radix-2^ED_WIDE_BW table at the
// end: the B digits need no doublings, so they all go after the last window (12 additions instead
// of the 26 of the round-1 radix-2^10 table spread over the windows). `Signed`: entries by |digit|,
// the sign through ge_madd_signed / ge_madd_half_signed (the form k_ed_ladder_pf runs).
// S' B over the constant radix-2^ED_WIDE_BW table, in the radix-2^29 arithmetic of its entries
// (fe9.h): R (extended, radix 2^25.5) in, q (projective, radix 2^25.5) out. Entries by |digit|,
// the sign through ge9_madd_half.
CG_HD void ed_add_b_wide9(ge_p2& q, const ge_p3& R, const uint32_t* esb, const EdBWideTab& TB) {
  ge9_p3 R9;
  ge9_from_p3(R9, R);
  for (int u = 0; u < EdWideCfg::kBDigits; ++u) {
    const int dg = sc_digit_at<EdWideCfg::kBBits>(esb, u);
    const int dp = dg < 0 ? -dg : dg;
    const ge9_niels n = dp == 0 ? TB.ident : TB.t[u][dp - 1];
    if (u + 1 < EdWideCfg::kBDigits) ge9_madd_half<true>(R9, R9, n, dg < 0);
    else ge9_madd_half<false>(R9, R9, n, dg < 0);
  }
  ge9_to_p2(q, R9);
}

template <int W, int K, bool Signed = false, class RowA, class PickA, class PickB>
CG_HD void ed_double_scalar_fw(ge_p2& out, const uint32_t* eh, const uint32_t* esb, const RowA& TA,
                               const EdBWideTab& TB, PickA pick_a, PickB pick_b) {
  typedef EdRowsCfg<W, K> C;
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int i = K - 1; i >= 0; --i) {
    if (i != K - 1) {  // R arrives as p2 (q) from the previous window's last addition
      for (int d = 0; d < W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    const int n_a = (C::kDigits - i + K - 1) / K;  // rows with a digit in this window
    for (int k = 0; k < n_a; ++k) {
      const int dg = sc_digit_b(eh, K * k + i);
      const int dp = Signed && dg < 0 ? -dg : dg;
      ge_niels n;
      pick_a(n, TA.t[k], dp);
      if (Signed) ge_madd_signed(t, R, n, dg < 0);
      else ge_madd(t, R, n);
      if (i != 0 && k + 1 == n_a) ge_p1p1_to_p2(q, t);  // next: doublings, which need no T
      else ge_p1p1_to_p3(R, t);
    }
  }
  (void)pick_b;
  ed_add_b_wide9(q, R, esb, TB);
  out = q;
}

template <int W, int K, class PickA, class PickB>
CG_HD void ed_double_scalar_row0w(ge_p2& out, const uint32_t* eh, const uint32_t* esb, const ge_niels* row0,
                                  const EdBWideTab& TB, PickA pick_a, PickB pick_b) {
  typedef EdRowsCfg<W, K> C;
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int td = C::kDigits - 1; td >= 0; --td) {
    if (td != C::kDigits - 1) {
      for (int d = 0; d < W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    ge_niels n;
    pick_a(n, row0, sc_digit_b(eh, td));
    ge_madd(t, R, n);
    if (td != 0) ge_p1p1_to_p2(q, t);
    else ge_p1p1_to_p3(R, t);
  }
  (void)pick_b;
  ed_add_b_wide9(q, R, esb, TB);
  out = q;
}
