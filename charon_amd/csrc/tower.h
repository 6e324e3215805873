// Extension tower:  Fp2 = Fp[u]/(u^2+1),  Fp6 = Fp2[v]/(v^3 - xi) with xi = 1+u,
//                   Fp12 = Fp6[w]/(w^2 - v)   (so w^6 = xi; the G2 twist is M-type).
#pragma once
#include "fp.h"

namespace hb {

struct Fp2 {
  Fp c0, c1;
};
struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 c0, c1;
};

// ---------------------------------- Fp2 ----------------------------------
HD Fp2 f2_from_const(const uint32_t (*c)[12]) { return {fp_from_const(c[0]), fp_from_const(c[1])}; }
HD Fp2 f2_zero() { return {fp_zero(), fp_zero()}; }
HD Fp2 f2_one() { return {fp_one(), fp_zero()}; }
#if defined(__HIP_DEVICE_COMPILE__)
// Device: the two components' carry chains are interleaved (c0 and c1 sums, then their 2p
// corrections one limb behind), so consecutive dependent carry ops are 4 instructions apart
// and gfx950's carry-forwarding wait states need no s_nop.
HD Fp2 f2_add(const Fp2& a, const Fp2& b) {
  Fp s0, s1, d0, d1;
  unsigned c0 = 0, c1 = 0, e0 = 0, e1 = 0;
  s0.v[0] = __builtin_addc(a.c0.v[0], b.c0.v[0], c0, &c0);
  s1.v[0] = __builtin_addc(a.c1.v[0], b.c1.v[0], c1, &c1);
  HB_UNROLL for (int i = 1; i < NL; i++) {
    s0.v[i] = __builtin_addc(a.c0.v[i], b.c0.v[i], c0, &c0);
    s1.v[i] = __builtin_addc(a.c1.v[i], b.c1.v[i], c1, &c1);
    d0.v[i - 1] = __builtin_subc(s0.v[i - 1], P2_RAW[i - 1], e0, &e0);
    d1.v[i - 1] = __builtin_subc(s1.v[i - 1], P2_RAW[i - 1], e1, &e1);
  }
  d0.v[NL - 1] = __builtin_subc(s0.v[NL - 1], P2_RAW[NL - 1], e0, &e0);
  d1.v[NL - 1] = __builtin_subc(s1.v[NL - 1], P2_RAW[NL - 1], e1, &e1);
  Fp2 r;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.c0.v[i] = e0 ? s0.v[i] : d0.v[i];  // s < 2p: keep s
    r.c1.v[i] = e1 ? s1.v[i] : d1.v[i];
  }
  return r;
}
HD Fp2 f2_sub(const Fp2& a, const Fp2& b) {
  Fp s0, s1, d0, d1;
  unsigned c0 = 0, c1 = 0, e0 = 0, e1 = 0;
  s0.v[0] = __builtin_subc(a.c0.v[0], b.c0.v[0], c0, &c0);
  s1.v[0] = __builtin_subc(a.c1.v[0], b.c1.v[0], c1, &c1);
  HB_UNROLL for (int i = 1; i < NL; i++) {
    s0.v[i] = __builtin_subc(a.c0.v[i], b.c0.v[i], c0, &c0);
    s1.v[i] = __builtin_subc(a.c1.v[i], b.c1.v[i], c1, &c1);
    d0.v[i - 1] = __builtin_addc(s0.v[i - 1], P2_RAW[i - 1], e0, &e0);
    d1.v[i - 1] = __builtin_addc(s1.v[i - 1], P2_RAW[i - 1], e1, &e1);
  }
  d0.v[NL - 1] = __builtin_addc(s0.v[NL - 1], P2_RAW[NL - 1], e0, &e0);
  d1.v[NL - 1] = __builtin_addc(s1.v[NL - 1], P2_RAW[NL - 1], e1, &e1);
  Fp2 r;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.c0.v[i] = c0 ? d0.v[i] : s0.v[i];  // borrow: add 2p back
    r.c1.v[i] = c1 ? d1.v[i] : s1.v[i];
  }
  return r;
}
#else
HD Fp2 f2_add(const Fp2& a, const Fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
HD Fp2 f2_sub(const Fp2& a, const Fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
#endif
HD Fp2 f2_neg(const Fp2& a) { return f2_sub(f2_zero(), a); }
HD Fp2 f2_dbl(const Fp2& a) { return f2_add(a, a); }
HD Fp2 f2_conj(const Fp2& a) { return {a.c0, fp_neg(a.c1)}; }

// Fp2 product and square as single lazily reduced passes (fp.h fp2_mul_core / fp2_sqr_core).
// Counted as 3 and 2 Fp products, the unit of the op counts (charon_amd/opcounts.py).
HD Fp2 f2_mul(const Fp2& a, const Fp2& b) {
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  Fp2 r;
  fp2_mul_pair(r.c0, r.c1, a.c0, a.c1, b.c0, b.c1);
  return r;
}

HD Fp2 f2_sqr(const Fp2& a) {
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  Fp2 r;
  fp2_sqr_pair(r.c0, r.c1, a.c0, a.c1);
  return r;
}

HD Fp2 f2_mul_fp(const Fp2& a, const Fp& b) { return {fp_mul(a.c0, b), fp_mul(a.c1, b)}; }

// multiply by xi = 1 + u
HD Fp2 f2_mul_xi(const Fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

HD bool f2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
HD bool f2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }

template <bool kEarlyExit>
HDNI Fp2 f2_inv_t(const Fp2& a) {
  Fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fp ni = fp_inv_t<kEarlyExit>(n);
  return {fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}
HD Fp2 f2_inv(const Fp2& a) { return f2_inv_t<true>(a); }
HD Fp2 f2_inv_ct(const Fp2& a) { return f2_inv_t<false>(a); }

HD Fp2 f2_mul_small(const Fp2& a, int k) { return {fp_mul_small(a.c0, k), fp_mul_small(a.c1, k)}; }

// a is a square in Fp2 iff its norm a0^2 + a1^2 is a square in Fp.
HD bool f2_is_square(const Fp2& a) { return fp_is_square(fp_add(fp_sqr(a.c0), fp_sqr(a.c1))); }

// Square root in Fp2 with two Fp exponentiations (norm method, inverse-free):
//   n = a0^2 + a1^2, s = sqrt(n), c = (a0 + s)/2, t = c^((p-3)/4), y = c t
//   y^2 == c :  x = y + (a1 t / 2) u        (1/y = t)
//   y^2 == -c:  x = (-a1 t / 2) + y u       (y = sqrt(-c), 1/y = -t)
// Any root is fine: every caller fixes the sign afterwards.  Returns false if a is not a square.
HDNI bool f2_sqrt(Fp2& x, const Fp2& a) {
  if (f2_is_zero(a)) {
    x = f2_zero();
    return true;
  }
  Fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  Fp s;
  if (!fp_sqrt(s, n)) return false;
  Fp inv2 = fp_from_const(FP_INV2);
  Fp c = fp_mul(fp_add(a.c0, s), inv2);
  if (fp_is_zero(c)) c = fp_mul(fp_sub(a.c0, s), inv2);
  Fp t = fp_pow_win(c, WIN_P_M3_4, WIN_P_M3_4_N);
  Fp y = fp_mul(c, t);
  Fp h = fp_mul(fp_mul(a.c1, t), inv2);
  if (fp_eq(fp_sqr(y), c)) {
    x = {y, h};
  } else {
    x = {fp_neg(h), y};
  }
  return f2_eq(f2_sqr(x), a);
}

// RFC 9380 sgn0 for m = 2 (on canonical values)
HD int f2_sgn0(const Fp2& a) {
  Fp c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  int sign0 = c0.v[0] & 1;
  uint32_t z = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) z |= c0.v[i];
  int zero0 = z == 0;
  int sign1 = c1.v[0] & 1;
  return sign0 | (zero0 & sign1);
}

// ZCash "lexicographically largest" for Fp2: compare c1 first, c0 if c1 == 0.
HD bool f2_is_lex_largest(const Fp2& a) {
  Fp c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t z = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) z |= c1.v[i];
  return z ? fp_raw_is_lex_largest(c1) : fp_raw_is_lex_largest(c0);
}

// a^e, e a fixed multi-limb exponent (left-to-right binary)
HDNI Fp2 f2_pow_const(const Fp2& a, const uint32_t* e, int top_bit) {
  Fp2 r = f2_one();
  HB_NOUNROLL for (int i = top_bit; i >= 0; i--) {
    r = f2_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = f2_mul(r, a);
  }
  return r;
}

// ---------------------------------- Fp6 ----------------------------------
HD Fp6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
HD Fp6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
HD Fp6 f6_add(const Fp6& a, const Fp6& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
HD Fp6 f6_sub(const Fp6& a, const Fp6& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
HD Fp6 f6_neg(const Fp6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }

// multiply by v: (c0, c1, c2) v = (xi c2, c0, c1)
HD Fp6 f6_mul_v(const Fp6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba-style (6 Fp2 products)
HDNI Fp6 f6_mul(const Fp6& a, const Fp6& b) {
  Fp2 t0 = f2_mul(a.c0, b.c0);
  Fp2 t1 = f2_mul(a.c1, b.c1);
  Fp2 t2 = f2_mul(a.c2, b.c2);
  Fp2 c0 = f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2));
  c0 = f2_add(f2_mul_xi(f2_sub(f2_sub(c0, t1), t2)), t0);
  Fp2 c1 = f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1));
  c1 = f2_add(f2_sub(f2_sub(c1, t0), t1), f2_mul_xi(t2));
  Fp2 c2 = f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2));
  c2 = f2_add(f2_sub(f2_sub(c2, t0), t2), t1);
  return {c0, c1, c2};
}

HD Fp6 f6_sqr(const Fp6& a) { return f6_mul(a, a); }

// a * (b0 + b1 v)
HDNI Fp6 f6_mul_01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  Fp2 t0 = f2_mul(a.c0, b0);
  Fp2 t1 = f2_mul(a.c1, b1);
  Fp2 c0 = f2_add(f2_mul_xi(f2_sub(f2_mul(f2_add(a.c1, a.c2), b1), t1)), t0);
  Fp2 c1 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b0, b1)), t0), t1);
  Fp2 c2 = f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c2), b0), t0), t1);
  return {c0, c1, c2};
}

// a * (b1 v)
HDNI Fp6 f6_mul_1(const Fp6& a, const Fp2& b1) {
  return {f2_mul_xi(f2_mul(a.c2, b1)), f2_mul(a.c0, b1), f2_mul(a.c1, b1)};
}

HDNI Fp6 f6_inv(const Fp6& a) {
  Fp2 t0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  Fp2 t1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  Fp2 t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  Fp2 d = f2_add(f2_mul(a.c0, t0), f2_mul_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2))));
  Fp2 di = f2_inv(d);
  return {f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}

HD bool f6_is_zero(const Fp6& a) { return f2_is_zero(a.c0) && f2_is_zero(a.c1) && f2_is_zero(a.c2); }

// ---------------------------------- Fp12 ----------------------------------
HD Fp12 f12_one() { return {f6_one(), f6_zero()}; }

HDNI Fp12 f12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = f6_mul(a.c0, b.c0);
  Fp6 t1 = f6_mul(a.c1, b.c1);
  Fp6 c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  Fp6 c0 = f6_add(t0, f6_mul_v(t1));
  return {c0, c1};
}

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w, with two Fp6 products
HDNI Fp12 f12_sqr(const Fp12& a) {
  Fp6 t = f6_mul(a.c0, a.c1);
  Fp6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
  Fp6 c0 = f6_sub(f6_sub(s, t), f6_mul_v(t));
  return {c0, f6_add(t, t)};
}

// f * l where the line is l = a0 + a1 v + b1 v w   (L0 = (a0, a1, 0), L1 = (0, b1, 0))
HDNI Fp12 f12_mul_line(const Fp12& f, const Fp2& a0, const Fp2& a1, const Fp2& b1) {
  Fp6 t0 = f6_mul_01(f.c0, a0, a1);
  Fp6 t1 = f6_mul_1(f.c1, b1);
  Fp6 c1 = f6_sub(f6_sub(f6_mul_01(f6_add(f.c0, f.c1), a0, f2_add(a1, b1)), t0), t1);
  Fp6 c0 = f6_add(t0, f6_mul_v(t1));
  return {c0, c1};
}

HD Fp12 f12_conj(const Fp12& a) { return {a.c0, f6_neg(a.c1)}; }

HDNI Fp12 f12_inv(const Fp12& a) {
  // (a0 + a1 w)^-1 = (a0 - a1 w) / (a0^2 - v a1^2)
  Fp6 d = f6_sub(f6_sqr(a.c0), f6_mul_v(f6_sqr(a.c1)));
  Fp6 di = f6_inv(d);
  return {f6_mul(a.c0, di), f6_neg(f6_mul(a.c1, di))};
}

// Frobenius x -> x^(p^j): conjugate the Fp2 coefficients j times and scale the coefficient
// of w^k (k = 2i for c0.ci, 2i+1 for c1.ci) by FROBj[k].
template <int J>
HDNI Fp12 f12_frob(const Fp12& a) {
  const uint32_t(*g)[2][12] = (J == 1) ? FROB1 : (J == 2) ? FROB2 : FROB3;
  auto cj = [](const Fp2& x) { return (J & 1) ? f2_conj(x) : x; };
  Fp12 r;
  r.c0.c0 = cj(a.c0.c0);
  r.c0.c1 = f2_mul(cj(a.c0.c1), f2_from_const(g[2]));
  r.c0.c2 = f2_mul(cj(a.c0.c2), f2_from_const(g[4]));
  r.c1.c0 = f2_mul(cj(a.c1.c0), f2_from_const(g[1]));
  r.c1.c1 = f2_mul(cj(a.c1.c1), f2_from_const(g[3]));
  r.c1.c2 = f2_mul(cj(a.c1.c2), f2_from_const(g[5]));
  return r;
}

HDNI bool f12_is_one(const Fp12& a) {
  return f2_eq(a.c0.c0, f2_one()) && f2_is_zero(a.c0.c1) && f2_is_zero(a.c0.c2) && f6_is_zero(a.c1);
}

}  // namespace hb
