// G1 (y^2 = x^3 + 4 over Fp) and G2 (y^2 = x^3 + 4(1+u) over Fp2) group law in Jacobian
// coordinates (x = X/Z^2, y = Y/Z^3, Z = 0 is the point at infinity), templated over the
// coordinate field.  Formulas: dbl-2009-l, madd-2007-bl, add-2007-bl (a = 0 curves).
#pragma once
#include "tower.h"

namespace hb {

// ---- uniform field interface for the templates ----
HD Fp f_add(const Fp& a, const Fp& b) { return fp_add(a, b); }
HD Fp f_sub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
HD Fp f_mul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
HD Fp f_sqr(const Fp& a) { return fp_sqr(a); }
HD Fp f_neg(const Fp& a) { return fp_neg(a); }
HD Fp f_dbl(const Fp& a) { return fp_dbl(a); }
HD Fp f_inv(const Fp& a) { return fp_inv(a); }
HD Fp f_inv_ct(const Fp& a) { return fp_inv_ct(a); }
HD bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
HD bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
HD void f_set_zero(Fp& a) { a = fp_zero(); }
HD void f_set_one(Fp& a) { a = fp_one(); }

HD Fp2 f_add(const Fp2& a, const Fp2& b) { return f2_add(a, b); }
HD Fp2 f_sub(const Fp2& a, const Fp2& b) { return f2_sub(a, b); }
HD Fp2 f_mul(const Fp2& a, const Fp2& b) { return f2_mul(a, b); }
HD Fp2 f_sqr(const Fp2& a) { return f2_sqr(a); }
HD Fp2 f_neg(const Fp2& a) { return f2_neg(a); }
HD Fp2 f_dbl(const Fp2& a) { return f2_dbl(a); }
HD Fp2 f_inv(const Fp2& a) { return f2_inv(a); }
HD Fp2 f_inv_ct(const Fp2& a) { return f2_inv_ct(a); }
HD bool f_is_zero(const Fp2& a) { return f2_is_zero(a); }
HD bool f_eq(const Fp2& a, const Fp2& b) { return f2_eq(a, b); }
HD void f_set_zero(Fp2& a) { a = f2_zero(); }
HD void f_set_one(Fp2& a) { a = f2_one(); }

template <class F>
struct Jac {
  F X, Y, Z;
};
template <class F>
struct Aff {
  F x, y;
  bool inf;
};

using G1J = Jac<Fp>;
using G2J = Jac<Fp2>;
using G1A = Aff<Fp>;
using G2A = Aff<Fp2>;

template <class F>
HD Jac<F> jac_infinity() {
  Jac<F> r;
  f_set_one(r.X);
  f_set_one(r.Y);
  f_set_zero(r.Z);
  return r;
}

template <class F>
HD bool jac_is_inf(const Jac<F>& p) {
  return f_is_zero(p.Z);
}

template <class F>
HD Jac<F> jac_from_aff(const Aff<F>& a) {
  if (a.inf) return jac_infinity<F>();
  Jac<F> r;
  r.X = a.x;
  r.Y = a.y;
  f_set_one(r.Z);
  return r;
}

template <class F>
HD Jac<F> jac_neg(const Jac<F>& p) {
  return {p.X, f_neg(p.Y), p.Z};
}

// dbl-2009-l: 2M + 5S
template <class F>
HDNI Jac<F> jac_dbl(const Jac<F>& p) {
  F A = f_sqr(p.X);
  F B = f_sqr(p.Y);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add(p.X, B)), A), C));
  F E = f_add(f_dbl(A), A);
  F Fv = f_sqr(E);
  Jac<F> r;
  r.X = f_sub(Fv, f_dbl(D));
  F C8 = f_dbl(f_dbl(f_dbl(C)));
  r.Y = f_sub(f_mul(E, f_sub(D, r.X)), C8);
  r.Z = f_dbl(f_mul(p.Y, p.Z));
  return r;  // Z = 0 propagates for infinity (and Y=0 never occurs on these curves' r-torsion)
}

// madd-2007-bl: p + q with q affine (q not infinity)
template <class F>
HDNI Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) {
  if (q.inf) return p;
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = f_sqr(p.Z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.Z), Z1Z1);
  F H = f_sub(U2, p.X);
  F rr = f_dbl(f_sub(S2, p.Y));
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.X, I);
  Jac<F> r;
  r.X = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.Y = f_sub(f_mul(rr, f_sub(V, r.X)), f_dbl(f_mul(p.Y, J)));
  r.Z = f_sub(f_sub(f_sqr(f_add(p.Z, H)), Z1Z1), HH);
  return r;
}

// add-2007-bl: general Jacobian addition
template <class F>
HDNI Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = f_sqr(p.Z);
  F Z2Z2 = f_sqr(q.Z);
  F U1 = f_mul(p.X, Z2Z2);
  F U2 = f_mul(q.X, Z1Z1);
  F S1 = f_mul(f_mul(p.Y, q.Z), Z2Z2);
  F S2 = f_mul(f_mul(q.Y, p.Z), Z1Z1);
  F H = f_sub(U2, U1);
  F rr = f_dbl(f_sub(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  Jac<F> r;
  r.X = f_sub(f_sub(f_sqr(rr), J), f_dbl(V));
  r.Y = f_sub(f_mul(rr, f_sub(V, r.X)), f_dbl(f_mul(S1, J)));
  r.Z = f_mul(f_sub(f_sub(f_sqr(f_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return r;
}

// kSecret: p depends on a secret key (Sign, SecretToPublicKey): the fixed-trip inversion
template <class F, bool kSecret = false>
HDNI Aff<F> jac_to_aff(const Jac<F>& p) {
  Aff<F> r;
  if (jac_is_inf(p)) {
    f_set_zero(r.x);
    f_set_zero(r.y);
    r.inf = true;
    return r;
  }
  F zi = kSecret ? f_inv_ct(p.Z) : f_inv(p.Z);
  F zi2 = f_sqr(zi);
  r.x = f_mul(p.X, zi2);
  r.y = f_mul(p.Y, f_mul(zi2, zi));
  r.inf = false;
  return r;
}

// projective equality of two Jacobian points
template <class F>
HDNI bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.Z), Z2Z2 = f_sqr(q.Z);
  if (!f_eq(f_mul(p.X, Z2Z2), f_mul(q.X, Z1Z1))) return false;
  return f_eq(f_mul(p.Y, f_mul(q.Z, Z2Z2)), f_mul(q.Y, f_mul(p.Z, Z1Z1)));
}

// [|x|] p for the curve parameter |x| = 0xd201000000010000 (63 doublings, 5 additions)
template <class F>
HDNI Jac<F> jac_mul_by_xabs(const Jac<F>& p) {
  Jac<F> r = p;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = jac_dbl(r);
    if ((HB_X_ABS >> i) & 1) r = jac_add(r, p);
  }
  return r;
}

// [|x|] q for q affine (not infinity): the five additions are mixed ones
template <class F>
HDNI Jac<F> jac_mul_by_xabs_aff(const Aff<F>& q) {
  Jac<F> r = jac_from_aff(q);
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = jac_dbl(r);
    if ((HB_X_ABS >> i) & 1) r = jac_add_aff(r, q);
  }
  return r;
}

// [k] q for q affine, k given as little-endian 32-bit words (nbits significant bits)
template <class F>
HDNI Jac<F> jac_mul_aff(const Aff<F>& q, const uint32_t* k, int nbits) {
  Jac<F> r = jac_infinity<F>();
  HB_NOUNROLL for (int i = nbits - 1; i >= 0; i--) {
    r = jac_dbl(r);
    if ((k[i >> 5] >> (i & 31)) & 1) r = jac_add_aff(r, q);
  }
  return r;
}

// ---------------------------------------------------------------------------------------
// Endomorphisms and subgroup membership
// ---------------------------------------------------------------------------------------

// psi(x, y) = (conj(x) cx, conj(y) cy), applied to Jacobian coordinates (Z conjugated).
HDNI G2J g2_psi(const G2J& p) {
  return {f2_mul(f2_conj(p.X), f2_from_const(PSI_CX)), f2_mul(f2_conj(p.Y), f2_from_const(PSI_CY)),
          f2_conj(p.Z)};
}

HDNI G2J g2_psi2(const G2J& p) {
  return {f2_mul(p.X, f2_from_const(PSI2_CX)), f2_mul(p.Y, f2_from_const(PSI2_CY)), p.Z};
}

// Q in G2  <=>  psi(Q) == [x] Q  (Scott, "A note on group membership tests for G1, G2 and GT
// on BLS pairing-friendly curves", 2021); x < 0 so [x]Q = -[|x|]Q.
HDNI bool g2_in_subgroup(const G2A& q) {
  if (q.inf) return true;
  G2J Q = jac_from_aff(q);
  G2J xq = jac_neg(jac_mul_by_xabs_aff(q));
  return jac_eq(g2_psi(Q), xq);
}

// P in G1  <=>  phi(P) == [-x^2] P with phi(x, y) = (beta x, y).
HDNI bool g1_in_subgroup(const G1A& p) {
  if (p.inf) return true;
  G1J t = jac_mul_by_xabs(jac_mul_by_xabs_aff(p));  // [x^2] P
  G1J phi = jac_from_aff(G1A{fp_mul(p.x, fp_from_const(G1_BETA)), p.y, false});
  return jac_eq(phi, jac_neg(t));
}

HD bool g1_on_curve(const G1A& p) {
  if (p.inf) return true;
  Fp rhs = fp_add(fp_mul(fp_sqr(p.x), p.x), fp_from_const(G1_B));
  return fp_eq(fp_sqr(p.y), rhs);
}

HD bool g2_on_curve(const G2A& p) {
  if (p.inf) return true;
  Fp2 rhs = f2_add(f2_mul(f2_sqr(p.x), p.x), f2_from_const(G2_B));
  return f2_eq(f2_sqr(p.y), rhs);
}

}  // namespace hb
