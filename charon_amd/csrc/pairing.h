// Optimal-ate pairing for BLS12-381 (M-type twist, |x| = 0xd201000000010000).
//
// Miller loop: G2 point T in homogeneous projective coordinates on the twist, lines scaled by
// w^3 and an Fp2 factor (both killed by the final exponentiation), giving the sparse form
//     l = a0 + a1 v + b1 v w   (a0, a1, b1 in Fp2)
// doubling:  a0 = Y^2 - 3b'Z^2,  a1 = -3X^2 xP,  b1 = 2YZ yP
// addition:  a0 = th xq - la yq, a1 = -th xP,    b1 = la yP   (th = Y - yq Z, la = X - xq Z)
// We return f_{|x|,Q}(P) without the final conjugation: verdicts prod e(Pi,Qi) == 1 are
// unchanged (it is the inverse pairing).
//
// Final exponentiation: easy part f^((p^6-1)(p^2+1)), hard part via
//     3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
// i.e. we compute e^3; e == 1 <=> e^3 == 1 since gcd(3, r) = 1.
#pragma once
#include "ec.h"

namespace hb {

struct LineCoeffs {
  Fp2 a0, a1, b1;
};

struct G2Proj {
  Fp2 X, Y, Z;
};

HD Fp fp_half(const Fp& a) {
  // a in [0,2p): (a even ? a : a + p) / 2  -> [0, 1.5p)
  Fp t = a;
  Fp s;
  uint32_t carry = 0;
  if (a.v[0] & 1) carry = raw_add_const(s, a, P_RAW), t = s;
  Fp r;
  HB_UNROLL for (int i = 0; i < NL - 1; i++) r.v[i] = (t.v[i] >> 1) | (t.v[i + 1] << 31);
  r.v[NL - 1] = (t.v[NL - 1] >> 1) | (carry << 31);
  return r;
}

HD Fp2 f2_half(const Fp2& a) { return {fp_half(a.c0), fp_half(a.c1)}; }

// 3b' = 12 (1 + u) times z  =  12 * mul_xi(z)
HD Fp2 f2_mul_b3(const Fp2& z) {
  Fp2 t = f2_mul_xi(z);
  Fp2 t4 = f2_dbl(f2_dbl(t));
  return f2_add(f2_add(t4, t4), t4);
}

// T <- 2T, returns the tangent line at T evaluated at P = (xP, yP)
HDNI LineCoeffs miller_dbl(G2Proj& T, const Fp& xP, const Fp& yP) {
  Fp2 A = f2_sqr(T.Y);
  Fp2 B = f2_sqr(T.Z);
  Fp2 C = f2_mul_b3(B);               // 3b' Z^2
  Fp2 E = f2_add(f2_dbl(C), C);      // 9b' Z^2
  Fp2 D = f2_mul(T.Y, T.Z);          // YZ
  Fp2 XX = f2_sqr(T.X);
  LineCoeffs l;
  l.a0 = f2_sub(A, C);
  l.a1 = f2_neg(f2_mul_fp(f2_add(f2_dbl(XX), XX), xP));
  l.b1 = f2_mul_fp(f2_dbl(D), yP);
  Fp2 XY = f2_mul(T.X, T.Y);
  Fp2 X3 = f2_half(f2_mul(XY, f2_sub(A, E)));
  Fp2 H = f2_half(f2_add(A, E));
  Fp2 Y3 = f2_sub(f2_sqr(H), f2_add(f2_dbl(f2_sqr(C)), f2_sqr(C)));
  Fp2 Z3 = f2_dbl(f2_mul(A, D));     // 2 Y^3 Z
  T.X = X3;
  T.Y = Y3;
  T.Z = Z3;
  return l;
}

// T <- T + Q (Q affine), returns the chord through T and Q evaluated at P
HDNI LineCoeffs miller_add(G2Proj& T, const Fp2& xq, const Fp2& yq, const Fp& xP, const Fp& yP) {
  Fp2 th = f2_sub(T.Y, f2_mul(yq, T.Z));
  Fp2 la = f2_sub(T.X, f2_mul(xq, T.Z));
  Fp2 C = f2_sqr(th);
  Fp2 D = f2_sqr(la);
  Fp2 E = f2_mul(la, D);
  Fp2 F = f2_mul(T.Z, C);
  Fp2 G = f2_mul(T.X, D);
  Fp2 H = f2_sub(f2_add(E, F), f2_dbl(G));
  LineCoeffs l;
  l.a0 = f2_sub(f2_mul(th, xq), f2_mul(la, yq));
  l.a1 = f2_neg(f2_mul_fp(th, xP));
  l.b1 = f2_mul_fp(la, yP);
  T.X = f2_mul(la, H);
  T.Y = f2_sub(f2_mul(th, f2_sub(G, H)), f2_mul(T.Y, E));
  T.Z = f2_mul(T.Z, E);
  return l;
}

// ---- unevaluated lines for the lane-group Miller loop (pair3.h) ----
// A line of the loop as three Fp2 coefficients (a0, c1, c2): evaluated at P = (xP, yP) it is
// a0 + (c1 xP) v + (c2 yP) v w, i.e. the (a0, a1, b1) of LineCoeffs with a1 = c1 xP, b1 = c2 yP.
// The loop visits 63 doubling lines and, after the doublings at the 5 set bits of |x| below the
// top, one addition line each: N_LINES = 68, in loop order.
constexpr int N_LINES = 68;

HD LineCoeffs miller_dbl_c(G2Proj& T) {
  Fp2 A = f2_sqr(T.Y);
  Fp2 B = f2_sqr(T.Z);
  Fp2 C = f2_mul_b3(B);
  Fp2 E = f2_add(f2_dbl(C), C);
  Fp2 D = f2_mul(T.Y, T.Z);
  Fp2 XX = f2_sqr(T.X);
  LineCoeffs l;
  l.a0 = f2_sub(A, C);
  l.a1 = f2_neg(f2_add(f2_dbl(XX), XX));
  l.b1 = f2_dbl(D);
  Fp2 XY = f2_mul(T.X, T.Y);
  Fp2 X3 = f2_half(f2_mul(XY, f2_sub(A, E)));
  Fp2 H = f2_half(f2_add(A, E));
  Fp2 C2 = f2_sqr(C);
  Fp2 Y3 = f2_sub(f2_sqr(H), f2_add(f2_dbl(C2), C2));
  Fp2 Z3 = f2_dbl(f2_mul(A, D));
  T.X = X3;
  T.Y = Y3;
  T.Z = Z3;
  return l;
}

HD LineCoeffs miller_add_c(G2Proj& T, const Fp2& xq, const Fp2& yq) {
  Fp2 th = f2_sub(T.Y, f2_mul(yq, T.Z));
  Fp2 la = f2_sub(T.X, f2_mul(xq, T.Z));
  Fp2 C = f2_sqr(th);
  Fp2 D = f2_sqr(la);
  Fp2 E = f2_mul(la, D);
  Fp2 F = f2_mul(T.Z, C);
  Fp2 G = f2_mul(T.X, D);
  Fp2 H = f2_sub(f2_add(E, F), f2_dbl(G));
  LineCoeffs l;
  l.a0 = f2_sub(f2_mul(th, xq), f2_mul(la, yq));
  l.a1 = f2_neg(th);
  l.b1 = la;
  T.X = f2_mul(la, H);
  T.Y = f2_sub(f2_mul(th, f2_sub(G, H)), f2_mul(T.Y, E));
  T.Z = f2_mul(T.Z, E);
  return l;
}

HD void line_eval(LineCoeffs& l, const Fp& xP, const Fp& yP) {
  l.a1 = f2_mul_fp(l.a1, xP);
  l.b1 = f2_mul_fp(l.b1, yP);
}

// f_{|x|,Q1}(P1) * f_{|x|,Q2}(P2); all inputs affine and not infinity.
HDNI Fp12 miller_loop2(const G1A& P1, const G2A& Q1, const G1A& P2, const G2A& Q2) {
  G2Proj T1 = {Q1.x, Q1.y, f2_one()};
  G2Proj T2 = {Q2.x, Q2.y, f2_one()};
  Fp12 f = f12_one();
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    if (i != 62) f = f12_sqr(f);
    LineCoeffs l = miller_dbl(T1, P1.x, P1.y);
    f = f12_mul_line(f, l.a0, l.a1, l.b1);
    l = miller_dbl(T2, P2.x, P2.y);
    f = f12_mul_line(f, l.a0, l.a1, l.b1);
    if ((HB_X_ABS >> i) & 1) {
      l = miller_add(T1, Q1.x, Q1.y, P1.x, P1.y);
      f = f12_mul_line(f, l.a0, l.a1, l.b1);
      l = miller_add(T2, Q2.x, Q2.y, P2.x, P2.y);
      f = f12_mul_line(f, l.a0, l.a1, l.b1);
    }
  }
  return f;
}

HDNI Fp12 miller_loop1(const G1A& P1, const G2A& Q1) {
  G2Proj T1 = {Q1.x, Q1.y, f2_one()};
  Fp12 f = f12_one();
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    if (i != 62) f = f12_sqr(f);
    LineCoeffs l = miller_dbl(T1, P1.x, P1.y);
    f = f12_mul_line(f, l.a0, l.a1, l.b1);
    if ((HB_X_ABS >> i) & 1) {
      l = miller_add(T1, Q1.x, Q1.y, P1.x, P1.y);
      f = f12_mul_line(f, l.a0, l.a1, l.b1);
    }
  }
  return f;
}

// (x + y s)^2 in Fp4 = Fp2[s]/(s^2 - xi): returns (x^2 + xi y^2, 2xy) with 3 Fp2 squarings.
HD void fp4_sqr(Fp2& r0, Fp2& r1, const Fp2& x, const Fp2& y) {
  Fp2 t0 = f2_sqr(x), t1 = f2_sqr(y);
  r0 = f2_add(f2_mul_xi(t1), t0);
  r1 = f2_sub(f2_sub(f2_sqr(f2_add(x, y)), t0), t1);
}

// Squaring in the cyclotomic subgroup G_{Phi_6}(p^2) (Granger-Scott, "Faster squaring in the
// cyclotomic subgroup of sixth degree extensions", PKC 2010): with s = w^3 the element is three
// Fp4 values (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2); 9 Fp2 squarings (18 Fp products)
// instead of f12_sqr's 36.  Valid only after the easy part of the final exponentiation.
HDNI Fp12 f12_cyclo_sqr(const Fp12& a) {
  Fp2 t00, t01, t10, t11, t20, t21;
  fp4_sqr(t00, t01, a.c0.c0, a.c1.c1);
  fp4_sqr(t10, t11, a.c1.c0, a.c0.c2);
  fp4_sqr(t20, t21, a.c0.c1, a.c1.c2);
  Fp12 r;
  r.c0.c0 = f2_add(f2_dbl(f2_sub(t00, a.c0.c0)), t00);  // 3 t00 - 2 a
  r.c0.c1 = f2_add(f2_dbl(f2_sub(t10, a.c0.c1)), t10);
  r.c0.c2 = f2_add(f2_dbl(f2_sub(t20, a.c0.c2)), t20);
  Fp2 x = f2_mul_xi(t21);
  r.c1.c0 = f2_add(f2_dbl(f2_add(x, a.c1.c0)), x);      // 3 xi t21 + 2 a
  r.c1.c1 = f2_add(f2_dbl(f2_add(t01, a.c1.c1)), t01);
  r.c1.c2 = f2_add(f2_dbl(f2_add(t11, a.c1.c2)), t11);
  return r;
}

// f^|x| in the cyclotomic subgroup
HDNI Fp12 f12_pow_xabs(const Fp12& f) {
  Fp12 r = f;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = f12_cyclo_sqr(r);
    if ((HB_X_ABS >> i) & 1) r = f12_mul(r, f);
  }
  return r;
}

// f^x for x < 0 (cyclotomic: inverse = conjugate)
HD Fp12 f12_pow_x(const Fp12& f) { return f12_conj(f12_pow_xabs(f)); }

// returns f^(3 (p^12-1)/r)
HDNI Fp12 final_exponentiation(const Fp12& f) {
  Fp12 t = f12_mul(f12_conj(f), f12_inv(f));  // ^(p^6 - 1)
  t = f12_mul(f12_frob<2>(t), t);                 // ^(p^2 + 1)
  // hard part: a = t^((x-1)^2)
  Fp12 a = f12_mul(f12_pow_x(t), f12_conj(t));
  a = f12_mul(f12_pow_x(a), f12_conj(a));
  // b = a^(x+p)
  Fp12 b = f12_mul(f12_pow_x(a), f12_frob<1>(a));
  // c = b^(x^2 + p^2 - 1)
  Fp12 c = f12_mul(f12_mul(f12_pow_x(f12_pow_x(b)), f12_frob<2>(b)), f12_conj(b));
  // result = c * t^3
  return f12_mul(c, f12_mul(f12_cyclo_sqr(t), t));
}

}  // namespace hb
