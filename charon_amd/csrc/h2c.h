// hash_to_curve for G2, RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_ with the Ethereum
// proof-of-possession DST (herumi ETH mode, tbls/herumi.go:32 bls.SetETHmode):
//   expand_message_xmd(msg, DST, 256) -> 4 Fp elements -> u0, u1 in Fp2
//   -> simplified SWU on E2' (A' = 240u, B' = 1012(1+u), Z = -(2+u))
//   -> 3-isogeny E2' -> E2 -> Q0 + Q1 -> clear_cofactor (Budroni-Pintore, = h_eff).
#pragma once
#include "ec.h"
#include "sha256.h"

namespace hb {

// "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" || I2OSP(43, 1)
HB_CONST uint8_t DST_PRIME[44] = {'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8',
                                  '1', 'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6',
                                  '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_', 43};
constexpr int DST_PRIME_LEN = 44;

// byte k of the xmd tail after msg: I2OSP(256, 2) || I2OSP(0, 1) || DST_prime
HD uint8_t xmd_tail_byte(int k) {
  if (k == 0) return 0x01;
  if (k < 3) return 0x00;
  return DST_PRIME[k - 3];
}
constexpr int XMD_TAIL_LEN = 3 + DST_PRIME_LEN;

HD uint32_t be_word(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
  return ((uint32_t)a << 24) | ((uint32_t)b << 16) | ((uint32_t)c << 8) | d;
}

// b0 = SHA256(Z_pad || msg || I2OSP(256,2) || 0x00 || DST_prime)
HDNI Sha256State xmd_b0(const uint8_t* msg, uint32_t len) {
  Sha256State st = sha256_init();
  uint32_t zero[16];
  HB_UNROLL for (int j = 0; j < 16; j++) zero[j] = 0;
  sha256_compress(st, zero);  // Z_pad block
  uint32_t body = len + XMD_TAIL_LEN;                       // bytes after Z_pad
  uint32_t total_bits = (64u + body) * 8u;
  uint32_t nblk = (body + 8u) / 64u + 1u;                  // blocks after Z_pad incl. padding
  HB_NOUNROLL for (uint32_t b = 0; b < nblk; b++) {
    uint32_t w[16];
    HB_UNROLL for (int j = 0; j < 16; j++) {
      uint8_t by[4];
      HB_UNROLL for (int k = 0; k < 4; k++) {
        uint32_t pos = b * 64u + (uint32_t)(4 * j + k);
        uint8_t v;
        if (pos < len) {
          v = msg[pos];
        } else if (pos < body) {
          v = xmd_tail_byte((int)(pos - len));
        } else if (pos == body) {
          v = 0x80;
        } else if (pos >= nblk * 64u - 4u) {
          v = (uint8_t)(total_bits >> (8 * (int)(nblk * 64u - 1u - pos)));
        } else {
          v = 0;
        }
        by[k] = v;
      }
      w[j] = be_word(by[0], by[1], by[2], by[3]);
    }
    sha256_compress(st, w);
  }
  return st;
}

// b_i = SHA256(x || I2OSP(i,1) || DST_prime), x = 32 bytes (8 words); 77 bytes -> 2 blocks
HDNI Sha256State xmd_bi(const uint32_t* x, uint32_t i) {
  Sha256State st = sha256_init();
  uint32_t w[16];
  HB_UNROLL for (int j = 0; j < 8; j++) w[j] = x[j];
  w[8] = be_word((uint8_t)i, DST_PRIME[0], DST_PRIME[1], DST_PRIME[2]);
  HB_UNROLL for (int j = 9; j < 16; j++) {
    int o = 4 * j - 33;
    w[j] = be_word(DST_PRIME[o], DST_PRIME[o + 1], DST_PRIME[o + 2], DST_PRIME[o + 3]);
  }
  sha256_compress(st, w);
  // second block: DST_prime[31..43] (13 bytes), 0x80, zeros, bit length 616
  uint8_t tb[64];
  HB_UNROLL for (int k = 0; k < 64; k++) tb[k] = 0;
  HB_UNROLL for (int k = 0; k < 13; k++) tb[k] = DST_PRIME[31 + k];
  tb[13] = 0x80;
  tb[62] = (uint8_t)(616 >> 8);
  tb[63] = (uint8_t)(616 & 0xff);
  HB_UNROLL for (int j = 0; j < 16; j++) w[j] = be_word(tb[4 * j], tb[4 * j + 1], tb[4 * j + 2], tb[4 * j + 3]);
  sha256_compress(st, w);
  return st;
}

// 64-byte big-endian integer (as 16 BE words) mod p, in Montgomery form
HD Fp fp_from_be512(const uint32_t* W) {
  Fp lo, hi = fp_zero();
  HB_UNROLL for (int i = 0; i < 12; i++) lo.v[i] = W[15 - i];
  HB_UNROLL for (int i = 0; i < 4; i++) hi.v[i] = W[3 - i];
  // lo may exceed 2p: it must be the second (unbounded) operand of the Montgomery product,
  // whose intermediate value stays below a + p for the first operand a.
  return fp_add(fp_mul(fp_from_const(FP_R2), lo), fp_mul(fp_from_const(FP_R3), hi));
}

// hash_to_field(msg, count = 2) for Fp2 with L = 64
HDNI void hash_to_field_fp2(Fp2& u0, Fp2& u1, const uint8_t* msg, uint32_t len) {
  Sha256State b0 = xmd_b0(msg, len);
  Fp e[4];
  uint32_t prev[8];
  HB_UNROLL for (int j = 0; j < 8; j++) prev[j] = b0.h[j];
  // b1 = H(b0 || 1 || DST'), b_i = H((b0 ^ b_{i-1}) || i || DST')
  HB_NOUNROLL for (int k = 0; k < 4; k++) {
    uint32_t W[16];
    HB_UNROLL for (int half = 0; half < 2; half++) {
      uint32_t i = (uint32_t)(2 * k + half + 1);
      uint32_t x[8];
      HB_UNROLL for (int j = 0; j < 8; j++) x[j] = (i == 1) ? b0.h[j] : (b0.h[j] ^ prev[j]);
      Sha256State bi = xmd_bi(x, i);
      HB_UNROLL for (int j = 0; j < 8; j++) {
        prev[j] = bi.h[j];
        W[8 * half + j] = bi.h[j];
      }
    }
    Fp v = fp_from_be512(W);
    // k is a runtime loop index: place without dynamic register indexing
    if (k == 0) e[0] = v;
    if (k == 1) e[1] = v;
    if (k == 2) e[2] = v;
    if (k == 3) e[3] = v;
  }
  u0 = {e[0], e[1]};
  u1 = {e[2], e[3]};
}

// simplified SWU for E2' (RFC 9380 6.6.2); returns affine point on E2'.  Straight-line with three
// Fp exponentiations (1/tv1, one norm square root, one (p-3)/4 power), so the lanes of a wave do
// not diverge on the square / non-square case:
//   s1 = N(gx1)^((p+1)/4) is sqrt(N(gx1)) if gx1 is a square, else sqrt(-N(gx1)); in that case
//   gx2 = (Z u^2)^3 gx1 is the square and sqrt(N(gx2)) = s1 N(u)^3 sqrt(-N(Z)^3).
// The Fp2 root of the chosen g(x) then follows the norm method of f2_sqrt.
HDNI void sswu_map(Fp2& x, Fp2& y, const Fp2& u) {
  Fp2 A = f2_from_const(SSWU_A), B = f2_from_const(SSWU_B), Z = f2_from_const(SSWU_Z);
  Fp2 u2 = f2_sqr(u);
  Fp2 zu2 = f2_mul(Z, u2);
  Fp2 tv1 = f2_add(f2_sqr(zu2), zu2);
  const bool tv1_zero = f2_is_zero(tv1);
  Fp2 x1 = f2_mul(f2_from_const(SSWU_MINUS_B_OVER_A), f2_add(f2_one(), f2_inv(tv1)));
  if (tv1_zero) x1 = f2_from_const(SSWU_B_OVER_ZA);
  Fp2 gx1 = f2_add(f2_mul(f2_add(f2_sqr(x1), A), x1), B);
  Fp2 x2 = f2_mul(zu2, x1);
  Fp2 gx2 = f2_add(f2_mul(f2_add(f2_sqr(x2), A), x2), B);
  Fp n1 = fp_add(fp_sqr(gx1.c0), fp_sqr(gx1.c1));
  Fp s1 = fp_pow_win(n1, WIN_SQRT, WIN_SQRT_N);
  const bool sq1 = fp_eq(fp_sqr(s1), n1);
  Fp nu = fp_add(fp_sqr(u.c0), fp_sqr(u.c1));
  Fp s2 = fp_mul(fp_mul(s1, fp_mul(fp_sqr(nu), nu)), fp_from_const(SSWU_SQRT_MNZ3));
  Fp2 a = sq1 ? gx1 : gx2;
  Fp s = sq1 ? s1 : s2;
  x = sq1 ? x1 : x2;
  Fp inv2 = fp_from_const(FP_INV2);
  Fp c = fp_mul(fp_add(a.c0, s), inv2);
  if (fp_is_zero(c)) c = fp_mul(fp_sub(a.c0, s), inv2);
  Fp t = fp_pow_win(c, WIN_P_M3_4, WIN_P_M3_4_N);
  Fp y0 = fp_mul(c, t);
  Fp h = fp_mul(fp_mul(a.c1, t), inv2);
  if (fp_eq(fp_sqr(y0), c)) {
    y = {y0, h};
  } else {
    y = {fp_neg(h), y0};
  }
  if (f2_sgn0(u) != f2_sgn0(y)) y = f2_neg(y);
}

HDNI Fp2 f2_poly_eval(const uint32_t (*c)[2][12], int n, const Fp2& x) {
  Fp2 acc = f2_from_const(c[n - 1]);
  for (int i = n - 2; i >= 0; i--) acc = f2_add(f2_mul(acc, x), f2_from_const(c[i]));
  return acc;
}

// 3-isogeny E2' -> E2 (RFC 9380 E.3), output in Jacobian coordinates (no inversion):
//   x = xn/xd, y = y' yn/yd;  Z = xd yd, X = xn xd yd^2, Y = y' yn xd^3 yd^2
HDNI G2J iso3_map(const Fp2& x, const Fp2& y) {
  Fp2 xn = f2_poly_eval(ISO_XNUM, 4, x);
  Fp2 xd = f2_poly_eval(ISO_XDEN, 3, x);
  Fp2 yn = f2_poly_eval(ISO_YNUM, 4, x);
  Fp2 yd = f2_poly_eval(ISO_YDEN, 4, x);
  G2J r;
  Fp2 yd2 = f2_sqr(yd);
  Fp2 xdyd2 = f2_mul(xd, yd2);
  r.Z = f2_mul(xd, yd);
  r.X = f2_mul(xn, xdyd2);
  r.Y = f2_mul(f2_mul(y, yn), f2_mul(xdyd2, f2_sqr(xd)));
  return r;
}

// A polynomial (coefficients c[0..n-1]) homogenised at x = X / Zh: sum c_i X^i Zh^(n-1-i), with
// zp[k] = Zh^k.
HDNI Fp2 f2_poly_eval_h(const uint32_t (*c)[2][12], int n, const Fp2& X, const Fp2* zp) {
  Fp2 acc = f2_from_const(c[n - 1]);
  for (int i = n - 2; i >= 0; i--) acc = f2_add(f2_mul(acc, X), f2_mul(f2_from_const(c[i]), zp[n - 1 - i]));
  return acc;
}

// sswu_map followed by iso3_map without an inversion: two Fp exponentiations instead of three.
//   x1 = xn / xd (xn = -B (tv1 + 1), xd = A tv1; B, Z A if tv1 = 0),  g(x1) = gn / xd^3 = a / n with
//   a = gn conj(xd^3), n = N(xd^3) in Fp.  The norm method of f2_sqrt on a / n:
//     S = N(a)^((p+1)/4)                      [sqrt(N(g(x1))) n, or sqrt(-N(g(x1))) n]
//     c = cn / n,  cn = (a0 + S) / 2
//     T = (cn n^3)^((p-3)/4),  so c^((p-3)/4) = T n^2,  y0 = c^((p+1)/4) = cn T n,  h = a1 T n / 2
//   (g(x2) = (Z u^2)^3 g(x1) shares the denominator n).  The isogeny is evaluated homogeneously at
//   x = X / Zh; with D1 = XD Zh, D2 = YD: x' = XN / D1, y' = y YN / D2, Jacobian (XN D1 D2^2,
//   y YN D1^3 D2^2, D1 D2).  Same point as iso3_map(sswu_map(u)).
HDNI G2J sswu_iso_map(const Fp2& u) {
  const Fp2 A = f2_from_const(SSWU_A), B = f2_from_const(SSWU_B), Z = f2_from_const(SSWU_Z);
  const Fp2 zu2 = f2_mul(Z, f2_sqr(u));
  const Fp2 tv1 = f2_add(f2_sqr(zu2), zu2);
  const bool tv1_zero = f2_is_zero(tv1);
  Fp2 xn = f2_neg(f2_mul(B, f2_add(tv1, f2_one())));
  Fp2 xd = f2_mul(A, tv1);
  if (tv1_zero) {
    xn = B;
    xd = f2_mul(Z, A);
  }
  const Fp2 xd2 = f2_sqr(xd);
  const Fp2 gd = f2_mul(xd2, xd);
  const Fp2 gn = f2_add(f2_mul(f2_add(f2_sqr(xn), f2_mul(A, xd2)), xn), f2_mul(B, gd));
  const Fp2 a = f2_mul(gn, f2_conj(gd));
  const Fp n = fp_add(fp_sqr(gd.c0), fp_sqr(gd.c1));
  const Fp na = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  const Fp s1 = fp_pow_win(na, WIN_SQRT, WIN_SQRT_N);
  const bool sq1 = fp_eq(fp_sqr(s1), na);
  const Fp nu = fp_add(fp_sqr(u.c0), fp_sqr(u.c1));
  const Fp s2 = fp_mul(fp_mul(s1, fp_mul(fp_sqr(nu), nu)), fp_from_const(SSWU_SQRT_MNZ3));
  const Fp2 zu2_3 = f2_mul(f2_sqr(zu2), zu2);
  const Fp2 as = sq1 ? a : f2_mul(zu2_3, a);
  const Fp S = sq1 ? s1 : s2;
  const Fp2 X = sq1 ? xn : f2_mul(zu2, xn);
  const Fp inv2 = fp_from_const(FP_INV2);
  Fp cn = fp_mul(fp_add(as.c0, S), inv2);
  if (fp_is_zero(cn)) cn = fp_mul(fp_sub(as.c0, S), inv2);
  const Fp T = fp_pow_win(fp_mul(cn, fp_mul(fp_sqr(n), n)), WIN_P_M3_4, WIN_P_M3_4_N);
  const Fp Tn = fp_mul(T, n);
  const Fp y0 = fp_mul(cn, Tn);
  const Fp h = fp_mul(fp_mul(as.c1, Tn), inv2);
  Fp2 y;
  if (fp_eq(fp_mul(fp_sqr(y0), n), cn)) {
    y = {y0, h};
  } else {
    y = {fp_neg(h), y0};
  }
  if (f2_sgn0(u) != f2_sgn0(y)) y = f2_neg(y);
  Fp2 zp[4];
  zp[0] = f2_one();
  zp[1] = xd;
  zp[2] = xd2;
  zp[3] = gd;
  const Fp2 XN = f2_poly_eval_h(ISO_XNUM, 4, X, zp);
  const Fp2 XD = f2_poly_eval_h(ISO_XDEN, 3, X, zp);
  const Fp2 YN = f2_poly_eval_h(ISO_YNUM, 4, X, zp);
  const Fp2 YD = f2_poly_eval_h(ISO_YDEN, 4, X, zp);
  const Fp2 D1 = f2_mul(XD, xd), D2 = YD;
  const Fp2 D22 = f2_sqr(D2);
  const Fp2 D1D22 = f2_mul(D1, D22);
  G2J r;
  r.Z = f2_mul(D1, D2);
  r.X = f2_mul(XN, D1D22);
  r.Y = f2_mul(f2_mul(y, YN), f2_mul(D1D22, f2_sqr(D1)));
  return r;
}

// h_eff * P via  [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)  (RFC 9380 G.3), x < 0.
HDNI G2J g2_clear_cofactor(const G2J& P) {
  G2J t1 = jac_neg(jac_mul_by_xabs(P));  // [x]P
  G2J t2 = g2_psi(P);
  G2J t3 = g2_psi2(jac_dbl(P));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(jac_mul_by_xabs(t2));  // [x](xP + psi(P))
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(P));
}

HDNI G2J hash_to_g2(const uint8_t* msg, uint32_t len) {
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msg, len);
  const G2J q0 = sswu_iso_map(u0);
  const G2J q1 = sswu_iso_map(u1);
  return g2_clear_cofactor(jac_add(q0, q1));
}

}  // namespace hb
