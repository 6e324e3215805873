// The Miller loop's arithmetic in lazily reduced 28-bit limbs (round 4).
//
// pairing.h / pair3.h run the Miller chain (G2 point + lines) and the three-lane Fp12 accumulator
// on stored 12-word Fp: every Fp2 product splits its four operands into 28-bit limbs and joins
// its two results, and every addition is a carry chain plus a conditional subtraction of 2p.
// Here both stay in 14 x 28-bit limbs (ec28.h L28 / F2L): the products take and return limbs,
// additions are limb-wise, subtractions add a multiple K = s p of p that dominates the
// subtrahend limb by limb (ec28.h K28<s, t>), and carries run only where a bound needs them.
// Values do not grow from step to step: every step ends with l_red, a partial reduction that
// needs no product (q = floor(v / p) or one less, read off the top 56 bits; v - q p < 2p), so
// the chain's point and the accumulator's lane values are below 2p at every step boundary.
// Reduced values are valid stored words after a join (fp.h fp_join28): the lines written to
// memory and the loop's result keep the stored-word layouts of layout.h without a product.
//
// charon_amd/tools/lazy28.py restates every formula here (ldbl, ladd, f4_mul, f4_sqr, g4_sqr,
// g4_mul_line) over per-limb intervals and proves that no limb leaves 32 bits, no product column
// 64 bits, every K dominates its subtrahend and the step outputs are reduced below 2p; the site
// constants below are the ones lazy28.KSITE holds ("3*": the chain, "4*": the Fp4 lane values),
// tests/test_lazy28.py compares them.
#pragma once
#include "pair3.h"
#include "pair6.h"

namespace hb {

HD L28 l_zero() {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = 0;
  return r;
}
HD L28 l_select(bool take_b, const L28& a, const L28& b) {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = take_b ? b.l[i] : a.l[i];
  return r;
}
// a reduced value (< 2p, normalised) as stored words, no product
HD Fp l_join(const L28& a) {
  Fp r;
  fp_join28(r.v, a.l);
  return r;
}

HD F2L f2l_zero() { return {l_zero(), l_zero()}; }
HD F2L f2l_one() { return {l_from(fp_one()), l_zero()}; }
HD F2L f2l_select(bool take_b, const F2L& a, const F2L& b) {
  return {l_select(take_b, a.c0, b.c0), l_select(take_b, a.c1, b.c1)};
}
HD Fp2 f2l_join(const F2L& a) { return {l_join(a.c0), l_join(a.c1)}; }
// (a0 + a1 u)(1 + u) = (a0 + K - a1) + (a0 + a1) u
template <uint32_t S, uint32_t T>
HD F2L f2l_xi(const F2L& a) {
  return {l_sub<S, T>(a.c0, a.c1), l_add(a.c0, a.c1)};
}

// ---- the Miller chain: T in homogeneous projective coordinates on the twist (pairing.h
// miller_dbl_c / miller_add_c), the line as (a0, c1, c2) -- evaluated at P it is
// a0 + (c1 xP) v + (c2 yP) v w.  Coordinates and line coefficients reduced (< 2p).
struct G2P28 {
  F2L X, Y, Z;
};
struct Line28 {
  F2L a0, a1, b1;
};

// lazy28.py ldbl: the doubling step scaled by 4 (X3 = 2 X Y (A - E), Y3 = (A + E)^2 - 12 C^2,
// Z3 = 8 A D -- the same projective point as miller_dbl_c's, no halving), A = Y^2, B = Z^2,
// C = 3 b' B = 12 xi B, E = 3 C, D = Y Z; line (A - C, -3 X^2, 2 D), handed to put(Line28) as
// soon as it exists.  The products run in the order that ends their inputs' live ranges first.
template <class Put, class M = F2One>
HD void l2_dbl_line(G2P28& T, const Put& put, M m = M()) {
  const F2L XX = fs<78, 1>(m, T.X);
  const F2L XY = fm(m, f2l_shl(T.X, 1), T.Y);
  const F2L D = fm(m, T.Y, T.Z);
  const F2L A = fs<78, 1>(m, T.Y);
  const F2L B = fs<78, 1>(m, T.Z);
  const F2L xb = f2l_norm(f2l_xi<2, 1>(B));
  const F2L C = f2l_norm(f2l_add(f2l_shl(xb, 3), f2l_shl(xb, 2)));
  put(Line28{f2l_red(f2l_sub<38, 1>(A, C)), f2l_red(f2l_sub<4, 3>(f2l_zero(), f2l_add(f2l_shl(XX, 1), XX))),
             f2l_red(f2l_shl(D, 1))});
  T.Z = f2l_red(f2l_shl(fm(m, A, D), 3));
  const F2L E = f2l_add(f2l_shl(C, 1), C);
  T.X = f2l_red(fm(m, XY, f2l_norm(f2l_sub<113, 3>(A, E))));
  const F2L C2 = fs<78, 1>(m, C);
  T.Y = f2l_red(f2l_sub<47, 12>(fs<78, 1>(m, f2l_norm(f2l_add(A, E))), f2l_add(f2l_shl(C2, 3), f2l_shl(C2, 2))));
}

// lazy28.py ladd: T + Q (Q affine, reduced), the chord through T and Q, put(Line28) as above
template <class Put, class M = F2One>
HD void l2_add_line(G2P28& T, const F2L& xq, const F2L& yq, const Put& put, M m = M()) {
  const F2L th = f2l_norm(f2l_sub<2, 1>(T.Y, fm(m, yq, T.Z)));
  const F2L la = f2l_norm(f2l_sub<2, 1>(T.X, fm(m, xq, T.Z)));
  put(Line28{f2l_red(f2l_sub<2, 1>(fm(m, th, xq), fm(m, la, yq))), f2l_red(f2l_sub<5, 1>(f2l_zero(), th)),
             f2l_red(la)});
  const F2L C = fs<78, 1>(m, th);
  const F2L D = fs<78, 1>(m, la);
  const F2L E = fm(m, la, D);
  const F2L G = fm(m, T.X, D);
  const F2L H = f2l_norm(f2l_sub<3, 2>(f2l_add(E, fm(m, T.Z, C)), f2l_shl(G, 1)));
  T.Z = f2l_red(fm(m, T.Z, E));
  T.Y = f2l_red(f2l_sub<2, 1>(fm(m, th, f2l_norm(f2l_sub<6, 1>(G, H))), fm(m, T.Y, E)));
  T.X = f2l_red(fm(m, la, H));
}

// a chain line as stored words; EVAL: evaluated at -g1 (c1 xP, c2 yP: products of reduced values
// are below 2p, joined as they are; counted like pairing.h line_eval's)
template <bool EVAL>
HD LineCoeffs line28_store(const Line28& l) {
  if (EVAL) {
    const L28 xp = l_from(fp_from_const(G1_GEN_X)), yp = l_from(fp_from_const(G1_GEN_NEG_Y));
    return {f2l_join(l.a0), {l_join(l_mul(l.a1.c0, xp)), l_join(l_mul(l.a1.c1, xp))},
            {l_join(l_mul(l.b1.c0, yp)), l_join(l_mul(l.b1.c1, yp))}};
  }
  return {f2l_join(l.a0), f2l_join(l.a1), f2l_join(l.b1)};
}

// The Miller chain of an affine G2 point (lines.h line_chain in lazy limbs): 68 lines, line j
// handed to put(j, LineCoeffs) (the stored-word line, pairing.h / layout.h LineEntry layout).
// load() returns Q again at each of the five additions (not held across the chain).
// line_chain28_st: each lazy line handed to store() first (e.g. evaluated at a variable P).
template <class LoadQ, class Store, class Put>
HD void line_chain28_st(const LoadQ& load, const Store& store, const Put& put) {
  const G2A Q = load();
  G2P28 T = {f2l_from(Q.x), f2l_from(Q.y), f2l_one()};
  int j = 0;
  auto emit = [&](const Line28& l) { put(j++, store(l)); };
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    l2_dbl_line(T, emit);
    if ((HB_X_ABS >> i) & 1) {
#if defined(__HIP_DEVICE_COMPILE__)
      __asm__ volatile("" ::: "memory");
#endif
      const G2A q2 = load();
      l2_add_line(T, f2l_from(q2.x), f2l_from(q2.y), emit);
    }
  }
}
template <bool EVAL, class LoadQ, class Put>
HD void line_chain28(const LoadQ& load, const Put& put) {
  line_chain28_st(load, [](const Line28& l) { return line28_store<EVAL>(l); }, put);
}

// ---- Fp4 = Fp2[s]/(s^2 - xi) in lazy limbs: the lane values of pair3.h's three-lane Fp12
struct F4L {
  F2L x, y;  // x + y s
};
HD F4L f4l_add(const F4L& a, const F4L& b) { return {f2l_add(a.x, b.x), f2l_add(a.y, b.y)}; }
template <uint32_t S, uint32_t T>
HD F4L f4l_sub(const F4L& a, const F4L& b) {
  return {f2l_sub<S, T>(a.x, b.x), f2l_sub<S, T>(a.y, b.y)};
}
HD F4L f4l_norm(const F4L& a) { return {f2l_norm(a.x), f2l_norm(a.y)}; }
HD F4L f4l_red(const F4L& a) { return {f2l_red(a.x), f2l_red(a.y)}; }
HD F4L f4l_select(bool take_b, const F4L& a, const F4L& b) {
  return {f2l_select(take_b, a.x, b.x), f2l_select(take_b, a.y, b.y)};
}
HD F4L f4l_from(const Fp2& x, const Fp2& y) { return {f2l_from(x), f2l_from(y)}; }
// (x + y s) s = xi y + x s
template <uint32_t S, uint32_t T>
HD F4L f4l_mul_s(const F4L& a) {
  return {f2l_xi<S, T>(a.y), a.x};
}
// lazy28.py f4_mul (Karatsuba, normalised): (t0 + xi t1, t2 - t0 - t1)
template <uint32_t XS, uint32_t XT, uint32_t YS, uint32_t YT, class M = F2One>
HD F4L f4l_mul(const F4L& a, const F4L& b, M m = M()) {
  F2L t0, t1, t2;
  fm3(m, a.x, b.x, a.y, b.y, f2l_add(a.x, a.y), f2l_add(b.x, b.y), t0, t1, t2);
  return f4l_norm({f2l_add(t0, f2l_xi<XS, XT>(t1)), f2l_sub<YS, YT>(t2, f2l_add(t0, t1))});
}
// lazy28.py f4_sqr: (x^2 + xi y^2, (x + y)^2 - x^2 - y^2), normalised
template <uint32_t XS, uint32_t XT, uint32_t YS, uint32_t YT, class M = F2One>
HD F4L f4l_sqr(const F4L& a, M m = M()) {
  F2L t0, t1, t2;
  fs3<9, 2>(m, a.x, a.y, f2l_norm(f2l_add(a.x, a.y)), t0, t1, t2);
  return f4l_norm({f2l_add(f2l_xi<XS, XT>(t1), t0), f2l_sub<YS, YT>(t2, f2l_add(t0, t1))});
}

// The lane operations of pair3.h in two phases around their lane exchanges, so that the host
// harness can run the three roles one after the other (tests/native/hostcheck.cpp) and the device
// (g4_sqr / g4_mul_line below) between ds_bpermutes.
// square (pair3.h g_sqr): phase 1 -- v = A^2, w = (A_p + A_q)^2 from the two roles != e(k);
// phase 2 -- D = w - v_p - v_q, C = Y + [k != 2] s X with (X, Y) = (D, v_e) for k = 0, else
// (v_e, D); reduced
template <class M = F2One>
HD void g4_sqr_p1(const F4L& A, const F4L& Ap, const F4L& Aq, F4L& v, F4L& w, M m = M()) {
  v = f4l_sqr<2, 1, 3, 2>(A, m);
  w = f4l_sqr<2, 1, 3, 2>(f4l_add(Ap, Aq), m);
}
HD F4L g4_sqr_p2(int k, const F4L& w, const F4L& vp, const F4L& vq, const F4L& ve) {
  const F4L D = f4l_sub<9, 2>(w, f4l_add(vp, vq));
  const F4L X = f4l_select(k != 0, D, ve), Y = f4l_select(k != 0, ve, D);
  const F4L sx = f4l_select(k == 2, f4l_mul_s<14, 4>(X), X);
  return f4l_red(f4l_add(Y, sx));
}
// product by a sparse line a0 + a1 v + b1 v w (pair3.h g_mul_line): phase 1 -- F a1, sent to the
// role before; phase 2 -- C = F (a0 + b1 s) + [k == 2 ? s : 1] (F_{k+1} a1); reduced
template <class M = F2One>
HD F4L g4_line_p1(const F4L& F, const F2L& a1, M m = M()) {
  F4L r;
  fm2(m, F.x, a1, F.y, a1, r.x, r.y);
  return r;
}
template <class M = F2One>
HD F4L g4_line_p2(int k, const F4L& F, const F2L& a0, const F2L& b1, const F4L& Qn, M m = M()) {
  const F4L Qs = f4l_select(k == 2, f4l_mul_s<2, 1>(Qn), Qn);  // k == 2 ? Qn : s Qn
  return f4l_red(f4l_add(f4l_mul<2, 1, 3, 2>(F, F4L{a0, b1}, m), Qs));
}
// ---- the final exponentiation's lane operations (pair3.h g_cyclo_sqr / g_mul / g_conj / g_frob)
// in lazy limbs: lane values reduced (< 2p) in and out (lazy28.py g4_cyc / g4_mul / g4_conj /
// g4_frob, sites "4C*", "4M*", "4J*", "4F*").
// cyclotomic square: phase 1 -- t = A^2, sent to role e(k); phase 2 -- from the received te,
// ts = s te for k = 1, else te; (3 ts.x - 2 A.x, 3 ts.y + 2 A.y), for k = 1 (3 ts.x + 2 A.x,
// 3 ts.y - 2 A.y), the negated terms as K - 2A
template <class M = F2One>
HD F4L g4_cyc_p1(const F4L& A, M m = M()) { return f4l_sqr<2, 1, 3, 2>(A, m); }
HD F4L g4_cyc_p2(int k, const F4L& te, const F4L& A) {
  const F4L ts = f4l_select(k == 1, te, f4l_mul_s<5, 1>(te));
  const F2L x3 = f2l_add(f2l_shl(ts.x, 1), ts.x), y3 = f2l_add(f2l_shl(ts.y, 1), ts.y);
  const F2L ax2 = f2l_shl(A.x, 1), ay2 = f2l_shl(A.y, 1);
  const F2L nx = f2l_sub<5, 2>(f2l_zero(), ax2), ny = f2l_sub<5, 2>(f2l_zero(), ay2);
  return f4l_red({f2l_add(x3, f2l_select(k == 1, nx, ax2)), f2l_add(y3, f2l_select(k == 1, ay2, ny))});
}
// product (Karatsuba over the roles): phase 1 -- v = A B, w = (A_p + A_q)(B_p + B_q), the sums
// normalised; phase 2 -- g4_sqr_p2's recombination (the same constants suffice, lazy28.py g4_mul)
// (sa = A_p + A_q, sb = B_p + B_q: formed by the caller as the exchanged values arrive)
template <class M = F2One>
HD void g4_mul_p1(const F4L& A, const F4L& B, const F4L& sa, const F4L& sb, F4L& v, F4L& w, M m = M()) {
  v = f4l_mul<2, 1, 3, 2>(A, B, m);
  w = f4l_mul<2, 1, 3, 2>(f4l_norm(sa), f4l_norm(sb), m);
}
// f -> f^(p^6): (-x, y) for k = 1, else (x, -y); reduced
HD F4L g4_conj(int k, const F4L& A) {
  const F2L nx = f2l_sub<3, 1>(f2l_zero(), A.x), ny = f2l_sub<3, 1>(f2l_zero(), A.y);
  return f4l_red({f2l_select(k == 1, A.x, nx), f2l_select(k == 1, ny, A.y)});
}
// f -> f^(p^J): the Fp2 coefficients conjugated for odd J, times FROBJ[k], FROBJ[k + 3] (products
// of reduced values: below 2p as they come)
template <int J, class M = F2One>
HD F4L g4_frob(int k, const F4L& A, M m = M()) {
  const uint32_t(*tab)[2][12] = (J == 1) ? FROB1 : (J == 2) ? FROB2 : FROB3;
  const F2L cx = f2l_from(f2_from_const(tab[k])), cy = f2l_from(f2_from_const(tab[k + 3]));
  F2L x = A.x, y = A.y;
  if (J & 1) {
    x.c1 = l_sub<3, 1>(l_zero(), x.c1);
    y.c1 = l_sub<3, 1>(l_zero(), y.c1);
  }
  F4L r;
  fm2(m, x, cx, y, cy, r.x, r.y);
  return r;
}
HD Fp4 f4l_join(const F4L& a) { return {f2l_join(a.x), f2l_join(a.y)}; }

HD F4L g4_one_role(int k) {
  F4L r = {f2l_zero(), f2l_zero()};
  if (k == 0) r.x = f2l_one();
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// The lane steps on the device: pair3.h's exchanges (ds_bpermute) around the two phases
__device__ __forceinline__ L28 xch(const L28& a, int addr) {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = xch(a.l[i], addr);
  return r;
}
__device__ __forceinline__ F2L xch(const F2L& a, int addr) { return {xch(a.c0, addr), xch(a.c1, addr)}; }
__device__ __forceinline__ F4L xch(const F4L& a, int addr) { return {xch(a.x, addr), xch(a.y, addr)}; }

// Eighteen lanes per Fp12 value: each role k of pair3.h held by SIX lanes j = 0..5 (lane = 18 grp +
// 6 k + j, three values per wavefront, lanes 54..63 shadow a group), which run a role's independent
// Fp2 products side by side -- lane j computes coefficient j & 1 of product j >> 1 of a batch of
// three (fm3 / fs3; fm2 leaves lanes 4, 5 duplicating) and every lane gathers the six results.  The
// lane values stay duplicated over the six lanes; each lane's stream holds one Fp product per batch
// instead of the three (Grp6) or six (Grp) -- the final exponentiations of single calls and of the
// slot-wide check, which nothing else hides.
struct F2Hex {
  int j;
  int at[6];  // the role's six lanes (ds_bpermute addresses)
};
struct Grp18 {
  int k, j;
  int n1, n2, e, p, q;  // pair3.h Grp's exchanges, between lanes of the same j
  F2Hex hx;
};
__device__ __forceinline__ Grp18 grp18_make() {
  const int lane = (int)(threadIdx.x & 63u);
  const int grp = lane / 18, r = lane - 18 * grp;
  Grp18 g;
  g.k = r / 6;
  g.j = r - 6 * g.k;
  const int base = 18 * grp;
  auto at = [&](int role, int jj) { return ((base + 6 * role + jj) & 63) << 2; };
  g.n1 = at((g.k + 1) % 3, g.j);
  g.n2 = at((g.k + 2) % 3, g.j);
  g.e = at((3 - g.k) % 3, g.j);
  g.p = at(g.k == 0 ? 1 : 0, g.j);
  g.q = at(g.k == 0 ? 2 : g.k, g.j);
  g.hx.j = g.j;
  HB_UNROLL for (int jj = 0; jj < 6; jj++) g.hx.at[jj] = at(g.k, jj);
  return g;
}
// the pair3.h lane group seen from one j (the inversion and the final test run duplicated)
__device__ __forceinline__ Grp grp_of(const Grp18& g) { return {g.k, g.n1, g.n2, g.e, g.p, g.q}; }

__device__ __forceinline__ F2L f2hex_pick3(int w, const F2L& a0, const F2L& a1, const F2L& a2) {
  return f2l_select(w == 2, f2l_select(w == 1, a0, a1), a2);
}
__device__ __forceinline__ void f2hex_gather(const F2Hex& m, const L28& mine, F2L& t0, F2L& t1, F2L& t2) {
  t0 = {l_xch(mine, m.at[0]), l_xch(mine, m.at[1])};
  t1 = {l_xch(mine, m.at[2]), l_xch(mine, m.at[3])};
  t2 = {l_xch(mine, m.at[4]), l_xch(mine, m.at[5])};
}
// coefficient j & 1 of a_w b_w, w = j >> 1 (ec28.h fm(F2Half)'s operand choice)
__device__ __forceinline__ L28 f2hex_dot(const F2Hex& m, const F2L& a, const F2L& b) {
  L28 na1;
  HB_UNROLL for (int i = 0; i < 14; i++) na1.l[i] = kF2N.l[i] - a.c1.l[i];
  const bool h = (m.j & 1) != 0;
  return l_dot(a.c0, l_pick(h, na1, a.c1), l_pick(h, b.c0, b.c1), l_pick(h, b.c1, b.c0));
}
__device__ __forceinline__ void fm3(const F2Hex& m, const F2L& a0, const F2L& b0, const F2L& a1, const F2L& b1,
                                    const F2L& a2, const F2L& b2, F2L& t0, F2L& t1, F2L& t2) {
  const int w = m.j >> 1;
  f2hex_gather(m, f2hex_dot(m, f2hex_pick3(w, a0, a1, a2), f2hex_pick3(w, b0, b1, b2)), t0, t1, t2);
}
__device__ __forceinline__ void fm2(const F2Hex& m, const F2L& a0, const F2L& b0, const F2L& a1, const F2L& b1, F2L& t0,
                                    F2L& t1) {
  const bool w1 = m.j >= 2;  // lanes 4, 5 repeat product 1
  F2L u0, u1, u2;
  f2hex_gather(m, f2hex_dot(m, f2l_select(w1, a0, a1), f2l_select(w1, b0, b1)), u0, u1, u2);
  t0 = u0;
  t1 = u1;
}
template <uint32_t S, uint32_t T>
__device__ __forceinline__ void fs3(const F2Hex& m, const F2L& a0, const F2L& a1, const F2L& a2, F2L& t0, F2L& t1,
                                    F2L& t2) {
  const F2L u = f2hex_pick3(m.j >> 1, a0, a1, a2);
  const bool h = (m.j & 1) != 0;
  f2hex_gather(m, l_mul(l_pick(h, l_add(u.c0, u.c1), l_shl(u.c0, 1)), l_pick(h, l_sub<S, T>(u.c0, u.c1), u.c1)), t0,
               t1, t2);
}

// Over a lane group G: Grp (three lanes, pair3.h; each lane its products alone), Grp6 (six lanes,
// pair6.h; each Fp2 product split over the role's two lanes, ec28.h F2Half) or Grp18 (above)
__device__ __forceinline__ F2One fe_m(const Grp&) { return {}; }
__device__ __forceinline__ F2Half fe_m(const Grp6& g) { return {g.h, g.partner}; }
__device__ __forceinline__ const F2Hex& fe_m(const Grp18& g) { return g.hx; }
template <class G>
__device__ __forceinline__ F4L g4_one(const G& g) { return g4_one_role(g.k); }
template <class G>
__device__ __forceinline__ F4L g4_sqr(const G& g, const F4L& A) {
  F4L v, w;
  g4_sqr_p1(A, xch(A, g.p), xch(A, g.q), v, w, fe_m(g));
  return g4_sqr_p2(g.k, w, xch(v, g.p), xch(v, g.q), xch(v, g.e));
}
template <class G>
__device__ __forceinline__ F4L g4_mul_line(const G& g, const F4L& F, const F2L& a0, const F2L& a1, const F2L& b1) {
  return g4_line_p2(g.k, F, a0, b1, xch(g4_line_p1(F, a1, fe_m(g)), g.n1), fe_m(g));
}

// The final exponentiation in lazy limbs over G.  The one inversion runs in stored words (pair3.h
// g_inv / pair6.h g6_inv).
__device__ __forceinline__ Fp4 fe_inv(const Grp& g, const Fp4& A) { return g_inv(g, A); }
__device__ __forceinline__ Fp4 fe_inv(const Grp6& g, const Fp4& A) { return g6_inv(g, A); }
__device__ __forceinline__ bool fe_is_one(const Grp& g, const Fp4& A) { return g_is_one(g, A); }
__device__ __forceinline__ bool fe_is_one(const Grp6& g, const Fp4& A) { return g6_is_one(g, A); }
__device__ __forceinline__ Fp4 fe_inv(const Grp18& g, const Fp4& A) { return g_inv(grp_of(g), A); }
__device__ __forceinline__ bool fe_is_one(const Grp18& g, const Fp4& A) { return g_is_one(grp_of(g), A); }

template <class G>
__device__ __forceinline__ F4L g4_cyc(const G& g, const F4L& A) {
  return g4_cyc_p2(g.k, xch(g4_cyc_p1(A, fe_m(g)), g.e), A);
}
template <class G>
__device__ __forceinline__ F4L g4_mul(const G& g, const F4L& A, const F4L& B) {
  F4L v, w;
  const F4L sa = f4l_add(xch(A, g.p), xch(A, g.q));
  const F4L sb = f4l_add(xch(B, g.p), xch(B, g.q));
  g4_mul_p1(A, B, sa, sb, v, w, fe_m(g));
  return g4_sqr_p2(g.k, w, xch(v, g.p), xch(v, g.q), xch(v, g.e));
}
template <class G>
__device__ __forceinline__ F4L g4_pow_x(const G& g, const F4L& f) {
  F4L r = f;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = g4_cyc(g, r);
    if ((HB_X_ABS >> i) & 1) r = g4_mul(g, r, f);
  }
  return g4_conj(g.k, r);
}
// pair3.h g_final_exp's chain
template <class G>
__device__ __forceinline__ F4L g4_final_exp(const G& g, const F4L& f) {
  const Fp4 fi = fe_inv(g, f4l_join(f));
  F4L t = g4_mul(g, g4_conj(g.k, f), f4l_from(fi.x, fi.y));
  t = g4_mul(g, g4_frob<2>(g.k, t, fe_m(g)), t);
  F4L x = t, b = t;
  HB_NOUNROLL for (int s = 0; s < 5; s++) {
    const F4L px = g4_pow_x(g, x);
    if (s == 3) b = x;
    if (s < 2) x = g4_mul(g, px, g4_conj(g.k, x));
    else if (s == 2) x = g4_mul(g, px, g4_frob<1>(g.k, x, fe_m(g)));
    else x = px;
  }
  const F4L c = g4_mul(g, g4_mul(g, x, g4_frob<2>(g.k, b, fe_m(g))), g4_conj(g.k, b));
  return g4_mul(g, c, g4_mul(g, g4_cyc(g, t), t));
}
template <class G>
__device__ __forceinline__ bool g4_is_one(const G& g, const F4L& A) { return fe_is_one(g, f4l_join(A)); }
#endif

}  // namespace hb
