// Lane-group pairing: one Fp12 value spread over THREE lanes of a wavefront.
//
// Why: a one-lane pairing holds f (144 VGPRs) + the G2 line state + temporaries, which does not
// fit in 256 VGPRs, and a slot of 40k partials gives only 625 waves for 1024 SIMDs.  Viewing
// Fp12 as a cubic extension of Fp4,
//     Fp4  = Fp2[s]/(s^2 - xi),  s = w^3          (xi = 1 + u)
//     Fp12 = Fp4[w]/(w^3 - s),   f = A0 + A1 w + A2 w^2,
// lane k of a group owns A_k (48 VGPRs).  In the tower basis of tower.h (f = c0 + c1 w over
// Fp6 = Fp2[v], v = w^2) the coefficient of w^i is z_i with
//     z0 = c0.c0, z1 = c1.c0, z2 = c0.c1, z3 = c1.c1, z4 = c0.c2, z5 = c1.c2,
// and A_k = (z_k, z_{k+3}).  Every Fp12 operation becomes the same instruction stream in the
// three lanes (no divergence) plus a few lane exchanges (ds_bpermute):
//   product      Karatsuba over Fp4: 6 Fp4 products = 2 per lane  (18 Fp-mul per lane)
//   square       3 Fp4 squares + 3 cross squares = 2 per lane     (12 Fp-mul per lane)
//   cyclotomic   Granger-Scott: one Fp4 square per lane            ( 6 Fp-mul per lane)
//   line product sparse line (a0 + a1 v + b1 v w)                  (15 Fp-mul per lane)
// A wavefront holds 21 groups (lanes 0..62; lane 63 computes on garbage and is never stored).
// The lines of the Miller loop are precomputed (pairing.h miller_*_c) by one-lane kernels and
// streamed from memory, so the lane group carries no G2 state.
//
// Device-only (uses the LDS crossbar permute); the host path keeps the one-lane tower code.
#pragma once
#include "ops.h"

namespace hb {

struct Fp4 {
  Fp2 x, y;  // x + y s
};

HD Fp4 f4_add(const Fp4& a, const Fp4& b) { return {f2_add(a.x, b.x), f2_add(a.y, b.y)}; }
HD Fp4 f4_sub(const Fp4& a, const Fp4& b) { return {f2_sub(a.x, b.x), f2_sub(a.y, b.y)}; }
HD Fp4 f4_zero() { return {f2_zero(), f2_zero()}; }
// (x + y s) s = xi y + x s
HD Fp4 f4_mul_s(const Fp4& a) { return {f2_mul_xi(a.y), a.x}; }

// 3 Fp2 products (9 Fp products)
HD Fp4 f4_mul(const Fp4& a, const Fp4& b) {
  Fp2 t0 = f2_mul(a.x, b.x);
  Fp2 t1 = f2_mul(a.y, b.y);
  Fp2 t2 = f2_mul(f2_add(a.x, a.y), f2_add(b.x, b.y));
  return {f2_add(t0, f2_mul_xi(t1)), f2_sub(f2_sub(t2, t0), t1)};
}

HD Fp4 f4_sqr(const Fp4& a) {
  Fp4 r;
  fp4_sqr(r.x, r.y, a.x, a.y);
  return r;
}

HD Fp4 f4_mul_f2(const Fp4& a, const Fp2& b) { return {f2_mul(a.x, b), f2_mul(a.y, b)}; }

HD void f4_select(Fp4& r, bool take_b, const Fp4& a, const Fp4& b) {
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.x.c0.v[i] = take_b ? b.x.c0.v[i] : a.x.c0.v[i];
    r.x.c1.v[i] = take_b ? b.x.c1.v[i] : a.x.c1.v[i];
    r.y.c0.v[i] = take_b ? b.y.c0.v[i] : a.y.c0.v[i];
    r.y.c1.v[i] = take_b ? b.y.c1.v[i] : a.y.c1.v[i];
  }
}

#if defined(__HIP_DEVICE_COMPILE__)

// The three lanes of a group: k = role (0, 1, 2).  Exchange addresses (ds_bpermute byte
// addresses = lane << 2), precomputed per lane:
//   n1, n2  lanes of roles k+1, k+2
//   e       lane of role e(k) = (3 - k) % 3   (0 -> 0, 1 -> 2, 2 -> 1)
//   p, q    the two roles other than e(k)
struct Grp {
  int k;
  int n1, n2, e, p, q;
};

__device__ __forceinline__ Grp grp_make() {
  int lane = (int)(threadIdx.x & 63u);
  int grp = lane / 3;
  Grp g;
  g.k = lane - 3 * grp;
  int base = 3 * grp;
  g.n1 = ((base + (g.k + 1) % 3) & 63) << 2;
  g.n2 = ((base + (g.k + 2) % 3) & 63) << 2;
  g.e = ((base + (3 - g.k) % 3) & 63) << 2;
  // roles != e(k): k=0 -> {1, 2}; k=1 -> {0, 1}; k=2 -> {0, 2}
  g.p = ((base + (g.k == 0 ? 1 : 0)) & 63) << 2;
  g.q = ((base + (g.k == 0 ? 2 : g.k)) & 63) << 2;
  return g;
}

__device__ __forceinline__ uint32_t xch(uint32_t v, int addr) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
}
__device__ __forceinline__ Fp xch(const Fp& a, int addr) {
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = xch(a.v[i], addr);
  return r;
}
__device__ __forceinline__ Fp2 xch(const Fp2& a, int addr) { return {xch(a.c0, addr), xch(a.c1, addr)}; }
__device__ __forceinline__ Fp4 xch(const Fp4& a, int addr) { return {xch(a.x, addr), xch(a.y, addr)}; }

// pick one of three per-lane candidates by role (selects: no divergence)
__device__ __forceinline__ Fp4 pick3(int role, const Fp4& r0, const Fp4& r1, const Fp4& r2) {
  Fp4 t;
  f4_select(t, role == 1, r0, r1);
  f4_select(t, role == 2, t, r2);
  return t;
}

// ---- conversions between the tower Fp12 and the lane form ----
__device__ __forceinline__ Fp4 g_from_f12(const Grp& g, const Fp12& f) {
  return pick3(g.k, Fp4{f.c0.c0, f.c1.c1}, Fp4{f.c1.c0, f.c0.c2}, Fp4{f.c0.c1, f.c1.c2});
}

__device__ __forceinline__ Fp4 g_one(const Grp& g) {
  Fp4 r;
  f4_select(r, g.k != 0, Fp4{f2_one(), f2_zero()}, f4_zero());
  return r;
}

// Karatsuba recombination shared by g_mul / g_sqr.  With v_k = A_k B_k,
// w_k = (A_p + A_q)(B_p + B_q) over the two roles p, q != e(k), and D = w_k - v_p - v_q:
//   k = 0: C0 = v0 + s D          (D = w0 - v1 - v2)
//   k = 1: C1 = D + s v2          (D = w1 - v0 - v1)
//   k = 2: C2 = D + v1            (D = w2 - v0 - v2)
// i.e. C = Y + [k != 2] s X with (X, Y) = (D, v_e) for k = 0 and (v_e, D) otherwise.
__device__ __forceinline__ Fp4 g_recombine(const Grp& g, const Fp4& v, const Fp4& w) {
  Fp4 D = f4_sub(f4_sub(w, xch(v, g.p)), xch(v, g.q));
  Fp4 ve = xch(v, g.e);
  Fp4 X, Y, sx;
  f4_select(X, g.k != 0, D, ve);
  f4_select(Y, g.k != 0, ve, D);
  f4_select(sx, g.k == 2, f4_mul_s(X), X);
  return f4_add(Y, sx);
}

// f * f' (Karatsuba over Fp4: 2 Fp4 products per lane)
__device__ __forceinline__ Fp4 g_mul(const Grp& g, const Fp4& A, const Fp4& B) {
  Fp4 sa = f4_add(xch(A, g.p), xch(A, g.q));
  Fp4 sb = f4_add(xch(B, g.p), xch(B, g.q));
  Fp4 v = f4_mul(A, B);
  Fp4 w = f4_mul(sa, sb);
  return g_recombine(g, v, w);
}

// general square (Miller loop): 2 Fp4 squares per lane
__device__ __forceinline__ Fp4 g_sqr(const Grp& g, const Fp4& A) {
  Fp4 sa = f4_add(xch(A, g.p), xch(A, g.q));
  Fp4 v = f4_sqr(A);
  Fp4 w = f4_sqr(sa);
  return g_recombine(g, v, w);
}

// cyclotomic square (Granger-Scott, cf. f12_cyclo_sqr): lane k squares its own Fp4 and takes
// the square t of lane e(k):
//   k = 0: (3 t.x - 2 A.x, 3 t.y + 2 A.y)
//   k = 1: (3 xi t.y + 2 A.x, 3 t.x - 2 A.y)
//   k = 2: (3 t.x - 2 A.x, 3 t.y + 2 A.y)
__device__ __forceinline__ Fp4 g_cyclo_sqr(const Grp& g, const Fp4& A) {
  Fp4 te = xch(f4_sqr(A), g.e);
  Fp4 ts;
  f4_select(ts, g.k == 1, te, f4_mul_s(te));  // k = 1 uses (xi t.y, t.x)
  Fp2 x3 = f2_add(f2_dbl(ts.x), ts.x), y3 = f2_add(f2_dbl(ts.y), ts.y);
  Fp2 ax2 = f2_dbl(A.x), ay2 = f2_dbl(A.y);
  Fp4 r;
  f4_select(r, g.k == 1, Fp4{f2_sub(x3, ax2), f2_add(y3, ay2)}, Fp4{f2_add(x3, ax2), f2_sub(y3, ay2)});
  return r;
}

// f * (a0 + a1 v + b1 v w):  L0 = (a0, b1), L1 = 0, L2 = (a1, 0)
//   C0 = F0 L0 + s F1 a1,  C1 = F1 L0 + s F2 a1,  C2 = F2 L0 + F0 a1
__device__ __forceinline__ Fp4 g_mul_line(const Grp& g, const Fp4& F, const Fp2& a0, const Fp2& a1, const Fp2& b1) {
  Fp4 Qn = xch(f4_mul_f2(F, a1), g.n1);
  Fp4 Qs;
  f4_select(Qs, g.k == 2, f4_mul_s(Qn), Qn);
  return f4_add(f4_mul(F, Fp4{a0, b1}), Qs);
}

// conjugation f -> f^(p^6): c1 -> -c1, i.e. z1, z3, z5 negated
__device__ __forceinline__ Fp4 g_conj(const Grp& g, const Fp4& A) {
  Fp4 r;
  f4_select(r, g.k == 1, Fp4{A.x, f2_neg(A.y)}, Fp4{f2_neg(A.x), A.y});
  return r;
}

// Frobenius x -> x^(p^J): conjugate the Fp2 coefficients (J odd) and scale z_i by FROBJ[i]
template <int J>
__device__ __forceinline__ Fp4 g_frob(const Grp& g, const Fp4& A) {
  const uint32_t(*tab)[2][12] = (J == 1) ? FROB1 : (J == 2) ? FROB2 : FROB3;
  Fp2 cx = f2_from_const(tab[g.k]), cy = f2_from_const(tab[g.k + 3]);
  Fp2 x = (J & 1) ? f2_conj(A.x) : A.x;
  Fp2 y = (J & 1) ? f2_conj(A.y) : A.y;
  return {f2_mul(x, cx), f2_mul(y, cy)};
}

// inverse via the cubic adjugate: B0 = A0^2 - s A1 A2, B1 = s A2^2 - A0 A1, B2 = A1^2 - A0 A2,
// N = A0 B0 + s (A1 B2 + A2 B1) in Fp4, A^-1 = B / N.  Once per final exponentiation.
__device__ __forceinline__ Fp4 g_inv(const Grp& g, const Fp4& A) {
  Fp4 A1 = xch(A, g.n1), A2 = xch(A, g.n2);  // A_{k+1}, A_{k+2}
  Fp4 X0 = pick3(g.k, A, A2, A1);            // A_0, A_1, A_2 seen from lane k
  Fp4 X1 = pick3(g.k, A1, A, A2);
  Fp4 X2 = pick3(g.k, A2, A1, A);
  Fp4 sq = f4_sqr(pick3(g.k, X0, X2, X1));                           // A0^2 | A2^2 | A1^2
  Fp4 pr = f4_mul(pick3(g.k, X1, X0, X0), pick3(g.k, X2, X1, X2));  // A1A2 | A0A1 | A0A2
  Fp4 B = pick3(g.k, f4_sub(sq, f4_mul_s(pr)), f4_sub(f4_mul_s(sq), pr), f4_sub(sq, pr));
  Fp4 T = f4_mul(A, xch(B, g.e));  // T_k = A_k B_e: A0B0 | A1B2 | A2B1
  Fp4 T1 = xch(T, g.n1), T2 = xch(T, g.n2);
  Fp4 N = f4_add(pick3(g.k, T, T2, T1), f4_mul_s(f4_add(pick3(g.k, T1, T, T2), pick3(g.k, T2, T1, T))));
  // (x + y s)^-1 = (x - y s) / (x^2 - xi y^2)
  Fp2 d = f2_sub(f2_sqr(N.x), f2_mul_xi(f2_sqr(N.y)));
  Fp2 di = f2_inv(d);
  return f4_mul(B, Fp4{f2_mul(N.x, di), f2_neg(f2_mul(N.y, di))});
}

__device__ __forceinline__ Fp4 g_pow_xabs(const Grp& g, const Fp4& f) {
  Fp4 r = f;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = g_cyclo_sqr(g, r);
    if ((HB_X_ABS >> i) & 1) r = g_mul(g, r, f);
  }
  return r;
}
__device__ __forceinline__ Fp4 g_pow_x(const Grp& g, const Fp4& f) { return g_conj(g, g_pow_xabs(g, f)); }

// f^(3 (p^12 - 1) / r), same chain as final_exponentiation (pairing.h).  The five f^x share one
// loop (stage s), so the exponentiation code exists once:
//   s0: a = t^x conj(t)   s1: a = a^x conj(a)   s2: b = a^x frob1(a)   s3: c = b^x   s4: c = c^x
__device__ __forceinline__ Fp4 g_final_exp(const Grp& g, const Fp4& f) {
  Fp4 t = g_mul(g, g_conj(g, f), g_inv(g, f));
  t = g_mul(g, g_frob<2>(g, t), t);
  Fp4 x = t, b = t;
  HB_NOUNROLL for (int s = 0; s < 5; s++) {
    Fp4 px = g_pow_x(g, x);
    if (s == 3) b = x;  // keep b for the last step
    if (s < 2) x = g_mul(g, px, g_conj(g, x));  // s is wave-uniform: plain branches
    else if (s == 2) x = g_mul(g, px, g_frob<1>(g, x));
    else x = px;
  }
  Fp4 c = g_mul(g, g_mul(g, x, g_frob<2>(g, b)), g_conj(g, b));
  return g_mul(g, c, g_mul(g, g_cyclo_sqr(g, t), t));
}

// true in every lane of the group iff f == 1
__device__ __forceinline__ bool g_is_one(const Grp& g, const Fp4& A) {
  bool mine = g.k == 0 ? (f2_eq(A.x, f2_one()) && f2_is_zero(A.y)) : (f2_is_zero(A.x) && f2_is_zero(A.y));
  uint32_t m = mine ? 1u : 0u;
  return (m & xch(m, g.n1) & xch(m, g.n2)) != 0;
}

#endif  // __HIP_DEVICE_COMPILE__

}  // namespace hb
