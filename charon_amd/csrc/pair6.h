// Six-lane final exponentiation: the lane-group Fp12 of pair3.h (role k = 0, 1, 2 owns A_k in Fp4)
// with each role held by TWO lanes h = 0, 1 that split every Fp2 product: lane h computes output
// coefficient h only and takes the other from its partner (one 12-dword exchange).
//
// Why: a slot's verification ends in ONE final exponentiation (the slot-wide check, or one per
// batch of groups), a chain of ~320 cyclotomic squarings and ~40 products that no amount of other
// work hides for small slots and single calls (C2, one tbls.Verify).  Its latency is the length of
// each lane's dependent instruction stream; with the Fp2 products split, every product in the chain
// costs each lane one two-term Montgomery pass (2 x 196 + 196 multiply-adds) instead of the full
// single-pass Fp2 product (6 x 196), and a square one plain product.  The additions stay duplicated
// in both lanes (cheap), so both lanes of a role always hold the whole Fp4 value.
//
//   coefficient 0 of a b:  a0 b0 - a1 b1        coefficient 1: a0 b1 + a1 b0
//   coefficient 0 of a^2:  (a0 + a1)(a0 - a1)   coefficient 1: 2 a0 a1
//
// The same uniform instruction stream in every lane (operands chosen by select), so the halves
// never diverge.  Lane layout: lane = 6 grp + 2 k + h, ten groups per wavefront (lanes 60..63 idle).
// Device-only; the results equal pair3.h g_final_exp's (the same formulas, the same group element).
#pragma once
#include "pair3.h"

namespace hb {

#if defined(__HIP_DEVICE_COMPILE__)

// c = x0 y0 + (neg ? -1 : 1) x1 y1, one Montgomery reduction (R = 2^392), result in [0, 2p): the
// single-accumulator pass of fp2_mul_core with the sign a per-lane operand (signed multiply-adds
// against the conditionally negated limbs of x1; a negative column total gets p added at the end)
HD void fp_dot2_core(uint32_t* out, const uint32_t* x0w, const uint32_t* y0w, const uint32_t* x1w,
                     const uint32_t* y1w, bool neg) {
  uint32_t x0[14], y0[14], x1[14], y1[14], m[14], r[14];
  int32_t s1[14];
  fp_split28(x0, x0w);
  fp_split28(y0, y0w);
  fp_split28(x1, x1w);
  fp_split28(y1, y1w);
  HB_UNROLL for (int j = 0; j < 14; j++) s1[j] = neg ? -(int32_t)x1[j] : (int32_t)x1[j];
  uint64_t acc = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      acc += (uint64_t)x0[j] * y0[k - j];
      acc += (uint64_t)((int64_t)s1[j] * (int64_t)(int32_t)y1[k - j]);
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P28[k - j];
    HB_MONT28_TAIL_S(acc, m, k, r)
  }
  r[13] = (uint32_t)acc;
  fp2_fix_neg(out, r, (int64_t)acc < 0);
}

// leaf: x0, x1 in registers, y0, y1 through the per-lane LDS slot of fp2_mul_leaf
__device__ __noinline__ static u32x12 fp_dot2_leaf(u32x24 a, uint32_t neg) {
  uint32_t x0[12], x1[12], y0[12], y1[12], r[12];
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 6; k++) {
    const uint2 v = hb_fp2_arg[k * HB_ARG_LANES + lane], w = hb_fp2_arg[(6 + k) * HB_ARG_LANES + lane];
    y0[2 * k] = v.x;
    y0[2 * k + 1] = v.y;
    y1[2 * k] = w.x;
    y1[2 * k + 1] = w.y;
  }
  HB_UNROLL for (int i = 0; i < 12; i++) {
    x0[i] = a[i];
    x1[i] = a[12 + i];
  }
  fp_dot2_core(r, x0, y0, x1, y1, neg != 0);
  u32x12 o;
  HB_UNROLL for (int i = 0; i < 12; i++) o[i] = r[i];
  return o;
}

__device__ __forceinline__ Fp fp_dot2(const Fp& x0, const Fp& y0, const Fp& x1, const Fp& y1, bool neg) {
  u32x24 av;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    av[i] = x0.v[i];
    av[12 + i] = x1.v[i];
  }
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 6; k++) {
    hb_fp2_arg[k * HB_ARG_LANES + lane] = make_uint2(y0.v[2 * k], y0.v[2 * k + 1]);
    hb_fp2_arg[(6 + k) * HB_ARG_LANES + lane] = make_uint2(y1.v[2 * k], y1.v[2 * k + 1]);
  }
  const u32x12 rv = fp_dot2_leaf(av, neg ? 1u : 0u);
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = rv[i];
  return r;
}

// Roles as pair3.h's Grp, each lane also knowing its half and its partner
struct Grp6 {
  int k, h;
  int n1, n2, e, p, q, partner;
};

__device__ __forceinline__ Grp6 grp6_make() {
  const int lane = (int)(threadIdx.x & 63u);
  const int grp = lane / 6;
  Grp6 g;
  const int r = lane - 6 * grp;
  g.k = r >> 1;
  g.h = r & 1;
  const int base = 6 * grp;
  auto at = [&](int role) { return ((base + 2 * role + g.h) & 63) << 2; };
  g.n1 = at((g.k + 1) % 3);
  g.n2 = at((g.k + 2) % 3);
  g.e = at((3 - g.k) % 3);
  g.p = at(g.k == 0 ? 1 : 0);
  g.q = at(g.k == 0 ? 2 : g.k);
  g.partner = ((lane ^ 1) & 63) << 2;
  return g;
}

// the Fp2 from this lane's coefficient and the partner's
__device__ __forceinline__ Fp2 h_join(const Grp6& g, const Fp& mine) {
  const Fp other = xch(mine, g.partner);
  Fp2 r;
  fp_select(r.c0, g.h != 0, mine, other);
  fp_select(r.c1, g.h != 0, other, mine);
  return r;
}

__device__ __forceinline__ Fp2 h2_mul(const Grp6& g, const Fp2& a, const Fp2& b) {
  HB_COUNT_FP_MUL();
  Fp y0, y1;
  fp_select(y0, g.h != 0, b.c0, b.c1);
  fp_select(y1, g.h != 0, b.c1, b.c0);
  return h_join(g, fp_dot2(a.c0, y0, a.c1, y1, g.h == 0));
}

__device__ __forceinline__ Fp2 h2_sqr(const Grp6& g, const Fp2& a) {
  HB_COUNT_FP_MUL();
  Fp x, y;
  fp_select(x, g.h != 0, fp_add(a.c0, a.c1), fp_dbl(a.c0));
  fp_select(y, g.h != 0, fp_sub(a.c0, a.c1), a.c1);
  return h_join(g, fp_mul(x, y));
}

// Fp4 = Fp2[s]/(s^2 - xi) with the split products (f4_mul / fp4_sqr of pair3.h / pairing.h)
__device__ __forceinline__ Fp4 h4_mul(const Grp6& g, const Fp4& a, const Fp4& b) {
  const Fp2 t0 = h2_mul(g, a.x, b.x);
  const Fp2 t1 = h2_mul(g, a.y, b.y);
  const Fp2 t2 = h2_mul(g, f2_add(a.x, a.y), f2_add(b.x, b.y));
  return {f2_add(t0, f2_mul_xi(t1)), f2_sub(f2_sub(t2, t0), t1)};
}

__device__ __forceinline__ Fp4 h4_sqr(const Grp6& g, const Fp4& a) {
  const Fp2 t0 = h2_sqr(g, a.x), t1 = h2_sqr(g, a.y);
  return {f2_add(f2_mul_xi(t1), t0), f2_sub(f2_sub(h2_sqr(g, f2_add(a.x, a.y)), t0), t1)};
}

// ---- pair3.h's lane-group Fp12 operations over six lanes ----
__device__ __forceinline__ Fp4 g6_one(const Grp6& g) {
  Fp4 r;
  f4_select(r, g.k != 0, Fp4{f2_one(), f2_zero()}, f4_zero());
  return r;
}

__device__ __forceinline__ Fp4 g6_recombine(const Grp6& g, const Fp4& v, const Fp4& w) {
  Fp4 D = f4_sub(f4_sub(w, xch(v, g.p)), xch(v, g.q));
  Fp4 ve = xch(v, g.e);
  Fp4 X, Y, sx;
  f4_select(X, g.k != 0, D, ve);
  f4_select(Y, g.k != 0, ve, D);
  f4_select(sx, g.k == 2, f4_mul_s(X), X);
  return f4_add(Y, sx);
}

__device__ __forceinline__ Fp4 g6_mul(const Grp6& g, const Fp4& A, const Fp4& B) {
  const Fp4 sa = f4_add(xch(A, g.p), xch(A, g.q));
  const Fp4 sb = f4_add(xch(B, g.p), xch(B, g.q));
  const Fp4 v = h4_mul(g, A, B);
  const Fp4 w = h4_mul(g, sa, sb);
  return g6_recombine(g, v, w);
}

__device__ __forceinline__ Fp4 g6_cyclo_sqr(const Grp6& g, const Fp4& A) {
  const Fp4 te = xch(h4_sqr(g, A), g.e);
  Fp4 ts;
  f4_select(ts, g.k == 1, te, f4_mul_s(te));
  const Fp2 x3 = f2_add(f2_dbl(ts.x), ts.x), y3 = f2_add(f2_dbl(ts.y), ts.y);
  const Fp2 ax2 = f2_dbl(A.x), ay2 = f2_dbl(A.y);
  Fp4 r;
  f4_select(r, g.k == 1, Fp4{f2_sub(x3, ax2), f2_add(y3, ay2)}, Fp4{f2_add(x3, ax2), f2_sub(y3, ay2)});
  return r;
}

__device__ __forceinline__ Fp4 g6_conj(const Grp6& g, const Fp4& A) {
  Fp4 r;
  f4_select(r, g.k == 1, Fp4{A.x, f2_neg(A.y)}, Fp4{f2_neg(A.x), A.y});
  return r;
}

template <int J>
__device__ __forceinline__ Fp4 g6_frob(const Grp6& g, const Fp4& A) {
  const uint32_t(*tab)[2][12] = (J == 1) ? FROB1 : (J == 2) ? FROB2 : FROB3;
  const Fp2 cx = f2_from_const(tab[g.k]), cy = f2_from_const(tab[g.k + 3]);
  const Fp2 x = (J & 1) ? f2_conj(A.x) : A.x;
  const Fp2 y = (J & 1) ? f2_conj(A.y) : A.y;
  return {h2_mul(g, x, cx), h2_mul(g, y, cy)};
}

// inverse via the cubic adjugate (g_inv); the one Fp2 inversion runs in both halves
__device__ __forceinline__ Fp4 g6_inv(const Grp6& g, const Fp4& A) {
  const Fp4 A1 = xch(A, g.n1), A2 = xch(A, g.n2);
  const Fp4 X0 = pick3(g.k, A, A2, A1);
  const Fp4 X1 = pick3(g.k, A1, A, A2);
  const Fp4 X2 = pick3(g.k, A2, A1, A);
  const Fp4 sq = h4_sqr(g, pick3(g.k, X0, X2, X1));
  const Fp4 pr = h4_mul(g, pick3(g.k, X1, X0, X0), pick3(g.k, X2, X1, X2));
  const Fp4 B = pick3(g.k, f4_sub(sq, f4_mul_s(pr)), f4_sub(f4_mul_s(sq), pr), f4_sub(sq, pr));
  const Fp4 T = h4_mul(g, A, xch(B, g.e));
  const Fp4 T1 = xch(T, g.n1), T2 = xch(T, g.n2);
  const Fp4 N = f4_add(pick3(g.k, T, T2, T1), f4_mul_s(f4_add(pick3(g.k, T1, T, T2), pick3(g.k, T2, T1, T))));
  const Fp2 d = f2_sub(h2_sqr(g, N.x), f2_mul_xi(h2_sqr(g, N.y)));
  const Fp2 di = f2_inv(d);
  return h4_mul(g, B, Fp4{h2_mul(g, N.x, di), f2_neg(h2_mul(g, N.y, di))});
}

__device__ __forceinline__ Fp4 g6_pow_x(const Grp6& g, const Fp4& f) {
  Fp4 r = f;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    r = g6_cyclo_sqr(g, r);
    if ((HB_X_ABS >> i) & 1) r = g6_mul(g, r, f);
  }
  return g6_conj(g, r);
}

// g_final_exp (pair3.h) over six lanes
__device__ __forceinline__ Fp4 g6_final_exp(const Grp6& g, const Fp4& f) {
  Fp4 t = g6_mul(g, g6_conj(g, f), g6_inv(g, f));
  t = g6_mul(g, g6_frob<2>(g, t), t);
  Fp4 x = t, b = t;
  HB_NOUNROLL for (int s = 0; s < 5; s++) {
    const Fp4 px = g6_pow_x(g, x);
    if (s == 3) b = x;
    if (s < 2) x = g6_mul(g, px, g6_conj(g, x));
    else if (s == 2) x = g6_mul(g, px, g6_frob<1>(g, x));
    else x = px;
  }
  const Fp4 c = g6_mul(g, g6_mul(g, x, g6_frob<2>(g, b)), g6_conj(g, b));
  return g6_mul(g, c, g6_mul(g, g6_cyclo_sqr(g, t), t));
}

__device__ __forceinline__ bool g6_is_one(const Grp6& g, const Fp4& A) {
  const bool mine = g.k == 0 ? (f2_eq(A.x, f2_one()) && f2_is_zero(A.y)) : (f2_is_zero(A.x) && f2_is_zero(A.y));
  const uint32_t m = mine ? 1u : 0u;
  return (m & xch(m, g.n1) & xch(m, g.n2)) != 0;
}

#endif  // __HIP_DEVICE_COMPILE__

}  // namespace hb
