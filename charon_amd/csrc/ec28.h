// Lazily reduced 28-bit-limb point arithmetic for the subgroup ladders (round 3).
//
// fp.h stores Fp in 12 x 32-bit words reduced to [0, 2p): every Montgomery product re-splits its
// operands into 14 limbs of 28 bits and joins its result back (≈ 80 of its ≈ 540 VALU
// instructions), and every addition is a 12-word carry chain plus a conditional subtraction of
// 2p (36 instructions).  Here the G1 Jacobian coordinates stay in 14 x 28-bit limbs across a
// whole ladder: the products take and return limbs directly (fp_mul28_leaf / fp_sqr28_leaf), an
// addition is 14 independent limb additions, a subtraction a + K - b adds a multiple K = s p of p
// whose limbs are spread so that each dominates the subtrahend's (no borrows), and a carry pass
// (`l_norm`) runs only where a value feeds a subtraction or must fit a product's input bound.
// Nothing is reduced modulo p outside the products, so values grow up to VMAX p between them;
// charon_amd/tools/lazy28.py restates every formula below over per-limb intervals and proves
// (tests/test_lazy28.py) that no limb exceeds 32 bits, no product column 64 bits, every K
// dominates its subtrahend and the coordinates return below VMAX p -- the ladders' invariant.
// The site constants K28<s, t> below are the ones lazy28.KSITE holds (the test compares them).
#pragma once
#include "ec.h"

namespace hb {

struct L28 {
  uint32_t l[14];
};

// K = s p as 14 limbs of 28 bits spread with redundancy t: K_0 = c_0 + t 2^28,
// K_i = c_i + t 2^28 - t (0 < i < 13), K_13 = c_13 - t (lazy28.py kconst)
struct K28v {
  uint32_t l[14];
};
constexpr uint32_t kP28_[14] = {0x0fffaaabu, 0x0fefffffu, 0x03ffffb9u, 0x0fffeb15u, 0x06241eabu,
                                0x0a0f6b0fu, 0x0f6730d2u, 0x0f38512bu, 0x04774b84u, 0x04bacd76u,
                                0x0ba7b643u, 0x0e69a4b1u, 0x01ea397fu, 0x0001a011u};  // = P28
constexpr K28v k28_make(uint32_t s, uint32_t t) {
  K28v k{};
  uint64_t c = 0;
  for (int i = 0; i < 14; i++) {
    const uint64_t v = (uint64_t)kP28_[i] * s + c;
    k.l[i] = (uint32_t)(v & 0x0FFFFFFFu);
    c = v >> 28;
  }
  k.l[13] += (uint32_t)(c << 28);  // s p < 2^392: no carry out of the top limb
  k.l[0] += t << 28;
  for (int i = 1; i < 13; i++) k.l[i] += (t << 28) - t;
  k.l[13] -= t;
  return k;
}
template <uint32_t S, uint32_t T>
struct K28 {
  static constexpr K28v v = k28_make(S, T);
};

HD L28 l_add(const L28& a, const L28& b) {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
HD L28 l_shl(const L28& a, int s) {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = a.l[i] << s;
  return r;
}
template <uint32_t S, uint32_t T>
HD L28 l_sub(const L28& a, const L28& b) {  // a + S p - b, limb-wise
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = a.l[i] + (K28<S, T>::v.l[i] - b.l[i]);
  return r;
}
HD L28 l_norm(L28 a) {  // carries: limbs 0..12 below 2^28, the value unchanged
  HB_UNROLL for (int i = 0; i < 13; i++) {
    a.l[i + 1] += a.l[i] >> 28;
    a.l[i] &= 0x0FFFFFFFu;
  }
  return a;
}
HD L28 l_from(const Fp& a) {
  L28 r;
  fp_split28(r.l, a.v);
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// (lanes 14, 15 of the argument vectors are left undefined: no moves for them around the call)
HD L28 l_mul_nc(const L28& a, const L28& b) {  // not counted: membership / conversion helpers
  u32x16 x, y;
  HB_UNROLL for (int i = 0; i < 14; i++) {
    x[i] = a.l[i];
    y[i] = b.l[i];
  }
  const u32x16 o = fp_mul28_leaf(x, y);
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = o[i];
  return r;
}
HD L28 l_mul(const L28& a, const L28& b) {
  HB_COUNT_FP_MUL();
  return l_mul_nc(a, b);
}
HD L28 l_sqr(const L28& a) {
  HB_COUNT_FP_MUL();
  u32x16 x;
  HB_UNROLL for (int i = 0; i < 14; i++) x[i] = a.l[i];
  const u32x16 o = fp_sqr28_leaf(x);
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = o[i];
  return r;
}
#else  // host: fp.h's choice of cores (hostmul64.h unless HB_HOST_MUL28)
HD L28 l_mul_nc(const L28& a, const L28& b) {
  L28 r;
#if defined(HB_HOST_MUL28)
  fp_mul28_core(r.l, a.l, b.l);
#else
  hm64::mul_limbs28(r.l, a.l, b.l);
#endif
  return r;
}
HD L28 l_mul(const L28& a, const L28& b) {
  HB_COUNT_FP_MUL();
  return l_mul_nc(a, b);
}
HD L28 l_sqr(const L28& a) {
  HB_COUNT_FP_MUL();
  L28 r;
#if defined(HB_HOST_MUL28)
  fp_sqr28_core(r.l, a.l);
#else
  hm64::mul_limbs28(r.l, a.l, a.l);
#endif
  return r;
}
#endif

// ---- Two independent products in one leaf, for the G1 formulas (g1l_dbl): the two column chains
// interleaved, each seeded with its own carry (HB_MADD keeps the compiler from reassociating
// them).  A lone chain makes the compiler start every column's multiply-adds at zero and add the
// shifted carry afterwards (one v_lshl_add_u64 per column) to keep dependent multiply-adds apart;
// with two chains the other chain's multiply-add sits between them.  Measured (round 5,
// profiles/r05c_leaf_ab.txt): the G1 kernels gain (k_dec_pk 24.7 -> 23.6-24.5 ms, k_rlc 10.6-10.9
// -> 10.2-10.3 ms alone), the same pairing of the G2 formulas' Fp2 products -- and an interleaved
// Fp2 product -- lose (k_msm_bucket +25 %, k_ta_small +13 %, hashing +2.5 %): G2 keeps the lone
// chains.  Same values as two l_mul / l_sqr.
// r0 = a0 b0 / R, r1 = a1 b1 / R (SQ: a0 = b0, a1 = b1, the squares' halved cross products)
template <bool SQ>
HD void mul28x2_core(uint32_t* r0, uint32_t* r1, const uint32_t* a0, const uint32_t* b0, const uint32_t* a1,
                     const uint32_t* b1) {
  uint32_t m0[14], m1[14], d0[14], d1[14];
  if (SQ)
    HB_UNROLL for (int j = 0; j < 14; j++) {
      d0[j] = a0[j] << 1;
      d1[j] = a1[j] << 1;
    }
  uint64_t c0 = 0, c1 = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      if (SQ) {
        if (2 * j < k) {
          HB_MADD(c0, d0[j], a0[k - j]);
          HB_MADD(c1, d1[j], a1[k - j]);
        } else if (2 * j == k) {
          HB_MADD(c0, a0[j], a0[j]);
          HB_MADD(c1, a1[j], a1[j]);
        }
      } else {
        HB_MADD(c0, a0[j], b0[k - j]);
        HB_MADD(c1, a1[j], b1[k - j]);
      }
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) {
        HB_MADD(c0, m0[j], P28[k - j]);
        HB_MADD(c1, m1[j], P28[k - j]);
      }
    if (k < 14) {
      m0[k] = ((uint32_t)c0 * HB_P_N0_28) & 0x0FFFFFFFu;
      m1[k] = ((uint32_t)c1 * HB_P_N0_28) & 0x0FFFFFFFu;
      HB_MADD(c0, m0[k], P28[0]);
      HB_MADD(c1, m1[k], P28[0]);
    } else {
      r0[k - 14] = (uint32_t)c0 & 0x0FFFFFFFu;
      r1[k - 14] = (uint32_t)c1 & 0x0FFFFFFFu;
    }
    c0 >>= 28;
    c1 >>= 28;
  }
  r0[13] = (uint32_t)c0;
  r1[13] = (uint32_t)c1;
}
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
// first operands in the argument VGPRs (a0: limbs 0..13, a1: 16..29), second operands through the
// per-lane LDS slot of fp.h (pairs (b0_k, b1_k)), as f2l_mul_leaf
__device__ __noinline__ static u32x32 l_mul2_leaf(u32x32 a) {
  uint32_t x0[14], x1[14], y0[14], y1[14], r0[14], r1[14];
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    const uint2 v = hb_fp2_arg[k * HB_ARG_LANES + lane];
    y0[k] = v.x;
    y1[k] = v.y;
    x0[k] = a[k];
    x1[k] = a[16 + k];
  }
  mul28x2_core<false>(r0, r1, x0, y0, x1, y1);
  u32x32 o;
  HB_UNROLL for (int k = 0; k < 14; k++) {
    o[k] = r0[k];
    o[16 + k] = r1[k];
  }
  return o;
}
__device__ __noinline__ static u32x32 l_sqr2_leaf(u32x32 a) {
  uint32_t x0[14], x1[14], r0[14], r1[14];
  HB_UNROLL for (int k = 0; k < 14; k++) {
    x0[k] = a[k];
    x1[k] = a[16 + k];
  }
  mul28x2_core<true>(r0, r1, x0, x0, x1, x1);
  u32x32 o;
  HB_UNROLL for (int k = 0; k < 14; k++) {
    o[k] = r0[k];
    o[16 + k] = r1[k];
  }
  return o;
}
#endif
// (a b, c d) and (a^2, c^2): one dual-chain leaf on the device, two products on the host
HD void l_mul2(const L28& a, const L28& b, const L28& c, const L28& d, L28& r0, L28& r1) {
#if defined(__HIP_DEVICE_COMPILE__)
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  u32x32 av;
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    av[k] = a.l[k];
    av[16 + k] = c.l[k];
    hb_fp2_arg[k * HB_ARG_LANES + lane] = make_uint2(b.l[k], d.l[k]);
  }
  const u32x32 o = l_mul2_leaf(av);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    r0.l[k] = o[k];
    r1.l[k] = o[16 + k];
  }
#else
  r0 = l_mul(a, b);
  r1 = l_mul(c, d);
#endif
}
HD void l_sqr2(const L28& a, const L28& c, L28& r0, L28& r1) {
#if defined(__HIP_DEVICE_COMPILE__)
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  u32x32 av;
  HB_UNROLL for (int k = 0; k < 14; k++) {
    av[k] = a.l[k];
    av[16 + k] = c.l[k];
  }
  const u32x32 o = l_sqr2_leaf(av);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    r0.l[k] = o[k];
    r1.l[k] = o[16 + k];
  }
#else
  r0 = l_sqr(a);
  r1 = l_sqr(c);
#endif
}

// a == 0 mod p for a NORMALISED value a < 2^392 without a product: a is k p only for
// k = rint(a / p), read off the top 56 bits (the low 336 bits of p move the ratio by < 2^-38 for
// the k < 2^20 of any lazy value), then one pass compares a with k p limb by limb
constexpr double kInvPTop = 1.0 / (double)(((uint64_t)0x0001a011u << 28) | 0x01ea397fu);  // 1 / (p >> 336)
HD bool l_is_zero_n(const L28& a) {
  const double top = (double)a.l[13] * 268435456.0 + (double)a.l[12];
  const uint32_t k = (uint32_t)__builtin_rint(top * kInvPTop);
  uint64_t c = 0;
  uint32_t diff = 0;
  HB_UNROLL for (int i = 0; i < 13; i++) {
    c += (uint64_t)k * kP28_[i];
    diff |= ((uint32_t)c & 0x0FFFFFFFu) ^ a.l[i];
    c >>= 28;
  }
  c += (uint64_t)k * kP28_[13];
  diff |= (uint32_t)c ^ a.l[13];
  return diff == 0;
}
HD bool l_is_zero(const L28& a) { return l_is_zero_n(l_norm(a)); }
// reference form of the same test (the Montgomery product by the integer 1 is a R^-1 mod p and
// lies in [0, p]), for tests/test_lazy28.py
HD bool l_is_zero_mul(const L28& a) {
  L28 one;
  one.l[0] = 1;
  HB_UNROLL for (int i = 1; i < 14; i++) one.l[i] = 0;
  const L28 t = l_mul_nc(a, one);
  uint32_t z = 0, q = 0;
  HB_UNROLL for (int i = 0; i < 14; i++) {
    z |= t.l[i];
    q |= t.l[i] ^ kP28_[i];
  }
  return z == 0 || q == 0;
}
// back to the stored form: the product by R mod p (Montgomery one) is < p + 1 -> [0, 2p) words
HD Fp l_to(const L28& a) {
  const L28 t = l_mul_nc(a, l_from(fp_one()));
  Fp r;
  fp_join28(r.v, t.l);
  return r;
}

// ---- G1 Jacobian points in lazy limbs; infinity as a flag (E(Fp) has no 2-torsion: the
// cofactor (x - 1)^2 / 3 and r are odd, so a doubling never reaches Z = 0 from a finite point)
struct G1L {
  L28 X, Y, Z;
  bool inf;
};

// Who computes the G1 formulas' pairs of independent products.  G1One: this lane, both in one
// dual-chain leaf (l_mul2 / l_sqr2).  G1Half (device, below): the two lanes of a pair, each one of
// the two products, then an exchange -- for the latency-bound small calls, like F2Half for Fp2.
struct G1One {
  static constexpr bool kSplit = false;
};
HD void p_mul2(G1One, const L28& a, const L28& b, const L28& c, const L28& d, L28& r0, L28& r1) { l_mul2(a, b, c, d, r0, r1); }
HD void p_sqr2(G1One, const L28& a, const L28& c, L28& r0, L28& r1) { l_sqr2(a, c, r0, r1); }

// dbl-2009-l (lazy28.py dbl)
template <class M = G1One>
HDNI G1L g1l_dbl(const G1L& p, M m = M()) {
  L28 A, B, C, T;
  p_sqr2(m, p.X, p.Y, A, B);
  p_sqr2(m, B, l_add(p.X, B), C, T);
  const L28 E = l_add(l_add(A, A), A);
  const L28 F = l_sqr(E);
  const L28 D = l_norm(l_shl(l_sub<3, 2>(T, l_add(A, C)), 1));
  G1L r;
  r.X = l_norm(l_sub<17, 2>(F, l_shl(D, 1)));
  const L28 W = l_sub<19, 1>(D, r.X);
  L28 EW;
  p_mul2(m, E, W, l_shl(p.Y, 1), p.Z, EW, r.Z);
  r.Y = l_norm(l_sub<9, 8>(EW, l_shl(C, 3)));
  r.inf = p.inf;
  return r;
}

// the common tail of the additions (I = 4 HH folded into shifts: J = 4 H HH, V = 4 U1 HH)
// (G1Half pairs the products that G1One, measured on the C3 ladders, keeps single)
template <class M = G1One>
HD G1L g1l_add_tail(const L28& H, const L28& rr, const L28& U1, const L28& S1, const L28& Zs, M m = M()) {
  L28 HH, Z3;
  if constexpr (M::kSplit) {
    p_mul2(m, H, H, Zs, H, HH, Z3);
  } else {
    HH = l_sqr(H);
  }
  L28 J1, V1;
  p_mul2(m, H, HH, U1, HH, J1, V1);
  G1L r;
  r.X = l_norm(l_sub<13, 12>(l_sqr(rr), l_add(l_shl(J1, 2), l_shl(V1, 3))));
  L28 t, sj;
  p_mul2(m, rr, l_sub<15, 1>(l_shl(V1, 2), r.X), S1, J1, t, sj);
  r.Y = l_norm(l_sub<9, 8>(t, l_shl(sj, 3)));
  if constexpr (M::kSplit) {
    r.Z = Z3;
  } else {
    r.Z = l_mul(Zs, H);
  }
  r.inf = false;
  return r;
}

HD G1L g1l_infinity() {
  G1L r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.X.l[i] = r.Y.l[i] = r.Z.l[i] = 0;
  r.inf = true;
  return r;
}

// madd-2007-bl: p + (x2, y2), the affine point finite and normalised below 2p (lazy28.py madd)
template <class M = G1One>
HDNI G1L g1l_madd(const G1L& p, const L28& x2, const L28& y2, M m = M()) {
  if (p.inf) return {x2, y2, l_from(fp_one()), false};
  L28 Z1Z1, U2, S2;
  if constexpr (M::kSplit) {
    L28 yZ;
    p_mul2(m, p.Z, p.Z, y2, p.Z, Z1Z1, yZ);
    p_mul2(m, x2, Z1Z1, yZ, Z1Z1, U2, S2);
  } else {
    Z1Z1 = l_sqr(p.Z);
    U2 = l_mul(x2, Z1Z1);
    S2 = l_mul(l_mul(y2, p.Z), Z1Z1);
  }
  const L28 H = l_sub<21, 1>(U2, p.X);
  const L28 rr = l_norm(l_sub<41, 2>(l_shl(S2, 1), l_shl(p.Y, 1)));
  if (l_is_zero(H)) {
    if (l_is_zero(rr)) return g1l_dbl(p, m);
    return g1l_infinity();
  }
  return g1l_add_tail(H, rr, p.X, p.Y, l_shl(p.Z, 1), m);
}

// add-2007-bl (lazy28.py jadd)
template <class M = G1One>
HDNI G1L g1l_add(const G1L& p, const G1L& q, M m = M()) {
  if (p.inf) return q;
  if (q.inf) return p;
  L28 Z1Z1, Z2Z2, U1, U2, S1, S2;
  if constexpr (M::kSplit) {
    L28 pYqZ, qYpZ;
    p_sqr2(m, p.Z, q.Z, Z1Z1, Z2Z2);
    p_mul2(m, p.Y, q.Z, q.Y, p.Z, pYqZ, qYpZ);
    p_mul2(m, p.X, Z2Z2, q.X, Z1Z1, U1, U2);
    p_mul2(m, pYqZ, Z2Z2, qYpZ, Z1Z1, S1, S2);
  } else {
    Z1Z1 = l_sqr(p.Z);
    Z2Z2 = l_sqr(q.Z);
    U1 = l_mul(p.X, Z2Z2);
    U2 = l_mul(q.X, Z1Z1);
    S1 = l_mul(l_mul(p.Y, q.Z), Z2Z2);
    S2 = l_mul(l_mul(q.Y, p.Z), Z1Z1);
  }
  const L28 H = l_sub<21, 1>(U2, U1);
  const L28 rr = l_norm(l_sub<41, 2>(l_shl(S2, 1), l_shl(S1, 1)));
  if (l_is_zero(H)) {
    if (l_is_zero(rr)) return g1l_dbl(p, m);
    return g1l_infinity();
  }
  return g1l_add_tail(H, rr, U1, S1, l_mul(l_shl(p.Z, 1), q.Z), m);
}

HD G1J g1l_to_jac(const G1L& p) {
  if (p.inf) return jac_infinity<Fp>();
  return {l_to(p.X), l_to(p.Y), l_to(p.Z)};
}

// P in G1  <=>  phi(P) == [-x^2] P (ec.h g1_in_subgroup), the two ladders in lazy limbs
template <class M = G1One>
HDNI bool g1_in_subgroup28(const G1A& p, M m = M()) {
  if (p.inf) return true;
  const L28 x = l_from(p.x), y = l_from(p.y);
  G1L t = {x, y, l_from(fp_one()), false};
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    t = g1l_dbl(t, m);
    if ((HB_X_ABS >> i) & 1) t = g1l_madd(t, x, y, m);
  }
  G1L u = t;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    u = g1l_dbl(u, m);
    if ((HB_X_ABS >> i) & 1) u = g1l_add(u, t, m);
  }
  const G1J phi = jac_from_aff(G1A{fp_mul(p.x, fp_from_const(G1_BETA)), p.y, false});
  return jac_eq(phi, jac_neg(g1l_to_jac(u)));
}


// ---- Fp2 (u^2 = -1) in lazy limbs (lazy28.py Fp2Ops)
struct F2L {
  L28 c0, c1;
};
HD F2L f2l_add(const F2L& a, const F2L& b) { return {l_add(a.c0, b.c0), l_add(a.c1, b.c1)}; }
HD F2L f2l_shl(const F2L& a, int s) { return {l_shl(a.c0, s), l_shl(a.c1, s)}; }
template <uint32_t S, uint32_t T>
HD F2L f2l_sub(const F2L& a, const F2L& b) {
  return {l_sub<S, T>(a.c0, b.c0), l_sub<S, T>(a.c1, b.c1)};
}
HD F2L f2l_norm(const F2L& a) { return {l_norm(a.c0), l_norm(a.c1)}; }
HD F2L f2l_from(const Fp2& a) { return {l_from(a.c0), l_from(a.c1)}; }
HD Fp2 f2l_to(const F2L& a) { return {l_to(a.c0), l_to(a.c1)}; }
HD bool f2l_is_zero(const F2L& a) { return l_is_zero(a.c0) && l_is_zero(a.c1); }

// (a0 + a1 u)(b0 + b1 u) in one product-scanning pass with two accumulators:
//   real = a0 b0 + (K - a1) b1,   imag = a0 b1 + a1 b0,   K = 33 p (lazy28.KSITE["2N"]),
// so both columns are sums of non-negative terms (no signed accumulator, no final correction)
// and both results come out normalised.
constexpr K28v kF2N = k28_make(33, 6);
HD void f2l_dot_core(uint32_t* r, const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1) {
  uint32_t m[14];  // r = (a0 b0 + a1 b1) / R: one column pass, one accumulator
  uint64_t acc = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      acc += (uint64_t)a0[j] * b0[k - j];
      acc += (uint64_t)a1[j] * b1[k - j];
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P28[k - j];
    HB_MONT28_TAIL(acc, m, k, r)
  }
  r[13] = (uint32_t)acc;
}
HD void f2l_mul_core(uint32_t* r0, uint32_t* r1, const uint32_t* a0, const uint32_t* a1, const uint32_t* b0,
                     const uint32_t* b1) {
  uint32_t na1[14];
  HB_UNROLL for (int j = 0; j < 14; j++) na1[j] = kF2N.l[j] - a1[j];
  f2l_dot_core(r0, a0, na1, b0, b1);  // real = a0 b0 + (K - a1) b1
  f2l_dot_core(r1, a0, a1, b1, b0);   // imag = a0 b1 + a1 b0
}

#if defined(__HIP_DEVICE_COMPILE__)
// first operand in the 32 argument VGPRs (limbs 0..13 | 16..29), the second through the per-lane
// LDS slot of fp.h (14 pairs (b0_k, b1_k), k-major: conflict-free 64-bit accesses)
static_assert(HB_FP2_ARG_SLOTS >= 14, "hb_fp2_arg holds 14 pairs per lane");
__device__ __noinline__ static u32x32 f2l_mul_leaf(u32x32 a) {
  uint32_t x0[14], x1[14], y0[14], y1[14], r0[14], r1[14];
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    const uint2 v = hb_fp2_arg[k * HB_ARG_LANES + lane];
    y0[k] = v.x;
    y1[k] = v.y;
    x0[k] = a[k];
    x1[k] = a[16 + k];
  }
  f2l_mul_core(r0, r1, x0, x1, y0, y1);
  u32x32 o;
  HB_UNROLL for (int k = 0; k < 14; k++) {
    o[k] = r0[k];
    o[16 + k] = r1[k];
  }
  return o;
}
HD F2L f2l_mul(const F2L& a, const F2L& b) {
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  u32x32 av;
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    av[k] = a.c0.l[k];
    av[16 + k] = a.c1.l[k];
    hb_fp2_arg[k * HB_ARG_LANES + lane] = make_uint2(b.c0.l[k], b.c1.l[k]);
  }
  const u32x32 o = f2l_mul_leaf(av);
  F2L r;
  HB_UNROLL for (int k = 0; k < 14; k++) {
    r.c0.l[k] = o[k];
    r.c1.l[k] = o[16 + k];
  }
  return r;
}
#else
HD F2L f2l_mul(const F2L& a, const F2L& b) {
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  F2L r;
#if defined(HB_HOST_MUL28)
  f2l_mul_core(r.c0.l, r.c1.l, a.c0.l, a.c1.l, b.c0.l, b.c1.l);
#else
  uint32_t na1[14];
  HB_UNROLL for (int j = 0; j < 14; j++) na1[j] = kF2N.l[j] - a.c1.l[j];
  hm64::dot_limbs28(r.c0.l, a.c0.l, na1, b.c0.l, b.c1.l);
  hm64::dot_limbs28(r.c1.l, a.c0.l, a.c1.l, b.c1.l, b.c0.l);
#endif
  return r;
}
#endif
// (a0 + a1)(a0 + K - a1) + 2 a0 a1 u, K = 36 p (lazy28.KSITE["2Q"]): two Fp products
HD F2L f2l_sqr(const F2L& a) {
  return {l_mul(l_add(a.c0, a.c1), l_sub<36, 1>(a.c0, a.c1)), l_mul(l_shl(a.c0, 1), a.c1)};
}
// f2l_sqr with the site's constant K = S p
template <uint32_t S, uint32_t T>
HD F2L f2l_sqr_k(const F2L& a) {
  return {l_mul(l_add(a.c0, a.c1), l_sub<S, T>(a.c0, a.c1)), l_mul(l_shl(a.c0, 1), a.c1)};
}

// Who computes a formula's Fp2 products.  F2One: this lane alone (f2l_mul / f2l_sqr_k).  F2Half
// (device, below): the two lanes of a pair, both holding the operands, each computing one output
// coefficient and taking the other from its partner -- half the multiply-adds on each lane's
// dependent path, for the latency-bound calls.  The formulas below take the policy as their last
// argument and multiply through fm / fs; the values are the same either way.
struct F2One {};
HD F2L fm(F2One, const F2L& a, const F2L& b) { return f2l_mul(a, b); }
template <uint32_t S, uint32_t T>
HD F2L fs(F2One, const F2L& a) { return f2l_sqr_k<S, T>(a); }
// Independent products in one call, so that a policy spreading them over more lanes (pair28.h
// F2Hex: six lanes, one coefficient each) can run them side by side; the default runs them in turn.
template <class M>
HD void fm2(M m, const F2L& a0, const F2L& b0, const F2L& a1, const F2L& b1, F2L& t0, F2L& t1) {
  t0 = fm(m, a0, b0);
  t1 = fm(m, a1, b1);
}
template <class M>
HD void fm3(M m, const F2L& a0, const F2L& b0, const F2L& a1, const F2L& b1, const F2L& a2, const F2L& b2, F2L& t0,
            F2L& t1, F2L& t2) {
  t0 = fm(m, a0, b0);
  t1 = fm(m, a1, b1);
  t2 = fm(m, a2, b2);
}
template <uint32_t S, uint32_t T, class M>
HD void fs3(M m, const F2L& a0, const F2L& a1, const F2L& a2, F2L& t0, F2L& t1, F2L& t2) {
  t0 = fs<S, T>(m, a0);
  t1 = fs<S, T>(m, a1);
  t2 = fs<S, T>(m, a2);
}

#if defined(__HIP_DEVICE_COMPILE__)
// x0 y0 + x1 y1 (one Montgomery pass, f2l_dot_core): x0 | x1 in the argument VGPRs, y0, y1 through
// the per-lane LDS slot as f2l_mul_leaf's
__device__ __noinline__ static u32x16 l_dot_leaf(u32x32 a) {
  uint32_t x0[14], x1[14], y0[14], y1[14], r[14];
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    const uint2 v = hb_fp2_arg[k * HB_ARG_LANES + lane];
    y0[k] = v.x;
    y1[k] = v.y;
    x0[k] = a[k];
    x1[k] = a[16 + k];
  }
  f2l_dot_core(r, x0, x1, y0, y1);
  u32x16 o;
  HB_UNROLL for (int k = 0; k < 14; k++) o[k] = r[k];
  return o;
}
__device__ __forceinline__ L28 l_dot(const L28& x0, const L28& x1, const L28& y0, const L28& y1) {
  HB_COUNT_FP_MUL();
  HB_COUNT_FP_MUL();
  u32x32 av;
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 14; k++) {
    av[k] = x0.l[k];
    av[16 + k] = x1.l[k];
    hb_fp2_arg[k * HB_ARG_LANES + lane] = make_uint2(y0.l[k], y1.l[k]);
  }
  const u32x16 o = l_dot_leaf(av);
  L28 r;
  HB_UNROLL for (int k = 0; k < 14; k++) r.l[k] = o[k];
  return r;
}
__device__ __forceinline__ L28 l_pick(bool take_b, const L28& a, const L28& b) {
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = take_b ? b.l[i] : a.l[i];
  return r;
}
__device__ __forceinline__ L28 l_xch(const L28& a, int addr) {  // the limbs of lane addr / 4
  L28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)a.l[i]);
  return r;
}
// h: the coefficient this lane computes; partner: the other lane of the pair (ds_bpermute address).
// Both lanes run the same instruction stream (operands chosen by select) and hold the same values.
struct F2Half {
  int h, partner;
};
__device__ __forceinline__ F2Half f2half_make() {  // pairs (2i, 2i + 1) of the wavefront
  const int lane = (int)(threadIdx.x & 63u);
  return {lane & 1, (lane ^ 1) << 2};
}
__device__ __forceinline__ F2L f2h_join(F2Half m, const L28& mine) {
  const L28 other = l_xch(mine, m.partner);
  return {l_pick(m.h != 0, mine, other), l_pick(m.h != 0, other, mine)};
}
// G1Half: lane h of the pair computes product h of the two and takes the other from its partner
struct G1Half {
  static constexpr bool kSplit = true;
  int h, partner;
};
__device__ __forceinline__ G1Half g1half_make() {
  const F2Half f = f2half_make();
  return {f.h, f.partner};
}
__device__ __forceinline__ void g1h_join(G1Half m, const L28& mine, L28& r0, L28& r1) {
  const L28 other = l_xch(mine, m.partner);
  r0 = l_pick(m.h != 0, mine, other);
  r1 = l_pick(m.h != 0, other, mine);
}
__device__ __forceinline__ void p_mul2(G1Half m, const L28& a, const L28& b, const L28& c, const L28& d, L28& r0,
                                       L28& r1) {
  const bool h = m.h != 0;
  g1h_join(m, l_mul(l_pick(h, a, c), l_pick(h, b, d)), r0, r1);
}
__device__ __forceinline__ void p_sqr2(G1Half m, const L28& a, const L28& c, L28& r0, L28& r1) {
  g1h_join(m, l_sqr(l_pick(m.h != 0, a, c)), r0, r1);
}

// coefficient 0: a0 b0 + (K - a1) b1 (K = kF2N, as f2l_mul_core), coefficient 1: a0 b1 + a1 b0
__device__ __forceinline__ F2L fm(F2Half m, const F2L& a, const F2L& b) {
  L28 na1;
  HB_UNROLL for (int j = 0; j < 14; j++) na1.l[j] = kF2N.l[j] - a.c1.l[j];
  const bool h = m.h != 0;
  return f2h_join(m, l_dot(a.c0, l_pick(h, na1, a.c1), l_pick(h, b.c0, b.c1), l_pick(h, b.c1, b.c0)));
}
// coefficient 0: (a0 + a1)(a0 + K - a1), coefficient 1: (2 a0) a1 (f2l_sqr_k's two products)
template <uint32_t S, uint32_t T>
__device__ __forceinline__ F2L fs(F2Half m, const F2L& a) {
  const bool h = m.h != 0;
  return f2h_join(m, l_mul(l_pick(h, l_add(a.c0, a.c1), l_shl(a.c0, 1)), l_pick(h, l_sub<S, T>(a.c0, a.c1), a.c1)));
}
#endif

// ---- G2 Jacobian points in lazy limbs (E'(Fp2) has no 2-torsion either: h2 and r are odd)
struct G2L {
  F2L X, Y, Z;
  bool inf;
};

// v mod p up to a multiple of p: the same residue, normalised, below 2p.  a: limbs below 2^32
// (not necessarily carried), value below 2^390.  The top estimate l13 2^28 + l12 is within 17 of
// v / 2^336 (the lower limbs carry at most 16 into limb 12), so top / (p >> 336) is within 2^-40
// of v / p; minus 2^-20 and truncated it gives floor(v / p) or one less.  The subtraction runs
// with a signed carry (q < 2^10, so q p_i < 2^38).  (pair28.h's steps end with it.)
HD L28 l_red(const L28& a) {
  const double top = (double)a.l[13] * 268435456.0 + (double)a.l[12];
  const double qd = top * kInvPTop - 0x1p-20;
  const int32_t q = qd > 0.0 ? (int32_t)qd : 0;
  L28 r;
  int64_t c = 0;
  HB_UNROLL for (int i = 0; i < 13; i++) {
    c += (int64_t)a.l[i] - (int64_t)q * (int64_t)kP28_[i];
    r.l[i] = (uint32_t)c & 0x0FFFFFFFu;
    c >>= 28;
  }
  r.l[13] = (uint32_t)(c + (int64_t)a.l[13] - (int64_t)q * (int64_t)kP28_[13]);
  return r;
}
HD F2L f2l_red(const F2L& a) { return {l_red(a.c0), l_red(a.c1)}; }

// lazy28.py dbl2: dbl-2009-l (2M + 5S) with D = 2((X + B)^2 - A - C) partially reduced (l_red, no
// product -- unreduced, its subtraction constant grows the point past the invariant), X + B and
// E = 3A normalised before their squares, W first in E W (33p - W.c1 dominates it); the products
// in the order that ends the inputs' live ranges first (Z3 before B = Y^2, T right after A)
template <class M = F2One>
HDNI G2L g2l_dbl(const G2L& p, M m = M()) {
  G2L r;
  r.Z = fm(m, f2l_shl(p.Y, 1), p.Z);
  const F2L B = fs<36, 1>(m, p.Y);
  const F2L A = fs<36, 1>(m, p.X);
  const F2L T = fs<36, 1>(m, f2l_norm(f2l_add(p.X, B)));
  const F2L C = fs<36, 1>(m, B);
  const F2L E = f2l_norm(f2l_add(f2l_shl(A, 1), A));
  const F2L D = f2l_red(f2l_shl(f2l_sub<3, 2>(T, f2l_add(A, C)), 1));
  r.X = f2l_norm(f2l_sub<5, 2>(fs<36, 1>(m, E), f2l_shl(D, 1)));
  const F2L W = f2l_sub<7, 1>(D, r.X);
  r.Y = f2l_norm(f2l_sub<9, 8>(fm(m, W, E), f2l_shl(C, 3)));
  r.inf = p.inf;
  return r;
}

HD G2L g2l_infinity() {
  G2L r;
  HB_UNROLL for (int i = 0; i < 14; i++)
    r.X.c0.l[i] = r.X.c1.l[i] = r.Y.c0.l[i] = r.Y.c1.l[i] = r.Z.c0.l[i] = r.Z.c1.l[i] = 0;
  r.inf = true;
  return r;
}

// lazy28.py madd2: madd-2007-bl with H normalised (its square is an Fp2 square)
template <class M = F2One>
HDNI G2L g2l_madd(const G2L& p, const F2L& x2, const F2L& y2, M m = M()) {
  if (p.inf) return {x2, y2, {l_from(fp_one()), l_from(fp_zero())}, false};
  const F2L Z1Z1 = fs<36, 1>(m, p.Z);
  const F2L U2 = fm(m, x2, Z1Z1);
  const F2L S2 = fm(m, fm(m, y2, p.Z), Z1Z1);
  const F2L H = f2l_norm(f2l_sub<17, 1>(U2, p.X));
  const F2L rr = f2l_norm(f2l_sub<33, 2>(f2l_shl(S2, 1), f2l_shl(p.Y, 1)));
  if (f2l_is_zero(H)) {
    if (f2l_is_zero(rr)) return g2l_dbl(p, m);
    return g2l_infinity();
  }
  const F2L HH = fs<36, 1>(m, H);
  const F2L J1 = fm(m, H, HH), V1 = fm(m, p.X, HH);
  G2L r;
  r.X = f2l_norm(f2l_sub<13, 12>(fs<36, 1>(m, rr), f2l_add(f2l_shl(J1, 2), f2l_shl(V1, 3))));
  r.Y = f2l_norm(
      f2l_sub<9, 8>(fm(m, f2l_sub<16, 1>(f2l_shl(V1, 2), r.X), rr), f2l_shl(fm(m, p.Y, J1), 3)));
  r.Z = fm(m, f2l_shl(p.Z, 1), H);
  r.inf = false;
  return r;
}

// sum_i [a_i] T_i1 + [b_i] T_i2 over a chunk, the joint 32-step ladder of vbatch.hip k_rlc_msm in
// lazy limbs: tab[3i + s - 1] is the affine point (Z = 1 record) added for bit pair s = a_i | 2 b_i
// (T_i1, T_i2, T_i1 + T_i2); the same group element as its stored-word msm_ladder<Fp, true>
template <class Pair>  // uint2 on the device
HD G1J g1l_msm_ladder(const G1J* __restrict__ tab, const Pair* __restrict__ coef, uint32_t first, uint32_t cnt) {
  G1L R = g1l_infinity();
  HB_NOUNROLL for (int bit = 31; bit >= 0; bit--) {
    R = g1l_dbl(R);
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const Pair ab = coef[i];
      const uint32_t sel = ((ab.x >> bit) & 1u) | (((ab.y >> bit) & 1u) << 1);
      const G1J T = tab[3ull * i + (sel ? sel - 1u : 0u)];
      const G1L S = g1l_madd(R, l_from(T.X), l_from(T.Y));
      if (sel) R = S;
    }
  }
  return g1l_to_jac(R);
}

// The sparse coefficient format of the chunk ladders when no bucket MSM reads the coefficients
// (vbatch.hip rlc_digits): r = A + B lambda, A = sum_j u_j 4^j and B = sum_j v_j 4^j over
// RLC_DIGITS = 22 positions, every (u_j, v_j) one of the eight nonzero pairs of {-1, 0, 1}^2 --
// three random bits d: entry d & 3 of (1, 0), (0, 1), (1, 1), (1, -1), negated when d & 4.  Base 4
// with digits in {-1, 0, 1} is a unique representation and |A|, |B| < 2^44 are far below the
// shortest nonzero (a, b) with a + b lambda = 0 mod r (~2^127), so the 8^22 = 2^66 digit strings
// are 2^66 distinct coefficients mod r; one addition per digit: 22 per item where the dense
// 32-bit pair takes 32 (and every digit is nonzero, so no lane adds a point it then drops).
// Digit j of an item's record: bits 3 (j mod 10) .. +2 of word j / 10; word 3 nonzero = usable.
constexpr int RLC_DIGITS = 22;
template <class Quad>
HD uint32_t rlc_digit(const Quad& c, int j) {
  const uint32_t w = j < 10 ? c.x : (j < 20 ? c.y : c.z);
  return (w >> (3 * (j % 10))) & 7u;
}

// sum_i [A_i] T_i1 + [B_i] T_i2 over a chunk in the sparse format: tab[4i + e] the affine points
// T1, T2, T1 + T2, T1 - T2 (Z = 1 records); the 44 doublings shared by the chunk's items
template <class Quad>  // uint4 on the device
HD G1J g1l_msm_ladder_sparse(const G1J* __restrict__ tab, const Quad* __restrict__ coef4, uint32_t first,
                             uint32_t cnt) {
  G1L R = g1l_infinity();
  HB_NOUNROLL for (int j = RLC_DIGITS - 1; j >= 0; j--) {
    if (j != RLC_DIGITS - 1) {
      R = g1l_dbl(R);
      R = g1l_dbl(R);
    }
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const Quad c = coef4[i];
      if (!c.w) continue;
      const uint32_t d = rlc_digit(c, j);
      const G1J T = tab[4ull * i + (d & 3u)];
      R = g1l_madd(R, l_from(T.X), l_from((d & 4u) ? fp_neg(T.Y) : T.Y));
    }
  }
  return g1l_to_jac(R);
}

// lazy28.py jadd2: add-2007-bl as g1l_add with H normalised (its square is an Fp2 square)
template <class M = F2One>
HDNI G2L g2l_add(const G2L& p, const G2L& q, M m = M()) {
  if (p.inf) return q;
  if (q.inf) return p;
  const F2L Z1Z1 = fs<36, 1>(m, p.Z), Z2Z2 = fs<36, 1>(m, q.Z);
  const F2L U1 = fm(m, p.X, Z2Z2), U2 = fm(m, q.X, Z1Z1);
  const F2L S1 = fm(m, fm(m, p.Y, q.Z), Z2Z2);
  const F2L S2 = fm(m, fm(m, q.Y, p.Z), Z1Z1);
  const F2L H = f2l_norm(f2l_sub<2, 1>(U2, U1));
  const F2L rr = f2l_norm(f2l_sub<3, 2>(f2l_shl(S2, 1), f2l_shl(S1, 1)));
  if (f2l_is_zero(H)) {
    if (f2l_is_zero(rr)) return g2l_dbl(p, m);
    return g2l_infinity();
  }
  const F2L HH = fs<36, 1>(m, H);
  const F2L J1 = fm(m, H, HH), V1 = fm(m, U1, HH);
  G2L r;
  r.X = f2l_norm(f2l_sub<13, 12>(fs<36, 1>(m, rr), f2l_add(f2l_shl(J1, 2), f2l_shl(V1, 3))));
  r.Y = f2l_norm(
      f2l_sub<9, 8>(fm(m, f2l_sub<15, 1>(f2l_shl(V1, 2), r.X), rr), f2l_shl(fm(m, S1, J1), 3)));
  r.Z = fm(m, fm(m, f2l_shl(p.Z, 1), q.Z), H);
  r.inf = false;
  return r;
}

HD G2L g2l_from_jac(const G2J& p) {
  return {f2l_from(p.X), f2l_from(p.Y), f2l_from(p.Z), f2_is_zero(p.Z)};
}
HD G2J g2l_to_jac(const G2L& p) {
  if (p.inf) return jac_infinity<Fp2>();
  return {f2l_to(p.X), f2l_to(p.Y), f2l_to(p.Z)};
}

// [|x|] P for a Jacobian P in stored words (ec.h jac_mul_by_xabs), the ladder in lazy limbs;
// `load` returns P again at each of the five additions (not held across the product calls)
template <class LoadP, class M = F2One>
HDNI G2J g2l_mul_by_xabs_l(const LoadP& load, M m = M()) {
  G2L t = g2l_from_jac(load());
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    t = g2l_dbl(t, m);
    if ((HB_X_ABS >> i) & 1) {
#if defined(__HIP_DEVICE_COMPILE__)
      __asm__ volatile("" ::: "memory");
#endif
      t = g2l_add(t, g2l_from_jac(load()), m);
    }
  }
  return g2l_to_jac(t);
}

// the G2 twin of g1l_msm_ladder (k_rlc_msm's per-group signature side): tab[3i + s - 1] affine
template <class Pair>
HD G2J g2l_msm_ladder(const G2J* __restrict__ tab, const Pair* __restrict__ coef, uint32_t first, uint32_t cnt) {
  G2L R = g2l_infinity();
  HB_NOUNROLL for (int bit = 31; bit >= 0; bit--) {
    R = g2l_dbl(R);
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const Pair ab = coef[i];
      const uint32_t sel = ((ab.x >> bit) & 1u) | (((ab.y >> bit) & 1u) << 1);
      if (sel) {
        const G2J T = tab[3ull * i + sel - 1u];
        R = g2l_madd(R, f2l_from(T.X), f2l_from(T.Y));
      }
    }
  }
  return g2l_to_jac(R);
}

// the G2 twin of g1l_msm_ladder_sparse: tab[4i + e] affine S, -psi^2(S), their sum and difference
template <class Quad>
HD G2J g2l_msm_ladder_sparse(const G2J* __restrict__ tab, const Quad* __restrict__ coef4, uint32_t first,
                             uint32_t cnt) {
  G2L R = g2l_infinity();
  HB_NOUNROLL for (int j = RLC_DIGITS - 1; j >= 0; j--) {
    if (j != RLC_DIGITS - 1) {
      R = g2l_dbl(R);
      R = g2l_dbl(R);
    }
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const Quad c = coef4[i];
      if (!c.w) continue;
      const uint32_t d = rlc_digit(c, j);
      const G2J T = tab[4ull * i + (d & 3u)];
      R = g2l_madd(R, f2l_from(T.X), f2l_from((d & 4u) ? f2_neg(T.Y) : T.Y));
    }
  }
  return g2l_to_jac(R);
}

// Q in G2  <=>  psi(Q) == [x] Q (ec.h g2_in_subgroup), the ladder in lazy limbs.  `load` returns
// Q again at each of the five mixed additions instead of the ladder holding its 56 limbs across
// every product call (the kernel re-reads its entry; LICM is kept from hoisting that read)
template <class LoadQ, class M = F2One>
HDNI bool g2_in_subgroup28_l(const LoadQ& load, M m = M()) {
  const G2A q = load();
  if (q.inf) return true;
  G2L t = {f2l_from(q.x), f2l_from(q.y), {l_from(fp_one()), l_from(fp_zero())}, false};
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    t = g2l_dbl(t, m);
    if ((HB_X_ABS >> i) & 1) {
#if defined(__HIP_DEVICE_COMPILE__)
      __asm__ volatile("" ::: "memory");
#endif
      const G2A q2 = load();
      t = g2l_madd(t, f2l_from(q2.x), f2l_from(q2.y), m);
    }
  }
  const G2A q3 = load();
  const G2J xq = t.inf ? jac_infinity<Fp2>() : G2J{f2l_to(t.X), f2l_to(t.Y), f2l_to(t.Z)};
  return jac_eq(g2_psi(jac_from_aff(q3)), jac_neg(xq));
}
HDNI bool g2_in_subgroup28(const G2A& q) {
  return g2_in_subgroup28_l([&]() { return q; });
}

}  // namespace hb
