// Fp: the 381-bit BLS12-381 base field, 12 x 32-bit little-endian limbs, Montgomery form
// (R = 2^392, see fp_mul).  Elements are kept *lazily reduced* in [0, 2p): since 4p < 2^384 the
// no-final-subtraction Montgomery product of two such values is again < 2p, so the
// hot multiply skips the conditional subtraction; canonical form ([0, p)) is produced only
// for comparisons and serialisation.
//
// The product (fp_mul) re-splits its operands into 14 limbs of 28 bits and reduces with
// R = 2^392; all other operations work on the 12 stored words.
#pragma once
#include "hd.h"
#include "consts.h"

namespace hb {

constexpr int NL = 12;

struct Fp {
  uint32_t v[NL];
};

HD Fp fp_from_const(const uint32_t* c) {
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = c[i];
  return r;
}

HD Fp fp_zero() {
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = 0;
  return r;
}

HD Fp fp_one() { return fp_from_const(FP_ONE); }

#if defined(__HIP_DEVICE_COMPILE__)
// Device: explicit carry chains (v_add_co_u32 / v_addc_co_u32, v_sub_co_u32 / v_subb_co_u32).
// The compiler sees them (clang carry builtins), so it can interleave independent chains and
// insert the wait states gfx950 needs between a carry write and its read.
HD uint32_t raw_add(Fp& r, const Fp& a, const Fp& b) {
  unsigned c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  return c;
}
HD uint32_t raw_sub(Fp& r, const Fp& a, const Fp& b) {
  unsigned c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], c, &c);
  return c;
}
HD uint32_t raw_sub_const(Fp& r, const Fp& a, const uint32_t* b) {
  unsigned c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = __builtin_subc(a.v[i], b[i], c, &c);
  return c;
}
HD uint32_t raw_add_const(Fp& r, const Fp& a, const uint32_t* b) {
  unsigned c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = __builtin_addc(a.v[i], b[i], c, &c);
  return c;
}
#else
// a + b over 12 limbs, returns carry
HD uint32_t raw_add(Fp& r, const Fp& a, const Fp& b) {
  uint64_t c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}

// a - b over 12 limbs, returns borrow (1 if a < b)
HD uint32_t raw_sub(Fp& r, const Fp& a, const Fp& b) {
  int64_t c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    c += (int64_t)a.v[i] - (int64_t)b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;  // arithmetic shift: 0 or -1
  }
  return (uint32_t)(c & 1);
}

HD uint32_t raw_sub_const(Fp& r, const Fp& a, const uint32_t* b) {
  int64_t c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    c += (int64_t)a.v[i] - (int64_t)b[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)(c & 1);
}

HD uint32_t raw_add_const(Fp& r, const Fp& a, const uint32_t* b) {
  uint64_t c = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    c += (uint64_t)a.v[i] + b[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
#endif

HD void fp_select(Fp& r, bool take_b, const Fp& a, const Fp& b) {
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = take_b ? b.v[i] : a.v[i];
}

// [0,2p) + [0,2p) -> [0,2p)
HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s, d;
  raw_add(s, a, b);  // < 4p < 2^383: no carry out
  uint32_t borrow = raw_sub_const(d, s, P2_RAW);
  fp_select(s, borrow == 0, s, d);
  return s;
}

HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp d, e;
  uint32_t borrow = raw_sub(d, a, b);
  raw_add_const(e, d, P2_RAW);
  fp_select(d, borrow != 0, d, e);
  return d;
}

HD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }

HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

// ---------------------------------------------------------------------------------------
// Montgomery product over 14 limbs of 28 bits (R = 2^392), carry-free.
//
// The operands are stored as 12 x 32-bit words (cheap exact additions with carry chains); the
// product re-splits them into 14 limbs of 28 bits, so that every partial product a_j b_i (and
// m_j p_i) is < 2^56 and a whole column of product scanning -- at most 14 + 14 such terms plus
// the incoming carry, < 2^61 -- accumulates in ONE 64-bit register with plain 64-bit
// multiply-adds (v_mad_u64_u32) and no carry words: 406 multiply-adds against the 288
// multiply-adds + 288 carry additions of 32-bit limbs.  Column k < 14 fixes m_k = low28 * (-p^-1)
// mod 2^28 so that its low 28 bits cancel; columns 14..26 emit the result limbs.
// Bounds: inputs a, b < 2^384 with a*b < 2^392 p (in particular both < 2p, or one < 2^384 and the
// other < p) give a result < 2p, so the [0, 2p) lazy reduction of the rest of the code holds.
// All of it is plain C++: the compiler schedules it and handles every gfx950 hazard (the r01
// hand-written register-convention subroutine is gone).
HD void fp_split28(uint32_t* l, const uint32_t* w) {  // 12 x 32 -> 14 x 28
  HB_UNROLL for (int j = 0; j < 14; j++) {
    const int bit = 28 * j, i = bit >> 5, s = bit & 31;
    uint32_t v = w[i] >> s;
    if (s > 4 && i + 1 < 12) v |= w[i + 1] << (32 - s);
    l[j] = v & 0x0FFFFFFFu;
  }
}
HD void fp_join28(uint32_t* w, const uint32_t* l) {  // 14 x 28 (normalised, < 2^384) -> 12 x 32
  HB_UNROLL for (int i = 0; i < 12; i++) {
    const int bit = 32 * i, j = bit / 28, s = bit % 28;  // s <= 24: two limbs cover a word
    w[i] = (l[j] >> s) | (l[j + 1] << (28 - s));
  }
}

// HB_MADD: a multiply-add whose accumulator the compiler may not reassociate (a register barrier;
// ec28.h mul28x2_core, the paired G1 products).
#if defined(__HIP_DEVICE_COMPILE__)
#define HB_MADD(acc, x, y)                \
  do {                                    \
    acc += (uint64_t)(x) * (y);           \
    __asm__("" : "+v"(acc));              \
  } while (0)
#else
#define HB_MADD(acc, x, y) acc += (uint64_t)(x) * (y)
#endif

// one column of the reduction: m_k p_{k-j} terms for the columns k >= 14 (and j < k below)
#define HB_MONT28_TAIL(acc, m, k, r)                                                     \
  if ((k) < 14) {                                                                       \
    m[(k)] = ((uint32_t)(acc) * HB_P_N0_28) & 0x0FFFFFFFu;                               \
    acc += (uint64_t)m[(k)] * P28[0];                                                    \
  } else {                                                                              \
    r[(k) - 14] = (uint32_t)(acc) & 0x0FFFFFFFu;                                          \
  }                                                                                     \
  acc >>= 28;

// the products on operands already in 14 x 28-bit limbs (values < 2p; the outputs are again
// normalised 28-bit limbs of a value < 2p, so they chain without a join / split in between)
HD void fp_mul28_core(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[14];
  uint64_t acc = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) acc += (uint64_t)a[j] * b[k - j];
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P28[k - j];
    HB_MONT28_TAIL(acc, m, k, r)
  }
  r[13] = (uint32_t)acc;
}

// squaring: the cross products a_j a_{k-j}, j < k - j, once against the doubled limb
HD void fp_sqr28_core(uint32_t* r, const uint32_t* a) {
  uint32_t a2[14], m[14];
  HB_UNROLL for (int j = 0; j < 14; j++) a2[j] = a[j] << 1;
  uint64_t acc = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      if (2 * j < k) acc += (uint64_t)a2[j] * a[k - j];
      else if (2 * j == k) acc += (uint64_t)a[j] * a[j];
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P28[k - j];
    HB_MONT28_TAIL(acc, m, k, r)
  }
  r[13] = (uint32_t)acc;
}

HD void fp_mul_core(uint32_t* out, const uint32_t* aw, const uint32_t* bw) {
  uint32_t a[14], b[14], r[14];
  fp_split28(a, aw);
  fp_split28(b, bw);
  fp_mul28_core(r, a, b);
  fp_join28(out, r);
}

HD void fp_sqr_core(uint32_t* out, const uint32_t* aw) {
  uint32_t a[14], r[14];
  fp_split28(a, aw);
  fp_sqr28_core(r, a);
  fp_join28(out, r);
}

// Fp2 products without intermediate reductions (xi = -1 + ... tower: u^2 = -1):
//   real = (a0 b0 - a1 b1) / R   imag = (a0 b1 + a1 b0) / R
// one product-scanning pass per output coefficient, both in the same column loop (two independent
// multiply-add chains).  The real part's negative terms are signed multiply-adds against negated
// limbs (two's complement in the same 64-bit accumulator, arithmetic carry shifts); its result lies
// in (-p, 2p) and is moved to [0, 2p) by one conditional addition of p.  Same multiply-add count as
// three Montgomery products (Karatsuba) but no Fp additions/subtractions around them, two operand
// splits fewer and one output conversion fewer.
#define HB_MONT28_TAIL_S(acc, m, k, r)                                                   \
  if ((k) < 14) {                                                                       \
    m[(k)] = ((uint32_t)(acc) * HB_P_N0_28) & 0x0FFFFFFFu;                               \
    acc += (uint64_t)m[(k)] * P28[0];                                                    \
  } else {                                                                              \
    r[(k) - 14] = (uint32_t)(acc) & 0x0FFFFFFFu;                                          \
  }                                                                                     \
  acc = (uint64_t)((int64_t)(acc) >> 28);

HD void fp2_fix_neg(uint32_t* out, const uint32_t* r, bool neg) {  // r (mod 2^384) + p if neg
  uint32_t w[12], s[12];
  fp_join28(w, r);
  unsigned c = 0;
  HB_UNROLL for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)w[i] + P_RAW[i] + c;
    s[i] = (uint32_t)t;
    c = (unsigned)(t >> 32);
  }
  HB_UNROLL for (int i = 0; i < 12; i++) out[i] = neg ? s[i] : w[i];
}

HD void fp2_mul_core(uint32_t* o0, uint32_t* o1, const uint32_t* a0w, const uint32_t* a1w, const uint32_t* b0w,
                     const uint32_t* b1w) {
  uint32_t a0[14], a1[14], b0[14], b1[14], m0[14], m1[14], r0[14], r1[14];
  int32_t na1[14];
  fp_split28(a0, a0w);
  fp_split28(a1, a1w);
  fp_split28(b0, b0w);
  fp_split28(b1, b1w);
  HB_UNROLL for (int j = 0; j < 14; j++) na1[j] = -(int32_t)a1[j];
  uint64_t ar = 0, ai = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      ar += (uint64_t)a0[j] * b0[k - j];
      ar += (uint64_t)((int64_t)na1[j] * (int64_t)(int32_t)b1[k - j]);
      ai += (uint64_t)a0[j] * b1[k - j];
      ai += (uint64_t)a1[j] * b0[k - j];
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) {
        ar += (uint64_t)m0[j] * P28[k - j];
        ai += (uint64_t)m1[j] * P28[k - j];
      }
    HB_MONT28_TAIL_S(ar, m0, k, r0)
    HB_MONT28_TAIL(ai, m1, k, r1)
  }
  r0[13] = (uint32_t)ar;
  r1[13] = (uint32_t)ai;
  fp2_fix_neg(o0, r0, (int64_t)ar < 0);
  fp_join28(o1, r1);
}

// (a0 + a1 u)^2 = (a0^2 - a1^2) + 2 a0 a1 u, squares with the doubled-limb cross products
HD void fp2_sqr_core(uint32_t* o0, uint32_t* o1, const uint32_t* a0w, const uint32_t* a1w) {
  uint32_t a0[14], a1[14], d0[14], m0[14], m1[14], r0[14], r1[14];
  int32_t na1[14], nd1[14];
  fp_split28(a0, a0w);
  fp_split28(a1, a1w);
  HB_UNROLL for (int j = 0; j < 14; j++) {
    d0[j] = a0[j] << 1;
    na1[j] = -(int32_t)a1[j];
    nd1[j] = -(int32_t)(a1[j] << 1);
  }
  uint64_t ar = 0, ai = 0;
  HB_UNROLL for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    HB_UNROLL for (int j = lo; j <= hi; j++) {
      if (2 * j < k) {
        ar += (uint64_t)d0[j] * a0[k - j];
        ar += (uint64_t)((int64_t)nd1[j] * (int64_t)(int32_t)a1[k - j]);
      } else if (2 * j == k) {
        ar += (uint64_t)a0[j] * a0[j];
        ar += (uint64_t)((int64_t)na1[j] * (int64_t)(int32_t)a1[j]);
      }
      ai += (uint64_t)d0[j] * a1[k - j];
    }
    HB_UNROLL for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) {
        ar += (uint64_t)m0[j] * P28[k - j];
        ai += (uint64_t)m1[j] * P28[k - j];
      }
    HB_MONT28_TAIL_S(ar, m0, k, r0)
    HB_MONT28_TAIL(ai, m1, k, r1)
  }
  r0[13] = (uint32_t)ar;
  r1[13] = (uint32_t)ai;
  fp2_fix_neg(o0, r0, (int64_t)ar < 0);
  fp_join28(o1, r1);
}

#if defined(__HIP_DEVICE_COMPILE__)
// Device: one out-of-line copy per code object (standard calling convention: the operands travel
// in VGPRs as 12-wide vectors; struct arguments would go through scratch).  Everything around it
// is inlined in the kernels (HB_FAST_FPMUL), so the product is the only call.
typedef uint32_t u32x12 __attribute__((ext_vector_type(12)));
__device__ __noinline__ static u32x12 fp_mul_leaf(u32x12 a, u32x12 b) {
  uint32_t x[12], y[12], r[12];
  HB_UNROLL for (int i = 0; i < 12; i++) {
    x[i] = a[i];
    y[i] = b[i];
  }
  fp_mul_core(r, x, y);
  u32x12 o;
  HB_UNROLL for (int i = 0; i < 12; i++) o[i] = r[i];
  return o;
}
__device__ __noinline__ static u32x12 fp_sqr_leaf(u32x12 a) {
  uint32_t x[12], r[12];
  HB_UNROLL for (int i = 0; i < 12; i++) x[i] = a[i];
  fp_sqr_core(r, x);
  u32x12 o;
  HB_UNROLL for (int i = 0; i < 12; i++) o[i] = r[i];
  return o;
}
typedef uint32_t u32x24 __attribute__((ext_vector_type(24)));
// The Fp2 product has 48 argument dwords; the calling convention passes 32 in VGPRs and the rest
// on the scratch stack (dword stores and loads around every call).  The second operand therefore
// travels through this per-lane LDS slot instead (k-major pairs: conflict-free 64-bit accesses).
// Every kernel runs 64-lane workgroups, one wave each (BLOCK / dim3(64) at every launch).
// HB_ARG_LANES: threads of the largest workgroup of the translation unit (64: one wave; the
// pairing unit's two-wave producer/consumer kernel needs a slot per thread of both waves)
#ifndef HB_ARG_LANES
#define HB_ARG_LANES 64
#endif
#define HB_FP2_ARG_SLOTS 14  // 12 pairs for the stored-word product, 14 for ec28.h's lazy one
__shared__ uint2 hb_fp2_arg[HB_FP2_ARG_SLOTS * HB_ARG_LANES];
__device__ __noinline__ static u32x24 fp2_mul_leaf(u32x24 a) {
  uint32_t x0[12], x1[12], y0[12], y1[12], r0[12], r1[12];
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
  fp2_mul_core(r0, r1, x0, x1, y0, y1);
  u32x24 o;
  HB_UNROLL for (int i = 0; i < 12; i++) {
    o[i] = r0[i];
    o[12 + i] = r1[i];
  }
  return o;
}
__device__ __noinline__ static u32x24 fp2_sqr_leaf(u32x24 a) {
  uint32_t x0[12], x1[12], r0[12], r1[12];
  HB_UNROLL for (int i = 0; i < 12; i++) {
    x0[i] = a[i];
    x1[i] = a[12 + i];
  }
  fp2_sqr_core(r0, r1, x0, x1);
  u32x24 o;
  HB_UNROLL for (int i = 0; i < 12; i++) {
    o[i] = r0[i];
    o[12 + i] = r1[i];
  }
  return o;
}
HD void fp2_mul_pair(Fp& r0, Fp& r1, const Fp& a0, const Fp& a1, const Fp& b0, const Fp& b1) {
  u32x24 av;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    av[i] = a0.v[i];
    av[12 + i] = a1.v[i];
  }
  const uint32_t lane = threadIdx.x & (HB_ARG_LANES - 1u);
  HB_UNROLL for (int k = 0; k < 6; k++) {
    hb_fp2_arg[k * HB_ARG_LANES + lane] = make_uint2(b0.v[2 * k], b0.v[2 * k + 1]);
    hb_fp2_arg[(6 + k) * HB_ARG_LANES + lane] = make_uint2(b1.v[2 * k], b1.v[2 * k + 1]);
  }
  u32x24 rv = fp2_mul_leaf(av);
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r0.v[i] = rv[i];
    r1.v[i] = rv[12 + i];
  }
}
HD void fp2_sqr_pair(Fp& r0, Fp& r1, const Fp& a0, const Fp& a1) {
  u32x24 av;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    av[i] = a0.v[i];
    av[12 + i] = a1.v[i];
  }
  u32x24 rv = fp2_sqr_leaf(av);
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r0.v[i] = rv[i];
    r1.v[i] = rv[12 + i];
  }
}
HD Fp fp_mul(const Fp& a, const Fp& b) {
  HB_COUNT_FP_MUL();
  u32x12 av, bv;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    av[i] = a.v[i];
    bv[i] = b.v[i];
  }
  u32x12 rv = fp_mul_leaf(av, bv);
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = rv[i];
  return r;
}
HD Fp fp_sqr(const Fp& a) {
  HB_COUNT_FP_MUL();
  u32x12 av;
  HB_UNROLL for (int i = 0; i < NL; i++) av[i] = a.v[i];
  u32x12 rv = fp_sqr_leaf(av);
  Fp r;
  HB_UNROLL for (int i = 0; i < NL; i++) r.v[i] = rv[i];
  return r;
}
// chains of products in 28-bit limbs (the constant exponentiations): 14 limbs in a 16-wide vector
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
__device__ __noinline__ static u32x16 fp_mul28_leaf(u32x16 a, u32x16 b) {
  uint32_t x[14], y[14], r[14];
  HB_UNROLL for (int i = 0; i < 14; i++) {
    x[i] = a[i];
    y[i] = b[i];
  }
  fp_mul28_core(r, x, y);
  u32x16 o;
  HB_UNROLL for (int i = 0; i < 14; i++) o[i] = r[i];
  return o;
}
__device__ __noinline__ static u32x16 fp_sqr28_leaf(u32x16 a) {
  uint32_t x[14], r[14];
  HB_UNROLL for (int i = 0; i < 14; i++) x[i] = a[i];
  fp_sqr28_core(r, x);
  u32x16 o;
  HB_UNROLL for (int i = 0; i < 14; i++) o[i] = r[i];
  return o;
}
struct Fp28 {
  u32x16 l;
};
HD Fp28 fp28_mul(const Fp28& a, const Fp28& b) {
  HB_COUNT_FP_MUL();
  return {fp_mul28_leaf(a.l, b.l)};
}
HD Fp28 fp28_sqr(const Fp28& a) {
  HB_COUNT_FP_MUL();
  return {fp_sqr28_leaf(a.l)};
}
HD Fp28 fp28_from(const Fp& a) {
  uint32_t x[14];
  fp_split28(x, a.v);
  Fp28 r;
  HB_UNROLL for (int i = 0; i < 14; i++) r.l[i] = x[i];
  r.l[14] = r.l[15] = 0;
  return r;
}
HD Fp fp28_to(const Fp28& a) {
  uint32_t x[14];
  HB_UNROLL for (int i = 0; i < 14; i++) x[i] = a.l[i];
  Fp r;
  fp_join28(r.v, x);
  return r;
}
#else
// Host (test harness, CPU baseline): the same products with 64-bit words (hostmul64.h: identical
// results); HB_HOST_MUL28 keeps the 28-bit cores
}  // namespace hb
#include "hostmul64.h"
namespace hb {
HD void fp2_mul_pair(Fp& r0, Fp& r1, const Fp& a0, const Fp& a1, const Fp& b0, const Fp& b1) {
#if defined(HB_HOST_MUL28)
  fp2_mul_core(r0.v, r1.v, a0.v, a1.v, b0.v, b1.v);
#else
  hm64::fp2_mul_words(r0.v, r1.v, a0.v, a1.v, b0.v, b1.v);
#endif
}
HD void fp2_sqr_pair(Fp& r0, Fp& r1, const Fp& a0, const Fp& a1) {
#if defined(HB_HOST_MUL28)
  fp2_sqr_core(r0.v, r1.v, a0.v, a1.v);
#else
  hm64::fp2_mul_words(r0.v, r1.v, a0.v, a1.v, a0.v, a1.v);
#endif
}
HD Fp fp_mul(const Fp& a, const Fp& b) {
  HB_COUNT_FP_MUL();
  Fp r;
#if defined(HB_HOST_MUL28)
  fp_mul_core(r.v, a.v, b.v);
#else
  hm64::mul_words(r.v, a.v, b.v);
#endif
  return r;
}
HD Fp fp_sqr(const Fp& a) {
  HB_COUNT_FP_MUL();
  Fp r;
#if defined(HB_HOST_MUL28)
  fp_sqr_core(r.v, a.v);
#else
  hm64::mul_words(r.v, a.v, a.v);
#endif
  return r;
}
struct Fp28 {
  uint32_t l[14];
};
HD Fp28 fp28_mul(const Fp28& a, const Fp28& b) {
  HB_COUNT_FP_MUL();
  Fp28 r;
#if defined(HB_HOST_MUL28)
  fp_mul28_core(r.l, a.l, b.l);
#else
  hm64::mul_limbs28(r.l, a.l, b.l);
#endif
  return r;
}
HD Fp28 fp28_sqr(const Fp28& a) {
  HB_COUNT_FP_MUL();
  Fp28 r;
#if defined(HB_HOST_MUL28)
  fp_sqr28_core(r.l, a.l);
#else
  hm64::mul_limbs28(r.l, a.l, a.l);
#endif
  return r;
}
HD Fp28 fp28_from(const Fp& a) {
  Fp28 r;
  fp_split28(r.l, a.v);
  return r;
}
HD Fp fp28_to(const Fp28& a) {
  Fp r;
  fp_join28(r.v, a.l);
  return r;
}
#endif



// reduce [0,2p) -> [0,p)
HD Fp fp_canon(const Fp& a) {
  Fp d;
  uint32_t borrow = raw_sub_const(d, a, P_RAW);
  Fp r;
  fp_select(r, borrow == 0, a, d);
  return r;
}

HD bool fp_is_zero(const Fp& a) {
  Fp c = fp_canon(a);
  uint32_t acc = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) acc |= c.v[i];
  return acc == 0;
}

HD bool fp_eq(const Fp& a, const Fp& b) { return fp_is_zero(fp_sub(a, b)); }

HD Fp fp_to_mont(const Fp& a) { return fp_mul(a, fp_from_const(FP_R2)); }

HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.v[0] = 1;
  return fp_canon(fp_mul(a, one));
}

HD Fp fp_mul_small(const Fp& a, int k) {
  // k in {2,3,4,8,...}: repeated doubling/adding keeps lazily reduced range
  Fp r = a;
  Fp acc = fp_zero();
  while (k) {
    if (k & 1) acc = fp_add(acc, r);
    r = fp_dbl(r);
    k >>= 1;
  }
  return acc;
}

// a^e for a fixed exponent given as 12 little-endian limbs (left-to-right binary).
HDNI Fp fp_pow_const(const Fp& a, const uint32_t* e, int top_bit) {
  Fp r = fp_one();
  HB_NOUNROLL for (int i = top_bit; i >= 0; i--) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = fp_mul(r, a);
  }
  return r;
}

// Sliding-window exponentiation by a constant schedule (consts.h WIN_*, w = 4): 7 products for
// the odd powers a^1 .. a^15, then per window its squarings and one product -- 79 windows, i.e.
// about 86 products against the 229 set bits the binary method above multiplies by.  The table
// entry of the next window is read before that window's squarings, so its load (the table is
// indexed by a wave-uniform digit) overlaps them.
//
// The whole chain stays in 14 x 28-bit limbs (fp28_*): every product's output is a valid input of
// the next, so the split of both operands and the join of the result -- ~45 of a product's ~545
// instructions -- happen once per exponentiation instead of once per product.
HDNI Fp fp_pow_win(const Fp& a, const uint8_t* sch, int n) {
  Fp28 tab[8];
  tab[0] = fp28_from(a);
  const Fp28 a2 = fp28_sqr(tab[0]);
  HB_UNROLL for (int i = 1; i < 8; i++) tab[i] = fp28_mul(tab[i - 1], a2);
  Fp28 r = tab[(sch[1] >> 1) & 7];
  HB_NOUNROLL for (int k = 1; k < n; k++) {
    const int sq = sch[2 * k], d = sch[2 * k + 1];
    const Fp28 m = tab[(d >> 1) & 7];
    HB_NOUNROLL for (int j = 0; j < sq; j++) r = fp28_sqr(r);
    if (d) r = fp28_mul(r, m);
  }
  return fp28_to(r);
}

// a^(p-2): the inversion by exponentiation (86 products + 380 squarings), kept for tests and A/B
HD Fp fp_inv_pow(const Fp& a) { return fp_pow_win(a, WIN_P_MINUS_2, WIN_P_MINUS_2_N); }

// ---------------------------------------------------------------------------------------
// Inversion by divsteps (round 4): the extended binary GCD of Bernstein and Yang ("Fast
// constant-time gcd computation and modular inversion", 2019) in batches of 30 divsteps, on
// signed 30-bit limbs -- the low 32 bits of f and g decide a batch's 2x2 transition matrix,
// which is then applied to the full f, g (exactly) and to the cofactors d, e (mod p, with a
// multiple of p that clears their low 30 bits).  The step structure (divsteps_30, update_fg_30,
// update_de_30, normalize_30 and the branch-free c1/c2/c3 masks with zeta) follows the published
// safegcd implementation of libsecp256k1's modinv32 (Bernstein & Yang, "Fast constant-time gcd
// computation and modular inversion", 2019; MIT licence), with BLS12-381's modulus, limb count and
// constants.  About 15 32-bit operations per divstep and
// ~300 per batch for the updates; the values are public, so the loop stops once g = 0 (on the
// device: once every lane of the wave has g = 0).  ~25-35 batches for random 381-bit inputs
// against the 466 Montgomery products of fp_inv_pow.  The result is the integer inverse z of
// the Montgomery representative, turned back into Montgomery form by one product with R^3.
struct S30 {
  int32_t v[13];  // value = sum v[i] 2^(30 i); limbs 0..11 in [0, 2^30) after an update, 12 signed
};
constexpr int32_t kM30 = 0x3FFFFFFF;

// 30 divsteps of (zeta, f, g) on the low bits (f odd); t = (u, v, q, r), the transition matrix
// scaled by 2^30: 2^30 f' = u f + v g, 2^30 g' = q f + r g.  zeta = -(delta + 1/2), branch-free.
HD int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, int32_t* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  HB_UNROLL for (int i = 0; i < 30; i++) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t c2 = 0u - (g & 1u);           // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    const uint32_t c3 = c1 & c2;  // swap: zeta < 0 and g odd
    zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
    f += g & c3;
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return zeta;
}

// (f, g) <- t (f, g) / 2^30, exactly
HD void update_fg_30(S30& f, S30& g, const int32_t* t) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];  // 32 x 32 -> 64-bit products (v_mad_i64_i32)
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0], cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
  HB_UNROLL for (int i = 1; i < 13; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)cf & kM30;
    g.v[i - 1] = (int32_t)cg & kM30;
    cf >>= 30;
    cg >>= 30;
  }
  f.v[12] = (int32_t)cf;
  g.v[12] = (int32_t)cg;
}

// (d, e) <- (t (d, e) + p (md, me)) / 2^30 with md, me making the low 30 bits zero; d, e stay in
// (-2p, p)
HD void update_de_30(S30& d, S30& e, const int32_t* t) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[12] >> 31, se = e.v[12] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0], ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((HB_P_INV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)((HB_P_INV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)P30[0] * md;
  ce += (int64_t)P30[0] * me;
  cd >>= 30;
  ce >>= 30;
  HB_UNROLL for (int i = 1; i < 13; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)P30[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)P30[i] * me;
    d.v[i - 1] = (int32_t)cd & kM30;
    e.v[i - 1] = (int32_t)ce & kM30;
    cd >>= 30;
    ce >>= 30;
  }
  d.v[12] = (int32_t)cd;
  e.v[12] = (int32_t)ce;
}

// d in (-2p, p), negated if f = -1 -> [0, p)
HD void normalize_30(S30& d, int32_t f_sign) {
  int32_t c = d.v[12] >> 31;  // d < 0: + p
  HB_UNROLL for (int i = 0; i < 13; i++) d.v[i] += P30[i] & c;
  const int32_t n = f_sign >> 31;  // f = -1: negate
  HB_UNROLL for (int i = 0; i < 13; i++) d.v[i] = (d.v[i] ^ n) - n;
  HB_UNROLL for (int i = 0; i < 12; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= kM30;
  }
  c = d.v[12] >> 31;
  HB_UNROLL for (int i = 0; i < 13; i++) d.v[i] += P30[i] & c;
  HB_UNROLL for (int i = 0; i < 12; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= kM30;
  }
}

constexpr int FP_INV_BATCHES = 40;  // 1200 divsteps >= the 1101 that 381-bit inputs can need

// a^-1 (0 -> 0, like a^(p-2)); batches: optional count of the batches run (tests).  Public data
// (kEarlyExit): the loop stops once g = 0 in every lane of the wave.  Secret-dependent values
// (fp_inv_ct: the affine conversion of sk * H(m) and sk * g1 in k_sign / k_sk_to_pk) always run
// the FP_INV_BATCHES batches, so the trip count does not depend on the input.
template <bool kEarlyExit>
HDNI Fp fp_inv_t(const Fp& a, int* batches = nullptr) {
  const Fp c = fp_canon(a);
  S30 f, g, d, e;
  HB_UNROLL for (int i = 0; i < 13; i++) {  // g = c in 30-bit limbs
    const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
    uint32_t x = c.v[w] >> sh;
    if (sh > 2 && w + 1 < 12) x |= c.v[w + 1] << (32 - sh);
    g.v[i] = (int32_t)(x & (uint32_t)kM30);
    f.v[i] = P30[i];
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  int32_t zeta = -1;
  int b = 0;
  HB_NOUNROLL for (; b < FP_INV_BATCHES; b++) {
    int32_t t[4];
    zeta = divsteps_30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30(d, e, t);
    update_fg_30(f, g, t);
    if (kEarlyExit) {
      int32_t nz = 0;
      HB_UNROLL for (int i = 0; i < 13; i++) nz |= g.v[i];
#if defined(__HIP_DEVICE_COMPILE__)
      if (!__any(nz != 0)) {  // every lane of the wave is done
        b++;
        break;
      }
#else
      if (nz == 0) {
        b++;
        break;
      }
#endif
    }
  }
  if (batches) *batches = b;
  normalize_30(d, f.v[12]);
  Fp z;  // d (< p) in 32-bit words
  HB_UNROLL for (int i = 0; i < 12; i++) {
    const int bit = 32 * i, j = bit / 30, sh = bit % 30;
    uint32_t x = (uint32_t)d.v[j] >> sh;
    if (j + 1 < 13) x |= (uint32_t)d.v[j + 1] << (30 - sh);
    if (sh > 28 && j + 2 < 13) x |= (uint32_t)d.v[j + 2] << (60 - sh);
    z.v[i] = x;
  }
  return fp_mul(z, fp_from_const(FP_RCUBE));
}
HD Fp fp_inv(const Fp& a, int* batches = nullptr) { return fp_inv_t<true>(a, batches); }
HD Fp fp_inv_ct(const Fp& a, int* batches = nullptr) { return fp_inv_t<false>(a, batches); }

// Legendre-style squareness check via a^((p-1)/2) (1: square, 0: zero).
HD bool fp_is_square(const Fp& a) {
  Fp t = fp_pow_win(a, WIN_LEGENDRE, WIN_LEGENDRE_N);
  return fp_is_zero(a) || fp_eq(t, fp_one());
}

// sqrt for p = 3 mod 4; returns false if a is not a square.
HDNI bool fp_sqrt(Fp& r, const Fp& a) {
  r = fp_pow_win(a, WIN_SQRT, WIN_SQRT_N);
  return fp_eq(fp_sqr(r), a);
}

// ---- byte conversions (big-endian, canonical) ----
HD void fp_from_be_raw(Fp& r, const uint8_t* b) {  // 48 bytes -> raw limbs (not reduced)
  HB_UNROLL for (int i = 0; i < NL; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

HD void fp_to_be_raw(uint8_t* b, const Fp& a) {
  HB_UNROLL for (int i = 0; i < NL; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.v[i] >> 24);
    q[1] = (uint8_t)(a.v[i] >> 16);
    q[2] = (uint8_t)(a.v[i] >> 8);
    q[3] = (uint8_t)a.v[i];
  }
}

// raw < p ?
HD bool fp_raw_lt_p(const Fp& a) {
  Fp d;
  return raw_sub_const(d, a, P_RAW) != 0;
}

// canonical (non-Montgomery) value > (p-1)/2 ?  i.e. 2*v > p-1  <=>  2*v >= p
HD bool fp_raw_is_lex_largest(const Fp& v) {
  Fp d;
  raw_add(d, v, v);  // v < p < 2^381 so no carry
  Fp e;
  return raw_sub_const(e, d, P_RAW) == 0;
}

}  // namespace hb
