// Fp: the 381-bit BLS12-381 base field, 12 x 32-bit little-endian limbs, Montgomery form
// (R = 2^384).  Elements are kept *lazily reduced* in [0, 2p): since 4p < R the
// no-final-subtraction Montgomery product of two such values is again < 2p, so the
// hot multiply skips the conditional subtraction; canonical form ([0, p)) is produced only
// for comparisons and serialisation.
//
// The product computes x*y+acc with v_mad_u64_u32 (see fp_mul); the limb count and layout
// match the structure-of-arrays layout the kernels load from HBM.
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

// Montgomery product, CIOS with the "no-carry" simplification (top limb of p < 2^31-1).
// Inputs in [0,2p), output in [0,2p).  (b may be any value < 2^384 if a < p: the
// intermediate stays below a + p; the result is then < 2p as well.)
HD Fp fp_mul_generic(const Fp& a, const Fp& b) {
  HB_COUNT_FP_MUL();
  uint32_t t[NL];
  HB_UNROLL for (int j = 0; j < NL; j++) t[j] = 0;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    uint64_t A = (uint64_t)a.v[0] * b.v[i] + t[0];
    t[0] = (uint32_t)A;
    A >>= 32;
    uint32_t m = t[0] * HB_P_N0;
    uint64_t C = (uint64_t)m * P_RAW[0] + t[0];
    C >>= 32;
    HB_UNROLL for (int j = 1; j < NL; j++) {
      A = (uint64_t)a.v[j] * b.v[i] + t[j] + A;
      t[j] = (uint32_t)A;
      A >>= 32;
      C = (uint64_t)m * P_RAW[j] + t[j] + C;
      t[j - 1] = (uint32_t)C;
      C >>= 32;
    }
    t[NL - 1] = (uint32_t)(C + A);
  }
  Fp r;
  HB_UNROLL for (int j = 0; j < NL; j++) r.v[j] = t[j];
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Device: product-scanning ("FIPS") Montgomery product on v_mad_u64_u32 carry chains.
// Column k of a*b + m*p is accumulated in a 64-bit VGPR pair `acc` plus a third word `c2`
// that collects the carry-outs of the 64-bit multiply-adds (VCC -> v_addc_co_u32).  Per
// column the low word of the first 12 columns selects m_k = acc_lo * (-p^-1) mod 2^32 so that
// it cancels; columns 12..22 emit the result limbs.  288 v_mad_u64_u32 + 288 v_addc_co_u32 +
// ~70 moves per product (the compiler's own lowering of the CIOS loop spent 764 extra v_movs).
// Same bounds as fp_mul_generic: inputs < 2p, output < 2p (4p < 2^384).
// The asm blocks carry 1 or 2 (a_j b_{k-j}, m_j p_{k-j}) pairs each: fewer blocks means fewer
// of the s_nop's the hazard recognizer places after every inline-asm statement.
__device__ __forceinline__ void fips_mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void fips_mac_s(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2) : "v"(a), "s"(b) : "vcc");
}
__device__ __forceinline__ void fips_mac2(uint64_t& acc, uint32_t& c2, uint32_t a0, uint32_t b0, uint32_t m0,
                                          uint32_t p0) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2) : "v"(a0), "v"(b0), "v"(m0), "s"(p0) : "vcc");
}
__device__ __forceinline__ void fips_mac4(uint64_t& acc, uint32_t& c2, uint32_t a0, uint32_t b0, uint32_t m0,
                                          uint32_t p0, uint32_t a1, uint32_t b1, uint32_t m1, uint32_t p1) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2)
      : "v"(a0), "v"(b0), "v"(m0), "s"(p0), "v"(a1), "v"(b1), "v"(m1), "s"(p1)
      : "vcc");
}

#if defined(HB_FAST_FPMUL)
// pipeline.hip: the product is the hand-scheduled subroutine hb_fpmul (fpmul_asm.inc,
// generated by charon_amd/tools/gen_fpmul_asm.py: the same FIPS schedule), entered with a fixed
// register convention: a in v0-v11, b in v12-v23, result in v24-v35, clobbering only v36-v50,
// vcc and s30-s48.  The standard calling convention would force every value a caller keeps
// across the call into the 112 callee-saved VGPRs; with this one the caller's state lives in
// v51-v255.  The subroutine is emitted once per code object, inside the never-launched kernel
// hb_fpmul_holder (HB_DEFINE_FPMUL_SUBROUTINE).
#include "fpmul_asm.inc"

HD Fp fp_mul(const Fp& a, const Fp& b) {
  HB_COUNT_FP_MUL();
  Fp r;
  asm volatile(
      "s_getpc_b64 s[34:35]\n\t"
      "s_add_u32 s34, s34, hb_fpmul@rel32@lo+4\n\t"
      "s_addc_u32 s35, s35, hb_fpmul@rel32@hi+12\n\t"
      "s_swappc_b64 s[30:31], s[34:35]"
      : HB_FPMUL_OUTPUTS(r)
      : HB_FPMUL_INPUTS(a, b)
      : HB_FPMUL_CLOBBERS);
  return r;
}

#define HB_DEFINE_FPMUL_SUBROUTINE(holder)                           \
  __global__ void holder() {                                \
    asm volatile("\ts_endpgm\n\t.p2align 8\n\t.globl hb_fpmul\n"     \
                 "\t.hidden hb_fpmul\n\t.type hb_fpmul,@function\n" \
                 "hb_fpmul:\n" HB_FPMUL_ASM_BODY);                     \
  }
#else
// hipbls.hip: one out-of-line copy of the product (standard calling convention); operands travel
// in VGPRs as 12-wide vectors (struct arguments would be passed through scratch memory).
typedef uint32_t u32x12 __attribute__((ext_vector_type(12)));
__device__ __noinline__ static u32x12 fp_mul_leaf(u32x12 a, u32x12 b) {
  uint32_t m[NL];
  u32x12 t;
  uint64_t acc = 0;
  uint32_t c2 = 0;
  HB_UNROLL for (int k = 0; k < 2 * NL - 1; k++) {
    const int lo = k < NL ? 0 : k - (NL - 1);
    const int hi = k < NL ? k - 1 : NL - 1;  // pairs j in [lo, hi]
    int j = lo;
    HB_UNROLL for (; j + 1 <= hi; j += 2)
      fips_mac4(acc, c2, a[j], b[k - j], m[j], P_RAW[k - j], a[j + 1], b[k - j - 1], m[j + 1], P_RAW[k - j - 1]);
    if (j <= hi) fips_mac2(acc, c2, a[j], b[k - j], m[j], P_RAW[k - j]);
    if (k < NL) {
      fips_mac(acc, c2, a[k], b[0]);
      m[k] = (uint32_t)acc * HB_P_N0;
      fips_mac_s(acc, c2, m[k], P_RAW[0]);  // low word becomes 0
    } else {
      t[k - NL] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  t[NL - 1] = (uint32_t)acc;
  return t;
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
#endif
#else
HD Fp fp_mul(const Fp& a, const Fp& b) { return fp_mul_generic(a, b); }
#endif

HD Fp fp_sqr(const Fp& a) { return fp_mul(a, a); }

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

HD Fp fp_inv(const Fp& a) { return fp_pow_const(a, EXP_P_MINUS_2, 380); }

// Legendre-style squareness check via a^((p-1)/2) (1: square, 0: zero).
HD bool fp_is_square(const Fp& a) {
  Fp t = fp_pow_const(a, EXP_LEGENDRE, 379);
  return fp_is_zero(a) || fp_eq(t, fp_one());
}

// sqrt for p = 3 mod 4; returns false if a is not a square.
HDNI bool fp_sqrt(Fp& r, const Fp& a) {
  r = fp_pow_const(a, EXP_SQRT, 379);
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
