// Fr: the 255-bit scalar field of BLS12-381 (8 x 32-bit limbs, Montgomery form, R = 2^256).
// Used for Lagrange coefficients lambda_i(0) = prod_{j!=i} x_j / (x_j - x_i)
// (ThresholdAggregate, herumi.go:249-286 -> mcl LagrangeInterpolation) and for the
// polynomial evaluation of ThresholdSplit / RecoverSecret (herumi.go:137-223).
// Canonical [0, r) representation (r's top limb is too large for lazy tricks).
#pragma once
#include "hd.h"
#include "consts.h"

namespace hb {

constexpr int NLR = 8;

struct Fr {
  uint32_t v[NLR];
};

HD Fr fr_from_const(const uint32_t* c) {
  Fr r;
  HB_UNROLL for (int i = 0; i < NLR; i++) r.v[i] = c[i];
  return r;
}

HD Fr fr_zero() {
  Fr r;
  HB_UNROLL for (int i = 0; i < NLR; i++) r.v[i] = 0;
  return r;
}

HD Fr fr_one() { return fr_from_const(FR_ONE); }

HD uint32_t fr_raw_sub(Fr& r, const Fr& a, const uint32_t* b) {
  int64_t c = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    c += (int64_t)a.v[i] - (int64_t)b[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)(c & 1);
}

HD Fr fr_add(const Fr& a, const Fr& b) {
  Fr s;
  uint64_t c = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    c += (uint64_t)a.v[i] + b.v[i];
    s.v[i] = (uint32_t)c;
    c >>= 32;
  }
  Fr d;
  uint32_t borrow = fr_raw_sub(d, s, R_RAW);
  // s < 2r < 2^256 so no carry out; subtract r if s >= r
  return (borrow == 0) ? d : s;
}

HD Fr fr_sub(const Fr& a, const Fr& b) {
  Fr d;
  int64_t c = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    c += (int64_t)a.v[i] - (int64_t)b.v[i];
    d.v[i] = (uint32_t)c;
    c >>= 32;
  }
  if (c) {
    uint64_t cc = 0;
    HB_UNROLL for (int i = 0; i < NLR; i++) {
      cc += (uint64_t)d.v[i] + R_RAW[i];
      d.v[i] = (uint32_t)cc;
      cc >>= 32;
    }
  }
  return d;
}

// Montgomery product (CIOS with explicit top carry; r's top limb is ~0x73ed... > 2^31).
HDNI Fr fr_mul(const Fr& a, const Fr& b) {
  HB_COUNT_FR_MUL();
  uint32_t t[NLR + 2];
  HB_UNROLL for (int j = 0; j < NLR + 2; j++) t[j] = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    uint64_t C = 0;
    HB_UNROLL for (int j = 0; j < NLR; j++) {
      C = (uint64_t)a.v[j] * b.v[i] + t[j] + C;
      t[j] = (uint32_t)C;
      C >>= 32;
    }
    C += t[NLR];
    t[NLR] = (uint32_t)C;
    t[NLR + 1] = (uint32_t)(C >> 32);
    uint32_t m = t[0] * HB_R_N0;
    C = (uint64_t)m * R_RAW[0] + t[0];
    C >>= 32;
    HB_UNROLL for (int j = 1; j < NLR; j++) {
      C = (uint64_t)m * R_RAW[j] + t[j] + C;
      t[j - 1] = (uint32_t)C;
      C >>= 32;
    }
    C += t[NLR];
    t[NLR - 1] = (uint32_t)C;
    t[NLR] = t[NLR + 1] + (uint32_t)(C >> 32);
  }
  Fr r, d;
  HB_UNROLL for (int j = 0; j < NLR; j++) r.v[j] = t[j];
  uint32_t borrow = fr_raw_sub(d, r, R_RAW);
  return (t[NLR] != 0 || borrow == 0) ? d : r;
}

HD Fr fr_to_mont(const Fr& a) { return fr_mul(a, fr_from_const(FR_R2)); }

HD Fr fr_from_mont(const Fr& a) {
  Fr one = fr_zero();
  one.v[0] = 1;
  return fr_mul(a, one);
}

HD bool fr_is_zero(const Fr& a) {
  uint32_t acc = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) acc |= a.v[i];
  return acc == 0;
}

HD bool fr_eq(const Fr& a, const Fr& b) {
  uint32_t acc = 0;
  HB_UNROLL for (int i = 0; i < NLR; i++) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

HDNI Fr fr_inv(const Fr& a) {
  Fr r = fr_one();
  HB_NOUNROLL for (int i = 254; i >= 0; i--) {
    r = fr_mul(r, r);
    if ((EXP_R_MINUS_2[i >> 5] >> (i & 31)) & 1) r = fr_mul(r, a);
  }
  return r;
}

// int64 share index -> Fr (Montgomery); negative indices map to r - |idx|
// (mcl's ID.SetDecString of a negative decimal; SURVEY App. A, unpinned).
HD Fr fr_from_i64(int64_t idx) {
  uint64_t mag = idx < 0 ? (uint64_t)(-(idx + 1)) + 1 : (uint64_t)idx;
  Fr a = fr_zero();
  a.v[0] = (uint32_t)mag;
  a.v[1] = (uint32_t)(mag >> 32);
  Fr m = fr_to_mont(a);
  return idx < 0 ? fr_sub(fr_zero(), m) : m;
}

// 32-byte big-endian -> raw limbs; returns false if >= r
HD bool fr_from_be(Fr& r, const uint8_t* b) {
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  Fr d;
  return fr_raw_sub(d, r, R_RAW) != 0;
}

HD void fr_to_be(uint8_t* b, const Fr& a) {
  HB_UNROLL for (int i = 0; i < NLR; i++) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(a.v[i] >> 24);
    q[1] = (uint8_t)(a.v[i] >> 16);
    q[2] = (uint8_t)(a.v[i] >> 8);
    q[3] = (uint8_t)a.v[i];
  }
}

}  // namespace hb
