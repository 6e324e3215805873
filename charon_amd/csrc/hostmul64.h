// hostmul64.h: the host builds' Montgomery products with 64-bit words (the test harness and the
// CPU baseline, tests/native/hostcheck.cpp; never the device).  They return exactly what the
// 28-bit-limb cores of fp.h / ec28.h return -- the same lazily reduced representation, bit for
// bit -- because that result is a function of the operands' values alone: with T the product (or
// signed sum of products), the Montgomery quotient M = -T p^-1 mod 2^392 is unique in
// [0, 2^392), so V = (T + M p) / 2^392 does not depend on the digit size that computes it.  Here
// M is found as six 64-bit digits and one 8-bit digit (2^392 = 2^384 * 2^8).  The 28-bit cores
// take 392 32 x 32-bit multiply-adds per product; these take ~80 64 x 64-bit multiplies, which is
// what a CPU does well (tests/test_hostcheck.py test_host_mul64_matches_r28 checks the equality on
// random and lazy operands).
#pragma once
#if !defined(__HIP_DEVICE_COMPILE__)
#include <stdint.h>

#include "consts.h"

namespace hb {
namespace hm64 {

typedef unsigned __int128 u128;
constexpr int NW = 14;  // words of the working integer: products and sums below 2^800

constexpr uint64_t p64(int i) { return (uint64_t)P_RAW[2 * i] | ((uint64_t)P_RAW[2 * i + 1] << 32); }
constexpr uint64_t neg_inv64(uint64_t x) {  // -x^-1 mod 2^64 (x odd), Newton's iteration
  uint64_t y = x;
  for (int i = 0; i < 6; i++) y *= 2 - x * y;
  return (uint64_t)0 - y;
}
constexpr uint64_t kN64 = neg_inv64(p64(0));
constexpr uint64_t kN8 = kN64 & 0xff;  // -p^-1 mod 2^8

// the value of 12 stored words (6 words) / of 14 limbs of 28 bits, any limb below 2^32 (7 words)
inline void from_words(uint64_t* o, const uint32_t* w) {
  for (int i = 0; i < 6; i++) o[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  o[6] = 0;
}
inline void from_limbs28(uint64_t* o, const uint32_t* l) {
  for (int i = 0; i < 7; i++) o[i] = 0;
  for (int j = 0; j < 14; j++) {
    const int bit = 28 * j, i = bit >> 6, s = bit & 63;
    const u128 t = (u128)l[j] << s;
    u128 c = (u128)o[i] + (uint64_t)t;
    o[i] = (uint64_t)c;
    c = (c >> 64) + (uint64_t)(t >> 64);
    for (int k = i + 1; k < 7 && c; k++) {
      c += o[k];
      o[k] = (uint64_t)c;
      c >>= 64;
    }
  }
}

// t (NW words, two's complement) += or -= a * b (7-word operands)
inline void mac(uint64_t* t, const uint64_t* a, const uint64_t* b, bool sub) {
  uint64_t p[NW] = {};
  for (int i = 0; i < 7; i++) {
    if (!a[i]) continue;
    u128 c = 0;
    for (int j = 0; j < 7; j++) {
      c += (u128)a[i] * b[j] + p[i + j];
      p[i + j] = (uint64_t)c;
      c >>= 64;
    }
    for (int k = i + 7; k < NW && c; k++) {
      c += p[k];
      p[k] = (uint64_t)c;
      c >>= 64;
    }
  }
  if (sub) {
    unsigned __int128 bor = 0;
    for (int k = 0; k < NW; k++) {
      const u128 d = (u128)t[k] - p[k] - bor;
      t[k] = (uint64_t)d;
      bor = (d >> 64) ? 1 : 0;
    }
  } else {
    u128 c = 0;
    for (int k = 0; k < NW; k++) {
      c += (u128)t[k] + p[k];
      t[k] = (uint64_t)c;
      c >>= 64;
    }
  }
}

// t <- (t + M p) / 2^392 (two's complement, the result in t[0..7], sign-extended)
inline void redc392(uint64_t* t) {
  for (int d = 0; d < 6; d++) {
    const uint64_t m = t[d] * kN64;
    u128 c = 0;
    for (int k = 0; k < 6; k++) {
      c += (u128)m * p64(k) + t[d + k];
      t[d + k] = (uint64_t)c;
      c >>= 64;
    }
    for (int k = d + 6; k < NW; k++) {
      c += t[k];
      t[k] = (uint64_t)c;
      c >>= 64;
    }
  }
  const uint64_t m8 = (t[6] * kN8) & 0xff;
  u128 c = 0;
  for (int k = 0; k < 6; k++) {
    c += (u128)m8 * p64(k) + t[6 + k];
    t[6 + k] = (uint64_t)c;
    c >>= 64;
  }
  for (int k = 12; k < NW; k++) {
    c += t[k];
    t[k] = (uint64_t)c;
    c >>= 64;
  }
  for (int k = 0; k < 8; k++) t[k] = (t[6 + k] >> 8) | (k + 7 < NW ? t[7 + k] << 56 : (uint64_t)((int64_t)t[NW - 1] >> 63) << 56);
}

// V -> 12 stored words (V mod 2^384), plus p when `neg` (fp.h fp2_fix_neg)
inline void to_words(uint32_t* w, const uint64_t* v, bool add_p) {
  uint64_t x[6];
  u128 c = 0;
  for (int i = 0; i < 6; i++) {
    c += (u128)v[i] + (add_p ? p64(i) : 0);
    x[i] = (uint64_t)c;
    c >>= 64;
  }
  for (int i = 0; i < 6; i++) {
    w[2 * i] = (uint32_t)x[i];
    w[2 * i + 1] = (uint32_t)(x[i] >> 32);
  }
}
// V -> 14 limbs: 28-bit digits 0..12, limb 13 = the low 32 bits of V >> 364
inline void to_limbs28(uint32_t* l, const uint64_t* v) {
  for (int j = 0; j < 14; j++) {
    const int bit = 28 * j, i = bit >> 6, s = bit & 63;
    uint64_t x = v[i] >> s;
    if (s && i + 1 < 8) x |= v[i + 1] << (64 - s);
    l[j] = j < 13 ? (uint32_t)(x & 0x0FFFFFFFu) : (uint32_t)x;
  }
}

inline void mul_words(uint32_t* out, const uint32_t* aw, const uint32_t* bw) {
  uint64_t a[7], b[7], t[NW] = {};
  from_words(a, aw);
  from_words(b, bw);
  mac(t, a, b, false);
  redc392(t);
  to_words(out, t, false);
}
inline void fp2_mul_words(uint32_t* o0, uint32_t* o1, const uint32_t* a0w, const uint32_t* a1w, const uint32_t* b0w,
                          const uint32_t* b1w) {
  uint64_t a0[7], a1[7], b0[7], b1[7], t0[NW] = {}, t1[NW] = {};
  from_words(a0, a0w);
  from_words(a1, a1w);
  from_words(b0, b0w);
  from_words(b1, b1w);
  mac(t0, a0, b0, false);
  mac(t0, a1, b1, true);
  mac(t1, a0, b1, false);
  mac(t1, a1, b0, false);
  redc392(t0);
  redc392(t1);
  to_words(o0, t0, (int64_t)t0[7] < 0);
  to_words(o1, t1, false);
}
inline void mul_limbs28(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint64_t x[7], y[7], t[NW] = {};
  from_limbs28(x, a);
  from_limbs28(y, b);
  mac(t, x, y, false);
  redc392(t);
  to_limbs28(r, t);
}
inline void dot_limbs28(uint32_t* r, const uint32_t* a0, const uint32_t* a1, const uint32_t* b0, const uint32_t* b1) {
  uint64_t x0[7], x1[7], y0[7], y1[7], t[NW] = {};
  from_limbs28(x0, a0);
  from_limbs28(x1, a1);
  from_limbs28(y0, b0);
  from_limbs28(y1, b1);
  mac(t, x0, y0, false);
  mac(t, x1, y1, false);
  redc392(t);
  to_limbs28(r, t);
}

}  // namespace hm64
}  // namespace hb
#endif
