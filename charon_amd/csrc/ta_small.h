// Small-scalar form of a ThresholdAggregate's Lagrange coefficients (tbls.ThresholdAggregate,
// herumi.go:249-286: sigma = sum_j lambda_j(0) sigma_j over the share indices x_j).
//
// With P = prod_m x_m, E_j = x_j prod_{m != j} (x_m - x_j) and L = lcm_j |E_j|:
//     lambda_j = prod_{m != j} x_m / (x_m - x_j) = P / E_j = s c_j,
//     c_j = L / E_j  (a signed integer dividing L),   s = P / L mod r,
// so  sigma = [s] (sum_j [c_j] sigma_j).  Charon's share indices are small (1..n, n the number of
// operators), so the c_j are small integers -- for any t-subset of 1..10 every |c_j| divides
// lcm(1..10) * 9! and is below 2^22 -- and the aggregation is ONE joint ladder of ~22 bits over
// the t members plus ONE 255-bit multiplication (4-dimensional via psi) per validator, instead
// of a 255-bit multiplication per member.  The result is the same group element, hence the same
// 96-byte aggregate.  The split is refused (the general path runs) for t outside 2..TA_SMALL_MAX,
// index 0, duplicated indices (herumi's combine failure), indices of 2^31 or more in magnitude, or
// any intermediate beyond 63 bits.
#pragma once
#include "fr.h"

namespace hb {

constexpr int TA_SMALL_MAX = 16;  // members per group of the small-scalar path

HD int64_t ta_gcd(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// c[0..t) and s (Montgomery form) as above; false when the split does not apply.
HD bool ta_small_split(const int64_t* x, int t, int64_t* c, Fr& s) {
  if (t < 2 || t > TA_SMALL_MAX) return false;
  const int64_t lim = (int64_t)1 << 31;
  for (int j = 0; j < t; j++)
    if (x[j] == 0 || x[j] <= -lim || x[j] >= lim) return false;
  int64_t L = 1;
  for (int j = 0; j < t; j++) {
    int64_t e = x[j];
    for (int m = 0; m < t; m++) {
      if (m == j) continue;
      const int64_t d = x[m] - x[j];  // |d| < 2^32
      if (d == 0) return false;
      if (__builtin_mul_overflow(e, d, &e)) return false;
    }
    // E_j = -2^63 passes the overflow checks (e.g. x_j = -2^30 among {2^30, -2^30 + 1, -2^30 + 4}),
    // but its magnitude does not fit: refuse it (the general path aggregates the group)
    if (e == INT64_MIN) return false;
    c[j] = e;  // E_j for now
    const int64_t ae = e < 0 ? -e : e;
    const int64_t g = ta_gcd(L, ae);
    int64_t l2;
    if (__builtin_mul_overflow(L / g, ae, &l2)) return false;
    L = l2;
  }
  Fr p = fr_one();
  for (int j = 0; j < t; j++) {
    c[j] = L / c[j];  // exact: E_j divides L
    p = fr_mul(p, fr_from_i64(x[j]));
  }
  s = fr_mul(p, fr_inv(fr_from_i64(L)));
  return true;
}

}  // namespace hb
