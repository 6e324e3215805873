// threshold.hip: staged ThresholdAggregate / Aggregate kernels of libhipbls.so
// (tbls.ThresholdAggregate -> Herumi.ThresholdAggregate, herumi.go:249-286; tbls.Aggregate,
// herumi.go:225-247).  Compiled like pipeline.hip (HB_FAST_FPMUL: everything but the Fp
// product inlined).
//
//   k_dec_sig_pt (vbatch.hip) 1 lane / partial: decompress + subgroup-check sigma_j (or, in the
//              slot entry point, the verification's decompressed points through src[])
//   k_ta_lambda 1 lane / partial: lambda_j(0) over its group's share indices (Fr, 1/d table for
//              the denominators), and the base-|x| digits of lambda_j
//   k_ta_straus 1 lane / partial: lambda_j sigma_j = sum_i [a_i] (-1)^i psi^i(sigma_j), one
//              joint 64-step ladder over the four digits (15-entry subset table)
//   k_group_sum (hipbls.hip) 1 lane / group: sum, affine, compress
//
// The split of lambda uses the G2 endomorphism psi, which acts on G2 as multiplication by the
// curve parameter x (this is the subgroup test of ec.h, psi(Q) == [x]Q).  With z = |x| = -x and
// lambda = a0 + a1 z + a2 z^2 + a3 z^3 (0 <= a_i < z; lambda < r < z^4):
//   [lambda] Q = [a0] Q - [a1] psi(Q) + [a2] psi^2(Q) - [a3] psi^3(Q),
// a 4-scalar multiplication with 64-bit scalars instead of one 255-bit one.  The result is the
// same group element, so the 96-byte output is byte-identical to herumi's Sign.Recover.
#define HB_FAST_FPMUL 1
#include "layout.h"
#include "ta_small.h"
#include <type_traits>

namespace hb {

static inline unsigned blocks_of(size_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

// u (8 little-endian limbs, < 2^256) <- u / z, returns u mod z   (z = |x|, bit-serial: the three
// divisions per partial cost a few Fp products)
__device__ __forceinline__ uint64_t divmod_xabs(uint32_t* u) {
  uint64_t r = 0;
  HB_UNROLL for (int li = NLR - 1; li >= 0; li--) {
    uint32_t word = u[li], qw = 0;
    HB_NOUNROLL for (int bit = 31; bit >= 0; bit--) {
      uint64_t nr = (r << 1) | ((word >> bit) & 1u);
      bool ge = (r >> 63) != 0 || nr >= HB_X_ABS;
      r = ge ? nr - HB_X_ABS : nr;
      qw = (qw << 1) | (ge ? 1u : 0u);
    }
    u[li] = qw;
  }
  return r;
}

__device__ __forceinline__ uint32_t find_group_ta(const uint32_t* grp_off, uint32_t n_groups, uint32_t j) {
  uint32_t lo = 0, hi = n_groups;  // invariant: grp_off[lo] <= j < grp_off[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (grp_off[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One lane per partial: lambda_j(0) over its group's share indices (Fr) and its base-|x|
// digits.  mode 0: ThresholdAggregate, mode 1: Aggregate (lambda = 1).  A combine failure (an
// index 0 mod r, or duplicated) is flagged unless the partial is already undecodable.
__global__ __launch_bounds__(64) void k_ta_lambda(const int64_t* __restrict__ idx, const uint32_t* __restrict__ grp_off,
                                                  uint32_t n_groups, uint32_t n_partials, int mode,
                                                  TaDigits* __restrict__ dig, uint8_t* __restrict__ mstat,
                                                  uint32_t t_u, uint8_t* __restrict__ nonuni,
                                                  const uint8_t* __restrict__ skip) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_partials) return;
  TaDigits d;
  d.a[0] = 1;
  d.a[1] = d.a[2] = d.a[3] = 0;
  uint32_t g = find_group_ta(grp_off, n_groups, j);
  uint32_t b = grp_off[g], en = grp_off[g + 1];
  if (nonuni && t_u && (en - b != t_u || b != g * t_u)) *nonuni = 1;
  if (skip && skip[g]) return;  // aggregated by the small-scalar path: no digits needed
  if (mode == 0 && en - b > 1) {  // k = 1: the single partial is returned as is
    // lambda_j = prod_m x_m / prod_m (x_m - x_j).  Share indices are small integers, so each
    // denominator factor normally comes from the 1/d table (no Fr inversion); anything else
    // (large or duplicated indices) goes through one Fermat inversion of their product.
    const int64_t ij = idx[j];
    const bool ij_small = ij > -(int64_t(1) << 62) && ij < (int64_t(1) << 62);
    Fr num = fr_one(), den_inv = fr_one(), den = fr_one();
    bool slow = false;
    for (uint32_t m = b; m < en; m++) {
      if (m == j) continue;
      const int64_t im = idx[m];
      num = fr_mul(num, fr_from_i64(im));
      const int64_t dd = im - ij;  // only used when both indices are below 2^62 in magnitude
      const bool small = ij_small && im > -(int64_t(1) << 62) && im < (int64_t(1) << 62) && dd != 0 &&
                         dd >= -FR_SMALL_INV_N && dd <= FR_SMALL_INV_N;
      if (small) {
        Fr t = fr_from_const(FR_SMALL_INV[(dd < 0 ? -dd : dd) - 1]);
        den_inv = fr_mul(den_inv, dd < 0 ? fr_sub(fr_zero(), t) : t);
      } else {
        den = fr_mul(den, fr_sub(fr_from_i64(im), fr_from_i64(ij)));
        slow = true;
      }
    }
    if (fr_is_zero(num) || fr_is_zero(den)) {
      if (mstat[j] == M_OK) mstat[j] = M_BAD_IDX;
    } else {
      if (slow) den_inv = fr_mul(den_inv, fr_inv(den));
      Fr lam = fr_from_mont(fr_mul(num, den_inv));
      uint32_t u[NLR];
      HB_UNROLL for (int i = 0; i < NLR; i++) u[i] = lam.v[i];
      d.a[0] = divmod_xabs(u);
      d.a[1] = divmod_xabs(u);
      d.a[2] = divmod_xabs(u);
      d.a[3] = ((uint64_t)u[1] << 32) | u[0];
    }
  }
  dig[j] = d;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Per-lane subset table, lane-interleaved so that one 16-byte load per (entry, quad) coalesces
// over the lanes that picked the same entry: uint4 index ((wave * 15 + e) * 18 + q) * 64 + lane.
constexpr int TA_TAB_QUADS = (int)(sizeof(G2JEntry) / 16);  // 18
__device__ __forceinline__ void tab_store(uint4* wt, int e, const G2J& p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&p);
  static_assert(sizeof(G2J) == sizeof(G2JEntry), "G2J layout");
  HB_UNROLL for (int q = 0; q < TA_TAB_QUADS; q++)
    wt[(e * TA_TAB_QUADS + q) * 64] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
__device__ __forceinline__ G2J tab_load(const uint4* wt, int e) {
  G2J p;
  uint32_t* w = reinterpret_cast<uint32_t*>(&p);
  HB_UNROLL for (int q = 0; q < TA_TAB_QUADS; q++) {
    uint4 v = wt[(e * TA_TAB_QUADS + q) * 64];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  return p;
}
__device__ __forceinline__ void f2_select(Fp2& r, bool take_b, const Fp2& a, const Fp2& b) {
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.c0.v[i] = take_b ? b.c0.v[i] : a.c0.v[i];
    r.c1.v[i] = take_b ? b.c1.v[i] : a.c1.v[i];
  }
}
// Fp2 values (6 quads) at quad offset q0 of entry e; affine points (x, y: 12 quads) at entry e
__device__ __forceinline__ void f2_store_q(uint4* wt, int e, int q0, const Fp2& a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  HB_UNROLL for (int q = 0; q < 6; q++)
    wt[(e * TA_TAB_QUADS + q0 + q) * 64] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
__device__ __forceinline__ Fp2 f2_load_q(const uint4* wt, int e, int q0) {
  Fp2 a;
  uint32_t* w = reinterpret_cast<uint32_t*>(&a);
  HB_UNROLL for (int q = 0; q < 6; q++) {
    const uint4 v = wt[(e * TA_TAB_QUADS + q0 + q) * 64];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  return a;
}
__device__ __forceinline__ void aff_store(uint4* wt, int e, const Fp2& x, const Fp2& y) {
  f2_store_q(wt, e, 0, x);
  f2_store_q(wt, e, 6, y);
}
#endif

// One lane per partial: lambda sigma = sum_i [a_i] P_i with P_i = (-1)^i psi^i(sigma), as a
// 4-scalar Straus ladder over the 15-entry subset table T[s] = sum_{i in s} P_i (built with 11
// mixed additions, kept in global memory): 64 doublings + 64 table additions per partial, against
// 4 x 64 of each for four independent ladders.  Uniform control flow: the table addition of
// every step is computed and kept or dropped per lane by select.
__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_straus(const HmEntry* __restrict__ pts, const uint32_t* __restrict__ src,
                                                     const TaDigits* __restrict__ dig,
                                                     uint32_t n_partials, uint32_t n_groups, uint32_t t_uniform,
                                                     uint4* __restrict__ tab, G2JEntry* __restrict__ out,
                                                     const uint8_t* __restrict__ skip, const uint8_t* __restrict__ guard) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ int8_t naf[4][66];
  __shared__ int naf_top;
  if (guard && *guard == 0) return;
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t item = blockIdx.x * 64 + (uint32_t)lane;
  const uint32_t it = item < n_partials ? item : n_partials - 1;
  // member of this lane: with t members in every group, lane L takes member j = L / n_groups of
  // validator v = L % n_groups, so a wave holds the same share position of 64 validators -- whose
  // Lagrange digits agree whenever the validators' index sets do (the common slot)
  const uint32_t m = t_uniform ? (it % n_groups) * t_uniform + it / n_groups : it;
  // skip (nullable, t_uniform only): groups the small-scalar path aggregated
  const bool valid = item < n_partials && !(skip && t_uniform && skip[m / t_uniform]);
  if (!__any(valid)) return;
  uint4* wt = tab + (size_t)blockIdx.x * 16 * TA_TAB_QUADS * 64 + lane;
  // skipped lanes' digits are never computed (k_ta_lambda skips their groups): they read a
  // neutral value and stay out of the uniformity test, which runs over the valid lanes only
  TaDigits d;
  if (valid) {
    d = dig[m];
  } else {
    d.a[0] = 1;
    d.a[1] = d.a[2] = d.a[3] = 0;
  }
  bool same = true;
  if (valid) {
    HB_UNROLL for (int k = 0; k < 4; k++) {
      const uint32_t lo = (uint32_t)d.a[k], hi = (uint32_t)(d.a[k] >> 32);
      same = same && lo == (uint32_t)__builtin_amdgcn_readfirstlane((int)lo) &&
             hi == (uint32_t)__builtin_amdgcn_readfirstlane((int)hi);
    }
  }
  const HmEntry e = pts[src ? src[m] : m];
  const G2A P0 = {e.x, e.y, e.inf != 0};
  G2J R = jac_infinity<Fp2>();
  if (__all(same)) {
    // wave-uniform digits: signed width-4 NAF of each digit (one shared schedule, uniform
    // branches) over the odd multiples {1, 3, 5, 7} of the four bases B_k = P0, -psi(P0),
    // psi^2(P0), -psi^3(P0): ~13 additions per 64-bit digit instead of one per ladder step.
    // The schedule comes from the first valid lane.
    const int fl = __ffsll((unsigned long long)__ballot(valid)) - 1;
    uint64_t da[4];
    HB_UNROLL for (int k = 0; k < 4; k++) {
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)d.a[k], fl);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(d.a[k] >> 32), fl);
      da[k] = ((uint64_t)hi << 32) | lo;
    }
    if (lane == 0) {
      int top = 0;
      HB_UNROLL for (int k = 0; k < 4; k++) {
        uint64_t v = da[k];  // < |x| < 2^64 - 7: v + 7 cannot overflow
        for (int i = 0; i < 66; i++) {
          int dg = 0;
          if (v & 1u) {
            dg = (int)(v & 15u);
            if (dg >= 8) dg -= 16;
            v = dg > 0 ? v - (uint64_t)dg : v + (uint64_t)(-dg);
          }
          naf[k][i] = (int8_t)dg;
          if (dg && i > top) top = i;
          v >>= 1;
        }
      }
      naf_top = top;
    }
    __syncthreads();
    const G2J J1 = jac_from_aff(P0);
    const G2J J2 = jac_dbl(J1);
    const G2J J3 = jac_add_aff(J2, P0);
    const G2J J5 = jac_add(J3, J2);
    const G2J J7 = jac_add(J5, J2);
    const Fp2 cx = f2_from_const(PSI_CX), cy = f2_from_const(PSI_CY);
    const Fp2 c2x = f2_from_const(PSI2_CX), c2y = f2_from_const(PSI2_CY);
    HB_NOUNROLL for (int j = 0; j < 4; j++) {
      const G2J J = j == 0 ? J1 : j == 1 ? J3 : j == 2 ? J5 : J7;
      tab_store(wt, j, J);
      // -psi: (conj(X) cx, -conj(Y) cy, conj(Z));  psi^2: (X c2x, Y c2y, Z)
      const G2J N1 = {f2_mul(f2_conj(J.X), cx), f2_neg(f2_mul(f2_conj(J.Y), cy)), f2_conj(J.Z)};
      const G2J N2 = {f2_mul(J.X, c2x), f2_mul(J.Y, c2y), J.Z};
      const G2J N3 = {f2_mul(f2_conj(N2.X), cx), f2_neg(f2_mul(f2_conj(N2.Y), cy)), f2_conj(N2.Z)};
      tab_store(wt, 4 + j, N1);
      tab_store(wt, 8 + j, N2);
      tab_store(wt, 12 + j, N3);
    }
    const int top = naf_top;
    HB_NOUNROLL for (int i = top; i >= 0; i--) {
      R = jac_dbl(R);
      HB_NOUNROLL for (int k = 0; k < 4; k++) {
        const int dg = naf[k][i];
        if (dg != 0) {  // wave-uniform
          G2J T = tab_load(wt, 4 * k + ((dg < 0 ? -dg : dg) >> 1));
          if (dg < 0) T.Y = f2_neg(T.Y);
          R = jac_add(R, T);
        }
      }
    }
  } else {
    // general case: one joint 64-step ladder over the 15-entry subset table of the four bases
    {
      G2A P1 = {f2_mul(f2_conj(e.x), f2_from_const(PSI_CX)), f2_neg(f2_mul(f2_conj(e.y), f2_from_const(PSI_CY))),
                P0.inf};
      G2A P2 = {f2_mul(e.x, f2_from_const(PSI2_CX)), f2_mul(e.y, f2_from_const(PSI2_CY)), P0.inf};
      G2A P3 = {f2_mul(f2_conj(P2.x), f2_from_const(PSI_CX)), f2_neg(f2_mul(f2_conj(P2.y), f2_from_const(PSI_CY))),
                P0.inf};
      tab_store(wt, 0, jac_from_aff(P0));
      tab_store(wt, 1, jac_from_aff(P1));
      tab_store(wt, 3, jac_from_aff(P2));
      tab_store(wt, 7, jac_from_aff(P3));
    }
    // T[s] (entry s - 1) = T[s - hi] + T[hi], hi the top bit of s; T[hi] is affine (Z = 1 or infinity)
    HB_NOUNROLL for (int sidx = 3; sidx < 16; sidx++) {
      const int hi = sidx >= 8 ? 8 : (sidx >= 4 ? 4 : 2);
      if (sidx == hi) continue;
      const G2J h = tab_load(wt, hi - 1);
      const G2A ha = {h.X, h.Y, f2_is_zero(h.Z)};
      tab_store(wt, sidx - 1, jac_add_aff(tab_load(wt, sidx - hi - 1), ha));
    }
    HB_NOUNROLL for (int b = 63; b >= 0; b--) {
      R = jac_dbl(R);
      const uint32_t sel = (uint32_t)((d.a[0] >> b) & 1) | ((uint32_t)((d.a[1] >> b) & 1) << 1) |
                           ((uint32_t)((d.a[2] >> b) & 1) << 2) | ((uint32_t)((d.a[3] >> b) & 1) << 3);
      const G2J S = jac_add(R, tab_load(wt, sel == 0 ? 0 : (int)sel - 1));
      f2_select(R.X, sel != 0, R.X, S.X);
      f2_select(R.Y, sel != 0, R.Y, S.Y);
      f2_select(R.Z, sel != 0, R.Z, S.Z);
    }
  }
  if (valid) out[m] = {R.X, R.Y, R.Z};
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
// Affine odd-multiple tables of the `cnt` members of a joint lane (k_ta_jtab): member k's entries
// 16 k + 4 b + (|d| >> 1) hold the affine odd multiples {1, 3, 5, 7} of the bases B_b = P0, -psi(P0),
// psi^2(P0), -psi^3(P0), so the ladder adds them with mixed additions (7M + 4S instead of 11M + 5S
// over Fp2).  3P0, 5P0, 7P0 of all members are made affine with ONE inversion (Montgomery's trick):
// pass 1 keeps them Jacobian in entries 16 k + 1..3 and the running product of their Z before each
// in entries 16 k + 5..7; pass 2 walks back, recovering every 1 / Z.  A member at infinity (an
// undecodable partial: the validator's aggregate is discarded) multiplies Z = 1 into the product.
__device__ __forceinline__ void odd_tables_affine(uint4* wt, const HmEntry* __restrict__ pts,
                                                  const uint32_t* __restrict__ src, uint32_t m0, uint32_t cnt) {
  Fp2 acc = f2_one();
  HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
    const HmEntry e = pts[src ? src[m0 + k] : m0 + k];
    const G2A P0 = {e.x, e.y, e.inf != 0};
    const G2J J1 = jac_from_aff(P0);
    const G2J J2 = jac_dbl(J1);
    const G2J J3 = jac_add_aff(J2, P0);
    const G2J J5 = jac_add(J3, J2);
    const G2J J7 = jac_add(J5, J2);
    HB_NOUNROLL for (int j = 1; j < 4; j++) {
      G2J J = j == 1 ? J3 : j == 2 ? J5 : J7;
      if (f2_is_zero(J.Z)) J.Z = f2_one();
      tab_store(wt, 16 * (int)k + j, J);
      f2_store_q(wt, 16 * (int)k + 4 + j, 0, acc);
      acc = f2_mul(acc, J.Z);
    }
    aff_store(wt, 16 * (int)k, P0.x, P0.y);
  }
  Fp2 inv = f2_inv(acc);
  const Fp2 cx = f2_from_const(PSI_CX), cy = f2_from_const(PSI_CY);
  const Fp2 c2x = f2_from_const(PSI2_CX), c2y = f2_from_const(PSI2_CY);
  HB_NOUNROLL for (int k = (int)cnt - 1; k >= 0; k--) {
    HB_NOUNROLL for (int j = 3; j >= 0; j--) {
      const int e = 16 * k + j;
      Fp2 x, y;
      if (j == 0) {
        x = f2_load_q(wt, e, 0);
        y = f2_load_q(wt, e, 6);
      } else {
        const G2J J = tab_load(wt, e);
        const Fp2 zi = f2_mul(inv, f2_load_q(wt, 16 * k + 4 + j, 0));  // 1 / Z
        inv = f2_mul(inv, J.Z);
        const Fp2 zi2 = f2_sqr(zi);
        x = f2_mul(J.X, zi2);
        y = f2_mul(J.Y, f2_mul(zi2, zi));
        aff_store(wt, e, x, y);
      }
      // -psi: (conj(x) cx, -conj(y) cy);  psi^2: (x c2x, y c2y);  -psi^3 = -psi(psi^2)
      const Fp2 x2 = f2_mul(x, c2x), y2 = f2_mul(y, c2y);
      aff_store(wt, e + 4, f2_mul(f2_conj(x), cx), f2_neg(f2_mul(f2_conj(y), cy)));
      aff_store(wt, e + 8, x2, y2);
      aff_store(wt, e + 12, f2_mul(f2_conj(x2), cx), f2_neg(f2_mul(f2_conj(y2), cy)));
    }
  }
}

// signed width-4 NAF of a 64-bit digit (< |x| < 2^64 - 7, so v + 7 cannot overflow) into out[66];
// returns the top nonzero position (0 if none)
__device__ __forceinline__ int naf4_digits(uint64_t v, int8_t* out) {
  int top = 0;
  for (int i = 0; i < 66; i++) {
    int dg = 0;
    if (v & 1u) {
      dg = (int)(v & 15u);
      if (dg >= 8) dg -= 16;
      v = dg > 0 ? v - (uint64_t)dg : v + (uint64_t)(-dg);
    }
    out[i] = (int8_t)dg;
    if (dg && i > top) top = i;
    v >>= 1;
  }
  return top;
}

// lambda sigma for one member with arbitrary digits: the joint 64-step ladder over its 15-entry
// subset table (entries e0 .. e0 + 14)
__device__ __forceinline__ G2J member_general(uint4* wt, int e0, const HmEntry& e, const TaDigits& d) {
  const G2A P0 = {e.x, e.y, e.inf != 0};
  {
    G2A P1 = {f2_mul(f2_conj(e.x), f2_from_const(PSI_CX)), f2_neg(f2_mul(f2_conj(e.y), f2_from_const(PSI_CY))),
              P0.inf};
    G2A P2 = {f2_mul(e.x, f2_from_const(PSI2_CX)), f2_mul(e.y, f2_from_const(PSI2_CY)), P0.inf};
    G2A P3 = {f2_mul(f2_conj(P2.x), f2_from_const(PSI_CX)), f2_neg(f2_mul(f2_conj(P2.y), f2_from_const(PSI_CY))),
              P0.inf};
    tab_store(wt, e0 + 0, jac_from_aff(P0));
    tab_store(wt, e0 + 1, jac_from_aff(P1));
    tab_store(wt, e0 + 3, jac_from_aff(P2));
    tab_store(wt, e0 + 7, jac_from_aff(P3));
  }
  HB_NOUNROLL for (int sidx = 3; sidx < 16; sidx++) {
    const int hi = sidx >= 8 ? 8 : (sidx >= 4 ? 4 : 2);
    if (sidx == hi) continue;
    const G2J h = tab_load(wt, e0 + hi - 1);
    const G2A ha = {h.X, h.Y, f2_is_zero(h.Z)};
    tab_store(wt, e0 + sidx - 1, jac_add_aff(tab_load(wt, e0 + sidx - hi - 1), ha));
  }
  G2J R = jac_infinity<Fp2>();
  HB_NOUNROLL for (int b = 63; b >= 0; b--) {
    R = jac_dbl(R);
    const uint32_t sel = (uint32_t)((d.a[0] >> b) & 1) | ((uint32_t)((d.a[1] >> b) & 1) << 1) |
                         ((uint32_t)((d.a[2] >> b) & 1) << 2) | ((uint32_t)((d.a[3] >> b) & 1) << 3);
    const G2J S = jac_add(R, tab_load(wt, e0 + (sel == 0 ? 0 : (int)sel - 1)));
    f2_select(R.X, sel != 0, R.X, S.X);
    f2_select(R.Y, sel != 0, R.Y, S.Y);
    f2_select(R.Z, sel != 0, R.Z, S.Z);
  }
  return R;
}
#endif

// Joint aggregation ladders: one lane per CHUNK of c members of one validator (the validator's t
// members in ceil(t / c) chunks), lane L taking chunk q = L / n_groups of validator v = L % n_groups
// so that a wave holds the same members of 64 validators.  When their Lagrange digits agree
// across the wave (every validator aggregates the same share indices -- the common slot), ONE
// signed width-4 NAF schedule runs over all c members' odd-multiple tables: top + 1 doublings for
// the chunk instead of per member, one addition per nonzero digit as before.  Otherwise each member
// takes the general 15-entry ladder.  The chunk's sum goes to its first member's slot of `out`,
// infinity to the others (k_group_sum adds a group's t slots).
constexpr int TA_JOINT_MAX = 8;
// Three kernels over the same lanes, so that each holds only its own working set (one kernel with
// both ladders and the table build spilled 2.9 KB per lane): k_ta_jtab builds the affine tables,
// k_ta_jladder runs the shared NAF schedule, k_ta_jgeneral the per-member ladders; the last two
// return at once on the waves that are not theirs (the uniformity test is repeated in each).
#if defined(__HIP_DEVICE_COMPILE__)
struct JointLane {
  uint32_t L, cnt, m0;
  bool valid, uniform, any;
  uint4* wt;
};
// skip (nullable): groups already aggregated by the small-scalar path (k_ta_small); their lanes
// neither compute for the uniformity test's sake nor store.  nonuni (nullable): the groups are not
// all of t members (k_ta_lambda): no lane is valid (the per-member ladders run instead)
__device__ __forceinline__ JointLane joint_lane(const TaDigits* __restrict__ dig, uint32_t n_groups, uint32_t t,
                                                uint32_t c, uint4* __restrict__ tab, const uint8_t* __restrict__ skip,
                                                const uint8_t* __restrict__ nonuni) {
  JointLane j;
  if (nonuni && *nonuni) {
    j.valid = j.uniform = j.any = false;
    j.L = j.cnt = j.m0 = 0;
    j.wt = tab;
    return j;
  }
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t n_chunks = (t + c - 1) / c, n_lanes = n_groups * n_chunks;
  j.L = blockIdx.x * 64 + (uint32_t)lane;
  j.valid = j.L < n_lanes && !(skip && skip[j.L % n_groups]);
  const uint32_t Lc = j.valid ? j.L : n_lanes - 1;
  const uint32_t q = Lc / n_groups, v = Lc % n_groups;
  const uint32_t j0 = q * c;
  j.cnt = min(c, t - j0);
  j.m0 = v * t + j0;
  j.wt = tab + (size_t)blockIdx.x * (16 * c) * TA_TAB_QUADS * 64 + lane;
  // the uniformity test runs over the valid lanes only (readfirstlane inside the branch reads the
  // first valid lane): skipped groups' digits are never computed (k_ta_lambda skips them)
  bool same = true;
  if (j.valid) {
    same = j.cnt == (uint32_t)__builtin_amdgcn_readfirstlane((int)j.cnt);
    HB_NOUNROLL for (uint32_t k = 0; k < c; k++) {
      const TaDigits d = dig[j.m0 + (k < j.cnt ? k : 0)];
      HB_UNROLL for (int i = 0; i < 4; i++) {
        const uint32_t lo = (uint32_t)d.a[i], hi = (uint32_t)(d.a[i] >> 32);
        same = same && lo == (uint32_t)__builtin_amdgcn_readfirstlane((int)lo) &&
               hi == (uint32_t)__builtin_amdgcn_readfirstlane((int)hi);
      }
    }
  }
  j.uniform = __all(same);
  j.any = __any(j.valid);
  return j;
}
// the first valid lane of the wave (j.any): its members' digits are the wave's schedule
__device__ __forceinline__ int joint_first_lane(const JointLane& j) {
  return __ffsll((unsigned long long)__ballot(j.valid)) - 1;
}
__device__ __forceinline__ void joint_store(G2JEntry* __restrict__ out, const JointLane& j, const G2J& R) {
  if (!j.valid) return;
  out[j.m0] = {R.X, R.Y, R.Z};
  const G2J z = jac_infinity<Fp2>();
  for (uint32_t k = 1; k < j.cnt; k++) out[j.m0 + k] = {z.X, z.Y, z.Z};
}
#endif

__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_jtab(const HmEntry* __restrict__ pts, const uint32_t* __restrict__ src,
                                                   const TaDigits* __restrict__ dig, uint32_t n_groups, uint32_t t,
                                                   uint32_t c, uint4* __restrict__ tab, const uint8_t* __restrict__ skip,
                                                   const uint8_t* __restrict__ nonuni) {
#if defined(__HIP_DEVICE_COMPILE__)
  const JointLane j = joint_lane(dig, n_groups, t, c, tab, skip, nonuni);
  if (j.any && j.uniform) odd_tables_affine(j.wt, pts, src, j.m0, j.cnt);
#endif
}

__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_jladder(const TaDigits* __restrict__ dig, uint32_t n_groups, uint32_t t,
                                                      uint32_t c, uint4* __restrict__ tab, G2JEntry* __restrict__ out,
                                                      const uint8_t* __restrict__ skip, const uint8_t* __restrict__ nonuni) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ int8_t naf[TA_JOINT_MAX][4][66];
  __shared__ int naf_top;
  const JointLane j = joint_lane(dig, n_groups, t, c, tab, skip, nonuni);
  if (!j.any || !j.uniform) return;  // wave-uniform
  const int fl = joint_first_lane(j);
  const uint32_t m0f = (uint32_t)__shfl((int)j.m0, fl), cntf = (uint32_t)__shfl((int)j.cnt, fl);
  if ((threadIdx.x & 63u) == 0) {
    int top = 0;
    for (uint32_t k = 0; k < cntf; k++) {
      const TaDigits d = dig[m0f + k];
      for (int i = 0; i < 4; i++) top = max(top, naf4_digits(d.a[i], naf[k][i]));
    }
    naf_top = top;
  }
  __syncthreads();
  G2J R = jac_infinity<Fp2>();
  const int top = naf_top;
  HB_NOUNROLL for (int i = top; i >= 0; i--) {
    R = jac_dbl(R);
    HB_NOUNROLL for (uint32_t k = 0; k < cntf; k++) {
      HB_NOUNROLL for (int b = 0; b < 4; b++) {
        const int dg = naf[k][b][i];
        if (dg != 0) {  // wave-uniform
          const int e = 16 * (int)k + 4 * b + ((dg < 0 ? -dg : dg) >> 1);
          G2A T = {f2_load_q(j.wt, e, 0), f2_load_q(j.wt, e, 6), false};
          if (dg < 0) T.y = f2_neg(T.y);
          R = jac_add_aff(R, T);
        }
      }
    }
  }
  joint_store(out, j, R);
#endif
}

__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_jgeneral(const HmEntry* __restrict__ pts, const uint32_t* __restrict__ src,
                                                       const TaDigits* __restrict__ dig, uint32_t n_groups, uint32_t t,
                                                       uint32_t c, uint4* __restrict__ tab, G2JEntry* __restrict__ out,
                                                       const uint8_t* __restrict__ skip, const uint8_t* __restrict__ nonuni) {
#if defined(__HIP_DEVICE_COMPILE__)
  const JointLane j = joint_lane(dig, n_groups, t, c, tab, skip, nonuni);
  if (!j.any || j.uniform) return;  // wave-uniform
  G2J R = jac_infinity<Fp2>();
  HB_NOUNROLL for (uint32_t k = 0; k < j.cnt; k++) {
    const HmEntry e = pts[src ? src[j.m0 + k] : j.m0 + k];
    R = jac_add(R, member_general(j.wt, 0, e, dig[j.m0 + k]));
  }
  joint_store(out, j, R);
#endif
}

// ---------------------------------------------------------------------------------------
// Small-scalar aggregation (ta_small.h): sigma_v = [s] (sum_j [c_j] sigma_{v,j}) with small
// integers c_j and one scalar s per index set.  One lane per validator; a wave whose validators
// share the index set (the common slot: parsigdb fires with the partials of the same t operators,
// parsigex exchanges whole sets per peer) runs
//   k_ta_small    the joint NAF ladder of the c_j (~22 bits for any index set of a cluster of up to
//                 10 operators, shared doublings, mixed additions of +-sigma_j), then the affine
//                 odd-multiple tables of Q = sum_j [c_j] sigma_j (one inversion), and
//   k_ta_sladder  [s] Q: the signed width-4 NAF schedule over the four base-|x| digits of s,
// about 5.4k Fp products per validator against 1 856 per MEMBER on the per-member ladders (13k at
// t = 7).  Waves with mixed index sets (or splits refused by ta_small_split) leave `done` at 0 and
// take the per-member ladders (k_ta_jtab / k_ta_jladder / k_ta_jgeneral, or k_ta_straus), which
// skip the done groups.
// ---------------------------------------------------------------------------------------

// One lane per group of exactly t members: the split of the group's index set.
__global__ __launch_bounds__(64) void k_ta_sprep(const int64_t* __restrict__ idx, uint32_t n_groups, uint32_t t,
                                                 int64_t* __restrict__ csm, TaDigits* __restrict__ sdig,
                                                 uint8_t* __restrict__ sok, const uint8_t* __restrict__ nonuni) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  int64_t x[TA_SMALL_MAX], c[TA_SMALL_MAX];
  const uint32_t tt = (t <= (uint32_t)TA_SMALL_MAX && !(nonuni && *nonuni)) ? t : 0u;
  for (uint32_t k = 0; k < tt; k++) x[k] = idx[(size_t)g * t + k];
  Fr s = fr_zero();
  const bool ok = tt && ta_small_split(x, (int)tt, c, s);
  for (uint32_t k = 0; k < tt; k++) csm[(size_t)g * t + k] = ok ? c[k] : 0;
  TaDigits d;
  d.a[0] = d.a[1] = d.a[2] = d.a[3] = 0;
  if (ok) {
    const Fr sc = fr_from_mont(s);
    uint32_t u[NLR];
    HB_UNROLL for (int i = 0; i < NLR; i++) u[i] = sc.v[i];
    d.a[0] = divmod_xabs(u);
    d.a[1] = divmod_xabs(u);
    d.a[2] = divmod_xabs(u);
    d.a[3] = ((uint64_t)u[1] << 32) | u[0];
  }
  sdig[g] = d;
  sok[g] = ok ? 1 : 0;
}

#if defined(__HIP_DEVICE_COMPILE__)
// The affine odd multiples {1, 3, 5, 7} of the four bases B_b = Q, -psi(Q), psi^2(Q), -psi^3(Q) of a
// Jacobian Q into entries 4 b + (|d| >> 1) (the layout k_ta_jladder reads, one member), with ONE
// inversion over the four Z (Montgomery's trick; entries 4..7 hold the running products until the
// psi images overwrite them).  Returns false if Q is the point at infinity (the table is then
// garbage and [s] Q = infinity).
__device__ __forceinline__ bool odd_tables_affine_jac(uint4* wt, const G2J& Q) {
  const bool qinf = jac_is_inf(Q);
  Fp2 acc = f2_one();
  {
    const G2J J2 = jac_dbl(Q);
    const G2J J3 = jac_add(Q, J2);
    const G2J J5 = jac_add(J3, J2);
    const G2J J7 = jac_add(J5, J2);
    HB_NOUNROLL for (int j = 0; j < 4; j++) {
      G2J J = j == 0 ? Q : j == 1 ? J3 : j == 2 ? J5 : J7;
      if (f2_is_zero(J.Z)) J.Z = f2_one();
      tab_store(wt, j, J);
      f2_store_q(wt, 4 + j, 0, acc);
      acc = f2_mul(acc, J.Z);
    }
  }
  Fp2 inv = f2_inv(acc);
  const Fp2 cx = f2_from_const(PSI_CX), cy = f2_from_const(PSI_CY);
  const Fp2 c2x = f2_from_const(PSI2_CX), c2y = f2_from_const(PSI2_CY);
  HB_NOUNROLL for (int j = 3; j >= 0; j--) {
    const G2J J = tab_load(wt, j);
    const Fp2 zi = f2_mul(inv, f2_load_q(wt, 4 + j, 0));  // 1 / Z
    inv = f2_mul(inv, J.Z);
    const Fp2 zi2 = f2_sqr(zi);
    const Fp2 x = f2_mul(J.X, zi2), y = f2_mul(J.Y, f2_mul(zi2, zi));
    aff_store(wt, j, x, y);
    const Fp2 x2 = f2_mul(x, c2x), y2 = f2_mul(y, c2y);
    aff_store(wt, j + 4, f2_mul(f2_conj(x), cx), f2_neg(f2_mul(f2_conj(y), cy)));
    aff_store(wt, j + 8, x2, y2);
    aff_store(wt, j + 12, f2_mul(f2_conj(x2), cx), f2_neg(f2_mul(f2_conj(y2), cy)));
  }
  return !qinf;
}

// wave-uniform small path?  ok flag, the t scalars and the digits of s agree across the wave
__device__ __forceinline__ bool ta_small_uniform(const int64_t* __restrict__ csm, const TaDigits* __restrict__ sdig,
                                                 const uint8_t* __restrict__ sok, uint32_t v, uint32_t t) {
  bool same = sok[v] != 0;
  for (uint32_t k = 0; k < t; k++) {
    const uint64_t c = (uint64_t)csm[(size_t)v * t + k];
    same = same && (uint32_t)c == (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c) &&
           (uint32_t)(c >> 32) == (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(c >> 32));
  }
  const TaDigits d = sdig[v];
  HB_UNROLL for (int i = 0; i < 4; i++) {
    const uint32_t lo = (uint32_t)d.a[i], hi = (uint32_t)(d.a[i] >> 32);
    same = same && lo == (uint32_t)__builtin_amdgcn_readfirstlane((int)lo) &&
           hi == (uint32_t)__builtin_amdgcn_readfirstlane((int)hi);
  }
  return __all(same);
}
#endif


// One lane per validator: Q = sum_j [c_j] sigma_j (joint signed-binary NAF, the doublings shared by
// the t members) into out[v t]; done[v] = 1, or 0 when the wave is not uniform.
__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_small(const HmEntry* __restrict__ pts, const uint32_t* __restrict__ src,
                                                    const int64_t* __restrict__ csm, const TaDigits* __restrict__ sdig,
                                                    const uint8_t* __restrict__ sok, uint32_t n_groups, uint32_t t,
                                                    G2JEntry* __restrict__ out, uint8_t* __restrict__ done) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ int8_t naf[TA_SMALL_MAX][64];
  __shared__ int naf_top;
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t v = blockIdx.x * 64 + (uint32_t)lane;
  const bool valid = v < n_groups;
  const uint32_t vc = valid ? v : n_groups - 1;
  if (t < 2 || t > (uint32_t)TA_SMALL_MAX || !ta_small_uniform(csm, sdig, sok, vc, t)) {
    if (valid) done[v] = 0;
    return;  // wave-uniform
  }
  if (lane == 0) {  // NAF (digits +-1) of |c_k|, the sign folded in
    int top = 0;
    for (uint32_t k = 0; k < t; k++) {
      const int64_t c = csm[(size_t)vc * t + k];
      uint64_t m = (uint64_t)(c < 0 ? -c : c);  // < 2^63
      const int sg = c < 0 ? -1 : 1;
      for (int i = 0; i < 64; i++) {
        int dg = 0;
        if (m & 1u) {
          dg = (m & 2u) ? -1 : 1;
          m = dg > 0 ? m - 1 : m + 1;
        }
        naf[k][i] = (int8_t)(dg * sg);
        if (dg && i > top) top = i;
        m >>= 1;
      }
    }
    naf_top = top;
  }
  __syncthreads();
  const uint32_t m0 = vc * t;
  const int top = naf_top;
  // the joint ladder in lazily reduced 28-bit limbs (ec28.h g2l_dbl / g2l_madd, as k_ta_sladder);
  // a member at infinity (an undecodable partial, replaced by infinity in k_dec_sig_pt; its group's
  // status comes from the member flags) is skipped, as jac_add_aff's infinity operand
  G2L RL = g2l_infinity();
  HB_NOUNROLL for (int i = top; i >= 0; i--) {
    RL = g2l_dbl(RL);
    HB_NOUNROLL for (uint32_t k = 0; k < t; k++) {
      const int dg = naf[k][i];
      if (dg != 0) {  // wave-uniform
        const HmEntry e = pts[src ? src[m0 + k] : m0 + k];
        const G2L S = g2l_madd(RL, f2l_from(e.x), f2l_from(dg < 0 ? f2_neg(e.y) : e.y));
        if (!e.inf) RL = S;
      }
    }
  }
  const G2J R = g2l_to_jac(RL);
  if (valid) {
    out[(size_t)v * t] = {R.X, R.Y, R.Z};
    done[v] = 1;
  }
#endif
}

// One lane per validator of a wave k_ta_small took: Q's affine odd-multiple tables; done[v] = 2 when
// Q is the point at infinity ([s] Q is then infinity).
__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_stab(const G2JEntry* __restrict__ q, uint32_t n_groups, uint32_t t,
                                                   uint4* __restrict__ tab, uint8_t* __restrict__ done) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t v = blockIdx.x * 64 + (uint32_t)lane;
  const bool valid = v < n_groups;
  const uint32_t vc = valid ? v : n_groups - 1;
  if (done[vc] == 0) return;  // wave-uniform
  const G2JEntry e = q[(size_t)vc * t];
  uint4* wt = tab + (size_t)blockIdx.x * 16 * TA_TAB_QUADS * 64 + lane;
  const bool finite = odd_tables_affine_jac(wt, G2J{e.X, e.Y, e.Z});
  if (valid && !finite) done[v] = 2;
#endif
}

// One lane per validator of a wave k_ta_small took: [s] Q over Q's tables (k_ta_jladder's schedule
// for one member), into the validator's first member slot of `out`, infinity into the others.
// PAIR: each validator's ladder split over a lane pair (ec28.h F2Half: each lane one coefficient of
// every Fp2 product), 32 validators per wave, for slots too small to fill the chip, where this
// ladder is on the slot's critical path (aggregation -> the aggregates' combination -> the check).
template <bool PAIR>
__global__ KB_OCC(HB_OCC_STRAUS) void k_ta_sladder(const TaDigits* __restrict__ sdig, const uint8_t* __restrict__ done,
                                                      uint32_t n_groups, uint32_t t, uint4* __restrict__ tab,
                                                      G2JEntry* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ int8_t naf[4][66];
  __shared__ int naf_top;
  const int lane = (int)(threadIdx.x & 63u);
  constexpr uint32_t VPW = PAIR ? 32u : 64u;  // validators per wave
  const uint32_t v = blockIdx.x * VPW + (uint32_t)(PAIR ? lane >> 1 : lane);
  const bool valid = v < n_groups;
  const uint32_t vc = valid ? v : n_groups - 1;
  const uint8_t dn = done[vc];
  if (dn == 0) return;  // wave-uniform (k_ta_small decides per wave of 64, which holds this wave)
  if (lane == 0) {
    const TaDigits d = sdig[vc];
    int top = 0;
    for (int i = 0; i < 4; i++) top = max(top, naf4_digits(d.a[i], naf[i]));
    naf_top = top;
  }
  __syncthreads();
  // k_ta_stab's table layout: per wave of 64 validators, one column per validator
  const uint4* wt = tab + (size_t)(vc / 64) * 16 * TA_TAB_QUADS * 64 + (vc % 64);
  using M = typename std::conditional<PAIR, F2Half, F2One>::type;
  M m{};
  if constexpr (PAIR) m = f2half_make();
  G2L RL = g2l_infinity();  // the ladder in lazily reduced 28-bit limbs (ec28.h)
  const int top = naf_top;
  HB_NOUNROLL for (int i = top; i >= 0; i--) {
    RL = g2l_dbl(RL, m);
    HB_NOUNROLL for (int b = 0; b < 4; b++) {
      const int dg = naf[b][i];
      if (dg != 0) {  // wave-uniform
        const int e = 4 * b + ((dg < 0 ? -dg : dg) >> 1);
        G2A T = {f2_load_q(wt, e, 0), f2_load_q(wt, e, 6), false};
        if (dg < 0) T.y = f2_neg(T.y);
        RL = g2l_madd(RL, f2l_from(T.x), f2l_from(T.y), m);
      }
    }
  }
  if (!valid) return;
  if constexpr (PAIR) {
    if (lane & 1) return;  // both lanes hold the result
  }
  G2J R = g2l_to_jac(RL);
  if (dn == 2) R = jac_infinity<Fp2>();
  out[(size_t)v * t] = {R.X, R.Y, R.Z};
  const G2J z = jac_infinity<Fp2>();
  for (uint32_t k = 1; k < t; k++) out[(size_t)v * t + k] = {z.X, z.Y, z.Z};
#endif
}

// validators up to which the [s] ladder runs on lane pairs (HBLS_TA_PAIR_MAX at init via
// hbls_ta_pair_max; default 16384 as the hash's lane-pair threshold)
std::atomic<size_t> g_ta_pair_max{16384};
static size_t ta_pair_max() { return g_ta_pair_max.load(std::memory_order_relaxed); }

size_t ta_small_table_bytes(uint32_t n_groups) { return (size_t)blocks_of(n_groups, 64) * 16 * sizeof(G2JEntry) * 64; }

void launch_ta_small(const HmEntry* pts, const uint32_t* src, const int64_t* idx, uint32_t n_groups, uint32_t t,
                     int64_t* csm, TaDigits* sdig, uint8_t* sok, void* tab, uint8_t* done, G2JEntry* out,
                     hipStream_t s, const uint8_t* nonuni, hipEvent_t pts_ready) {
  if (!n_groups) {
    if (pts_ready) (void)hipStreamWaitEvent(s, pts_ready, 0);
    return;
  }
  const dim3 grid(blocks_of(n_groups, 64));
  // the split reads the share indices only: it runs while the members are still being decompressed
  hipLaunchKernelGGL(k_ta_sprep, grid, dim3(64), 0, s, idx, n_groups, t, csm, sdig, sok, nonuni);
  if (pts_ready) (void)hipStreamWaitEvent(s, pts_ready, 0);
  hipLaunchKernelGGL(k_ta_small, grid, dim3(64), 0, s, pts, src, csm, sdig, sok, n_groups, t, out, done);
  hipLaunchKernelGGL(k_ta_stab, grid, dim3(64), 0, s, (const G2JEntry*)out, n_groups, t, (uint4*)tab, done);
  if (n_groups <= ta_pair_max())
    hipLaunchKernelGGL(k_ta_sladder<true>, dim3(blocks_of(n_groups, 32)), dim3(64), 0, s, sdig, done, n_groups, t,
                       (uint4*)tab, out);
  else
    hipLaunchKernelGGL(k_ta_sladder<false>, grid, dim3(64), 0, s, sdig, done, n_groups, t, (uint4*)tab, out);
}

void launch_ta_lambda(const int64_t* idx, const uint32_t* grp_off, uint32_t n_groups,
                      uint32_t n_partials, int mode, TaDigits* dig, uint8_t* mstat, hipStream_t s, uint32_t t_u,
                      uint8_t* nonuni, const uint8_t* skip) {
  if (!n_partials) return;
  hipLaunchKernelGGL(k_ta_lambda, dim3(blocks_of(n_partials, 64)), dim3(64), 0, s, idx, grp_off, n_groups,
                     n_partials, mode, dig, mstat, t_u, nonuni, skip);
}

// one lane per group: does group g hold exactly t_u members at offset g t_u?  (vector stores only)
__global__ __launch_bounds__(64) void k_ta_layout(const uint32_t* __restrict__ grp_off, uint32_t n_groups, uint32_t t_u,
                                                  uint8_t* __restrict__ nonuni) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const uint32_t b = grp_off[g], en = grp_off[g + 1];
  if (en - b != t_u || b != g * t_u) *nonuni = 1;
}

void launch_ta_layout(const uint32_t* grp_off, uint32_t n_groups, uint32_t t_u, uint8_t* nonuni, hipStream_t s) {
  if (!n_groups) return;
  hipLaunchKernelGGL(k_ta_layout, dim3(blocks_of(n_groups, 64)), dim3(64), 0, s, grp_off, n_groups, t_u, nonuni);
}

size_t ta_table_bytes(uint32_t n_partials) { return (size_t)blocks_of(n_partials, 64) * 16 * sizeof(G2JEntry) * 64; }
size_t ta_joint_table_bytes(uint32_t n_groups, uint32_t t, uint32_t c) {
  const size_t lanes = (size_t)n_groups * ((t + c - 1) / c);
  return (size_t)blocks_of(lanes, 64) * 16 * c * sizeof(G2JEntry) * 64;
}
void launch_ta_joint(const HmEntry* pts, const uint32_t* src, const TaDigits* dig, uint32_t n_groups, uint32_t t,
                     uint32_t c, void* tab, G2JEntry* out, hipStream_t s, const uint8_t* skip,
                     const uint8_t* nonuni) {
  if (!n_groups || !t || !c || c > (uint32_t)TA_JOINT_MAX) return;
  const size_t lanes = (size_t)n_groups * ((t + c - 1) / c);
  const dim3 grid(blocks_of(lanes, 64));
  hipLaunchKernelGGL(k_ta_jtab, grid, dim3(64), 0, s, pts, src, dig, n_groups, t, c, (uint4*)tab, skip, nonuni);
  hipLaunchKernelGGL(k_ta_jladder, grid, dim3(64), 0, s, dig, n_groups, t, c, (uint4*)tab, out, skip, nonuni);
  hipLaunchKernelGGL(k_ta_jgeneral, grid, dim3(64), 0, s, pts, src, dig, n_groups, t, c, (uint4*)tab, out, skip,
                     nonuni);
}

void launch_ta_straus(const HmEntry* pts, const uint32_t* src, const TaDigits* dig, uint32_t n_partials,
                      uint32_t n_groups, void* tab, G2JEntry* out, hipStream_t s, const uint8_t* skip,
                      const uint8_t* guard) {
  if (!n_partials) return;
  // members laid out share-position-major when every group has the same size t (a permutation of
  // the members: right for any group structure); the guarded launch behind the joint path takes
  // them in plain order
  const uint32_t t = (!guard && n_groups && n_partials % n_groups == 0) ? n_partials / n_groups : 0;
  hipLaunchKernelGGL(k_ta_straus, dim3(blocks_of(n_partials, 64)), dim3(64), 0, s, pts, src, dig, n_partials,
                     n_groups, t, (uint4*)tab, out, guard ? nullptr : skip, guard);
}

// Member statuses of a ThresholdAggregate whose partials were decompressed by the verification
// of the same slot (member j = verified partial src[j]): undecodable there = undecodable here.
__global__ __launch_bounds__(64) void k_ta_member_status(const uint8_t* __restrict__ sig_st,
                                                         const uint32_t* __restrict__ src, uint32_t n_partials,
                                                         uint8_t* __restrict__ mstat) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_partials) return;
  mstat[j] = sig_st[src[j]] ? M_BAD_SIG : M_OK;
}

void launch_ta_member_status(const uint8_t* sig_st, const uint32_t* src, uint32_t n_partials, uint8_t* mstat,
                             hipStream_t s) {
  if (n_partials)
    hipLaunchKernelGGL(k_ta_member_status, dim3(blocks_of(n_partials, 64)), dim3(64), 0, s, sig_st, src,
                       n_partials, mstat);
}

}  // namespace hb
