// threshold.hip: staged ThresholdAggregate / Aggregate kernels of libhipbls.so
// (tbls.ThresholdAggregate -> Herumi.ThresholdAggregate, herumi.go:249-286; tbls.Aggregate,
// herumi.go:225-247).  Compiled like pipeline.hip (HB_FAST_FPMUL: register-convention Fp
// product, everything else inlined).
//
//   k_ta_dec   (hipbls.hip) 1 lane / partial: decompress + subgroup-check sigma_j
//   k_ta_lambda 1 lane / partial: lambda_j(0) over its group's share indices (Fr), and the
//              base-|x| digits of lambda_j
//   k_ta_mul4  4 lanes / partial: lambda_j sigma_j = sum_i [a_i] psi^i(sigma_j) (-1)^i, one
//              64-bit digit per lane, then a 2-round lane reduction
//   k_group_sum (hipbls.hip) 1 lane / group: sum, affine, compress
//
// The split of lambda uses the G2 endomorphism psi, which acts on G2 as multiplication by the
// curve parameter x (this is the subgroup test of ec.h, psi(Q) == [x]Q).  With z = |x| = -x and
// lambda = a0 + a1 z + a2 z^2 + a3 z^3 (0 <= a_i < z; lambda < r < z^4):
//   [lambda] Q = [a0] Q - [a1] psi(Q) + [a2] psi^2(Q) - [a3] psi^3(Q),
// four independent 64-bit scalar multiplications instead of one 255-bit one.  The result is the
// same group element, so the 96-byte output is byte-identical to herumi's Sign.Recover.
#define HB_FAST_FPMUL 1
#include "layout.h"

namespace hb {

#if defined(__HIP_DEVICE_COMPILE__)
// hb_fpmul has hidden visibility per code object: each translation unit carries its own copy
HB_DEFINE_FPMUL_SUBROUTINE(hb_fpmul_holder_threshold)
#else
__global__ void hb_fpmul_holder_threshold() {}
#endif

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
                                                  TaDigits* __restrict__ dig, uint8_t* __restrict__ mstat) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_partials) return;
  TaDigits d;
  d.a[0] = 1;
  d.a[1] = d.a[2] = d.a[3] = 0;
  uint32_t g = find_group_ta(grp_off, n_groups, j);
  uint32_t b = grp_off[g], en = grp_off[g + 1];
  if (mode == 0 && en - b > 1) {  // k = 1: the single partial is returned as is
    Fr xi = fr_from_i64(idx[j]);
    Fr num = fr_one(), den = fr_one();
    for (uint32_t m = b; m < en; m++) {
      if (m == j) continue;
      Fr xm = fr_from_i64(idx[m]);
      num = fr_mul(num, xm);
      den = fr_mul(den, fr_sub(xm, xi));
    }
    if (fr_is_zero(num) || fr_is_zero(den)) {
      if (mstat[j] == M_OK) mstat[j] = M_BAD_IDX;
    } else {
      Fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
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
__device__ __forceinline__ uint32_t xch4(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(lane << 2, (int)v);
}
__device__ __forceinline__ Fp2 xch4(const Fp2& a, int lane) {
  Fp2 r;
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.c0.v[i] = xch4(a.c0.v[i], lane);
    r.c1.v[i] = xch4(a.c1.v[i], lane);
  }
  return r;
}
__device__ __forceinline__ G2J xch4(const G2J& p, int lane) { return {xch4(p.X, lane), xch4(p.Y, lane), xch4(p.Z, lane)}; }

__device__ __forceinline__ void f2_select(Fp2& r, bool take_b, const Fp2& a, const Fp2& b) {
  HB_UNROLL for (int i = 0; i < NL; i++) {
    r.c0.v[i] = take_b ? b.c0.v[i] : a.c0.v[i];
    r.c1.v[i] = take_b ? b.c1.v[i] : a.c1.v[i];
  }
}
#endif

// Four lanes per partial (16 partials per wave): lane i computes (-1)^i [a_i] psi^i(sigma), the
// quad then sums its four points.  Uniform control flow: the add of every step is computed and
// kept or dropped per lane by select.
__global__ __launch_bounds__(64, 2) void k_ta_mul4(const HmEntry* __restrict__ pts, const TaDigits* __restrict__ dig,
                                                   uint32_t n_partials, G2JEntry* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int lane = (int)(threadIdx.x & 63u);
  const int i = lane & 3;
  const uint32_t item = blockIdx.x * 16 + (uint32_t)(lane >> 2);
  const bool valid = item < n_partials;
  const uint32_t it = valid ? item : n_partials - 1;
  const HmEntry e = pts[it];
  const uint64_t a = dig[it].a[i];
  // psi^i(sigma): psi^2 (x, y) = (x c2x, y c2y); psi (x, y) = (conj(x) c1x, conj(y) c1y)
  Fp2 x = e.x, y = e.y;
  {
    Fp2 x2 = f2_mul(x, f2_from_const(PSI2_CX)), y2 = f2_mul(y, f2_from_const(PSI2_CY));
    f2_select(x, (i & 2) != 0, x, x2);
    f2_select(y, (i & 2) != 0, y, y2);
    Fp2 x1 = f2_mul(f2_conj(x), f2_from_const(PSI_CX)), y1 = f2_mul(f2_conj(y), f2_from_const(PSI_CY));
    f2_select(x, (i & 1) != 0, x, x1);
    f2_select(y, (i & 1) != 0, y, y1);
    Fp2 ny = f2_neg(y);  // (-1)^i
    f2_select(y, (i & 1) != 0, y, ny);
  }
  const G2A P = {x, y, e.inf != 0};
  G2J R = jac_infinity<Fp2>();
  HB_NOUNROLL for (int b = 63; b >= 0; b--) {
    R = jac_dbl(R);
    G2J S = jac_add_aff(R, P);
    const bool take = ((a >> b) & 1) != 0;
    f2_select(R.X, take, R.X, S.X);
    f2_select(R.Y, take, R.Y, S.Y);
    f2_select(R.Z, take, R.Z, S.Z);
  }
  R = jac_add(R, xch4(R, lane ^ 1));
  R = jac_add(R, xch4(R, lane ^ 2));
  if (valid && i == 0) out[item] = {R.X, R.Y, R.Z};
#endif
}

static inline unsigned blocks_of(size_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

void launch_ta_lambda(const int64_t* idx, const uint32_t* grp_off, uint32_t n_groups,
                      uint32_t n_partials, int mode, TaDigits* dig, uint8_t* mstat, hipStream_t s) {
  if (!n_partials) return;
  hipLaunchKernelGGL(k_ta_lambda, dim3(blocks_of(n_partials, 64)), dim3(64), 0, s, idx, grp_off, n_groups,
                     n_partials, mode, dig, mstat);
}

void launch_ta_mul4(const HmEntry* pts, const TaDigits* dig, uint32_t n_partials, G2JEntry* out, hipStream_t s) {
  if (n_partials)
    hipLaunchKernelGGL(k_ta_mul4, dim3(blocks_of(n_partials, 16)), dim3(64), 0, s, pts, dig, n_partials, out);
}

}  // namespace hb
