// Random linear combinations for batched verification (vbatch.hip; host-compiled by the test
// harness for op counts).  r = a + b * lambda with 32-bit a, b and lambda = -x^2 mod r, the
// eigenvalue of phi(x, y) = (beta x, y) on G1 (ec.h g1_in_subgroup: phi(P) = [-x^2] P) and of
// -psi^2 on G2 (psi^2(Q) = [x^2] Q), so [r] P = [a] P + [b] phi(P) and [r] S = [a] S + [b] (-psi^2(S)).
#pragma once
#include "ec.h"

namespace hb {

template <class F>
HD Jac<F> jac_select(bool take_b, const Jac<F>& a, const Jac<F>& b) {
  Jac<F> r;
  const uint32_t* pa = reinterpret_cast<const uint32_t*>(&a);
  const uint32_t* pb = reinterpret_cast<const uint32_t*>(&b);
  uint32_t* pr = reinterpret_cast<uint32_t*>(&r);
  HB_UNROLL for (int k = 0; k < (int)(sizeof(Jac<F>) / 4); k++) pr[k] = take_b ? pb[k] : pa[k];
  return r;
}

// [a] T1 + [b] T2 for affine T1, T2 (T1 != +-T2): joint 32-step ladder over {T1, T2, T1 + T2};
// uniform control flow (the addition of every step is computed and kept or dropped per lane).
template <class F>
HDNI Jac<F> joint_mul32(const Aff<F>& T1, const Aff<F>& T2, uint32_t a, uint32_t b) {
  const Jac<F> J1 = jac_from_aff(T1), J2 = jac_from_aff(T2);
  const Jac<F> J3 = jac_add_aff(J1, T2);
  Jac<F> R = jac_infinity<F>();
  HB_NOUNROLL for (int i = 31; i >= 0; i--) {
    R = jac_dbl(R);
    const uint32_t sel = ((a >> i) & 1u) | (((b >> i) & 1u) << 1);
    const Jac<F> T = jac_select(sel == 3, jac_select(sel == 2, J1, J2), J3);
    const Jac<F> S = jac_add(R, T);
    R = jac_select(sel != 0, R, S);
  }
  return R;
}

HD G1J rlc_g1(const G1A& P, uint32_t a, uint32_t b) {
  const G1A P2 = {fp_mul(P.x, fp_from_const(G1_BETA)), P.y, false};
  return joint_mul32(P, P2, a, b);
}

HD G2J rlc_g2(const G2A& S, uint32_t a, uint32_t b) {
  const G2A S2 = {f2_mul(S.x, f2_from_const(PSI2_CX)), f2_neg(f2_mul(S.y, f2_from_const(PSI2_CY))), false};
  return joint_mul32(S, S2, a, b);
}

// The chunk ladders' points in ec28.h's sparse coefficient format: per item T1, T2, T1 + T2,
// T1 - T2 at t[4i .. 4i + 3], affine with ONE inversion per chunk (Montgomery's trick).  Forward
// pass (sparse_put, items in order): the four records, entry 0's Z holding the running product of
// the sums' Z before this item; returns the product through it.  Then inv = 1 / that product and
// the backward pass (sparse_fix, items in reverse) makes the records affine, returning the inverse
// of the product before the item.  A sum at infinity (T1 = -+T2: never for points of the prime
// subgroups) keeps Z = 1 so the product stays invertible; such an item's record is never read.
template <class F>
HD F sparse_put(Jac<F>* t, uint64_t i, const Aff<F>& P, const Aff<F>& P2, const F& acc) {
  const Jac<F> J1 = jac_from_aff(P), J2 = jac_from_aff(P2);
  Jac<F> J3 = jac_add_aff(J1, P2);
  Jac<F> J4 = jac_add_aff(J1, Aff<F>{P2.x, f_neg(P2.y), false});
  if (f_is_zero(J3.Z)) J3.Z = J1.Z;
  if (f_is_zero(J4.Z)) J4.Z = J1.Z;
  t[4 * i] = {J1.X, J1.Y, acc};
  t[4 * i + 1] = J2;
  t[4 * i + 2] = J3;
  t[4 * i + 3] = J4;
  return f_mul(f_mul(acc, J3.Z), J4.Z);
}
template <class F>
HD F sparse_fix(Jac<F>* t, uint64_t i, const F& inv_through) {
  Jac<F> J1 = t[4 * i];
  const Jac<F> J3 = t[4 * i + 2], J4 = t[4 * i + 3];
  const F one = t[4 * i + 1].Z;
  const F z34 = f_mul(inv_through, J1.Z);  // 1 / (Z3 Z4)
  const F inv_before = f_mul(f_mul(inv_through, J3.Z), J4.Z);
  const F z3 = f_mul(z34, J4.Z), z4 = f_mul(z34, J3.Z);
  const F z3s = f_sqr(z3), z4s = f_sqr(z4);
  J1.Z = one;
  t[4 * i] = J1;
  t[4 * i + 2] = {f_mul(J3.X, z3s), f_mul(J3.Y, f_mul(z3s, z3)), one};
  t[4 * i + 3] = {f_mul(J4.X, z4s), f_mul(J4.Y, f_mul(z4s, z4)), one};
  return inv_before;
}

}  // namespace hb
