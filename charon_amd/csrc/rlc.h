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

}  // namespace hb
