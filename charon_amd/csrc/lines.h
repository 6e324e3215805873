// The Miller chain of an affine G2 point (shared by pipeline.hip and vbatch.hip).
#pragma once
#include "layout.h"

namespace hb {

// The Miller chain of an affine G2 point Q: 68 lines, stored at out[j * stride].  EVAL: evaluate
// each line at -g1 (pair (-g1, S) of the verification equation); otherwise store (a0, c1, c2).
template <bool EVAL>
__device__ __forceinline__ void line_chain(const G2A& Q, LineEntry* __restrict__ out, size_t stride) {
  G2Proj T = {Q.x, Q.y, f2_one()};
  int j = 0;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    LineCoeffs l = miller_dbl_c(T);
    if (EVAL) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
    out[(size_t)j * stride] = {l.a0, l.a1, l.b1};
    j++;
    if ((HB_X_ABS >> i) & 1) {
      l = miller_add_c(T, Q.x, Q.y);
      if (EVAL) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
      out[(size_t)j * stride] = {l.a0, l.a1, l.b1};
      j++;
    }
  }
}

}  // namespace hb
