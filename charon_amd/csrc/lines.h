// The Miller chain of an affine G2 point (shared by pipeline.hip and vbatch.hip).
#pragma once
#include "layout.h"
#include "pair28.h"

namespace hb {

// pair28.h's lazy-limb chain, whose lines equal pairing.h's stored-word ones up to one nonzero Fp2
// factor per line (its doubling keeps T scaled by 4), which the final exponentiation removes
// (tests/test_lazy28.py)

// The Miller chain of an affine G2 point Q: 68 lines, stored at out[j * stride].  EVAL: evaluate
// each line at -g1 (pair (-g1, S) of the verification equation); otherwise store (a0, c1, c2).
template <bool EVAL>
__device__ __forceinline__ void line_chain(const G2A& Q, LineEntry* __restrict__ out, size_t stride) {
  line_chain28<EVAL>([&]() { return Q; }, [&](int j, const LineCoeffs& l) { out[(size_t)j * stride] = {l.a0, l.a1, l.b1}; });
}

// line_chain of an affine point read from memory (re-read at the chain's additions instead of
// held in registers across it)
template <bool EVAL>
__device__ __forceinline__ void line_chain_ld(const HmEntry* src, LineEntry* __restrict__ out, size_t stride) {
  line_chain28<EVAL>([src]() { return hm_load(*src); },
                     [&](int j, const LineCoeffs& l) { out[(size_t)j * stride] = {l.a0, l.a1, l.b1}; });
}

#if defined(__HIP_DEVICE_COMPILE__)
// a stored-word line (evaluated, < 2p) as limbs, and a reduced lane value as the stored Fp4Entry
__device__ __forceinline__ void line_split(const LineEntry& L, F2L& a0, F2L& a1, F2L& b1) {
  a0 = f2l_from(L.a0);
  a1 = f2l_from(L.a1);
  b1 = f2l_from(L.b1);
}
__device__ __forceinline__ Fp4Entry f4l_store(const F4L& f) { return {f2l_join(f.x), f2l_join(f.y)}; }
#endif

}  // namespace hb
