// vgroup.hip: the per-group stage of the batched verification (vbatch.hip).
//
// History: built with r01's register-convention product subroutine (a hand-written routine
// entered through inline asm the compiler could not see into), this kernel returned a wrong group
// sum -- a point off the curve -- on the GPU, deterministically, while the same source built with
// a compiler-visible product was exact (tests/native/devcheck_vb.hip).  That
// subroutine is gone; the kernel is compiled like the other fast units.
#define HB_FAST_FPMUL 1
#include "lines.h"

namespace hb {

__device__ __forceinline__ bool item_usable_g(const G1AEntry& p, uint8_t pst, const HmEntry& s, uint8_t sst) {
  return !pst && !sst && !p.inf && !s.inf;
}

// One lane per verification group: sum the combined points of its usable items (plus the folded
// aggregate), affine, and the Miller lines of the signature side evaluated at -g1.
__global__ KB_OCC(HB_OCC_PREP) void k_group_prep(GroupPrepArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (lg >= a.ng) return;
  const uint32_t g = a.g0 + lg;
  const uint32_t b = a.grp_off ? a.grp_off[g] : g, e = a.grp_off ? a.grp_off[g + 1] : g + 1;
  uint32_t cnt = 0, first = b, m = 0;
  bool consistent = true;
  for (uint32_t i = b; i < e; i++) {
    if (!item_usable_g(a.pk[i], a.pk_st[i], a.sig[i], a.sig_st[i])) continue;
    const uint32_t mi = a.msg_idx[i];
    if (cnt == 0) {
      first = i;
      m = mi;
    } else if (mi != m) {
      consistent = false;
    }
    cnt++;
  }
  const bool with_agg = a.agg_pk && !a.agg_st[g] && !a.agg_pk_st[g] && !a.agg_pk[g].inf && !a.agg_sig[g].inf &&
                        cnt > 0;  // the aggregate takes its message from the group's partials
  if (cnt == 0 && e > b) m = a.msg_idx[b];  // the folded aggregate's message (a fallback may need it)
  a.gmsg[g] = m;
  if (cnt == 0 || a.hm[m].h.inf) {
    a.gst[lg] = G_EMPTY;
    return;
  }
  if (!consistent) {
    a.gst[lg] = G_FALLBACK;
    return;
  }
  G1A P;
  G2A S;
  if (cnt == 1 && !with_agg) {
    P = g1a_load(a.pk[first]);
    S = hm_load(a.sig[first]);
  } else {
    // unusable items hold the point at infinity (k_rlc): a plain sum
    G1J pacc = jac_infinity<Fp>();
    G2J sacc = jac_infinity<Fp2>();
    for (uint32_t i = b; i < e; i++) {
      const G1JEntry pj = a.pr[i];
      const G2JEntry sj = a.sr[i];
      pacc = jac_add(pacc, G1J{pj.X, pj.Y, pj.Z});
      sacc = jac_add(sacc, G2J{sj.X, sj.Y, sj.Z});
    }
    if (with_agg) {
      const G1JEntry pj = a.agg_pr[g];
      const G2JEntry sj = a.agg_sr[g];
      pacc = jac_add(pacc, G1J{pj.X, pj.Y, pj.Z});
      sacc = jac_add(sacc, G2J{sj.X, sj.Y, sj.Z});
    }
    P = jac_to_aff(pacc);
    S = jac_to_aff(sacc);
  }
  if (P.inf || S.inf) {  // a degenerate combination (probability ~2^-64): check every item alone
    a.gst[lg] = G_FALLBACK;
    return;
  }
  G1AEntry pe;
  pe.x = P.x;
  pe.y = P.y;
  pe.inf = 0;
  pe.pad[0] = pe.pad[1] = pe.pad[2] = 0;
  a.gP[lg] = pe;
  a.gst[lg] = G_READY;
  line_chain<true>(S, a.glines + lg, a.ng);
#endif
}


void launch_group_prep(const GroupPrepArgs& a, hipStream_t s) {
  if (a.ng) hipLaunchKernelGGL(k_group_prep, dim3((a.ng + 63) / 64), dim3(64), 0, s, a);
}

}  // namespace hb
