// vgroup.hip: the per-group stage of the batched verification (vbatch.hip).
//
// History: built with r01's register-convention product subroutine (a hand-written routine
// entered through inline asm the compiler could not see into), this kernel returned a wrong group
// sum -- a point off the curve -- on the GPU, deterministically, while the same source built with
// a compiler-visible product was exact (tests/native/devcheck_vb.hip).  That
// subroutine is gone; the kernel is compiled like the other fast units.
#define HB_FAST_FPMUL 1
#include "lines.h"
#include "pair3.h"

namespace hb {

__device__ __forceinline__ bool item_usable_g(const G1AEntry& p, uint8_t pst, const HmEntry& s, uint8_t sst) {
  return !pst && !sst && !p.inf && !s.inf;
}

// The group's state; when READY, P = its combined public key (affine, finite) and its combined
// signature as S (Jacobian; BATCH) or Sa (affine).  Group sizes of one without an aggregate keep
// r = 1 (k_rlc) and take the decoded points directly unless BATCH (random r for every item).
// P_ONLY (the slot-wide check, msm.hip): no signature side at all; a degenerate S is caught by
// the slot-wide check failing.
template <bool BATCH, bool P_ONLY = false>
__device__ __forceinline__ uint8_t group_scan(const GroupPrepArgs& a, uint32_t lg, G1A& P, G2J& S, G2A& Sa) {
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
  if (cnt == 0 || (!a.skip_hm && a.hm[m].h.inf)) return G_EMPTY;
  if (!consistent) return G_FALLBACK;
  if (!BATCH && cnt == 1 && !with_agg) {
    P = g1a_load(a.pk[first]);
    Sa = hm_load(a.sig[first]);
    return G_READY;
  }
  // unusable items hold the point at infinity (k_rlc, k_rlc_msm: a chunk's sum sits in its first
  // item's slot): a plain sum -- except a key side combined from the keys alone (keys_only, one
  // item per slot), where a key whose signature then failed is skipped here
  G1J pacc = jac_infinity<Fp>();
  G2J sacc = jac_infinity<Fp2>();
  for (uint32_t i = b; i < e; i++) {
    if (a.keys_only && !item_usable_g(a.pk[i], a.pk_st[i], a.sig[i], a.sig_st[i])) continue;
    const G1JEntry pj = a.pr[i];
    pacc = jac_add(pacc, G1J{pj.X, pj.Y, pj.Z});
    if (!P_ONLY) {
      const G2JEntry sj = a.sr[i];
      sacc = jac_add(sacc, G2J{sj.X, sj.Y, sj.Z});
    }
  }
  if (with_agg) {
    const G1JEntry pj = a.agg_pr[g];
    pacc = jac_add(pacc, G1J{pj.X, pj.Y, pj.Z});
    if (!P_ONLY) {
      const G2JEntry sj = a.agg_sr[g];
      sacc = jac_add(sacc, G2J{sj.X, sj.Y, sj.Z});
    }
  }
  P = jac_to_aff(pacc);
  bool s_inf;
  if (P_ONLY) {
    s_inf = false;
  } else if (BATCH) {
    S = sacc;
    s_inf = jac_is_inf(sacc);
  } else {
    Sa = jac_to_aff(sacc);
    s_inf = Sa.inf;
  }
  // a degenerate combination (probability ~2^-64): check every item alone
  return (P.inf || s_inf) ? G_FALLBACK : G_READY;
}

__device__ __forceinline__ void store_gp(G1AEntry* out, const G1A& P) {
  G1AEntry pe;
  pe.x = P.x;
  pe.y = P.y;
  pe.inf = 0;
  pe.pad[0] = pe.pad[1] = pe.pad[2] = 0;
  *out = pe;
}

// One lane per verification group: sum the combined points of its usable items (plus the folded
// aggregate), affine, and the Miller lines of the signature side evaluated at -g1.
__global__ KB_OCC(HB_OCC_PREP) void k_group_prep(GroupPrepArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (lg >= a.ng) return;
  G1A P;
  G2J S;
  G2A Sa;
  const uint8_t st = group_scan<false>(a, lg, P, S, Sa);
  a.gst[lg] = st;
  if (st != G_READY) return;
  store_gp(a.gP + lg, P);
  line_chain<true>(Sa, a.glines + lg, a.ng);
#endif
}

// Batched final exponentiation: one lane per group as above but no lines; the group's S is kept
// (gS) and each batch of fe_batch consecutive groups of the wave sums its S into bS (butterfly
// over the batch's lanes).
__global__ KB_OCC(HB_OCC_PREP) void k_group_prep_b(GroupPrepArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (a.guard && *a.guard == 0) return;
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  G2J S = jac_infinity<Fp2>();
  if (lg < a.ng) {
    G1A P;
    G2J Sg;
    G2A Sa;
    const uint8_t st = group_scan<true>(a, lg, P, Sg, Sa);
    a.gst[lg] = st;
    if (st == G_READY) {
      store_gp(a.gP + lg, P);
      S = Sg;
    }
    a.gS[lg] = {S.X, S.Y, S.Z};
  }
  const int lane = (int)(threadIdx.x & 63u);
  const int fb = a.fe_batch ? (int)a.fe_batch : (int)FE_BATCH;
  HB_NOUNROLL for (int off = fb >> 1; off; off >>= 1) {
    const int addr = (lane ^ off) << 2;
    const G2J T = {xch(S.X, addr), xch(S.Y, addr), xch(S.Z, addr)};
    S = jac_add(S, T);
  }
  if (a.bS && (lane & (fb - 1)) == 0 && lg < a.ng) a.bS[lg / (uint32_t)fb] = {S.X, S.Y, S.Z};
#endif
}

// Behind a failed slot-wide check: one lane per batch of k consecutive groups (a multi-Miller
// loop's chunk), the sum of their signature sides S_g (infinity for groups that are not READY).
__global__ KB_OCC(HB_OCC_PREP) void k_batch_sum(const G2JEntry* __restrict__ gS, uint32_t ng, uint32_t k,
                                              G2JEntry* __restrict__ bS, const uint8_t* __restrict__ guard) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (guard && *guard == 0) return;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t first = b * k;
  if (first >= ng) return;
  const uint32_t last = min(first + k, ng);
  G2J S = jac_infinity<Fp2>();
  for (uint32_t i = first; i < last; i++) {
    const G2JEntry e = gS[i];
    S = jac_add(S, G2J{e.X, e.Y, e.Z});
  }
  bS[b] = {S.X, S.Y, S.Z};
#endif
}

// Slot-wide check (msm.hip): one lane per verification group, its combined public key and state
// only (the signature side is one multi-scalar multiplication over the whole call).
__global__ KB_OCC(HB_OCC_PREP) void k_group_prep_p(GroupPrepArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (lg >= a.ng) return;
  G1A P;
  G2J Sg;
  G2A Sa;
  const uint8_t st = group_scan<true, true>(a, lg, P, Sg, Sa);
  a.gst[lg] = st;
  if (st == G_READY) store_gp(a.gP + lg, P);
#endif
}

__global__ KB_OCC(HB_OCC_LINES) void k_slines(const G2JEntry* __restrict__ pts, const uint32_t* __restrict__ list,
                                             const uint32_t* __restrict__ count, uint32_t n,
                                             LineEntry* __restrict__ lines, uint32_t stride, uint8_t* __restrict__ bad,
                                             const uint8_t* __restrict__ guard) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (guard && *guard == 0) return;
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t avail = list ? min(*count, n) : n;
  if (u >= avail) return;
  const uint32_t e = list ? list[u] : u;
  const G2JEntry pe = pts[e];
  const G2A S = jac_to_aff(G2J{pe.X, pe.Y, pe.Z});
  if (bad) bad[u] = S.inf ? 1 : 0;
  if (S.inf) return;  // the verdict comes from bad[u]; the lines are never used
  line_chain<true>(S, lines + u, stride);
#endif
}

__global__ __launch_bounds__(64) void k_batch_verdict(const uint8_t* __restrict__ gst, const uint8_t* __restrict__ bver, uint32_t ng,
                                   uint8_t* __restrict__ gver, uint32_t* __restrict__ list,
                                   uint32_t* __restrict__ count, const uint8_t* __restrict__ guard, uint32_t fb,
                                   const uint32_t* __restrict__ first, uint32_t g0) {
  if (guard && *guard == 0) return;
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (lg >= ng) return;
  if (gst[lg] != G_READY) gver[lg] = GV_NOT_READY;
  else if (bver[lg / fb] == 0) gver[lg] = GV_PASS;
  else if (first && g0 + (lg / fb) * fb != *first) gver[lg] = GV_UNCHECKED;
  else list[atomicAdd(count, 1u)] = lg;
}
// first-error mode, before k_batch_verdict: the key of the first failing batch of READY groups
__global__ __launch_bounds__(64) void k_first_batch(const uint8_t* __restrict__ gst, const uint8_t* __restrict__ bver,
                                                     uint32_t ng, const uint8_t* __restrict__ guard, uint32_t fb,
                                                     uint32_t* __restrict__ first, uint32_t g0) {
  if (guard && *guard == 0) return;
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (lg >= ng || gst[lg] != G_READY || bver[lg / fb] == 0) return;
  atomicMin(first, g0 + (lg / fb) * fb);
}
__global__ __launch_bounds__(64) void k_first_group(const uint8_t* __restrict__ gver, uint32_t ng,
                                                     uint32_t* __restrict__ first) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng && gv_failed(gver[g])) atomicMin(first, g);
}
__global__ __launch_bounds__(64) void k_first_item(const uint8_t* __restrict__ st, uint32_t n,
                                                    uint32_t* __restrict__ first) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && st[i] != ST_OK && st[i] != ST_UNCHECKED) atomicMin(first, i);
}

// sfail[0]: the slot-wide check's outcome; sfail[1] (zeroed before): set when anything will read
// the messages' unevaluated Miller lines -- the per-batch check behind a failed slot-wide check,
// or a group that was not READY (inconsistent messages, a degenerate combination), whose items
// the per-item fallback checks alone.  The deferred k_lines_msg is guarded by it.
__global__ __launch_bounds__(64) void k_slot_verdict(const uint8_t* __restrict__ gst, uint8_t* __restrict__ sfail,
                                                      uint32_t ng, uint8_t* __restrict__ gver) {
  const uint32_t lg = blockIdx.x * blockDim.x + threadIdx.x;
  if (sfail[0] != 0) {
    if (lg == 0) sfail[1] = 1;
    return;
  }
  if (lg < ng) {
    const bool fb = gst[lg] != G_READY;
    gver[lg] = fb ? GV_NOT_READY : GV_PASS;
    if (fb) sfail[1] = 1;
  }
}

void launch_group_prep(const GroupPrepArgs& a, hipStream_t s) {
  if (!a.ng) return;
  if (a.p_only) hipLaunchKernelGGL(k_group_prep_p, dim3((a.ng + 63) / 64), dim3(64), 0, s, a);
  else if (a.gS) hipLaunchKernelGGL(k_group_prep_b, dim3((a.ng + 63) / 64), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(k_group_prep, dim3((a.ng + 63) / 64), dim3(64), 0, s, a);
}
void launch_batch_sum(const G2JEntry* gS, uint32_t ng, uint32_t k, G2JEntry* bS, hipStream_t s, const uint8_t* guard) {
  const uint32_t nb = (ng + k - 1) / k;
  if (nb) hipLaunchKernelGGL(k_batch_sum, dim3((nb + 63) / 64), dim3(64), 0, s, gS, ng, k, bS, guard);
}
void launch_slines(const G2JEntry* pts, const uint32_t* list, const uint32_t* count, uint32_t n, LineEntry* lines,
                   uint32_t stride, uint8_t* bad, hipStream_t s, const uint8_t* guard) {
  if (n)
    hipLaunchKernelGGL(k_slines, dim3((n + 63) / 64), dim3(64), 0, s, pts, list, count, n, lines, stride, bad, guard);
}
void launch_batch_verdict(const uint8_t* gst, const uint8_t* bver, uint32_t ng, uint8_t* gver, uint32_t* list,
                          uint32_t* count, hipStream_t s, const uint8_t* guard, uint32_t fe_batch, uint32_t* first,
                          uint32_t g0) {
  if (!ng) return;
  const uint32_t fb = fe_batch ? fe_batch : FE_BATCH;
  if (first)
    hipLaunchKernelGGL(k_first_batch, dim3((ng + 63) / 64), dim3(64), 0, s, gst, bver, ng, guard, fb, first, g0);
  hipLaunchKernelGGL(k_batch_verdict, dim3((ng + 63) / 64), dim3(64), 0, s, gst, bver, ng, gver, list, count, guard,
                     fb, (const uint32_t*)first, g0);
}
void launch_first_group(const uint8_t* gver, uint32_t n_groups, uint32_t* first_group, hipStream_t s) {
  if (n_groups) hipLaunchKernelGGL(k_first_group, dim3((n_groups + 63) / 64), dim3(64), 0, s, gver, n_groups, first_group);
}
void launch_first_item(const uint8_t* status, uint32_t n, uint32_t* first_item, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_first_item, dim3((n + 63) / 64), dim3(64), 0, s, status, n, first_item);
}
void launch_slot_verdict(const uint8_t* gst, uint8_t* sfail, uint32_t ng, uint8_t* gver, hipStream_t s) {
  if (ng) hipLaunchKernelGGL(k_slot_verdict, dim3((ng + 63) / 64), dim3(64), 0, s, gst, sfail, ng, gver);
}

}  // namespace hb
