// vbatch.hip: batched verification of partial signatures (tbls.Verify, herumi.go:288-304, for a
// whole slot at once; callers core/parsigex/parsigex.go:93-98, core/sigagg/sigagg.go:117).
//
// Items are partitioned into verification groups of partials over the same message (one
// validator's n partials in a slot).  A group of k usable items is checked with ONE pairing
// product through a random linear combination with secret 64-bit coefficients r_i:
//     e(sum_i r_i pk_i, H(m)) * e(-g1, sum_i r_i sig_i) == 1.
// If every item is valid the equation holds; if any item is invalid it fails except with
// probability <= 2^-64 over the choice of the r_i (each r_i is drawn from 2^64 distinct values mod
// r; the subgroup checks of decompression make the argument sound).  Every item of a failing
// group is then verified on its own (fallback), so per-item verdicts equal herumi's.
//
// r_i = a + b * lambda with 32-bit a, b (rlc.h: a 32-step joint ladder over the point and its
// endomorphism image instead of a 64-bit ladder).  The coefficients come from SHA-256(key || item), with the key
// drawn from the OS CSPRNG per call (hipbls.hip), so no party can predict them.
//
// Compiled like pipeline.hip (HB_FAST_FPMUL).
#define HB_FAST_FPMUL 1
#include "lines.h"
#include "rlc.h"

namespace hb {

#define KB __launch_bounds__(64)
constexpr int BLOCK = 64;

__device__ __forceinline__ uint32_t find_group_vb(const uint32_t* grp_off, uint32_t n_groups, uint32_t j) {
  uint32_t lo = 0, hi = n_groups;  // invariant: grp_off[lo] <= j < grp_off[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (grp_off[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// item -> verification group (grp_off nullable: every item its own group)
__global__ KB void k_item_group(const uint32_t* __restrict__ grp_off, uint32_t n_groups, uint32_t n,
                                uint32_t* __restrict__ item_grp) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  item_grp[i] = grp_off ? find_group_vb(grp_off, n_groups, i) : i;
}

// One lane per partial: decompress + subgroup-check the public key (herumi.go:290
// PublicKey.Deserialize).  A rejected key is replaced by g1 so later stages run the same
// arithmetic on well-formed values; its status byte decides the verdict.
__global__ KB_OCC(HB_OCC_DECPK) void k_dec_pk(const uint8_t* __restrict__ pks, uint32_t n, G1AEntry* __restrict__ out,
                            uint8_t* __restrict__ st) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A p;
  uint8_t bad = g1_decompress(p, pks + 48ull * i);
  if (bad) p = g1_generator();
  G1AEntry e;
  e.x = p.x;
  e.y = p.y;
  e.inf = p.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[i] = e;
  st[i] = bad;
}

// One lane per signature: decompress + subgroup-check (herumi.go:295 / :257 Sign.Deserialize),
// affine point + status (1 = undecodable or off the subgroup).  Serves the verification and,
// through index arrays, the ThresholdAggregate of the same partials.
__global__ KB_OCC(HB_OCC_DECSIG) void k_dec_sig_pt(const uint8_t* __restrict__ sigs, uint32_t n, HmEntry* __restrict__ out,
                                uint8_t* __restrict__ st) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2A q;
  uint8_t bad = g2_decompress(q, sigs + 96ull * i);
  if (bad) q = {f2_zero(), f2_zero(), true};
  HmEntry e;
  e.x = q.x;
  e.y = q.y;
  e.inf = q.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[i] = e;
  st[i] = bad;
}

// the random coefficient r = a + b lambda of entry `item` (SHA-256 of key || item, one block)
__device__ __forceinline__ void rlc_coeffs(const RlcKey& key, uint32_t item, uint32_t& a, uint32_t& b) {
  uint32_t w[16];
  HB_UNROLL for (int j = 0; j < 8; j++) w[j] = key.w[j];
  w[8] = item;
  w[9] = 0x80000000u;
  HB_UNROLL for (int j = 10; j < 15; j++) w[j] = 0;
  w[15] = 36 * 8;
  Sha256State st = sha256_init();
  sha256_compress(st, w);
  a = st.h[0];
  b = st.h[1];
  if ((a | b) == 0) a = 1;  // r != 0
}

__device__ __forceinline__ bool item_usable(const G1AEntry& p, uint8_t pst, const HmEntry& s, uint8_t sst) {
  return !pst && !sst && !p.inf && !s.inf;
}

// One lane per item (key_base + i is the item's index in the coefficient stream):
// P' = r pk, S' = r sig, written for every item so that the group sums need no branches: unusable
// items (undecodable, infinity) contribute the point at infinity, items of singleton groups keep
// r = 1 unless `always` (the folded aggregates).
__global__ KB_OCC(HB_OCC_RLC) void k_rlc(const G1AEntry* __restrict__ pk, const uint8_t* __restrict__ pk_st,
                         const HmEntry* __restrict__ sig, const uint8_t* __restrict__ sig_st,
                         const uint32_t* __restrict__ item_grp, const uint32_t* __restrict__ grp_off, int always,
                         uint32_t n, uint32_t key_base, RlcKey key, G1JEntry* __restrict__ pout,
                         G2JEntry* __restrict__ sout) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1AEntry pe = pk[i];
  const HmEntry se = sig[i];
  const G1A P = {pe.x, pe.y, false};
  const G2A S = {se.x, se.y, false};
  G1J rp;
  G2J rs;
  if (!item_usable(pe, pk_st[i], se, sig_st[i])) {
    rp = jac_infinity<Fp>();
    rs = jac_infinity<Fp2>();
  } else if (!always && (!grp_off || grp_off[item_grp[i] + 1] - grp_off[item_grp[i]] <= 1)) {
    rp = jac_from_aff(P);
    rs = jac_from_aff(S);
  } else {
    uint32_t a, b;
    rlc_coeffs(key, key_base + i, a, b);
    rp = rlc_g1(P, a, b);
    rs = rlc_g2(S, a, b);
  }
  pout[i] = {rp.X, rp.Y, rp.Z};
  sout[i] = {rs.X, rs.Y, rs.Z};
#endif
}

// One lane per item (then per folded aggregate): final status, or a place in the fallback list.
__global__ KB void k_scatter(ScatterArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < a.n) {
    const uint32_t i = t;
    uint8_t s;
    if (a.pk_st[i]) s = ST_BAD_PUBKEY;
    else if (a.sig_st[i]) s = ST_BAD_SIGNATURE;
    else if (a.pk[i].inf || a.sig[i].inf || a.hm[a.msg_idx[i]].h.inf) s = ST_NOT_VERIFIED;  // verify_core
    else if (a.gverdict[a.item_grp[i]] == 0) s = ST_OK;
    else {
      a.list[atomicAdd(a.count, 1u)] = i;
      return;
    }
    a.status[i] = s;
  } else if (t < a.n + a.n_agg) {
    const uint32_t v = t - a.n;
    uint8_t s;
    if (a.ta_status[v] != ST_OK) s = a.ta_status[v];  // no aggregate was produced
    else if (a.agg_pk_st[v]) s = ST_BAD_PUBKEY;
    else if (a.agg_pk[v].inf || a.agg_sig[v].inf) s = ST_NOT_VERIFIED;
    else if (a.gverdict[v] == 0) s = ST_OK;
    else {
      a.list[atomicAdd(a.count, 1u)] = t;
      return;
    }
    a.agg_status[v] = s;
  }
}

// Fallback: Miller lines at -g1 of the listed signatures, slot u = list position - base.
__global__ KB_OCC(HB_OCC_LINES) void k_fb_lines(const uint32_t* __restrict__ list, const uint32_t* __restrict__ count, uint32_t base,
                              uint32_t cap, const HmEntry* __restrict__ sig, const HmEntry* __restrict__ agg_sig,
                              uint32_t n_items, LineEntry* __restrict__ lines) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= cap || base + u >= *count) return;
  const uint32_t e = list[base + u];
  const G2A S = e < n_items ? hm_load(sig[e]) : hm_load(agg_sig[e - n_items]);
  line_chain<true>(S, lines + u, cap);
}

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

void launch_item_group(const uint32_t* grp_off, uint32_t n_groups, uint32_t n, uint32_t* item_grp, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_item_group, dim3(blocks_for(n)), dim3(BLOCK), 0, s, grp_off, n_groups, n, item_grp);
}
void launch_dec_pk(const uint8_t* pks, uint32_t n, G1AEntry* out, uint8_t* st, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_dec_pk, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pks, n, out, st);
}
void launch_dec_sig_pt(const uint8_t* sigs, uint32_t n, HmEntry* out, uint8_t* st, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_dec_sig_pt, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sigs, n, out, st);
}
void launch_rlc(const G1AEntry* pk, const uint8_t* pk_st, const HmEntry* sig, const uint8_t* sig_st,
                const uint32_t* item_grp, const uint32_t* grp_off, int always, uint32_t n, uint32_t key_base,
                const RlcKey& key, G1JEntry* pout, G2JEntry* sout, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_rlc, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pk, pk_st, sig, sig_st, item_grp, grp_off,
                       always, n, key_base, key, pout, sout);
}
void launch_scatter(const ScatterArgs& a, hipStream_t s) {
  const size_t tot = (size_t)a.n + a.n_agg;
  if (tot) hipLaunchKernelGGL(k_scatter, dim3(blocks_for(tot)), dim3(BLOCK), 0, s, a);
}
void launch_fb_lines(const uint32_t* list, const uint32_t* count, uint32_t base, uint32_t cap, const HmEntry* sig,
                     const HmEntry* agg_sig, uint32_t n_items, LineEntry* lines, hipStream_t s) {
  if (cap)
    hipLaunchKernelGGL(k_fb_lines, dim3(blocks_for(cap)), dim3(BLOCK), 0, s, list, count, base, cap, sig, agg_sig,
                       n_items, lines);
}

// ---------------------------------------------------------------------------------------
// FastAggregateVerify at scale (tbls.VerifyAggregate, herumi.go:318-342; the startup check of
// cluster/lock.go:185 runs it over every validator's every public share): the public keys of a
// group are summed by a segmented tree reduction -- pass 1 sums segments of affine decompressed
// keys, later passes sum segments of the previous pass's Jacobian partials -- so a group of 7M
// keys takes a few launches of many lanes instead of one lane walking 7M points.
// ---------------------------------------------------------------------------------------

// One lane per segment [seg_off[s], seg_off[s+1]): sum of the points, OR of the bad flags.
template <bool AFFINE>
__global__ KB void k_seg_sum(const void* __restrict__ pts, const uint8_t* __restrict__ st_in,
                             const uint32_t* __restrict__ seg_off, uint32_t n_seg, G1JEntry* __restrict__ out,
                             uint8_t* __restrict__ st_out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t sgi = blockIdx.x * blockDim.x + threadIdx.x;
  if (sgi >= n_seg) return;
  const uint32_t b = seg_off[sgi], e = seg_off[sgi + 1];
  G1J acc = jac_infinity<Fp>();
  uint8_t bad = 0;
  for (uint32_t i = b; i < e; i++) {
    bad |= st_in[i];
    if (AFFINE) {
      const G1AEntry q = reinterpret_cast<const G1AEntry*>(pts)[i];
      acc = jac_add_aff(acc, G1A{q.x, q.y, q.inf != 0});
    } else {
      const G1JEntry q = reinterpret_cast<const G1JEntry*>(pts)[i];
      acc = jac_add(acc, G1J{q.X, q.Y, q.Z});
    }
  }
  out[sgi] = {acc.X, acc.Y, acc.Z};
  st_out[sgi] = bad;
#endif
}

// One lane per group: the reduced key sum (nullable for empty groups) -> affine, for the pairing.
__global__ KB void k_va_point(const G1JEntry* __restrict__ sums, const uint32_t* __restrict__ sum_of_group,
                              uint32_t n_groups, G1AEntry* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  G1A a = {fp_zero(), fp_zero(), true};
  const uint32_t k = sum_of_group[g];
  if (k != 0xffffffffu) {
    const G1JEntry q = sums[k];
    a = jac_to_aff(G1J{q.X, q.Y, q.Z});
  }
  G1AEntry e;
  e.x = a.x;
  e.y = a.y;
  e.inf = a.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[g] = e;
}

// One lane per signature: its Miller lines evaluated at -g1 (lines[j * stride + i]).
__global__ KB_OCC(HB_OCC_LINES) void k_sig_lines(const HmEntry* __restrict__ sig, uint32_t n, LineEntry* __restrict__ lines,
                               uint32_t stride) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  line_chain<true>(hm_load(sig[i]), lines + i, stride);
}

// One lane per group: herumi's order of checks -- signature decoding, public key decoding, then
// the pairing verdict (pv) of the aggregated key.  An empty group, and an identity signature
// (verify_core, ops.h), never verify; the pairing kernel sees an identity key sum itself.
__global__ KB void k_va_status(const HmEntry* __restrict__ sig, const uint8_t* __restrict__ sig_st,
                               const uint8_t* __restrict__ key_bad, const uint32_t* __restrict__ sum_of_group,
                               const uint8_t* __restrict__ pv, uint32_t n_groups, uint8_t* __restrict__ status) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const uint32_t k = sum_of_group[g];
  uint8_t s;
  if (sig_st[g]) s = ST_BAD_SIGNATURE;
  else if (k != 0xffffffffu && key_bad[k]) s = ST_BAD_PUBKEY;
  else if (k == 0xffffffffu || sig[g].inf) s = ST_NOT_VERIFIED;
  else s = pv[g] == ST_OK ? ST_OK : ST_NOT_VERIFIED;
  status[g] = s;
}

void launch_seg_sum(bool affine, const void* pts, const uint8_t* st_in, const uint32_t* seg_off, uint32_t n_seg,
                    G1JEntry* out, uint8_t* st_out, hipStream_t s) {
  if (!n_seg) return;
  if (affine)
    hipLaunchKernelGGL(k_seg_sum<true>, dim3(blocks_for(n_seg)), dim3(BLOCK), 0, s, pts, st_in, seg_off, n_seg, out,
                       st_out);
  else
    hipLaunchKernelGGL(k_seg_sum<false>, dim3(blocks_for(n_seg)), dim3(BLOCK), 0, s, pts, st_in, seg_off, n_seg, out,
                       st_out);
}
void launch_va_point(const G1JEntry* sums, const uint32_t* sum_of_group, uint32_t n_groups, G1AEntry* out,
                     hipStream_t s) {
  if (n_groups)
    hipLaunchKernelGGL(k_va_point, dim3(blocks_for(n_groups)), dim3(BLOCK), 0, s, sums, sum_of_group, n_groups, out);
}
void launch_sig_lines(const HmEntry* sig, uint32_t n, LineEntry* lines, uint32_t stride, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_sig_lines, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sig, n, lines, stride);
}
void launch_va_status(const HmEntry* sig, const uint8_t* sig_st, const uint8_t* key_bad,
                      const uint32_t* sum_of_group, const uint8_t* pv, uint32_t n_groups, uint8_t* status,
                      hipStream_t s) {
  if (n_groups)
    hipLaunchKernelGGL(k_va_status, dim3(blocks_for(n_groups)), dim3(BLOCK), 0, s, sig, sig_st, key_bad,
                       sum_of_group, pv, n_groups, status);
}

}  // namespace hb
