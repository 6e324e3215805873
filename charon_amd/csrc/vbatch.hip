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
  uint8_t bad = g1_decompress(p, pks + 48ull * i, false);  // the subgroup check: k_g1_subgroup
  if (bad) p = g1_generator();
  G1AEntry e;
  e.x = p.x;
  e.y = p.y;
  e.inf = p.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[i] = e;
  st[i] = bad;
}

// The subgroup check of k_dec_pk's points, a kernel of its own like k_g2_subgroup (the fused
// kernel spilled the square root's window table beside the ladder).  The ladders run in lazily
// reduced 28-bit limbs (ec28.h g1_in_subgroup28 / g2_in_subgroup28_l).
__global__ KB_OCC(HB_OCC_SUBG) void k_g1_subgroup(uint32_t n, G1AEntry* __restrict__ pts, uint8_t* __restrict__ st) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1AEntry e = pts[i];
  if (st[i] || e.inf) return;
  if (!g1_in_subgroup28(G1A{e.x, e.y, false})) {
    const G1A g = g1_generator();
    G1AEntry z;
    z.x = g.x;
    z.y = g.y;
    z.inf = 0u;
    z.pad[0] = z.pad[1] = z.pad[2] = 0;
    pts[i] = z;
    st[i] = 1;
  }
}

// One lane per signature: decompress + subgroup-check (herumi.go:295 / :257 Sign.Deserialize),
// affine point + status (1 = undecodable or off the subgroup).  Serves the verification and,
// through index arrays, the ThresholdAggregate of the same partials.
// Two kernels: the square root (k_dec_sig_pt) and the subgroup check (k_g2_subgroup), so that
// neither holds the other's working set (one kernel spilled 4 KB per lane to scratch).
// skip (nullable): items already filled from the decompressed-signature cache (k_sc_get)
__global__ KB_OCC(HB_OCC_DECSIG) void k_dec_sig_pt(const uint8_t* __restrict__ sigs, uint32_t n, HmEntry* __restrict__ out,
                                uint8_t* __restrict__ st, const uint8_t* __restrict__ skip) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (skip && skip[i])) return;
  G2A q;
  uint8_t bad = g2_decompress(q, sigs + 96ull * i, false);
  if (bad) q = {f2_zero(), f2_zero(), true};
  HmEntry e;
  e.x = q.x;
  e.y = q.y;
  e.inf = q.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[i] = e;
  st[i] = bad;
}

__global__ KB_OCC(HB_OCC_SUBG) void k_g2_subgroup(uint32_t n, HmEntry* __restrict__ pts, uint8_t* __restrict__ st,
                                                   const uint8_t* __restrict__ skip) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (skip && skip[i])) return;
  const HmEntry e = pts[i];
  if (st[i] || e.inf) return;
  const HmEntry* src = pts + i;
  if (!g2_in_subgroup28_l([src]() { return G2A{src->x, src->y, false}; })) {
    HmEntry z;
    z.x = f2_zero();
    z.y = f2_zero();
    z.inf = 1u;
    z.pad[0] = z.pad[1] = z.pad[2] = 0;
    pts[i] = z;
    st[i] = 1;
  }
}

// The subgroup checks with each item's ladder split over a lane pair (ec28.h G1Half: each lane one
// of every pair of independent products; F2Half: each lane one coefficient of every Fp2 product),
// for calls with too few items to fill the chip, where the ladders' latency, not their
// lane-cycles, is what the slot waits for.  Same outputs as k_g1_subgroup / k_g2_subgroup.
__global__ KB_OCC(HB_OCC_SUBG) void k_g1_subgroup_h(uint32_t n, G1AEntry* __restrict__ pts, uint8_t* __restrict__ st) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (i >= n) return;  // both lanes of a pair
  const G1AEntry e = pts[i];
  if (st[i] || e.inf) return;
  const G1Half m = g1half_make();
  if (!g1_in_subgroup28(G1A{e.x, e.y, false}, m) && m.h == 0) {
    const G1A g = g1_generator();
    G1AEntry z;
    z.x = g.x;
    z.y = g.y;
    z.inf = 0u;
    z.pad[0] = z.pad[1] = z.pad[2] = 0;
    pts[i] = z;
    st[i] = 1;
  }
#endif
}
__global__ KB_OCC(HB_OCC_SUBG) void k_g2_subgroup_h(uint32_t n, HmEntry* __restrict__ pts, uint8_t* __restrict__ st,
                                                     const uint8_t* __restrict__ skip) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (i >= n || (skip && skip[i])) return;
  const HmEntry e = pts[i];
  if (st[i] || e.inf) return;
  const F2Half m = f2half_make();
  const HmEntry* src = pts + i;
  if (!g2_in_subgroup28_l([src]() { return G2A{src->x, src->y, false}; }, m) && m.h == 0) {
    HmEntry z;
    z.x = f2_zero();
    z.y = f2_zero();
    z.inf = 1u;
    z.pad[0] = z.pad[1] = z.pad[2] = 0;
    pts[i] = z;
    st[i] = 1;
  }
#endif
}

// items up to which the subgroup checks run on lane pairs (HBLS_DEC_PAIR_MAX at init,
// hbls_dec_pair_max at run time; 0 = never: measured neutral at C2, profiles/r05_scheduling_ab.txt)
std::atomic<size_t> g_dec_pair_max{0};
static size_t dec_pair_max() { return g_dec_pair_max.load(std::memory_order_relaxed); }

// ---- decompressed-signature cache (host-buffer calls: hbls_verify_batch fills it,
// hbls_threshold_aggregate_batch reads it -- charon's parsigex Verify -> parsigdb -> sigagg flow,
// where the aggregation's partials are exactly partials verified before).  A ring of `cap`
// entries (the compressed bytes, the decompressed point, its status) and an open-addressing index
// of 2 cap slots (entry + 1, 0 = empty) probed linearly from a keyed hash of the bytes, at most
// SC_PROBES slots.  Slots are never emptied: a slot whose entry was overwritten by the ring or no
// longer hashes within SC_PROBES of it is stale and may be taken.  A lookup compares all 96 bytes,
// so a stale or raced slot can only cause a miss (the partial is then decompressed), never a wrong
// point.  Puts and gets are ordered on the device by the host (one event per device).
constexpr uint32_t SC_PROBES = 16;
__device__ __forceinline__ uint32_t sc_hash(const uint4* k, uint64_t k0, uint64_t k1) {
  uint64_t h = k0;
  HB_UNROLL for (int j = 0; j < 6; j++) {
    const uint64_t v = ((uint64_t)k[j].y << 32 | k[j].x) ^ ((uint64_t)k[j].w << 32 | k[j].z) * 0x9e3779b97f4a7c15ull;
    h = (h ^ v) * 0xff51afd7ed558ccdull + k1;
    h ^= h >> 29;
  }
  h *= 0xc4ceb9fe1a85ec53ull;
  return (uint32_t)(h >> 32);
}
__device__ __forceinline__ bool sc_eq(const uint4* a, const uint4* b) {
  bool eq = true;
  HB_UNROLL for (int j = 0; j < 6; j++) eq = eq && a[j].x == b[j].x && a[j].y == b[j].y && a[j].z == b[j].z && a[j].w == b[j].w;
  return eq;
}
// entries (base + i) & (cap - 1) take item i: bytes, point, status (k_sc_write); then, once all of
// them are written, the index (k_sc_index).  An occupied slot is taken over only when its entry
// holds the same bytes (put again: the newer entry wins) or no longer hashes within SC_PROBES of
// the slot (its ring entry was rewritten with other bytes); an entry of this very put with other
// bytes is live.  (One kernel judging slots by "rewritten by this put" let lanes of one put evict
// each other: 4.5 % of a 1M-signature put went unindexed.)
__global__ __launch_bounds__(64) void k_sc_write(const uint8_t* __restrict__ sigs, const HmEntry* __restrict__ pts,
                                                 const uint8_t* __restrict__ st, uint32_t n, uint32_t base, uint32_t cap,
                                                 uint4* __restrict__ key, HmEntry* __restrict__ ent,
                                                 uint8_t* __restrict__ est) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = (base + i) & (cap - 1);
  HB_UNROLL for (int j = 0; j < 6; j++) key[6ull * e + j] = ((const uint4*)(sigs + 96ull * i))[j];
  ent[e] = pts[i];
  est[e] = st[i];
}
__global__ __launch_bounds__(64) void k_sc_index(uint32_t n, uint32_t base, uint32_t cap, const uint4* __restrict__ key,
                                                 uint32_t* __restrict__ tab, uint32_t tcap, uint64_t k0, uint64_t k1) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = (base + i) & (cap - 1);
  uint4 kb[6];
  HB_UNROLL for (int j = 0; j < 6; j++) kb[j] = key[6ull * e + j];
  const uint32_t home = sc_hash(kb, k0, k1) & (tcap - 1);
  for (uint32_t q = 0; q < SC_PROBES; q++) {
    const uint32_t slot = (home + q) & (tcap - 1);
    const uint32_t old = atomicCAS(&tab[slot], 0u, e + 1);
    if (old == 0 || old == e + 1) return;
    const uint4* ko = key + 6ull * (old - 1);
    const bool dead = sc_eq(ko, kb) || ((slot - (sc_hash(ko, k0, k1) & (tcap - 1))) & (tcap - 1)) >= SC_PROBES;
    if (dead && atomicCAS(&tab[slot], old, e + 1) == old) return;
  }
}
// one lane per signature: the cached point and status when its bytes are cached (hit = 1).
// Ring entries [busy_lo, busy_lo + busy_len) (mod cap) belong to puts that may still be writing
// them (sc_get): an index pointing there is a miss, whatever the bytes there say.
__global__ __launch_bounds__(64) void k_sc_get(const uint8_t* __restrict__ sigs, uint32_t n,
                                               const uint4* __restrict__ key, const HmEntry* __restrict__ ent,
                                               const uint8_t* __restrict__ est, const uint32_t* __restrict__ tab,
                                               uint32_t tcap, uint64_t k0, uint64_t k1, HmEntry* __restrict__ out,
                                               uint8_t* __restrict__ st, uint8_t* __restrict__ hit, uint32_t cap,
                                               uint32_t busy_lo, uint32_t busy_len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 kb[6];
  HB_UNROLL for (int j = 0; j < 6; j++) kb[j] = ((const uint4*)(sigs + 96ull * i))[j];
  const uint32_t home = sc_hash(kb, k0, k1) & (tcap - 1);
  uint8_t h = 0;
  for (uint32_t q = 0; q < SC_PROBES; q++) {
    const uint32_t v = tab[(home + q) & (tcap - 1)];
    if (v == 0) break;
    if (((v - 1 - busy_lo) & (cap - 1)) < busy_len) continue;
    if (sc_eq(key + 6ull * (v - 1), kb)) {
      out[i] = ent[v - 1];
      st[i] = est[v - 1];
      h = 1;
      break;
    }
  }
  hit[i] = h;
}

// ---- public-key cache on the device (hbls_pubkey_cache_add): the compressed keys of the table's
// entries and an open-addressing index of them (entry + 1, 0 = empty; SC_PROBES slots from a keyed
// hash of the 48 bytes), so a host-buffer verification finds its keys on the device instead of
// looking each one up on the host (1 M host lookups cost ~0.3 s).  Entries are only added (and the
// whole table dropped by hbls_pubkey_cache_clear), so no slot is ever stale.
__device__ __forceinline__ uint32_t kc_hash(const uint4* k, uint64_t k0, uint64_t k1) {
  uint64_t h = k1;
  HB_UNROLL for (int j = 0; j < 3; j++) {
    const uint64_t v = ((uint64_t)k[j].y << 32 | k[j].x) ^ ((uint64_t)k[j].w << 32 | k[j].z) * 0x9e3779b97f4a7c15ull;
    h = (h ^ v) * 0xff51afd7ed558ccdull + k0;
    h ^= h >> 29;
  }
  h *= 0xc4ceb9fe1a85ec53ull;
  return (uint32_t)(h >> 32);
}
__device__ __forceinline__ void kc_key_load(const uint8_t* p, uint4* k) {
  HB_UNROLL for (int j = 0; j < 3; j++) k[j] = ((const uint4*)p)[j];
}
// entries first .. first + m - 1 (keys already at keys[48 e]) into the index
__global__ __launch_bounds__(64) void k_kc_index(const uint8_t* __restrict__ keys, uint32_t first, uint32_t m,
                                                 uint32_t* __restrict__ tab, uint32_t tcap, uint64_t k0, uint64_t k1) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t e = first + i;
  uint4 kb[3];
  kc_key_load(keys + 48ull * e, kb);
  const uint32_t home = kc_hash(kb, k0, k1) & (tcap - 1);
  for (uint32_t q = 0; q < tcap; q++)  // load factor <= 1/2: a free slot exists
    if (atomicCAS(&tab[(home + q) & (tcap - 1)], 0u, e + 1) == 0u) return;
}
// One lane per public key: the cached entry when its 48 bytes are in the index, else decompressed
// here like k_dec_pk (+ the subgroup check)
__global__ KB_OCC(HB_OCC_DECPK) void k_pk_cached(const uint8_t* __restrict__ pks, uint32_t n,
                                                 const uint8_t* __restrict__ keys, const G1AEntry* __restrict__ tabe,
                                                 const uint8_t* __restrict__ tst, const uint32_t* __restrict__ tab,
                                                 uint32_t tcap, uint64_t k0, uint64_t k1, G1AEntry* __restrict__ out,
                                                 uint8_t* __restrict__ st) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 kb[3];
  kc_key_load(pks + 48ull * i, kb);
  const uint32_t home = kc_hash(kb, k0, k1) & (tcap - 1);
  for (uint32_t q = 0; q < tcap; q++) {
    const uint32_t v = tab[(home + q) & (tcap - 1)];
    if (v == 0) break;
    uint4 ke[3];
    kc_key_load(keys + 48ull * (v - 1), ke);
    bool eq = true;
    HB_UNROLL for (int j = 0; j < 3; j++)
      eq = eq && ke[j].x == kb[j].x && ke[j].y == kb[j].y && ke[j].z == kb[j].z && ke[j].w == kb[j].w;
    if (eq) {
      out[i] = tabe[v - 1];
      st[i] = tst[v - 1];
      return;
    }
  }
  G1A p;
  uint8_t bad = g1_decompress(p, pks + 48ull * i);
  if (bad) p = {fp_zero(), fp_zero(), true};
  G1AEntry e;
  e.x = p.x;
  e.y = p.y;
  e.inf = p.inf ? 1u : 0u;
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

// the sparse-format digits of entry `item` (ec28.h RLC_DIGITS: 66 random bits of the same hash
// block, 10 three-bit digits per word), word 3 = 1 (usable)
__device__ __forceinline__ uint4 rlc_digits(const RlcKey& key, uint32_t item) {
  uint32_t w[16];
  HB_UNROLL for (int j = 0; j < 8; j++) w[j] = key.w[j];
  w[8] = item;
  w[9] = 0x80000000u;
  HB_UNROLL for (int j = 10; j < 15; j++) w[j] = 0;
  w[15] = 36 * 8;
  Sha256State st = sha256_init();
  sha256_compress(st, w);
  return make_uint4(st.h[0] & 0x3fffffffu, st.h[1] & 0x3fffffffu, st.h[2] & 0x3fu, 1u);
}

__device__ __forceinline__ bool item_usable(const G1AEntry& p, uint8_t pst, const HmEntry& s, uint8_t sst) {
  return !pst && !sst && !p.inf && !s.inf;
}

// One lane per item (key_base + i is the item's index in the coefficient stream):
// P' = r pk, S' = r sig, written for every item so that the group sums need no branches: unusable
// items (undecodable, infinity) contribute the point at infinity, items of singleton groups keep
// r = 1 unless `always` (the folded aggregates).  coef (nullable): the item's (a, b), (0, 0) when
// unusable; sides 1 computes P' only and writes coef, sides 2 computes S' only from coef.  sig and
// sig_st null (sides 1 only): usability by the key alone, the signature's applied by the consumer.
template <int sides>
__global__ KB_OCC(HB_OCC_RLC) void k_rlc(const G1AEntry* __restrict__ pk, const uint8_t* __restrict__ pk_st,
                         const HmEntry* __restrict__ sig, const uint8_t* __restrict__ sig_st,
                         const uint32_t* __restrict__ item_grp, const uint32_t* __restrict__ grp_off, int always,
                         uint32_t n, uint32_t key_base, RlcKey key, G1JEntry* __restrict__ pout,
                         G2JEntry* __restrict__ sout, uint2* __restrict__ coef, const uint8_t* __restrict__ guard) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (guard && *guard == 0) return;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1AEntry pe = pk[i];
  const HmEntry se = sig ? sig[i] : HmEntry{};
  const G1A P = {pe.x, pe.y, false};
  const G2A S = {se.x, se.y, false};
  G1J rp;
  G2J rs;
  uint32_t a = 0, b = 0;
  if (sig ? !item_usable(pe, pk_st[i], se, sig_st[i]) : (pk_st[i] || pe.inf)) {
    rp = jac_infinity<Fp>();
    rs = jac_infinity<Fp2>();
  } else if (!always && (!grp_off || grp_off[item_grp[i] + 1] - grp_off[item_grp[i]] <= 1)) {
    a = 1;
    rp = jac_from_aff(P);
    rs = jac_from_aff(S);
  } else {
    if (sides == 2) {
      const uint2 ab = coef[i];
      a = ab.x;
      b = ab.y;
    } else {
      rlc_coeffs(key, key_base + i, a, b);
    }
    if (sides & 1) rp = rlc_g1(P, a, b);
    if (sides & 2) rs = rlc_g2(S, a, b);
  }
  if (sides & 1) pout[i] = {rp.X, rp.Y, rp.Z};
  if (sides & 2) sout[i] = {rs.X, rs.Y, rs.Z};
  if (coef && sides != 2) coef[i] = make_uint2(a, b);
#endif
}

// ---------------------------------------------------------------------------------------
// Chunk plans: the items of every group [grp_off[g], grp_off[g+1]) cut into ceil(size / cmax)
// nearly equal chunks of consecutive items (group g's chunks are coff[g] .. coff[g+1]-1; chunk c covers
// cfirst[c] .. cfirst[c] + (ccount[c] & 0x7fffffff) - 1; bit 31 of ccount marks a group of ONE
// item).  A chunk is one lane of the multi-scalar kernels below, which share the doublings of a
// ladder over the chunk's items.
// ---------------------------------------------------------------------------------------
__global__ KB void k_plan_count(const uint32_t* __restrict__ grp_off, uint32_t ng, uint32_t cmax,
                                uint32_t* __restrict__ cnt) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  cnt[g] = (grp_off[g + 1] - grp_off[g] + cmax - 1) / cmax;
}

// one workgroup: exclusive scan of cnt[0..ng) into coff[0..ng], coff[ng] = total
__global__ __launch_bounds__(1024) void k_plan_scan(const uint32_t* __restrict__ cnt, uint32_t ng,
                                                    uint32_t* __restrict__ coff) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x, per = (ng + 1023u) / 1024u;
  const uint32_t b = t * per < ng ? t * per : ng, e = b + per < ng ? b + per : ng;
  uint32_t sum = 0;
  for (uint32_t i = b; i < e; i++) sum += cnt[i];
  part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 1024u; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t i = b; i < e; i++) {
    coff[i] = run;
    run += cnt[i];
  }
  if (t == 1023u) coff[ng] = part[1023];
}

__global__ KB void k_plan_fill(const uint32_t* __restrict__ grp_off, uint32_t ng, uint32_t cmax,
                               const uint32_t* __restrict__ coff, uint32_t* __restrict__ cfirst,
                               uint32_t* __restrict__ ccount) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  // the group's items split into nc nearly equal chunks (a wave's lanes then run equal loops)
  const uint32_t b = grp_off[g], sz = grp_off[g + 1] - b, c0 = coff[g], nc = coff[g + 1] - c0;
  for (uint32_t k = 0; k < nc; k++) {
    const uint32_t lo = (uint32_t)((uint64_t)k * sz / nc), hi = (uint32_t)((uint64_t)(k + 1) * sz / nc);
    cfirst[c0 + k] = b + lo;
    ccount[c0 + k] = (hi - lo) | (sz == 1 ? 0x80000000u : 0u);
  }
}

// One lane per chunk of a verification group: sum_i [r_i] pk_i and sum_i [r_i] sig_i over the
// chunk's items with r_i = a_i + b_i lambda (rlc.h), as ONE joint 32-step ladder per side whose
// doublings all items share (32 doublings + 32 additions per item before: 32 doublings per chunk
// + 32 additions per item now).  Each item's three ladder points {T1, phi(T1), T1 + phi(T1)} go to
// the workspace as Jacobian records and are read back by the step's selection; unusable items
// contribute nothing; a group of one item keeps r = 1.  The chunk's sum is written at its first
// item, infinity at the others, so k_group_prep sums the items as before.
// AFF: the ladder points are affine (Z = 1 in the records): mixed additions
template <class F, bool AFF = false>
__device__ __forceinline__ Jac<F> msm_ladder(const Jac<F>* __restrict__ tab, const uint2* __restrict__ coef,
                                             uint32_t first, uint32_t cnt) {
  Jac<F> R = jac_infinity<F>();
  HB_NOUNROLL for (int bit = 31; bit >= 0; bit--) {
    R = jac_dbl(R);
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const uint2 ab = coef[i];
      const uint32_t sel = ((ab.x >> bit) & 1u) | (((ab.y >> bit) & 1u) << 1);
      const Jac<F> T = tab[3ull * i + (sel ? sel - 1u : 0u)];
      const Jac<F> S = AFF ? jac_add_aff(R, Aff<F>{T.X, T.Y, false}) : jac_add(R, T);
      R = jac_select(sel != 0, R, S);
    }
  }
  return R;
}

// the stored-word twin of ec28.h g1l/g2l_msm_ladder_sparse (HB_G1_LAZY=0 / HB_G2_LAZY=0 builds)
template <class F>
__device__ __forceinline__ Jac<F> msm_ladder_sparse(const Jac<F>* __restrict__ tab, const uint4* __restrict__ coef4,
                                                    uint32_t first, uint32_t cnt) {
  Jac<F> R = jac_infinity<F>();
  HB_NOUNROLL for (int j = RLC_DIGITS - 1; j >= 0; j--) {
    if (j != RLC_DIGITS - 1) R = jac_dbl(jac_dbl(R));
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const uint4 c = coef4[i];
      if (!c.w) continue;
      const uint32_t d = rlc_digit(c, j);
      const Jac<F> T = tab[4ull * i + (d & 3u)];
      R = jac_add_aff(R, Aff<F>{T.X, (d & 4u) ? f_neg(T.Y) : T.Y, false});
    }
  }
  return R;
}

// The pieces of the chunk kernels, split: one kernel builds the coefficients and ladder tables,
// then one kernel per side runs the ladder -- each kernel holds only its own phase's state (a fused
// kernel spilled 1.6 KB per lane: the SHA schedule, the inversion and both ladders in one register
// allocation; time-neutral, profiles/r04s_rlc_split_ab.txt).

// a group of ONE item keeps r = 1 (unless `always`): its records written here; true if so
template <int SIDES>
__device__ __forceinline__ bool rlc_single(const RlcMsmArgs& a, uint32_t first, uint32_t cc, bool write) {
  if (!((cc & 0x80000000u) != 0 && !a.always)) return false;
  if (!write) return true;
  const uint32_t i = first;
  const bool usable = !a.pk_st[i] && !a.sig_st[i] && !a.pk[i].inf && !a.sig[i].inf;
  const G1AEntry pe = a.pk[i];
  if (SIDES & 1) {
    const G1J rp = usable ? jac_from_aff(G1A{pe.x, pe.y, false}) : jac_infinity<Fp>();
    a.pout[i] = {rp.X, rp.Y, rp.Z};
    a.coef[i] = make_uint2(usable ? 1u : 0u, 0u);
  }
  if (SIDES & 2) {
    const HmEntry se = a.sig[i];
    const G2J rs = usable ? jac_from_aff(G2A{se.x, se.y, false}) : jac_infinity<Fp2>();
    a.sout[i] = {rs.X, rs.Y, rs.Z};
  }
  return true;
}

// coefficients and the G1 ladder points of a chunk's items: P, phi(P), P + phi(P) (dense) or
// P, phi(P), P + phi(P), P - phi(P) (sparse), affine with ONE inversion per chunk (Montgomery's
// trick), so the ladder adds affine points (7M + 4S instead of 11M + 5S)
__device__ __forceinline__ void rlc_tab_g1(const RlcMsmArgs& a, uint32_t first, uint32_t cnt) {
  Fp acc = fp_one();
  if (a.sparse) {
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const bool usable = !a.pk_st[i] && !a.sig_st[i] && !a.pk[i].inf && !a.sig[i].inf;
      a.coef4[i] = usable ? rlc_digits(a.key, a.key_base + i) : make_uint4(0u, 0u, 0u, 0u);
      const G1AEntry pe = a.pk[i];
      const G1A P = {pe.x, pe.y, false};
      acc = sparse_put(a.t1, i, P, G1A{fp_mul(P.x, fp_from_const(G1_BETA)), P.y, false}, acc);
    }
    Fp inv = fp_inv(acc);
    HB_NOUNROLL for (int k = (int)cnt - 1; k >= 0; k--) inv = sparse_fix(a.t1, first + (uint32_t)k, inv);
    return;
  }
  HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
    const uint32_t i = first + k;
    const bool usable = !a.pk_st[i] && !a.sig_st[i] && !a.pk[i].inf && !a.sig[i].inf;
    uint32_t ca = 0, cb = 0;
    if (usable) rlc_coeffs(a.key, a.key_base + i, ca, cb);
    a.coef[i] = make_uint2(ca, cb);
    const G1AEntry pe = a.pk[i];
    const G1A P = {pe.x, pe.y, false};
    const G1A P2 = {fp_mul(P.x, fp_from_const(G1_BETA)), P.y, false};
    const G1J J1 = jac_from_aff(P), J2 = jac_from_aff(P2);
    G1J J3 = jac_add_aff(J1, P2);
    if (fp_is_zero(J3.Z)) J3.Z = fp_one();  // never for a point of G1; keeps the product invertible
    a.t1[3ull * i] = {J1.X, J1.Y, acc};     // the running product of the Z before this item
    a.t1[3ull * i + 1] = J2;
    a.t1[3ull * i + 2] = J3;
    acc = fp_mul(acc, J3.Z);
  }
  Fp inv = fp_inv(acc);
  HB_NOUNROLL for (int k = (int)cnt - 1; k >= 0; k--) {
    const uint32_t i = first + (uint32_t)k;
    const G1J J3 = a.t1[3ull * i + 2];
    G1J J1 = a.t1[3ull * i];
    const Fp zi = fp_mul(inv, J1.Z);
    inv = fp_mul(inv, J3.Z);
    const Fp zi2 = fp_sqr(zi);
    J1.Z = fp_one();
    a.t1[3ull * i] = J1;
    a.t1[3ull * i + 2] = {fp_mul(J3.X, zi2), fp_mul(J3.Y, fp_mul(zi2, zi)), fp_one()};
  }
}

// the G2 ladder points: S, -psi^2(S), their sum (and difference when sparse), affine likewise
__device__ __forceinline__ void rlc_tab_g2(const RlcMsmArgs& a, uint32_t first, uint32_t cnt) {
  Fp2 acc2 = f2_one();
  if (a.sparse) {
    HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
      const uint32_t i = first + k;
      const HmEntry se = a.sig[i];
      const G2A S = {se.x, se.y, false};
      const G2A S2 = {f2_mul(S.x, f2_from_const(PSI2_CX)), f2_neg(f2_mul(S.y, f2_from_const(PSI2_CY))), false};
      acc2 = sparse_put(a.t2, i, S, S2, acc2);
    }
    Fp2 inv2 = f2_inv(acc2);
    HB_NOUNROLL for (int k = (int)cnt - 1; k >= 0; k--) inv2 = sparse_fix(a.t2, first + (uint32_t)k, inv2);
    return;
  }
  HB_NOUNROLL for (uint32_t k = 0; k < cnt; k++) {
    const uint32_t i = first + k;
    const HmEntry se = a.sig[i];
    const G2A S = {se.x, se.y, false};
    const G2A S2 = {f2_mul(S.x, f2_from_const(PSI2_CX)), f2_neg(f2_mul(S.y, f2_from_const(PSI2_CY))), false};
    const G2J J1 = jac_from_aff(S), J2 = jac_from_aff(S2);
    G2J J3 = jac_add_aff(J1, S2);
    if (f2_is_zero(J3.Z)) J3.Z = f2_one();  // an unusable item's placeholder: keeps the product invertible
    a.t2[3ull * i] = {J1.X, J1.Y, acc2};     // the running product of the Z before this item
    a.t2[3ull * i + 1] = J2;
    a.t2[3ull * i + 2] = J3;
    acc2 = f2_mul(acc2, J3.Z);
  }
  Fp2 inv2 = f2_inv(acc2);
  HB_NOUNROLL for (int k = (int)cnt - 1; k >= 0; k--) {
    const uint32_t i = first + (uint32_t)k;
    const G2J J3 = a.t2[3ull * i + 2];
    G2J J1 = a.t2[3ull * i];
    const Fp2 zi = f2_mul(inv2, J1.Z);
    inv2 = f2_mul(inv2, J3.Z);
    const Fp2 zi2 = f2_sqr(zi);
    J1.Z = f2_one();
    a.t2[3ull * i] = J1;
    a.t2[3ull * i + 2] = {f2_mul(J3.X, zi2), f2_mul(J3.Y, f2_mul(zi2, zi)), f2_one()};
  }
}

// the chunk's sums (ec28.h ladders; coefficients from the workspace) at its first item, infinity
// at the others, so k_group_prep sums the items as before
__device__ __forceinline__ void rlc_lad_g1(const RlcMsmArgs& a, uint32_t first, uint32_t cnt) {
  const G1J rp = a.sparse ? g1l_msm_ladder_sparse(a.t1, a.coef4, first, cnt) : g1l_msm_ladder(a.t1, a.coef, first, cnt);
  a.pout[first] = {rp.X, rp.Y, rp.Z};
  const G1J zi = jac_infinity<Fp>();
  for (uint32_t k = 1; k < cnt; k++) a.pout[first + k] = {zi.X, zi.Y, zi.Z};
}
__device__ __forceinline__ void rlc_lad_g2(const RlcMsmArgs& a, uint32_t first, uint32_t cnt) {
  const G2J rs = a.sparse ? g2l_msm_ladder_sparse(a.t2, a.coef4, first, cnt) : g2l_msm_ladder(a.t2, a.coef, first, cnt);
  a.sout[first] = {rs.X, rs.Y, rs.Z};
  const G2J zs = jac_infinity<Fp2>();
  for (uint32_t k = 1; k < cnt; k++) a.sout[first + k] = {zs.X, zs.Y, zs.Z};
}

// One lane per chunk.  PHASE 1: coefficients and tables of SIDES; 2: the ladder of side SIDES (1
// or 2).  SIDES as RlcMsmArgs::sides, a template argument so that the public-key-only launch of
// the slot-wide check does not allocate registers for the G2 side.
template <int SIDES, int PHASE>
__global__ KB_OCC(HB_OCC_RLC) void k_rlc_msm(RlcMsmArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (a.guard && *a.guard == 0) return;
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= *a.total) return;
  const uint32_t first = a.cfirst[c], cc = a.ccount[c], cnt = cc & 0x7fffffffu;
  if (rlc_single<SIDES>(a, first, cc, PHASE != 2)) return;
  if (PHASE == 2) {
    if (SIDES == 1) rlc_lad_g1(a, first, cnt);
    else rlc_lad_g2(a, first, cnt);
    return;
  }
  if (SIDES & 1) rlc_tab_g1(a, first, cnt);
  if (SIDES & 2) rlc_tab_g2(a, first, cnt);
#endif
}

void launch_plan(const uint32_t* grp_off, uint32_t ng, uint32_t cmax, uint32_t* cnt, uint32_t* coff,
                 uint32_t* cfirst, uint32_t* ccount, hipStream_t s) {
  if (!ng) return;
  const unsigned nb = (ng + BLOCK - 1) / BLOCK;
  hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(BLOCK), 0, s, grp_off, ng, cmax, cnt);
  hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, s, cnt, ng, coff);
  hipLaunchKernelGGL(k_plan_fill, dim3(nb), dim3(BLOCK), 0, s, grp_off, ng, cmax, coff, cfirst, ccount);
}
void launch_scan(const uint32_t* cnt, uint32_t n, uint32_t* off, hipStream_t s) {
  hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, s, cnt, n, off);
}
void launch_rlc_msm(const RlcMsmArgs& a, uint32_t max_chunks, hipStream_t s) {
  if (!max_chunks) return;
  const dim3 grid((max_chunks + BLOCK - 1) / BLOCK);
  if (a.sides == 1) hipLaunchKernelGGL((k_rlc_msm<1, 1>), grid, dim3(BLOCK), 0, s, a);
  else if (a.sides == 2) hipLaunchKernelGGL((k_rlc_msm<2, 1>), grid, dim3(BLOCK), 0, s, a);
  else hipLaunchKernelGGL((k_rlc_msm<3, 1>), grid, dim3(BLOCK), 0, s, a);
  if (a.sides & 1) hipLaunchKernelGGL((k_rlc_msm<1, 2>), grid, dim3(BLOCK), 0, s, a);
  if (a.sides & 2) hipLaunchKernelGGL((k_rlc_msm<2, 2>), grid, dim3(BLOCK), 0, s, a);
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
    else if (a.gverdict[a.item_grp[i]] == GV_PASS) s = ST_OK;
    else if (a.first_group && (a.gverdict[a.item_grp[i]] == GV_UNCHECKED ||
                               (gv_failed(a.gverdict[a.item_grp[i]]) && a.item_grp[i] != *a.first_group)))
      s = ST_UNCHECKED;  // first-error mode: after the first failing group, not resolved
    else if (!a.n_agg && (!a.grp_off || a.grp_off[a.item_grp[i] + 1] - a.grp_off[a.item_grp[i]] <= 1))
      s = ST_NOT_VERIFIED;  // a group of one item (with a folded aggregate it has a second member)
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
  line_chain_ld<true>(e < n_items ? sig + e : agg_sig + (e - n_items), lines + u, cap);
}

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

void launch_item_group(const uint32_t* grp_off, uint32_t n_groups, uint32_t n, uint32_t* item_grp, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_item_group, dim3(blocks_for(n)), dim3(BLOCK), 0, s, grp_off, n_groups, n, item_grp);
}
void launch_dec_pk(const uint8_t* pks, uint32_t n, G1AEntry* out, uint8_t* st, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_dec_pk, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pks, n, out, st);
  if (n <= dec_pair_max())
    hipLaunchKernelGGL(k_g1_subgroup_h, dim3(blocks_for(2 * n)), dim3(BLOCK), 0, s, n, out, st);
  else
    hipLaunchKernelGGL(k_g1_subgroup, dim3(blocks_for(n)), dim3(BLOCK), 0, s, n, out, st);
}
void launch_kc_index(const uint8_t* keys, uint32_t first, uint32_t m, uint32_t* tab, uint32_t tcap, uint64_t k0,
                     uint64_t k1, hipStream_t s) {
  if (m) hipLaunchKernelGGL(k_kc_index, dim3(blocks_for(m)), dim3(BLOCK), 0, s, keys, first, m, tab, tcap, k0, k1);
}
void launch_pk_cached(const uint8_t* pks, uint32_t n, const uint8_t* keys, const G1AEntry* tabe, const uint8_t* tst,
                      const uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1, G1AEntry* out, uint8_t* st,
                      hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_pk_cached, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pks, n, keys, tabe, tst, tab, tcap, k0, k1,
                       out, st);
}
void launch_dec_sig_pt(const uint8_t* sigs, uint32_t n, HmEntry* out, uint8_t* st, hipStream_t s, const uint8_t* skip,
                       hipEvent_t decoded) {
  if (!n) {
    if (decoded) (void)hipEventRecord(decoded, s);
    return;
  }
  hipLaunchKernelGGL(k_dec_sig_pt, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sigs, n, out, st, skip);
  if (decoded) (void)hipEventRecord(decoded, s);
  if (n <= dec_pair_max())
    hipLaunchKernelGGL(k_g2_subgroup_h, dim3(blocks_for(2 * n)), dim3(BLOCK), 0, s, n, out, st, skip);
  else
    hipLaunchKernelGGL(k_g2_subgroup, dim3(blocks_for(n)), dim3(BLOCK), 0, s, n, out, st, skip);
}
void launch_sc_put(const uint8_t* sigs, const HmEntry* pts, const uint8_t* st, uint32_t n, uint32_t base, uint32_t cap,
                   void* key, HmEntry* ent, uint8_t* est, uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1,
                   hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sc_write, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sigs, pts, st, n, base, cap, (uint4*)key, ent,
                     est);
  hipLaunchKernelGGL(k_sc_index, dim3(blocks_for(n)), dim3(BLOCK), 0, s, n, base, cap, (const uint4*)key, tab, tcap, k0, k1);
}
void launch_sc_get(const uint8_t* sigs, uint32_t n, const void* key, const HmEntry* ent, const uint8_t* est,
                   const uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1, HmEntry* out, uint8_t* st, uint8_t* hit,
                   uint32_t cap, uint32_t busy_lo, uint32_t busy_len, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sc_get, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sigs, n, (const uint4*)key, ent, est, tab, tcap,
                     k0, k1, out, st, hit, cap, busy_lo, busy_len);
}
void launch_rlc(const G1AEntry* pk, const uint8_t* pk_st, const HmEntry* sig, const uint8_t* sig_st,
                const uint32_t* item_grp, const uint32_t* grp_off, int always, uint32_t n, uint32_t key_base,
                const RlcKey& key, G1JEntry* pout, G2JEntry* sout, hipStream_t s, uint2* coef, int sides,
                const uint8_t* guard) {
  if (!n) return;
  if (sides == 1)
    hipLaunchKernelGGL(k_rlc<1>, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pk, pk_st, sig, sig_st, item_grp, grp_off,
                       always, n, key_base, key, pout, sout, coef, guard);
  else if (sides == 2)
    hipLaunchKernelGGL(k_rlc<2>, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pk, pk_st, sig, sig_st, item_grp, grp_off,
                       always, n, key_base, key, pout, sout, coef, guard);
  else
    hipLaunchKernelGGL(k_rlc<3>, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pk, pk_st, sig, sig_st, item_grp, grp_off,
                       always, n, key_base, key, pout, sout, coef, guard);
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
  line_chain_ld<true>(sig + i, lines + i, stride);
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
