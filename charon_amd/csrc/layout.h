// Device-side storage formats and kernel launchers shared by the translation units of
// libhipbls.so (hipbls.hip: host runtime + one-lane kernels; pipeline.hip: hashing and the
// pairing kernel; vbatch.hip: batched verification; threshold.hip: ThresholdAggregate).
#pragma once
#include <atomic>
#include "ops.h"
#include "ta_small.h"

// Occupancy targets (waves per SIMD) of the heavy kernels: 1 lets the compiler use all 512
// registers of a lane, 2 gives each wave 256, 3 gives 168 (spilling the rest to scratch).  Chosen
// per kernel by measurement (DESIGN.md §4 "Occupancy"; the alternatives measured slower).
#define HB_OCC_HASH 2
#define HB_OCC_LINES 1
#define HB_OCC_DECPK 2
#define HB_OCC_DECSIG 2
#define HB_OCC_SUBG 2  // k_g1_subgroup, k_g2_subgroup
#define HB_OCC_RLC 2
#define HB_OCC_PREP 2
#define HB_OCC_PAIR3 1
#define HB_OCC_STRAUS 2
#define KB_OCC(n) __launch_bounds__(64, n)

namespace hb {

struct HmEntry {  // affine G2 point (Montgomery limbs) + infinity flag
  Fp2 x, y;
  uint32_t inf;
  uint32_t pad[3];
};

struct G2JEntry {  // Jacobian G2 point
  Fp2 X, Y, Z;
};

struct G1AEntry {  // affine G1 point
  Fp x, y;
  uint32_t inf;
  uint32_t pad[3];
};

struct G1JEntry {  // Jacobian G1 point
  Fp X, Y, Z;
};

struct LineEntry {  // one Miller-loop line: (a0, c1, c2) unevaluated or (a0, a1, b1)
  Fp2 a0, a1, b1;
};

struct Fp4Entry {  // one lane's third of an Fp12 value in the lane-group form of pair3.h
  Fp2 x, y;
};

// Per distinct message: H(m) and the 68 unevaluated lines of its Miller chain (pairing.h
// miller_dbl_c / miller_add_c), shared by every partial signed over that message.
struct MsgEntry {
  HmEntry h;
  LineEntry lines[N_LINES];
};

__device__ __forceinline__ G2A hm_load(const HmEntry& e) { return {e.x, e.y, e.inf != 0}; }
__device__ __forceinline__ G1A g1a_load(const G1AEntry& e) { return {e.x, e.y, e.inf != 0}; }

// ThresholdAggregate member status flags (threshold.hip -> k_group_sum)
enum : uint8_t { M_OK = 0, M_BAD_SIG = 1, M_BAD_IDX = 2 };

// base-|x| digits of a Lagrange coefficient (threshold.hip)
struct TaDigits {
  uint64_t a[4];
};

// Verification group state (vbatch.hip): READY groups go through the pairing kernel; EMPTY
// groups have no item left to check; FALLBACK groups send every usable item to the per-item
// path (inconsistent messages inside the group, or a degenerate combination).
enum : uint8_t { G_READY = 0, G_FALLBACK = 1, G_EMPTY = 2 };

// Key of the random linear combination (32 bytes drawn from the OS CSPRNG per call).
struct RlcKey {
  uint32_t w[8];
};

// Staged ThresholdAggregate (threshold.hip).  src (nullable): member j's point is pts[src[j]].
// nonuni (nullable, zeroed by the caller): set when t_u != 0 and some group does not hold exactly
// t_u members at offset g t_u -- the joint and small-scalar paths then stand down (nonuni below)
// and the per-member ladders run instead.  launch_ta_layout sets it alone (one lane per group);
// k_ta_lambda sets it too.  skip (nullable, per group): groups the small-scalar path aggregated --
// their lambda digits are not needed and not computed.
void launch_ta_layout(const uint32_t* grp_off, uint32_t n_groups, uint32_t t_u, uint8_t* nonuni, hipStream_t s);
void launch_ta_lambda(const int64_t* idx, const uint32_t* grp_off, uint32_t n_groups, uint32_t n_partials, int mode,
                      TaDigits* dig, uint8_t* mstat, hipStream_t s, uint32_t t_u = 0, uint8_t* nonuni = nullptr,
                      const uint8_t* skip = nullptr);
size_t ta_table_bytes(uint32_t n_partials);
// guard (nullable): nothing unless *guard != 0 (then one lane per member in plain order, skip unused)
void launch_ta_straus(const HmEntry* pts, const uint32_t* src, const TaDigits* dig, uint32_t n_partials,
                      uint32_t n_groups, void* tab, G2JEntry* out, hipStream_t s, const uint8_t* skip = nullptr,
                      const uint8_t* guard = nullptr);
// joint ladders over chunks of c (<= 8) members of a validator, every group of exactly t members
// (threshold.hip k_ta_jtab, k_ta_jladder, k_ta_jgeneral); table workspace of ta_joint_table_bytes
size_t ta_joint_table_bytes(uint32_t n_groups, uint32_t t, uint32_t c);
void launch_ta_joint(const HmEntry* pts, const uint32_t* src, const TaDigits* dig, uint32_t n_groups, uint32_t t,
                     uint32_t c, void* tab, G2JEntry* out, hipStream_t s, const uint8_t* skip = nullptr,
                     const uint8_t* nonuni = nullptr);
// small-scalar aggregation (threshold.hip k_ta_sprep / k_ta_small / k_ta_sladder, ta_small.h): groups
// of exactly t members (idx: their share indices); done[g] != 0 for the groups it aggregated (their
// sums at out[g t], infinity at the other members), the rest left to the per-member ladders
// (skip = done).  Workspace: csm [n_groups t], sdig / sok / done [n_groups], tab ta_small_table_bytes.
// pts_ready (nullable): waited for after the index-only split (k_ta_sprep), before pts is read.
size_t ta_small_table_bytes(uint32_t n_groups);
void launch_ta_small(const HmEntry* pts, const uint32_t* src, const int64_t* idx, uint32_t n_groups, uint32_t t,
                     int64_t* csm, TaDigits* sdig, uint8_t* sok, void* tab, uint8_t* done, G2JEntry* out,
                     hipStream_t s, const uint8_t* nonuni, hipEvent_t pts_ready = nullptr);
void launch_ta_member_status(const uint8_t* sig_st, const uint32_t* src, uint32_t n_partials, uint8_t* mstat,
                             hipStream_t s);

// Hashing and the pairing kernel (pipeline.hip).
constexpr int GROUPS_PER_WAVE = 21;  // k_pair3: 3 lanes per pairing, 21 pairings per wave
void launch_hash_to_g2(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                       hipStream_t s);
// the staged form (hashsplit.hip): uses hm[i].lines[0..3] as hand-over space (k_lines_msg overwrites it)
void launch_hash_to_g2_split(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                             hipStream_t s);
void launch_lines_msg(MsgEntry* hm, uint32_t n, hipStream_t s, const uint8_t* guard = nullptr);

// k_pair3 arguments.  Unit u of a launch pairs (P, H(m)) and (-g1, S) where S's lines evaluated at
// -g1 are sig_lines[j * stride + u].  Direct mode (list == nullptr): unit u is entry u of pk /
// msg_idx / status.  List mode: unit u is entry e = list[base + u] when base + u < *count, where
// entries e >= n_items denote the folded aggregate of validator e - n_items (agg_pk, agg_msg,
// agg_status).  Statuses: a nonzero pk_st / sig_st byte (nullable arrays) decides the verdict
// without the pairing; otherwise OK iff the product of the two pairings is one.
//
// Batched final exponentiation (launch_pair3_ml / launch_pair3_fin): the ML launch runs only the
// Miller loop of (P, H(m)) of entry e and stores it, unexponentiated, at f_out[3 e .. 3 e + 2] (one
// where pk_st[e] is nonzero).  The FIN launch runs the Miller loop of (-g1, S) from sig_lines,
// multiplies in the stored values f_in of entries [e f_range, min((e + 1) f_range, f_n)), then
// exponentiates: status[e] = nonzero pk_st[e] ? 1 : (OK iff the product is one).
struct Pair3Args {
  const G1AEntry* pk;
  const uint8_t* pk_st;
  const uint8_t* sig_st;
  const uint8_t* sig_inf;
  const uint32_t* msg_idx;
  const MsgEntry* hm;
  const LineEntry* sig_lines;
  uint32_t stride;
  uint32_t n;
  const uint32_t* list;
  const uint32_t* count;
  uint32_t base;
  uint32_t n_items;
  const G1AEntry* agg_pk;
  const uint32_t* agg_msg;
  uint8_t* status;
  uint8_t* agg_status;
  Fp4Entry* f_out;
  const Fp4Entry* f_in;
  uint32_t f_range, f_n;
  const uint8_t* guard;  // nullable: the launch does nothing unless *guard != 0 (slot-wide check failed)
  // PROD / MLS / ML / MML outputs: entry e goes to f_out[e * f_out_stride + f_out_off] (stride 0 = 1),
  // so that a final exponentiation's two factors (product tree root, signature-side loop) sit side
  // by side
  uint32_t f_out_stride, f_out_off;
  // ML (nullable): one byte per unit, nonzero when the unit fails without its pairing (state, P or
  // H(m) at infinity); a six-lane final exponentiation over the stored loop takes it as pk_st
  uint8_t* f_bad;
};
void launch_pair3(const Pair3Args& a, hipStream_t s);
void launch_pair3_ml(const Pair3Args& a, hipStream_t s);
void launch_pair3_fin(const Pair3Args& a, hipStream_t s);
// PROD: f_out[e] = product of the stored values f_in of entries [e f_range, min((e + 1) f_range, f_n))
void launch_pair3_prod(const Pair3Args& a, hipStream_t s);
// MML: f_out[e] = ONE Miller loop over the pairs i in [e f_range, min((e + 1) f_range, f_n)) with
// the shared squarings; the lines come from sig_lines as evaluated by launch_mml_eval (pk, pk_st,
// msg_idx, hm, f_n of the same arguments), line j of pair i at sig_lines[j f_n + i]
void launch_pair3_mml(const Pair3Args& a, hipStream_t s);
void launch_mml_eval(const Pair3Args& a, LineEntry* ev, hipStream_t s);
// the same evaluated lines computed from H(m_g) directly (pipeline.hip k_lines_at_p; calls that
// deferred the messages' unevaluated lines)
void launch_lines_at_p(const Pair3Args& a, LineEntry* ev, hipStream_t s);
// MLS: f_out[e] = the Miller loop of (-g1, S) alone from sig_lines (unit e at sig_lines[j stride + e]),
// stored unexponentiated; the final exponentiation then runs with sig_lines == nullptr (FIN: no loop
// of its own, the product of its f_range stored values, exponentiated)
void launch_pair3_mls(const Pair3Args& a, hipStream_t s);
// the (-g1, S) loop of each of n Jacobian points S straight from the points (lines produced and
// consumed in one two-wave workgroup per point): f_out[e f_stride + f_off], bad[e] = S infinite
void launch_lml(const G2JEntry* pts, uint32_t n, Fp4Entry* f_out, uint32_t f_stride, uint32_t f_off, uint8_t* bad,
                hipStream_t s, const uint8_t* guard = nullptr);
struct LmlArgs {
  const G2JEntry* pts;     // side 0: the points S
  const G1AEntry* pk;      // side 1: P per unit, its state (pk_st), message (msg_idx) and table (hm)
  const uint8_t* pk_st;
  const uint32_t* msg_idx;
  const MsgEntry* hm;
  uint32_t n;
  Fp4Entry* f_out;
  uint32_t f_stride, f_off;
  uint8_t* bad;
  const uint8_t* guard;
};
// side 1: the (P, H(m)) loop of each unit, H(m) affine (its lines are produced in the kernel)
void launch_lml_p(const LmlArgs& a, hipStream_t s);
constexpr uint32_t PROD_FAN = 8;  // fan-in of the product trees in front of a final exponentiation
// FIN without sig_lines over six lanes per unit (pair6.h: Fp2 products split across lane pairs):
// the same statuses at about half the latency
void launch_pair6_fin(const Pair3Args& a, hipStream_t s);
constexpr uint32_t MML_PAIRS = 4;  // pairs per multi-Miller loop of the slot-wide check

// Batched verification (vbatch.hip).
void launch_item_group(const uint32_t* grp_off, uint32_t n_groups, uint32_t n, uint32_t* item_grp, hipStream_t s);
extern std::atomic<size_t> g_dec_pair_max;
extern std::atomic<size_t> g_ta_pair_max;
extern std::atomic<size_t> g_hash_pair_max;
extern std::atomic<size_t> g_hash_one_lane, g_hash_split;  // hash.hip (the unsplit kernels, a cross-check)
extern std::atomic<size_t> g_fe18_max;  // pipeline.hip: final exponentiations over eighteen lanes up to this many units  // hashsplit.hip: the cofactor ladders on lane pairs up to this many messages  // threshold.hip: the aggregation's [s] ladder on lane pairs up to this many validators  // vbatch.hip: subgroup checks on lane pairs up to this many items
void launch_dec_pk(const uint8_t* pks, uint32_t n, G1AEntry* out, uint8_t* st, hipStream_t s);
// decoded (nullable): recorded between the decompression and the subgroup checks (which set a
// failing point to infinity and its status)
void launch_dec_sig_pt(const uint8_t* sigs, uint32_t n, HmEntry* out, uint8_t* st, hipStream_t s,
                       const uint8_t* skip = nullptr, hipEvent_t decoded = nullptr);
void launch_sc_put(const uint8_t* sigs, const HmEntry* pts, const uint8_t* st, uint32_t n, uint32_t base, uint32_t cap,
                   void* key, HmEntry* ent, uint8_t* est, uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1,
                   hipStream_t s);
void launch_sc_get(const uint8_t* sigs, uint32_t n, const void* key, const HmEntry* ent, const uint8_t* est,
                   const uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1, HmEntry* out, uint8_t* st, uint8_t* hit,
                   uint32_t cap, uint32_t busy_lo, uint32_t busy_len, hipStream_t s);
void launch_kc_index(const uint8_t* keys, uint32_t first, uint32_t m, uint32_t* tab, uint32_t tcap, uint64_t k0,
                     uint64_t k1, hipStream_t s);
void launch_pk_cached(const uint8_t* pks, uint32_t n, const uint8_t* keys, const G1AEntry* tabe, const uint8_t* tst,
                      const uint32_t* tab, uint32_t tcap, uint64_t k0, uint64_t k1, G1AEntry* out, uint8_t* st,
                      hipStream_t s);
// Chunk plans and the multi-scalar random linear combination (vbatch.hip k_plan_*, k_rlc_msm).
constexpr uint32_t RLC_CHUNK = 16;  // items per lane of k_rlc_msm
struct RlcMsmArgs {
  const G1AEntry* pk;
  const uint8_t* pk_st;
  const HmEntry* sig;
  const uint8_t* sig_st;
  const uint32_t* cfirst;
  const uint32_t* ccount;
  const uint32_t* total;  // device: number of chunks
  uint32_t key_base;
  RlcKey key;
  uint2* coef;    // per item (the dense (a, b) pairs a bucket MSM reads)
  uint4* coef4;   // per item in the sparse format (ec28.h RLC_DIGITS), when `sparse`
  int sparse;     // 1: sparse coefficients (sides 1 and 3 only; nothing reads coef)
  G1J* t1;        // 3 per item (4 when sparse)
  G2J* t2;        // 3 per item (4 when sparse)
  G1JEntry* pout;
  G2JEntry* sout;
  int always;     // random r for groups of one item too (batched final exponentiation)
  int sides;      // 1: public-key side only (coef written); 2: signature side only (coef read); 3: both
  const uint8_t* guard;  // nullable: nothing unless *guard != 0
};
void launch_plan(const uint32_t* grp_off, uint32_t ng, uint32_t cmax, uint32_t* cnt, uint32_t* coff,
                 uint32_t* cfirst, uint32_t* ccount, hipStream_t s);
void launch_rlc_msm(const RlcMsmArgs& a, uint32_t max_chunks, hipStream_t s);
// per item; coef (nullable) as RlcMsmArgs::coef with `sides`, guard as RlcMsmArgs::guard
void launch_rlc(const G1AEntry* pk, const uint8_t* pk_st, const HmEntry* sig, const uint8_t* sig_st,
                const uint32_t* item_grp, const uint32_t* grp_off, int always, uint32_t n, uint32_t key_base,
                const RlcKey& key, G1JEntry* pout, G2JEntry* sout, hipStream_t s, uint2* coef = nullptr,
                int sides = 3, const uint8_t* guard = nullptr);
// exclusive scan of cnt[0..n) into off[0..n], off[n] = total (one workgroup)
void launch_scan(const uint32_t* cnt, uint32_t n, uint32_t* off, hipStream_t s);
struct GroupPrepArgs {
  const uint32_t* grp_off;  // nullable: group g = item g
  uint32_t g0, ng;          // groups [g0, g0 + ng) of this launch
  const uint32_t* msg_idx;
  const MsgEntry* hm;
  const G1AEntry* pk;
  const uint8_t* pk_st;
  const HmEntry* sig;
  const uint8_t* sig_st;
  const G1JEntry* pr;
  const G2JEntry* sr;
  // folded aggregate of validator g (nullable): its pk / signature / decode statuses / combinations
  const G1AEntry* agg_pk;
  const uint8_t* agg_pk_st;
  const HmEntry* agg_sig;
  const uint8_t* agg_st;
  const G1JEntry* agg_pr;
  const G2JEntry* agg_sr;
  G1AEntry* gP;      // [ng]
  uint32_t* gmsg;    // [n_groups] (indexed by g)
  uint8_t* gst;      // [ng]
  LineEntry* glines; // [N_LINES][ng]
  // batched final exponentiation (non-null): no lines; the group's S (Jacobian, infinity unless
  // READY) and the sum over each batch of fe_batch consecutive groups
  G2JEntry* gS;      // [ng]
  G2JEntry* bS;      // [ceil(ng / fe_batch)]
  uint32_t fe_batch; // groups per batch (a power of two <= FE_BATCH; 0 = FE_BATCH)
  int p_only;        // slot-wide check (msm.hip): the public-key side and the state only, no S
  int keys_only;     // pr combined from the keys alone (per item, k_rlc): skip unusable items' pr
  const uint8_t* guard;  // nullable: nothing unless *guard != 0
  // small calls: do not read hm (the launch need not wait for the hashing); a message hashing to
  // infinity is then caught by the group's pairing check (its status, k_pair3<FML>) instead of
  // G_EMPTY -- either way the group fails and its items are checked alone
  int skip_hm;
};
constexpr uint32_t FE_BATCH = 64;  // groups per batched final exponentiation (one wave of k_group_prep)
void launch_group_prep(const GroupPrepArgs& a, hipStream_t s);
void launch_batch_sum(const G2JEntry* gS, uint32_t ng, uint32_t k, G2JEntry* bS, hipStream_t s, const uint8_t* guard);
// lines at -g1 of the affine images of pts[e], e = list ? list[u] (u < *count) : u, into
// lines[j * stride + u]; bad[u] (nullable) = the point is infinity
void launch_slines(const G2JEntry* pts, const uint32_t* list, const uint32_t* count, uint32_t n, LineEntry* lines,
                   uint32_t stride, uint8_t* bad, hipStream_t s, const uint8_t* guard = nullptr);
// Group verdicts (gver) of the batched paths: 0 passed; 1 .. 0x7f its own check failed (the
// pairing kernels write their status byte); GV_UNCHECKED a failing batch the first-error mode did
// not descend into; GV_NOT_READY not in any combined check (inconsistent messages, a degenerate
// combination): its items are checked alone.
enum : uint8_t { GV_PASS = 0, GV_UNCHECKED = 0x80, GV_NOT_READY = 0x81 };
HD bool gv_failed(uint8_t v) { return v != GV_PASS && v < GV_UNCHECKED; }
// group verdicts from the batch verdicts: not READY -> GV_NOT_READY, READY in a passing batch ->
// GV_PASS, else the group joins list (its verdict comes from the per-group check).  first
// (nullable, first-error mode): first[0] is the smallest key g0 + (first group of the batch) over
// the failing batches (atomicMin, 0xffffffff before the first chunk); only that batch's groups join
// the list, the other failing batches' groups get GV_UNCHECKED.
void launch_batch_verdict(const uint8_t* gst, const uint8_t* bver, uint32_t ng, uint8_t* gver, uint32_t* list,
                          uint32_t* count, hipStream_t s, const uint8_t* guard = nullptr, uint32_t fe_batch = FE_BATCH,
                          uint32_t* first = nullptr, uint32_t g0 = 0);
// slot-wide check passed (*sfail == 0): gver[g] = GV_NOT_READY or GV_PASS; else nothing (the
// per-group path decides)
void launch_slot_verdict(const uint8_t* gst, uint8_t* sfail, uint32_t ng, uint8_t* gver, hipStream_t s);
// first-error mode: *first_group = the smallest g whose own check failed (atomicMin; 0xffffffff
// before); *first_item = the smallest i with status[i] decided and not OK
void launch_first_group(const uint8_t* gver, uint32_t n_groups, uint32_t* first_group, hipStream_t s);
void launch_first_item(const uint8_t* status, uint32_t n, uint32_t* first_item, hipStream_t s);

// The signature side of a whole verification as one multi-scalar multiplication (msm.hip):
// S = sum over the items i of READY groups of [a_i] sig_i + [b_i] (-psi^2 sig_i), bucket method
// with MSM_WINDOWS windows of MSM_C bits.
constexpr uint32_t MSM_C = 16, MSM_WINDOWS = 2, MSM_MASK = (1u << MSM_C) - 1;
constexpr uint32_t MSM_KEYS = MSM_WINDOWS << MSM_C;  // buckets (window, digit); digit 0 unused
// buckets per lane of the weighing pass: 4 (32 768 lanes) rather than 16 -- the pass is a latency
// tail of every slot (one round of waves), so more, shorter lanes halve it for ~20 M more products
constexpr uint32_t MSM_CHUNK = 4;
constexpr uint32_t MSM_PARTS = MSM_KEYS / MSM_CHUNK;
struct G2MsmArgs {
  const HmEntry* sig;      // items [0, n)
  const uint8_t* sig_st;   // [n] their decompression / subgroup statuses (nonzero: not in the sum)
  const HmEntry* agg_sig;  // items [n, n + n_agg): the folded aggregates (group i - n)
  const uint8_t* agg_st;   // [n_agg] their ThresholdAggregate statuses (nonzero: not in the sum)
  const uint2* coef;       // [n + n_agg]; (0, 0) = the item is not in the combination
  const uint32_t* igrp;    // [n] item -> group
  const uint8_t* gst;      // [groups] group state (G_READY ones enter)
  uint32_t n, n_agg;
  uint32_t* cnt;           // [MSM_KEYS] zeroed
  uint32_t* off;           // [MSM_KEYS + 1]
  uint32_t* cur;           // [MSM_KEYS] zeroed
  uint32_t* ent;           // [2 MSM_WINDOWS (n + n_agg)]
  uint32_t* order;         // [MSM_KEYS] buckets by decreasing size
  G2JEntry* bucket;        // [MSM_KEYS]
  G2JEntry* part;          // [MSM_PARTS]
  G2JEntry* part2;         // [MSM_PARTS / 128]
  G2JEntry* total;         // [1]
};
void launch_msm_count(const G2MsmArgs& a, hipStream_t s);
void launch_msm_fill(const G2MsmArgs& a, hipStream_t s);
void launch_msm_bucket(const G2MsmArgs& a, hipStream_t s);
void launch_msm_reduce(const G2MsmArgs& a, hipStream_t s);
void launch_msm_sum(const G2MsmArgs& a, hipStream_t s);
struct ScatterArgs {
  uint32_t n;
  const uint32_t* item_grp;
  const uint32_t* msg_idx;
  const MsgEntry* hm;
  const G1AEntry* pk;
  const uint8_t* pk_st;
  const HmEntry* sig;
  const uint8_t* sig_st;
  const uint8_t* gverdict;  // [n_groups], 0 = the group's combined check passed
  // [n_groups + 1] group offsets (nullable: every item its own group).  A failing group of one
  // item is that item's verdict (its check is the item's own up to a nonzero exponent r): no
  // re-check alone -- unless aggregates are folded in (n_agg), which join their group's check
  const uint32_t* grp_off;
  // folded aggregates (nullable)
  uint32_t n_agg;
  const uint8_t* ta_status;
  const G1AEntry* agg_pk;
  const uint8_t* agg_pk_st;
  const HmEntry* agg_sig;
  uint8_t* agg_status;
  uint8_t* status;
  uint32_t* list;
  uint32_t* count;
  // first-error mode (nullable): first_group[0] = the first group whose own check failed; items of
  // GV_FAIL groups after it and of GV_UNCHECKED groups get ST_UNCHECKED instead of a re-check
  const uint32_t* first_group;
};
void launch_scatter(const ScatterArgs& a, hipStream_t s);
// fallback: lines at -g1 of the listed signatures (entries >= n_items: folded aggregates)
void launch_fb_lines(const uint32_t* list, const uint32_t* count, uint32_t base, uint32_t cap, const HmEntry* sig,
                     const HmEntry* agg_sig, uint32_t n_items, LineEntry* lines, hipStream_t s);

// Signing roots (roots.hip): SSZ AttestationData -> GetDataRoot, and SigningData of object roots.
void launch_duty_roots(int kind, const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                       const uint8_t* domains, uint32_t n_domains, const uint32_t* dom_idx, uint8_t* roots,
                       uint8_t* status, hipStream_t s);
void launch_attestation_roots(const uint8_t* data, uint32_t n, const uint8_t* domains, uint32_t n_domains,
                              const uint32_t* dom_idx, uint8_t* roots, hipStream_t s);
void launch_signing_roots(const uint8_t* obj, uint32_t n, const uint8_t* domains, uint32_t n_domains,
                          const uint32_t* dom_idx, uint8_t* roots, hipStream_t s);

// FastAggregateVerify at scale (vbatch.hip): segmented G1 reduction, then the pairing kernel.
void launch_seg_sum(bool affine, const void* pts, const uint8_t* st_in, const uint32_t* seg_off, uint32_t n_seg,
                    G1JEntry* out, uint8_t* st_out, hipStream_t s);
void launch_va_point(const G1JEntry* sums, const uint32_t* sum_of_group, uint32_t n_groups, G1AEntry* out,
                     hipStream_t s);
void launch_sig_lines(const HmEntry* sig, uint32_t n, LineEntry* lines, uint32_t stride, hipStream_t s);
void launch_va_status(const HmEntry* sig, const uint8_t* sig_st, const uint8_t* key_bad,
                      const uint32_t* sum_of_group, const uint8_t* pv, uint32_t n_groups, uint8_t* status,
                      hipStream_t s);

}  // namespace hb
