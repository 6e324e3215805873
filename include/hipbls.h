/*
 * hipbls.h -- C ABI of libhipbls.so, the MI355X (gfx950) BLS12-381 backend for charon's tbls
 * package.  Plain pointers and sizes only; every hot-path entry point runs as HIP kernels.
 *
 * Each entry point replaces one method of charon's tbls.Implementation
 * (/root/reference/tbls/tbls.go:27-69) as implemented by tbls.Herumi
 * (/root/reference/tbls/herumi.go), in batched form; see INTEGRATION.md for the cgo binding.
 *
 * Byte formats (identical to herumi ETH mode):
 *   public key  48 B  compressed G1 (ZCash flags 0x80/0x40/0x20, big-endian x)   tbls.go:18
 *   signature   96 B  compressed G2 (x.c1 || x.c0, flags in byte 0)             tbls.go:24
 *   secret key  32 B  big-endian scalar < r                                     tbls.go:21
 *
 * Per-item status codes (the Go shim maps them to herumi's error strings):
 */
#ifndef HIPBLS_H
#define HIPBLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum hbls_status {
  HBLS_OK = 0,
  HBLS_BAD_PUBKEY = 1,     /* "cannot set compressed public key in Herumi format"   herumi.go:291 */
  HBLS_BAD_SIGNATURE = 2,  /* "cannot unmarshal signature into Herumi signature"    herumi.go:296 */
  HBLS_NOT_VERIFIED = 3,   /* "signature not verified" (Verify, herumi.go:300) /
                              "signature verification failed" (VerifyAggregate, herumi.go:338) */
  HBLS_COMBINE_FAILED = 4, /* "cannot combine signatures"                           herumi.go:282 */
  HBLS_BAD_SECRET = 5,     /* "cannot unmarshal secret into Herumi secret key"      herumi.go:310 */
  HBLS_BAD_INPUT = 6,      /* malformed batch description (offsets/lengths)  -- new, batch-only */
  HBLS_UNCHECKED = 7       /* first-error calls only: after the first failing item, not resolved */
};

/* Return codes of the entry points themselves: 0 on success, <0 on a HIP/runtime error or a
 * malformed batch description (text via hbls_last_error()).  Per-item verdicts are in the status
 * arrays. */

/* Select and initialise the devices the library drives (herumi.go:18-36 init(), idempotent and
 * thread-safe).  device_mask: bit k = HIP device k; 0 = HBLS_DEVICE_MASK from the environment
 * (default: device 0); 0xffffffff = every visible device.  Host-buffer calls shard their items
 * over the devices of the mask (one process, several GPUs: charon runs as one Go process,
 * app/app.go:131).  Calling again with a different mask fails. */
int hbls_init(uint32_t device_mask);
const char* hbls_last_error(void);
/* Nonzero if a gfx950 device is present and the kernels are loadable. */
int hbls_available(void);
/* Devices driven by the library (after hbls_init). */
int hbls_device_count(void);
/* Build provenance (new, no herumi counterpart): "hbls-build:<sha256 prefix of the charon_amd/csrc files
 * and this header>[+<compile defines>]", embedded at compile time by charon_amd/build.py.  The
 * loader (charon_amd/_lib.py) recomputes the source hash from the tree and refuses a library built
 * from other sources. */
const char* hbls_build_id(void);

/* ---------------------------------------------------------------------------------------
 * Host-buffer entry points (the drop-in boundary for the Go shim).  Blocking; the library
 * copies inputs to device memory, runs the kernels and copies results back.
 * --------------------------------------------------------------------------------------- */

/* Verify: n independent (pk, msg, sig) triples.  tbls.Verify / Herumi.Verify
 * (tbls.go:121, herumi.go:288-304).  Message i is msgs[msg_off[i] .. msg_off[i]+msg_len[i]).
 * Identical messages are hashed to G2 once; items over one message are checked together by a
 * random linear combination (one pairing per group, each item re-checked alone if its group
 * fails), so every status equals the per-item verdict.  status[i] in {OK, BAD_PUBKEY,
 * BAD_SIGNATURE, NOT_VERIFIED}.  Thread-safe: concurrent calls (one goroutine per libp2p stream,
 * p2p/receive.go:52) are coalesced into one launch after at most HBLS_COALESCE_US microseconds
 * (default 200; 0 disables). */
int hbls_verify_batch(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs,
                      const uint64_t* msg_off, const uint32_t* msg_len, size_t n, uint8_t* status);

/* Verify an ORDERED set up to its first failure (new; the callers' loops that stop at the first
 * failing item: core/parsigex/parsigex.go:93-98 drops a peer's set, core/sigagg/sigagg.go:56-63
 * and core/validatorapi/validatorapi.go:302-306 return the first error).  Same inputs as
 * hbls_verify_batch.  *first = the smallest i whose tbls.Verify fails (-1: every item verifies)
 * and *first_status (nullable) its status, exactly as hbls_verify_batch would report it.
 * status (nullable, n bytes): every item before *first is OK; after it an item is either its
 * exact status or HBLS_UNCHECKED.  Runs of consecutive items over one message are checked
 * together and, behind a failing check, only the first failing batch of runs and the first failing
 * run are resolved -- under attack the cost stays near a clean call's instead of one pairing per
 * item of every failing run.  One device; not coalesced. */
int hbls_verify_batch_first_error(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs,
                                  const uint64_t* msg_off, const uint32_t* msg_len, size_t n, int64_t* first,
                                  uint8_t* first_status, uint8_t* status);

/* ThresholdAggregate over groups: group g holds partials grp_off[g] .. grp_off[g+1]-1 with
 * 96-byte signatures sigs[j] and share indices idx[j].  out[g] = sum_j lambda_j(0) sig_j,
 * tbls.ThresholdAggregate / Herumi.ThresholdAggregate (tbls.go:115, herumi.go:249-286).
 * status[g] in {OK, BAD_SIGNATURE, COMBINE_FAILED}. */
int hbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off,
                                   size_t n_groups, uint8_t* out, uint8_t* status);

/* Aggregate: plain sum of each group's signatures (tbls.Aggregate, herumi.go:225-247).
 * An empty group yields the infinity encoding 0xc0||0^95. status in {OK, BAD_SIGNATURE}. */
int hbls_aggregate_batch(const uint8_t* sigs, const uint32_t* grp_off, size_t n_groups, uint8_t* out,
                         uint8_t* status);

/* VerifyAggregate (FastAggregateVerify): group g verifies sigs[g] on message g against the sum of
 * pks[grp_off[g] .. grp_off[g+1]).  tbls.VerifyAggregate / Herumi.VerifyAggregate
 * (tbls.go:133, herumi.go:318-342).  status in {OK, BAD_SIGNATURE, BAD_PUBKEY, NOT_VERIFIED}.
 * The keys of a group are summed by a parallel segmented reduction, so one group may hold all
 * public shares of a cluster lock (cluster/lock.go:185). */
int hbls_verify_aggregate_batch(const uint8_t* pks, const uint32_t* grp_off, const uint8_t* sigs,
                                const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                                size_t n_groups, uint8_t* status);

/* Signing roots (eth2util/signing/signing.go:63-77 GetDataRoot = SSZ SigningData{object_root,
 * domain}.HashTreeRoot), the 32-byte messages every verification hashes to G2.
 *   attestation: data[i] is the 128-byte SSZ encoding of a phase0.AttestationData (object root =
 *                its hash-tree-root, core/signeddata.go Attestation.MessageRoot);
 *   generic:     object_roots[i] is a 32-byte object root computed by the caller.
 * domains: n_domains 32-byte domains (signing.GetDomain); item i uses domains[dom_idx[i]]
 * (dom_idx NULL: domain 0).  roots: n x 32 bytes. */
int hbls_attestation_signing_roots(const uint8_t* data, size_t n, const uint8_t* domains, size_t n_domains,
                                   const uint32_t* dom_idx, uint8_t* roots);
int hbls_signing_roots(const uint8_t* object_roots, size_t n, const uint8_t* domains, size_t n_domains,
                       const uint32_t* dom_idx, uint8_t* roots);
/* The signing roots of the other duty types charon verifies per slot, from their SSZ encodings
 * (core/signeddata.go MessageRoot; no host SSZ pass): object i is data[off[i] .. off[i]+len[i]).
 *   kind 1  phase0.AggregateAndProof          (SignedAggregateAndProof.MessageRoot, :979)
 *   kind 2  altair.ContributionAndProof, 264 B (SignedSyncContributionAndProof.MessageRoot, :1227)
 *   kind 3  altair.SyncAggregatorSelectionData{slot, subcommittee_index}, 16 B
 *           (SyncContributionAndProof / SyncCommitteeSelection.MessageRoot, :1135 / :915)
 *   kind 4  uint64 slot, 8 B little-endian (BeaconCommitteeSelection, eth2util.SlotHashRoot, :852)
 *   kind 5  beacon block root, 32 B (SignedSyncMessage.MessageRoot, :1056)
 *   kind 6  v1.ValidatorRegistration{fee_recipient, gas_limit, timestamp, pubkey}, 84 B
 *           (VersionedSignedValidatorRegistration.MessageRoot, :661; one per validator per epoch)
 *   kind 7  phase0.VoluntaryExit{epoch, validator_index}, 16 B (SignedVoluntaryExit.MessageRoot, :580)
 *   kind 8  uint64 epoch, 8 B little-endian (SignedRandao.MessageRoot = eth2util.SignedEpoch, :791)
 *   kind 9  phase0.BeaconBlockHeader{slot, proposer_index, parent_root, state_root, body_root}, 112 B
 *           (VersionedSignedProposal.MessageRoot, :301: a block's root is its header's; the
 *           caller supplies the body root, which the beacon node's block already carries)
 * roots: n x 32 bytes; status: 0, or HBLS_BAD_INPUT for a malformed object (its root all zero). */
int hbls_duty_signing_roots(int kind, const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n,
                            const uint8_t* domains, size_t n_domains, const uint32_t* dom_idx, uint8_t* roots,
                            uint8_t* status);

/* Public-key cache for the host-buffer verification (hbls_verify_batch): keys added here are
 * decompressed and subgroup-checked once, on every device of the mask; later calls take cached
 * keys from the cache and decompress only the others.  charon adds every pubshare of its cluster
 * lock at startup (cluster/lock.go; the keys never change while it runs).  Statuses and verdicts
 * are unchanged: an undecodable cached key still yields HBLS_BAD_PUBKEY. */
int hbls_pubkey_cache_add(const uint8_t* pks, size_t n);
int hbls_pubkey_cache_clear(void);
size_t hbls_pubkey_cache_size(void);
/* Decompressed-signature cache (new, no herumi counterpart): hbls_verify_batch keeps the
 * decompressed, subgroup-checked points of the partials it verified (a ring of `entries` per
 * device, keyed by all 96 bytes), and hbls_threshold_aggregate_batch takes its members from it
 * instead of decompressing them again -- charon aggregates exactly the partials parsigex verified
 * (core/parsigdb/memory.go:197-225 -> core/sigagg/sigagg.go:105).  Results are identical with or
 * without it.  Sets the capacity (rounded down to a power of two; 0 = off; default 2^21, or
 * HBLS_SIG_CACHE), drops the contents and returns the previous capacity.  Call while no host-buffer
 * call is in flight. */
size_t hbls_sig_cache(size_t entries);

/* Test switch of the in-process multi-device split (charon is one process over every GPU of the
 * node, app/app.go:131): every device of the mask is driven through `copies` contexts (own streams,
 * workspaces and host thread), so the host-buffer entry points shard their items over them exactly
 * as over several GPUs, on a one-GPU machine.  1 restores one context per device.  Call while no
 * other call is in flight.  Results never depend on it. */
int hbls_debug_split(uint32_t copies);

/* Sign (herumi.go:306-316) and SecretToPublicKey (herumi.go:66-79), batched.
 * Sign status in {OK, BAD_SECRET}; SecretToPublicKey additionally rejects the zero key. */
int hbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_off,
                    const uint32_t* msg_len, size_t n, uint8_t* sigs, uint8_t* status);
int hbls_secret_to_public_key_batch(const uint8_t* sks, size_t n, uint8_t* pks, uint8_t* status);

/* ThresholdSplit core (herumi.go:137-185): shares[i-1] = f(i) for i = 1..total where
 * f(z) = secret + sum_k coeffs[k-1] z^k (threshold-1 coefficients, 32 B big-endian each; the
 * caller draws them from a CSPRNG or, for ThresholdSplitInsecure, from its reader).
 * RecoverSecret (herumi.go:187-223): Lagrange interpolation at 0 over k shares. */
int hbls_threshold_split(const uint8_t* secret, const uint8_t* coeffs, uint32_t total, uint32_t threshold,
                         uint8_t* shares, uint8_t* status);
int hbls_recover_secret(const uint8_t* shares, const int64_t* idx, size_t k, uint8_t* out, uint8_t* status);

/* ---------------------------------------------------------------------------------------
 * Device-buffer entry points (inputs already resident in HBM; asynchronous on `stream`, a
 * hipStream_t passed as void*; 0 = the first device's null stream).  The device is the one the
 * stream belongs to.  All pointers are device pointers.  Work is ordered after prior work on
 * `stream` and complete when later work on `stream` starts; library workspaces are ordered by
 * events, so calls on different streams never race on them.
 *
 * verify: msg_idx[i] indexes the table of distinct messages hashed by hbls_hash_to_g2_device
 * into `hm` (hbls_hm_entry_bytes() per message, library layout).  vgrp_off (nullable): groups
 * of consecutive partials over one message (group g = [vgrp_off[g], vgrp_off[g+1])), checked
 * together; NULL = every partial on its own.
 * --------------------------------------------------------------------------------------- */
int hbls_hash_to_g2_device(const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                           size_t n_msgs, void* hm, void* stream);
/* hbls_verify_batch_first_error on device buffers: the items in set order with vgrp_off's groups
 * (consecutive items over one message); status as there; *first (a device uint32) = the first
 * failing item, 0xffffffff when every item verifies. */
int hbls_verify_device_first_error(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, const void* hm,
                                   size_t n, const uint32_t* vgrp_off, size_t n_vgroups, uint8_t* status,
                                   uint32_t* first, void* stream);
int hbls_verify_device(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, const void* hm,
                       size_t n, const uint32_t* vgrp_off, size_t n_vgroups, uint8_t* status, void* stream);
int hbls_threshold_aggregate_device(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off,
                                    size_t n_groups, size_t n_partials, uint8_t* out, uint8_t* status,
                                    void* stream);

/* Attestation signing roots on device buffers (see hbls_attestation_signing_roots); dom_idx
 * entries must be < n_domains: the device path cannot return a per-call error without a host
 * synchronisation, so an out-of-range entry yields the all-zero root (never a root under another
 * domain; no signature over a real signing root verifies against it -- the item fails closed).
 * Writes the messages a slot then hashes (hbls_hash_to_g2_device / hbls_slot_device msgs). */
int hbls_attestation_signing_roots_device(const uint8_t* data, size_t n, const uint8_t* domains, size_t n_domains,
                                          const uint32_t* dom_idx, uint8_t* roots, void* stream);

/* Decompressed-key tables for hbls_slot pk_table / dv_pk_table: n compressed public keys ->
 * n entries of hbls_pk_entry_bytes() (library layout) + a status byte each (0 = valid, else the
 * key is undecodable or outside G1 and every partial under it gets HBLS_BAD_PUBKEY). */
size_t hbls_pk_entry_bytes(void);
int hbls_decompress_pubkeys_device(const uint8_t* pks, size_t n, void* table, uint8_t* status, void* stream);

/* VerifyAggregate on device buffers: pks (48 B each), sigs (96 B per group), hm (one hashed message
 * per group, hbls_hash_to_g2_device), status (n_groups) are device pointers; grp_off is a HOST
 * array of n_groups + 1 non-decreasing offsets into pks (the reduction is planned from it). */
int hbls_verify_aggregate_device(const uint8_t* pks, const uint32_t* grp_off, size_t n_groups,
                                 const uint8_t* sigs, const void* hm, uint8_t* status, void* stream);

/* One attestation slot in one call: the batch entry point of SURVEY.md section 8b for
 * sigagg/parsigex (core/parsigex/parsigex.go:93-98, core/sigagg/sigagg.go:56-63,105,117).
 *   - hash the n_msgs distinct messages (+ their Miller lines) into hm;
 *   - verify the n partials (msg_idx[i] indexes the messages, vgrp_off groups as in
 *     hbls_verify_device) into vstatus;
 *   - threshold-aggregate n_groups groups (grp_off over n_ta_partials members with share indices
 *     ta_idx) into ta_out / ta_status.  Members are either verified partials (ta_src[j] = index
 *     of member j among the n partials: their decompression is shared) or their own 96-byte
 *     signatures ta_sigs (ta_src == NULL);
 *   - optionally (dv_pks != NULL, requires n_vgroups == n_groups with group g = validator g):
 *     verify each aggregate under the validator's DV public key (sigagg.go:117) into
 *     agg_vstatus, folded into group g's combined check.  agg_vstatus[g] is the aggregation
 *     status when no aggregate was produced.
 * Semantics per item as hbls_verify_batch / hbls_threshold_aggregate_batch. */
typedef struct hbls_slot {
  const uint8_t* msgs;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  size_t n_msgs;
  void* hm;
  const uint8_t* pks;
  const uint8_t* sigs;
  const uint32_t* msg_idx;
  size_t n;
  const uint32_t* vgrp_off;
  size_t n_vgroups;
  uint8_t* vstatus;
  const uint8_t* ta_sigs;
  const uint32_t* ta_src;
  const int64_t* ta_idx;
  const uint32_t* grp_off;
  size_t n_groups;
  size_t n_ta_partials;
  uint8_t* ta_out;
  uint8_t* ta_status;
  const uint8_t* dv_pks;
  uint8_t* agg_vstatus;
  /* Optional decompressed-key tables (hbls_decompress_pubkeys_device): when non-NULL the slot
   * reads entry i of pk_table (status pk_table_st[i]) instead of decompressing pks[i], and
   * entry g of dv_pk_table instead of dv_pks[g].  Pubshares are static per cluster lock, so a
   * node decompresses and subgroup-checks them once (SURVEY.md 8e pubshare cache). */
  const void* pk_table;
  const uint8_t* pk_table_st;
  const void* dv_pk_table;
  const uint8_t* dv_pk_table_st;
} hbls_slot;
int hbls_slot_device(const hbls_slot* args, void* stream);
/* Bytes of the `hm` table entry per message. */
size_t hbls_hm_entry_bytes(void);
/* Measurement: with timing enabled (which also resets the record), every kernel launch of the
 * verification, aggregation and hashing paths is bracketed by HIP events on the stream it runs
 * on; hbls_timing_read returns kernel names (static strings) and durations in milliseconds, in
 * launch order.  enable: 0 off, 1 on, 2 on and serialised (each timed launch completes before
 * the call enqueues the next one, so every duration is the kernel alone on the device: the
 * per-kernel roofline; calls then block). */
int hbls_timing(int enable);
int hbls_timing_read(const char** names, float* ms, size_t max_n, size_t* n_out);
/* Verification statistics, collected only with HBLS_STATS=1 in the environment (each call then
 * synchronises): out[0] items verified, out[1] verification groups, out[2] items re-checked
 * alone because their group's combined check failed, out[3] groups checked alone because their
 * batch's shared final exponentiation failed, out[4] slot-wide checks run, out[5] slot-wide
 * checks that failed (the call then took the per-batch check), out[6] ThresholdAggregate /
 * Aggregate members looked up in the decompressed-signature cache, out[7] those found.  n <= 8. */
int hbls_stats(uint64_t* out, size_t n);
/* Tuning: verifications of at least min_groups groups share one final exponentiation among 64
 * groups (0 = one per group; default 128, HBLS_FE_BATCH).  Returns the previous value.  Verdicts
 * do not depend on it. */
size_t hbls_fe_batch(size_t min_groups);
/* Tuning: batched verifications of at least min_items items (partials + folded aggregates) first
 * check every group at once -- the signature side as one multi-scalar multiplication, one final
 * exponentiation for the call -- and take the per-batch check only if that fails (0 = never;
 * default 32768, HBLS_SLOT_MSM).  Returns the previous value and clears the adaptive history
 * below.  Verdicts do not depend on it. */
size_t hbls_slot_msm(size_t min_items);
/* Tuning: adaptive slot-wide check (1 = on, the default; HBLS_ADAPTIVE): after a call whose
 * slot-wide check failed, the next calls take the per-batch check directly until one passes every
 * batch.  Returns the previous setting.  Verdicts do not depend on it. */
int hbls_adaptive(int on);
/* Host Verify batches of fewer than `items` check every item alone (no random-combination ladder
 * on the latency path); SIZE_MAX = the default (the batched final exponentiation's threshold).
 * Returns the previous setting (HBLS_SINGLE_MAX at init).  Verdicts never depend on it. */
size_t hbls_single_max(size_t items);
/* Tuning: decompressions of at most `items` keys or signatures run their subgroup checks with each
 * item's ladder split over a lane pair (latency for calls that do not fill the chip; 0 = never, the
 * default, HBLS_DEC_PAIR_MAX).  Returns the previous value.  Verdicts do not depend on it. */
size_t hbls_dec_pair_max(size_t items);
/* Tuning by name (read from the environment at init; verdicts and outputs never depend on them):
 * the layouts of the latency-bound small calls "HBLS_HASH_PAIR_MAX", "HBLS_HASH_ONE_LANE",
 * "HBLS_HASH_SPLIT" (0: the unstaged hashing kernels), "HBLS_FE18_MAX", "HBLS_TA_PAIR_MAX",
 * "HBLS_DEC_PAIR_MAX"; the chunking of large verifications "HBLS_GROUP_CHUNK" (groups per pairing
 * chunk), "HBLS_FALLBACK_CHUNK" (items per fallback pass), "HBLS_GROUP_MAX" (items per group of a
 * host call).  *previous (if not NULL) receives the old value.  Returns 0, or -1 for an unknown
 * name. */
int hbls_tune(const char* name, size_t value, size_t* previous);
/* Tuning: the random linear combination's public-key side groups a verification group's items
 * into shared-doubling chunks sized to keep about `lanes` lanes busy (at most 16 items per chunk;
 * calls of fewer than 2 lanes' worth keep one ladder per item).  0 restores the default 65536
 * (HBLS_RLC_LANES).  Returns the previous value.  Verdicts do not depend on it. */
size_t hbls_rlc_lanes(size_t lanes);
/* Tuning: ThresholdAggregate calls whose groups all have t members run joint ladders over chunks
 * of `members` (<= 8) members of a validator, sharing the doublings; 0 = auto (HBLS_TA_JOINT), 1 =
 * one ladder per member.  Returns the previous value.  Outputs do not depend on it. */
size_t hbls_ta_joint(size_t members);
/* Wait for all work the library queued on `stream`. */
int hbls_sync(void* stream);
/* Device: the verify bitmap of n statuses (bit i of bits[i / 8], least significant bit first, set
 * when status[i] == HBLS_OK; bits holds ceil(n / 8) bytes), on `stream` -- the compact form of a
 * slot's verdicts that the ranks all-gather (north_star: "all-gather verify bitmaps"); the
 * failure classes stay in the owning rank's status bytes. */
int hbls_status_bitmap(const uint8_t* status, size_t n, uint8_t* bits, void* stream);

/* ---------------------------------------------------------------------------------------
 * Exchange of slot results between processes that drive one GPU each:
 * RCCL over xGMI.  Rank 0 creates the id, every rank passes it to hbls_comm_init, then
 * hbls_allgather_device gathers `bytes` from every rank into recv (rank order) on `stream`.
 * --------------------------------------------------------------------------------------- */
size_t hbls_comm_id_bytes(void);
int hbls_comm_unique_id(uint8_t* id);
int hbls_comm_init(int nranks, int rank, const uint8_t* id);
int hbls_allgather_device(const void* send, void* recv, size_t bytes, void* stream);
/* The number of ranks of the communicator as RCCL reports it (ncclCommCount), 0 without one:
 * bench.py puts it in its line beside n_gpus. */
int hbls_comm_size(void);
int hbls_comm_destroy(void);

#ifdef __cplusplus
}
#endif
#endif /* HIPBLS_H */
