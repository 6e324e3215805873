// libhipbls.so: gfx950 kernels + C ABI (include/hipbls.h) for charon's BLS hot path.
//
// Reference interface replaced: tbls.Implementation (/root/reference/tbls/tbls.go:27-69) as
// implemented by tbls.Herumi (/root/reference/tbls/herumi.go).  This file holds the one-lane
// kernels of the cold entry points (Sign, SecretToPublicKey, split/recover, group sums) and the
// host runtime: per-device contexts (one process may drive every GPU in its device mask),
// workspace sets ordered by events, the batched verification pipeline, a coalescing queue for
// concurrent callers (charon calls tbls.Verify from one goroutine per libp2p stream,
// p2p/receive.go:52) and the RCCL exchange of slot results between processes.
#include "layout.h"
#include "../../include/hipbls.h"
#include "coalesce.h"
#include "msgtable.h"

#include <rccl/rccl.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <numeric>
#include <string>
#include <string.h>
#include <thread>
#include <unordered_map>
#include <vector>

using namespace hb;

#define KERNEL_BOUNDS __launch_bounds__(64)
constexpr int BLOCK = 64;

// ---------------------------------------------------------------------------------------
// One-lane kernels (standard calling convention product: code size over speed)
// ---------------------------------------------------------------------------------------

// One lane per group: sum the member points, compress (herumi Sign.Recover / Sign.Aggregate +
// Serialize).  Status precedence follows herumi: any undecodable partial -> BAD_SIGNATURE
// (deserialisation happens first, herumi.go:255-264), then combine failure.  agg_pt (nullable):
// the affine result, for the folded post-aggregate verification of the slot entry point.
//
// Invariant the slot path relies on: a group with a member whose status is M_BAD_SIG never uses
// its ladders' outputs (pts) -- it is zeroed here whatever they hold.  In hbls_slot_device the
// aggregation ladders start once the partials are decoded (ev_dec) and only the Lagrange digits
// wait for the subgroup statuses (mst_ready), so k_g2_subgroup may overwrite a failing member's
// point with infinity while a ladder reads it; such a member's status is M_BAD_SIG by the time
// this kernel runs (it is ordered after mst_ready), so the raced values are never published.
__global__ KERNEL_BOUNDS void k_group_sum(const uint32_t* __restrict__ grp_off, uint32_t n_groups, int mode,
                                          const G2JEntry* __restrict__ pts, const uint8_t* __restrict__ mstat,
                                          uint8_t* __restrict__ out, uint8_t* __restrict__ status,
                                          HmEntry* __restrict__ agg_pt) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  uint8_t st = ST_OK;
  if (e == b && mode == 0) st = ST_COMBINE_FAILED;  // Recover of an empty set fails
  for (uint32_t m = b; m < e; m++) {
    if (mstat[m] == M_BAD_SIG) st = ST_BAD_SIGNATURE;
  }
  if (st == ST_OK) {
    for (uint32_t m = b; m < e; m++)
      if (mstat[m] == M_BAD_IDX) st = ST_COMBINE_FAILED;
  }
  uint8_t* o = out + 96ull * g;
  if (st != ST_OK) {
    for (int k = 0; k < 96; k++) o[k] = 0;
    status[g] = st;
    if (agg_pt) agg_pt[g].inf = 1;
    return;
  }
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t m = b; m < e; m++) {
    G2JEntry q = pts[m];
    acc = jac_add(acc, G2J{q.X, q.Y, q.Z});
  }
  const G2A a = jac_to_aff(acc);
  uint8_t buf[96];
  g2_compress(buf, a);
  for (int k = 0; k < 96; k++) o[k] = buf[k];
  status[g] = ST_OK;
  if (agg_pt) {
    HmEntry h;
    h.x = a.x;
    h.y = a.y;
    h.inf = a.inf ? 1u : 0u;
    h.pad[0] = h.pad[1] = h.pad[2] = 0;
    agg_pt[g] = h;
  }
}

// Sign: one lane per (sk, message): sigma = sk * H(m)   (herumi.go:306-316)
__global__ KERNEL_BOUNDS void k_sign(const uint8_t* __restrict__ sks, const uint32_t* __restrict__ msg_idx,
                                     const MsgEntry* __restrict__ hm, uint32_t n, uint8_t* __restrict__ sigs,
                                     uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t skb[32];
  for (int k = 0; k < 32; k++) skb[k] = sks[32ull * i + k];
  Fr s;
  uint8_t buf[96];
  if (!fr_from_be(s, skb)) {
    status[i] = ST_BAD_SECRET;
    for (int k = 0; k < 96; k++) sigs[96ull * i + k] = 0;
    return;
  }
  G2J sg = jac_mul_aff(hm_load(hm[msg_idx[i]].h), s.v, 255);
  g2_compress(buf, jac_to_aff<Fp2, true>(sg));  // secret-dependent: fixed-trip inversion
  for (int k = 0; k < 96; k++) sigs[96ull * i + k] = buf[k];
  status[i] = ST_OK;
}

// SecretToPublicKey: pk = sk * g1 (herumi.go:66-79; GetSafePublicKey rejects sk = 0)
__global__ KERNEL_BOUNDS void k_sk_to_pk(const uint8_t* __restrict__ sks, uint32_t n, uint8_t* __restrict__ pks,
                                         uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t skb[32];
  for (int k = 0; k < 32; k++) skb[k] = sks[32ull * i + k];
  Fr s;
  uint8_t buf[48];
  if (!fr_from_be(s, skb) || fr_is_zero(s)) {
    status[i] = ST_BAD_SECRET;
    for (int k = 0; k < 48; k++) pks[48ull * i + k] = 0;
    return;
  }
  G1J p = jac_mul_aff(g1_generator(), s.v, 255);
  g1_compress(buf, jac_to_aff<Fp, true>(p));  // secret-dependent: fixed-trip inversion
  for (int k = 0; k < 48; k++) pks[48ull * i + k] = buf[k];
  status[i] = ST_OK;
}

// ThresholdSplit core: share i = f(i), f(z) = secret + sum coeffs[k-1] z^k over Fr.
__global__ KERNEL_BOUNDS void k_split(const uint8_t* __restrict__ poly, uint32_t threshold, uint32_t total,
                                      uint8_t* __restrict__ shares, uint8_t* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  Fr x = fr_from_i64((int64_t)i + 1);
  Fr acc = fr_zero();
  for (int k = (int)threshold - 1; k >= 0; k--) {
    Fr c;
    if (!fr_from_be(c, poly + 32ull * k)) {
      status[i] = ST_BAD_SECRET;
      return;
    }
    acc = fr_add(fr_mul(acc, x), fr_to_mont(c));
  }
  fr_to_be(shares + 32ull * i, fr_from_mont(acc));
  status[i] = ST_OK;
}

// RecoverSecret: single lane (k small), Lagrange at 0 over Fr.
__global__ void k_recover(const uint8_t* __restrict__ shares, const int64_t* __restrict__ idx, uint32_t k,
                          uint8_t* __restrict__ out, uint8_t* __restrict__ status) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Fr acc = fr_zero();
  for (uint32_t i = 0; i < k; i++) {
    Fr si;
    if (!fr_from_be(si, shares + 32ull * i)) {
      status[0] = ST_BAD_SECRET;
      return;
    }
    Fr lam = fr_one();
    if (k > 1) {
      Fr xi = fr_from_i64(idx[i]);
      Fr num = fr_one(), den = fr_one();
      for (uint32_t m = 0; m < k; m++) {
        if (m == i) continue;
        Fr xm = fr_from_i64(idx[m]);
        num = fr_mul(num, xm);
        den = fr_mul(den, fr_sub(xm, xi));
      }
      if (fr_is_zero(num) || fr_is_zero(den)) {
        status[0] = ST_COMBINE_FAILED;
        return;
      }
      lam = fr_mul(num, fr_inv(den));
    }
    acc = fr_add(acc, fr_mul(lam, fr_to_mont(si)));
  }
  if (k == 0) {
    status[0] = ST_COMBINE_FAILED;
    return;
  }
  fr_to_be(out, fr_from_mont(acc));
  status[0] = ST_OK;
}

// ---------------------------------------------------------------------------------------
// Host runtime
// ---------------------------------------------------------------------------------------
namespace {

thread_local std::string g_err;

int set_err(const std::string& what) {
  g_err = what;
  return -1;
}
int set_err(const char* what, hipError_t e) { return set_err(std::string(what) + ": " + hipGetErrorString(e)); }

#define HCHK(expr)                                         \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return set_err(#expr, _e);       \
  } while (0)

inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

// Host-buffer Verify on one device: the caller's keys and signatures go up as they are, and the
// device puts them in group order (one lane per item: 48 + 96 bytes as 16-byte words) and the
// statuses back in the caller's order -- no host-side copy of the 144 bytes per item.
__global__ KERNEL_BOUNDS void k_gather_items(const uint4* __restrict__ pk_in, const uint4* __restrict__ sig_in,
                                             const uint32_t* __restrict__ order, uint32_t n, uint4* __restrict__ pk_out,
                                             uint4* __restrict__ sig_out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t i = order[k];
  HB_UNROLL for (int w = 0; w < 3; w++) pk_out[3ull * k + w] = pk_in[3ull * i + w];
  HB_UNROLL for (int w = 0; w < 6; w++) sig_out[6ull * k + w] = sig_in[6ull * i + w];
}
__global__ KERNEL_BOUNDS void k_scatter_status(const uint8_t* __restrict__ st_in, const uint32_t* __restrict__ order,
                                               uint32_t n, uint8_t* __restrict__ st_out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) st_out[order[k]] = st_in[k];
}

// the verify bitmap of a slot (bit i of byte i / 8, least significant first: status[i] == OK): one
// ballot per wave, eight bytes per wave -- what the ranks all-gather
__global__ KERNEL_BOUNDS void k_status_bitmap(const uint8_t* __restrict__ st, uint32_t n, uint8_t* __restrict__ bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = __ballot(i < n && st[i] == ST_OK);
  const uint32_t lane = threadIdx.x & 63u, first = i - lane;  // the wave's first item (a multiple of 64)
  if (lane < 8 && first + 8 * lane < n) bits[first / 8 + lane] = (uint8_t)(m >> (8 * lane));
}

#define LAUNCH(kern, n, stream, ...)                                                              \
  do {                                                                                            \
    if ((n) > 0) {                                                                                \
      hipLaunchKernelGGL(kern, dim3(blocks_for(n)), dim3(BLOCK), 0, (stream), __VA_ARGS__);       \
      HCHK(hipGetLastError());                                                                    \
    }                                                                                             \
  } while (0)

size_t env_size(const char* name, size_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 0);
  return (end && *end == 0) ? (size_t)x : dflt;
}

// Verification groups are chunked for the line buffers: GCAP groups per pairing launch, FB_CAP
// fallback items per pass (HBLS_GROUP_CHUNK / HBLS_FALLBACK_CHUNK).  Host-buffer calls build
// groups of at most GMAX items over one message (HBLS_GROUP_MAX).
std::atomic<size_t> g_gcap{131072}, g_fbcap{65536}, g_gmax{16};
std::atomic<size_t> g_rlc_lanes{65536};   // HBLS_RLC_LANES: lanes the chunk size aims to keep busy
// public-key cache: compressed key -> entry index (the same on every device).  Lock order: an
// adder (or clear) takes g_kc_add_mu, then one Dev::mu at a time to fill that device's table, then
// g_kc_mu to publish; verifications hold their Dev::mu and take g_kc_mu for the lookup.  g_kc_mu is
// always the innermost lock, so adds and verifications never wait on each other in a cycle.  A
// lookup made under a Dev::mu stays valid for everything enqueued while it is held: entries are
// only written under it, and kc_fill first waits for every launch already enqueued on the device
// (which covers indices reused after hbls_pubkey_cache_clear).
std::mutex g_kc_add_mu;
std::mutex g_kc_mu;
std::unordered_map<std::string, uint32_t> g_kc_map;
size_t g_kc_n = 0;             // published entries (g_kc_mu; written under g_kc_add_mu too)
std::vector<uint8_t> g_kc_keys;  // their compressed bytes, 48 B each (g_kc_add_mu): fills new devices
// HBLS_TA_JOINT: members per lane of the joint aggregation ladders (k_ta_jtab, k_ta_jladder, k_ta_jgeneral) when every group has
// the same size t; 0 = auto (about TA_JOINT_LANES lanes, at most t and 8), 1 = one ladder per member
// (k_ta_straus)
std::atomic<size_t> g_ta_joint{0};
constexpr size_t TA_JOINT_LANES = 98304;
// HBLS_FE_BATCH: verifications of at least this many groups check FE_BATCH groups per final
// exponentiation (vgroup.hip; 0 = one final exponentiation per group)
std::atomic<size_t> g_fe_batch_min{2 * FE_BATCH};
// HBLS_SLOT_MSM: batched verifications of at least this many items (partials + folded aggregates,
// one chunk of groups) check every group at once -- the signature side as one multi-scalar
// multiplication (msm.hip), one final exponentiation for the call -- and fall back to the
// per-batch check when that fails (0 = never).  32 768: at C2 (40 k partials + 10 k folded
// aggregates) the slot-wide check beats the per-batch one since the multi-Miller loops and the
// six-lane final exponentiation (14.4 vs 15.3 ms per slot, profiles/r03s_ab_summary.txt)
std::atomic<size_t> g_slot_msm_min{32768};
// HBLS_ADAPTIVE=0: always try the slot-wide check.  Default: after a call whose slot-wide check
// failed (invalid partials or aggregates that only a pairing catches), the next calls go straight
// to the per-batch check -- a failing slot-wide check is work thrown away -- until a call passes
// every batch; under a sustained attack (C5: 1 % of the partials invalid in every slot) that
// saves the signature-side MSM, its lines and Miller loop, the product tree and one final
// exponentiation per slot.  Verdicts are the same either way.
std::atomic<bool> g_adaptive{true};
// HBLS_SINGLE_MAX / hbls_single_max: host Verify batches of fewer items check every item alone
// (SINGLE_MAX_DEFAULT: the batched final exponentiation's threshold, g_fe_batch_min)
constexpr size_t SINGLE_MAX_DEFAULT = ~size_t(0);
std::atomic<size_t> g_single_max{SINGLE_MAX_DEFAULT};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

// workspace buffers of one set
enum WsId {
  W_VPK, W_VPKST, W_VSIG, W_VSIGST, W_IGRP, W_PR, W_SR, W_GP, W_GST, W_GMSG, W_GVER, W_GLINES, W_LIST, W_COUNT,
  W_FBLINES,
  W_APK, W_APKST, W_ASIG, W_APR, W_ASR,          // folded aggregates (post-aggregate verification)
  W_TAPTS, W_TADST, W_TAMST, W_TADIG, W_TATAB, W_TAJ, W_TAHIT,  // ThresholdAggregate / Aggregate
  W_TACSM, W_TASDIG, W_TASOK, W_TASDONE, W_TASTAB, W_TANONUNI,  // its small-scalar path
  W_SEGA, W_SEGB, W_SEGSTA, W_SEGSTB, W_VAPT, W_VAPV, W_PLAN,  // VerifyAggregate key reduction
  W_PCNT, W_PCOFF, W_PCFIRST, W_PCCOUNT, W_COEF, W_COEF4, W_RT1, W_RT2,  // chunk plan + multi-scalar RLC
  W_FBUF, W_GS, W_BS, W_BLINES, W_BBAD, W_BVER, W_GLIST, W_GCOUNT,  // batched final exponentiation
  W_MCNT, W_MOFF, W_MCUR, W_MORDER, W_MENT, W_MBUCKET, W_MPART, W_MPART2, W_MTOT, W_PBUF1, W_PBUF2, W_PBUF3, W_SFAIL,  // slot-wide check
  W_MLEV,                                                                          // its evaluated Miller lines
  W_PFIN, W_TBUF, W_F1, W_F1BAD, W_F1S, W_FIRST,                                                                  // final exponentiations' factors
  W_COUNT_
};

// A workspace set: grow-only device buffers plus the event recorded after the last kernel that
// used them.  Every user waits on `free_ev` in each stream it launches on before touching the
// set, so two calls never share a set concurrently, whatever streams they run on.
//
// Each set also owns the side streams its calls fork onto (decompression, hashing, aggregation)
// and their fork/join events, so two calls in flight on different user streams -- consecutive
// slots, say -- overlap instead of queueing behind each other on shared side streams.
constexpr int N_SIDE = 4;
struct Ws {
  DevBuf b[W_COUNT_];
  hipEvent_t free_ev = nullptr;
  bool used = false;
  hipStream_t side[N_SIDE] = {};
  hipEvent_t ev_fork = nullptr, ev_side[N_SIDE] = {}, ev_ta = nullptr, ev_msm = nullptr;
  hipEvent_t ev_pk = nullptr;  // the partials' keys decompressed (side 0, before the DV keys)
  hipEvent_t ev_dec = nullptr;  // the partials' signatures decompressed (side 1, before their subgroup checks)
  hipEvent_t ev_h = nullptr;  // host calls: the hashing done (before the messages' lines)
};

// host-call staging buffers (inputs and outputs of the host-buffer entry points)
enum IoId { I_PK, I_SIG, I_MSG, I_OFF, I_LEN, I_MIDX, I_HM, I_STAT, I_IDX, I_GOFF, I_OUT, I_SK, I_VGOFF, I_HM2, I_COUNT };

constexpr int N_WS_MAX = 8;  // workspace sets per device: HBLS_WS_SETS (default 3)
int g_ws_sets = 3;

struct Timed {
  const char* name;
  hipEvent_t a, b;
};

// Host-call contexts: a blocking host-buffer call (Verify / ThresholdAggregate / VerifyAggregate
// batches: what the Go shim calls from its goroutines) owns one from its first upload to its last
// download -- its own stream and staging buffers -- and holds the device lock only while it
// enqueues.  Several calls from different threads therefore overlap on the device (one workspace
// set each), as consecutive slots do on the device-buffer path.  g_ws_sets contexts per device; a
// caller beyond them waits for one to finish.
struct Hc {
  hipStream_t s = nullptr;
  DevBuf io[I_COUNT];
  bool busy = false;
  hipEvent_t ev = nullptr;  // a chunked call's hand-overs between contexts (verify_large)
  // pinned staging for uploads queued behind the call's own kernels: a pageable hipMemcpyAsync is
  // staged by the runtime and returns only once staged, so one queued behind the decompression
  // held the calling thread until that finished (verify_large's grouping: 20 ms measured; on a
  // stream of its own beside the kernels the pageable copies took over a second)
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
  // a signature-cache put (on the device's cache stream, after the call returned) still reading
  // this context's staging buffers: the context's next call waits for it before it uploads into
  // them (hc_acquire)
  hipEvent_t put_ev = nullptr;
  bool put_pending = false;
  hipStream_t put_s = nullptr;  // its signature-cache puts (sc_put_release)
};

// host arrays packed into a context's pinned staging, then one asynchronous copy each
struct PinnedUploads {
  struct Item {
    IoId id;
    const void* src;
    size_t bytes;
    void** dst;
  };
  std::vector<Item> items;
  template <class T>
  void add(IoId id, const T* src, size_t count, T** dst) {
    items.push_back({id, src, count * sizeof(T), (void**)dst});
  }
};

// one record per call that could take the slot-wide check: did it fail (or, skipped, did any batch
// fail the per-batch check)
struct SlotRes {
  uint8_t sfail, skipped, pad[2];
  uint32_t gcount;
};
constexpr unsigned N_RES = 16;

struct Dev {
  int ord = -1;
  int n_cu = 256;  // compute units (4 SIMDs each)
  hipStream_t stream = nullptr;  // the library stream of host-buffer calls
  Ws ws[N_WS_MAX];
  unsigned next_ws = 0;
  DevBuf io[I_COUNT];
  std::mutex mu;  // one call at a time enqueues on this device
  Hc hc[N_WS_MAX];
  std::mutex hc_mu;  // hc[].busy
  std::condition_variable hc_cv;
  // public-key cache (hbls_pubkey_cache_add): decompressed entries + statuses, every device holds
  // all g_kc_n of them
  DevBuf kc_tab, kc_st;
  // its compressed keys and their open-addressing index (vbatch.hip k_kc_index / k_pk_cached):
  // kc_n entries indexed, kc_tcap slots (a power of two >= 2 kc_n)
  DevBuf kc_keys, kc_hidx;
  size_t kc_n = 0, kc_tcap = 0;
  // decompressed-signature cache (vbatch.hip k_sc_write / k_sc_index / k_sc_get): filled by host-buffer Verify
  // batches, read by host-buffer ThresholdAggregate batches; enqueued under `mu` like everything
  // else.  A put runs on its host-call context's own put stream, off the Verify call's critical
  // path and beside other contexts' puts: it waits for its call's pipeline (`pipe`), for every get
  // enqueued before it (a put rewrites ring entries a get may read) and for any put still in flight
  // whose ring range overlaps its own, and records `done`.  A get waits only for puts whose
  // pipeline has already completed (a short kernel pair); the ring entries of puts still behind
  // their pipeline are passed to it as a range of misses.  Ring positions are also counted without
  // the wrap (`pos`), so the span of the in-flight puts is exact.
  DevBuf sc_key, sc_ent, sc_st, sc_tab;
  size_t sc_cap = 0, sc_cursor = 0, sc_filled = 0;
  uint64_t sc_pos = 0;
  struct ScPut {
    size_t start, m;
    uint64_t pos;
    hipEvent_t pipe, done;
  };
  std::deque<ScPut> sc_inflight;       // enqueue (= ring) order
  std::vector<hipEvent_t> sc_gets;     // gets not yet known complete
  std::vector<hipEvent_t> sc_ev_pool;  // spare events
  // adaptive slot-wide check (HBLS_ADAPTIVE): outcomes of recent checked calls, copied to pinned host
  // memory asynchronously and read once their event has completed -- never a synchronisation
  SlotRes* res_host = nullptr;
  hipEvent_t res_ev[N_RES] = {};
  unsigned res_head = 0, res_tail = 0;  // records [tail, head) not yet read
  bool attack = false;                  // the last known call had invalid items a pairing caught
  // timing (hbls_timing)
  bool timing = false;
  bool serial = false;  // timing mode 2: every timed launch completes before the next is enqueued
  std::vector<Timed> tev;
  size_t tev_used = 0;
};

// HBLS_SIG_CACHE / hbls_sig_cache: entries of each device's decompressed-signature cache (a power
// of two; 0 = off).  2^21 (two C3 slots of partials): 2 M x 305 B = 640 MB per device.
std::atomic<size_t> g_sc_cap{size_t(1) << 21};
uint64_t g_sc_k0 = 0x243f6a8885a308d3ull, g_sc_k1 = 0x13198a2e03707344ull;  // keyed hash (getrandom at init)

std::mutex g_init_mu;
std::vector<Dev*> g_devs;  // in device-mask order (hbls_debug_split: each ordinal repeated); g_devs_mu
std::mutex g_devs_mu;      // hbls_debug_split swaps g_devs while calls may be in flight
// a snapshot of g_devs: Dev objects are never freed (split contexts are pooled), so the pointers
// stay valid after the lock is released
std::vector<Dev*> devs() {
  std::lock_guard<std::mutex> l(g_devs_mu);
  return g_devs;
}
std::vector<Dev*> g_base_devs;   // one per device of the mask
std::vector<std::vector<Dev*>> g_split_pool;  // per base device: extra contexts of hbls_debug_split (reused)
uint32_t g_mask = 0;
std::atomic<bool> g_ready{false};

int ensure_buf(DevBuf& b, size_t bytes, void** out) {
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) HCHK(hipFree(b.p));
    b.p = nullptr;
    size_t cap = bytes + bytes / 4;
    HCHK(hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  *out = b.p;
  return 0;
}

template <class T>
int wsbuf(Ws& w, WsId id, size_t count, T** out) {
  // growing a buffer frees the old one: its last user (on any stream) must be done with it
  if (w.used && w.b[id].cap < std::max<size_t>(count * sizeof(T), 16)) HCHK(hipEventSynchronize(w.free_ev));
  void* p;
  if (ensure_buf(w.b[id], count * sizeof(T), &p)) return -1;
  *out = (T*)p;
  return 0;
}

// Acquire a workspace set for a call whose kernels run on `s` and the set's side streams.
Ws& ws_acquire(Dev& d, hipStream_t s) {
  Ws& w = d.ws[d.next_ws++ % (unsigned)g_ws_sets];
  if (w.used) {
    (void)hipStreamWaitEvent(s, w.free_ev, 0);
    for (hipStream_t x : w.side) (void)hipStreamWaitEvent(x, w.free_ev, 0);
  }
  return w;
}
int ws_release(Ws& w, hipStream_t last) {
  HCHK(hipEventRecord(w.free_ev, last));
  w.used = true;
  return 0;
}

// --- timing of kernel launches (hbls_timing): event pairs on the launch's stream -------------
int timed_begin(Dev& d, const char* name, hipStream_t s, Timed** t) {
  *t = nullptr;
  if (!d.timing) return 0;
  if (d.tev_used == d.tev.size()) {
    Timed x{name, nullptr, nullptr};
    HCHK(hipEventCreate(&x.a));
    HCHK(hipEventCreate(&x.b));
    d.tev.push_back(x);
  }
  Timed& x = d.tev[d.tev_used++];
  x.name = name;
  HCHK(hipEventRecord(x.a, s));
  *t = &x;
  return 0;
}
int timed_end(Dev& d, Timed* t, hipStream_t s) {
  if (t) {
    HCHK(hipEventRecord(t->b, s));
    if (d.serial) HCHK(hipEventSynchronize(t->b));  // the kernel ran alone on the device
  }
  return 0;
}
#define TIMED(dev, name, s, call)                  \
  do {                                             \
    Timed* _t;                                     \
    if (timed_begin((dev), (name), (s), &_t)) return -1; \
    call;                                          \
    HCHK(hipGetLastError());                       \
    if (timed_end((dev), _t, (s))) return -1;      \
  } while (0)

int dev_create(int ord, Dev** out) {
  HCHK(hipSetDevice(ord));
  hipDeviceProp_t prop;
  HCHK(hipGetDeviceProperties(&prop, ord));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(std::string("libhipbls is built for gfx950, device ") + std::to_string(ord) + " is " +
                   prop.gcnArchName);
  Dev* d = new Dev();
  d->ord = ord;
  d->n_cu = std::max(1, prop.multiProcessorCount);
  // the verification's side streams (decompression, hashing) get the highest priority: they
  // gate the pairing kernel; the library stream is the lowest
  int prio_lo = 0, prio_hi = 0;
  HCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  HCHK(hipStreamCreateWithPriority(&d->stream, hipStreamNonBlocking, prio_lo));
  for (int k_ws = 0; k_ws < g_ws_sets; k_ws++) {
    Ws& w = d->ws[k_ws];
    HCHK(hipEventCreateWithFlags(&w.free_ev, hipEventDisableTiming));
    for (int k = 0; k < N_SIDE; k++) {
      // side 3 (the slot's ThresholdAggregate) at high priority like the others (the lowest measured
      // 135.7-135.9 against 134.2-134.9 ms per C3 slot, three slots in flight)
      HCHK(hipStreamCreateWithPriority(&w.side[k], hipStreamNonBlocking, prio_hi));
      HCHK(hipEventCreateWithFlags(&w.ev_side[k], hipEventDisableTiming));
    }
    HCHK(hipEventCreateWithFlags(&w.ev_fork, hipEventDisableTiming));
    HCHK(hipEventCreateWithFlags(&w.ev_ta, hipEventDisableTiming));
    HCHK(hipEventCreateWithFlags(&w.ev_msm, hipEventDisableTiming));
    HCHK(hipEventCreateWithFlags(&w.ev_h, hipEventDisableTiming));
    HCHK(hipEventCreateWithFlags(&w.ev_pk, hipEventDisableTiming));
    HCHK(hipEventCreateWithFlags(&w.ev_dec, hipEventDisableTiming));
    HCHK(hipStreamCreateWithPriority(&d->hc[k_ws].s, hipStreamNonBlocking, prio_lo));
    HCHK(hipEventCreateWithFlags(&d->hc[k_ws].ev, hipEventDisableTiming));
  }
  HCHK(hipHostMalloc((void**)&d->res_host, N_RES * sizeof(SlotRes), hipHostMallocDefault));
  for (unsigned k = 0; k < N_RES; k++) HCHK(hipEventCreateWithFlags(&d->res_ev[k], hipEventDisableTiming));
  *out = d;
  return 0;
}

// hbls_init: mask 0 = HBLS_DEVICE_MASK from the environment, else device 0; 0xffffffff = every
// visible device.  Idempotent for the same mask; a different mask afterwards is an error.
int init_mask(uint32_t mask) {
  if (g_ready.load()) {
    if (mask != 0 && mask != g_mask && !(mask == 0xffffffffu && g_mask == ((1u << g_base_devs.size()) - 1)))
      return set_err("hipbls already initialised with device mask " + std::to_string(g_mask));
    return 0;
  }
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_ready.load()) return init_mask(mask);
  int n = 0;
  HCHK(hipGetDeviceCount(&n));
  if (n <= 0) return set_err("no HIP device");
  if (mask == 0) mask = (uint32_t)env_size("HBLS_DEVICE_MASK", 1);
  const uint32_t visible = n >= 32 ? 0xffffffffu : ((1u << n) - 1);
  if (mask == 0xffffffffu) mask = visible;
  if ((mask & visible) != mask || mask == 0)
    return set_err("device mask " + std::to_string(mask) + " names devices that are not visible (" +
                   std::to_string(n) + " devices)");
  g_gcap = std::max<size_t>(1, env_size("HBLS_GROUP_CHUNK", g_gcap.load()));
  g_fbcap = std::max<size_t>(1, env_size("HBLS_FALLBACK_CHUNK", g_fbcap.load()));
  g_gmax = std::max<size_t>(1, env_size("HBLS_GROUP_MAX", g_gmax.load()));
  g_rlc_lanes = std::max<size_t>(1, env_size("HBLS_RLC_LANES", g_rlc_lanes.load()));
  g_ta_joint = std::min<size_t>(8, env_size("HBLS_TA_JOINT", g_ta_joint.load()));
  g_fe_batch_min = env_size("HBLS_FE_BATCH", g_fe_batch_min.load());
  g_slot_msm_min = env_size("HBLS_SLOT_MSM", g_slot_msm_min.load());
  g_adaptive = env_size("HBLS_ADAPTIVE", 1) != 0;
  g_single_max = env_size("HBLS_SINGLE_MAX", SINGLE_MAX_DEFAULT);
  g_dec_pair_max = env_size("HBLS_DEC_PAIR_MAX", 0);
  g_ta_pair_max = env_size("HBLS_TA_PAIR_MAX", g_ta_pair_max.load());
  g_hash_pair_max = env_size("HBLS_HASH_PAIR_MAX", g_hash_pair_max.load());
  g_hash_one_lane = env_size("HBLS_HASH_ONE_LANE", g_hash_one_lane.load());
  g_hash_split = env_size("HBLS_HASH_SPLIT", 1) != 0;
  g_fe18_max = env_size("HBLS_FE18_MAX", g_fe18_max.load());
  g_ws_sets = (int)std::min<size_t>(N_WS_MAX, std::max<size_t>(1, env_size("HBLS_WS_SETS", 3)));
  {
    size_t sc = env_size("HBLS_SIG_CACHE", g_sc_cap.load());
    while (sc & (sc - 1)) sc &= sc - 1;  // a power of two
    g_sc_cap = std::min<size_t>(sc, size_t(1) << 30);
    uint64_t k[2];
    if (getrandom(k, sizeof(k), 0) == (ssize_t)sizeof(k)) {  // otherwise the fixed key (a miss costs time only)
      g_sc_k0 = k[0];
      g_sc_k1 = k[1] | 1;
    }
  }
  std::vector<Dev*> devs;
  for (int k = 0; k < 32; k++)
    if (mask & (1u << k)) {
      Dev* d;
      if (dev_create(k, &d)) return -1;
      devs.push_back(d);
    }
  {
    std::lock_guard<std::mutex> l(g_devs_mu);
    g_devs = devs;
  }
  g_base_devs = devs;
  g_mask = mask;
  g_ready.store(true);
  return 0;
}

int ensure_init() { return g_ready.load() ? 0 : init_mask(0); }

// the device of a caller's stream (device entry points); stream 0: the first device
int dev_of_stream(hipStream_t s, Dev** out) {
  if (ensure_init()) return -1;
  const std::vector<Dev*> ds = devs();
  int ord = ds[0]->ord;
  if (s) {
    hipDevice_t dv;
    HCHK(hipStreamGetDevice(s, &dv));
    ord = (int)dv;
  }
  for (Dev* d : ds)
    if (d->ord == ord) {
      HCHK(hipSetDevice(ord));
      *out = d;
      return 0;
    }
  return set_err("stream belongs to device " + std::to_string(ord) + ", outside the library's device mask");
}

// a host call's stream and staging buffers: its context's, or the device's own (h == nullptr: the
// small entry points, which hold the device lock throughout)
inline hipStream_t call_stream(Dev& d, Hc* h) { return h ? h->s : d.stream; }
inline DevBuf* call_io(Dev& d, Hc* h) { return h ? h->io : d.io; }

template <class T>
int upload(Dev& d, IoId id, const T* src, size_t count, T** dst, Hc* h = nullptr) {
  void* p;
  if (ensure_buf(call_io(d, h)[id], count * sizeof(T), &p)) return -1;
  if (count) HCHK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, call_stream(d, h)));
  *dst = (T*)p;
  return 0;
}

// the uploads through h's pinned staging, on h's stream (never blocks the calling thread; the
// staging is reused by the context's next call only, after this one's stream synchronisation)
int upload_pinned(Dev& d, Hc& h, const PinnedUploads& u) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  size_t total = 0;
  for (const auto& it : u.items) total += al(it.bytes);
  if (total > h.pin_cap) {
    if (h.pin) HCHK(hipHostFree(h.pin));
    h.pin = nullptr;
    h.pin_cap = 0;
    const size_t cap = std::max(total + total / 4, size_t(1) << 20);
    HCHK(hipHostMalloc((void**)&h.pin, cap, hipHostMallocDefault));
    h.pin_cap = cap;
  }
  size_t o = 0;
  for (const auto& it : u.items) {
    void* p;
    if (ensure_buf(h.io[it.id], it.bytes, &p)) return -1;
    if (it.bytes) {
      memcpy(h.pin + o, it.src, it.bytes);
      HCHK(hipMemcpyAsync(p, h.pin + o, it.bytes, hipMemcpyHostToDevice, h.s));
    }
    *it.dst = p;
    o += al(it.bytes);
  }
  return 0;
}

// a context's staging buffers are free once the signature-cache put of its previous call has read
// them (a short kernel pair that started when that call's pipeline ended)
void hc_ready(Hc& h) {
  if (h.put_pending) {
    (void)hipEventSynchronize(h.put_ev);
    h.put_pending = false;
  }
}
Hc& hc_acquire(Dev& d) {
  Hc* got = nullptr;
  {
    std::unique_lock<std::mutex> lk(d.hc_mu);
    while (!got) {
      for (int k = 0; k < g_ws_sets && !got; k++)
        if (!d.hc[k].busy) {
          d.hc[k].busy = true;
          got = &d.hc[k];
        }
      if (!got) d.hc_cv.wait(lk);
    }
  }
  hc_ready(*got);
  return *got;
}
void hc_release(Dev& d, Hc& h) {
  {
    std::lock_guard<std::mutex> lk(d.hc_mu);
    h.busy = false;
  }
  d.hc_cv.notify_one();
}
// a free context or nullptr (never waits: a chunked call takes only what is idle)
Hc* hc_try_acquire(Dev& d) {
  Hc* got = nullptr;
  {
    std::lock_guard<std::mutex> lk(d.hc_mu);
    for (int k = 0; k < g_ws_sets && !got; k++)
      if (!d.hc[k].busy) {
        d.hc[k].busy = true;
        got = &d.hc[k];
      }
  }
  if (got) hc_ready(*got);
  return got;
}

// per-call random linear combination key (OS CSPRNG)
int rlc_key(RlcKey& k) {
  uint8_t* p = reinterpret_cast<uint8_t*>(k.w);
  size_t got = 0;
  while (got < sizeof(k.w)) {
    ssize_t r = getrandom(p + got, sizeof(k.w) - got, 0);
    if (r <= 0) return set_err("getrandom failed");
    got += (size_t)r;
  }
  return 0;
}

// ---------------------------------------------------------------------------------------
// Batched verification of n partials already in device memory (vbatch.hip):
//   side 0: k_dec_pk            side 1: k_dec_sig_pt
//   s:      k_item_group, k_rlc, then per chunk of groups k_group_prep -> k_pair3,
//           k_scatter, then the fallback passes (k_fb_lines -> k_pair3 over the listed items)
// Optional fold of the slot's ThresholdAggregate (reusing the decompressed partials) and of the
// post-aggregate verification under the DV keys (sigagg.go:117) into the same groups.
// ---------------------------------------------------------------------------------------
// verification statistics (HBLS_STATS=1): items, groups, items re-checked alone
std::atomic<uint64_t> g_stats[8];
bool stats_on() {
  const char* v = getenv("HBLS_STATS");
  return v && v[0] == '1';
}

struct TaFold {
  // aggregation members: verified partial src[j] (src == nullptr: decompress sigs instead)
  const uint8_t* ta_sigs;
  const uint32_t* ta_src;
  const int64_t* ta_idx;
  const uint32_t* grp_off;
  size_t n_groups, n_partials;
  uint8_t* ta_out;
  uint8_t* ta_status;
  // post-aggregate verification (nullable): DV public key per group, verdict per group
  const uint8_t* dv_pks;
  uint8_t* agg_status;
  // decompressed-key tables (hbls_decompress_pubkeys_device; nullable): used instead of
  // decompressing pks / dv_pks in this call
  const G1AEntry* pk_table;
  const uint8_t* pk_table_st;
  const G1AEntry* dv_pk_table;
  const uint8_t* dv_pk_table_st;
};


// ThresholdAggregate (mode 0) / Aggregate (mode 1) of groups whose members are already
// decompressed (pts, mst) into ta_out / ta_status; agg_pt (nullable) gets the affine results.
int ta_tail(Dev& d, Ws& w, const HmEntry* pts, const uint32_t* src, const uint8_t* mst_in, const int64_t* didx,
            const uint32_t* dgoff, size_t n_groups, size_t np, int mode, uint8_t* out, uint8_t* status,
            HmEntry* agg_pt, hipStream_t s, hipEvent_t mst_ready = nullptr, hipEvent_t pts_ready = nullptr) {
  uint8_t* mst;
  TaDigits* dig;
  void* tab;
  G2JEntry* pj;
  if (wsbuf(w, W_TAMST, np, &mst) || wsbuf(w, W_TADIG, np, &dig) || wsbuf(w, W_TAJ, np, &pj)) return -1;
  // joint ladders over chunks of a validator's members (k_ta_jtab, k_ta_jladder, k_ta_jgeneral) when every group has t members
  const size_t t_u = (n_groups && np % n_groups == 0) ? np / n_groups : 0;
  size_t jc = 0;
  if (mode == 0 && t_u > 1) {
    const size_t knob = g_ta_joint.load();
    jc = knob ? knob : np / TA_JOINT_LANES;
    jc = std::min<size_t>(std::min<size_t>(jc, t_u), 8);
    if (jc <= 1) jc = 0;
  }
  // (the joint path's guarded per-member fallback reads the same buffer: the larger of the two)
  const size_t tab_bytes = jc ? std::max(ta_joint_table_bytes((uint32_t)n_groups, (uint32_t)t_u, (uint32_t)jc),
                                         ta_table_bytes((uint32_t)np))
                              : ta_table_bytes((uint32_t)np);
  if (wsbuf(w, W_TATAB, tab_bytes, (uint8_t**)&tab)) return -1;
  if (np) {
    // t_u > 1: the joint and small-scalar paths assume groups of exactly t_u members; k_ta_layout
    // flags any other layout in nonuni (the per-member ladders then run instead)
    uint8_t* nonuni = nullptr;
    if (mode == 0 && t_u > 1) {
      if (wsbuf(w, W_TANONUNI, 1, &nonuni)) return -1;
      HCHK(hipMemsetAsync(nonuni, 0, 1, s));
      TIMED(d, "k_ta_lambda", s, launch_ta_layout(dgoff, (uint32_t)n_groups, (uint32_t)t_u, nonuni, s));
    }
    // small-scalar path first (groups of exactly t members, wave-uniform index sets); the Lagrange
    // digits and the per-member ladders below skip the groups it aggregated
    uint8_t* sdone = nullptr;
    if (mode == 0 && t_u >= 2 && t_u <= (size_t)TA_SMALL_MAX) {
      int64_t* csm;
      TaDigits* sdig;
      uint8_t *sok, *stab;
      if (wsbuf(w, W_TACSM, np, &csm) || wsbuf(w, W_TASDIG, n_groups, &sdig) || wsbuf(w, W_TASOK, n_groups, &sok) ||
          wsbuf(w, W_TASDONE, n_groups, &sdone) || wsbuf(w, W_TASTAB, ta_small_table_bytes((uint32_t)n_groups), &stab))
        return -1;
      TIMED(d, "k_ta_small", s,
            launch_ta_small(pts, src, didx, (uint32_t)n_groups, (uint32_t)t_u, csm, sdig, sok, stab, sdone, pj, s,
                            nonuni, pts_ready));
      pts_ready = nullptr;  // waited for inside, after the index-only split
    }
    if (pts_ready) HCHK(hipStreamWaitEvent(s, pts_ready, 0));
    // the members' statuses are first read by the Lagrange digits: the small-scalar ladders above
    // run on the decompressed points while their subgroup checks (mst_ready) finish; a member that
    // fails them makes its group's status and output below whatever the ladders computed
    if (mst_ready) HCHK(hipStreamWaitEvent(s, mst_ready, 0));
    if (src) launch_ta_member_status(mst_in, src, (uint32_t)np, mst, s);
    else HCHK(hipMemcpyAsync(mst, mst_in, np, hipMemcpyDeviceToDevice, s));
    HCHK(hipGetLastError());
    TIMED(d, "k_ta_lambda", s,
          launch_ta_lambda(didx, dgoff, (uint32_t)n_groups, (uint32_t)np, mode, dig, mst, s, (uint32_t)t_u, nonuni,
                           sdone));
    if (jc) {
      TIMED(d, "k_ta_straus", s,
            launch_ta_joint(pts, src, dig, (uint32_t)n_groups, (uint32_t)t_u, (uint32_t)jc, tab, pj, s, sdone, nonuni));
      // groups not all of t_u members: the per-member ladders instead (nothing unless nonuni)
      TIMED(d, "k_ta_straus", s,
            launch_ta_straus(pts, src, dig, (uint32_t)np, (uint32_t)n_groups, tab, pj, s, nullptr, nonuni));
    } else {
      TIMED(d, "k_ta_straus", s, launch_ta_straus(pts, src, dig, (uint32_t)np, (uint32_t)n_groups, tab, pj, s, sdone));
    }
  }
  TIMED(d, "k_group_sum", s,
        LAUNCH(k_group_sum, n_groups, s, dgoff, (uint32_t)n_groups, mode, (const G2JEntry*)pj, (const uint8_t*)mst,
               out, status, agg_pt));
  return 0;
}

// defer_hm / defer_msgs: the caller hashed the defer_msgs messages at defer_hm (the call's messages
// or a contiguous range of them) without their Miller lines (callers whose messages have about one
// verification group each, batched final exponentiation sizes): the slot-wide check evaluates each
// group's chain at P directly (k_lines_at_p) and the unevaluated lines are computed only behind a
// failed check; any other path computes them first.
int verify_pipeline(Dev& d, Ws& w, const uint8_t* dpk, const uint8_t* dsig, const uint32_t* didx,
                    const MsgEntry* hm, size_t n, const uint32_t* dgoff, size_t n_groups, uint8_t* dst,
                    hipStream_t s, hipEvent_t hm_ready, const TaFold* fold, bool kc = false,
                    hipEvent_t h_ready = nullptr, MsgEntry* defer_hm = nullptr, size_t defer_msgs = 0,
                    uint32_t* first_out = nullptr) {
  if (!dgoff) n_groups = n;
  G1AEntry* vpk;
  HmEntry* vsig;
  uint8_t *vpkst, *vsigst, *gst, *gver;
  uint32_t *igrp, *gmsg, *list, *count;
  G1JEntry* pr;
  G2JEntry* sr;
  G1AEntry* gP;
  LineEntry *glines, *fbl;
  const size_t gcap = std::min(std::max<size_t>(1, g_gcap.load()), std::max<size_t>(n_groups, 1));
  const size_t n_agg = (fold && fold->dv_pks) ? fold->n_groups : 0;
  const size_t fbcap = std::min(std::max<size_t>(1, g_fbcap.load()), std::max<size_t>(n + n_agg, 1));
  if (wsbuf(w, W_VPK, n, &vpk) || wsbuf(w, W_VPKST, n, &vpkst) || wsbuf(w, W_VSIG, n, &vsig) ||
      wsbuf(w, W_VSIGST, n, &vsigst) || wsbuf(w, W_IGRP, n, &igrp) || wsbuf(w, W_PR, n, &pr) ||
      wsbuf(w, W_SR, n, &sr) || wsbuf(w, W_GP, gcap, &gP) || wsbuf(w, W_GST, gcap, &gst) ||
      wsbuf(w, W_GMSG, n_groups, &gmsg) || wsbuf(w, W_GVER, n_groups, &gver) ||
      wsbuf(w, W_GLINES, gcap * N_LINES, &glines) || wsbuf(w, W_LIST, n + n_agg, &list) ||
      wsbuf(w, W_COUNT, 1, &count) || wsbuf(w, W_FBLINES, fbcap * N_LINES, &fbl))
    return -1;
  G1AEntry* apk = nullptr;
  uint8_t* apkst = nullptr;
  HmEntry* asig = nullptr;
  G1JEntry* apr = nullptr;
  G2JEntry* asr = nullptr;
  if (n_agg && (wsbuf(w, W_APK, n_agg, &apk) || wsbuf(w, W_APKST, n_agg, &apkst) ||
                wsbuf(w, W_ASIG, n_agg, &asig) || wsbuf(w, W_APR, n_agg, &apr) || wsbuf(w, W_ASR, n_agg, &asr)))
    return -1;
  RlcKey key;
  if (rlc_key(key)) return -1;
  // Coefficients: at most ONE fixed (r = 1) coefficient per combined check.  Items of a singleton
  // group keep r = 1 only when nothing else joins their group's check; with a folded aggregate
  // (which keeps r = 1 without the batched final exponentiation) every item takes a random one --
  // otherwise an error +D on a group's single partial and -D on its aggregate would cancel.
  // Batched final exponentiation: a batch of groups (FE_BATCH; behind a failed slot-wide check the
  // multi-Miller loops' chunks of mmlk groups) shares one final exponentiation and one Miller
  // loop of the signature side, checking prod_g e(P_g, H(m_g)) * e(-g1, sum_g S_g) == 1.  Every
  // item (singletons and folded aggregates included) then takes a random coefficient: with two
  // fixed coefficients in one combination, errors of two items could cancel.
  const size_t fe_min = g_fe_batch_min.load();
  const bool bfe = fe_min && n_groups >= fe_min;
  const int item_always = (bfe || n_agg) ? 1 : 0;  // see the coefficient rule above
  // First-error mode (first_out, the callers' contract: parsigex.go:93-98, sigagg.go:56-63 stop at
  // the first failing item): behind a failed combined check only the FIRST failing batch descends
  // to its groups and only the first failing group to its items -- groups and batches are in item
  // order, so every item before the first failure has passed a check and every item left
  // unresolved (ST_UNCHECKED) comes after it.  Without the batched final exponentiation every
  // group is checked anyway (exact statuses).  *first_out: the first item whose status is decided
  // and not OK (0xffffffff: none).
  if (first_out && n_agg) return set_err("verify: the first-error mode takes no folded aggregates");
  const bool first_only = first_out && bfe;
  uint32_t* wfirst = nullptr;
  if (first_only) {
    if (wsbuf(w, W_FIRST, 2, &wfirst)) return -1;
    HCHK(hipMemsetAsync(wfirst, 0xff, 2 * sizeof(uint32_t), s));
  }
  // pairs per multi-Miller loop of the slot-wide check: enough that the loops fill at most one
  // round of waves (21 groups per wave, one wave per SIMD) -- a second, partial round would double
  // the kernel's span
  const size_t mmlk = std::min<size_t>(16, std::max<size_t>(1, (std::min(gcap, n_groups) + GROUPS_PER_WAVE * 4 * d.n_cu - 1) /
                                                              (GROUPS_PER_WAVE * 4 * d.n_cu)));
  const size_t nb1 = (gcap + mmlk - 1) / mmlk, nb2 = (nb1 + PROD_FAN - 1) / PROD_FAN;
  // batches of >= 2 groups (FE_BATCH), or behind a failed slot-wide check its multi-Miller loops' chunks
  const size_t nbcap = std::max((gcap + 1) / 2, nb1);
  Fp4Entry* fbuf = nullptr;
  G2JEntry *gS = nullptr, *bS = nullptr;
  LineEntry* blines = nullptr;
  uint8_t *bbad = nullptr, *bver = nullptr;
  uint32_t *glist = nullptr, *gcount = nullptr;
  // the two factors of each final exponentiation side by side (product tree root, signature-side
  // loop), and the product tree's intermediate level
  Fp4Entry *pfin = nullptr, *tbuf = nullptr;
  if (bfe && (wsbuf(w, W_FBUF, 3 * gcap, &fbuf) || wsbuf(w, W_GS, gcap, &gS) || wsbuf(w, W_BS, nbcap, &bS) ||
              wsbuf(w, W_BLINES, nbcap * N_LINES, &blines) || wsbuf(w, W_BBAD, nbcap, &bbad) ||
              wsbuf(w, W_BVER, nbcap, &bver) || wsbuf(w, W_GLIST, gcap, &glist) || wsbuf(w, W_GCOUNT, 1, &gcount) ||
              wsbuf(w, W_PFIN, 3 * 2 * std::max<size_t>(nbcap, 1), &pfin) || wsbuf(w, W_TBUF, 3 * nbcap, &tbuf)))
    return -1;
  // Slot-wide check (msm.hip): every group of the call at once, the signature side as one
  // multi-scalar multiplication; the per-batch path below runs only if it fails (its kernels wait
  // on the device flag sfail).  Needs all groups in one chunk.
  const size_t smin = g_slot_msm_min.load();
  const bool smsm = bfe && smin && n_groups <= gcap && n + n_agg >= smin;
  G2MsmArgs ma{};
  // pbuf1: the multi-Miller loops (kept: behind a failed slot-wide check they are the per-batch
  // check's public-key sides); pbuf2 / pbuf3: the product tree's levels
  Fp4Entry *pbuf1 = nullptr, *pbuf2 = nullptr, *pbuf3 = nullptr;
  uint8_t* sfail = nullptr;
  LineEntry* mlev = nullptr;
  if (smsm && (wsbuf(w, W_MCNT, MSM_KEYS, &ma.cnt) || wsbuf(w, W_MOFF, MSM_KEYS + 1, &ma.off) ||
               wsbuf(w, W_MCUR, MSM_KEYS, &ma.cur) || wsbuf(w, W_MORDER, MSM_KEYS, &ma.order) ||
               wsbuf(w, W_MENT, 2 * MSM_WINDOWS * (n + n_agg), &ma.ent) ||
               wsbuf(w, W_MBUCKET, MSM_KEYS, &ma.bucket) || wsbuf(w, W_MPART, MSM_PARTS, &ma.part) ||
               wsbuf(w, W_MPART2, MSM_PARTS / 128, &ma.part2) || wsbuf(w, W_MTOT, 1, &ma.total) ||
               wsbuf(w, W_PBUF1, 3 * nb1, &pbuf1) || wsbuf(w, W_PBUF2, 3 * nb2, &pbuf2) ||
               wsbuf(w, W_PBUF3, 3 * nb2, &pbuf3) ||
               wsbuf(w, W_SFAIL, 2, &sfail) || wsbuf(w, W_MLEV, N_LINES * gcap, &mlev)))
    return -1;
  // adaptive: the outcome of the last completed checked call decides whether this one tries the
  // slot-wide check at all (skip: the fallback's kernels run unguarded, sfail set to 1)
  bool skip_msm = false;
  if (smsm && g_adaptive.load()) {
    while (d.res_tail != d.res_head && hipEventQuery(d.res_ev[d.res_tail % N_RES]) == hipSuccess) {
      const SlotRes& r = d.res_host[d.res_tail % N_RES];
      d.attack = r.skipped ? r.gcount != 0 : r.sfail != 0;
      d.res_tail++;
    }
    skip_msm = d.attack;
  }
  // first pass: the public-key side only when the MSM takes the other
  const int sides1 = smsm && !skip_msm ? 1 : 3;

  // fork: decompression on the side streams (after the previous verification's decompression)
  HCHK(hipEventRecord(w.ev_fork, s));
  for (int k = 0; k < 2; k++) HCHK(hipStreamWaitEvent(w.side[k], w.ev_fork, 0));
  // public keys: from the caller's decompressed-key tables when given (static per cluster lock:
  // decompressed and subgroup-checked once), else decompressed here
  if (fold && fold->pk_table) {
    vpk = const_cast<G1AEntry*>(fold->pk_table);
    vpkst = const_cast<uint8_t*>(fold->pk_table_st);
  } else if (kc && d.kc_n) {  // host-buffer call with the key cache: cached entries, the rest decompressed
    TIMED(d, "k_dec_pk", w.side[0],
          launch_pk_cached(dpk, (uint32_t)n, (const uint8_t*)d.kc_keys.p, (const G1AEntry*)d.kc_tab.p,
                           (const uint8_t*)d.kc_st.p, (const uint32_t*)d.kc_hidx.p, (uint32_t)d.kc_tcap, g_sc_k0,
                           g_sc_k1, vpk, vpkst, w.side[0]));
  } else {
    TIMED(d, "k_dec_pk", w.side[0], launch_dec_pk(dpk, (uint32_t)n, vpk, vpkst, w.side[0]));
  }
  HCHK(hipEventRecord(w.ev_pk, w.side[0]));
  if (n_agg && fold->dv_pk_table) {
    apk = const_cast<G1AEntry*>(fold->dv_pk_table);
    apkst = const_cast<uint8_t*>(fold->dv_pk_table_st);
  } else if (n_agg) {
    TIMED(d, "k_dec_pk", w.side[0], launch_dec_pk(fold->dv_pks, (uint32_t)n_agg, apk, apkst, w.side[0]));
  }
  TIMED(d, "k_dec_sig_pt", w.side[1], launch_dec_sig_pt(dsig, (uint32_t)n, vsig, vsigst, w.side[1], nullptr, w.ev_dec));
  HCHK(hipEventRecord(w.ev_side[0], w.side[0]));
  HCHK(hipEventRecord(w.ev_side[1], w.side[1]));

  // the slot's ThresholdAggregate on side 3 (needs the decompressed partials when it reuses them)
  const bool ta = fold && fold->n_groups;
  if (ta) {
    hipStream_t st = w.side[3];
    HCHK(hipStreamWaitEvent(st, w.ev_fork, 0));
    const HmEntry* pts = vsig;
    const uint8_t* mst_in = vsigst;
    hipEvent_t mst_ready = nullptr, pts_ready = nullptr;
    if (fold->ta_src) {  // the points once decompressed; their subgroup statuses before the digits
      pts_ready = w.ev_dec;
      mst_ready = w.ev_side[1];
    } else {  // the aggregation members come as their own bytes: decompress them here
      HmEntry* tpts;
      uint8_t* tdst;
      if (wsbuf(w, W_TAPTS, fold->n_partials, &tpts) || wsbuf(w, W_TADST, fold->n_partials, &tdst)) return -1;
      TIMED(d, "k_dec_sig_pt", st, launch_dec_sig_pt(fold->ta_sigs, (uint32_t)fold->n_partials, tpts, tdst, st));
      pts = tpts;
      mst_in = tdst;
    }
    if (ta_tail(d, w, pts, fold->ta_src, mst_in, fold->ta_idx, fold->grp_off, fold->n_groups, fold->n_partials, 0,
                fold->ta_out, fold->ta_status, asig, st, mst_ready, pts_ready))
      return -1;
    HCHK(hipEventRecord(w.ev_ta, st));
  }

  // random linear combinations per item, then per group (the partials' keys only: the DV keys'
  // decompression behind them on side 0 is waited for by the aggregates' combination below)
  HCHK(hipStreamWaitEvent(s, w.ev_pk, 0));
  // the partials' key side from the keys alone when the slot-wide MSM takes the signature side
  // (sides1 1, the per-lane combination): it runs beside the signatures' subgroup checks, whose
  // statuses group_scan and msm_take apply; otherwise the signatures' statuses first
  const uint32_t rlc_cmax = (uint32_t)std::min<size_t>(RLC_CHUNK, std::max<size_t>(1, n / g_rlc_lanes.load()));
  const bool keys_only = sides1 == 1 && !(dgoff && rlc_cmax > 1);
  if (!keys_only) HCHK(hipStreamWaitEvent(s, w.ev_side[1], 0));
  TIMED(d, "k_item_group", s, launch_item_group(dgoff, (uint32_t)n_groups, (uint32_t)n, igrp, s));
  RlcMsmArgs rlc_fallback{};
  uint32_t rlc_fallback_chunks = 0;
  uint2* coef_pi = nullptr;  // per-item path's coefficients (slot-wide check)
  if (dgoff && rlc_cmax > 1) {
    // chunks of a group's items share their ladders' doublings (k_rlc_msm); the chunk size keeps
    // about g_rlc_lanes lanes busy (at most RLC_CHUNK items, one item per lane for small calls)
    const uint32_t cmax = rlc_cmax;
    const size_t max_chunks = n / cmax + n_groups;
    uint32_t *pcnt, *pcoff, *pcf, *pcc;
    uint2* coef;
    uint4* coef4 = nullptr;
    G1J* t1;
    G2J* t2;
    // the sparse coefficient format (22 additions per item instead of 32) unless the slot-wide
    // bucket MSM reads the coefficients: under attack (skip_msm), or a chunked call without the
    // slot-wide check (HBLS_SLOT_MSM above its size)
    const bool sparse = !(smsm && !skip_msm);
    if (wsbuf(w, W_PCNT, n_groups, &pcnt) || wsbuf(w, W_PCOFF, n_groups + 1, &pcoff) ||
        wsbuf(w, W_PCFIRST, max_chunks, &pcf) || wsbuf(w, W_PCCOUNT, max_chunks, &pcc) ||
        wsbuf(w, W_COEF, n + n_agg, &coef) || wsbuf(w, W_RT1, 4 * n, &t1) || wsbuf(w, W_RT2, 4 * n, &t2) ||
        (sparse && wsbuf(w, W_COEF4, n, &coef4)))
      return -1;
    TIMED(d, "k_plan", s, launch_plan(dgoff, (uint32_t)n_groups, cmax, pcnt, pcoff, pcf, pcc, s));
    RlcMsmArgs ra{};
    ra.pk = vpk;
    ra.pk_st = vpkst;
    ra.sig = vsig;
    ra.sig_st = vsigst;
    ra.cfirst = pcf;
    ra.ccount = pcc;
    ra.total = pcoff + n_groups;
    ra.key_base = 0;
    ra.key = key;
    ra.coef = coef;
    ra.coef4 = coef4;
    ra.sparse = sparse ? 1 : 0;
    ra.t1 = t1;
    ra.t2 = t2;
    ra.pout = pr;
    ra.sout = sr;
    ra.always = item_always;
    ra.sides = sides1;
    TIMED(d, "k_rlc", s, launch_rlc_msm(ra, (uint32_t)max_chunks, s));
    if (smsm && !skip_msm) {  // the per-item signature side, only if the slot-wide check fails
      ra.sides = 2;
      ra.guard = sfail;
      rlc_fallback = ra;
      rlc_fallback_chunks = (uint32_t)max_chunks;
    }
  } else {
    if (smsm && wsbuf(w, W_COEF, n + n_agg, &coef_pi)) return -1;
    TIMED(d, "k_rlc", s,
          launch_rlc(vpk, vpkst, keys_only ? nullptr : vsig, keys_only ? nullptr : vsigst, igrp, dgoff, item_always,
                     (uint32_t)n, 0, key, pr, sr, s, coef_pi, sides1));
    HCHK(hipStreamWaitEvent(s, w.ev_side[1], 0));  // the groups' states below read the signatures
  }
  if (n_agg) {
    // without the batched final exponentiation the folded aggregate keeps r = 1: one coefficient
    // per combination may be fixed without losing soundness (an invalid aggregate alone fails the
    // combined check exactly; with an invalid partial j beside it the check passes for one value
    // of the random r_j only) -- the group's items all take random coefficients (item_always)
    //
    // Key side only (sides1 1, the slot-wide check's MSM takes the signature side): the DV keys
    // are all it reads, so it runs beside the slot's ThresholdAggregate; the aggregates' statuses
    // and points are applied where the signature side is read (group_scan's with_agg, msm_take)
    const bool key_only = sides1 == 1;
    if (!key_only) HCHK(hipStreamWaitEvent(s, w.ev_ta, 0));
    HCHK(hipStreamWaitEvent(s, w.ev_side[0], 0));
    uint2* acoef = smsm && !skip_msm ? (coef_pi ? coef_pi : rlc_fallback.coef) + n : nullptr;
    TIMED(d, "k_rlc", s,
          launch_rlc(apk, apkst, key_only ? nullptr : asig, key_only ? nullptr : fold->ta_status, nullptr, nullptr,
                     bfe ? 1 : 0, (uint32_t)n_agg, (uint32_t)n, key, apr, asr, s, acoef, sides1));
    HCHK(hipStreamWaitEvent(s, w.ev_ta, 0));  // the groups' states below read the aggregates
  }
  // small calls (no batched final exponentiation): the groups' sums and signature lines do not
  // need the hashed messages, so they overlap the hashing; the wait comes before the pairing
  if (hm_ready && bfe) HCHK(hipStreamWaitEvent(s, hm_ready, 0));
  if (defer_msgs && !bfe) return set_err("verify: deferred Miller lines need the batched final exponentiation");
  const bool lines_at_p = defer_msgs && smsm && !skip_msm;
  if (defer_msgs && !lines_at_p)  // the per-batch check reads the unevaluated lines
    TIMED(d, "k_lines_msg", s, launch_lines_msg(defer_hm, (uint32_t)defer_msgs, s));
  Fp4Entry* f1 = nullptr;
  uint8_t* f1bad = nullptr;
  G2JEntry* f1S = nullptr;
  if (!bfe && (wsbuf(w, W_F1, 3 * 2 * gcap, &f1) || wsbuf(w, W_F1BAD, gcap, &f1bad) || wsbuf(w, W_F1S, gcap, &f1S)))
    return -1;
  for (size_t g0 = 0; g0 < n_groups; g0 += gcap) {
    const uint32_t ng = (uint32_t)std::min(gcap, n_groups - g0);
    GroupPrepArgs ga{};
    ga.keys_only = keys_only ? 1 : 0;
    ga.grp_off = dgoff;
    ga.g0 = (uint32_t)g0;
    ga.ng = ng;
    ga.msg_idx = didx;
    ga.hm = hm;
    ga.pk = vpk;
    ga.pk_st = vpkst;
    ga.sig = vsig;
    ga.sig_st = vsigst;
    ga.pr = pr;
    ga.sr = sr;
    if (n_agg) {
      ga.agg_pk = apk;
      ga.agg_pk_st = apkst;
      ga.agg_sig = asig;
      ga.agg_st = fold->ta_status;
      ga.agg_pr = apr;
      ga.agg_sr = asr;
    }
    ga.gP = gP;
    ga.gmsg = gmsg;
    ga.gst = gst;
    ga.glines = glines;
    if (bfe) {
      const uint32_t fb = FE_BATCH;
      const uint32_t nb = (ng + fb - 1) / fb;
      ga.fe_batch = fb;
      Pair3Args pm{};
      pm.pk = gP;
      pm.pk_st = gst;
      pm.msg_idx = gmsg + g0;
      pm.hm = hm;
      pm.sig_lines = glines;
      pm.stride = ng;
      pm.n = ng;
      pm.f_out = fbuf;
      if (smsm) {
        // the groups' public-key sides and states; then beside each other: the (P_g, H(m_g))
        // Miller loops and their product tree (s), the MSM of the signature side and its lines (side 0)
        ga.p_only = 1;
        TIMED(d, "k_group_prep", s, launch_group_prep(ga, s));
        if (skip_msm) HCHK(hipMemsetAsync(sfail, 1, 1, s));  // the per-batch check runs unconditionally
        HCHK(hipEventRecord(w.ev_msm, s));
        hipStream_t sm = w.side[0];
        if (!skip_msm) {
        // the bucket counters zeroed before the wait (side 0 is idle since the keys' decompression;
        // under three slots these fills wait for free CUs: ~1 ms on the check's chain otherwise)
        HCHK(hipMemsetAsync(ma.cnt, 0, MSM_KEYS * sizeof(uint32_t), sm));
        HCHK(hipMemsetAsync(ma.cur, 0, MSM_KEYS * sizeof(uint32_t), sm));
        HCHK(hipStreamWaitEvent(sm, w.ev_msm, 0));
        ma.sig = vsig;
        ma.sig_st = vsigst;
        ma.agg_sig = asig;
        ma.agg_st = n_agg ? fold->ta_status : nullptr;
        ma.coef = coef_pi ? coef_pi : rlc_fallback.coef;
        ma.igrp = igrp;
        ma.gst = gst;
        ma.n = (uint32_t)n;
        ma.n_agg = (uint32_t)n_agg;
        TIMED(d, "k_msm_count", sm, launch_msm_count(ma, sm));
        TIMED(d, "k_msm_scan", sm, launch_scan(ma.cnt, MSM_KEYS, ma.off, sm));
        TIMED(d, "k_msm_fill", sm, launch_msm_fill(ma, sm));
        TIMED(d, "k_msm_bucket", sm, launch_msm_bucket(ma, sm));
        TIMED(d, "k_msm_reduce", sm, launch_msm_reduce(ma, sm));
        TIMED(d, "k_msm_sum", sm, launch_msm_sum(ma, sm));
        // the signature side's Miller loop, beside the multi-Miller loops and their product tree:
        // the final exponentiation's second factor, pfin[1] (lines and loop in one kernel, k_lml)
        TIMED(d, "k_pair3_mls", sm, launch_lml(ma.total, 1, pfin, 1, 1, bbad, sm));
        }
        HCHK(hipEventRecord(w.ev_side[0], sm));
        // multi-Miller loops over mmlk groups (shared squarings), then a product tree of fan-in
        // PROD_FAN down to ONE value, pfin[0] (ping-pong between pbuf1 and pbuf2): eight products
        // per level in each lane group instead of a chain of 64
        Pair3Args pp{};
        pp.pk = gP;
        pp.pk_st = gst;
        pp.msg_idx = gmsg + g0;
        pp.hm = hm;
        pp.n = (uint32_t)((ng + mmlk - 1) / mmlk);
        pp.f_range = (uint32_t)mmlk;
        pp.f_n = ng;
        pp.f_out = pbuf1;
        pp.sig_lines = mlev;
        if (lines_at_p) TIMED(d, "k_lines_at_p", s, launch_lines_at_p(pp, mlev, s));
        else TIMED(d, "k_mml_eval", s, launch_mml_eval(pp, mlev, s));
        TIMED(d, "k_pair3_mml", s, launch_pair3_mml(pp, s));
        Fp4Entry* cur = pbuf1;
        uint32_t cur_n = pp.n;
        if (!skip_msm) do {
          Pair3Args pr{};
          pr.n = (cur_n + PROD_FAN - 1) / PROD_FAN;
          pr.f_in = cur;
          pr.f_range = PROD_FAN;
          pr.f_n = cur_n;
          pr.f_out = pr.n == 1 ? pfin : (cur == pbuf2 ? pbuf3 : pbuf2);
          TIMED(d, "k_pair3_prod", s, launch_pair3_prod(pr, s));
          cur = pr.f_out;
          cur_n = pr.n;
        } while (cur_n > 1);
        HCHK(hipStreamWaitEvent(s, w.ev_side[0], 0));
        Pair3Args pf{};
        pf.pk_st = bbad;
        pf.n = 1;
        pf.f_in = pfin;
        pf.f_range = 2;
        pf.f_n = 2;
        pf.status = sfail;
        if (!skip_msm) {
          TIMED(d, "k_pair3_fin", s, launch_pair6_fin(pf, s));
          HCHK(hipMemsetAsync(sfail + 1, 0, 1, s));
          TIMED(d, "k_slot_verdict", s, launch_slot_verdict(gst, sfail, ng, gver + g0, s));
          // deferred lines: read by the per-batch check behind a failed slot-wide check and by
          // the per-item fallback of any group that was not READY (k_slot_verdict sets sfail[1])
          if (lines_at_p)
            TIMED(d, "k_lines_msg", s, launch_lines_msg(defer_hm, (uint32_t)defer_msgs, s, sfail + 1));
          // the slot-wide check failed: the per-batch check (signature sides per item and group;
          // computed in the first pass when the check was skipped)
          if (rlc_fallback_chunks) {
            TIMED(d, "k_rlc", s, launch_rlc_msm(rlc_fallback, rlc_fallback_chunks, s));
          } else {
            TIMED(d, "k_rlc", s,
                  launch_rlc(vpk, vpkst, vsig, vsigst, igrp, dgoff, 1, (uint32_t)n, 0, key, pr, sr, s, coef_pi, 2,
                             sfail));
          }
          if (n_agg)
            TIMED(d, "k_rlc", s,
                  launch_rlc(apk, apkst, asig, fold->ta_status, nullptr, nullptr, 1, (uint32_t)n_agg, (uint32_t)n,
                             key, apr, asr, s, const_cast<uint2*>(ma.coef) + n, 2, sfail));
        }
        ga.p_only = 0;
        ga.guard = sfail;
        pm.guard = sfail;
        // the per-batch check over the multi-Miller loops' chunks (mmlk consecutive groups): their
        // stored loops (pbuf1) are the batches' public-key sides, so no group's (P_g, H(m_g)) loop
        // is recomputed unless its batch fails.  Per batch: the signature sides S_g summed, the
        // lines of the sum, its loop times the stored one, one final exponentiation (3 lanes: one
        // round of waves for the chip-sized batch count, where six lanes would take two)
        const uint32_t nbm = (uint32_t)((ng + mmlk - 1) / mmlk);
        ga.gS = gS;
        ga.bS = nullptr;
        ga.fe_batch = 1;
        TIMED(d, "k_group_prep", s, launch_group_prep(ga, s));
        TIMED(d, "k_group_prep", s, launch_batch_sum(gS, ng, (uint32_t)mmlk, bS, s, sfail));
        TIMED(d, "k_slines", s, launch_slines(bS, nullptr, nullptr, nbm, blines, nbm, bbad, s, sfail));
        Pair3Args pb{};
        pb.sig_lines = blines;
        pb.stride = nbm;
        pb.n = nbm;
        pb.f_in = pbuf1;
        pb.f_range = 1;
        pb.f_n = nbm;
        pb.pk_st = bbad;
        pb.status = bver;
        pb.guard = sfail;
        TIMED(d, "k_pair3_fin", s, launch_pair3_fin(pb, s));
        HCHK(hipMemsetAsync(gcount, 0, sizeof(uint32_t), s));
        TIMED(d, "k_batch_verdict", s,
              launch_batch_verdict(gst, bver, ng, gver + g0, glist, gcount, s, sfail, (uint32_t)mmlk, wfirst,
                                   (uint32_t)g0));
        // groups of a failing batch: their own (P_g, H(m_g)) loops, then each group alone below
        pm.list = glist;
        pm.count = gcount;
        TIMED(d, "k_pair3_ml", s, launch_pair3_ml(pm, s));
        // the call's outcome for the next calls' choice (read when its event has completed)
        if (g_adaptive.load() && d.res_head - d.res_tail < N_RES) {
          const unsigned k = d.res_head % N_RES;
          d.res_host[k].skipped = skip_msm ? 1 : 0;
          HCHK(hipMemcpyAsync(&d.res_host[k].sfail, sfail, 1, hipMemcpyDeviceToHost, s));
          HCHK(hipMemcpyAsync(&d.res_host[k].gcount, gcount, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
          HCHK(hipEventRecord(d.res_ev[k], s));
          d.res_head++;
        }
      }
      if (!smsm) {  // the per-batch check of FE_BATCH groups (below the slot-wide check's size)
        ga.gS = gS;
        ga.bS = bS;
        TIMED(d, "k_group_prep", s, launch_group_prep(ga, s));
        // the (P_g, H(m_g)) Miller loops, stored unexponentiated
        TIMED(d, "k_pair3_ml", s, launch_pair3_ml(pm, s));
        // per batch: the lines of sum_g S_g, one Miller loop times the batch's stored loops, one
        // final exponentiation
        const uint8_t* guard = nullptr;
        TIMED(d, "k_slines", s, launch_slines(bS, nullptr, nullptr, nb, blines, nb, bbad, s, guard));
        // the batches' signature-side loops (pfin[2b + 1]), the product trees of their stored loops
        // (fan-in PROD_FAN, the last level into pfin[2b]), then each batch's final exponentiation
        // multiplies just the two.  All on s: with several slots in flight a side stream here would
        // share a hardware queue with another slot's long kernels (C2 24.4 vs 19.1 ms per slot)
        {
          Pair3Args ps{};
          ps.sig_lines = blines;
          ps.stride = nb;
          ps.n = nb;
          ps.f_out = pfin;
          ps.f_out_stride = 2;
          ps.f_out_off = 1;
          ps.guard = guard;
          TIMED(d, "k_pair3_mls", s, launch_pair3_mls(ps, s));
        }
        {
          const Fp4Entry* cur = fbuf;
          uint32_t cur_n = ng, span = 1;
          while (span < fb) {
            const uint32_t fan = std::min<uint32_t>(PROD_FAN, fb / span);
            Pair3Args pr{};
            pr.n = (cur_n + fan - 1) / fan;
            pr.f_in = cur;
            pr.f_range = fan;
            pr.f_n = cur_n;
            pr.guard = guard;
            span *= fan;
            if (span == fb) {
              pr.f_out = pfin;
              pr.f_out_stride = 2;
            } else {
              pr.f_out = tbuf;
            }
            TIMED(d, "k_pair3_prod", s, launch_pair3_prod(pr, s));
            cur = pr.f_out;
            cur_n = pr.n;
          }
        }
        Pair3Args pf{};
        pf.pk_st = bbad;
        pf.n = nb;
        pf.f_in = pfin;
        pf.f_range = 2;
        pf.f_n = 2 * nb;
        pf.status = bver;
        pf.guard = guard;
        TIMED(d, "k_pair3_fin", s, launch_pair6_fin(pf, s));
        // groups of a failing batch: checked one by one (their stored loop, their own S lines)
        HCHK(hipMemsetAsync(gcount, 0, sizeof(uint32_t), s));
        TIMED(d, "k_batch_verdict", s,
              launch_batch_verdict(gst, bver, ng, gver + g0, glist, gcount, s, guard, fb, wfirst, (uint32_t)g0));
      }
      TIMED(d, "k_slines", s, launch_slines(gS, glist, gcount, ng, glines, ng, nullptr, s));
      Pair3Args pg{};
      pg.sig_lines = glines;
      pg.stride = ng;
      pg.n = ng;
      pg.list = glist;
      pg.count = gcount;
      pg.f_in = fbuf;
      pg.f_range = 1;
      pg.f_n = ng;
      pg.status = gver + g0;
      TIMED(d, "k_pair3_fin", s, launch_pair3_fin(pg, s));
      continue;
    }
    ga.skip_hm = 1;
    // these calls are single Verifies and small batches, latency-bound: each group's sums (S kept
    // Jacobian, no lines), then its signature side's Miller loop -- lines produced and consumed in
    // one kernel (k_lml) -- on side stream 0 while the messages still hash; after the hashing (not
    // its lines) the (P, H(m)) loop the same way on s, beside it; then ONE six-lane final
    // exponentiation of the two stored loops (f1[2g], f1[2g + 1])
    ga.gS = f1S;
    ga.bS = nullptr;
    ga.fe_batch = 1;
    TIMED(d, "k_group_prep", s, launch_group_prep(ga, s));
    hipStream_t sl = w.side[0];
    HCHK(hipEventRecord(w.ev_msm, s));
    HCHK(hipStreamWaitEvent(sl, w.ev_msm, 0));
    TIMED(d, "k_pair3", sl, launch_lml(f1S, ng, f1, 2, 1, nullptr, sl));
    HCHK(hipEventRecord(w.ev_side[0], sl));
    if (g0 == 0 && (h_ready || hm_ready)) HCHK(hipStreamWaitEvent(s, h_ready ? h_ready : hm_ready, 0));
    LmlArgs pa{};
    pa.pk = gP;
    pa.pk_st = gst;
    pa.msg_idx = gmsg + g0;
    pa.hm = hm;
    pa.n = ng;
    pa.f_out = f1;
    pa.f_stride = 2;
    pa.bad = f1bad;
    TIMED(d, "k_pair3", s, launch_lml_p(pa, s));
    HCHK(hipStreamWaitEvent(s, w.ev_side[0], 0));
    Pair3Args pf{};
    pf.pk_st = f1bad;
    pf.n = ng;
    pf.f_in = f1;
    pf.f_range = 2;
    pf.f_n = 2 * ng;
    pf.status = gver + g0;
    TIMED(d, "k_pair3", s, launch_pair6_fin(pf, s));
  }
  // the per-item fallback reads the messages' lines (the small calls' group checks did not wait)
  if (!bfe && hm_ready && h_ready) HCHK(hipStreamWaitEvent(s, hm_ready, 0));
  HCHK(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
  ScatterArgs sa{};
  sa.n = (uint32_t)n;
  sa.item_grp = igrp;
  sa.msg_idx = didx;
  sa.hm = hm;
  sa.pk = vpk;
  sa.pk_st = vpkst;
  sa.sig = vsig;
  sa.sig_st = vsigst;
  sa.gverdict = gver;
  sa.grp_off = dgoff;
  sa.n_agg = (uint32_t)n_agg;
  if (n_agg) {
    sa.ta_status = fold->ta_status;
    sa.agg_pk = apk;
    sa.agg_pk_st = apkst;
    sa.agg_sig = asig;
    sa.agg_status = fold->agg_status;
  }
  sa.status = dst;
  sa.list = list;
  sa.count = count;
  if (first_only) {
    TIMED(d, "k_first_group", s, launch_first_group(gver, (uint32_t)n_groups, wfirst + 1, s));
    sa.first_group = wfirst + 1;
  }
  TIMED(d, "k_scatter", s, launch_scatter(sa, s));
  // fallback: every item of a failing group on its own; passes beyond the list end exit at once
  for (size_t base = 0; base < n + n_agg; base += fbcap) {
    TIMED(d, "k_fb_lines", s,
          launch_fb_lines(list, count, (uint32_t)base, (uint32_t)fbcap, vsig, asig, (uint32_t)n, fbl, s));
    Pair3Args pa{};
    pa.pk = vpk;
    pa.msg_idx = didx;
    pa.hm = hm;
    pa.sig_lines = fbl;
    pa.stride = (uint32_t)fbcap;
    pa.n = (uint32_t)fbcap;
    pa.list = list;
    pa.count = count;
    pa.base = (uint32_t)base;
    pa.n_items = (uint32_t)n;
    pa.agg_pk = apk;
    pa.agg_msg = gmsg;
    pa.status = dst;
    pa.agg_status = n_agg ? fold->agg_status : nullptr;
    TIMED(d, "k_pair3_fallback", s, launch_pair3(pa, s));
  }
  if (first_out) {
    HCHK(hipMemsetAsync(first_out, 0xff, sizeof(uint32_t), s));
    TIMED(d, "k_first_item", s, launch_first_item(dst, (uint32_t)n, first_out, s));
  }
  if (ta && !n_agg) {  // the aggregation ran beside the verification: join it
    HCHK(hipStreamWaitEvent(s, w.ev_ta, 0));
  }
  if (stats_on()) {  // HBLS_STATS=1: count the fallback items (synchronises; tests and diagnosis)
    uint32_t c = 0;
    HCHK(hipMemcpyAsync(&c, count, sizeof(c), hipMemcpyDeviceToHost, s));
    HCHK(hipStreamSynchronize(s));
    g_stats[0] += n + n_agg;
    g_stats[1] += n_groups;
    g_stats[2] += c;
    if (bfe) {  // only the last chunk's count is still in gcount: enough for the tests' sizes
      HCHK(hipMemcpyAsync(&c, gcount, sizeof(c), hipMemcpyDeviceToHost, s));
      HCHK(hipStreamSynchronize(s));
      g_stats[3] += c;
    }
    if (smsm && !skip_msm) {
      uint8_t f = 0;
      HCHK(hipMemcpyAsync(&f, sfail, 1, hipMemcpyDeviceToHost, s));
      HCHK(hipStreamSynchronize(s));
      g_stats[4] += 1;
      g_stats[5] += f ? 1 : 0;
    }
  }
  return 0;
}

// hash every distinct message to G2 (+ its Miller line chain) into hm, on stream s
int hash_messages(Dev& d, const uint8_t* dmsg, const uint64_t* doff, const uint32_t* dlen, size_t n_msgs,
                  MsgEntry* hm, hipStream_t s, bool lines = true) {
  TIMED(d, "k_hash_to_g2", s, launch_hash_to_g2(dmsg, doff, dlen, (uint32_t)n_msgs, hm, s));
  if (lines) TIMED(d, "k_lines_msg", s, launch_lines_msg(hm, (uint32_t)n_msgs, s));
  return 0;
}

// Whether a verification defers its messages' Miller lines (verify_pipeline defer_msgs): messages
// with about one group each (the chain per group is then no extra work) and the batched sizes.
bool defer_lines(size_t n_groups, size_t n_msgs) {
  const size_t fe_min = g_fe_batch_min.load();
  return fe_min && n_groups >= fe_min && n_groups <= n_msgs;
}

// ---------------------------------------------------------------------------------------
// Host-buffer calls: staging, message dedup, multi-device sharding
// ---------------------------------------------------------------------------------------
// Upload the distinct messages (library stream) and hash them; with a workspace set, the hashing
// runs on its side stream 2 (beside the decompression the verification forks next) and *ready is
// the event the verification waits on before it needs H(m).
int hash_table(Dev& d, const MsgTable& t, MsgEntry** hm_out, bool lines, Ws* w = nullptr,
               hipEvent_t* ready = nullptr, Hc* h = nullptr, hipEvent_t* h_ready = nullptr) {
  uint8_t* dmsg;
  uint64_t* doff;
  uint32_t* dlen;
  void* hm;
  if (upload(d, I_MSG, t.bytes.data(), t.bytes.size(), &dmsg, h)) return -1;
  if (upload(d, I_OFF, t.off.data(), t.off.size(), &doff, h)) return -1;
  if (upload(d, I_LEN, t.len.data(), t.len.size(), &dlen, h)) return -1;
  if (ensure_buf(call_io(d, h)[I_HM], t.len.size() * sizeof(MsgEntry), &hm)) return -1;
  hipStream_t hs = call_stream(d, h);
  if (w) {
    HCHK(hipEventRecord(w->ev_ta, hs));  // the uploads (ev_ta is free until the verification)
    hs = w->side[2];
    HCHK(hipStreamWaitEvent(hs, w->ev_ta, 0));
  }
  TIMED(d, "k_hash_to_g2", hs, launch_hash_to_g2(dmsg, doff, dlen, (uint32_t)t.len.size(), (MsgEntry*)hm, hs));
  if (w && h_ready) {
    HCHK(hipEventRecord(w->ev_h, hs));
    *h_ready = w->ev_h;
  }
  if (lines) TIMED(d, "k_lines_msg", hs, launch_lines_msg((MsgEntry*)hm, (uint32_t)t.len.size(), hs));
  if (w) {
    HCHK(hipEventRecord(w->ev_side[2], hs));
    *ready = w->ev_side[2];
  }
  *hm_out = (MsgEntry*)hm;
  return 0;
}

// Run fn(dev, shard) for each device's shard concurrently (one host thread per extra device).
int for_each_device(size_t n_units, const std::function<int(Dev&, size_t, size_t)>& fn) {
  const std::vector<Dev*> ds = devs();
  const size_t nd = std::min(ds.size(), std::max<size_t>(n_units, 1));
  if (nd <= 1) {
    Dev& d = *ds[0];
    std::lock_guard<std::mutex> lk(d.mu);
    if (hipSetDevice(d.ord) != hipSuccess) return set_err("hipSetDevice failed");
    return fn(d, 0, n_units);
  }
  std::vector<int> rc(nd, 0);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (size_t k = 0; k < nd; k++) {
    const size_t b = n_units * k / nd, e = n_units * (k + 1) / nd;
    th.emplace_back([&, k, b, e]() {
      Dev& d = *ds[k];
      std::lock_guard<std::mutex> lk(d.mu);
      if (hipSetDevice(d.ord) != hipSuccess) {
        rc[k] = -1;
        errs[k] = "hipSetDevice failed";
        return;
      }
      rc[k] = fn(d, b, e);
      if (rc[k]) errs[k] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (size_t k = 0; k < nd; k++)
    if (rc[k]) return set_err("device " + std::to_string(ds[k]->ord) + ": " + errs[k]);
  return 0;
}

// for_each_device for the heavy host-buffer calls: each device's share runs in a host-call context
// (acquired before the device lock); fn may release the lock once everything is enqueued and then
// wait for its own stream only
using HcFn = std::function<int(Dev&, Hc&, size_t, size_t, std::unique_lock<std::mutex>&)>;
int for_each_device_hc(size_t n_units, const HcFn& fn) {
  auto run = [&fn](Dev& d, size_t b, size_t e) -> int {
    Hc& h = hc_acquire(d);
    struct Rel {
      Dev& d;
      Hc& h;
      ~Rel() { hc_release(d, h); }
    } rel{d, h};
    std::unique_lock<std::mutex> lk(d.mu);
    if (hipSetDevice(d.ord) != hipSuccess) return set_err("hipSetDevice failed");
    return fn(d, h, b, e, lk);
  };
  const std::vector<Dev*> ds = devs();
  const size_t nd = std::min(ds.size(), std::max<size_t>(n_units, 1));
  if (nd <= 1) return run(*ds[0], 0, n_units);
  std::vector<int> rc(nd, 0);
  std::vector<std::string> errs(nd);
  std::vector<std::thread> th;
  for (size_t k = 0; k < nd; k++) {
    const size_t b = n_units * k / nd, e = n_units * (k + 1) / nd;
    th.emplace_back([&, k, b, e]() {
      rc[k] = run(*ds[k], b, e);
      if (rc[k]) errs[k] = g_err;
    });
  }
  for (auto& t : th) t.join();
  for (size_t k = 0; k < nd; k++)
    if (rc[k]) return set_err("device " + std::to_string(ds[k]->ord) + ": " + errs[k]);
  return 0;
}

// Verify n host-buffer items (tbls.Verify per item): items are ordered by message and grouped
// (at most g_gmax per group), the groups sharded over the devices, statuses scattered back.
// Decompress m compressed keys into entries first .. first+m-1 of d's key table (grown, keeping
// the entries before `first`).  Caller holds d.mu.
int kc_fill(Dev& d, const uint8_t* keys, size_t first, size_t m) {
  HCHK(hipSetDevice(d.ord));
  // launches enqueued earlier may still read the table: its only reader, launch_pk_cached of a
  // host-buffer verification, runs on a workspace side stream, so the library's own streams (the
  // library stream, the host-call contexts' and the workspaces' side streams) are drained before
  // any entry is rewritten or the table moves -- not the whole device: caller, torch and RCCL
  // streams keep running.  No new reader can be enqueued meanwhile (they look indices up under
  // d.mu, held here); cache adds are rare (cluster locks).
  HCHK(hipStreamSynchronize(d.stream));
  for (int k = 0; k < N_WS_MAX; k++) {
    if (d.hc[k].s) HCHK(hipStreamSynchronize(d.hc[k].s));
    for (int j = 0; j < N_SIDE; j++)
      if (d.ws[k].side[j]) HCHK(hipStreamSynchronize(d.ws[k].side[j]));
  }
  const size_t tot = first + m;
  if (d.kc_tab.cap < tot * sizeof(G1AEntry) || d.kc_st.cap < tot) {  // grow, keeping the old entries
    DevBuf nt, ns;
    void* p;
    if (ensure_buf(nt, tot * sizeof(G1AEntry), &p) || ensure_buf(ns, tot, &p)) return -1;
    if (first) {
      HCHK(hipMemcpyAsync(nt.p, d.kc_tab.p, first * sizeof(G1AEntry), hipMemcpyDeviceToDevice, d.stream));
      HCHK(hipMemcpyAsync(ns.p, d.kc_st.p, first, hipMemcpyDeviceToDevice, d.stream));
      HCHK(hipStreamSynchronize(d.stream));
    }
    if (d.kc_tab.p) HCHK(hipFree(d.kc_tab.p));
    if (d.kc_st.p) HCHK(hipFree(d.kc_st.p));
    d.kc_tab = nt;
    d.kc_st = ns;
  }
  uint8_t* dpk;
  if (upload(d, I_PK, keys, 48 * m, &dpk)) return -1;
  TIMED(d, "k_dec_pk", d.stream,
        launch_dec_pk(dpk, (uint32_t)m, (G1AEntry*)d.kc_tab.p + first, (uint8_t*)d.kc_st.p + first, d.stream));
  // the keys and the device index (grown to >= 2 x the entries: every entry re-inserted)
  if (d.kc_keys.cap < tot * 48) {
    DevBuf nk;
    void* p;
    if (ensure_buf(nk, tot * 48, &p)) return -1;
    if (first) HCHK(hipMemcpyAsync(nk.p, d.kc_keys.p, first * 48, hipMemcpyDeviceToDevice, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    if (d.kc_keys.p) HCHK(hipFree(d.kc_keys.p));
    d.kc_keys = nk;
  }
  HCHK(hipMemcpyAsync((uint8_t*)d.kc_keys.p + 48 * first, dpk, 48 * m, hipMemcpyDeviceToDevice, d.stream));
  size_t tcap = std::max<size_t>(d.kc_tcap, 1024);
  while (tcap < 2 * tot) tcap *= 2;
  size_t from = first;
  if (tcap != d.kc_tcap || first < d.kc_n) {  // a new index: every entry
    void* p;
    if (ensure_buf(d.kc_hidx, tcap * sizeof(uint32_t), &p)) return -1;
    HCHK(hipMemsetAsync(d.kc_hidx.p, 0, tcap * sizeof(uint32_t), d.stream));
    d.kc_tcap = tcap;
    from = 0;
  }
  TIMED(d, "k_kc_index", d.stream,
        launch_kc_index((const uint8_t*)d.kc_keys.p, (uint32_t)from, (uint32_t)(tot - from), (uint32_t*)d.kc_hidx.p,
                        (uint32_t)tcap, g_sc_k0, g_sc_k1, d.stream));
  HCHK(hipStreamSynchronize(d.stream));
  d.kc_n = tot;
  return 0;
}


// ---- decompressed-signature cache (Dev::sc_*; kernels in vbatch.hip).  Both run under d.mu.
// sc_ready: the device's cache at the current capacity (allocated on first use; a capacity change
// drops the old contents), false when the cache is off.
hipEvent_t sc_event(Dev& d) {
  hipEvent_t e = nullptr;
  if (!d.sc_ev_pool.empty()) {
    e = d.sc_ev_pool.back();
    d.sc_ev_pool.pop_back();
  } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    return nullptr;
  }
  return e;
}
// drop the records of completed puts and gets (wait: block until every one has completed)
void sc_prune(Dev& d, bool wait) {
  std::deque<Dev::ScPut> live_puts;
  for (Dev::ScPut& p : d.sc_inflight) {
    if (wait) (void)hipEventSynchronize(p.done);
    if (wait || hipEventQuery(p.done) == hipSuccess) {
      d.sc_ev_pool.push_back(p.pipe);
      d.sc_ev_pool.push_back(p.done);
    } else {
      live_puts.push_back(p);
    }
  }
  d.sc_inflight.swap(live_puts);
  std::vector<hipEvent_t> live;
  for (hipEvent_t e : d.sc_gets) {
    if (wait) (void)hipEventSynchronize(e);
    if (wait || hipEventQuery(e) == hipSuccess) d.sc_ev_pool.push_back(e);
    else live.push_back(e);
  }
  d.sc_gets.swap(live);
}
bool sc_ready(Dev& d, bool alloc) {
  const size_t cap = g_sc_cap.load();
  if (cap == 0) return false;
  if (d.sc_cap == cap) return true;
  if (!alloc) return false;
  sc_prune(d, true);  // the buffers may be reallocated: nothing may still use them
  void* p;
  if (ensure_buf(d.sc_key, cap * 96, &p) || ensure_buf(d.sc_ent, cap * sizeof(HmEntry), &p) ||
      ensure_buf(d.sc_st, cap, &p) || ensure_buf(d.sc_tab, 2 * cap * sizeof(uint32_t), &p))
    return false;
  if (hipMemset(d.sc_tab.p, 0, 2 * cap * sizeof(uint32_t)) != hipSuccess) return false;
  d.sc_cap = cap;
  d.sc_cursor = d.sc_filled = 0;
  return true;
}
// After a Verify batch's pipeline on s: its m signatures (bytes in group order, sig: in the staging
// buffers of the host-call context `owner`) and their decompressed points and statuses (pts, st:
// the verification's workspace w) enter the ring on the owner's put stream; the workspace is
// released behind the put -- or on s when nothing is put -- and the owner's next call waits for it
// (hc_ready).
int sc_put_release(Dev& d, Ws& w, const uint8_t* sig, const HmEntry* pts, const uint8_t* st, size_t m, hipStream_t s,
                   Hc& owner) {
  if (!m || !sc_ready(d, true)) return ws_release(w, s);
  const size_t cap = d.sc_cap;
  if (m > cap) {  // only the last cap items fit
    sig += 96 * (m - cap);
    pts += m - cap;
    st += m - cap;
    m = cap;
  }
  sc_prune(d, false);
  if (!owner.put_s) HCHK(hipStreamCreateWithFlags(&owner.put_s, hipStreamNonBlocking));
  if (!owner.put_ev) HCHK(hipEventCreateWithFlags(&owner.put_ev, hipEventDisableTiming));
  hipStream_t ps = owner.put_s;
  hipEvent_t pipe = sc_event(d), done = sc_event(d);
  if (!pipe || !done) return set_err("signature cache: no event");
  HCHK(hipEventRecord(pipe, s));
  HCHK(hipStreamWaitEvent(ps, pipe, 0));
  for (hipEvent_t g : d.sc_gets) HCHK(hipStreamWaitEvent(ps, g, 0));
  // an in-flight put [q, q + mq) (absolute positions, before this one's [P, P + m)) shares ring
  // entries with this one only if some position of this one lies a whole ring after one of its:
  // P + m - 1 - q >= cap (only when more than the ring is in flight)
  for (const Dev::ScPut& p : d.sc_inflight)
    if (p.pos + cap < d.sc_pos + m) HCHK(hipStreamWaitEvent(ps, p.done, 0));
  TIMED(d, "k_sc_put", ps,
        launch_sc_put(sig, pts, st, (uint32_t)m, (uint32_t)d.sc_cursor, (uint32_t)cap, d.sc_key.p, (HmEntry*)d.sc_ent.p,
                      (uint8_t*)d.sc_st.p, (uint32_t*)d.sc_tab.p, (uint32_t)(2 * cap), g_sc_k0, g_sc_k1, ps));
  HCHK(hipEventRecord(done, ps));
  // sig lives in the owner context's staging buffers: its next call waits for this put
  HCHK(hipEventRecord(owner.put_ev, ps));
  owner.put_pending = true;
  d.sc_inflight.push_back({d.sc_cursor, m, d.sc_pos, pipe, done});
  d.sc_cursor = (d.sc_cursor + m) & (cap - 1);
  d.sc_pos += m;
  d.sc_filled = std::min(cap, d.sc_filled + m);
  return ws_release(w, ps);
}
// before an aggregation's decompression: the cached points of its n members into pts / st, hit[i]
// set for those (k_dec_sig_pt then skips them).  Returns whether the cache was consulted.  Never
// waits for a Verify still in its pipeline: the entries its put will write are misses.
bool sc_get(Dev& d, const uint8_t* sig, size_t n, HmEntry* pts, uint8_t* st, uint8_t* hit, hipStream_t s) {
  if (!n || !d.sc_filled || !sc_ready(d, false)) return false;
  sc_prune(d, false);
  // puts whose pipeline is done: wait for them; the others: their span is a range of misses
  uint64_t busy_first = 0, busy_end = 0;
  bool busy = false;
  for (const Dev::ScPut& p : d.sc_inflight) {
    if (hipEventQuery(p.pipe) == hipSuccess) {
      if (hipStreamWaitEvent(s, p.done, 0) != hipSuccess) return false;
      continue;
    }
    if (!busy) busy_first = p.pos;
    busy = true;
    busy_end = p.pos + p.m;
  }
  size_t busy_lo = 0, busy_len = 0;
  if (busy) {
    if (busy_end - busy_first >= d.sc_cap) return false;  // every entry may be rewritten
    busy_lo = (size_t)(busy_first & (d.sc_cap - 1));
    busy_len = (size_t)(busy_end - busy_first);
  }
  hipEvent_t e = sc_event(d);
  if (!e) return false;
  TIMED(d, "k_sc_get", s,
        launch_sc_get(sig, (uint32_t)n, d.sc_key.p, (const HmEntry*)d.sc_ent.p, (const uint8_t*)d.sc_st.p,
                      (const uint32_t*)d.sc_tab.p, (uint32_t)(2 * d.sc_cap), g_sc_k0, g_sc_k1, pts, st, hit,
                      (uint32_t)d.sc_cap, (uint32_t)busy_lo, (uint32_t)busy_len, s));
  if (hipEventRecord(e, s) != hipSuccess) return false;
  d.sc_gets.push_back(e);
  return true;
}

// HBLS_HOST_TIMING=1: phases of a host-buffer Verify batch on stderr (diagnosis)
static bool host_timing() {
  static const bool on = [] {
    const char* v = getenv("HBLS_HOST_TIMING");
    return v && v[0] == '1';
  }();
  return on;
}
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A large one-device Verify batch.  Its keys and signatures go up in the caller's order while the
// host groups them (message dedup and sort, ~7-12 ms for a slot's million partials: beside the
// PCIe upload instead of in front of it); then the groups run in chunks of whole groups, each on
// its own host-call context (stream) and workspace set, so that -- like consecutive slots in
// flight -- one chunk's gather, decompression and hashing overlap the previous chunk's pairings
// and latency-bound tail.  Each chunk gathers its items in group order on the device
// (k_gather_items), hashes its own contiguous range of the message table (items are sorted by
// message; chunks only when every message has one group), verifies, enters its signatures into
// the signature cache and scatters its statuses into the call's status array, downloaded once.
// Extra contexts are taken only if idle (hc_try_acquire).
constexpr size_t CHUNK_MIN_ITEMS = size_t(1) << 18;
int verify_large(Dev& d, const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                 const uint32_t* msg_len, size_t n, uint8_t* status) {
  const double t_start = now_ms();
  Hc& h0 = hc_acquire(d);
  struct Rel0 {
    Dev& d;
    Hc& h;
    ~Rel0() { hc_release(d, h); }
  } rel0{d, h0};
  std::unique_lock<std::mutex> lk(d.mu);
  if (hipSetDevice(d.ord) != hipSuccess) return set_err("hipSetDevice failed");
  const double t_locked0 = now_ms();
  // 1. keys and signatures up in the caller's order
  uint8_t *rpk, *rsig;
  if (upload(d, I_PK, pks, 48 * n, &rpk, &h0) || upload(d, I_SIG, sigs, 96 * n, &rsig, &h0)) return -1;
  lk.unlock();
  const double t_up = now_ms();
  // 2. the grouping on the host, beside the upload: message ids, items ordered by message (a
  // counting sort), groups of <= g_gmax items over one message
  MsgTable all;
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw >= 4)
    dedup_messages_par(msgs, msg_off, msg_len, n, all, hw >= 8 ? 8u : 4u);
  else
    dedup_messages(msgs, msg_off, msg_len, n, nullptr, all);
  const size_t nm = all.len.size();
  std::vector<uint32_t> order32(n), mstart(nm + 1, 0);
  for (size_t k = 0; k < n; k++) mstart[all.idx[k] + 1]++;
  for (size_t j = 0; j < nm; j++) mstart[j + 1] += mstart[j];
  for (size_t k = 0; k < n; k++) order32[mstart[all.idx[k]]++] = (uint32_t)k;
  std::vector<size_t> gstart;
  std::vector<uint32_t> midx(n);
  for (size_t k = 0; k < n; k++) {
    midx[k] = all.idx[order32[k]];
    if (k == 0 || midx[k] != midx[k - 1] || k - gstart.back() >= g_gmax.load()) gstart.push_back(k);
  }
  const size_t n_groups = gstart.size();
  gstart.push_back(n);
  const bool defer = defer_lines(n_groups, nm);
  // chunks (one per idle context, messages of one group each) at group starts, ~n / K items each
  std::vector<Hc*> hcs{&h0};
  const size_t k_want = defer ? std::min<size_t>((size_t)g_ws_sets, std::max<size_t>(1, n / CHUNK_MIN_ITEMS)) : 1;
  while (hcs.size() < k_want) {
    Hc* x = hc_try_acquire(d);
    if (!x) break;
    hcs.push_back(x);
  }
  struct RelExtra {
    Dev& d;
    std::vector<Hc*>& h;
    ~RelExtra() {
      for (size_t c = 1; c < h.size(); c++) hc_release(d, *h[c]);
    }
  } rel{d, hcs};
  const size_t K = hcs.size();
  std::vector<size_t> cg{0};
  for (size_t c = 1; c < K; c++) {
    const size_t g = (size_t)(std::lower_bound(gstart.begin(), gstart.begin() + n_groups, n * c / K) - gstart.begin());
    if (g > cg.back() && g < n_groups) cg.push_back(g);
  }
  cg.push_back(n_groups);
  // the chunks' group offsets, concatenated (chunk c's at goff_base[c])
  std::vector<uint32_t> goffs;
  std::vector<size_t> goff_base;
  for (size_t c = 0; c + 1 < cg.size(); c++) {
    goff_base.push_back(goffs.size());
    for (size_t g = cg[c]; g <= cg[c + 1]; g++) goffs.push_back((uint32_t)(gstart[g] - gstart[cg[c]]));
  }
  const double t_grouped = now_ms();
  lk.lock();
  const double t_locked = now_ms();
  // 3. the grouping up (pinned: queued behind the raw upload without waiting for it), then the chunks
  uint32_t *dord, *dmidx, *dlen, *dgoffs;
  uint8_t* dmsg;
  uint64_t* doff;
  void *hmp, *stp, *gp;
  PinnedUploads up;
  up.add(I_IDX, order32.data(), n, &dord);
  up.add(I_MIDX, midx.data(), n, &dmidx);
  up.add(I_MSG, all.bytes.data(), all.bytes.size(), &dmsg);
  up.add(I_OFF, all.off.data(), all.off.size(), &doff);
  up.add(I_LEN, all.len.data(), all.len.size(), &dlen);
  up.add(I_VGOFF, goffs.data(), goffs.size(), &dgoffs);
  if (upload_pinned(d, h0, up) || ensure_buf(h0.io[I_HM], nm * sizeof(MsgEntry), &hmp) ||
      ensure_buf(h0.io[I_HM2], n, &stp) || ensure_buf(h0.io[I_OUT], 144 * n, &gp))
    return -1;
  MsgEntry* hm = (MsgEntry*)hmp;
  uint8_t* dst_out = (uint8_t*)stp;
  uint8_t *gpk = (uint8_t*)gp, *gsig = gpk + 48 * n;  // group order
  HCHK(hipEventRecord(h0.ev, h0.s));
  for (size_t c = 0; c + 1 < cg.size(); c++) {
    Hc& hc = *hcs[c];
    hipStream_t sc = hc.s;
    if (c) HCHK(hipStreamWaitEvent(sc, h0.ev, 0));
    const size_t ib = gstart[cg[c]], m = gstart[cg[c + 1]] - ib, ng = cg[c + 1] - cg[c];
    // the chunk's messages: all of them for one chunk, else its contiguous range
    const size_t mfirst = K == 1 ? 0 : midx[ib], mcount = K == 1 ? nm : midx[ib + m - 1] + 1 - midx[ib];
    // deferred lines per chunk: verify_pipeline decides its batched final exponentiation from the
    // chunk's own group count, so a chunk below that size computes its lines here
    const bool cdefer = defer && defer_lines(ng, mcount);
    Ws& w = ws_acquire(d, sc);
    void* sio;
    if (ensure_buf(hc.io[I_STAT], m, &sio)) return -1;
    uint8_t* dst = (uint8_t*)sio;
    uint8_t *cpk = gpk + 48 * ib, *csig = gsig + 96 * ib;
    LAUNCH(k_gather_items, m, sc, (const uint4*)rpk, (const uint4*)rsig, dord + ib, (uint32_t)m, (uint4*)cpk,
           (uint4*)csig);
    HCHK(hipEventRecord(w.ev_ta, sc));
    hipStream_t hs = w.side[2];
    HCHK(hipStreamWaitEvent(hs, w.ev_ta, 0));
    TIMED(d, "k_hash_to_g2", hs, launch_hash_to_g2(dmsg, doff + mfirst, dlen + mfirst, (uint32_t)mcount, hm + mfirst, hs));
    HCHK(hipEventRecord(w.ev_h, hs));
    if (!cdefer) TIMED(d, "k_lines_msg", hs, launch_lines_msg(hm + mfirst, (uint32_t)mcount, hs));
    HCHK(hipEventRecord(w.ev_side[2], hs));
    // the key cache is looked up on the device (k_pk_cached): its tables are only rewritten under
    // Dev::mu, held while this call enqueues, after every launch that may still read them
    if (verify_pipeline(d, w, cpk, csig, dmidx + ib, hm, m, dgoffs + goff_base[c], ng, dst, sc, w.ev_side[2], nullptr,
                        true, w.ev_h, hm + mfirst, cdefer ? mcount : 0))
      return -1;
    {  // the decompressed partials into the signature cache (the aggregation of these partials reads them)
      HmEntry* vsig;
      uint8_t* vsigst;
      if (wsbuf(w, W_VSIG, m, &vsig) || wsbuf(w, W_VSIGST, m, &vsigst) ||
          sc_put_release(d, w, csig, vsig, vsigst, m, sc, h0))
        return -1;
    }
    LAUNCH(k_scatter_status, m, sc, dst, dord + ib, (uint32_t)m, dst_out);
    if (c) {
      HCHK(hipEventRecord(hc.ev, sc));
      HCHK(hipStreamWaitEvent(h0.s, hc.ev, 0));
    }
  }
  lk.unlock();  // enqueued: other callers may enqueue while this one waits
  const double t_enq = now_ms();
  HCHK(hipMemcpyAsync(status, dst_out, n, hipMemcpyDeviceToHost, h0.s));
  HCHK(hipStreamSynchronize(h0.s));
  if (host_timing())
    fprintf(stderr, "hbls verify_large n=%zu chunks=%zu: lock %.2f ms, upload enqueue %.2f, grouping %.2f (beside the "
            "upload), lock wait %.2f, enqueue %.2f, device %.2f\n", n, cg.size() - 1, t_locked0 - t_start,
            t_up - t_locked0, t_grouped - t_up, t_locked - t_grouped, t_enq - t_locked, now_ms() - t_enq);
  return 0;
}

int verify_host(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                const uint32_t* msg_len, size_t n, uint8_t* status) {
  if (n == 0) return 0;
  if (n >= 0xffffffffull) return set_err("verify batch: too many items");
  {
    const std::vector<Dev*> ds = devs();
    if (ds.size() == 1 && n >= 2 * CHUNK_MIN_ITEMS && g_ws_sets > 1)
      return verify_large(*ds[0], pks, sigs, msgs, msg_off, msg_len, n, status);
  }
  const double t_start = now_ms();
  // global message ids, order items by (message, position), groups of <= g_gmax
  MsgTable all;
  const unsigned hw = std::thread::hardware_concurrency();
  if (n >= (1u << 16) && hw >= 4)
    dedup_messages_par(msgs, msg_off, msg_len, n, all, hw >= 8 ? 8u : 4u);
  else
    dedup_messages(msgs, msg_off, msg_len, n, nullptr, all);
  // items ordered by message id, stable (a counting sort: one pass, no comparisons)
  std::vector<size_t> order(n), mstart(all.len.size() + 1, 0);
  for (size_t k = 0; k < n; k++) mstart[all.idx[k] + 1]++;
  for (size_t j = 0; j < all.len.size(); j++) mstart[j + 1] += mstart[j];
  for (size_t k = 0; k < n; k++) order[mstart[all.idx[k]]++] = k;
  // a call below the batched final exponentiation's size (the latency-bound small calls, e.g. the
  // coalesced single-item callers) checks every item alone: a group of several items needs random
  // coefficients, i.e. a 64-bit scalar ladder per item on the call's critical path (~3.7 ms for a
  // lone lane), where separate checks only add lanes to kernels that have them to spare
  // (HBLS_SINGLE_MAX at init, hbls_single_max at run time: items below which every item is its own
  // group; default the batched final exponentiation's group threshold)
  const size_t sm = g_single_max.load();
  const size_t single_max = sm == SINGLE_MAX_DEFAULT ? g_fe_batch_min.load() : sm;
  const size_t gmax = n < single_max ? 1 : std::max<size_t>(1, g_gmax.load());
  std::vector<size_t> gstart;  // group starts in `order`
  for (size_t k = 0; k < n; k++)
    if (k == 0 || all.idx[order[k]] != all.idx[order[k - 1]] || k - gstart.back() >= gmax) gstart.push_back(k);
  const size_t n_groups = gstart.size();
  gstart.push_back(n);
  if (n >= 0xffffffffull) return set_err("verify batch: too many items");
  std::vector<uint32_t> order32(order.begin(), order.end());
  const double t_grouped = now_ms();
  return for_each_device_hc(n_groups, [&](Dev& d, Hc& h, size_t gb, size_t ge, std::unique_lock<std::mutex>& lk) -> int {
    const size_t ib = gstart[gb], ie = gstart[ge], m = ie - ib;
    if (m == 0) return 0;
    const bool whole = gb == 0 && ge == n_groups;
    // host preparation without the device lock (other callers enqueue meanwhile): the shard's
    // distinct messages and each item's message index in group order -- the whole call's table
    // when one device takes every group
    lk.unlock();
    MsgTable tl;
    std::vector<uint32_t> midx;
    if (whole) {
      midx.resize(m);
      for (size_t k = 0; k < m; k++) midx[k] = all.idx[order[k]];
    } else {
      dedup_messages(msgs, msg_off, msg_len, m, order.data() + ib, tl);
    }
    const MsgTable& t = whole ? all : tl;
    const std::vector<uint32_t>& tidx = whole ? midx : tl.idx;
    std::vector<uint8_t> hpk, hsig;  // several devices: each uploads only its shard, in group order
    if (!whole) {
      hpk.resize(48 * m);
      hsig.resize(96 * m);
      for (size_t k = 0; k < m; k++) {
        memcpy(&hpk[48 * k], pks + 48 * order[ib + k], 48);
        memcpy(&hsig[96 * k], sigs + 96 * order[ib + k], 96);
      }
    }
    std::vector<uint32_t> goff(ge - gb + 1);
    for (size_t g = gb; g <= ge; g++) goff[g - gb] = (uint32_t)(gstart[g] - ib);
    const double t_prep = now_ms();
    lk.lock();
    const double t_locked = now_ms();
    // the messages hash on a side stream while the keys and signatures decompress (latency of
    // one call: the two chains run side by side)
    Ws& w = ws_acquire(d, h.s);
    MsgEntry* hm;
    hipEvent_t hm_ready = nullptr, h_ready = nullptr;
    const bool defer = defer_lines(ge - gb, t.len.size());
    if (hash_table(d, t, &hm, !defer, &w, &hm_ready, &h, &h_ready)) return -1;
    uint8_t *dpk, *dsig, *dst, *dst_out = nullptr;
    uint32_t *didx, *dgoff, *dord = nullptr;
    if (whole) {  // caller order up, group order on the device
      uint8_t *rpk, *rsig;
      void *p1, *p2, *p3;
      if (upload(d, I_PK, pks, 48 * m, &rpk, &h) || upload(d, I_SIG, sigs, 96 * m, &rsig, &h) ||
          upload(d, I_IDX, order32.data(), m, &dord, &h) || ensure_buf(h.io[I_OUT], 144 * m, &p1) ||
          ensure_buf(h.io[I_HM2], m, &p2) || ensure_buf(h.io[I_STAT], m, &p3))
        return -1;
      dpk = (uint8_t*)p1;
      dsig = dpk + 48 * m;
      dst_out = (uint8_t*)p2;
      dst = (uint8_t*)p3;
      LAUNCH(k_gather_items, m, h.s, (const uint4*)rpk, (const uint4*)rsig, dord, (uint32_t)m, (uint4*)dpk,
             (uint4*)dsig);
    } else {
      void* p;
      if (upload(d, I_PK, hpk.data(), hpk.size(), &dpk, &h) || upload(d, I_SIG, hsig.data(), hsig.size(), &dsig, &h) ||
          ensure_buf(h.io[I_STAT], m, &p))
        return -1;
      dst = (uint8_t*)p;
    }
    if (upload(d, I_MIDX, tidx.data(), m, &didx, &h) || upload(d, I_VGOFF, goff.data(), goff.size(), &dgoff, &h))
      return -1;
    // the key cache is looked up on the device (k_pk_cached): its tables are only rewritten under
    // Dev::mu, held while this call enqueues, after every launch that may still read them
    if (verify_pipeline(d, w, dpk, dsig, didx, hm, m, dgoff, ge - gb, dst, h.s, hm_ready, nullptr, true, h_ready, hm,
                        defer ? t.len.size() : 0))
      return -1;
    {  // the decompressed partials into the signature cache (the aggregation of these partials reads them)
      HmEntry* vsig;
      uint8_t* vsigst;
      if (wsbuf(w, W_VSIG, m, &vsig) || wsbuf(w, W_VSIGST, m, &vsigst) ||
          sc_put_release(d, w, dsig, vsig, vsigst, m, h.s, h))
        return -1;
    }
    if (whole) LAUNCH(k_scatter_status, m, h.s, dst, dord, (uint32_t)m, dst_out);
    lk.unlock();  // enqueued: other callers may enqueue while this one waits for its stream
    const double t_enq = now_ms();
    if (whole) {
      HCHK(hipMemcpyAsync(status, dst_out, m, hipMemcpyDeviceToHost, h.s));
      HCHK(hipStreamSynchronize(h.s));
      if (host_timing())
        fprintf(stderr, "hbls verify_host n=%zu: group %.2f ms, prep %.2f, lock wait %.2f, enqueue+upload %.2f, device %.2f\n",
                n, t_grouped - t_start, t_prep - t_grouped, t_locked - t_prep, t_enq - t_locked, now_ms() - t_enq);
      return 0;
    }
    std::vector<uint8_t> hst(m);
    HCHK(hipMemcpyAsync(hst.data(), dst, m, hipMemcpyDeviceToHost, h.s));
    HCHK(hipStreamSynchronize(h.s));
    for (size_t k = 0; k < m; k++) status[order[ib + k]] = hst[k];
    return 0;
  });
}

// First-error Verify of an ordered set (hbls_verify_batch_first_error): the callers' loops that
// stop at their first failing item -- parsigex verifies a peer's set and drops it on the first
// bad partial (core/parsigex/parsigex.go:93-98), sigagg returns on the first failure
// (core/sigagg/sigagg.go:56-63), validatorapi on the first bad submission
// (core/validatorapi/validatorapi.go:302-306).  Groups are runs of consecutive items over one
// message in the caller's order (at most g_gmax items), so batches and groups are in item order
// and verify_pipeline's first-error mode resolves only the first failing batch's groups and the
// first failing group's items: under attack O(groups / batch + batch + group) checks instead of
// one per item of every failing group.  One device (the order must not be split).
int verify_first_host(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                      const uint32_t* msg_len, size_t n, int64_t* first, uint8_t* first_status, uint8_t* status) {
  *first = -1;
  if (first_status) *first_status = ST_OK;
  if (n == 0) return 0;
  if (n >= 0xffffffffull) return set_err("verify first error: too many items");
  MsgTable all;
  const unsigned hw = std::thread::hardware_concurrency();
  if (n >= (1u << 16) && hw >= 4)
    dedup_messages_par(msgs, msg_off, msg_len, n, all, hw >= 8 ? 8u : 4u);
  else
    dedup_messages(msgs, msg_off, msg_len, n, nullptr, all);
  std::vector<uint32_t> goff;
  for (size_t k = 0; k < n; k++)
    if (k == 0 || all.idx[k] != all.idx[k - 1] || k - goff.back() >= std::max<size_t>(1, g_gmax.load()))
      goff.push_back((uint32_t)k);
  const size_t n_groups = goff.size();
  goff.push_back((uint32_t)n);
  Dev& d = *devs()[0];
  Hc& h = hc_acquire(d);
  struct Rel {
    Dev& d;
    Hc& h;
    ~Rel() { hc_release(d, h); }
  } rel{d, h};
  std::unique_lock<std::mutex> lk(d.mu);
  if (hipSetDevice(d.ord) != hipSuccess) return set_err("hipSetDevice failed");
  Ws& w = ws_acquire(d, h.s);
  MsgEntry* hm;
  hipEvent_t hm_ready = nullptr, h_ready = nullptr;
  const bool defer = defer_lines(n_groups, all.len.size());
  if (hash_table(d, all, &hm, !defer, &w, &hm_ready, &h, &h_ready)) return -1;
  uint8_t *dpk, *dsig;
  uint32_t *didx, *dgoff;
  void *pst, *pfirst;
  if (upload(d, I_PK, pks, 48 * n, &dpk, &h) || upload(d, I_SIG, sigs, 96 * n, &dsig, &h) ||
      upload(d, I_MIDX, all.idx.data(), n, &didx, &h) || upload(d, I_VGOFF, goff.data(), goff.size(), &dgoff, &h) ||
      ensure_buf(h.io[I_STAT], n, &pst) || ensure_buf(h.io[I_HM2], sizeof(uint32_t), &pfirst))
    return -1;
  uint8_t* dst = (uint8_t*)pst;
  uint32_t* dfirst = (uint32_t*)pfirst;
  if (verify_pipeline(d, w, dpk, dsig, didx, hm, n, dgoff, n_groups, dst, h.s, hm_ready, nullptr, true, h_ready, hm,
                      defer ? all.len.size() : 0, dfirst))
    return -1;
  {  // the decoded signatures enter the signature cache as after hbls_verify_batch
    HmEntry* vsig;
    uint8_t* vsigst;
    if (wsbuf(w, W_VSIG, n, &vsig) || wsbuf(w, W_VSIGST, n, &vsigst) || sc_put_release(d, w, dsig, vsig, vsigst, n, h.s, h))
      return -1;
  }
  lk.unlock();
  uint32_t f = 0;
  std::vector<uint8_t> own;
  uint8_t* hst = status;
  if (!hst) {
    own.resize(n);
    hst = own.data();
  }
  HCHK(hipMemcpyAsync(&f, dfirst, sizeof(f), hipMemcpyDeviceToHost, h.s));
  HCHK(hipMemcpyAsync(hst, dst, n, hipMemcpyDeviceToHost, h.s));
  HCHK(hipStreamSynchronize(h.s));
  if (f != 0xffffffffu) {
    if (f >= n) return set_err("verify first error: index out of range");
    *first = (int64_t)f;
    if (first_status) *first_status = hst[f];
  }
  return 0;
}

int check_offsets(const uint32_t* grp_off, size_t n_groups) {
  if (grp_off[0] != 0) return set_err("grp_off[0] must be 0");
  for (size_t g = 0; g < n_groups; g++)
    if (grp_off[g + 1] < grp_off[g]) return set_err("grp_off must be non-decreasing");
  return 0;
}

// ThresholdAggregate (mode 0) / Aggregate (mode 1) of host-buffer groups, sharded over devices
int group_op_host(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups, int mode,
                  uint8_t* out, uint8_t* status) {
  if (check_offsets(grp_off, n_groups)) return -1;
  const double t_start = now_ms();
  return for_each_device_hc(n_groups, [&](Dev& d, Hc& h, size_t gb, size_t ge, std::unique_lock<std::mutex>& lk) -> int {
    const size_t ng = ge - gb, pb = grp_off[gb], np = grp_off[ge] - pb;
    if (ng == 0) return 0;
    const double t_locked = now_ms();
    std::vector<uint32_t> goff(ng + 1);
    for (size_t g = 0; g <= ng; g++) goff[g] = grp_off[gb + g] - (uint32_t)pb;
    uint8_t* dsig;
    int64_t* didx = nullptr;
    uint32_t* dgoff;
    if (upload(d, I_SIG, sigs + 96 * pb, np * 96, &dsig, &h)) return -1;
    if (mode == 0 && upload(d, I_IDX, idx + pb, np, &didx, &h)) return -1;
    if (upload(d, I_GOFF, goff.data(), ng + 1, &dgoff, &h)) return -1;
    void *dout, *dst;
    if (ensure_buf(h.io[I_OUT], ng * 96, &dout) || ensure_buf(h.io[I_STAT], ng, &dst)) return -1;
    Ws& w = ws_acquire(d, h.s);
    HmEntry* pts;
    uint8_t *mst0, *hit = nullptr;
    if (wsbuf(w, W_TAPTS, np, &pts) || wsbuf(w, W_TADST, np, &mst0)) return -1;
    // members verified by an earlier host-buffer Verify batch come from the signature cache; the
    // rest are decompressed (the same kernels, so the same points and statuses)
    if (mode == 0 && np && d.sc_filled) {
      if (wsbuf(w, W_TAHIT, np, &hit)) return -1;
      if (!sc_get(d, dsig, np, pts, mst0, hit, h.s)) hit = nullptr;
    }
    if (np) TIMED(d, "k_dec_sig_pt", h.s, launch_dec_sig_pt(dsig, (uint32_t)np, pts, mst0, h.s, hit));
    if (ta_tail(d, w, pts, nullptr, mst0, didx, dgoff, ng, np, mode, (uint8_t*)dout, (uint8_t*)dst, nullptr, h.s))
      return -1;
    // diagnosis (HBLS_STATS / HBLS_HOST_TIMING): the cache's hit flags, copied on the call's stream
    // before the workspace holding them is released to other callers
    std::vector<uint8_t> hh;
    if (hit && (host_timing() || stats_on())) {
      hh.resize(np);
      HCHK(hipMemcpyAsync(hh.data(), hit, np, hipMemcpyDeviceToHost, h.s));
    }
    if (ws_release(w, h.s)) return -1;
    lk.unlock();  // enqueued: other callers may enqueue while this one waits for its stream
    const double t_enq = now_ms();
    HCHK(hipMemcpyAsync(out + 96 * gb, dout, ng * 96, hipMemcpyDeviceToHost, h.s));
    HCHK(hipMemcpyAsync(status + gb, dst, ng, hipMemcpyDeviceToHost, h.s));
    HCHK(hipStreamSynchronize(h.s));
    size_t hits = 0;
    if (!hh.empty()) {
      for (uint8_t x : hh) hits += x;
      g_stats[6] += np;
      g_stats[7] += hits;
    }
    if (host_timing()) {
      fprintf(stderr, "hbls group_op mode=%d groups=%zu members=%zu cache=%d hits=%zu: lock wait %.2f ms, enqueue+upload "
              "%.2f, device %.2f\n", mode, ng, np, hit ? 1 : 0, hits, t_locked - t_start, t_enq - t_locked,
              now_ms() - t_enq);
    }
    return 0;
  });
}

// ---------------------------------------------------------------------------------------
// Coalescing of concurrent host calls (coalesce.h): the first caller of an idle queue becomes the
// leader, waits at most HBLS_COALESCE_US for more requests (or until HBLS_COALESCE_MAX items queue
// up), runs them as one batch and wakes every requester with its own statuses.  Requests that
// arrive while a batch runs form the next batch.
// ---------------------------------------------------------------------------------------
Coalescer g_vq;
CoalesceParams g_cp;
std::once_flag g_cp_once;

// read once, by the first caller, before any request is queued (std::call_once: concurrent first
// callers all see the three parameters set)
const CoalesceParams& coalesce_params() {
  std::call_once(g_cp_once, [] {
    g_cp.us = env_size("HBLS_COALESCE_US", 200);
    g_cp.max_items = env_size("HBLS_COALESCE_MAX", 1u << 16);
    // batches in flight at once (HBLS_COALESCE_INFLIGHT, default: the host-call contexts): the
    // requests that arrive while batches run form the next one, which starts at once instead of
    // behind them -- a small batch leaves most of the chip idle
    g_cp.inflight = std::max<size_t>(1, env_size("HBLS_COALESCE_INFLIGHT", (size_t)g_ws_sets));
  });
  return g_cp;
}

void run_verify_batch(std::vector<VReq*>& batch) {
  size_t tot = 0;
  for (VReq* r : batch) tot += r->n;
  std::vector<uint8_t> pk(48 * tot), sig(96 * tot), msg, st(tot);
  std::vector<uint64_t> off(tot);
  std::vector<uint32_t> len(tot);
  size_t k = 0;
  for (VReq* r : batch)
    for (size_t i = 0; i < r->n; i++, k++) {
      memcpy(&pk[48 * k], r->pk + 48 * i, 48);
      memcpy(&sig[96 * k], r->sig + 96 * i, 96);
      off[k] = msg.size();
      len[k] = r->len[i];
      msg.insert(msg.end(), r->msg + r->off[i], r->msg + r->off[i] + r->len[i]);
    }
  if (msg.empty()) msg.push_back(0);
  int rc = verify_host(pk.data(), sig.data(), msg.data(), off.data(), len.data(), tot, st.data());
  std::string err = rc ? g_err : std::string();
  k = 0;
  for (VReq* r : batch) {
    r->rc = rc;
    r->err = err;
    if (!rc) memcpy(r->st, &st[k], r->n);
    k += r->n;
  }
}

int verify_coalesced(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                     const uint32_t* msg_len, size_t n, uint8_t* status) {
  const CoalesceParams& p = coalesce_params();
  if (p.us == 0 || n >= p.max_items) return verify_host(pks, sigs, msgs, msg_off, msg_len, n, status);
  VReq me;
  me.pk = pks;
  me.sig = sigs;
  me.msg = msgs;
  me.off = msg_off;
  me.len = msg_len;
  me.n = n;
  me.st = status;
  coalesce_submit(g_vq, p, me, run_verify_batch);  // coalesce.h
  if (me.rc) g_err = me.err;
  return me.rc;
}

// ---------------------------------------------------------------------------------------
// VerifyAggregate (FastAggregateVerify, herumi.go:318-342) of n_groups groups whose public keys
// are pks[goff[g] .. goff[g+1]) (goff on the HOST, goff[0] == 0): every key decompressed in
// parallel (k_dec_pk), the keys of each group summed by a segmented tree reduction of segments of
// VA_SEG points (k_seg_sum; planned here from goff: a 7M-key group takes 5 launches), the sums
// paired with H(m_g) against the group's signature (k_pair3), herumi's checks applied in its
// order (k_va_status).  hm: one hashed message (with lines) per group, written by hash_fn (if
// given) on s while the side streams decompress: side 0 the keys and their reduction, side 1 the
// signatures and their lines.
// ---------------------------------------------------------------------------------------
constexpr uint32_t VA_SEG = 32;

int va_pipeline(Dev& d, Ws& w, const uint8_t* dpk, size_t np, const uint32_t* goff, size_t ng, const uint8_t* dsig,
                const MsgEntry* hm, uint8_t* dst, hipStream_t s, const std::function<int()>& hash_fn) {
  if (ng == 0) return 0;
  if (np > 0xffffffffull || ng > 0x7fffffffull) return set_err("verify aggregate: too many keys");
  // plan: boundaries of every pass, then the sum index of each group, then the identity map
  std::vector<uint32_t> plan, lo(ng), hi(ng);
  std::vector<size_t> pass_off, pass_n;
  for (size_t g = 0; g < ng; g++) lo[g] = goff[g], hi[g] = goff[g + 1];
  bool more = np > 0;
  while (more) {
    pass_off.push_back(plan.size());
    plan.push_back(0);
    uint32_t out = 0;
    more = false;
    for (size_t g = 0; g < ng; g++) {
      if (hi[g] == lo[g]) continue;
      const uint32_t first = out;
      for (uint32_t b = lo[g]; b < hi[g]; b += VA_SEG) {
        plan.push_back(std::min<uint32_t>(b + VA_SEG, hi[g]));
        out++;
      }
      lo[g] = first;
      hi[g] = out;
      more |= out - first > 1;
    }
    pass_n.push_back(out);
  }
  const size_t sog_off = plan.size();
  for (size_t g = 0; g < ng; g++) plan.push_back(hi[g] > lo[g] ? lo[g] : 0xffffffffu);
  const size_t iota_off = plan.size();
  for (size_t g = 0; g < ng; g++) plan.push_back((uint32_t)g);
  uint32_t* dplan;  // in the workspace set (event-ordered), copied on the call's stream
  if (wsbuf(w, W_PLAN, plan.size(), &dplan)) return -1;
  HCHK(hipMemcpyAsync(dplan, plan.data(), plan.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));

  G1AEntry *pts, *vapt;
  uint8_t *mst, *sigst, *pv, *sta, *stb;
  HmEntry* sigpt;
  G1JEntry *sa, *sb;
  LineEntry* lines;
  const size_t na = pass_n.empty() ? 1 : pass_n[0], nb = pass_n.size() > 1 ? pass_n[1] : 1;
  if (wsbuf(w, W_VPK, np, &pts) || wsbuf(w, W_VPKST, np, &mst) || wsbuf(w, W_VSIG, ng, &sigpt) ||
      wsbuf(w, W_VSIGST, ng, &sigst) || wsbuf(w, W_FBLINES, ng * N_LINES, &lines) || wsbuf(w, W_SEGA, na, &sa) ||
      wsbuf(w, W_SEGSTA, na, &sta) || wsbuf(w, W_SEGB, nb, &sb) || wsbuf(w, W_SEGSTB, nb, &stb) ||
      wsbuf(w, W_VAPT, ng, &vapt) || wsbuf(w, W_VAPV, ng, &pv))
    return -1;
  hipStream_t s0 = w.side[0], s1 = w.side[1];
  HCHK(hipEventRecord(w.ev_fork, s));
  HCHK(hipStreamWaitEvent(s0, w.ev_fork, 0));
  HCHK(hipStreamWaitEvent(s1, w.ev_fork, 0));
  TIMED(d, "k_dec_sig_pt", s1, launch_dec_sig_pt(dsig, (uint32_t)ng, sigpt, sigst, s1));
  TIMED(d, "k_sig_lines", s1, launch_sig_lines(sigpt, (uint32_t)ng, lines, (uint32_t)ng, s1));
  HCHK(hipEventRecord(w.ev_side[1], s1));
  if (hash_fn && hash_fn()) return -1;
  if (np) TIMED(d, "k_dec_pk", s0, launch_dec_pk(dpk, (uint32_t)np, pts, mst, s0));
  const void* in = pts;
  const uint8_t* in_st = mst;
  G1JEntry* out = sa;
  uint8_t* out_st = sta;
  for (size_t k = 0; k < pass_n.size(); k++) {
    out = (k & 1) ? sb : sa;
    out_st = (k & 1) ? stb : sta;
    TIMED(d, "k_seg_sum", s0,
          launch_seg_sum(k == 0, in, in_st, dplan + pass_off[k], (uint32_t)pass_n[k], out, out_st, s0));
    in = out;
    in_st = out_st;
  }
  HCHK(hipEventRecord(w.ev_side[0], s0));
  HCHK(hipStreamWaitEvent(s, w.ev_side[0], 0));
  HCHK(hipStreamWaitEvent(s, w.ev_side[1], 0));
  TIMED(d, "k_va_point", s, launch_va_point(out, dplan + sog_off, (uint32_t)ng, vapt, s));
  Pair3Args a{};
  a.pk = vapt;
  a.msg_idx = dplan + iota_off;
  a.hm = hm;
  a.sig_lines = lines;
  a.stride = (uint32_t)ng;
  a.n = (uint32_t)ng;
  a.n_items = (uint32_t)ng;
  a.status = pv;
  TIMED(d, "k_pair3", s, launch_pair3(a, s));
  TIMED(d, "k_va_status", s, launch_va_status(sigpt, sigst, out_st, dplan + sog_off, pv, (uint32_t)ng, dst, s));
  return 0;
}

// ---------------------------------------------------------------------------------------
// RCCL: one communicator per process (one GPU each) for the exchange of slot results
// ---------------------------------------------------------------------------------------
ncclComm_t g_comm = nullptr;
int g_comm_ranks = 0;

#define NCHK(expr)                                                                        \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess) return set_err(std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int hbls_init(uint32_t device_mask) { return init_mask(device_mask); }

const char* hbls_last_error(void) { return g_err.c_str(); }

int hbls_available(void) { return ensure_init() == 0 ? 1 : 0; }

#ifndef HBLS_BUILD_ID
#define HBLS_BUILD_ID "hbls-build:unversioned"
#endif
const char* hbls_build_id(void) { return HBLS_BUILD_ID; }

int hbls_device_count(void) { return ensure_init() ? -1 : (int)devs().size(); }

size_t hbls_hm_entry_bytes(void) { return sizeof(MsgEntry); }

int hbls_verify_batch(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                      const uint32_t* msg_len, size_t n, uint8_t* status) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  return verify_coalesced(pks, sigs, msgs, msg_off, msg_len, n, status);
}

int hbls_verify_batch_first_error(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                                  const uint32_t* msg_len, size_t n, int64_t* first, uint8_t* first_status,
                                  uint8_t* status) {
  if (ensure_init()) return -1;
  if (!first) return set_err("verify first error: no output for the index");
  return verify_first_host(pks, sigs, msgs, msg_off, msg_len, n, first, first_status, status);
}

int hbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups,
                                   uint8_t* out, uint8_t* status) {
  if (ensure_init()) return -1;
  if (n_groups == 0) return 0;
  return group_op_host(sigs, idx, grp_off, n_groups, 0, out, status);
}

int hbls_aggregate_batch(const uint8_t* sigs, const uint32_t* grp_off, size_t n_groups, uint8_t* out,
                         uint8_t* status) {
  if (ensure_init()) return -1;
  if (n_groups == 0) return 0;
  return group_op_host(sigs, nullptr, grp_off, n_groups, 1, out, status);
}

int hbls_verify_aggregate_batch(const uint8_t* pks, const uint32_t* grp_off, const uint8_t* sigs,
                                const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                                size_t n_groups, uint8_t* status) {
  if (ensure_init()) return -1;
  if (n_groups == 0) return 0;
  if (check_offsets(grp_off, n_groups)) return -1;
  return for_each_device_hc(n_groups, [&](Dev& d, Hc& h, size_t gb, size_t ge, std::unique_lock<std::mutex>& lk) -> int {
    const size_t ng = ge - gb, pb = grp_off[gb], np = grp_off[ge] - pb;
    if (ng == 0) return 0;
    MsgTable t;  // one hash per group (messages need not be distinct)
    t.idx.resize(ng);
    for (size_t g = gb; g < ge; g++) {
      t.off.push_back(t.bytes.size());
      t.len.push_back(msg_len[g]);
      t.bytes.insert(t.bytes.end(), msgs + msg_off[g], msgs + msg_off[g] + msg_len[g]);
    }
    std::vector<uint32_t> goff(ng + 1);
    for (size_t g = 0; g <= ng; g++) goff[g] = grp_off[gb + g] - (uint32_t)pb;
    uint8_t *dpk, *dsig;
    if (upload(d, I_PK, pks + 48 * pb, np * 48, &dpk, &h) || upload(d, I_SIG, sigs + 96 * gb, ng * 96, &dsig, &h))
      return -1;
    void* p;
    if (ensure_buf(h.io[I_STAT], ng, &p)) return -1;
    Ws& w = ws_acquire(d, h.s);
    uint8_t* dst = (uint8_t*)p;
    void* hmp;  // the message table's buffer (hash_table fills the same one on the call's stream)
    if (ensure_buf(h.io[I_HM], ng * sizeof(MsgEntry), &hmp)) return -1;
    MsgEntry* hm = (MsgEntry*)hmp;
    if (va_pipeline(d, w, dpk, np, goff.data(), ng, dsig, hm, dst, h.s,
                    [&]() -> int { MsgEntry* hx; return hash_table(d, t, &hx, true, nullptr, nullptr, &h); }))
      return -1;
    if (ws_release(w, h.s)) return -1;
    lk.unlock();  // enqueued: other callers may enqueue while this one waits for its stream
    HCHK(hipMemcpyAsync(status + gb, dst, ng, hipMemcpyDeviceToHost, h.s));
    HCHK(hipStreamSynchronize(h.s));
    return 0;
  });
}

// Signing roots (roots.hip).  mode 0: data = 128-byte SSZ AttestationData; 1: data = 32-byte
// object roots.  Host buffers; dom_idx nullable.
static int roots_host(int mode, const uint8_t* data, size_t n, const uint8_t* domains, size_t n_domains,
                      const uint32_t* dom_idx, uint8_t* roots) {
  if (n_domains == 0) return set_err("signing roots: no domain");
  if (dom_idx)
    for (size_t i = 0; i < n; i++)
      if (dom_idx[i] >= n_domains) return set_err("signing roots: domain index out of range");
  const size_t item = mode == 0 ? 128 : 32;
  return for_each_device(n, [&](Dev& d, size_t b, size_t e) -> int {
    const size_t m = e - b;
    uint8_t *dd, *ddom;
    uint32_t* didx = nullptr;
    if (upload(d, I_SIG, data + item * b, m * item, &dd) || upload(d, I_PK, domains, n_domains * 32, &ddom)) return -1;
    if (dom_idx && upload(d, I_MIDX, dom_idx + b, m, &didx)) return -1;
    void* out;
    if (ensure_buf(d.io[I_OUT], m * 32, &out)) return -1;
    if (mode == 0)
      TIMED(d, "k_attestation_roots", d.stream,
            launch_attestation_roots(dd, (uint32_t)m, ddom, (uint32_t)n_domains, didx, (uint8_t*)out, d.stream));
    else
      TIMED(d, "k_signing_roots", d.stream,
            launch_signing_roots(dd, (uint32_t)m, ddom, (uint32_t)n_domains, didx, (uint8_t*)out, d.stream));
    HCHK(hipMemcpyAsync(roots + 32 * b, out, m * 32, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int hbls_attestation_signing_roots(const uint8_t* data, size_t n, const uint8_t* domains, size_t n_domains,
                                   const uint32_t* dom_idx, uint8_t* roots) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  return roots_host(0, data, n, domains, n_domains, dom_idx, roots);
}

int hbls_signing_roots(const uint8_t* object_roots, size_t n, const uint8_t* domains, size_t n_domains,
                       const uint32_t* dom_idx, uint8_t* roots) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  return roots_host(1, object_roots, n, domains, n_domains, dom_idx, roots);
}

int hbls_duty_signing_roots(int kind, const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n,
                            const uint8_t* domains, size_t n_domains, const uint32_t* dom_idx, uint8_t* roots,
                            uint8_t* status) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  if (kind < 1 || kind > 9) return set_err("duty signing roots: unknown kind");
  if (n_domains == 0) return set_err("signing roots: no domain");
  if (dom_idx)
    for (size_t i = 0; i < n; i++)
      if (dom_idx[i] >= n_domains) return set_err("signing roots: domain index out of range");
  return for_each_device(n, [&](Dev& d, size_t b, size_t e) -> int {
    const size_t m = e - b;
    // the shard's objects packed: their bytes from the first object's offset on, offsets rebased
    uint64_t lo = ~0ull, hi = 0;
    for (size_t i = b; i < e; i++) {
      lo = std::min(lo, off[i]);
      hi = std::max(hi, off[i] + len[i]);
    }
    std::vector<uint64_t> roff(m);
    for (size_t i = 0; i < m; i++) roff[i] = off[b + i] - lo;
    uint8_t *dd, *ddom;
    uint64_t* doff;
    uint32_t *dlen, *didx = nullptr;
    if (upload(d, I_SIG, data + lo, hi - lo, &dd) || upload(d, I_PK, domains, n_domains * 32, &ddom) ||
        upload(d, I_OFF, roff.data(), m, &doff) || upload(d, I_LEN, len + b, m, &dlen))
      return -1;
    if (dom_idx && upload(d, I_MIDX, dom_idx + b, m, &didx)) return -1;
    void *out, *st;
    if (ensure_buf(d.io[I_OUT], m * 32, &out) || ensure_buf(d.io[I_STAT], m, &st)) return -1;
    TIMED(d, "k_duty_roots", d.stream,
          launch_duty_roots(kind, dd, doff, dlen, (uint32_t)m, ddom, (uint32_t)n_domains, didx, (uint8_t*)out,
                            (uint8_t*)st, d.stream));
    HCHK(hipMemcpyAsync(roots + 32 * b, out, m * 32, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipMemcpyAsync(status + b, st, m, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int hbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                    size_t n, uint8_t* sigs, uint8_t* status) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  return for_each_device(n, [&](Dev& d, size_t b, size_t e) -> int {
    const size_t m = e - b;
    std::vector<size_t> items(m);
    std::iota(items.begin(), items.end(), b);
    MsgTable t;
    dedup_messages(msgs, msg_off, msg_len, m, items.data(), t);
    MsgEntry* hm;
    if (hash_table(d, t, &hm, false)) return -1;
    uint8_t* dsk;
    uint32_t* didx;
    if (upload(d, I_SK, sks + 32 * b, m * 32, &dsk) || upload(d, I_MIDX, t.idx.data(), m, &didx)) return -1;
    void *dout, *dst;
    if (ensure_buf(d.io[I_OUT], m * 96, &dout) || ensure_buf(d.io[I_STAT], m, &dst)) return -1;
    LAUNCH(k_sign, m, d.stream, dsk, didx, hm, (uint32_t)m, (uint8_t*)dout, (uint8_t*)dst);
    HCHK(hipMemcpyAsync(sigs + 96 * b, dout, m * 96, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipMemcpyAsync(status + b, dst, m, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int hbls_secret_to_public_key_batch(const uint8_t* sks, size_t n, uint8_t* pks, uint8_t* status) {
  if (ensure_init()) return -1;
  if (n == 0) return 0;
  return for_each_device(n, [&](Dev& d, size_t b, size_t e) -> int {
    const size_t m = e - b;
    uint8_t* dsk;
    if (upload(d, I_SK, sks + 32 * b, m * 32, &dsk)) return -1;
    void *dout, *dst;
    if (ensure_buf(d.io[I_OUT], m * 48, &dout) || ensure_buf(d.io[I_STAT], m, &dst)) return -1;
    LAUNCH(k_sk_to_pk, m, d.stream, dsk, (uint32_t)m, (uint8_t*)dout, (uint8_t*)dst);
    HCHK(hipMemcpyAsync(pks + 48 * b, dout, m * 48, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipMemcpyAsync(status + b, dst, m, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int hbls_threshold_split(const uint8_t* secret, const uint8_t* coeffs, uint32_t total, uint32_t threshold,
                         uint8_t* shares, uint8_t* status) {
  if (ensure_init()) return -1;
  if (total == 0 || threshold == 0) return 0;
  std::vector<uint8_t> poly(32ull * threshold);
  memcpy(poly.data(), secret, 32);
  if (threshold > 1) memcpy(poly.data() + 32, coeffs, 32ull * (threshold - 1));
  return for_each_device(1, [&](Dev& d, size_t, size_t) -> int {
    uint8_t* dpoly;
    if (upload(d, I_SK, poly.data(), poly.size(), &dpoly)) return -1;
    void *dout, *dst;
    if (ensure_buf(d.io[I_OUT], 32ull * total, &dout) || ensure_buf(d.io[I_STAT], total, &dst)) return -1;
    LAUNCH(k_split, total, d.stream, dpoly, threshold, total, (uint8_t*)dout, (uint8_t*)dst);
    HCHK(hipMemcpyAsync(shares, dout, 32ull * total, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipMemcpyAsync(status, dst, total, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

int hbls_recover_secret(const uint8_t* shares, const int64_t* idx, size_t k, uint8_t* out, uint8_t* status) {
  if (ensure_init()) return -1;
  return for_each_device(1, [&](Dev& d, size_t, size_t) -> int {
    uint8_t* dsh;
    int64_t* didx;
    std::vector<uint8_t> dummy(32);
    if (upload(d, I_SK, k ? shares : dummy.data(), k ? 32 * k : 32, &dsh)) return -1;
    std::vector<int64_t> di(k ? k : 1, 0);
    if (k) memcpy(di.data(), idx, 8 * k);
    if (upload(d, I_IDX, di.data(), di.size(), &didx)) return -1;
    void *dout, *dst;
    if (ensure_buf(d.io[I_OUT], 32, &dout) || ensure_buf(d.io[I_STAT], 1, &dst)) return -1;
    hipLaunchKernelGGL(k_recover, dim3(1), dim3(64), 0, d.stream, dsh, didx, (uint32_t)k, (uint8_t*)dout,
                       (uint8_t*)dst);
    HCHK(hipGetLastError());
    HCHK(hipMemcpyAsync(out, dout, 32, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipMemcpyAsync(status, dst, 1, hipMemcpyDeviceToHost, d.stream));
    HCHK(hipStreamSynchronize(d.stream));
    return 0;
  });
}

// ---- device-buffer entry points (slot pipeline) ----
int hbls_hash_to_g2_device(const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len, size_t n_msgs,
                           void* hm, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  return hash_messages(*d, msgs, msg_off, msg_len, n_msgs, (MsgEntry*)hm, s);
}

int hbls_verify_device(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, const void* hm, size_t n,
                       const uint32_t* vgrp_off, size_t n_vgroups, uint8_t* status, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(d->mu);
  Ws& w = ws_acquire(*d, s);
  if (verify_pipeline(*d, w, pks, sigs, msg_idx, (const MsgEntry*)hm, n, vgrp_off, n_vgroups, status, s, nullptr,
                      nullptr))
    return -1;
  return ws_release(w, s);
}

int hbls_verify_device_first_error(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, const void* hm,
                                   size_t n, const uint32_t* vgrp_off, size_t n_vgroups, uint8_t* status,
                                   uint32_t* first, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (!first) return set_err("verify first error: no output for the index");
  if (n == 0) {
    HCHK(hipMemsetAsync(first, 0xff, sizeof(uint32_t), s));
    return 0;
  }
  if (n >= 0xffffffffull) return set_err("verify first error: too many items");
  std::lock_guard<std::mutex> lk(d->mu);
  Ws& w = ws_acquire(*d, s);
  if (verify_pipeline(*d, w, pks, sigs, msg_idx, (const MsgEntry*)hm, n, vgrp_off, n_vgroups, status, s, nullptr,
                      nullptr, false, nullptr, nullptr, 0, first))
    return -1;
  return ws_release(w, s);
}

size_t hbls_pk_entry_bytes(void) { return sizeof(G1AEntry); }

int hbls_pubkey_cache_add(const uint8_t* pks, size_t n) {
  if (ensure_init()) return -1;
  std::lock_guard<std::mutex> al(g_kc_add_mu);
  std::vector<uint8_t> fresh;
  std::unordered_map<std::string, uint32_t> add;
  {
    std::lock_guard<std::mutex> lk(g_kc_mu);
    for (size_t k = 0; k < n; k++) {
      std::string key((const char*)pks + 48 * k, 48);
      if (g_kc_map.count(key) || add.count(key)) continue;
      add.emplace(key, (uint32_t)(g_kc_n + add.size()));
      fresh.insert(fresh.end(), pks + 48 * k, pks + 48 * k + 48);
    }
  }
  const size_t m = add.size();
  if (m == 0) return 0;
  if (g_kc_n + m > 0xffffffffull) return set_err("pubkey cache full");
  for (Dev* dp : devs()) {  // the device work under each Dev::mu in turn, g_kc_mu not held
    std::lock_guard<std::mutex> dl(dp->mu);
    if (kc_fill(*dp, fresh.data(), g_kc_n, m)) return -1;
  }
  g_kc_keys.insert(g_kc_keys.end(), fresh.begin(), fresh.end());
  std::lock_guard<std::mutex> lk(g_kc_mu);  // publish: lookups see the entries only now
  for (auto& kv : add) g_kc_map.emplace(kv.first, kv.second);
  g_kc_n += m;
  return 0;
}

size_t hbls_sig_cache(size_t entries) {
  if (ensure_init()) return 0;
  while (entries & (entries - 1)) entries &= entries - 1;
  entries = std::min<size_t>(entries, size_t(1) << 30);
  const size_t old = g_sc_cap.exchange(entries);
  for (Dev* d : devs()) {  // drop the contents: the next put allocates at the new capacity
    std::lock_guard<std::mutex> lk(d->mu);
    d->sc_filled = 0;
    d->sc_cap = 0;
  }
  return old;
}

int hbls_pubkey_cache_clear(void) {
  std::lock_guard<std::mutex> al(g_kc_add_mu);
  for (Dev* dp : devs()) {  // no verification enqueued after this sees the old entries
    std::lock_guard<std::mutex> dl(dp->mu);
    dp->kc_n = 0;
    dp->kc_tcap = 0;  // the next fill builds a fresh index
  }
  std::lock_guard<std::mutex> lk(g_kc_mu);
  g_kc_map.clear();
  g_kc_n = 0;
  g_kc_keys.clear();
  return 0;
}

size_t hbls_pubkey_cache_size(void) {
  std::lock_guard<std::mutex> lk(g_kc_mu);
  return g_kc_n;
}

// Test switch of the in-process multi-device split: every device of the mask is driven through
// `copies` contexts (streams, workspaces, host thread), so host-buffer calls shard over them as
// over several GPUs (for_each_device) on a one-GPU box.  Call while no other call is in flight.
int hbls_debug_split(uint32_t copies) {
  if (ensure_init()) return -1;
  if (copies == 0 || copies > 16) return set_err("hbls_debug_split: copies must be in 1..16");
  std::lock_guard<std::mutex> il(g_init_mu);
  std::lock_guard<std::mutex> al(g_kc_add_mu);
  std::vector<Dev*> devs;
  g_split_pool.resize(g_base_devs.size());
  for (size_t bi = 0; bi < g_base_devs.size(); bi++) {
    Dev* b = g_base_devs[bi];
    std::vector<Dev*>& pool = g_split_pool[bi];
    devs.push_back(b);
    for (uint32_t c = 1; c < copies; c++) {
      if (pool.size() < c) {
        Dev* d;
        if (dev_create(b->ord, &d)) return -1;
        pool.push_back(d);
      }
      Dev* d = pool[c - 1];
      d->timing = b->timing;
      d->serial = b->serial;
      std::lock_guard<std::mutex> dl(d->mu);
      if (hipSetDevice(d->ord) != hipSuccess) return set_err("hipSetDevice failed");
      if (g_kc_n && kc_fill(*d, g_kc_keys.data(), 0, g_kc_n)) return -1;  // the same key cache
      devs.push_back(d);
    }
  }
  std::lock_guard<std::mutex> l(g_devs_mu);
  g_devs = devs;
  return 0;
}

int hbls_decompress_pubkeys_device(const uint8_t* pks, size_t n, void* table, uint8_t* status, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (n == 0) return 0;
  if (n > 0xffffffffull) return set_err("decompress pubkeys: too many keys");
  std::lock_guard<std::mutex> lk(d->mu);
  TIMED(*d, "k_dec_pk", s, launch_dec_pk(pks, (uint32_t)n, (G1AEntry*)table, status, s));
  return 0;
}

int hbls_attestation_signing_roots_device(const uint8_t* data, size_t n, const uint8_t* domains, size_t n_domains,
                                          const uint32_t* dom_idx, uint8_t* roots, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (n == 0) return 0;
  if (n_domains == 0) return set_err("signing roots: no domain");
  if (n > 0xffffffffull) return set_err("signing roots: too many items");
  std::lock_guard<std::mutex> lk(d->mu);
  TIMED(*d, "k_attestation_roots", s,
        launch_attestation_roots(data, (uint32_t)n, domains, (uint32_t)n_domains, dom_idx, roots, s));
  return 0;
}

int hbls_verify_aggregate_device(const uint8_t* pks, const uint32_t* grp_off, size_t n_groups, const uint8_t* sigs,
                                 const void* hm, uint8_t* status, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (n_groups == 0) return 0;
  if (check_offsets(grp_off, n_groups)) return -1;
  std::vector<uint32_t> goff(n_groups + 1);
  for (size_t g = 0; g <= n_groups; g++) goff[g] = grp_off[g] - grp_off[0];
  std::lock_guard<std::mutex> lk(d->mu);
  Ws& w = ws_acquire(*d, s);
  if (va_pipeline(*d, w, pks + 48ull * grp_off[0], goff[n_groups], goff.data(), n_groups, sigs, (const MsgEntry*)hm,
                  status, s, nullptr))
    return -1;
  return ws_release(w, s);
}

int hbls_threshold_aggregate_device(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups,
                                    size_t n_partials, uint8_t* out, uint8_t* status, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  Ws& w = ws_acquire(*d, s);
  HmEntry* pts;
  uint8_t* mst0;
  if (wsbuf(w, W_TAPTS, n_partials, &pts) || wsbuf(w, W_TADST, n_partials, &mst0)) return -1;
  if (n_partials) TIMED(*d, "k_dec_sig_pt", s, launch_dec_sig_pt(sigs, (uint32_t)n_partials, pts, mst0, s));
  if (ta_tail(*d, w, pts, nullptr, mst0, idx, grp_off, n_groups, n_partials, 0, out, status, nullptr, s)) return -1;
  return ws_release(w, s);
}

int hbls_slot_device(const hbls_slot* a, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (!a) return set_err("hbls_slot_device: null arguments");
  if (a->n_groups && !a->ta_src && !a->ta_sigs) return set_err("hbls_slot_device: ta_src or ta_sigs is required");
  if (a->dv_pks && a->n_vgroups != a->n_groups)
    return set_err("hbls_slot_device: the folded post-aggregate verification needs one verification group per "
                   "aggregation group");
  std::lock_guard<std::mutex> lk(d->mu);
  Ws& w = ws_acquire(*d, s);
  HCHK(hipEventRecord(w.ev_fork, s));
  // messages: hash + Miller lines (side 2)
  hipStream_t sh = w.side[2];
  HCHK(hipStreamWaitEvent(sh, w.ev_fork, 0));
  const bool defer = defer_lines(a->n_vgroups, a->n_msgs);
  if (hash_messages(*d, a->msgs, a->msg_off, a->msg_len, a->n_msgs, (MsgEntry*)a->hm, sh, !defer)) return -1;
  HCHK(hipEventRecord(w.ev_side[2], sh));
  TaFold fold{};
  fold.ta_sigs = a->ta_sigs;
  fold.ta_src = a->ta_src;
  fold.ta_idx = a->ta_idx;
  fold.grp_off = a->grp_off;
  fold.n_groups = a->n_groups;
  fold.n_partials = a->n_ta_partials;
  fold.ta_out = a->ta_out;
  fold.ta_status = a->ta_status;
  fold.dv_pks = a->dv_pks;
  fold.agg_status = a->agg_vstatus;
  if ((a->pk_table != nullptr) != (a->pk_table_st != nullptr) ||
      (a->dv_pk_table != nullptr) != (a->dv_pk_table_st != nullptr))
    return set_err("hbls_slot_device: a key table needs its status array");
  fold.pk_table = (const G1AEntry*)a->pk_table;
  fold.pk_table_st = a->pk_table_st;
  fold.dv_pk_table = (const G1AEntry*)a->dv_pk_table;
  fold.dv_pk_table_st = a->dv_pk_table_st;
  if (verify_pipeline(*d, w, a->pks, a->sigs, a->msg_idx, (const MsgEntry*)a->hm, a->n, a->vgrp_off, a->n_vgroups,
                      a->vstatus, s, w.ev_side[2], &fold, false, nullptr, (MsgEntry*)a->hm, defer ? a->n_msgs : 0))
    return -1;
  HCHK(hipStreamWaitEvent(s, w.ev_side[2], 0));
  return ws_release(w, s);
}

int hbls_timing(int enable) {
  if (ensure_init()) return -1;
  for (Dev* d : devs()) {
    std::lock_guard<std::mutex> lk(d->mu);
    d->timing = enable != 0;
    d->serial = enable == 2;
    d->tev_used = 0;
  }
  return 0;
}

// Launch durations recorded since hbls_timing(1), in launch order over the devices of the mask:
// names[i] (kernel name, static storage) and ms[i].
int hbls_timing_read(const char** names, float* ms, size_t max_n, size_t* n_out) {
  if (ensure_init()) return -1;
  size_t k = 0;
  for (Dev* d : devs()) {
    std::lock_guard<std::mutex> lk(d->mu);
    HCHK(hipSetDevice(d->ord));
    for (size_t i = 0; i < d->tev_used && k < max_n; i++, k++) {
      HCHK(hipEventSynchronize(d->tev[i].b));
      HCHK(hipEventElapsedTime(&ms[k], d->tev[i].a, d->tev[i].b));
      if (names) names[k] = d->tev[i].name;
    }
  }
  *n_out = k;
  return 0;
}

int hbls_stats(uint64_t* out, size_t n) {
  for (size_t k = 0; k < n && k < 8; k++) out[k] = g_stats[k].load();
  return stats_on() ? 0 : set_err("statistics are collected only with HBLS_STATS=1");
}

size_t hbls_fe_batch(size_t min_groups) { return g_fe_batch_min.exchange(min_groups); }
int hbls_adaptive(int on) { return g_adaptive.exchange(on != 0) ? 1 : 0; }
// the latency-path layouts by name (tests switch between them within one process)
int hbls_tune(const char* name, size_t value, size_t* previous) {
  if (ensure_init()) return -1;
  if (!name) return set_err("hbls_tune: no name");
  static const std::pair<const char*, std::atomic<size_t>*> knobs[] = {
      {"HBLS_HASH_PAIR_MAX", &g_hash_pair_max}, {"HBLS_HASH_ONE_LANE", &g_hash_one_lane},
      {"HBLS_HASH_SPLIT", &g_hash_split},       {"HBLS_FE18_MAX", &g_fe18_max},
      {"HBLS_TA_PAIR_MAX", &g_ta_pair_max},     {"HBLS_DEC_PAIR_MAX", &g_dec_pair_max},
      // chunking of large verifications (tests run them at small sizes: several chunks per call)
      {"HBLS_GROUP_CHUNK", &g_gcap},            {"HBLS_FALLBACK_CHUNK", &g_fbcap},
      {"HBLS_GROUP_MAX", &g_gmax}};
  for (const auto& k : knobs)
    if (strcmp(k.first, name) == 0) {
      const size_t old = k.second->exchange(value);
      if (previous) *previous = old;
      return 0;
    }
  return set_err(std::string("hbls_tune: unknown setting ") + name);
}
size_t hbls_dec_pair_max(size_t items) {
  if (ensure_init()) return 0;
  return g_dec_pair_max.exchange(items);
}
size_t hbls_single_max(size_t items) {
  if (ensure_init()) return 0;
  return g_single_max.exchange(items);
}
size_t hbls_slot_msm(size_t min_items) {
  // a new setting starts from a clean history (tests count the slot-wide checks that ran)
  for (Dev* d : devs()) {
    std::lock_guard<std::mutex> lk(d->mu);
    for (; d->res_tail != d->res_head; d->res_tail++) (void)hipEventSynchronize(d->res_ev[d->res_tail % N_RES]);
    d->attack = false;
  }
  return g_slot_msm_min.exchange(min_items);
}
size_t hbls_ta_joint(size_t members) { return g_ta_joint.exchange(std::min<size_t>(members, 8)); }
size_t hbls_rlc_lanes(size_t lanes) { return g_rlc_lanes.exchange(lanes ? lanes : 65536); }

int hbls_sync(void* stream) {
  HCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int hbls_status_bitmap(const uint8_t* status, size_t n, uint8_t* bits, void* stream) {
  Dev* d;
  hipStream_t s = (hipStream_t)stream;
  if (dev_of_stream(s, &d)) return -1;
  if (n > 0xffffffffull) return set_err("status bitmap: too many items");
  LAUNCH(k_status_bitmap, n, s, status, (uint32_t)n, bits);
  return 0;
}

// ---- RCCL exchange between processes (one GPU each) ----
size_t hbls_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

int hbls_comm_unique_id(uint8_t* id) {
  ncclUniqueId u;
  NCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return 0;
}

int hbls_comm_init(int nranks, int rank, const uint8_t* id) {
  if (ensure_init()) return -1;
  const std::vector<Dev*> ds = devs();
  if (ds.size() != 1) return set_err("hbls_comm_init: one device per process");
  if (g_comm) return g_comm_ranks == nranks ? 0 : set_err("communicator already initialised");
  HCHK(hipSetDevice(ds[0]->ord));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  NCHK(ncclCommInitRank(&g_comm, nranks, u, rank));
  g_comm_ranks = nranks;
  return 0;
}

int hbls_allgather_device(const void* send, void* recv, size_t bytes, void* stream) {
  if (!g_comm) return set_err("hbls_allgather_device: no communicator (hbls_comm_init)");
  NCHK(ncclAllGather(send, recv, bytes, ncclUint8, g_comm, (hipStream_t)stream));
  return 0;
}

int hbls_comm_size(void) {
  if (!g_comm) return 0;
  int n = 0;
  if (ncclCommCount(g_comm, &n) != ncclSuccess) return -1;
  return n;
}

int hbls_comm_destroy(void) {
  if (g_comm) NCHK(ncclCommDestroy(g_comm));
  g_comm = nullptr;
  g_comm_ranks = 0;
  return 0;
}

}  // extern "C"
