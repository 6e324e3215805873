// libhipbls.so: gfx950 kernels + C ABI (include/hipbls.h) for charon's BLS hot path.
//
// Reference interface replaced: tbls.Implementation (/root/reference/tbls/tbls.go:27-69) as
// implemented by tbls.Herumi (/root/reference/tbls/herumi.go).  One lane = one item
// (partial signature, group or message); kernels are staged so that work shared between
// items (hash_to_curve of a message) runs once.
#include "layout.h"
#include "../../include/hipbls.h"

#include <mutex>
#include <string>
#include <string.h>
#include <unordered_map>
#include <vector>

using namespace hb;


#define KERNEL_BOUNDS __launch_bounds__(64)
constexpr int BLOCK = 64;

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t find_group(const uint32_t* grp_off, uint32_t n_groups, uint32_t j) {
  // largest g with grp_off[g] <= j  (groups may be empty)
  uint32_t lo = 0, hi = n_groups;  // invariant: grp_off[lo] <= j < grp_off[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (grp_off[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One lane per partial: decompress + subgroup-check sigma_j (herumi.go:257 Sign.Deserialize).
__global__ KERNEL_BOUNDS void k_ta_dec(const uint8_t* __restrict__ sigs, uint32_t n_partials,
                                               HmEntry* __restrict__ pts, uint8_t* __restrict__ mstat) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_partials) return;
  G2A s;
  uint8_t bad = g2_decompress(s, sigs + 96ull * j);
  HmEntry e;
  e.x = s.x;
  e.y = s.y;
  e.inf = (!bad && s.inf) ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  pts[j] = e;
  mstat[j] = bad ? M_BAD_SIG : M_OK;
}

// One lane per group: sum the member points, compress (herumi Sign.Recover / Sign.Aggregate +
// Serialize).  Status precedence follows herumi: any undecodable partial -> BAD_SIGNATURE
// (deserialisation happens first, herumi.go:255-264), then combine failure.
__global__ KERNEL_BOUNDS void k_group_sum(const uint32_t* __restrict__ grp_off, uint32_t n_groups, int mode,
                                          const G2JEntry* __restrict__ pts, const uint8_t* __restrict__ mstat,
                                          uint8_t* __restrict__ out, uint8_t* __restrict__ status) {
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
    return;
  }
  G2J acc = jac_infinity<Fp2>();
  for (uint32_t m = b; m < e; m++) {
    G2JEntry q = pts[m];
    acc = jac_add(acc, G2J{q.X, q.Y, q.Z});
  }
  uint8_t buf[96];
  g2_compress(buf, jac_to_aff(acc));
  for (int k = 0; k < 96; k++) o[k] = buf[k];
  status[g] = ST_OK;
}

// VerifyAggregate stage 1: one lane per public key.
__global__ KERNEL_BOUNDS void k_g1_member(const uint8_t* __restrict__ pks, uint32_t n, G1AEntry* __restrict__ pts,
                                          uint8_t* __restrict__ mstat) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  G1A p;
  if (g1_decompress(p, pks + 48ull * j)) {
    mstat[j] = 1;
    return;
  }
  mstat[j] = 0;
  G1AEntry e;
  e.x = p.x;
  e.y = p.y;
  e.inf = p.inf;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  pts[j] = e;
}

// VerifyAggregate stage 2: one lane per group (FastAggregateVerify, herumi.go:318-342).
__global__ KERNEL_BOUNDS void k_verify_aggregate(const uint32_t* __restrict__ grp_off, uint32_t n_groups,
                                                 const G1AEntry* __restrict__ pts, const uint8_t* __restrict__ mstat,
                                                 const uint8_t* __restrict__ sigs, const MsgEntry* __restrict__ hm,
                                                 uint8_t* __restrict__ status) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  G2A sig;
  if (g2_decompress(sig, sigs + 96ull * g)) {
    status[g] = ST_BAD_SIGNATURE;
    return;
  }
  uint32_t b = grp_off[g], e = grp_off[g + 1];
  G1J acc = jac_infinity<Fp>();
  for (uint32_t m = b; m < e; m++) {
    if (mstat[m]) {
      status[g] = ST_BAD_PUBKEY;
      return;
    }
    G1AEntry q = pts[m];
    acc = jac_add_aff(acc, G1A{q.x, q.y, q.inf != 0});
  }
  if (e == b) {
    status[g] = ST_NOT_VERIFIED;
    return;
  }
  G1A agg = jac_to_aff(acc);
  status[g] = verify_core(agg, hm_load(hm[g].h), sig) ? ST_OK : ST_NOT_VERIFIED;
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
  g2_compress(buf, jac_to_aff(sg));
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
  g1_compress(buf, jac_to_aff(p));
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
// Host runtime: device selection, grow-only workspaces, error reporting
// ---------------------------------------------------------------------------------------
namespace {

thread_local std::string g_err;
std::mutex g_mu;  // serialises host-buffer calls (shared workspace)
int g_device = -1;
hipStream_t g_stream = nullptr;
// fork/join streams: 0, 1 = the staged verify's decompression kernels, 2 = message hashing,
// 3 = unused (hbls_slot_device runs its ThresholdAggregate on g_stream)
constexpr int N_SIDE = 4;
hipStream_t g_side[N_SIDE] = {};
hipEvent_t g_ev_fork = nullptr, g_ev_slot = nullptr, g_ev_side[N_SIDE] = {};

// optional timing of the pairing kernel (hbls_timing): event pairs recorded on its stream
bool g_timing = false;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_tev;  // pool
size_t g_tev_used = 0;
int timing_pair(hipEvent_t* a, hipEvent_t* b);

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

enum BufId {
  B_PK, B_SIG, B_MSG, B_OFF, B_LEN, B_MIDX, B_HM, B_STAT, B_IDX, B_GOFF, B_PTS, B_MSTAT, B_OUT, B_SK, B_G1PTS,
  B_VPK, B_VPKST, B_VSIGINF, B_VSIGST, B_VLINES,  // staged verify: per-partial intermediates
  B_TAPTS, B_TADIG, B_TATAB,                      // staged ThresholdAggregate
  B_COUNT
};
DevBuf g_bufs[B_COUNT];

int set_err(const char* what, hipError_t e) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return -1;
}

#define HCHK(expr)                                         \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return set_err(#expr, _e);       \
  } while (0)

int ensure(BufId id, size_t bytes, void** out) {
  DevBuf& b = g_bufs[id];
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) HCHK(hipFree(b.p));
    size_t cap = bytes + bytes / 4;
    HCHK(hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  *out = b.p;
  return 0;
}

int timing_pair(hipEvent_t* a, hipEvent_t* b) {
  if (g_tev_used == g_tev.size()) {
    hipEvent_t x, y;
    HCHK(hipEventCreate(&x));
    HCHK(hipEventCreate(&y));
    g_tev.push_back({x, y});
  }
  *a = g_tev[g_tev_used].first;
  *b = g_tev[g_tev_used].second;
  g_tev_used++;
  return 0;
}

int init_locked(int device) {
  if (g_device >= 0) {
    HCHK(hipSetDevice(g_device));
    return 0;
  }
  int n = 0;
  HCHK(hipGetDeviceCount(&n));
  if (n <= 0) {
    g_err = "no HIP device";
    return -1;
  }
  if (device < 0) device = 0;
  HCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HCHK(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_err = std::string("libhipbls is built for gfx950, device is ") + prop.gcnArchName;
    return -1;
  }
  // the verify pipeline's streams (decompression, hashing) get the highest priority: they gate the
  // pairing kernel, while the aggregation chain on g_stream (lowest priority) has slack in the slot
  int prio_lo = 0, prio_hi = 0;
  HCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  HCHK(hipStreamCreateWithPriority(&g_stream, hipStreamNonBlocking, prio_lo));
  for (int k = 0; k < N_SIDE; k++) {
    HCHK(hipStreamCreateWithPriority(&g_side[k], hipStreamNonBlocking, prio_hi));
    HCHK(hipEventCreateWithFlags(&g_ev_side[k], hipEventDisableTiming));
  }
  HCHK(hipEventCreateWithFlags(&g_ev_fork, hipEventDisableTiming));
  HCHK(hipEventCreateWithFlags(&g_ev_slot, hipEventDisableTiming));
  g_device = device;
  return 0;
}

inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

#define LAUNCH(kern, n, stream, ...)                                                              \
  do {                                                                                            \
    if ((n) > 0) {                                                                                \
      hipLaunchKernelGGL(kern, dim3(blocks_for(n)), dim3(BLOCK), 0, (stream), __VA_ARGS__);       \
      HCHK(hipGetLastError());                                                                    \
    }                                                                                             \
  } while (0)

template <class T>
int upload(BufId id, const T* src, size_t count, T** dst) {
  void* p;
  if (ensure(id, count * sizeof(T), &p)) return -1;
  if (count) HCHK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, g_stream));
  *dst = (T*)p;
  return 0;
}

// Deduplicate messages: returns packed table + per-item index (host-side bookkeeping only).
struct MsgTable {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  std::vector<uint32_t> idx;
};

void dedup_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, MsgTable& t) {
  std::unordered_map<std::string, uint32_t> seen;
  seen.reserve(n * 2 + 1);
  t.idx.resize(n);
  for (size_t i = 0; i < n; i++) {
    std::string key((const char*)msgs + off[i], len[i]);
    auto it = seen.find(key);
    if (it == seen.end()) {
      uint32_t id = (uint32_t)t.len.size();
      seen.emplace(std::move(key), id);
      t.off.push_back(t.bytes.size());
      t.len.push_back(len[i]);
      t.bytes.insert(t.bytes.end(), msgs + off[i], msgs + off[i] + len[i]);
      t.idx[i] = id;
    } else {
      t.idx[i] = it->second;
    }
  }
}

// hash every distinct message to G2 (+ its Miller line chain when `lines`) into MsgEntry[].
int hash_table_locked(const MsgTable& t, MsgEntry** hm_out, bool lines) {
  uint8_t* dmsg;
  uint64_t* doff;
  uint32_t* dlen;
  void* hm;
  if (upload(B_MSG, t.bytes.data(), t.bytes.size(), &dmsg)) return -1;
  if (upload(B_OFF, t.off.data(), t.off.size(), &doff)) return -1;
  if (upload(B_LEN, t.len.data(), t.len.size(), &dlen)) return -1;
  if (ensure(B_HM, t.len.size() * sizeof(MsgEntry), &hm)) return -1;
  launch_hash_to_g2(dmsg, doff, dlen, (uint32_t)t.len.size(), (MsgEntry*)hm, g_stream);
  HCHK(hipGetLastError());
  if (lines) launch_lines_msg((MsgEntry*)hm, (uint32_t)t.len.size(), g_stream);
  *hm_out = (MsgEntry*)hm;
  return 0;
}

// Staged verify of n partials already in device memory (herumi.go:288-304 per item):
//   side stream 0: k_dec_pk          (1 lane / partial)
//   side stream 1: k_dec_sig_lines   (1 lane / partial: decompress sig + its 68 lines at -g1)
//   stream s:      k_pair3           (3 lanes / partial: Miller loop + final exponentiation)
// in chunks of at most VERIFY_CHUNK partials (the line buffer is 19.6 KB per partial).
constexpr size_t VERIFY_CHUNK = 1u << 17;
// hm_ready (optional): event after which `hm` is complete; only the pairing kernel waits for it,
// so the decompression kernels overlap the hashing.
int verify_pipeline_locked(const uint8_t* dpk, const uint8_t* dsig, const uint32_t* didx, const MsgEntry* hm,
                           size_t n, uint8_t* dst, hipStream_t s, hipEvent_t hm_ready = nullptr) {
  size_t cap = n < VERIFY_CHUNK ? n : VERIFY_CHUNK;
  void *vpk, *vpkst, *vsinf, *vsst, *vlines;
  if (ensure(B_VPK, cap * sizeof(G1AEntry), &vpk) || ensure(B_VPKST, cap, &vpkst) || ensure(B_VSIGINF, cap, &vsinf) ||
      ensure(B_VSIGST, cap, &vsst) || ensure(B_VLINES, cap * N_LINES * sizeof(LineEntry), &vlines))
    return -1;
  for (size_t c0 = 0; c0 < n; c0 += cap) {
    uint32_t cn = (uint32_t)((n - c0) < cap ? (n - c0) : cap);
    HCHK(hipEventRecord(g_ev_fork, s));
    for (int k = 0; k < 2; k++) HCHK(hipStreamWaitEvent(g_side[k], g_ev_fork, 0));
    launch_dec_pk(dpk + 48 * c0, cn, (G1AEntry*)vpk, (uint8_t*)vpkst, g_side[0]);
    HCHK(hipGetLastError());
    launch_dec_sig_lines(dsig + 96 * c0, cn, (uint8_t*)vsinf, (uint8_t*)vsst, (LineEntry*)vlines, g_side[1]);
    HCHK(hipGetLastError());
    for (int k = 0; k < 2; k++) {
      HCHK(hipEventRecord(g_ev_side[k], g_side[k]));
      HCHK(hipStreamWaitEvent(s, g_ev_side[k], 0));
    }
    if (hm_ready) HCHK(hipStreamWaitEvent(s, hm_ready, 0));
    hipEvent_t t0 = nullptr, t1 = nullptr;
    if (g_timing) {
      if (timing_pair(&t0, &t1)) return -1;
      HCHK(hipEventRecord(t0, s));
    }
    launch_pair3((const G1AEntry*)vpk, (const uint8_t*)vpkst, (const uint8_t*)vsinf, (const uint8_t*)vsst,
                 didx + c0, hm, (const LineEntry*)vlines, cn, dst + c0, s);
    if (g_timing) HCHK(hipEventRecord(t1, s));
    HCHK(hipGetLastError());
  }
  return 0;
}

// ThresholdAggregate / Aggregate members (herumi.go:249-286, 225-247): decompress + lambda
// digits (1 lane / partial), then lambda_j sigma_j as a 4-scalar Straus ladder (threshold.hip).
int ta_members_locked(const uint8_t* dsig, const int64_t* didx, const uint32_t* dgoff, size_t n_groups, size_t np,
                      int mode, G2JEntry* pts, uint8_t* mst, hipStream_t s) {
  if (np == 0) return 0;
  void *apts, *dig;
  void* tab;
  if (ensure(B_TAPTS, np * sizeof(HmEntry), &apts) || ensure(B_TADIG, np * sizeof(TaDigits), &dig) ||
      ensure(B_TATAB, ta_table_bytes((uint32_t)np), &tab))
    return -1;
  LAUNCH(k_ta_dec, np, s, dsig, (uint32_t)np, (HmEntry*)apts, mst);
  launch_ta_lambda(didx, dgoff, (uint32_t)n_groups, (uint32_t)np, mode, (TaDigits*)dig, mst, s);
  HCHK(hipGetLastError());
  launch_ta_straus((const HmEntry*)apts, (const TaDigits*)dig, (uint32_t)np, tab, pts, s);
  HCHK(hipGetLastError());
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int hbls_init(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  return init_locked(device);
}

const char* hbls_last_error(void) { return g_err.c_str(); }

int hbls_available(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return init_locked(-1) == 0 ? 1 : 0;
}

size_t hbls_hm_entry_bytes(void) { return sizeof(MsgEntry); }

int hbls_verify_batch(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, const uint64_t* msg_off,
                      const uint32_t* msg_len, size_t n, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n == 0) return 0;
  MsgTable t;
  dedup_messages(msgs, msg_off, msg_len, n, t);
  MsgEntry* hm;
  if (hash_table_locked(t, &hm, true)) return -1;
  uint8_t *dpk, *dsig, *dst;
  uint32_t* didx;
  if (upload(B_PK, pks, n * 48, &dpk)) return -1;
  if (upload(B_SIG, sigs, n * 96, &dsig)) return -1;
  if (upload(B_MIDX, t.idx.data(), n, &didx)) return -1;
  void* p;
  if (ensure(B_STAT, n, &p)) return -1;
  dst = (uint8_t*)p;
  if (verify_pipeline_locked(dpk, dsig, didx, hm, n, dst, g_stream)) return -1;
  HCHK(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

static int group_op_locked(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups,
                           int mode, uint8_t* out, uint8_t* status) {
  size_t np = grp_off[n_groups] - grp_off[0];
  if (grp_off[0] != 0) {
    g_err = "grp_off[0] must be 0";
    return -1;
  }
  for (size_t g = 0; g < n_groups; g++)
    if (grp_off[g + 1] < grp_off[g]) {
      g_err = "grp_off must be non-decreasing";
      return -1;
    }
  uint8_t* dsig;
  int64_t* didx = nullptr;
  uint32_t* dgoff;
  if (upload(B_SIG, sigs, np * 96, &dsig)) return -1;
  if (mode == 0 && upload(B_IDX, idx, np, &didx)) return -1;
  if (upload(B_GOFF, grp_off, n_groups + 1, &dgoff)) return -1;
  void *pts, *mst, *dout, *dst;
  if (ensure(B_PTS, np * sizeof(G2JEntry), &pts) || ensure(B_MSTAT, np, &mst) || ensure(B_OUT, n_groups * 96, &dout) ||
      ensure(B_STAT, n_groups, &dst))
    return -1;
  if (ta_members_locked(dsig, didx, dgoff, n_groups, np, mode, (G2JEntry*)pts, (uint8_t*)mst, g_stream)) return -1;
  LAUNCH(k_group_sum, n_groups, g_stream, dgoff, (uint32_t)n_groups, mode, (const G2JEntry*)pts, (const uint8_t*)mst,
         (uint8_t*)dout, (uint8_t*)dst);
  HCHK(hipMemcpyAsync(out, dout, n_groups * 96, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipMemcpyAsync(status, dst, n_groups, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

int hbls_threshold_aggregate_batch(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups,
                                   uint8_t* out, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n_groups == 0) return 0;
  return group_op_locked(sigs, idx, grp_off, n_groups, 0, out, status);
}

int hbls_aggregate_batch(const uint8_t* sigs, const uint32_t* grp_off, size_t n_groups, uint8_t* out,
                         uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n_groups == 0) return 0;
  return group_op_locked(sigs, nullptr, grp_off, n_groups, 1, out, status);
}

int hbls_verify_aggregate_batch(const uint8_t* pks, const uint32_t* grp_off, const uint8_t* sigs,
                                const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                                size_t n_groups, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n_groups == 0) return 0;
  size_t np = grp_off[n_groups];
  // one hash per group (messages need not be distinct)
  MsgTable t;
  t.idx.resize(n_groups);
  for (size_t g = 0; g < n_groups; g++) {
    t.off.push_back(t.bytes.size());
    t.len.push_back(msg_len[g]);
    t.bytes.insert(t.bytes.end(), msgs + msg_off[g], msgs + msg_off[g] + msg_len[g]);
  }
  MsgEntry* hm;
  if (hash_table_locked(t, &hm, false)) return -1;
  uint8_t *dpk, *dsig;
  uint32_t* dgoff;
  if (upload(B_PK, pks, np * 48, &dpk)) return -1;
  if (upload(B_SIG, sigs, n_groups * 96, &dsig)) return -1;
  if (upload(B_GOFF, grp_off, n_groups + 1, &dgoff)) return -1;
  void *pts, *mst, *dst;
  if (ensure(B_G1PTS, np * sizeof(G1AEntry), &pts) || ensure(B_MSTAT, np, &mst) || ensure(B_STAT, n_groups, &dst))
    return -1;
  LAUNCH(k_g1_member, np, g_stream, dpk, (uint32_t)np, (G1AEntry*)pts, (uint8_t*)mst);
  LAUNCH(k_verify_aggregate, n_groups, g_stream, dgoff, (uint32_t)n_groups, (const G1AEntry*)pts, (const uint8_t*)mst,
         dsig, (const MsgEntry*)hm, (uint8_t*)dst);
  HCHK(hipMemcpyAsync(status, dst, n_groups, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

int hbls_sign_batch(const uint8_t* sks, const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len,
                    size_t n, uint8_t* sigs, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n == 0) return 0;
  MsgTable t;
  dedup_messages(msgs, msg_off, msg_len, n, t);
  MsgEntry* hm;
  if (hash_table_locked(t, &hm, false)) return -1;
  uint8_t* dsk;
  uint32_t* didx;
  if (upload(B_SK, sks, n * 32, &dsk)) return -1;
  if (upload(B_MIDX, t.idx.data(), n, &didx)) return -1;
  void *dout, *dst;
  if (ensure(B_OUT, n * 96, &dout) || ensure(B_STAT, n, &dst)) return -1;
  LAUNCH(k_sign, n, g_stream, dsk, didx, hm, (uint32_t)n, (uint8_t*)dout, (uint8_t*)dst);
  HCHK(hipMemcpyAsync(sigs, dout, n * 96, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

int hbls_secret_to_public_key_batch(const uint8_t* sks, size_t n, uint8_t* pks, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (n == 0) return 0;
  uint8_t* dsk;
  if (upload(B_SK, sks, n * 32, &dsk)) return -1;
  void *dout, *dst;
  if (ensure(B_OUT, n * 48, &dout) || ensure(B_STAT, n, &dst)) return -1;
  LAUNCH(k_sk_to_pk, n, g_stream, dsk, (uint32_t)n, (uint8_t*)dout, (uint8_t*)dst);
  HCHK(hipMemcpyAsync(pks, dout, n * 48, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipMemcpyAsync(status, dst, n, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

int hbls_threshold_split(const uint8_t* secret, const uint8_t* coeffs, uint32_t total, uint32_t threshold,
                         uint8_t* shares, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  if (total == 0 || threshold == 0) return 0;
  std::vector<uint8_t> poly(32ull * threshold);
  memcpy(poly.data(), secret, 32);
  if (threshold > 1) memcpy(poly.data() + 32, coeffs, 32ull * (threshold - 1));
  uint8_t* dpoly;
  if (upload(B_SK, poly.data(), poly.size(), &dpoly)) return -1;
  void *dout, *dst;
  if (ensure(B_OUT, 32ull * total, &dout) || ensure(B_STAT, total, &dst)) return -1;
  LAUNCH(k_split, total, g_stream, dpoly, threshold, total, (uint8_t*)dout, (uint8_t*)dst);
  HCHK(hipMemcpyAsync(shares, dout, 32ull * total, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipMemcpyAsync(status, dst, total, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

int hbls_recover_secret(const uint8_t* shares, const int64_t* idx, size_t k, uint8_t* out, uint8_t* status) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  uint8_t* dsh;
  int64_t* didx;
  std::vector<uint8_t> dummy(32);
  if (upload(B_SK, k ? shares : dummy.data(), k ? 32 * k : 32, &dsh)) return -1;
  std::vector<int64_t> di(k ? k : 1, 0);
  if (k) memcpy(di.data(), idx, 8 * k);
  if (upload(B_IDX, di.data(), di.size(), &didx)) return -1;
  void *dout, *dst;
  if (ensure(B_OUT, 32, &dout) || ensure(B_STAT, 1, &dst)) return -1;
  hipLaunchKernelGGL(k_recover, dim3(1), dim3(64), 0, g_stream, dsh, didx, (uint32_t)k, (uint8_t*)dout,
                     (uint8_t*)dst);
  HCHK(hipGetLastError());
  HCHK(hipMemcpyAsync(out, dout, 32, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipMemcpyAsync(status, dst, 1, hipMemcpyDeviceToHost, g_stream));
  HCHK(hipStreamSynchronize(g_stream));
  return 0;
}

// ---- device-buffer entry points (bench / slot pipeline) ----
int hbls_hash_to_g2_device(const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len, size_t n_msgs,
                           void* hm, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  launch_hash_to_g2(msgs, msg_off, msg_len, (uint32_t)n_msgs, (MsgEntry*)hm, s);
  HCHK(hipGetLastError());
  launch_lines_msg((MsgEntry*)hm, (uint32_t)n_msgs, s);
  HCHK(hipGetLastError());
  return 0;
}

int hbls_verify_device(const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, const void* hm, size_t n,
                       uint8_t* status, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);  // the staged pipeline's workspaces are library-owned
  if (init_locked(-1)) return -1;
  if (n == 0) return 0;
  return verify_pipeline_locked(pks, sigs, msg_idx, (const MsgEntry*)hm, n, status, (hipStream_t)stream);
}

int hbls_threshold_aggregate_device(const uint8_t* sigs, const int64_t* idx, const uint32_t* grp_off, size_t n_groups,
                                    size_t n_partials, uint8_t* out, uint8_t* status, void* stream) {
  // workspace for member points is owned by the library (grow-only)
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  hipStream_t s = (hipStream_t)stream;
  void *pts, *mst;
  if (ensure(B_PTS, n_partials * sizeof(G2JEntry), &pts) || ensure(B_MSTAT, n_partials, &mst)) return -1;
  if (ta_members_locked(sigs, idx, grp_off, n_groups, n_partials, 0, (G2JEntry*)pts, (uint8_t*)mst, s)) return -1;
  LAUNCH(k_group_sum, n_groups, s, grp_off, (uint32_t)n_groups, 0, (const G2JEntry*)pts, (const uint8_t*)mst, out,
         status);
  return 0;
}

int hbls_slot_device(const uint8_t* msgs, const uint64_t* msg_off, const uint32_t* msg_len, size_t n_msgs, void* hm,
                     const uint8_t* pks, const uint8_t* sigs, const uint32_t* msg_idx, size_t n, uint8_t* vstatus,
                     const uint8_t* ta_sigs, const int64_t* ta_idx, const uint32_t* grp_off, size_t n_groups,
                     size_t n_ta_partials, uint8_t* ta_out, uint8_t* ta_status, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (init_locked(-1)) return -1;
  hipStream_t s = (hipStream_t)stream;
  HCHK(hipEventRecord(g_ev_slot, s));
  // messages: hash + Miller lines (side 2)
  hipStream_t sh = g_side[2];
  HCHK(hipStreamWaitEvent(sh, g_ev_slot, 0));
  launch_hash_to_g2(msgs, msg_off, msg_len, (uint32_t)n_msgs, (MsgEntry*)hm, sh);
  HCHK(hipGetLastError());
  launch_lines_msg((MsgEntry*)hm, (uint32_t)n_msgs, sh);
  HCHK(hipGetLastError());
  HCHK(hipEventRecord(g_ev_side[2], sh));
  // partial signatures (sides 0, 1, then s)
  if (n && verify_pipeline_locked(pks, sigs, msg_idx, (const MsgEntry*)hm, n, vstatus, s, g_ev_side[2])) return -1;
  // ThresholdAggregate on the library's own stream, which no other slot kernel uses: the runtime
  // has 4 hardware queues, and with five busy streams two would share one, serialising the
  // aggregation chain behind the hashing (profiles/r01h_slot_timeline.txt).  In-order with the
  // host-buffer entry points that share its workspaces.
  hipStream_t st = g_stream;
  HCHK(hipStreamWaitEvent(st, g_ev_slot, 0));
  if (n_groups) {
    void *pts, *mst;
    if (ensure(B_PTS, n_ta_partials * sizeof(G2JEntry), &pts) || ensure(B_MSTAT, n_ta_partials, &mst)) return -1;
    if (ta_members_locked(ta_sigs, ta_idx, grp_off, n_groups, n_ta_partials, 0, (G2JEntry*)pts, (uint8_t*)mst, st))
      return -1;
    LAUNCH(k_group_sum, n_groups, st, grp_off, (uint32_t)n_groups, 0, (const G2JEntry*)pts, (const uint8_t*)mst,
           ta_out, ta_status);
  }
  HCHK(hipEventRecord(g_ev_side[3], st));
  HCHK(hipStreamWaitEvent(s, g_ev_side[2], 0));
  HCHK(hipStreamWaitEvent(s, g_ev_side[3], 0));
  return 0;
}

int hbls_timing(int enable) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_timing = enable != 0;
  g_tev_used = 0;
  return 0;
}

int hbls_timing_read(float* ms, size_t max_n, size_t* n_out) {
  std::lock_guard<std::mutex> lk(g_mu);
  size_t n = g_tev_used < max_n ? g_tev_used : max_n;
  for (size_t i = 0; i < n; i++) {
    HCHK(hipEventSynchronize(g_tev[i].second));
    HCHK(hipEventElapsedTime(&ms[i], g_tev[i].first, g_tev[i].second));
  }
  *n_out = n;
  return 0;
}

int hbls_sync(void* stream) {
  HCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

}  // extern "C"
