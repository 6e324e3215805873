// hash.hip: hash_to_curve G2 of the distinct messages (RFC 9380, DST BLS_SIG_..._POP_), the
// first stage of tbls.Verify / Sign (herumi.go:288-316).
//
// Compiled WITHOUT HB_FAST_FPMUL: the hashing's building blocks (expand_message_xmd, SSWU, the
// 3-isogeny, cofactor clearing, the exponentiations) stay separate functions.  Inlined into one
// kernel they left the register allocator ~21 KB of spills per lane at two waves per SIMD, and the
// scratch the runtime must reserve for that (x 2 waves x 4 SIMDs x 256 CUs, per hardware queue)
// exhausted the device's scratch with two slots in flight.
#include "layout.h"

#include <stdlib.h>

namespace hb {

constexpr int BLOCK = 64;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ G2J xch_pair(const G2J& p) {  // the point of lane ^ 1
  G2J r;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* d = reinterpret_cast<uint32_t*>(&r);
  const int addr = (int)((threadIdx.x ^ 1u) << 2);
  HB_UNROLL for (int k = 0; k < (int)(sizeof(G2J) / 4); k++)
    d[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)s[k]);
  return r;
}
#endif

// Two lanes per distinct message: hash_to_curve G2 (RFC 9380, DST ..._POP_), affine.  Both lanes
// expand the message; the even lane maps u0, the odd lane u1 (SSWU + 3-isogeny, the larger half
// of the work, in parallel), then the even lane adds the pair and clears the cofactor.
__global__ KB_OCC(HB_OCC_HASH) void k_hash_to_g2(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ off,
                                           const uint32_t* __restrict__ len, uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = t >> 1;
  const bool odd = (t & 1u) != 0;
  const uint32_t ii = i < n ? i : n - 1;  // every lane takes part in the exchange
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msgs + off[ii], len[ii]);
  Fp2 x, y;
  sswu_map(x, y, odd ? u1 : u0);
  const G2J q = iso3_map(x, y);
  const G2J q1 = xch_pair(q);
  if (odd || i >= n) return;
  G2A h = jac_to_aff(g2_clear_cofactor(jac_add(q, q1)));
  HmEntry e;
  e.x = h.x;
  e.y = h.y;
  e.inf = h.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  hm[i].h = e;
#endif
}


// One lane per distinct message (hash_to_g2, h2c.h): the same result with no idle partner lane
// during the cofactor clearing and no duplicated expand_message -- fewer lane-cycles per
// message, half the lanes.  Used when the call has enough messages to fill the chip.
__global__ KB_OCC(HB_OCC_HASH) void k_hash_to_g2_1(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ off,
                                                   const uint32_t* __restrict__ len, uint32_t n,
                                                   MsgEntry* __restrict__ hm) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2A h = jac_to_aff(hash_to_g2(msgs + off[i], len[i]));
  HmEntry e;
  e.x = h.x;
  e.y = h.y;
  e.inf = h.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  hm[i].h = e;
}

// messages from which one lane per message fills the chip (HBLS_HASH_ONE_LANE, default 65536);
// g_hash_split = 0 (HBLS_HASH_SPLIT=0) takes the kernels of this file instead of hashsplit.hip's --
// kept as the cross-check of tests/test_gpu_scale.py.  Both read at init, set by hbls_tune.
std::atomic<size_t> g_hash_one_lane{65536}, g_hash_split{1};

void launch_hash_to_g2(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                       hipStream_t s) {
  if (!n) return;
  // default: the staged fast-unit kernels (hashsplit.hip)
  if (g_hash_split.load(std::memory_order_relaxed)) {
    launch_hash_to_g2_split(msgs, off, len, n, hm, s);
    return;
  }
  if (n >= g_hash_one_lane.load(std::memory_order_relaxed))
    hipLaunchKernelGGL(k_hash_to_g2_1, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, msgs, off, len,
                       n, hm);
  else
    hipLaunchKernelGGL(k_hash_to_g2, dim3((unsigned)((2 * (size_t)n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       msgs, off, len, n, hm);
}

}  // namespace hb
