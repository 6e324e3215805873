// hashsplit.hip: hash_to_curve G2 of the distinct messages (RFC 9380, DST BLS_SIG_..._POP_; the
// first stage of tbls.Verify / Sign, herumi.go:288-316) as six kernels compiled like the other
// fast units (HB_FAST_FPMUL: everything but the Fp product inlined).
//
//   k_h2c_field   one lane per message: expand_message_xmd (SHA-256) -> u0, u1 in Fp2
//   k_h2c_map     one lane per (message, i): the inversion-free SSWU map + 3-isogeny of u_i
//   k_h2c_clear1, 1b, 2, 3  one lane per message: Q0 + Q1, cofactor clearing, affine -> hm[i].h
//
// One kernel with the whole chain needs either the standard calling convention for its building
// blocks (hash.hip: 3.8 KB of call stack per lane, ~20 GB of scratch traffic per C3 slot) or, inlined,
// ~21 KB of spills; split, each stage holds only its own working set.  The stages hand over through
// the message's own MsgEntry: u0, u1 and Q0, Q1 sit in its line area (lines[0..2]) until k_lines_msg
// writes the lines there.
#define HB_FAST_FPMUL 1
#include "layout.h"

#include <stdlib.h>

namespace hb {

constexpr int HBLOCK = 64;

#if defined(__HIP_DEVICE_COMPILE__)
// the hand-over slots in a MsgEntry's line area (LineEntry = 3 Fp2 = 288 B)
__device__ __forceinline__ Fp2* h2c_u(MsgEntry* e) { return reinterpret_cast<Fp2*>(&e->lines[0]); }  // u0, u1
__device__ __forceinline__ G2JEntry* h2c_q(MsgEntry* e) { return reinterpret_cast<G2JEntry*>(&e->lines[1]); }  // Q0, Q1 / P, t1, t2
static_assert(2 * sizeof(Fp2) <= sizeof(LineEntry), "u0, u1 fit line 0");
static_assert(3 * sizeof(G2JEntry) <= 3 * sizeof(LineEntry), "Q0, Q1 (later P, t1, t2) fit lines 1..3");
#endif

__global__ __launch_bounds__(64) void k_h2c_field(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ len, uint32_t n,
                                                  MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msgs + off[i], len[i]);
  Fp2* u = h2c_u(hm + i);
  u[0] = u0;
  u[1] = u1;
#endif
}

__global__ KB_OCC(HB_OCC_HASH) void k_h2c_map(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  MsgEntry* e = hm + (t >> 1);
  const G2J q = sswu_iso_map(h2c_u(e)[t & 1u]);
  h2c_q(e)[t & 1u] = {q.X, q.Y, q.Z};
#endif
}

// Cofactor clearing h_eff P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P) (RFC 9380 G.3, as
// g2_clear_cofactor: with t1 = [x] P and t2 = [x](t1 + psi(P)), h = psi^2(2P) - psi(P) - P - t1 + t2)
// in four kernels, the points that must outlive a ladder parked in the message's line area rather
// than held in registers across it:
//   k_h2c_clear1  P = Q0 + Q1, t1 = [x] P                                                -> (P, t1)
//   k_h2c_clear1b u = t1 + psi(P), v = psi^2(2P) - psi(P) - P - t1                          -> (u, v)
//   k_h2c_clear2  h = [x] u + v                                                          -> h
//   k_h2c_clear3  h affine                                                               -> hm[i].h
// the two [x] ladders in lazily reduced 28-bit limbs (ec28.h)
__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear1(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2JEntry* q = h2c_q(hm + i);
  G2J P;
  {
    const G2JEntry a = q[0], b = q[1];
    P = jac_add(G2J{a.X, a.Y, a.Z}, G2J{b.X, b.Y, b.Z});
  }
  q[0] = {P.X, P.Y, P.Z};
  const G2JEntry* src = q;
  const G2J t1 = jac_neg(g2l_mul_by_xabs_l([src]() { return G2J{src->X, src->Y, src->Z}; }));  // [x] P (x < 0)
  q[1] = {t1.X, t1.Y, t1.Z};
#endif
}

__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear1b(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2JEntry* q = h2c_q(hm + i);
  const G2JEntry pe = q[0], te = q[1];
  const G2J P = {pe.X, pe.Y, pe.Z}, t1 = {te.X, te.Y, te.Z};
  const G2J pp = g2_psi(P);
  const G2J u = jac_add(t1, pp);
  q[1] = {u.X, u.Y, u.Z};
  const G2J v = jac_add(g2_psi2(jac_dbl(P)), jac_neg(jac_add(jac_add(pp, P), t1)));
  q[2] = {v.X, v.Y, v.Z};
#endif
}

__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear2(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2JEntry* q = h2c_q(hm + i);
  const G2JEntry* src = q + 1;
  const G2J t2 = jac_neg(g2l_mul_by_xabs_l([src]() { return G2J{src->X, src->Y, src->Z}; }));
  const G2JEntry ve = q[2];
  const G2J h = jac_add(t2, G2J{ve.X, ve.Y, ve.Z});
  q[0] = {h.X, h.Y, h.Z};
#endif
}

// The two ladder kernels with each message's G2 arithmetic split over a lane pair (ec28.h F2Half:
// each lane computes one coefficient of every Fp2 product, ~60 % of the one-lane instruction
// stream per lane): for calls with too few messages to fill the chip, where the ladders' latency,
// not their lane-cycles, is what the caller waits for.  Same outputs as k_h2c_clear1 / 2.
__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear1h(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (i >= n) return;  // both lanes of a pair
  const F2Half m = f2half_make();
  G2JEntry* q = h2c_q(hm + i);
  G2J P;
  {
    const G2JEntry a = q[0], b = q[1];
    P = jac_add(G2J{a.X, a.Y, a.Z}, G2J{b.X, b.Y, b.Z});
  }
  q[0] = {P.X, P.Y, P.Z};  // the same words from both lanes
  const G2JEntry* src = q;
  const G2J t1 = jac_neg(g2l_mul_by_xabs_l([src]() { return G2J{src->X, src->Y, src->Z}; }, m));
  if (m.h == 0) q[1] = {t1.X, t1.Y, t1.Z};
#endif
}

__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear2h(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (i >= n) return;
  const F2Half m = f2half_make();
  G2JEntry* q = h2c_q(hm + i);
  const G2JEntry* src = q + 1;
  const G2J t2 = jac_neg(g2l_mul_by_xabs_l([src]() { return G2J{src->X, src->Y, src->Z}; }, m));
  if (m.h) return;
  const G2JEntry ve = q[2];
  const G2J h = jac_add(t2, G2J{ve.X, ve.Y, ve.Z});
  q[0] = {h.X, h.Y, h.Z};
#endif
}

__global__ KB_OCC(HB_OCC_HASH) void k_h2c_clear3(uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G2JEntry he = h2c_q(hm + i)[0];
  const G2A ha = jac_to_aff(G2J{he.X, he.Y, he.Z});
  HmEntry e;
  e.x = ha.x;
  e.y = ha.y;
  e.inf = ha.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  hm[i].h = e;
#endif
}

// messages up to which the ladders run on lane pairs (HBLS_HASH_PAIR_MAX, read once at init;
// default 16384: 512 wavefronts, half a wave per SIMD -- below it the one-lane ladders leave the
// chip idle)
std::atomic<size_t> g_hash_pair_max{16384};
static size_t hash_pair_max() { return g_hash_pair_max.load(std::memory_order_relaxed); }

void launch_hash_to_g2_split(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                             hipStream_t s) {
  if (!n) return;
  const unsigned g1 = (unsigned)(((size_t)n + HBLOCK - 1) / HBLOCK), g2 = (unsigned)((2 * (size_t)n + HBLOCK - 1) / HBLOCK);
  const bool pair = n <= hash_pair_max();
  hipLaunchKernelGGL(k_h2c_field, dim3(g1), dim3(HBLOCK), 0, s, msgs, off, len, n, hm);
  hipLaunchKernelGGL(k_h2c_map, dim3(g2), dim3(HBLOCK), 0, s, n, hm);
  if (pair)
    hipLaunchKernelGGL(k_h2c_clear1h, dim3(g2), dim3(HBLOCK), 0, s, n, hm);
  else
    hipLaunchKernelGGL(k_h2c_clear1, dim3(g1), dim3(HBLOCK), 0, s, n, hm);
  hipLaunchKernelGGL(k_h2c_clear1b, dim3(g1), dim3(HBLOCK), 0, s, n, hm);
  if (pair)
    hipLaunchKernelGGL(k_h2c_clear2h, dim3(g2), dim3(HBLOCK), 0, s, n, hm);
  else
    hipLaunchKernelGGL(k_h2c_clear2, dim3(g1), dim3(HBLOCK), 0, s, n, hm);
  hipLaunchKernelGGL(k_h2c_clear3, dim3(g1), dim3(HBLOCK), 0, s, n, hm);
}

}  // namespace hb
