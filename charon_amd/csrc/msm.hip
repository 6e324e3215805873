// msm.hip: the signature side of a whole verification as ONE multi-scalar multiplication
// (bucket method), for the batched check of vbatch.hip / vgroup.hip.
//
// With random r_i = a_i + b_i lambda (rlc.h) the check over every READY group g of a call is
//     prod_g e(P_g, H(m_g)) * e(-g1, S) == 1,   S = sum_i [r_i] sig_i = sum_i [a_i] sig_i + [b_i] (-psi^2 sig_i),
// so the signature side needs no per-group sums: S is one MSM of 2 (n + n_agg) affine points with
// 32-bit scalars.  Bucket method with c = 16-bit windows (two windows): every (point, window) pair
// with a nonzero digit d is one entry of bucket (window, d); the entries are sorted by bucket with
// a counting sort (histogram, scan, scatter); one lane sums a bucket with mixed additions; buckets
// are weighed by running sums over chunks of 16 (plus one 16-bit multiple per chunk) and the chunk
// results summed by wave butterflies.  Per entry that is ONE mixed G2 addition (~29 Fp products)
// where the per-group ladders spent ~1 400 Fp products per item.
//
// Only items whose group is READY (group_scan, vgroup.hip) with a nonzero coefficient enter the
// sum.  If the slot-wide check fails, the per-group path runs (hipbls.hip verify_pipeline), so
// verdicts are those of the per-group check.
#define HB_FAST_FPMUL 1
#include "lines.h"
#include "pair3.h"

namespace hb {

constexpr int BLOCK = 64;

// The reduction and the butterflies run 128 and at most 64 waves: far fewer than the SIMDs, so
// they are latency-bound and take one wave per SIMD's full register file (no scratch spills).
#define HB_OCC_MSMBUCKET HB_OCC_RLC
#define HB_OCC_MSMTAIL 1

__device__ __forceinline__ bool msm_take(const G2MsmArgs& a, uint32_t i, uint2& ab) {
  ab = a.coef[i];
  if ((ab.x | ab.y) == 0) return false;
  // coefficients are drawn from the keys alone (the combination runs beside the signatures'
  // subgroup checks and the aggregation): an item enters as group_scan takes it -- signature
  // status OK, not at infinity
  if (i < a.n) return a.gst[a.igrp[i]] == G_READY && !a.sig_st[i] && !a.sig[i].inf;
  const uint32_t g = i - a.n;
  return a.gst[g] == G_READY && !a.agg_st[g] && !a.agg_sig[g].inf;
}

// one lane per item: bucket sizes
__global__ __launch_bounds__(64) void k_msm_count(G2MsmArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n + a.n_agg) return;
  uint2 ab;
  if (!msm_take(a, i, ab)) return;
  HB_UNROLL for (int h = 0; h < 2; h++) {
    const uint32_t s = h ? ab.y : ab.x;
    HB_UNROLL for (int w = 0; w < MSM_WINDOWS; w++) {
      const uint32_t d = (s >> (MSM_C * w)) & MSM_MASK;
      if (d) atomicAdd(a.cnt + ((uint32_t)w << MSM_C) + d, 1u);
    }
  }
}

// one lane per item: entries (item << 1 | half) into their buckets' ranges
__global__ __launch_bounds__(64) void k_msm_fill(G2MsmArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n + a.n_agg) return;
  uint2 ab;
  if (!msm_take(a, i, ab)) return;
  HB_UNROLL for (int h = 0; h < 2; h++) {
    const uint32_t s = h ? ab.y : ab.x;
    HB_UNROLL for (int w = 0; w < MSM_WINDOWS; w++) {
      const uint32_t d = (s >> (MSM_C * w)) & MSM_MASK;
      if (d) {
        const uint32_t k = ((uint32_t)w << MSM_C) + d;
        a.ent[a.off[k] + atomicAdd(a.cur + k, 1u)] = (i << 1) | (uint32_t)h;
      }
    }
  }
}

// one workgroup: the buckets in decreasing order of size (counting sort on the sizes, capped at
// 255), so that the lanes of a wave of k_msm_bucket sum buckets of nearly equal size (lane per
// bucket in key order: Poisson sizes, a wave waits for its largest)
__global__ __launch_bounds__(1024) void k_msm_order(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ order) {
  __shared__ uint32_t hist[256];
  const uint32_t t = threadIdx.x;
  if (t < 256) hist[t] = 0;
  __syncthreads();
  for (uint32_t k = t; k < MSM_KEYS; k += 1024) atomicAdd(&hist[255u - min(cnt[k], 255u)], 1u);
  __syncthreads();
  if (t == 0) {  // exclusive scan, largest sizes first
    uint32_t run = 0;
    for (int b = 0; b < 256; b++) {
      const uint32_t c = hist[b];
      hist[b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (uint32_t k = t; k < MSM_KEYS; k += 1024) order[atomicAdd(&hist[255u - min(cnt[k], 255u)], 1u)] = k;
}

// one lane per bucket (in the order of k_msm_order): the sum of its points (half 1: -psi^2 of the
// signature), in lazily reduced 28-bit limbs (ec28.h g2l_madd)
__global__ KB_OCC(HB_OCC_MSMBUCKET) void k_msm_bucket(G2MsmArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t L = blockIdx.x * blockDim.x + threadIdx.x;
  if (L >= MSM_KEYS) return;
  const uint32_t k = a.order[L];
  const uint32_t b = a.off[k], e = a.off[k + 1];
  G2L acc = g2l_infinity();
  HB_NOUNROLL for (uint32_t j = b; j < e; j++) {
    const uint32_t u = a.ent[j], i = u >> 1;
    const HmEntry se = i < a.n ? a.sig[i] : a.agg_sig[i - a.n];
    G2A P = {se.x, se.y, false};
    if (u & 1u) P = {f2_mul_fp(P.x, fp_from_const(PSI2_CX[0])), f2_neg(f2_mul_fp(P.y, fp_from_const(PSI2_CY[0]))), false};
    acc = g2l_madd(acc, f2l_from(P.x), f2l_from(P.y));
  }
  const G2J r = g2l_to_jac(acc);
  a.bucket[k] = {r.X, r.Y, r.Z};
#endif
}

// [m] p for a 16-bit m (uniform control flow: every step's addition computed, kept per lane)
__device__ __forceinline__ G2J mul16(const G2J& p, uint32_t m) {
  G2J r = jac_infinity<Fp2>();
  HB_NOUNROLL for (int bit = 15; bit >= 0; bit--) {
    r = jac_dbl(r);
    const G2J t = jac_add(r, p);
    const bool take = ((m >> bit) & 1u) != 0;
    r = {take ? t.X : r.X, take ? t.Y : r.Y, take ? t.Z : r.Z};
  }
  return r;
}

// one lane per chunk of MSM_CHUNK buckets of one window: sum_d d * 2^(16 w) B_d over the chunk,
// as running sums T = sum_j (j + 1) B_(lo + j), R = sum_j B_(lo + j), then T + (lo - 1) R
__global__ KB_OCC(HB_OCC_MSMTAIL) void k_msm_reduce(G2MsmArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= MSM_PARTS) return;
  constexpr uint32_t per_w = (1u << MSM_C) / MSM_CHUNK;
  const uint32_t w = c / per_w, lo = (c % per_w) * MSM_CHUNK;
  const G2JEntry* B = a.bucket + ((size_t)w << MSM_C) + lo;
  G2J R = jac_infinity<Fp2>(), T = jac_infinity<Fp2>();
  HB_NOUNROLL for (int j = (int)MSM_CHUNK - 1; j >= 0; j--) {
    const G2JEntry q = B[j];
    R = jac_add(R, G2J{q.X, q.Y, q.Z});
    T = jac_add(T, R);
  }
  G2J W;
  if (lo == 0) W = jac_add(T, jac_neg(R));  // (lo - 1) = -1
  else W = jac_add(T, mul16(R, lo - 1));
  HB_NOUNROLL for (uint32_t k = 0; k < MSM_C * w; k++) W = jac_dbl(W);  // wave-uniform
  a.part[c] = {W.X, W.Y, W.Z};
#endif
}

// sum of m Jacobian points: workgroup b (one wave) sums in[b * 64 q, (b + 1) * 64 q) into out[b]
__global__ KB_OCC(HB_OCC_MSMTAIL) void k_msm_sum(const G2JEntry* __restrict__ in, uint32_t m, uint32_t q,
                                             G2JEntry* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lane = threadIdx.x & 63u, base = blockIdx.x * 64u * q;
  G2J S = jac_infinity<Fp2>();
  HB_NOUNROLL for (uint32_t j = 0; j < q; j++) {
    const uint32_t i = base + j * 64u + lane;
    if (i < m) {
      const G2JEntry e = in[i];
      S = jac_add(S, G2J{e.X, e.Y, e.Z});
    }
  }
  HB_NOUNROLL for (int off = 32; off; off >>= 1) {
    const int addr = (int)((lane ^ (uint32_t)off) << 2);
    const G2J T = {xch(S.X, addr), xch(S.Y, addr), xch(S.Z, addr)};
    S = jac_add(S, T);
  }
  if (lane == 0) out[blockIdx.x] = {S.X, S.Y, S.Z};
#endif
}

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

void launch_msm_count(const G2MsmArgs& a, hipStream_t s) {
  const size_t n = (size_t)a.n + a.n_agg;
  if (n) hipLaunchKernelGGL(k_msm_count, dim3(blocks_for(n)), dim3(BLOCK), 0, s, a);
}
void launch_msm_fill(const G2MsmArgs& a, hipStream_t s) {
  const size_t n = (size_t)a.n + a.n_agg;
  if (n) hipLaunchKernelGGL(k_msm_fill, dim3(blocks_for(n)), dim3(BLOCK), 0, s, a);
}
void launch_msm_bucket(const G2MsmArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_msm_order, dim3(1), dim3(1024), 0, s, (const uint32_t*)a.cnt, a.order);
  hipLaunchKernelGGL(k_msm_bucket, dim3(blocks_for(MSM_KEYS)), dim3(BLOCK), 0, s, a);
}
void launch_msm_reduce(const G2MsmArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_msm_reduce, dim3(blocks_for(MSM_PARTS)), dim3(BLOCK), 0, s, a);
}
// part[MSM_PARTS] -> part2[n2 <= 64] -> total[0]: q entries per lane in the first pass
void launch_msm_sum(const G2MsmArgs& a, hipStream_t s) {
  constexpr uint32_t q = MSM_PARTS >= 64 * 64 ? MSM_PARTS / (64 * 64) : 1u, n2 = MSM_PARTS / (64 * q);
  static_assert(MSM_PARTS % (64 * q) == 0 && n2 <= 64 && n2 <= MSM_PARTS / 128, "two butterfly passes");
  hipLaunchKernelGGL(k_msm_sum, dim3(n2), dim3(BLOCK), 0, s, (const G2JEntry*)a.part, MSM_PARTS, q, a.part2);
  hipLaunchKernelGGL(k_msm_sum, dim3(1), dim3(BLOCK), 0, s, (const G2JEntry*)a.part2, n2, 1u, a.total);
}

}  // namespace hb
