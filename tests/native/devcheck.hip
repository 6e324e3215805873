// TEST-ONLY device harness: runs building blocks of the gfx950 kernels (charon_amd/csrc/*.h,
// compiled exactly as the product's fast translation units) one lane per case, so
// tests/test_gpu_blocks.py can compare them with the host harness and the oracle.  The product
// library never loads this.
#define HB_FAST_FPMUL 1
#include "../../charon_amd/csrc/layout.h"
#include "../../charon_amd/csrc/rlc.h"

using namespace hb;

// case i: (pk, sig, a, b) -> compressed [a + b lambda] pk, [a + b lambda] sig, and the sum of the
// two cases i, i+1 (Jacobian adds, affine) in sum48 / sum96 (last case: itself)
__global__ __launch_bounds__(64) void k_dc_rlc(const uint8_t* pks, const uint8_t* sigs, const uint32_t* ab, int n,
                                               uint8_t* out48, uint8_t* out96, uint8_t* sum48, uint8_t* sum96) {
#if defined(__HIP_DEVICE_COMPILE__)
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A p;
  G2A q;
  g1_decompress(p, pks + 48 * i);
  g2_decompress(q, sigs + 96 * i);
  const G1J rp = rlc_g1(p, ab[2 * i], ab[2 * i + 1]);
  const G2J rq = rlc_g2(q, ab[2 * i], ab[2 * i + 1]);
  uint8_t b48[48], b96[96];
  g1_compress(b48, jac_to_aff(rp));
  g2_compress(b96, jac_to_aff(rq));
  for (int k = 0; k < 48; k++) out48[48 * i + k] = b48[k];
  for (int k = 0; k < 96; k++) out96[96 * i + k] = b96[k];
  const int j = i + 1 < n ? i + 1 : i;
  G1A p2;
  G2A q2;
  g1_decompress(p2, pks + 48 * j);
  g2_decompress(q2, sigs + 96 * j);
  const G1J sp = j == i ? rp : jac_add(rp, rlc_g1(p2, ab[2 * j], ab[2 * j + 1]));
  const G2J sq = j == i ? rq : jac_add(rq, rlc_g2(q2, ab[2 * j], ab[2 * j + 1]));
  g1_compress(b48, jac_to_aff(sp));
  g2_compress(b96, jac_to_aff(sq));
  for (int k = 0; k < 48; k++) sum48[48 * i + k] = b48[k];
  for (int k = 0; k < 96; k++) sum96[96 * i + k] = b96[k];
#endif
}

extern "C" int dc_rlc(const uint8_t* pks, const uint8_t* sigs, const uint32_t* ab, int n, uint8_t* out48,
                      uint8_t* out96, uint8_t* sum48, uint8_t* sum96) {
  uint8_t *dpk, *dsig, *o48, *o96, *s48, *s96;
  uint32_t* dab;
  if (hipMalloc(&dpk, 48 * n) || hipMalloc(&dsig, 96 * n) || hipMalloc(&dab, 8 * n) || hipMalloc(&o48, 48 * n) ||
      hipMalloc(&o96, 96 * n) || hipMalloc(&s48, 48 * n) || hipMalloc(&s96, 96 * n))
    return -1;
  hipMemcpy(dpk, pks, 48 * n, hipMemcpyHostToDevice);
  hipMemcpy(dsig, sigs, 96 * n, hipMemcpyHostToDevice);
  hipMemcpy(dab, ab, 8 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_dc_rlc, dim3((n + 63) / 64), dim3(64), 0, 0, dpk, dsig, dab, n, o48, o96, s48, s96);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  hipMemcpy(out48, o48, 48 * n, hipMemcpyDeviceToHost);
  hipMemcpy(out96, o96, 96 * n, hipMemcpyDeviceToHost);
  hipMemcpy(sum48, s48, 48 * n, hipMemcpyDeviceToHost);
  hipMemcpy(sum96, s96, 96 * n, hipMemcpyDeviceToHost);
  for (void* p : {(void*)dpk, (void*)dsig, (void*)dab, (void*)o48, (void*)o96, (void*)s48, (void*)s96}) hipFree(p);
  return 0;
}

// jac_add of two Jacobian G1 / G2 points with Z != 1: case i adds [k1] Q and [k2] Q (Q = the
// case's decompressed pk / sig, k from the double-and-add of jac_mul_aff), compressed
__global__ __launch_bounds__(64) void k_dc_jac_add(const uint8_t* pks, const uint8_t* sigs, const uint32_t* ks, int n,
                                                   uint8_t* out48, uint8_t* out96) {
#if defined(__HIP_DEVICE_COMPILE__)
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A p;
  G2A q;
  g1_decompress(p, pks + 48 * i);
  g2_decompress(q, sigs + 96 * i);
  const uint32_t k1 = ks[2 * i], k2 = ks[2 * i + 1];
  const G1J a1 = jac_mul_aff(p, &k1, 32), a2 = jac_mul_aff(p, &k2, 32);
  const G2J b1 = jac_mul_aff(q, &k1, 32), b2 = jac_mul_aff(q, &k2, 32);
  uint8_t b48[48], b96[96];
  g1_compress(b48, jac_to_aff(jac_add(a1, a2)));
  g2_compress(b96, jac_to_aff(jac_add(b1, b2)));
  for (int k = 0; k < 48; k++) out48[48 * i + k] = b48[k];
  for (int k = 0; k < 96; k++) out96[96 * i + k] = b96[k];
#endif
}

extern "C" int dc_jac_add(const uint8_t* pks, const uint8_t* sigs, const uint32_t* ks, int n, uint8_t* out48,
                          uint8_t* out96) {
  uint8_t *dpk, *dsig, *o48, *o96;
  uint32_t* dk;
  if (hipMalloc(&dpk, 48 * n) || hipMalloc(&dsig, 96 * n) || hipMalloc(&dk, 8 * n) || hipMalloc(&o48, 48 * n) ||
      hipMalloc(&o96, 96 * n))
    return -1;
  hipMemcpy(dpk, pks, 48 * n, hipMemcpyHostToDevice);
  hipMemcpy(dsig, sigs, 96 * n, hipMemcpyHostToDevice);
  hipMemcpy(dk, ks, 8 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_dc_jac_add, dim3((n + 63) / 64), dim3(64), 0, 0, dpk, dsig, dk, n, o48, o96);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  hipMemcpy(out48, o48, 48 * n, hipMemcpyDeviceToHost);
  hipMemcpy(out96, o96, 96 * n, hipMemcpyDeviceToHost);
  for (void* p : {(void*)dpk, (void*)dsig, (void*)dk, (void*)o48, (void*)o96}) hipFree(p);
  return 0;
}
