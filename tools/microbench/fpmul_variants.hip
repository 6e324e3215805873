// Fp Montgomery-product variants on gfx950: throughput and bit-exact agreement.
//
//   generic  12 x 32-bit CIOS, plain C++ (the compiler lowers and schedules everything)
//   asm      12 x 32-bit product scanning, inline-asm v_mad_u64_u32 + v_addc_co_u32 pairs with
//            the carry read immediately after the VCC write (the r01 product, fp.h fips_mac*)
//   asmnop   the same with `s_nop 1` between the VCC write and its read (the wait states the
//            compiler's hazard recognizer inserts between a VALU carry write and a carry read)
//   r29      14 x 29-bit product scanning, one 64-bit accumulator per column, no carry word
//   r29x2    14 x 29-bit, two interleaved accumulators per column
//   r29sq    14 x 29-bit squaring (x <- x^2 chain; compared against generic's x*x chain)
//
// Every lane runs two independent chains of ITERS products; outputs are converted back to
// canonical 12 x 32-bit values and compared on the host with `generic`.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "fpmul_consts.h"

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr uint32_t M29 = (1u << 29) - 1;

// ------------------------------------------------------------------ 12 x 32 generic CIOS
__device__ __forceinline__ void mul_generic(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t A = (uint64_t)a[0] * b[i] + t[0];
    t[0] = (uint32_t)A;
    A >>= 32;
    uint32_t m = t[0] * N0_32;
    uint64_t C = (uint64_t)m * P32[0] + t[0];
    C >>= 32;
#pragma unroll
    for (int j = 1; j < 12; j++) {
      A = (uint64_t)a[j] * b[i] + t[j] + A;
      t[j] = (uint32_t)A;
      A >>= 32;
      C = (uint64_t)m * P32[j] + t[j] + C;
      t[j - 1] = (uint32_t)C;
      C >>= 32;
    }
    t[11] = (uint32_t)(C + A);
  }
#pragma unroll
  for (int j = 0; j < 12; j++) r[j] = t[j];
}

// ------------------------------------------------------------------ 12 x 32 inline-asm FIPS
template <bool NOP>
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  if (NOP)
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                 : "+v"(acc), "+v"(c2) : "v"(a), "v"(b) : "vcc");
  else
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                 : "+v"(acc), "+v"(c2) : "v"(a), "v"(b) : "vcc");
}

template <bool NOP>
__device__ __forceinline__ void mul_asm(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[12];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 23; k++) {
    const int lo = k < 12 ? 0 : k - 11;
    const int hi = k < 12 ? k - 1 : 11;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      mac<NOP>(acc, c2, a[j], b[k - j]);
      mac<NOP>(acc, c2, m[j], P32[k - j]);
    }
    if (k < 12) {
      mac<NOP>(acc, c2, a[k], b[0]);
      m[k] = (uint32_t)acc * N0_32;
      mac<NOP>(acc, c2, m[k], P32[0]);
    } else {
      r[k - 12] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  r[11] = (uint32_t)acc;
}

// ------------------------------------------------------------------ 14 x 29 product scanning
// a, b < 2^29 per limb; output limbs < 2^29, value < 2p for a, b < 2^12 p.
__device__ __forceinline__ void mul_r29(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
#pragma unroll
    for (int j = lo; j <= hi; j++) acc += (uint64_t)a[j] * b[k - j];
#pragma unroll
    for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P29[k - j];
    if (k < 14) {
      m[k] = ((uint32_t)acc * N0_29) & M29;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r[k - 14] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  r[13] = (uint32_t)acc;
}

__device__ __forceinline__ void mul_r29x2(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[14];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
    uint64_t s0 = carry, s1 = 0;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      if ((j & 1) == 0) s0 += (uint64_t)a[j] * b[k - j];
      else s1 += (uint64_t)a[j] * b[k - j];
    }
#pragma unroll
    for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) {
        if ((j & 1) == 0) s1 += (uint64_t)m[j] * P29[k - j];
        else s0 += (uint64_t)m[j] * P29[k - j];
      }
    uint64_t acc = s0 + s1;
    if (k < 14) {
      m[k] = ((uint32_t)acc * N0_29) & M29;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r[k - 14] = (uint32_t)acc & M29;
    }
    carry = acc >> 29;
  }
  r[13] = (uint32_t)carry;
}

// squaring: a_j a_{k-j} for j < k-j taken once against the doubled limb
__device__ __forceinline__ void sqr_r29(uint32_t* r, const uint32_t* a) {
  uint32_t m[14], a2[14];
#pragma unroll
  for (int j = 0; j < 14; j++) a2[j] = a[j] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      if (2 * j < k) acc += (uint64_t)a2[j] * a[k - j];
      else if (2 * j == k) acc += (uint64_t)a[j] * a[j];
    }
#pragma unroll
    for (int j = lo; j <= hi; j++)
      if (j < k || k >= 14) acc += (uint64_t)m[j] * P29[k - j];
    if (k < 14) {
      m[k] = ((uint32_t)acc * N0_29) & M29;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r[k - 14] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  r[13] = (uint32_t)acc;
}

// ------------------------------------------------------------------ conversions
__device__ __forceinline__ void to29(uint32_t* o, const uint32_t* w) {  // 12 x 32 -> 14 x 29
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t v = w[wi];
    if (wi + 1 < 12) v |= (uint64_t)w[wi + 1] << 32;
    o[i] = (uint32_t)(v >> sh) & M29;
  }
}
__device__ __forceinline__ void from29(uint32_t* w, const uint32_t* o) {  // 14 x 29 -> 12 x 32
#pragma unroll
  for (int i = 0; i < 12; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    w[wi] |= o[i] << sh;
    if (sh > 3 && wi + 1 < 12) w[wi + 1] |= o[i] >> (32 - sh);
  }
}
__device__ __forceinline__ void canon32(uint32_t* x) {  // [0, 2p) -> [0, p)
  uint32_t d[12];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (int64_t)x[i] - P32[i];
    d[i] = (uint32_t)c;
    c >>= 32;
  }
  const bool ge = c == 0;
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = ge ? d[i] : x[i];
}

enum { V_GENERIC, V_ASM, V_ASMNOP, V_R29, V_R29X2, V_R29SQ, V_GENERIC_SQ, NV };
static const char* NAMES[NV] = {"generic", "asm", "asmnop", "r29", "r29x2", "r29sq", "generic_sq"};

template <int V>
__global__ __launch_bounds__(64) void kbench(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x1[12], x2[12], y[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x1[i] = in[(3 * t + 0) * 12 + i];
    x2[i] = in[(3 * t + 1) * 12 + i];
    y[i] = in[(3 * t + 2) * 12 + i];
  }
  if (V == V_GENERIC || V == V_ASM || V == V_ASMNOP || V == V_GENERIC_SQ) {
    uint32_t r2[12], one[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
      r2[i] = R2_32[i];
      one[i] = i == 0;
    }
    mul_generic(x1, x1, r2);
    mul_generic(x2, x2, r2);
    mul_generic(y, y, r2);
    for (int it = 0; it < iters; it++) {
      if (V == V_GENERIC) {
        mul_generic(x1, x1, y);
        mul_generic(x2, x2, y);
      } else if (V == V_GENERIC_SQ) {
        mul_generic(x1, x1, x1);
        mul_generic(x2, x2, x2);
      } else {
        mul_asm<V == V_ASMNOP>(x1, x1, y);
        mul_asm<V == V_ASMNOP>(x2, x2, y);
      }
    }
    mul_generic(x1, x1, one);
    mul_generic(x2, x2, one);
  } else {
    uint32_t a1[14], a2[14], b[14], r2[14], one[14];
    to29(a1, x1);
    to29(a2, x2);
    to29(b, y);
#pragma unroll
    for (int i = 0; i < 14; i++) {
      r2[i] = R2_29[i];
      one[i] = i == 0;
    }
    mul_r29(a1, a1, r2);
    mul_r29(a2, a2, r2);
    mul_r29(b, b, r2);
    for (int it = 0; it < iters; it++) {
      if (V == V_R29) {
        mul_r29(a1, a1, b);
        mul_r29(a2, a2, b);
      } else if (V == V_R29X2) {
        mul_r29x2(a1, a1, b);
        mul_r29x2(a2, a2, b);
      } else {
        sqr_r29(a1, a1);
        sqr_r29(a2, a2);
      }
    }
    mul_r29(a1, a1, one);
    mul_r29(a2, a2, one);
    from29(x1, a1);
    from29(x2, a2);
  }
  canon32(x1);
  canon32(x2);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    out[(2 * t + 0) * 12 + i] = x1[i];
    out[(2 * t + 1) * 12 + i] = x2[i];
  }
}

typedef void (*kfn)(const uint32_t*, uint32_t*, int);

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2048;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d iters %d\n", prop.gcnArchName, cus, iters);
  kfn ks[NV] = {kbench<V_GENERIC>, kbench<V_ASM>, kbench<V_ASMNOP>, kbench<V_R29>,
                kbench<V_R29X2>,   kbench<V_R29SQ>, kbench<V_GENERIC_SQ>};
  // waves per SIMD: 1 (a wave alone, back-to-back issue) and 8
  for (int wps : {1, 2, 8}) {
    const int blocks = cus * 4 * wps;
    const size_t lanes = (size_t)blocks * 64;
    std::vector<uint32_t> hin(lanes * 3 * 12);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& v : hin) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      v = (uint32_t)s;
    }
    for (size_t i = 0; i < lanes * 3; i++) hin[i * 12 + 11] &= 0x0fffffffu;  // < p
    uint32_t *din, *dout;
    CHK(hipMalloc(&din, hin.size() * 4));
    CHK(hipMalloc(&dout, lanes * 2 * 12 * 4));
    CHK(hipMemcpy(din, hin.data(), hin.size() * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> ref(lanes * 24), refsq(lanes * 24), got(lanes * 24);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int v = 0; v < NV; v++) {
      hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(64), 0, 0, din, dout, 4);
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(64), 0, 0, din, dout, iters);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      CHK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
      if (v == V_GENERIC) ref = got;
      if (v == V_GENERIC_SQ) refsq = got;
      size_t bad = 0;
      if (v != V_GENERIC && v != V_GENERIC_SQ) {
        const std::vector<uint32_t>& r = (v == V_R29SQ) ? refsq : ref;
        if (v != V_R29SQ || !refsq.empty())
          for (size_t i = 0; i < lanes * 2; i++) bad += memcmp(&got[i * 12], &r[i * 12], 48) != 0;
      }
      const double muls = 2.0 * lanes * iters;
      // cycles per product per wave on one SIMD at 2.4 GHz nominal: SIMDs * clk * time / (products/64)
      const double cyc = (4.0 * cus) * 2.4e9 * (ms * 1e-3) / (muls / 64.0);
      printf("waves/SIMD %d  %-10s %8.3f ms  %8.3f G Fp-mul/s  %7.0f SIMD-cycles per wave-product  mismatches %zu%s\n",
             wps, NAMES[v], ms, muls / (ms * 1e-3) / 1e9, cyc, bad,
             (v == V_R29SQ && refsq.empty()) ? " (checked below)" : "");
    }
    // r29sq runs before generic_sq in the table; re-check it now
    {
      hipLaunchKernelGGL(ks[V_R29SQ], dim3(blocks), dim3(64), 0, 0, din, dout, iters);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < lanes * 2; i++) bad += memcmp(&got[i * 12], &refsq[i * 12], 48) != 0;
      printf("waves/SIMD %d  r29sq vs generic_sq mismatches %zu\n", wps, bad);
    }
    CHK(hipFree(din));
    CHK(hipFree(dout));
  }
  return 0;
}
