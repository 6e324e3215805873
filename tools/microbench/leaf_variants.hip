// Product-leaf variants on gfx950: throughput of chains of Montgomery products (14 x 28-bit limbs)
// at 1 / 2 / 4 waves per SIMD, plus the effective shader clock read inside the kernel (clock64 =
// shader cycles, wall_clock64 = the 100 MHz constant counter).  Decides which leaf form the library
// uses (DESIGN.md §4 "the product leaf").
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/leaf_variants.hip -o /tmp/leafv && /tmp/leafv
//
// Variants:
//   mul V0  the library's form up to round 4: the compiler starts each column's multiply-add chain at
//           zero and adds the shifted carry at the end (one v_lshl_add_u64 per column);
//   mul V1  the carry seeds the column's chain (a register barrier after every multiply-add keeps the
//           compiler from reassociating): no 64-bit adds, but back-to-back dependent multiply-adds
//           (the compiler inserts one wait state between them);
//   f2 F0   the Fp2 product as two one-accumulator passes in turn (ec28.h f2l_mul_core up to round 4);
//   f2 F1   both passes in ONE column loop, the two accumulators alternating, barriers as V1: no
//           64-bit adds and no wait states (the other chain's multiply-add sits between dependent ones).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);               \
      return 1;                                                                     \
    }                                                                               \
  } while (0)
#define UNR _Pragma("unroll")

static constexpr __device__ uint32_t P28[14] = {0x0fffaaabu, 0x0fefffffu, 0x03ffffb9u, 0x0fffeb15u, 0x06241eabu,
                                                0x0a0f6b0fu, 0x0f6730d2u, 0x0f38512bu, 0x04774b84u, 0x04bacd76u,
                                                0x0ba7b643u, 0x0e69a4b1u, 0x01ea397fu, 0x0001a011u};
#define N0 0x0ffcfffdu
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));

#define MADD0(acc, x, y) acc += (uint64_t)(x) * (y)
#define MADD1(acc, x, y)              \
  do {                                \
    acc += (uint64_t)(x) * (y);       \
    asm("" : "+v"(acc));              \
  } while (0)

template <int V>
__device__ __forceinline__ void mul_core(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[14];
  uint64_t acc = 0;
  UNR for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    UNR for (int j = lo; j <= hi; j++) {
      if (V == 0) MADD0(acc, a[j], b[k - j]);
      else MADD1(acc, a[j], b[k - j]);
    }
    UNR for (int j = lo; j <= hi; j++) if (j < k || k >= 14) {
      if (V == 0) MADD0(acc, m[j], P28[k - j]);
      else MADD1(acc, m[j], P28[k - j]);
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * N0) & 0x0FFFFFFFu;
      if (V == 0) MADD0(acc, m[k], P28[0]);
      else MADD1(acc, m[k], P28[0]);
    } else {
      r[k - 14] = (uint32_t)acc & 0x0FFFFFFFu;
    }
    acc >>= 28;
  }
  r[13] = (uint32_t)acc;
}

// r = (A B + C D) / R, one accumulator (ec28.h f2l_dot_core up to round 4)
__device__ __forceinline__ void dot_core(uint32_t* r, const uint32_t* A, const uint32_t* B, const uint32_t* C,
                                         const uint32_t* D) {
  uint32_t m[14];
  uint64_t acc = 0;
  UNR for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
    UNR for (int j = lo; j <= hi; j++) {
      MADD0(acc, A[j], B[k - j]);
      MADD0(acc, C[j], D[k - j]);
    }
    UNR for (int j = lo; j <= hi; j++) if (j < k || k >= 14) MADD0(acc, m[j], P28[k - j]);
    if (k < 14) {
      m[k] = ((uint32_t)acc * N0) & 0x0FFFFFFFu;
      MADD0(acc, m[k], P28[0]);
    } else {
      r[k - 14] = (uint32_t)acc & 0x0FFFFFFFu;
    }
    acc >>= 28;
  }
  r[13] = (uint32_t)acc;
}

// x0 y0 + x1 y1 and x0 y1 + x2 y0 (the two coefficients of an Fp2 product with x2 = K - a1 folded
// by the caller): F0 = two passes, F1 = one interleaved pass
template <int V>
__device__ __forceinline__ void dot2_core(uint32_t* r0, uint32_t* r1, const uint32_t* x0, const uint32_t* x1,
                                          const uint32_t* y0, const uint32_t* y1, const uint32_t* z0,
                                          const uint32_t* z1) {
  // r0 = x0 y0 + x1 y1, r1 = x0 z0 + z1 y0 ... generic: r0 = x0*y0 + x1*y1 ; r1 = x0*z0 + z1*y0
  if (V == 0) {
    dot_core(r0, x0, y0, x1, y1);
    dot_core(r1, x0, z0, z1, y0);
  } else {
    uint32_t m0[14], m1[14];
    uint64_t a0 = 0, a1 = 0;
    UNR for (int k = 0; k < 27; k++) {
      const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
      UNR for (int j = lo; j <= hi; j++) {
        MADD1(a0, x0[j], y0[k - j]);
        MADD1(a1, x0[j], z0[k - j]);
        MADD1(a0, x1[j], y1[k - j]);
        MADD1(a1, z1[j], y0[k - j]);
      }
      UNR for (int j = lo; j <= hi; j++) if (j < k || k >= 14) {
        MADD1(a0, m0[j], P28[k - j]);
        MADD1(a1, m1[j], P28[k - j]);
      }
      if (k < 14) {
        m0[k] = ((uint32_t)a0 * N0) & 0x0FFFFFFFu;
        m1[k] = ((uint32_t)a1 * N0) & 0x0FFFFFFFu;
        MADD1(a0, m0[k], P28[0]);
        MADD1(a1, m1[k], P28[0]);
      } else {
        r0[k - 14] = (uint32_t)a0 & 0x0FFFFFFFu;
        r1[k - 14] = (uint32_t)a1 & 0x0FFFFFFFu;
      }
      a0 >>= 28;
      a1 >>= 28;
    }
    r0[13] = (uint32_t)a0;
    r1[13] = (uint32_t)a1;
  }
}

template <int V>
__device__ __noinline__ u32x16 mul_leaf(u32x16 a, u32x16 b) {
  uint32_t x[14], y[14], r[14];
  UNR for (int i = 0; i < 14; i++) {
    x[i] = a[i];
    y[i] = b[i];
  }
  mul_core<V>(r, x, y);
  u32x16 o;
  UNR for (int i = 0; i < 14; i++) o[i] = r[i];
  o[14] = o[15] = 0;
  return o;
}

// Fp2 product (a0 + a1 u)(b0 + b1 u): real = a0 b0 + (K - a1) b1, imag = a0 b1 + a1 b0; the second
// operand is a kernel-wide constant here (the leaf's LDS operand slot is not what is measured)
__constant__ uint32_t KB[2][14];
template <int V>
__device__ __noinline__ u32x32 f2_leaf(u32x32 a) {
  uint32_t x0[14], x1[14], nx1[14], b0[14], b1[14], r0[14], r1[14];
  UNR for (int i = 0; i < 14; i++) {
    x0[i] = a[i];
    x1[i] = a[16 + i];
    nx1[i] = 0x0fffffffu - a[16 + i];
    b0[i] = KB[0][i];
    b1[i] = KB[1][i];
  }
  // r0 = x0 b0 + nx1 b1 ; r1 = x0 b1 + x1 b0
  dot2_core<V>(r0, r1, x0, nx1, b0, b1, b1, x1);
  u32x32 o;
  UNR for (int i = 0; i < 14; i++) {
    o[i] = r0[i];
    o[16 + i] = r1[i];
  }
  o[14] = o[15] = o[30] = o[31] = 0;
  return o;
}

struct Clk {
  unsigned long long c0, c1, w0, w1;
};

template <int V, int OCC>
__global__ __launch_bounds__(64, OCC) void k_mul(uint32_t* io, Clk* clk, int n) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  u32x16 x, y;
  UNR for (int i = 0; i < 16; i++) {
    x[i] = (io[i] + g * 7u + i) & 0x0fffffffu;
    y[i] = (io[16 + i] ^ (g * 13u)) & 0x0fffffffu;
  }
  x[13] &= 0xffffu;
  y[13] &= 0xffffu;
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < n; it++) x = mul_leaf<V>(x, y);
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  uint32_t s = 0;
  UNR for (int i = 0; i < 14; i++) s ^= x[i];
  io[64 + g] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = {c0, c1, w0, w1};
}

template <int V, int OCC>
__global__ __launch_bounds__(64, OCC) void k_f2(uint32_t* io, Clk* clk, int n) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  u32x32 x;
  UNR for (int i = 0; i < 32; i++) x[i] = (io[i & 15] + g * 7u + i) & 0x0fffffffu;
  x[13] &= 0xffffu;
  x[29] &= 0xffffu;
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  for (int it = 0; it < n; it++) x = f2_leaf<V>(x);
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  uint32_t s = 0;
  UNR for (int i = 0; i < 30; i++) s ^= x[i];
  io[64 + g] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = {c0, c1, w0, w1};
}

typedef void (*kfn)(uint32_t*, Clk*, int);

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d nominal clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  uint32_t kb[2][14];
  for (int i = 0; i < 14; i++) {
    kb[0][i] = (0x9e3779b9u * (i + 1)) & 0x0fffffffu;
    kb[1][i] = (0x85ebca6bu * (i + 3)) & 0x0fffffffu;
  }
  kb[0][13] &= 0xffffu;
  kb[1][13] &= 0xffffu;
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(KB), kb, sizeof(kb)));
  struct K {
    const char* name;
    kfn f;
    int occ;
    double fp_per_call;  // Fp-product equivalents per leaf call (Fp2 product = 4 a.b + 2 reductions = 3)
    int madds;           // v_mad_u64_u32 per call
  } ks[] = {
      {"mul V0", k_mul<0, 1>, 1, 1, 392}, {"mul V1", k_mul<1, 1>, 1, 1, 392},
      {"mul V0", k_mul<0, 2>, 2, 1, 392}, {"mul V1", k_mul<1, 2>, 2, 1, 392},
      {"mul V0", k_mul<0, 4>, 4, 1, 392}, {"mul V1", k_mul<1, 4>, 4, 1, 392},
      {"f2  F0", k_f2<0, 1>, 1, 3, 1176}, {"f2  F1", k_f2<1, 1>, 1, 3, 1176},
      {"f2  F0", k_f2<0, 2>, 2, 3, 1176}, {"f2  F1", k_f2<1, 2>, 2, 3, 1176},
  };
  const int n = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t* io;
  Clk* clk;
  const int max_blocks = cus * 4 * 4;
  CHK(hipMalloc(&io, (64 + max_blocks * 64) * 4));
  CHK(hipMemset(io, 0x5a, (64 + max_blocks * 64) * 4));
  CHK(hipMalloc(&clk, max_blocks * sizeof(Clk)));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  std::vector<Clk> h(max_blocks);
  for (auto& k : ks) {
    const int blocks = cus * 4 * k.occ;  // one wave per block, occ waves per SIMD
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, io, clk, n / 10);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, io, clk, n);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(h.data(), clk, blocks * sizeof(Clk), hipMemcpyDeviceToHost));
    double cyc = 0, wall = 0;
    for (int b = 0; b < blocks; b++) {
      cyc += (double)(h[b].c1 - h[b].c0);
      wall += (double)(h[b].w1 - h[b].w0);
    }
    const double ghz = cyc / wall * 0.1;  // wall_clock64 ticks at 100 MHz
    const double calls = (double)blocks * 64 * n;
    const double fp_rate = calls * k.fp_per_call / (ms * 1e-3);
    // issue slots: one wave64 VALU instruction per SIMD per 4 cycles; per call per wave, cycles
    const double cyc_per_call_wave = cyc / blocks / n;
    printf("%s occ %d: %8.3f ms  %7.2f G Fp-products/s  %6.2f T madd/s  clock %.3f GHz  %7.1f cycles per call per wave  (%5.1f per madd)\n",
           k.name, k.occ, ms, fp_rate / 1e9, calls * k.madds / (ms * 1e-3) / 1e12, ghz, cyc_per_call_wave,
           cyc_per_call_wave / k.madds);
  }
  return 0;
}
