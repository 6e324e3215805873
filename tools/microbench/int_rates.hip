// Per-instruction VALU throughput on gfx950 for the ops a 381-bit Montgomery product is built
// from: the roofline peak of bench.py (charon_amd/opcounts.py PEAK_MAD_TOPS) comes from here.
//
// Every timed kernel is a loop of ITERS x UNROLL copies of ONE instruction (inline asm, 8
// independent accumulators so no copy waits on the previous one) and nothing else in the loop
// but the loop's scalar counter.  The run prints, per kernel and occupancy:
//   * lane-ops/s from HIP events (copies x lanes / kernel time),
//   * the effective shader clock inside the kernel (clock64 = shader cycles, wall_clock64 = the
//     100 MHz constant counter, summed over every wave),
//   * lane-ops per clock per CU at that clock and at the nominal 2.4 GHz,
//   * the VALU instructions each wave is expected to issue (for the PMC cross-check:
//     tools/microbench/int_rates_pmc.py joins rocprofv3 --pmc SQ_INSTS_VALU / SQ_WAVES /
//     GRBM_GUI_ACTIVE with these lines).
// Instructions above 64 lane-ops/clk/CU at the effective clock issue faster than one wave64 VALU
// instruction per SIMD per 4 cycles (dual-issue of simple 32-bit ops); the multiply-adds do not.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/int_rates.hip -o tools/microbench/int_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                 \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

constexpr int ITERS = 16384;  // ~2 ms kernels: launch overhead below 1 % of the event-timed rate
constexpr int UNROLL = 16;  // copies per loop trip (2 x the 8 accumulators)

struct Clk {
  unsigned long long c0, c1, w0, w1;
};

#define BODY8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define CLOCK_BEGIN const unsigned long long c0 = clock64(), w0 = wall_clock64();
#define CLOCK_END                                                     \
  const unsigned long long c1 = clock64(), w1 = wall_clock64();       \
  if (threadIdx.x == 0) clk[blockIdx.x] = {c0, c1, w0, w1};

__global__ void k_mad64(uint32_t* out, Clk* clk, uint32_t seed) {
  uint64_t acc[8];
  uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  CLOCK_BEGIN
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
      BODY8(M)
#undef M
    }
  }
  CLOCK_END
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

#define SIMPLE_KERNEL(NAME, INSTR)                                                        \
  __global__ void NAME(uint32_t* out, Clk* clk, uint32_t seed) {                          \
    uint32_t acc[8];                                                                      \
    uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;                                    \
    for (int i = 0; i < 8; i++) acc[i] = a + i;                                           \
    CLOCK_BEGIN                                                                           \
    for (int it = 0; it < ITERS; it++) {                                                  \
      _Pragma("unroll") for (int u = 0; u < UNROLL / 8; u++) {                            \
        _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(INSTR : "+v"(acc[i]) : "v"(a), "v"(b)); \
      }                                                                                   \
    }                                                                                     \
    CLOCK_END                                                                             \
    uint32_t s = 0;                                                                       \
    for (int i = 0; i < 8; i++) s += acc[i];                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
  }

SIMPLE_KERNEL(k_mullo, "v_mul_lo_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mulhi, "v_mul_hi_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add, "v_add_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add3, "v_add3_u32 %0, %1, %2, %0")
SIMPLE_KERNEL(k_and, "v_and_b32 %0, %1, %0")
SIMPLE_KERNEL(k_mad24, "v_mad_u32_u24 %0, %1, %2, %0")

__global__ void k_lshr64(uint32_t* out, Clk* clk, uint32_t seed) {
  uint64_t acc[8];
  for (int i = 0; i < 8; i++) acc[i] = (uint64_t)(threadIdx.x ^ seed) << 20 | i;
  CLOCK_BEGIN
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc[i]));
      BODY8(M)
#undef M
    }
  }
  CLOCK_END
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_lshladd64(uint32_t* out, Clk* clk, uint32_t seed) {
  uint64_t acc[8];
  uint64_t a = threadIdx.x ^ seed;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  CLOCK_BEGIN
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
      BODY8(M)
#undef M
    }
  }
  CLOCK_END
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_fma64(uint32_t* out, Clk* clk, uint32_t seed) {
  double acc[8];
  double a = 1.0000001 * (threadIdx.x + seed), b = 0.999999;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  CLOCK_BEGIN
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
      BODY8(M)
#undef M
    }
  }
  CLOCK_END
  double s = 0;
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

typedef void (*kfn)(uint32_t*, Clk*, uint32_t);

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const double nominal_hz = prop.clockRate * 1e3;
  printf("device %s CUs %d nominal clock %.0f MHz; %d x %d copies per wave per launch\n", prop.gcnArchName, cus,
         nominal_hz / 1e6, ITERS, UNROLL);
  struct {
    const char* name;
    kfn f;
  } ks[] = {{"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
            {"v_add_u32", k_add},       {"v_add3_u32", k_add3},     {"v_and_b32", k_and},
            {"v_mad_u32_u24", k_mad24}, {"v_lshrrev_b64", k_lshr64}, {"v_lshl_add_u64", k_lshladd64},
            {"v_fma_f64", k_fma64}};
  const int block = 64;  // one wave per workgroup: waves per CU = grid / CUs
  for (int wpc : {8, 16}) {
    const int grid = cus * wpc;
    uint32_t* out;
    Clk* clk;
    CHK(hipMalloc(&out, (size_t)grid * block * 4));
    CHK(hipMalloc(&clk, (size_t)grid * sizeof(Clk)));
    std::vector<Clk> h(grid);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, clk, 7u);  // warm
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, clk, 11u);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      CHK(hipMemcpy(h.data(), clk, grid * sizeof(Clk), hipMemcpyDeviceToHost));
      double cyc = 0, wall = 0;
      for (int b = 0; b < grid; b++) {
        cyc += (double)(h[b].c1 - h[b].c0);
        wall += (double)(h[b].w1 - h[b].w0);
      }
      const double eff_hz = cyc / wall * 1e8;
      const double copies = (double)ITERS * UNROLL;
      const double lane_ops = copies * grid * block;
      const double rate = lane_ops / (ms * 1e-3);
      printf("waves/CU %2d  %-15s %8.3f T lane-ops/s  %7.3f ms  eff clock %6.0f MHz  %6.1f lane-ops/clk/CU (eff)  "
             "%6.1f (nominal)  expected VALU per wave %.0f\n",
             wpc, k.name, rate / 1e12, ms, eff_hz / 1e6, rate / (cus * eff_hz), rate / (cus * nominal_hz), copies);
    }
    CHK(hipFree(out));
    CHK(hipFree(clk));
  }
  return 0;
}
