// Measures per-instruction VALU throughput on gfx950 for the ops a 381-bit Montgomery
// multiply is built from.  Used to fix the roofline "peak" for bench.py.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int UNROLL = 16;

#define BODY8(ASM)  ASM(0) ASM(1) ASM(2) ASM(3) ASM(4) ASM(5) ASM(6) ASM(7)

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t acc[8]; uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
      BODY8(M)
#undef M
    }
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

#define SIMPLE_KERNEL(NAME, INSTR)                                                              \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                          \
    uint32_t acc[8]; uint32_t a = threadIdx.x ^ seed, b = seed * 3 + 1;                         \
    for (int i = 0; i < 8; i++) acc[i] = a + i;                                                 \
    for (int it = 0; it < ITERS; it++) {                                                        \
      _Pragma("unroll") for (int u = 0; u < UNROLL / 8; u++) {                                  \
        _Pragma("unroll") for (int i = 0; i < 8; i++)                                           \
          asm volatile(INSTR : "+v"(acc[i]) : "v"(a), "v"(b));                                 \
      }                                                                                         \
    }                                                                                           \
    uint32_t s = 0; for (int i = 0; i < 8; i++) s += acc[i];                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                             \
  }

SIMPLE_KERNEL(k_mullo, "v_mul_lo_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mulhi, "v_mul_hi_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add, "v_add_u32 %0, %1, %0")
SIMPLE_KERNEL(k_addco, "v_add_co_u32 %0, vcc, %1, %0")
SIMPLE_KERNEL(k_addc, "v_addc_co_u32 %0, vcc, %1, %0, vcc")
SIMPLE_KERNEL(k_add3, "v_add3_u32 %0, %1, %2, %0")
SIMPLE_KERNEL(k_mad24, "v_mad_u32_u24 %0, %1, %2, %0")
SIMPLE_KERNEL(k_mulhi24, "v_mul_hi_u32_u24 %0, %1, %0")
SIMPLE_KERNEL(k_cndmask, "v_cndmask_b32 %0, %1, %0, vcc")

__global__ void k_lshladd64(uint32_t* out, uint32_t seed) {
  uint64_t acc[8]; uint64_t a = threadIdx.x ^ seed;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
      BODY8(M)
#undef M
    }
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double acc[8]; double a = 1.0000001 * (threadIdx.x + seed), b = 0.999999;
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL / 8; u++) {
#define M(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
      BODY8(M)
#undef M
    }
  }
  double s = 0; for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_add_u32", k_add}, {"v_add_co_u32", k_addco}, {"v_addc_co_u32", k_addc},
    {"v_add3_u32", k_add3}, {"v_mad_u32_u24", k_mad24}, {"v_mul_hi_u32_u24", k_mulhi24},
    {"v_cndmask_b32", k_cndmask}, {"v_lshl_add_u64", k_lshladd64}, {"v_fma_f64", k_fma64}};
  const int block = 256;
  for (int wpc : {8, 16}) {
    int grid = cus * wpc / 4;  // wpc waves per CU
    uint32_t* out; CHK(hipMalloc(&out, (size_t)grid * block * 4));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 7u);  // warm
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      const int reps = 5;
      for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 7u + r);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double ops = (double)reps * grid * block * ITERS * UNROLL;  // lane-ops
      double rate = ops / (ms * 1e-3);
      // lane-ops per clock per CU at nominal clock
      double per_clk_cu = rate / (cus * (prop.clockRate * 1e3));
      printf("waves/CU %2d  %-18s %9.3f Tops/s (lane-ops)  %6.1f lane-ops/clk/CU @nominal\n", wpc, k.name, rate / 1e12, per_clk_cu);
    }
    CHK(hipFree(out));
  }
  return 0;
}
