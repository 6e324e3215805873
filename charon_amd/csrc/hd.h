// Host/device portability macros for the BLS12-381 arithmetic headers.
//
// The arithmetic headers are compiled two ways:
//   * by hipcc for gfx950 inside libhipbls.so (the product: every hot-path call runs as a
//     HIP kernel on the MI355X), and
//   * by g++ into tests/native/libhbls_hostcheck.so, a TEST-ONLY harness that runs the same
//     per-item functions on the CPU so arithmetic bugs are caught before GPU time.  The
//     product never loads that harness.
#pragma once
#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HD static __host__ __device__ __forceinline__
#if defined(HB_FAST_FPMUL)
// fast units: everything but the Fp product / square (fp.h leaves) is inlined
#define HDNI static __host__ __device__ __forceinline__
#else
#define HDNI static __host__ __device__ __noinline__
#endif
#define HB_CONST static constexpr __device__
#define HB_DEVICE_CODE 1
#else
#define HD static inline
#define HDNI static __attribute__((noinline))
#define HB_CONST static constexpr
#define HB_DEVICE_CODE 0
#endif

// Op counting (test harness only: the g++ build of tests/native/hostcheck.cpp defines
// HB_COUNT_OPS to freeze the algorithmic work per item).  Compiles to nothing
// in the product library.
#if defined(HB_COUNT_OPS) && !defined(__HIPCC__)
namespace hb {
extern thread_local unsigned long long g_cnt_fp_mul, g_cnt_fr_mul;
}
#define HB_COUNT_FP_MUL() (++hb::g_cnt_fp_mul)
#define HB_COUNT_FR_MUL() (++hb::g_cnt_fr_mul)
#else
#define HB_COUNT_FP_MUL() ((void)0)
#define HB_COUNT_FR_MUL() ((void)0)
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HB_UNROLL _Pragma("unroll")
#define HB_NOUNROLL _Pragma("nounroll")
#else
#define HB_UNROLL _Pragma("GCC unroll 16")
#define HB_NOUNROLL
#endif
