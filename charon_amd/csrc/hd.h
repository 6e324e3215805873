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
#define HDNI static __host__ __device__ __noinline__
#define HB_CONST static constexpr __device__
#define HB_DEVICE_CODE 1
#else
#define HD static inline
#define HDNI static __attribute__((noinline))
#define HB_CONST static constexpr
#define HB_DEVICE_CODE 0
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HB_UNROLL _Pragma("unroll")
#define HB_NOUNROLL _Pragma("nounroll")
#else
#define HB_UNROLL _Pragma("GCC unroll 16")
#define HB_NOUNROLL
#endif
