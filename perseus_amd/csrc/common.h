// Shared helpers for the perseus_amd HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <string>

#include "../../include/perseus_amd.h"
#include "../../include/perseus_amd_debug.h"

// Timing-only kernel variants (wrong results by construction: MFMAs, DMAs, waits, stores or
// offset arithmetic removed) exist only in a measurement build (PERSEUS_AMD_TIMING_VARIANTS=1 at
// build time, perseus_amd/build.py -> -DPA_TIMING_VARIANTS=1).  The release library has no code
// for them and pa_detector_debug_set_variant rejects their ids (detector.hip timing_only_variant).
#ifndef PA_TIMING_VARIANTS
#define PA_TIMING_VARIANTS 0
#endif

namespace pa {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

void set_error(const char* fmt, ...);

#define PA_HIP(call)                                                               \
  do {                                                                             \
    hipError_t _e = (call);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::pa::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(_e)); \
      return PA_EHIP;                                                              \
    }                                                                              \
  } while (0)

#define PA_CHECK(cond, ...)          \
  do {                               \
    if (!(cond)) {                   \
      ::pa::set_error(__VA_ARGS__);  \
      return PA_EINVAL;              \
    }                                \
  } while (0)

#define PA_LAUNCH_CHECK()                                                              \
  do {                                                                                 \
    hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess) {                                                            \
      ::pa::set_error("%s:%d launch: %s", __FILE__, __LINE__, hipGetErrorString(_e)); \
      return PA_EHIP;                                                                  \
    }                                                                                  \
  } while (0)

// Workgroup barrier that orders LDS only: lgkmcnt(0) + s_barrier.  __syncthreads()
// also waits vmcnt(0), which would drain every global prefetch in flight.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// kornia.geometry.conversions.denormalize_pixel_coordinates in f32, operation for
// operation: factor = 2 / (S - 1); px = (1 / factor) * (n + 1).  (1 / f32(2/255) is
// 127.49999237, not 127.5: the reference's pixels carry that rounding.)
__host__ __device__ __forceinline__ float kornia_denorm(float n, int S) {
  const float factor = 2.0f / (float)(S - 1);
  return (1.0f / factor) * (n + 1.0f);
}

}  // namespace pa
