// Shared helpers for the libanr_hip.so kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/anr.h"

namespace anr {

// ---------------------------------------------------------------- error reporting
void set_error(const char* fmt, ...);

#define ANR_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::anr::set_error(__VA_ARGS__);        \
      return ANR_E_INVALID;                 \
    }                                       \
  } while (0)

#define ANR_CHECK_LAUNCH(name)                                                     \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      ::anr::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));      \
      return ANR_E_LAUNCH;                                                         \
    }                                                                              \
  } while (0)

inline hipStream_t as_stream(anr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int kWave = 64;  // CDNA wavefront width

// ---------------------------------------------------------------- dtype helpers
template <typename T>
__device__ __forceinline__ float to_f32(T v);
template <>
__device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }

template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half_rn(v); }

// Load element i of a buffer whose dtype is only known at run time (wave-uniform).
__device__ __forceinline__ float load_dyn(const void* p, int32_t dtype, int64_t i) {
  return dtype == ANR_F32 ? static_cast<const float*>(p)[i]
                          : __half2float(static_cast<const __half*>(p)[i]);
}
__device__ __forceinline__ void store_dyn(void* p, int32_t dtype, int64_t i, float v) {
  if (dtype == ANR_F32)
    static_cast<float*>(p)[i] = v;
  else
    static_cast<__half*>(p)[i] = __float2half_rn(v);
}

// ---------------------------------------------------------------- wave primitives
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Shuffles over the 64-lane wavefront (ds_bpermute based).
__device__ __forceinline__ float shfl(float v, int src) { return __shfl(v, src, kWave); }
__device__ __forceinline__ float shfl_up(float v, int d) { return __shfl_up(v, d, kWave); }
__device__ __forceinline__ float shfl_down(float v, int d) { return __shfl_down(v, d, kWave); }
__device__ __forceinline__ float shfl_xor(float v, int m) { return __shfl_xor(v, m, kWave); }
__device__ __forceinline__ uint32_t shfl_up_u(uint32_t v, int d) {
  return static_cast<uint32_t>(__shfl_up(static_cast<int>(v), d, kWave));
}
__device__ __forceinline__ uint32_t shfl_down_u(uint32_t v, int d) {
  return static_cast<uint32_t>(__shfl_down(static_cast<int>(v), d, kWave));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor(v, m);
  return v;
}

}  // namespace anr
