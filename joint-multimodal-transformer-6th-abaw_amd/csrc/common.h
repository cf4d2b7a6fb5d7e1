// Shared definitions for the JMT HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/jmt.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace jmt {

// ------------------------------------------------------------------ error plumbing (abi.cpp)
int set_error(int code, const char* fmt, ...);

#define JMT_CHECK_ARG(cond, ...)                                                     \
  do {                                                                               \
    if (!(cond)) return ::jmt::set_error(JMT_ERR_ARG, __VA_ARGS__);                  \
  } while (0)

#define JMT_LAUNCH_CHECK(name)                                                       \
  do {                                                                               \
    hipError_t e_ = hipGetLastError();                                               \
    if (e_ != hipSuccess)                                                            \
      return ::jmt::set_error(JMT_ERR_HIP, "%s: launch failed: %s", name,            \
                              hipGetErrorString(e_));                                \
  } while (0)

// ------------------------------------------------------------------ element conversions
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(_Float16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float x) { return (__bf16)x; }
template <> __device__ __forceinline__ _Float16 from_f<_Float16>(float x) { return (_Float16)x; }

// runtime-dtype scalar load / store (used in epilogues and small kernels)
__device__ __forceinline__ float ld_dyn(const void* p, int64_t i, int dt) {
  if (dt == JMT_F32) return ((const float*)p)[i];
  if (dt == JMT_BF16) return (float)((const __bf16*)p)[i];
  return (float)((const _Float16*)p)[i];
}
__device__ __forceinline__ void st_dyn(void* p, int64_t i, int dt, float v) {
  if (dt == JMT_F32) ((float*)p)[i] = v;
  else if (dt == JMT_BF16) ((__bf16*)p)[i] = (__bf16)v;
  else ((_Float16*)p)[i] = (_Float16)v;
}

__host__ __device__ inline int dtype_size(int dt) { return dt == JMT_F32 ? 4 : 2; }

// ------------------------------------------------------------------ wave / block reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 64*NW; `red` must hold NW floats.  All threads get the sum.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  __syncthreads();
  return s;
}

inline hipStream_t as_stream(void* s) { return (hipStream_t)s; }

}  // namespace jmt
