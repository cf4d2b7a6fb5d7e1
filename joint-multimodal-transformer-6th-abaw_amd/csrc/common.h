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
typedef float f32x16 __attribute__((ext_vector_type(16)));

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

// ------------------------------------------------------------------ bounds-check build
// `make bounds` compiles the kernels with -DJMT_BOUNDS=1: JMT_DCHECK(cond) at the kernels' global
// index computations counts every failed check in a per-translation-unit device counter (a
// vector atomic — never a trap, so a bad index is reported, not turned into a GPU fault) that
// jmt_bounds_violations() (abi.cpp) sums over the library.  The default build compiles it out.
int register_bounds_counter(unsigned (*read)(bool reset));
#if defined(JMT_BOUNDS) && JMT_BOUNDS
static __device__ unsigned g_jmt_bounds_hits;
#define JMT_DCHECK(cond)                                                             \
  do {                                                                               \
    if (!(cond)) atomicAdd(&g_jmt_bounds_hits, 1u);                                  \
  } while (0)
static unsigned jmt_read_bounds_hits(bool reset) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_jmt_bounds_hits), sizeof(v)) != hipSuccess) return 0;
  if (reset) {
    const unsigned z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_jmt_bounds_hits), &z, sizeof(z));
  }
  return v;
}
static const int g_jmt_bounds_reg = register_bounds_counter(&jmt_read_bounds_hits);
#else
#define JMT_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

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

// ------------------------------------------------------------------ MFMA fragments (gfx950)
// 16-bit operand fragment of v_mfma_f32_16x16x32_{bf16,f16}: lane l holds row (l&15),
// k = 8*(l>>4) + j, j = 0..7.  C/D: lane l holds row 4*(l>>4) + r, column l&15.
template <typename T> struct Frag16;
template <> struct Frag16<__bf16> { typedef bf16x8 t; typedef bf16x4 h; };
template <> struct Frag16<_Float16> { typedef f16x8 t; typedef f16x4 h; };

typedef short i16x4 __attribute__((ext_vector_type(4)));
// ds_read_b64_tr_b16: the 16 lanes of a group that address k rows kb..kb+3 (lane i -> row
// kb + (i>>2), columns 4*(i&3)..+3) receive, per lane, column (i) of those 4 rows.
template <typename H>
__device__ __forceinline__ H tr_read(const char* p) {
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(i16x4, p));
  return __builtin_bit_cast(H, v);
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// v_mfma_f32_32x32x16_{bf16,f16}: A lane l holds row (l & 31), k = 8 (l >> 5) + j; B k = 8 (l >> 5)
// + j, column (l & 31); C/D lane l holds column (l & 31), rows (r & 3) + 8 (r >> 2) + 4 (l >> 5).
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// One LDS-DMA wave-instruction (global_load_lds_dwordx4: 16 B per lane from `src` to the
// wave-uniform LDS address `lds_dst` + 16 * lane), issued from inline asm so that the compiler
// does not track it: hipcc (ROCm 7.2) treats every pending LDS-DMA as a possible writer of any
// ds_read_b64_tr_b16 it schedules and puts an s_waitcnt vmcnt(0) in front of the first transposed
// read after it — draining the prefetch (the next K-tile in the GEMMs, the next K tile under the
// P V phase of the attention forward; visible in their .s).  Every kernel that stages through
// this waits for its DMA explicitly (vmcnt, then a barrier before the reads), and M0 is written
// and restored inside the statement (cdna_hip_programming.md §5.7).  The ASan build compiles
// device code at -O0, where the "s" operand cannot be proven uniform; its kernels are never
// launched, so it takes the builtin.
__device__ __forceinline__ void glds16_asm(const void* src, const void* lds_dst) {
#if !defined(__OPTIMIZE__)
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
#else
  const uint32_t a = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(a)
      : "memory");
#endif
}

// glds16_asm with the destination as a wave-uniform 32-bit LDS address (no generic->LDS cast:
// that cast costs a null check and a readfirstlane per instruction when the pointer is computed)
__device__ __forceinline__ void glds16_at(const void* src, uint32_t lds_addr) {
#if !defined(__OPTIMIZE__)
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(uintptr_t)lds_addr,
                                   16, 0, 0);
#else
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_addr)
      : "memory");
#endif
}

// The same instruction from the builtin: hipcc counts it in its own s_waitcnt bookkeeping (and
// drains it before transposed LDS reads, above).  The attention kernels load their row operands
// (Q, dO) into registers with plain loads that hipcc waits for by counting the VMEM operations
// issued after them; with the DMA hidden those counts come out short and every such wait
// over-waits for the DMA in flight (attention backward +10 %, scripts/bench_attn.py), so they
// keep the builtin.
__device__ __forceinline__ void glds16(const void* src, const void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

}  // namespace jmt
