// Shared pieces of the fused attention kernels (attn.hip: long sequences, attn_short.hip:
// Lq, Lk <= 32), head dim 512: the swizzled K / V / Q / dO row images in LDS and their fragment
// reads, LDS-DMA row staging, lane-group reductions, the register-direct output store.
#pragma once
#include "common.h"

namespace jmt {

constexpr int AT_DH = 512;          // head dim of the fused kernels
constexpr int AT_ROWB = 1024;       // bytes per image row (DH 16-bit values)

// arguments of the long-sequence attention backward (attn.hip attn_bwd_kernel)
struct AttnBwdArgs {
  const void* go;
  const void* o;
  const void* q;
  const void* k;
  const void* v;
  const float* lse;
  void* pbuf;
  void* dsbuf;
  void* dq;
  int64_t sgo_l, sgo_n, so_l, so_n, sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, sdq_l, sdq_n, ldp;
  int Lq, Lk, H, nitems;
  float scale, scale_log2;
};

// byte offset of logical byte b of row `row` in a swizzled image
__device__ __forceinline__ int img_off(int row, int b) {
  return row * AT_ROWB + ((((b >> 4) ^ ((row & 7) << 1))) << 4) + (b & 15);
}
// Per-lane base offsets of the fragment reads (the swizzle XOR touches chunk bits 1-3 only, so
// a read's offset = one of a few lane bases + a compile-time immediate):
//  row_base(m): ds_read_b128 fragment of row li (+16 kt), chunk 4 (4 a + m) + g of half h
//               -> row_base(m) + 256 a + 16384 kt
//  tr_base(c):  ds_read_b64_tr_b16 block rows 4 g + (li >> 2) (+16, +32 u), columns
//               16 (8 b + c) + 4 (li & 3) of half h -> tr_base(c) + 256 b + 16384 hi + 32768 u
__device__ __forceinline__ int row_base(int m, int li, int g, int h) {
  return li * AT_ROWB + ((((4 * m + g) ^ ((li & 7) << 1))) << 4) + 512 * h;
}
__device__ __forceinline__ int tr_base(int c, int li, int g, int h) {
  const int r = 4 * g + (li >> 2);
  return r * AT_ROWB + ((((2 * c + ((li & 3) >> 1)) ^ ((r & 7) << 1))) << 4) + 8 * (li & 1) +
         512 * h;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// stage R key rows k0.. (row r <- source row min(k0 + r, Lk - 1)) by LDS-DMA, R / 8 per wave.
// Row addresses are wave-uniform (scalar arithmetic, saddr + 32-bit lane offset); the lane's
// 16-B chunk is the swizzle of the image: LDS chunk `lane` of row r holds source chunk
// lane ^ ((r & 7) << 1).
// ASM: the DMA from inline asm (common.h glds16_asm, invisible to hipcc's wait bookkeeping).
// The forward takes it: hipcc otherwise drains the next K tile before the P V phase's
// transposed V reads (-4 % at L = 300, -9 % at L = 1024); the backward keeps the builtin: its
// register loads of Q / dO are waited for by hipcc's own counts, which the hidden DMA would make
// short (+5 %; profiles/r04/attn_glds_ab.txt).
template <typename T, int R, int NW = 8, bool ASM = false>
__device__ __forceinline__ void stage_rows(char* img, const T* base, int64_t ld, int k0, int Lk) {
  constexpr int NI = R / NW;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = wu * NI + i;
    const int src = min(k0 + r, Lk - 1);
    JMT_DCHECK(src >= 0 && src < Lk);
    const char* row = (const char*)(base + (int64_t)src * ld);
    const unsigned off = (unsigned)(lane ^ ((r & 7) << 1)) << 4;
    if constexpr (ASM) glds16_asm(row + off, img + r * AT_ROWB);
    else glds16(row + off, img + r * AT_ROWB);
  }
}

// pieces [i0, i1) of stage_rows (the NI = R / NW wave-instructions of this wave), so the DMA of a
// tile can be issued between the MFMA batches of a phase instead of in one burst
template <typename T, int R, int NW = 8, bool ASM = false>
__device__ __forceinline__ void stage_rows_part(char* img, const T* base, int64_t ld, int k0,
                                                int Lk, int i0, int i1) {
  constexpr int NI = R / NW;
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (i < i0 || i >= i1) continue;
    const int r = wu * NI + i;
    const int src = min(k0 + r, Lk - 1);
    JMT_DCHECK(src >= 0 && src < Lk);
    const char* row = (const char*)(base + (int64_t)src * ld);
    const unsigned off = (unsigned)(lane ^ ((r & 7) << 1)) << 4;
    if constexpr (ASM) glds16_asm(row + off, img + r * AT_ROWB);
    else glds16(row + off, img + r * AT_ROWB);
  }
}

// Reductions over the 4 lane groups g = lane >> 4 (lanes l, l ^ 16, l ^ 32, l ^ 48) with
// v_permlane16_swap / v_permlane32_swap (VALU, no LDS round trip as ds_bpermute has).  After a
// swap of (x, x) the pair holds (x of the even row, x of the odd row) in EVERY lane, so a sum is
// formed in one order on both partners (bitwise equal, as the shuffle form's commutative add).
__device__ __forceinline__ float pl_pair_max(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float pl_pair_sum(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// XCD-aware bijective remap of the block index (blocks % 8 share an XCD)
__device__ __forceinline__ int xcd_block() {
  const int nwg = gridDim.x;
  int wg = blockIdx.x;
  if (nwg >= 16) {
    const int qd = nwg / 8, rm = nwg % 8, x = blockIdx.x % 8;
    wg = (x < rm ? x * (qd + 1) : rm * (qd + 1) + (x - rm) * qd) + blockIdx.x / 8;
  }
  return wg;
}

// Persistent work distribution over `nitems` (n, h, q-tile) items, item = (n H + h) nqt + qt.
// A grid of one block per CU (a multiple of 8) deals the items to the 8 XCDs in contiguous
// ranges; block b (XCD b % 8, slot b / 8) takes items lo + slot, lo + slot + G/8, ...  so at any
// moment an XCD's blocks work on consecutive items and the q-tiles of one (n, h) share its K / V
// through that XCD's L2.  A grid of one block per item keeps the xcd_block() order.
__device__ __forceinline__ void item_range(int nitems, int& first, int& end, int& stride) {
  const int G = gridDim.x;
  if (G < nitems && G % 8 == 0) {
    const int x = blockIdx.x % 8, S8 = G / 8;
    first = (int)((int64_t)nitems * x / 8) + blockIdx.x / 8;
    end = (int)((int64_t)nitems * (x + 1) / 8);
    stride = S8;
  } else {
    first = G < nitems ? blockIdx.x : xcd_block();
    end = nitems;
    stride = G;
  }
}

// Store this wave's 16 x 256 accumulator half (lane: row li, dims 16 t + 4 g + r of `out`'s
// half, multiplied by `mul`) straight from registers: the accumulators of sub-tiles t, t+1 are
// paired with v_permlane16_swap so a lane holds 8 consecutive dims -> one 16-B store per lane and
// pair (as gemm.hip's epilogue).  No LDS, no barrier: the next item's tiles may already be landing.
template <typename T>
__device__ __forceinline__ void store_acc_direct(const f32x4* acc, float mul, T* orow, bool valid) {
  const int g = (threadIdx.x & 63) >> 4;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int jp = 0; jp < 8; ++jp) {
    uint32_t pk[2][2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        T two[2] = {from_f<T>(acc[2 * jp + hh][2 * q] * mul),
                    from_f<T>(acc[2 * jp + hh][2 * q + 1] * mul)};
        pk[hh][q] = *(const uint32_t*)two;
      }
    const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
    const int c = 16 * (2 * jp + (g & 1)) + 8 * (g >> 1);
    const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
    if (valid) __builtin_nontemporal_store(v, (u32x4*)(orow + c));
  }
}

}  // namespace jmt
