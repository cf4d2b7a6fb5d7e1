// Shared device code of the LDS-tiled MFMA GEMM (gemm.hip: one block per tile, split-K;
// gemm_persist.hip: persistent tile walk).  See gemm.hip for the design.
#pragma once
#include <cstdlib>

#include "common.h"

namespace jmt {

constexpr int MAXP = 8;

struct GemmParams {
  const void* a_ptr[MAXP];
  const void* b_ptr[MAXP];
  void* c_ptr[MAXP];
  const float* bias;
  const float* bias_tab[MAXP];  // per-b0 bias vectors (n_bias > 0)
  int n_bias;
  const void* aux;
  float* ws;
  int64_t lda, ldb, ldc, ldaux;
  int64_t sA0, sA1, sB0, sB1, sC0, sC1;
  int a_mode, b_mode, c_mode;   // 0 strided, 1 pointer per b0, 2 K-concat, 3 K-concat per b0
                                // (a/b only; mode 3: sA0 / sB0 hold the segments per b0)
  int a_kseg, b_kseg;           // K-concat segment length (multiple of the K-tile)
  int M, N, K;
  int batch0, batch1;
  int splits, k_per_split;
  float alpha, beta;
  int bias_mode;                // 0 none, 1 per column n, 2 per row m
  int relu;
  int c_dtype;
  int aux_dtype;
  int tiles_m, tiles_n;
  int c_vec4;                   // C (and aux) 4-element groups aligned for 4-element stores
  int c_vec8;                   // C rows / base 16-B aligned (16-bit C: paired 16-B stores)
  int dbg;                      // development ablations: 1 skip MFMA, 2 skip epilogue, 8 trace,
                                //   16 split-K work dealt per (batch, split) as without splits
  // row sums of A (the bias gradient of a weight-gradient GEMM dW = dY^T X: db = sum_k A[m][k]):
  // dbias_tab[b0][m] (+)= ..., per-split fp32 partials in dbias_ws when split
  float* dbias_tab[MAXP];
  float* dbias_ws;
  int n_dbias, dbias_acc;
};

// PF: A-fragment prefetch distance in MFMA rows; PRIO: s_setprio(1) around each MFMA row;
// SGB: sched_group_barrier pinning of each row's LDS reads ahead of its MFMAs.
// OCC: minimum resident blocks per CU requested from the compiler (0: 2 x 256 threads' worth).
// IL: the LDS-DMA of K-tile kt+S-1 is issued in pieces BETWEEN the MFMA rows of tile kt (per-lane
// source offsets precomputed once per block, the K advance in scalar registers), instead of all
// at once before the MFMAs: its issue overlaps the MFMA pipe (requires S >= 3).
template <int BM_, int BN_, int WM_, int WN_, int KB_, int S_, int PF_ = 1, int PRIO_ = 0,
          int SGB_ = 0, int OCC_ = 0, int IL_ = 0>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, KB = KB_, S = S_;
  static constexpr int PF = PF_, PRIO = PRIO_, SGB = SGB_, IL = IL_;
  static constexpr int OCC = OCC_ > 0 ? OCC_ : (2 * 256 / (64 * WM_ * WN_) > 0 ? 2 * 256 / (64 * WM_ * WN_) : 1);
  static constexpr int NT = 64 * WM * WN;          // threads per block
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 16, TN = WTN / 16;
  static constexpr int STAGE = (BM + BN) * KB;     // LDS bytes per stage (A image + B image)
  static constexpr int EPI = 64 * (BN + 4) * 4;     // epilogue staging of one 64-row pass
  static constexpr int LDS = S * STAGE > EPI ? S * STAGE : EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
};
using Cfg1 = TileCfg<128, 128, 2, 2, 128, 2>;
// s_setprio(1) around each MFMA row: 2-4% faster on every step shape than the same tile without
// it; a 2-row A prefetch with sched_group_barrier pinning gained nothing on top
// (profiles/r01_gemm_sched.txt); on the 128x128 tile setprio measured +-2% (kept without)
using Cfg5 = TileCfg<256, 256, 2, 4, 128, 2, 1, 1, 0>;
// 128x128 tiles with 64-B K-tiles at 4 resident blocks / CU (2 stages) or 3 (3 stages), so one
// block's epilogue and loads overlap the others' MFMAs; chosen by occupancy_override()
using Cfg10 = TileCfg<128, 128, 2, 2, 64, 2, 1, 1, 0, 4>;
using Cfg11 = TileCfg<128, 128, 2, 2, 64, 3, 1, 1, 0, 3>;
// 256x256, 64-B K-tiles, 4 stages (3 tiles in flight), DMA issue interleaved with the MFMAs
using Cfg20 = TileCfg<256, 256, 2, 4, 64, 4, 1, 1, 0, 0, 1>;
// 128x128, 64-B K-tiles, 4 stages, interleaved issue, 2 blocks / CU
using Cfg21 = TileCfg<128, 128, 2, 2, 64, 4, 1, 1, 0, 2, 1>;
// 160x256 (8 waves of 80x64): the M = B*T = 19,200-row problems are 120 row tiles, so a
// 512-wide output is 240 tiles — 0.94 of one wave on 256 CUs where the 256x256 tile leaves 150
// (0.59 of a wave, 41 % of the CUs idle) and batched launches quantise to 94 % instead of 88 %.
// K-major A only (the MN-major image swizzle needs a power-of-two row count); the 20 A
// instructions of a K-tile are dealt round-robin over the 8 waves (glds_tile, dma_count);
// 128-B K-tiles in 3 stages (two K-steps in flight, 156 KiB; uneven DMA dealing, per-wave
// waits).  (2 stages, round 3's form, and 64-B K-tiles in 4 stages measured 1 % / 12-17 % slower:
// profiles/r04/gemm_tile160_stages.txt.)
using Cfg32 = TileCfg<160, 256, 2, 4, 128, 3, 1, 1, 0>;
// (256x256 over 4 waves — 2x2, 128x128 each, 256 accumulators per lane in AGPRs, 64-B K-tiles,
// 4 stages, one block / CU: the macro tile hipBLASLt picks on these shapes, profiles/
// r02_hipblaslt_reference.txt — compiled without spills but measured 1.45-1.65x slower than
// Cfg5 / Cfg20 on every step shape, with and without interleaved DMA issue: one wave per SIMD
// leaves each wave's LDS-read latency exposed; profiles/r02_gemm_4wave_256.txt)
// (4-wave 256x128 / 128x256 tiles — a wave 128x64 / 64x128, 64-B K-tiles, 3 stages, 2 blocks /
// CU so one block's epilogue burst overlaps the other's K loop — measured 0-30 % slower than the
// chosen configs on every step shape: profiles/r02_gemm_4wave_rect.jsonl)
// (64x64 tiles — 4 waves of 32x32, 128-B K-tiles, 8 stages: a whole K = 512 reduction in flight —
// for the few-tile T=16 real-data launches measured 0-10 % slower than the 128x128 tile there, and
// up to 2x slower on larger launches: those launches sit on a ~15 us floor of launch, first-load
// and store-drain latency, not on per-K-tile latency; profiles/r02_gemm_small_tiles_realdata.jsonl)
// (without s_setprio the two measured the same: profiles/r01_gemm_occupancy.txt)
// (an epilogue that issues the beta*C / ReLU-mask loads of ALL its rows before the first store, to
// overlap their latencies: 8 B x TM x TN more live registers per lane — 62-133 VGPRs spilled on
// the 256x256 and 128x128/64-B tiles and 3 -> 2 blocks/CU on the others (hipcc
// -Rpass-analysis=kernel-resource-usage), so it was not run)
// (8-wave 128x256 / 256x128 tiles with 64-B K-tiles, 3 stages, 2 blocks / CU measured 20-100%
// slower on every step shape: profiles/r01_gemm_occupancy.txt)
// (deeper pipelines — 256x256 KB=64 with 3-4 stages, 128x128 with 3-4 stages — measured 0-40%
// slower on every JMT shape: profiles/r01_gemm_pipeline_depth.txt)

template <typename T> struct Vec { static constexpr int n = 16 / sizeof(T); };

// ------------------------------------------------------------------ operand addressing
template <typename T>
__device__ __forceinline__ const T* operand_base(const void* const* ptrs, int mode, int64_t s0,
                                                 int64_t s1, int b0, int b1, int kseg, int k0,
                                                 int& kloc) {
  if (mode >= 2) {               // K-concat: segment k0 / kseg (mode 3: of batch entry b0,
    const int seg = k0 / kseg;   // s0 segments per entry)
    kloc = k0 - seg * kseg;
    return (const T*)ptrs[mode == 3 ? b0 * (int)s0 + seg : seg];
  }
  kloc = k0;
  const T* p = (const T*)ptrs[mode == 1 ? b0 : 0];
  return p + (mode == 1 ? 0 : (int64_t)b0 * s0) + (int64_t)b1 * s1;
}

// Swizzles.  K-major image: ROWS rows of KB bytes; MN-major image: KB/sizeof(T) k-rows of
// RB = ROWS*sizeof(T) bytes.
// 64-B rows: a fragment read puts lane l on row l & 15, chunk l >> 4, and ds_read_b128 serves
// the lanes in the groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): the 16 (row % 4,
// chunk) pairs of a group must be distinct, i.e. s(q) for q = row >> 2 with {s0, s3, s1^1,
// s2^1} and {s1, s2, s0^1, s3^1} both permutations of 0..3: s = (0, 2, 3, 1).  (s(q) = q put
// q = 0 and q = 1 of every group on one bank quad: 40 % of the LDS cycles of the 64-B-row
// configs were bank conflicts, profiles/r04/pmc_gemm_vs_hipblaslt.txt.)  128-B rows: every
// group is conflict-free with (row >> 1) & 7.
template <int KB>
__device__ __forceinline__ int swz_k(int row) {
  if constexpr (KB == 128) return (row >> 1) & 7;
  else return (0x78 >> (2 * ((row >> 2) & 3))) & 3;
}
// (an MN-major k-row of RB bytes holds RB/32 pairs of 16-B chunks: the XOR stays inside it)
template <int RB>
__device__ __forceinline__ int swz_t(int k) {
  if constexpr (RB >= 256) return (k & 3) | (((k >> 3) & 1) << 2);
  else return (k & 3) & (RB / 32 - 1);
}

// Physical 16-B chunk `id` (image byte id*16) -> its logical source element (row index in the
// M/N dimension, k index) of one K-tile.  Shared by the LDS-DMA and the register paths, whose LDS
// writes are therefore both linear.
template <typename T, bool KMAJ, int KB, int ROWS>
__device__ __forceinline__ void chunk_src(int id, int& row, int& kk) {
  constexpr int V = Vec<T>::n;
  if constexpr (KMAJ) {
    constexpr int CPR = KB / 16;
    row = id / CPR;
    const int cp = id % CPR;
    kk = (cp ^ swz_k<KB>(row)) * V;
  } else {
    constexpr int CPR = ROWS * (int)sizeof(T) / 16;
    kk = id / CPR;
    const int cp = id % CPR;
    const int c = (sizeof(T) == 2) ? ((((cp >> 1) ^ swz_t<ROWS * (int)sizeof(T)>(kk)) << 1) | (cp & 1))
                                   : cp;
    row = c * V;
  }
}

// One LDS-DMA wave-instruction from inline asm (common.h glds16: why hipcc must not see it).
__device__ __forceinline__ void glds_asm(const void* src, const char* lds) { glds16_asm(src, lds); }

// LDS-DMA staging of one FULL K-tile of one operand (ROWS*KB bytes = ROWS*KB/1024 wave
// instructions spread over the block's waves).  Rows past the matrix edge are clamped to a valid
// row: their products only reach discarded outputs.
template <typename T, bool KMAJ, int KB, int ROWS, int NT>
__device__ __forceinline__ void glds_tile(char* img, const T* base, int64_t ld, int rows_lim,
                                          int r0, int kloc) {
  constexpr int V = Vec<T>::n;
  constexpr int NW = NT / 64;
  constexpr int TOT = ROWS * KB / 1024;    // wave-instructions (1 KiB each) of the image
  constexpr bool EVEN = TOT % NW == 0;
  constexpr int NI = (TOT + NW - 1) / NW;
  static_assert(TOT >= NW || !EVEN, "tile too small for the block");
  static_assert(ROWS * KB % 1024 == 0, "image not a whole number of wave-instructions");
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    // even split: wave w owns instructions [w NI, (w+1) NI); otherwise they are dealt
    // round-robin (wave w: w, w + NW, ...) and the last round is partial (tile_dma_count)
    const int q = EVEN ? w * NI + i : i * NW + w;
    if (!EVEN && q >= TOT) break;           // wave-uniform
    int row, kk;
    chunk_src<T, KMAJ, KB, ROWS>(q * 64 + lane, row, kk);
    const T* src;
    if constexpr (KMAJ) {
      const int gr = min(r0 + row, rows_lim - 1);
      JMT_DCHECK(gr >= 0 && kloc + kk >= 0);
      src = base + (int64_t)gr * ld + kloc + kk;
    } else {
      int gm = r0 + row;
      if (gm >= rows_lim) gm = ((rows_lim - 1) / V) * V;
      src = base + (int64_t)(kloc + kk) * ld + gm;
    }
    glds_asm(src, img + q * 1024);
  }
}

// Interleaved staging (Cfg IL): the per-lane byte offset of each of this wave's LDS-DMA
// instructions of one operand's K-tile, relative to the K-tile's scalar base (operand base +
// k0 along K).  Constant over the K loop of a block: computed once.
template <typename T, bool KMAJ, int KB, int ROWS, int NT>
__device__ __forceinline__ void glds_offsets(uint32_t* off, int64_t ld, int rows_lim, int r0) {
  constexpr int V = Vec<T>::n;
  constexpr int NW = NT / 64;
  constexpr int NI = ROWS * KB / 1024 / NW;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int q = w * NI + i;
    int row, kk;
    chunk_src<T, KMAJ, KB, ROWS>(q * 64 + lane, row, kk);
    int64_t e;
    if constexpr (KMAJ) {
      e = (int64_t)min(r0 + row, rows_lim - 1) * ld + kk;
    } else {
      int gm = r0 + row;
      if (gm >= rows_lim) gm = ((rows_lim - 1) / V) * V;
      e = (int64_t)kk * ld + gm;
    }
    off[i] = (uint32_t)(e * (int64_t)sizeof(T));
  }
}

// one LDS-DMA instruction i (this wave's slot) of an operand K-tile whose scalar base is `src`
template <int NI>
__device__ __forceinline__ void glds_slot(char* img, const char* src, const uint32_t* off, int i) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  glds_asm(src + off[i], img + (w * NI + i) * 1024);
}

// Register staging of one (partial, masked) K-tile: NC chunks of 16 B per thread.
template <typename T, bool KMAJ, int KB, int ROWS, int NT>
__device__ __forceinline__ void stage_tile(char* img, const T* base, int64_t ld, int rows_lim,
                                           int r0, int k_lim, int kloc) {
  constexpr int V = Vec<T>::n;
  constexpr int CH = ROWS * KB / 16;        // 16-B chunks of the image
  constexpr int NC = (CH + NT - 1) / NT;
  uint4 r[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int id = threadIdx.x + NT * i;
    if (CH % NT != 0 && id >= CH) {
      r[i] = make_uint4(0, 0, 0, 0);
      continue;
    }
    int row, kk;
    chunk_src<T, KMAJ, KB, ROWS>(id, row, kk);
    const int gr = r0 + row;
    const int gk = kloc + kk;
    uint4 v = make_uint4(0, 0, 0, 0);
    if constexpr (KMAJ) {
      if (gr < rows_lim && gk < k_lim) {
        const T* src = base + (int64_t)gr * ld + gk;
        if (gk + V <= k_lim) {
          v = *(const uint4*)src;
        } else {
          T tmp[V];
#pragma unroll
          for (int e = 0; e < V; ++e) tmp[e] = (gk + e < k_lim) ? src[e] : from_f<T>(0.f);
          v = *(uint4*)tmp;
        }
      }
    } else {
      if (gk < k_lim && gr < rows_lim) {
        const T* src = base + (int64_t)gk * ld + gr;
        if (gr + V <= rows_lim) {
          v = *(const uint4*)src;
        } else {
          T tmp[V];
#pragma unroll
          for (int e = 0; e < V; ++e) tmp[e] = (gr + e < rows_lim) ? src[e] : from_f<T>(0.f);
          v = *(uint4*)tmp;
        }
      }
    }
    r[i] = v;
  }
#pragma unroll
  for (int i = 0; i < NC; ++i)
    if (CH % NT == 0 || threadIdx.x + NT * i < CH) *(uint4*)(img + (threadIdx.x + NT * i) * 16) = r[i];
}

// ------------------------------------------------------------------ fragment reads
template <int KB>
__device__ __forceinline__ int kmaj_off(int row, int c) {
  return row * KB + ((c ^ swz_k<KB>(row)) << 4);
}
template <int RB>
__device__ __forceinline__ int mnmaj16_off(int k, int m) {
  const int c = m >> 3;
  const int cp = ((((c >> 1) ^ swz_t<RB>(k))) << 1) | (c & 1);
  return k * RB + (cp << 4) + ((m & 7) << 1);
}

// 16-bit A/B fragment of one 16-row sub-tile for k-step ks (32 wide) of the current K-tile:
// lane l holds X[row rbase + (l&15)][k = 32 ks + 8 (l>>4) + j], j = 0..7.
template <typename T, bool KMAJ, int KB, int ROWS>
__device__ __forceinline__ typename Frag16<T>::t read_frag16(const char* img, int rbase, int ks) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  const int lane = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *(const F*)(img + kmaj_off<KB>(row, c));
  } else {
    constexpr int RB = ROWS * 2;
    const int i = lane & 15;
    const int k0 = ks * 32 + (lane >> 4) * 8 + (i >> 2);
    const int m = rbase + (i & 3) * 4;
    Hf lo = tr_read<Hf>(img + mnmaj16_off<RB>(k0, m));
    Hf hi = tr_read<Hf>(img + mnmaj16_off<RB>(k0 + 4, m));
    F f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
}

// f32 fragment: element s (0..3) is the operand value at k = seg*16 + 4*(lane>>4) + s.
template <bool KMAJ, int KB, int ROWS>
__device__ __forceinline__ f32x4 read_frag32(const char* img, int rbase, int seg) {
  const int lane = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = seg * 4 + (lane >> 4);
    return *(const f32x4*)(img + kmaj_off<KB>(row, c));
  } else {
    const float* f = (const float*)img;
    const int m = rbase + (lane & 15);
    const int k = seg * 16 + 4 * (lane >> 4);
    f32x4 r;
    r[0] = f[(k + 0) * ROWS + m];
    r[1] = f[(k + 1) * ROWS + m];
    r[2] = f[(k + 2) * ROWS + m];
    r[3] = f[(k + 3) * ROWS + m];
    return r;
  }
}


__device__ __forceinline__ void sgb_ds_reads(int n) {   // sched_group_barrier needs literals
  switch (n) {
    case 1: __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); break;
    case 2: __builtin_amdgcn_sched_group_barrier(0x100, 2, 0); break;
    case 4: __builtin_amdgcn_sched_group_barrier(0x100, 4, 0); break;
    case 5: __builtin_amdgcn_sched_group_barrier(0x100, 5, 0); break;
    case 6: __builtin_amdgcn_sched_group_barrier(0x100, 6, 0); break;
    case 8: __builtin_amdgcn_sched_group_barrier(0x100, 8, 0); break;
    case 9: __builtin_amdgcn_sched_group_barrier(0x100, 9, 0); break;
    case 10: __builtin_amdgcn_sched_group_barrier(0x100, 10, 0); break;
    default: break;
  }
}

struct NoIssue {
  __device__ __forceinline__ void operator()(int) const {}
};

// Row sums of the A operand (launches with n_dbias > 0: the bias gradient db = sum_k dY^T[m][k]
// of a weight-gradient GEMM, taken from the A image already in LDS instead of a second pass over
// dY in HBM).  M-subtile i of a block's row panel is summed by wave wn = i % WN of the n-tile
// (i / WN) % tiles_n — spread over the waves and n-tiles, so a wave re-reads at most
// ceil(TM / WN) fragments per k-step (for the 256x256 tile of an N = 512 wgrad: one).  After
// the MFMAs of a K-tile (before the barrier that frees its stage) the owner reads the fragment
// again and adds its 8 k-values with four v_dot2 against the literal (1, 1): one fp32 per lane,
// the four k-groups folded at the end.  (Folded into the MFMA loop instead — as an MFMA against
// an all-ones fragment, or as dot2s on the fragments in flight — the extra registers or the
// owner branch inside the unrolled block spilled the 256x256 and 4-block tiles: +14-44 % on the
// qkv / cross-attention wgrads, profiles/r03_wgrad_dbias.jsonl.)
struct NoRowSums {
  static constexpr bool on = false;
};
template <class C> struct RowSums {
  static constexpr bool on = true;
  static constexpr int NV = (C::TM + C::WN - 1) / C::WN;
  float v[NV];
  uint32_t own;     // bit i: this wave sums m-subtile i (wave-uniform)
};

__device__ __forceinline__ float rowsum8(bf16x8 a, float c) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 0, 1), one, c, false);
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 2, 3), one, c, false);
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 4, 5), one, c, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 6, 7), one, c, false);
}
__device__ __forceinline__ float rowsum8(f16x8 a, float c) {
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  const f16x2 one = {(_Float16)1.0f, (_Float16)1.0f};
  c = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 0, 1), one, c, false);
  c = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 2, 3), one, c, false);
  c = __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 4, 5), one, c, false);
  return __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, 6, 7), one, c, false);
}
template <bool RS, class C> struct RowSumSel { typedef NoRowSums type; };
template <class C> struct RowSumSel<true, C> { typedef RowSums<C> type; };

template <typename T, bool AK, class C>
__device__ __forceinline__ void rowsum_tile(const char* imgA, int wm, int wn, RowSums<C>& rs) {
  constexpr int KS = C::KB / 64;
#pragma unroll
  for (int sl = 0; sl < RowSums<C>::NV; ++sl) {
    const int i = sl * C::WN + wn;
    if (i >= C::TM || !((rs.own >> i) & 1u)) continue;     // wave-uniform
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      rs.v[sl] = rowsum8(read_frag16<T, AK, C::KB, C::BM>(imgA, wm * C::WTM + i * 16, ks),
                         rs.v[sl]);
  }
}

// MODE (development ablations of the persistent kernel, gemm_persist.hip dbg 64 / 128): 1 = the
// fragments are read from LDS once per K-tile row 0 and reused (MFMAs without the LDS reads),
// 2 = the LDS reads without the MFMAs (one v_add per MFMA keeps the reads live)
template <typename T, bool AK, bool BK, class C, class ISSUE = NoIssue, int MODE = 0>
__device__ __forceinline__ void compute_tile(const char* imgA, const char* imgB, int wm, int wn,
                                             f32x4 (&acc)[C::TM][C::TN],
                                             const ISSUE& issue = ISSUE()) {
  if constexpr (sizeof(T) == 2) {
    // software-pipelined fragment reads: the A fragment of MFMA row i+1 (and, at the last row
    // of a k-step, the B fragments of the next k-step) are issued before the MFMAs of row i,
    // so LDS latency hides behind TN MFMAs instead of stalling on lgkmcnt(0)
    typedef typename Frag16<T>::t F;
    constexpr int KS = C::KB / 64;
    constexpr int NR = KS * C::TM;                 // MFMA rows of one K-tile
    constexpr int PF = C::PF;                      // A rows read ahead
    constexpr int BPF = PF < C::TM ? PF : C::TM - 1;   // B fragments read BPF rows ahead
    F fb[2][C::TN];
    F fa[PF + 1];
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
      fb[0][j] = read_frag16<T, BK, C::KB, C::BN>(imgB, wn * C::WTN + j * 16, 0);
#pragma unroll
    for (int r = 0; r < PF; ++r)
      if (r < NR) fa[r] = read_frag16<T, AK, C::KB, C::BM>(imgA, wm * C::WTM + (r % C::TM) * 16,
                                                          r / C::TM);
#pragma unroll
    for (int idx = 0; idx < NR; ++idx) {
      const int ks = idx / C::TM, i = idx % C::TM;
      int nreads = 0;
      if (MODE != 1 && i == C::TM - BPF && ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          fb[(ks + 1) & 1][j] = read_frag16<T, BK, C::KB, C::BN>(imgB, wn * C::WTN + j * 16,
                                                                 ks + 1);
        nreads += BK ? C::TN : 2 * C::TN;
      }
      if (MODE != 1 && idx + PF < NR) {
        const int r = idx + PF;
        fa[r % (PF + 1)] = read_frag16<T, AK, C::KB, C::BM>(imgA, wm * C::WTM + (r % C::TM) * 16,
                                                           r / C::TM);
        nreads += AK ? 1 : 2;
      }
      issue(idx);                                   // interleaved LDS-DMA pieces (Cfg IL)
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(1);
      if constexpr (MODE == 2) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j][0] += __builtin_bit_cast(float, __builtin_shufflevector(
                              fb[ks & 1][j], fa[idx % (PF + 1)], 0, 8)) ;
      } else if constexpr (MODE == 1) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = mfma16(fb[0][j], fa[0], acc[i][j]);
      } else {
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = mfma16(fb[ks & 1][j], fa[idx % (PF + 1)], acc[i][j]);   // C^T tile
      }
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (C::SGB) {
        sgb_ds_reads(nreads);                                                 // DS reads first
        __builtin_amdgcn_sched_group_barrier(0x008, C::TN, 0);               // then the MFMAs
      }
    }
  } else {
#pragma unroll
    for (int seg = 0; seg < C::KB / 64; ++seg) {
      f32x4 fb[C::TN];
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        fb[j] = read_frag32<BK, C::KB, C::BN>(imgB, wn * C::WTN + j * 16, seg);
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const f32x4 fa = read_frag32<AK, C::KB, C::BM>(imgA, wm * C::WTM + i * 16, seg);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < C::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[j][s], fa[s], acc[i][j], 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n <= 16 (wave-uniform)
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
  }
}

// LDS-DMA instructions this wave issues per K-tile of one operand image of `tot` instructions
// (glds_tile: an even split, or round-robin with a partial last round)
template <int TOT, int NW>
__device__ __forceinline__ int dma_count(int w) {
  if constexpr (TOT % NW == 0) return TOT / NW;
  else return w < TOT % NW ? TOT / NW + 1 : TOT / NW;
}

// wait until at most n (runtime, < 8) K-tiles of VMT DMA instructions each are outstanding
template <int N>
__device__ __forceinline__ void wait_vmcnt_capped() { wait_vmcnt<(N < 63 ? N : 63)>(); }
template <int VMT>
__device__ __forceinline__ void wait_tiles(int n) {
  switch (n) {
    case 0: wait_vmcnt<0>(); break;
    case 1: wait_vmcnt_capped<VMT>(); break;
    case 2: wait_vmcnt_capped<2 * VMT>(); break;
    case 3: wait_vmcnt_capped<3 * VMT>(); break;
    case 4: wait_vmcnt_capped<4 * VMT>(); break;
    case 5: wait_vmcnt_capped<5 * VMT>(); break;
    case 6: wait_vmcnt_capped<6 * VMT>(); break;
    default: wait_vmcnt_capped<7 * VMT>(); break;
  }
}

// 4 consecutive elements row[n..n+3] as floats (one vector load when aligned and in range;
// elements past `lim` read as 0)
template <typename O>
__device__ __forceinline__ void load4_guard(const O* row, int n, int lim, bool vec4, float (&v)[4]) {
  if (vec4 && n + 4 <= lim) {
    if constexpr (sizeof(O) == 4) {
      const float4 t = *(const float4*)(row + n);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
      const uint2 t = *(const uint2*)(row + n);
      const O* h = (const O*)&t;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = to_f(h[e]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (n + e < lim) ? to_f(row[n + e]) : 0.f;
  }
}

// The reduce + epilogue of W (1 or 4) consecutive outputs (b, m, n..n+W-1): the splits' fp32
// partial slabs summed in split order (the same order, so the same bits, wherever it runs),
// then alpha, bias, beta * C, ReLU, the ReLU mask; the A row sums' split partials folded by the
// thread of column 0.
template <typename O, int W>
__device__ __forceinline__ void reduce_outputs(const GemmParams& p, int b, int m, int n) {
  const int nb = p.batch0 * p.batch1;
  const int64_t per = (int64_t)p.M * p.N;
  const int64_t mn = (int64_t)m * p.N + n;
  float v[W];
#pragma unroll
  for (int i = 0; i < W; ++i) v[i] = 0.f;
  const int64_t sstride = (int64_t)nb * per;
  const float* src0 = p.ws + (int64_t)b * per + mn;
  int s = 0;
  if constexpr (W == 4) {
    // (every slab load of up to 32 splits issued before the first add measured slower: 19.7 vs
    // 17.3 us per reduce launch in the c3 step, profiles/r06/reduce_prof_all_loads_first.csv vs reduce_prof_rowsum_batched.csv)
    // (two lanes per output group, each summing half of the splits, then lo + hi: slower in
    // the c3 step, 4.014-4.024 vs 4.001-4.011 ms, profiles/r06/step_ab_skr_pair.txt)
    // eight (then four) slab loads in flight per step, summed in split order (the same sums as
    // four at a time: bit-identical; no measurable change in the step, profiles/r04/
    // splitk_reduce_depth_ab.txt)
    for (; s + 8 <= p.splits; s += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *(const float4*)(src0 + (s + u) * sstride);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[0] += t[u].x; v[1] += t[u].y; v[2] += t[u].z; v[3] += t[u].w;
      }
    }
    for (; s + 4 <= p.splits; s += 4) {
      float4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = *(const float4*)(src0 + (s + u) * sstride);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[0] += t[u].x; v[1] += t[u].y; v[2] += t[u].z; v[3] += t[u].w;
      }
    }
  }
  for (; s < p.splits; ++s) {
    const float* src = src0 + s * sstride;
    if constexpr (W == 4) {
      const float4 t = *(const float4*)src;
      v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
    } else {
      v[0] += *src;
    }
  }
  const int b0 = b / p.batch1, b1 = b % p.batch1;
  if (p.n_dbias > 0 && n == 0 && p.dbias_tab[b0]) {   // the A row sums' split partials
    const float* src = p.dbias_ws + (int64_t)b * p.M + m;
    const int64_t ts = (int64_t)nb * p.M;
    float r = 0.f;
    int t = 0;
    // eight loads in flight per step, summed in split order (a plain loop issued them one at a
    // time behind each add: ~20 dependent HBM round trips for the column-0 threads at 21 splits,
    // the tail of every row-summing reduce launch)
    for (; t + 8 <= p.splits; t += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = src[(t + u) * ts];
#pragma unroll
      for (int u = 0; u < 8; ++u) r += x[u];
    }
    for (; t < p.splits; ++t) r += src[t * ts];
    float* d = p.dbias_tab[b0];
    d[m] = (p.dbias_acc ? d[m] : 0.f) + r;
  }
  const float* biasp = p.n_bias > 0 ? p.bias_tab[b0] : p.bias;
  O* cp;
  int64_t cbase;
  if (p.c_mode == 1) {
    cp = (O*)p.c_ptr[b0];
    cbase = (int64_t)b1 * p.sC1;
  } else {
    cp = (O*)p.c_ptr[0];
    cbase = (int64_t)b0 * p.sC0 + (int64_t)b1 * p.sC1;
  }
  const int64_t co = cbase + (int64_t)m * p.ldc + n;
  const O* auxp = (const O*)p.aux;
  float cin[W], ain[W];
  if constexpr (W == 4) {
    if (p.beta != 0.f) load4_guard(cp + co, 0, 4, true, cin);
    if (auxp) load4_guard(auxp + cbase + (int64_t)m * p.ldaux + n, 0, 4, true, ain);
  } else {
    if (p.beta != 0.f) cin[0] = to_f(cp[co]);
    if (auxp) ain[0] = to_f(auxp[cbase + (int64_t)m * p.ldaux + n]);
  }
  O out[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    float x = v[i] * p.alpha;
    if (p.bias_mode == 1) x += biasp[n + i];
    else if (p.bias_mode == 2) x += biasp[m];
    if (p.beta != 0.f) x += p.beta * cin[i];
    if (p.relu) x = fmaxf(x, 0.f);
    if (auxp && !(ain[i] > 0.f)) x = 0.f;
    out[i] = from_f<O>(x);
  }
  if constexpr (W == 4) {
    if constexpr (sizeof(O) == 4) *(float4*)(cp + co) = *(const float4*)out;
    else *(uint2*)(cp + co) = *(const uint2*)out;
  } else {
    cp[co] = out[0];
  }
}

// gemm_persist.hip: launch the persistent kernel (cfg 40) on `blocks` blocks
int launch_gemm_persist(const GemmParams& p, int dt, int ak, int bk, int cfg, int blocks,
                        hipStream_t st);
int num_cus_persist();
// the persistent configuration (40) jmt_gemm launches for this descriptor, 0 = none: `forced`
// is jmt_gemm_set_debug's forced tile config (40 takes the persistent kernel where its
// preconditions hold); otherwise JMT_GEMM_PERSIST (0 off, 40 every eligible launch, unset: the
// measured default by layout and shape)
int persist_choice(const jmt_gemm_desc* d, const GemmParams& p, int splits, int forced);
// gemm_persist_kernel's limit on the per-column bias staged in LDS (floats, all tables)
constexpr int kPersistBias = 8192;
// gemm_persist.hip, split-K ping-pong (cfg 44): the launch (fp32 slabs + optional A row sums;
// the caller reduces), its preconditions, and the planner's split count for it (0: not used)
void launch_gemm_pp_split(const GemmParams& p, int dt, int ak, int bk, bool rs, int blocks,
                          hipStream_t st);
bool pp_split_ok(int dt, int M, int N, int K, int splits);
int pp_split_plan(int dt, int M, int N, int K, int batch);

}  // namespace jmt
