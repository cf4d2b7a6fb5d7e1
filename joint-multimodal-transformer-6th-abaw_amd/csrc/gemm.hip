// LDS-tiled MFMA GEMM for gfx950 (CDNA4), wave64.
//
//   C[b] = epilogue( alpha * A[b] (M x K) . B[b] (K x N) )
//
// Serves every matmul on the JMT path: nn.Linear forward (NT), its dgrad
// (NN) and wgrad (TN, split-K over the B*T tokens), and the attention products S = Q K^T,
// O = P V and their backward (batched over (batch, head) with two batch strides).
//
// Design:
//  * Tile configurations (TileCfg): block tile BM x BN computed by WM x WN waves, each wave a
//    (BM/WM) x (BN/WN) tile of 16x16 MFMA sub-tiles.  16-bit inputs: v_mfma_f32_16x16x32_{bf16,
//    f16}; f32 inputs (the fp32 parity mode): v_mfma_f32_16x16x4_f32 (exact f32 fma chain).
//      cfg 1: 128x128, 2x2 waves  (256 threads, 2 blocks / CU)   — small / batched problems
//      cfg 5: 256x256, 2x4 waves  (512 threads, 1 block / CU)    — large problems: 2x the
//             FLOPs per byte staged into LDS.  The planner (plan()) picks tile and split-K from
//             a cost model; 256x128 / 128x256 tiles and 3-5 stage KB=64 pipelines measured slower
//             on every JMT shape (profiles/r01_gemm_tiles.txt).
//    A K-tile is KB = 128 bytes per operand row (64 elements of 16-bit, 32 of f32).
//  * Operands are staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, no
//    VGPR round trip) into S = 2 LDS stages.  The LDS image depends on the operand's memory order:
//      K-major operand  -> image [row][k], 16-B chunks XOR-swizzled by (row>>1)&7, read with
//                          ds_read_b128 (conflict-free for the 16-row fragment reads);
//      MN-major operand -> image [k][row], 32-B pairs swizzled by t(k), read with
//                          ds_read_b64_tr_b16 (hardware transpose) for 16-bit types.
//    The LDS-DMA destination is linear per wave-instruction, so swizzles go on the per-lane
//    GLOBAL source address.  A trailing partial K-tile is staged through registers with masks.
//  * Operands may be K-concatenations of up to 8 tensors (cat(...) @ W^T without a concat copy)
//    or per-batch pointer tables; C may be a per-batch pointer table.
//  * The MFMA is fed (B, A), so each accumulator holds a TRANSPOSED 16x16 tile: a lane owns one
//    C row and 4 consecutive columns, and the epilogue stores straight from registers (8-B
//    bf16 / 16-B fp32 stores, 16 rows x 64 B per instruction) with alpha, bias (per column / per
//    row), beta*C, ReLU and the ReLU-backward mask fused — no LDS round trip, no barriers
//    (measured 10-15% faster than an LDS-staged 16-B-row epilogue).
//  * split-K writes fp32 partial slabs to a caller-owned workspace; jmt_gemm launches the
//    reduce + epilogue kernel afterwards (deterministic, no atomics).
//  * XCD-aware bijective block -> tile remap: blocks sharing an A row panel run on one XCD.
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
  int a_mode, b_mode, c_mode;   // 0 strided, 1 pointer per b0, 2 K-concat (a/b only)
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
// instructions of a K-tile are dealt round-robin over the 8 waves (glds_tile, dma_count).
using Cfg30 = TileCfg<160, 256, 2, 4, 128, 2, 1, 1, 0>;
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
  if (mode == 2) {
    const int seg = k0 / kseg;
    kloc = k0 - seg * kseg;
    return (const T*)ptrs[seg];
  }
  kloc = k0;
  const T* p = (const T*)ptrs[mode == 1 ? b0 : 0];
  return p + (mode == 1 ? 0 : (int64_t)b0 * s0) + (int64_t)b1 * s1;
}

// Swizzles.  K-major image: ROWS rows of KB bytes; MN-major image: KB/sizeof(T) k-rows of
// RB = ROWS*sizeof(T) bytes.
template <int KB>
__device__ __forceinline__ int swz_k(int row) {
  if constexpr (KB == 128) return (row >> 1) & 7;
  else return (row >> 2) & 3;
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
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + q * 1024),
                                     16, 0, 0);
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
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off[i]),
                                   (__attribute__((address_space(3))) void*)(img + (w * NI + i) * 1024),
                                   16, 0, 0);
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

template <typename T, bool AK, bool BK, class C, class ISSUE = NoIssue>
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
      if (i == C::TM - BPF && ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          fb[(ks + 1) & 1][j] = read_frag16<T, BK, C::KB, C::BN>(imgB, wn * C::WTN + j * 16,
                                                                 ks + 1);
        nreads += BK ? C::TN : 2 * C::TN;
      }
      if (idx + PF < NR) {
        const int r = idx + PF;
        fa[r % (PF + 1)] = read_frag16<T, AK, C::KB, C::BM>(imgA, wm * C::WTM + (r % C::TM) * 16,
                                                           r / C::TM);
        nreads += AK ? 1 : 2;
      }
      issue(idx);                                   // interleaved LDS-DMA pieces (Cfg IL)
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        acc[i][j] = mfma16(fb[ks & 1][j], fa[idx % (PF + 1)], acc[i][j]);   // C^T tile
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

// ------------------------------------------------------------------ main kernel
// one unit of work: an output tile of one batch entry and one K split
struct GemmWork {
  int m0, n0, b, b0, b1, split, kbeg, kend;
};

template <class C>
__device__ __forceinline__ GemmWork decode_work(const GemmParams& p, int w) {
  const int ntile = p.tiles_m * p.tiles_n;
  const int nb = p.batch0 * p.batch1;
  // split-K: every tile of one (batch entry, K split) reads the same K rows of both operands, so
  // the whole work list is remapped (bijectively) so that each XCD — the hardware deals blocks
  // to XCDs round-robin by linear id — runs a contiguous range of work items, i.e. whole
  // (batch, split) groups whose operand rows its own L2 serves to all of the group's tiles
  // (dealt across the XCDs, each group's operand panels were fetched ~3x from HBM / MALL)
  const bool global = p.splits > 1 && !(p.dbg & 16);
  if (global) {
    const int W = ntile * nb * p.splits;
    const int q = W / 8, rm = W % 8, x = w % 8;
    w = x * q + min(x, rm) + w / 8;
  }
  const int bid = w % ntile;
  const int rest = w / ntile;
  GemmWork r;
  r.b = rest % nb;
  r.split = rest / nb;
  // XCD-aware remap (bijective): consecutive logical tiles (same A row panel) on one XCD.
  int wg = bid;
  if (!global && ntile >= 16) {
    const int q = ntile / 8, rm = ntile % 8, x = bid % 8;
    wg = (x < rm ? x * (q + 1) : rm * (q + 1) + (x - rm) * q) + bid / 8;
  }
  r.m0 = (wg / p.tiles_n) * C::BM;
  r.n0 = (wg % p.tiles_n) * C::BN;
  r.b0 = r.b / p.batch1;
  r.b1 = r.b % p.batch1;
  r.kbeg = r.split * p.k_per_split;
  r.kend = min(p.K, r.kbeg + p.k_per_split);
  return r;
}

// LDS-DMA of K-tile kt of work item `wk` into stage `buf`
template <typename T, bool AK, bool BK, class C>
__device__ __forceinline__ void issue_ktile(const GemmParams& p, char* smem, const GemmWork& wk,
                                            int kt, int buf) {
  constexpr int BKE = C::KB / (int)sizeof(T);
  const int k0 = wk.kbeg + kt * BKE;
  int ka, kb;
  const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, wk.b0, wk.b1, p.a_kseg, k0, ka);
  const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, wk.b0, wk.b1, p.b_kseg, k0, kb);
  char* base = smem + buf * C::STAGE;
  glds_tile<T, AK, C::KB, C::BM, C::NT>(base, A, p.lda, p.M, wk.m0, ka);
  glds_tile<T, BK, C::KB, C::BN, C::NT>(base + C::BM * C::KB, B, p.ldb, p.N, wk.n0, kb);
}

template <typename T, typename O, class C>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, const GemmWork& wk,
                                              f32x4 (&acc)[C::TM][C::TN], int lane, int wm,
                                              int wn) {
  const int m0 = wk.m0, n0 = wk.n0, b = wk.b, b0 = wk.b0, b1 = wk.b1, split = wk.split;
  // ---- epilogue.  acc[i][j] holds the TRANSPOSED 16x16 tile (the MFMA was fed B as its first
  //      operand): lane owns C row (lane&15) and the 4 consecutive columns 4*(lane>>4) + r.
  const bool partial = p.splits > 1;
  const float* biasp = p.n_bias > 0 ? p.bias_tab[b0] : p.bias;
  O* cp;
  int64_t cbase;
  float alpha = p.alpha, beta = p.beta;
  int bias_mode = p.bias_mode, relu = p.relu;
  int64_t ldc = p.ldc;
  const O* auxp = partial ? nullptr : (const O*)p.aux;
  if (partial) {   // raw partial sums: no epilogue ops, row stride N
    const int nb = p.batch0 * p.batch1;
    cp = (O*)(p.ws + ((int64_t)split * nb + b) * (int64_t)p.M * p.N);
    cbase = 0;
    alpha = 1.f; beta = 0.f; bias_mode = 0; relu = 0; ldc = p.N;
  } else {
    if (p.c_mode == 1) {
      cp = (O*)p.c_ptr[b0];
      cbase = (int64_t)b1 * p.sC1;
    } else {
      cp = (O*)p.c_ptr[0];
      cbase = (int64_t)b0 * p.sC0 + (int64_t)b1 * p.sC1;
    }
  }
  if (p.dbg & 2) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 12345.678f) ((float*)cp)[0] = sum;   // keep acc live
    return;
  }
  if constexpr (sizeof(O) == 2 && C::TN % 2 == 0) {
    // 16-bit C, whole wave tile in range (wave-uniform): pair the accumulators of sub-tiles j and
    // j+1 with v_permlane16_swap so that every lane holds 8 consecutive columns of one row ->
    // one 16-B store per lane per tile pair (half the store instructions of the 8-B path; the
    // epilogue is store-issue-bound)
    const int g = lane >> 4, rl = lane & 15;
    if (!partial && p.c_vec8 && m0 + wm * C::WTM + C::WTM <= p.M &&
        n0 + wn * C::WTN + C::WTN <= p.N) {
      const bool plain = beta == 0.f && auxp == nullptr;
      float bias4[C::TN][4];
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int n = n0 + wn * C::WTN + 16 * j + 4 * g;
#pragma unroll
        for (int e = 0; e < 4; ++e) bias4[j][e] = (bias_mode == 1) ? biasp[n + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int m = m0 + wm * C::WTM + 16 * i + rl;
        const float bm = (bias_mode == 2) ? biasp[m] : 0.f;
        const int64_t rowo = cbase + (int64_t)m * ldc;
        const int64_t rowa = cbase + (int64_t)m * p.ldaux;
        float cin[C::TN][4], ain[C::TN][4];
        if (beta != 0.f) {
#pragma unroll
          for (int j = 0; j < C::TN; ++j)
            load4_guard(cp + rowo, n0 + wn * C::WTN + 16 * j + 4 * g, p.N, true, cin[j]);
        }
        if (auxp) {
#pragma unroll
          for (int j = 0; j < C::TN; ++j)
            load4_guard(auxp + rowa, n0 + wn * C::WTN + 16 * j + 4 * g, p.N, true, ain[j]);
        }
#pragma unroll
        for (int jp = 0; jp < C::TN / 2; ++jp) {
          uint32_t pk[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 2 * jp + h;
            float x[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              x[e] = acc[i][j][e] * alpha + bias4[j][e] + bm;
              if (!plain) {
                if (beta != 0.f) x[e] += beta * cin[j][e];
                if (relu) x[e] = fmaxf(x[e], 0.f);
                if (auxp && !(ain[j][e] > 0.f)) x[e] = 0.f;
              } else if (relu) {
                x[e] = fmaxf(x[e], 0.f);
              }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              O hh[2] = {from_f<O>(x[2 * q]), from_f<O>(x[2 * q + 1])};
              pk[h][q] = *(const uint32_t*)hh;
            }
          }
          const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          const int n = n0 + wn * C::WTN + 16 * (2 * jp + (g & 1)) + 8 * (g >> 1);
          typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
          // streaming (nontemporal) stores: measured 5-12% faster on the JMT shapes
          JMT_DCHECK(m < p.M && n + 8 <= p.N);
          if (p.dbg & 4) *(u32x4*)(cp + rowo + n) = v;
          else __builtin_nontemporal_store(v, (u32x4*)(cp + rowo + n));
        }
      }
      return;
    }
  }
  {
    // direct epilogue: 4 consecutive columns per lane -> one 8-B (16-bit) / 16-B (fp32) store,
    // 16 rows x 4 lanes per instruction; no LDS round trip, no block barriers.
    const int rl = lane & 15, cq = 4 * (lane >> 4);
    const bool vec4 = partial ? (p.N % 4) == 0 : p.c_vec4 != 0;
    float bias4[C::TN][4];
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int n = n0 + wn * C::WTN + 16 * j + cq;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        bias4[j][e] = (bias_mode == 1 && n + e < p.N) ? biasp[n + e] : 0.f;
    }
    const bool plain = beta == 0.f && auxp == nullptr;
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
      const int m = m0 + wm * C::WTM + 16 * i + rl;
      if (m >= p.M) continue;
      const float bm = (bias_mode == 2) ? biasp[m] : 0.f;
      const int64_t rowo = cbase + (int64_t)m * ldc;
      const int64_t rowa = cbase + (int64_t)m * p.ldaux;
      // beta*C / ReLU-mask operands: all TN 4-element groups of this row are loaded up front
      // (one 8-B / 16-B load each, uniform branches) so their latencies overlap
      float cin[C::TN][4], ain[C::TN][4];
      if (beta != 0.f) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j) load4_guard(cp + rowo, n0 + wn * C::WTN + 16 * j + cq, p.N, vec4, cin[j]);
      }
      if (auxp) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j) load4_guard(auxp + rowa, n0 + wn * C::WTN + 16 * j + cq, p.N, vec4, ain[j]);
      }
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int n = n0 + wn * C::WTN + 16 * j + cq;
        if (n >= p.N) continue;
        const bool full4 = vec4 && n + 4 <= p.N;
        JMT_DCHECK(m >= 0 && m < p.M && n >= 0);
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = acc[i][j][e] * alpha + bias4[j][e] + bm;
        if (!plain) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (beta != 0.f) x[e] += beta * cin[j][e];
            if (relu) x[e] = fmaxf(x[e], 0.f);
            if (auxp && !(ain[j][e] > 0.f)) x[e] = 0.f;
          }
        } else if (relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
        }
        if (full4) {
          if constexpr (sizeof(O) == 4) {
            *(float4*)(cp + rowo + n) = make_float4(x[0], x[1], x[2], x[3]);
          } else {
            O o4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o4[e] = from_f<O>(x[e]);
            *(uint2*)(cp + rowo + n) = *(const uint2*)o4;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) cp[rowo + n + e] = from_f<O>(x[e]);
        }
      }
    }
  }
}

// development timeline probe (dbg & 8): wave 0 of each block stamps s_memrealtime (100 MHz) at
// kernel entry, first K-tile landed, main loop done, epilogue done (scripts/gemm_timeline.py)
constexpr int kTraceBlocks = 8192;
__device__ uint64_t g_gemm_trace[kTraceBlocks * 4];
__device__ __forceinline__ void trace_stamp(const GemmParams& p, int slot) {
  if (!(p.dbg & 8) || threadIdx.x != 0) return;
  const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (b < kTraceBlocks) g_gemm_trace[b * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}

// One block per output tile (blockIdx.x, XCD-remapped), batch entry (blockIdx.y) and K split
// (blockIdx.z).  (A persistent form — blocks capped at the resident slots, the next tile's first
// K-tile prefetched under the epilogue — measured 3-5% slower: profiles/r01_gemm_persistent.txt.)
// A row sums of one block (RowSums above) -> dbias_tab[b0][m] (+)=, or the split's fp32 partial
template <class C>
__device__ __forceinline__ void rowsum_store(const GemmParams& p, const GemmWork& wk,
                                             const RowSums<C>& rs, int lane, int wm) {
  const int nb = p.batch0 * p.batch1;
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    if (!((rs.own >> i) & 1u)) continue;                  // wave-uniform
    float v = rs.v[i / C::WN];
    v += __shfl_xor(v, 16);                                // the four k-groups of row lane & 15
    v += __shfl_xor(v, 32);
    const int m = wk.m0 + wm * C::WTM + 16 * i + lane;
    if (lane >= 16 || m >= p.M) continue;
    if (p.splits > 1) {
      p.dbias_ws[((int64_t)wk.split * nb + wk.b) * p.M + m] = v;
    } else {
      float* d = p.dbias_tab[wk.b0];
      d[m] = (p.dbias_acc ? d[m] : 0.f) + v;
    }
  }
}

template <typename T, typename O, bool AK, bool BK, class C, bool RS = false>
__global__ __launch_bounds__(C::NT, C::OCC)
void gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BKE = C::KB / (int)sizeof(T);         // K elements per tile
  constexpr int IA = C::BM * C::KB;                   // A image bytes
  constexpr int NWV = C::NT / 64;
  // LDS-DMA instructions per wave per K-tile (the same for every wave unless an image's count is
  // not a multiple of the wave count, e.g. the 160-row tile: then it depends on the wave)
  constexpr int VMT = ((C::BM + C::BN) * C::KB / 1024 + NWV - 1) / NWV;

  const int ntile = p.tiles_m * p.tiles_n;
  const GemmWork cur = decode_work<C>(
      p, blockIdx.x + ntile * (blockIdx.y + p.batch0 * p.batch1 * blockIdx.z));
  const int klen = max(0, cur.kend - cur.kbeg);
  const int nfull = klen / BKE;
  const bool tail = (klen % BKE) != 0;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  trace_stamp(p, 0);

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  typedef typename RowSumSel<RS, C>::type RSumT;
  RSumT rsum;
  [[maybe_unused]] const int wnu = __builtin_amdgcn_readfirstlane(wn);
  if constexpr (RS) {
    const int tn = cur.n0 / C::BN;
    const bool want = p.dbias_tab[cur.b0] != nullptr;
    uint32_t own = 0;
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
      if (want && i % C::WN == wnu && (i / C::WN) % p.tiles_n == tn) own |= 1u << i;
    rsum.own = own;
#pragma unroll
    for (int v = 0; v < RSumT::NV; ++v) rsum.v[v] = 0.f;
  }

  if constexpr (C::S == 2) {
    // prefetch one tile, two barriers per tile
    if (nfull > 0) issue_ktile<T, AK, BK, C>(p, smem, cur, 0, 0);
    for (int kt = 0; kt < nfull; ++kt) {
      if (kt + 1 < nfull) {
        issue_ktile<T, AK, BK, C>(p, smem, cur, kt + 1, (kt + 1) & 1);
        // tile kt landed (one newer tile in flight)
        const int wu = __builtin_amdgcn_readfirstlane(wid);
        wait_vm(dma_count<C::BM * C::KB / 1024, NWV>(wu) + dma_count<C::BN * C::KB / 1024, NWV>(wu));
      } else {
        wait_vm(0);
      }
      __builtin_amdgcn_s_barrier();            // ... for every wave of the block
      if (kt == 0) trace_stamp(p, 1);
      const char* img = smem + (kt & 1) * C::STAGE;
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(img, img + IA, wm, wn, acc);
      if constexpr (RS) rowsum_tile<T, AK, C>(img, wm, wnu, rsum);
      __builtin_amdgcn_s_barrier();            // buffer (kt&1) free for tile kt+2
    }
  } else if constexpr (C::IL) {
    // S-1 tiles in flight, one barrier per tile; tile kt+S-1's DMA is issued in pieces between
    // the MFMA rows of tile kt (buffer (kt-1) % S: freed by this iteration's barrier)
    static_assert(C::S >= 3 && C::S <= 5, "interleaved staging needs 3-5 stages");
    static_assert(C::BM * C::KB / 1024 % NWV == 0 && C::BN * C::KB / 1024 % NWV == 0,
                  "an uneven LDS-DMA split needs the 2-stage pipeline");
    constexpr int NIA = C::BM * C::KB / 1024 / (C::NT / 64);
    constexpr int NIB = C::BN * C::KB / 1024 / (C::NT / 64);
    constexpr int NR = C::KB / 64 * C::TM;            // MFMA rows per K-tile
    uint32_t offa[NIA], offb[NIB];
    glds_offsets<T, AK, C::KB, C::BM, C::NT>(offa, p.lda, p.M, cur.m0);
    glds_offsets<T, BK, C::KB, C::BN, C::NT>(offb, p.ldb, p.N, cur.n0);
    auto bases = [&](int kt, const char*& sa, const char*& sb) {
      const int k0 = cur.kbeg + kt * BKE;
      int ka, kb;
      const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, cur.b0, cur.b1, p.a_kseg, k0,
                                   ka);
      const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, cur.b0, cur.b1, p.b_kseg, k0,
                                   kb);
      sa = (const char*)(AK ? A + ka : A + (int64_t)ka * p.lda);
      sb = (const char*)(BK ? B + kb : B + (int64_t)kb * p.ldb);
    };
#pragma unroll
    for (int t = 0; t < C::S - 1; ++t)
      if (t < nfull) {
        const char *sa, *sb;
        bases(t, sa, sb);
        char* img = smem + t * C::STAGE;
#pragma unroll
        for (int i = 0; i < NIA; ++i) glds_slot<NIA>(img, sa, offa, i);
#pragma unroll
        for (int i = 0; i < NIB; ++i) glds_slot<NIB>(img + IA, sb, offb, i);
      }
    for (int kt = 0; kt < nfull; ++kt) {
      wait_tiles<VMT>(min(C::S - 2, nfull - 1 - kt));
      __builtin_amdgcn_s_barrier();
      const int tn = kt + C::S - 1;
      const char *sa = nullptr, *sb = nullptr;
      char* nimg = smem + (tn % C::S) * C::STAGE;
      if (tn < nfull) bases(tn, sa, sb);
      const bool go = tn < nfull;
      // piece q of the NIA + NIB instructions goes before MFMA row q * NR / (NIA + NIB)
      auto issue = [&](int row) {
        if (!go) return;
#pragma unroll
        for (int q = 0; q < NIA + NIB; ++q) {
          if (row == q * NR / (NIA + NIB)) {
            if (q < NIA) glds_slot<NIA>(nimg, sa, offa, q);
            else glds_slot<NIB>(nimg + IA, sb, offb, q - NIA);
          }
        }
      };
      const char* img = smem + (kt % C::S) * C::STAGE;
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(img, img + IA, wm, wn, acc, issue);
      else issue(0);
      if constexpr (RS) rowsum_tile<T, AK, C>(img, wm, wnu, rsum);
    }
  } else {
    // S-1 tiles in flight, one barrier per tile: the barrier of iteration kt also certifies that
    // every wave finished computing tile kt-1, whose buffer receives tile kt+S-1.
    static_assert(C::S <= 9 && (C::S - 2) * VMT < 64, "wait_tiles covers up to 7 newer tiles");
    static_assert(C::BM * C::KB / 1024 % NWV == 0 && C::BN * C::KB / 1024 % NWV == 0,
                  "an uneven LDS-DMA split needs the 2-stage pipeline");
#pragma unroll
    for (int i = 0; i < C::S - 1; ++i)
      if (i < nfull) issue_ktile<T, AK, BK, C>(p, smem, cur, i, i);
    for (int kt = 0; kt < nfull; ++kt) {
      wait_tiles<VMT>(min(C::S - 2, nfull - 1 - kt));
      __builtin_amdgcn_s_barrier();
      if (kt + C::S - 1 < nfull)
        issue_ktile<T, AK, BK, C>(p, smem, cur, kt + C::S - 1, (kt + C::S - 1) % C::S);
      const char* img = smem + (kt % C::S) * C::STAGE;
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(img, img + IA, wm, wn, acc);
      if constexpr (RS) rowsum_tile<T, AK, C>(img, wm, wnu, rsum);
    }
  }
  if (tail) {   // trailing partial K-tile: masked register staging
    const int k0 = cur.kbeg + nfull * BKE;
    int ka, kb;
    const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, cur.b0, cur.b1, p.a_kseg, k0,
                                 ka);
    const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, cur.b0, cur.b1, p.b_kseg, k0,
                                 kb);
    const int ka_lim = (p.a_mode == 2) ? min(p.a_kseg, ka + (cur.kend - k0)) : cur.kend;
    const int kb_lim = (p.b_mode == 2) ? min(p.b_kseg, kb + (cur.kend - k0)) : cur.kend;
    char* base = smem + (nfull % C::S) * C::STAGE;
    stage_tile<T, AK, C::KB, C::BM, C::NT>(base, A, p.lda, p.M, cur.m0, ka_lim, ka);
    stage_tile<T, BK, C::KB, C::BN, C::NT>(base + IA, B, p.ldb, p.N, cur.n0, kb_lim, kb);
    __syncthreads();
    if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(base, base + IA, wm, wn, acc);
    if constexpr (RS) rowsum_tile<T, AK, C>(base, wm, wnu, rsum);
  }
  __syncthreads();
  trace_stamp(p, 2);
  gemm_epilogue<T, O, C>(p, cur, acc, lane, wm, wn);
  if constexpr (RS) rowsum_store<C>(p, cur, rsum, lane, wm);
  trace_stamp(p, 3);
}

// split-K reduction + epilogue.  Vector form (N % 4 == 0, C 4-element aligned): one thread per 4
// consecutive outputs, float4 slab loads; otherwise one thread per output element.
template <typename O, bool V4>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  constexpr int W = V4 ? 4 : 1;
  const int nb = p.batch0 * p.batch1;
  const int64_t per = (int64_t)p.M * p.N;
  const int64_t total = per * nb / W;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = e * W;
    const int b = (int)(idx / per);
    const int64_t mn = idx - (int64_t)b * per;
    const int m = (int)(mn / p.N), n = (int)(mn - (int64_t)m * p.N);
    float v[W];
#pragma unroll
    for (int i = 0; i < W; ++i) v[i] = 0.f;
    const int64_t sstride = (int64_t)nb * per;
    const float* src0 = p.ws + (int64_t)b * per + mn;
    int s = 0;
    if constexpr (V4) {
      // four slab loads in flight per step, summed in split order (the same order, and so the
      // same bits, as one at a time)
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
      if constexpr (V4) {
        const float4 t = *(const float4*)src;
        v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
      } else {
        v[0] += *src;
      }
    }
    const int b0 = b / p.batch1, b1 = b % p.batch1;
    if (p.n_dbias > 0 && n == 0 && p.dbias_tab[b0]) {   // the A row sums' split partials
      const float* src = p.dbias_ws + (int64_t)b * p.M + m;
      float r = 0.f;
      for (int t = 0; t < p.splits; ++t) r += src[(int64_t)t * nb * p.M];
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
    if constexpr (V4) {
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
    if constexpr (V4) {
      if constexpr (sizeof(O) == 4) *(float4*)(cp + co) = *(const float4*)out;
      else *(uint2*)(cp + co) = *(const uint2*)out;
    } else {
      cp[co] = out[0];
    }
  }
}

// ------------------------------------------------------------------ launch
template <typename T, typename O, bool AK, bool BK, class C, bool RS = false>
static void launch_cfg(const GemmParams& p, dim3 grid, hipStream_t st) {
  auto fn = gemm_kernel<T, O, AK, BK, C, RS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              C::LDS);
    attr = true;
  }
  hipLaunchKernelGGL(fn, grid, dim3(C::NT), (size_t)C::LDS, st, p);
}

template <typename T, typename O, bool AK, bool BK, bool RS = false>
static void launch_layout(const GemmParams& p, int cfg, dim3 grid, hipStream_t st) {
  switch (cfg) {
    case 5: launch_cfg<T, O, AK, BK, Cfg5, RS>(p, grid, st); break;
    case 30: if constexpr (AK) { launch_cfg<T, O, AK, BK, Cfg30, RS>(p, grid, st); break; }
             [[fallthrough]];
    case 10: if constexpr (sizeof(T) == 2) { launch_cfg<T, O, AK, BK, Cfg10, RS>(p, grid, st); break; }
             [[fallthrough]];
    case 11: if constexpr (sizeof(T) == 2) { launch_cfg<T, O, AK, BK, Cfg11, RS>(p, grid, st); break; }
             [[fallthrough]];
    case 20: if constexpr (sizeof(T) == 2) { launch_cfg<T, O, AK, BK, Cfg20, RS>(p, grid, st); break; }
             [[fallthrough]];
    case 21: if constexpr (sizeof(T) == 2) { launch_cfg<T, O, AK, BK, Cfg21, RS>(p, grid, st); break; }
             [[fallthrough]];
    default: launch_cfg<T, O, AK, BK, Cfg1, RS>(p, grid, st); break;
  }
}

template <typename T, typename O>
static void launch_to(const GemmParams& p, int ak, int bk, int cfg, dim3 grid, hipStream_t st) {
  if (ak && bk) launch_layout<T, O, true, true>(p, cfg, grid, st);
  else if (ak && !bk) launch_layout<T, O, true, false>(p, cfg, grid, st);
  else if (!ak && bk) launch_layout<T, O, false, true>(p, cfg, grid, st);
  else if constexpr (sizeof(T) == 2 && sizeof(O) == 4) {
    // weight gradients (fp32 out): A row sums only on this layout (jmt_gemm checks)
    if (p.n_dbias > 0) launch_layout<T, O, false, false, true>(p, cfg, grid, st);
    else launch_layout<T, O, false, false>(p, cfg, grid, st);
  } else {
    launch_layout<T, O, false, false>(p, cfg, grid, st);
  }
}

template <typename T>
static void launch_t(const GemmParams& p, int ak, int bk, int cfg, dim3 grid, hipStream_t st) {
  if (p.splits > 1 || p.c_dtype == JMT_F32) launch_to<T, float>(p, ak, bk, cfg, grid, st);
  else launch_to<T, T>(p, ak, bk, cfg, grid, st);
}

static void cfg_tile(int cfg, int& bm, int& bn) {
  switch (cfg) {
    case 5: case 20: bm = 256; bn = 256; break;
    case 30: bm = 160; bn = 256; break;
    default: bm = 128; bn = 128; break;
  }
}

// ------------------------------------------------------------------ planner
// Cost model fitted to the gfx950 microbenchmarks (scripts/bench_gemm.py, profiles/r01_*):
//   t(cfg, splits) = ceil(blocks / resident slots) * (tile FLOPs / per-block rate + overhead)
//                  + split-K reduce (fp32 slabs read once, output written once) when splits > 1
// 128x128 runs 2 blocks / CU (512 slots) at ~1.9 TFLOP/s each; 256x256 runs 1 block / CU at
// ~4.2 TFLOP/s (half the LDS traffic per FLOP) but quantises 4x coarser.  Waves are counted
// whole: the tail wave of a launch costs a full wave.
struct TileModel { int id, bm, bn, slots; double mflop_per_us, ovh_us; };
static const TileModel kModels16[] = {{1, 128, 128, 512, 1.91, 7.0},
                                      {5, 256, 256, 256, 4.2, 13.0}};
static const TileModel kModels32[] = {{1, 128, 128, 512, 0.5, 7.0}};

static double model_cost(const TileModel& t, int M, int N, int K, int batch, int splits, int bke) {
  const long tiles = (long)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn) * batch;
  int kps = ((K + splits - 1) / splits + bke - 1) / bke * bke;
  if (kps < bke) kps = bke;
  const long blocks = tiles * splits;
  const long waves = (blocks + t.slots - 1) / t.slots;
  const double tile_mflop = 2.0 * t.bm * t.bn * (double)kps / 1e6;
  double c = waves * (tile_mflop / t.mflop_per_us + t.ovh_us);
  if (splits > 1) c += ((double)splits + 1.0) * M * N * batch * 4.0 / 3.5e6 + 4.0;
  return c;
}

// Padding guard: the 256x256 tile is only considered when it wastes < 10% of its MACs.
static bool tile_ok(const TileModel& t, int M, int N) {
  const double pad = (double)((M + t.bm - 1) / t.bm * t.bm) * ((N + t.bn - 1) / t.bn * t.bn);
  return t.bm == 128 || (double)M * N >= 0.9 * pad;
}

// Launch families where a 128x128 tile at 3-4 resident blocks / CU (Cfg10 / Cfg11) beat the
// planner's choice by 3-11% in repeated step-shape sweeps (profiles/r01_gemm_occupancy.txt);
// elsewhere they tie or lose, so they are selected by layout and shape, not by the cost model.
// Round 2 (profiles/r02_gemm_step_shapes.txt, one process, cfg 0 / 5 / 20 / 21 interleaved):
// the grouped NN dgrads run fastest on the interleaved-DMA 256x256 tile (Cfg20: -2..-18 %), the
// grouped NT forwards on the plain 256x256 tile (-2..-7 % vs the round-1 128x128 overrides).
static int occupancy_override(int ak, int bk, int M, int N, int K, int batch, int splits) {
  // round 3: the 160x256 tile on the single (un-batched) B*T-row GEMMs — the 19,200-row output
  // of N <= 1024 is 240 / 480 tiles instead of 150 / 300 of 256x256 (0.94 / 1.88 waves on 256
  // CUs instead of 0.59 / 1.17): video linear fwd 69 -> 54 us, FcLayer fwd 42 -> 33, head dgrad
  // 45 -> 36, K-concat stream dgrad 94 -> 84 (was Cfg11); and the grouped qkv forward (b3,
  // N = 1536) 167 -> 161.  Batched N = 512 / 1024 launches stay on 256x256 (cfg 30 lost 6-15 %
  // there: 1.76 / 3.5 waves already quantise well).  profiles/r03_gemm_tile160.jsonl
  // These B*T-row overrides were measured at c3's 19,200 rows; at c2's 9,600 the planner's own
  // tile is faster (video linear fwd 51.5 -> 35.8 us, FcLayer fwd 30.5 -> 23.6, head dgrad 30.8
  // -> 24.5, K-concat stream dgrad 80.1 -> 66.7, qkv fwd b3 97.2 -> 77.1, qkv wgrad b3 101 ->
  // 81: profiles/r03_c2_gemm_tiles.jsonl), so they are keyed to >= 16,384 rows.
  if (splits <= 1 && ak && M >= 16384 && K >= 512 && K % 64 == 0 &&
      ((batch == 1 && N <= 1024) || (bk && batch == 3 && N == 1536 && K == 512)))
    return 30;
  // the stacked-stream dgrad of out_layer_pv (b2, beta = 1): 65 -> 57 us (1.17 waves of 256x256
  // tiles, 1.88 of 160x256; profiles/r03_nn_sweep.jsonl)
  if (splits <= 1 && ak && !bk && batch == 2 && M >= 4096 && N == 512 && K == 512) return 30;
  if (!ak && !bk && M >= 1536 && N >= 512 && batch >= 3 && K >= 16384)
    return 10;                                                   // split-K qkv wgrad
  if (!ak && !bk && batch == 6 && M == 1024 && N == 512 && K >= 8192)
    return 5;          // cross-attention k|v wgrad: 256x256 at the planner's splits (-8 %,
                       // profiles/r02_wgrad_splits_b6.jsonl)
  if (splits > 1) return 0;
  if (!ak && !bk && batch >= 64 && M <= 512 && N <= 512 && K >= 128 && K <= 512)
    return 11;                                                   // attn dK / dV
  if (ak && !bk && batch == 1 && K >= 3072 && M >= 16384) return 11;   // K-concat stream dgrad
  if (ak && !bk && batch == 1 && K <= 128 && M >= 4096 && N >= 512)
    return 11;         // short-K dgrad (the regressors' first layer, K = 128): 28.7 -> 23.3 us,
                       // profiles/r02_regressor_gemm_sweep.jsonl
  if (ak && !bk && batch >= 3 && batch <= 8 && K >= 512 && M >= 4096 && N >= 512)
    return 20;                                                   // grouped / head dgrads
  if (ak && bk && batch >= 3 && K == 512 && M >= 4096 && N >= 512) return 5;   // grouped fwd
  return 0;
}

static void plan(int dt, int M, int N, int K, int batch, int fixed_splits, int& cfg, int& splits) {
  const int bke = 128 / dtype_size(dt);
  const TileModel* ms = dt == JMT_F32 ? kModels32 : kModels16;
  const int nm = dt == JMT_F32 ? 1 : 2;
  double best = 1e300;
  cfg = 1;
  splits = fixed_splits > 0 ? fixed_splits : 1;
  for (int i = 0; i < nm; ++i) {
    if (!tile_ok(ms[i], M, N)) continue;
    // a handful of output tiles over a long K (the V / A regressors' 1 x 128 weight gradient over
    // all B*T rows): up to 256 splits, so the launch still covers the chip
    const long tiles = (long)((M + ms[i].bm - 1) / ms[i].bm) * ((N + ms[i].bn - 1) / ms[i].bn) *
                       batch;
    int s_lo = 1, s_hi = tiles <= 8 ? 256 : 32;
    if (fixed_splits > 0) s_lo = s_hi = fixed_splits;
    for (int s = s_lo; s <= s_hi; ++s) {
      if (fixed_splits <= 0 && s > 1 && K / s < 4 * bke) break;   // >= 4 K-tiles per split
      const double c = model_cost(ms[i], M, N, K, batch, s, bke);
      if (c < best * 0.999) { best = c; cfg = ms[i].id; splits = s; }
    }
  }
}

}  // namespace jmt

using namespace jmt;

static int g_gemm_dbg = 0;
static int g_gemm_cfg = 0;
extern "C" int jmt_gemm_trace_read(uint64_t* host, int nblocks) {
  if (nblocks > kTraceBlocks) nblocks = kTraceBlocks;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_trace), sizeof(uint64_t) * 4 * nblocks) !=
          hipSuccess)
    return -1;
  return nblocks;
}
extern "C" void jmt_gemm_set_debug(int flags) { g_gemm_dbg = flags & 0xff; g_gemm_cfg = flags >> 8; }

extern "C" int jmt_gemm_plan_splits(int ab_dtype, int M, int N, int K, int batch) {
  if (M <= 0 || N <= 0 || K <= 0) return 1;
  if (ab_dtype != JMT_F32 && ab_dtype != JMT_BF16 && ab_dtype != JMT_F16) return 1;
  int cfg, splits;
  plan(ab_dtype, M, N, K, batch < 1 ? 1 : batch, 0, cfg, splits);
  return splits;
}

extern "C" size_t jmt_gemm_workspace_bytes(int M, int N, int batch, int splits) {
  if (splits <= 1) return 0;
  return (size_t)splits * (size_t)batch * (size_t)M * (size_t)N * sizeof(float);
}

extern "C" int jmt_gemm(const jmt_gemm_desc* d, void* stream) {
  JMT_CHECK_ARG(d != nullptr, "jmt_gemm: null descriptor");
  const int dt = d->ab_dtype;
  JMT_CHECK_ARG(dt == JMT_F32 || dt == JMT_BF16 || dt == JMT_F16, "jmt_gemm: bad ab_dtype %d", dt);
  JMT_CHECK_ARG(d->c_dtype == JMT_F32 || d->c_dtype == dt, "jmt_gemm: c_dtype must be f32 or ab");
  JMT_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "jmt_gemm: negative size");
  JMT_CHECK_ARG(d->aux == nullptr || d->aux_dtype == d->c_dtype,
                "jmt_gemm: aux (ReLU mask) must have the output dtype");
  if (d->M == 0 || d->N == 0) return JMT_OK;
  const int batch0 = d->batch0 < 1 ? 1 : d->batch0;
  const int batch1 = d->batch1 < 1 ? 1 : d->batch1;
  JMT_CHECK_ARG(batch0 * batch1 <= 65535, "jmt_gemm: batch too large");
  const int es = dtype_size(dt);
  const int V = 16 / es;
  const int BKE = 128 / es;     // K elements per K-tile (all configs use 128-B tile rows)
  JMT_CHECK_ARG(d->n_a >= 1 && d->n_a <= MAXP && d->n_b >= 1 && d->n_b <= MAXP &&
                    d->n_c >= 1 && d->n_c <= MAXP, "jmt_gemm: pointer table size");
  JMT_CHECK_ARG(d->lda % V == 0 && d->ldb % V == 0, "jmt_gemm: lda/ldb must be multiples of %d", V);
  JMT_CHECK_ARG((d->sA0 % V == 0) && (d->sA1 % V == 0) && (d->sB0 % V == 0) && (d->sB1 % V == 0),
                "jmt_gemm: batch strides must be multiples of %d elements", V);
  for (int i = 0; i < d->n_a; ++i)
    JMT_CHECK_ARG(((uintptr_t)d->a[i] & 15) == 0, "jmt_gemm: A[%d] not 16-B aligned", i);
  for (int i = 0; i < d->n_b; ++i)
    JMT_CHECK_ARG(((uintptr_t)d->b[i] & 15) == 0, "jmt_gemm: B[%d] not 16-B aligned", i);
  if (d->a_mode == 2) JMT_CHECK_ARG(d->a_kseg % BKE == 0 && d->a_kseg * d->n_a >= d->K,
                                    "jmt_gemm: A K-concat segment must be a multiple of %d", BKE);
  if (d->b_mode == 2) JMT_CHECK_ARG(d->b_kseg % BKE == 0 && d->b_kseg * d->n_b >= d->K,
                                    "jmt_gemm: B K-concat segment must be a multiple of %d", BKE);
  if (d->a_mode == 1) JMT_CHECK_ARG(d->n_a >= batch0, "jmt_gemm: A pointer table < batch0");
  if (d->b_mode == 1) JMT_CHECK_ARG(d->n_b >= batch0, "jmt_gemm: B pointer table < batch0");
  if (d->c_mode == 1) JMT_CHECK_ARG(d->n_c >= batch0, "jmt_gemm: C pointer table < batch0");

  GemmParams p;
  for (int i = 0; i < MAXP; ++i) {
    p.a_ptr[i] = i < d->n_a ? d->a[i] : nullptr;
    p.b_ptr[i] = i < d->n_b ? d->b[i] : nullptr;
    p.c_ptr[i] = i < d->n_c ? d->c[i] : nullptr;
  }
  JMT_CHECK_ARG(d->n_bias >= 0 && d->n_bias <= MAXP, "jmt_gemm: bias table size");
  if (d->n_bias > 0)
    JMT_CHECK_ARG(d->n_bias >= batch0 && d->bias_mode != 0, "jmt_gemm: bias table < batch0");
  p.bias = d->bias;
  p.n_bias = d->n_bias;
  for (int i = 0; i < MAXP; ++i) p.bias_tab[i] = i < d->n_bias ? d->bias_tab[i] : nullptr;
  p.aux = d->aux;
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldaux = d->ldaux;
  p.sA0 = d->sA0; p.sA1 = d->sA1; p.sB0 = d->sB0; p.sB1 = d->sB1; p.sC0 = d->sC0; p.sC1 = d->sC1;
  p.a_mode = d->a_mode; p.b_mode = d->b_mode; p.c_mode = d->c_mode;
  p.a_kseg = d->a_mode == 2 ? d->a_kseg : 0;
  p.b_kseg = d->b_mode == 2 ? d->b_kseg : 0;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.batch0 = batch0; p.batch1 = batch1;
  p.alpha = d->alpha; p.beta = d->beta;
  p.bias_mode = (d->bias || d->n_bias > 0) ? d->bias_mode : 0;
  p.relu = d->relu;
  p.c_dtype = d->c_dtype;
  p.aux_dtype = d->aux_dtype;
  p.dbg = g_gemm_dbg;
  JMT_CHECK_ARG(d->n_dbias >= 0 && d->n_dbias <= MAXP, "jmt_gemm: dbias table size");
  p.n_dbias = d->n_dbias;
  p.dbias_acc = d->dbias_acc;
  p.dbias_ws = d->dbias_ws;
  for (int i = 0; i < MAXP; ++i) p.dbias_tab[i] = i < d->n_dbias ? d->dbias_tab[i] : nullptr;
  if (d->n_dbias > 0) {
    JMT_CHECK_ARG(dt != JMT_F32 && d->c_dtype == JMT_F32 && !d->a_kmajor && !d->b_kmajor &&
                      batch1 == 1 && d->n_dbias >= batch0,
                  "jmt_gemm: A row sums need 16-bit MN-major A and B, fp32 C, batch1 = 1 and a "
                  "dbias table of batch0 entries");
    bool any = false;   // null entries: no row sums for that batch entry (a K-concatenated
    for (int i = 0; i < batch0; ++i) any = any || d->dbias_tab[i] != nullptr;   // wgrad's segments
    JMT_CHECK_ARG(any, "jmt_gemm: every dbias_tab entry is null");
  }
  {
    const int ces = dtype_size(d->c_dtype);
    bool cv4 = d->ldc % 4 == 0 && d->sC0 % 4 == 0 && d->sC1 % 4 == 0;
    for (int i = 0; i < d->n_c; ++i) cv4 = cv4 && (((uintptr_t)d->c[i] & (4 * ces - 1)) == 0);
    if (d->aux) cv4 = cv4 && (((uintptr_t)d->aux & (4 * ces - 1)) == 0) && d->ldaux % 4 == 0;
    p.c_vec4 = cv4 ? 1 : 0;
    bool cv8 = cv4 && d->ldc % 8 == 0 && d->sC0 % 8 == 0 && d->sC1 % 8 == 0;
    for (int i = 0; i < d->n_c; ++i) cv8 = cv8 && (((uintptr_t)d->c[i] & 15) == 0);
    p.c_vec8 = cv8 ? 1 : 0;
  }

  int splits = d->splits < 1 ? 1 : d->splits;
  // each split owns whole K-tiles, so a K-concat segment boundary never cuts a tile
  int kps = ((d->K + splits - 1) / splits + BKE - 1) / BKE * BKE;
  if (kps < BKE) kps = BKE;
  splits = (d->K + kps - 1) / kps;
  if (splits < 1) splits = 1;
  p.splits = splits;
  p.k_per_split = splits > 1 ? kps : (d->K > 0 ? d->K : 1);
  p.ws = (float*)d->workspace;
  if (splits > 1) {
    const size_t need = jmt_gemm_workspace_bytes(d->M, d->N, batch0 * batch1, splits);
    JMT_CHECK_ARG(d->workspace != nullptr && d->ws_bytes >= need,
                  "jmt_gemm: split-K needs %zu workspace bytes", need);
    if (d->n_dbias > 0) {
      const size_t dneed = (size_t)splits * batch0 * (size_t)d->M * sizeof(float);
      JMT_CHECK_ARG(d->dbias_ws != nullptr && d->dbias_ws_bytes >= dneed,
                    "jmt_gemm: split-K A row sums need %zu dbias_ws bytes", dneed);
    }
  }
  int cfg = g_gemm_cfg;
  if (dt == JMT_F32 && cfg >= 10) cfg = 1;   // occupancy configs: 16-bit only
  if (cfg == 30 && !d->a_kmajor) cfg = 5;    // 160-row tile: K-major A only
  if (!cfg) {
    int s_unused;
    plan(dt, d->M, d->N, d->K, batch0 * batch1, splits, cfg, s_unused);
    if (dt != JMT_F32 && (cfg == 1 || splits == 1)) {   // same 128x128 split plan when split
      // (an override may pick a 256x256 tile: 5 or 20)
      const int t = occupancy_override(d->a_kmajor, d->b_kmajor, d->M, d->N, d->K,
                                       batch0 * batch1, splits);
      if (t) cfg = t;
    }
  }
  // A row sums: the 4-block 128x128 tile (128 VGPRs) spills with the extra per-lane sums; the
  // 256x256 tile does not and runs the split-K qkv / FFN wgrad shapes at least as fast
  // (profiles/r03_wgrad_dbias.jsonl)
  if (d->n_dbias > 0 && cfg == 10) cfg = 5;
  int bm, bn;
  cfg_tile(cfg, bm, bn);
  p.tiles_m = (d->M + bm - 1) / bm;
  p.tiles_n = (d->N + bn - 1) / bn;
  hipStream_t st = as_stream(stream);
  dim3 grid(p.tiles_m * p.tiles_n, batch0 * batch1, splits);
  if (dt == JMT_F32) launch_t<float>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  else if (dt == JMT_BF16) launch_t<__bf16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  else launch_t<_Float16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  JMT_LAUNCH_CHECK("jmt_gemm");
  if (splits > 1) {
    const bool v4 = d->N % 4 == 0 && p.c_vec4;
    const int64_t total = (int64_t)d->M * d->N * batch0 * batch1 / (v4 ? 4 : 1);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
#define JMT_SKR(O)                                                                          \
    if (v4) hipLaunchKernelGGL((splitk_reduce_kernel<O, true>), dim3(blocks), dim3(256), 0, st, p); \
    else hipLaunchKernelGGL((splitk_reduce_kernel<O, false>), dim3(blocks), dim3(256), 0, st, p);
    if (d->c_dtype == JMT_F32) { JMT_SKR(float) }
    else if (d->c_dtype == JMT_BF16) { JMT_SKR(__bf16) }
    else { JMT_SKR(_Float16) }
#undef JMT_SKR
    JMT_LAUNCH_CHECK("jmt_gemm(splitk_reduce)");
  }
  return JMT_OK;
}
