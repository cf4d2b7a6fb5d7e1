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
#include "gemm_tile.h"

namespace jmt {

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
    // an uneven DMA split (the 160-row tile) deals a K-tile's instructions round-robin, so a
    // wave's own count per K-tile depends on the wave: its waits count exactly those
    constexpr bool EVEN = C::BM * C::KB / 1024 % NWV == 0 && C::BN * C::KB / 1024 % NWV == 0;
    static_assert(EVEN || (C::S - 2) * VMT <= 16, "wait_vm covers up to 16");
    const int cw = dma_count<C::BM * C::KB / 1024, NWV>(__builtin_amdgcn_readfirstlane(wid)) +
                   dma_count<C::BN * C::KB / 1024, NWV>(__builtin_amdgcn_readfirstlane(wid));
#pragma unroll
    for (int i = 0; i < C::S - 1; ++i)
      if (i < nfull) issue_ktile<T, AK, BK, C>(p, smem, cur, i, i);
    for (int kt = 0; kt < nfull; ++kt) {
      if constexpr (EVEN) wait_tiles<VMT>(min(C::S - 2, nfull - 1 - kt));
      else wait_vm(min(C::S - 2, nfull - 1 - kt) * cw);
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
    const int ka_lim = (p.a_mode >= 2) ? min(p.a_kseg, ka + (cur.kend - k0)) : cur.kend;
    const int kb_lim = (p.b_mode >= 2) ? min(p.b_kseg, kb + (cur.kend - k0)) : cur.kend;
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

// (split-K reduced inside the GEMM launch by each tile's last-arriving split block — agent-scope
// release / acquire on a per-tile counter, bit-identical to the separate launch — measured slower:
// every tile of a weight gradient finishes in the last wave, so the fused reductions ran on one
// CU per tile at the end of the launch, TN b3 512x512x19200 58 -> 93 us, the step 4.65 -> 5.43 ms;
// profiles/r04/splitk_fused_ab.txt.  Removed in round 5.)

// split-K reduction + epilogue.  Vector form (N % 4 == 0, C 4-element aligned): one thread per 4
// consecutive outputs, float4 slab loads; otherwise one thread per output element.
template <typename O, bool V4>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  constexpr int W = V4 ? 4 : 1;
  const int64_t per = (int64_t)p.M * p.N;
  const int64_t total = per * p.batch0 * p.batch1 / W;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = e * W;
    const int b = (int)(idx / per);
    const int64_t mn = idx - (int64_t)b * per;
    const int m = (int)(mn / p.N), n = (int)(mn - (int64_t)m * p.N);
    reduce_outputs<O, W>(p, b, m, n);
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
    case 32: if constexpr (AK && sizeof(T) == 2) { launch_cfg<T, O, AK, BK, Cfg32, RS>(p, grid, st); break; }
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
    case 32: bm = 160; bn = 256; break;
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
    return 32;
  // the stacked-stream dgrad of out_layer_pv (b2, beta = 1): 65 -> 57 us (1.17 waves of 256x256
  // tiles, 1.88 of 160x256; profiles/r03_nn_sweep.jsonl)
  if (splits <= 1 && ak && !bk && batch == 2 && M >= 4096 && N == 512 && K == 512) return 32;
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

static int pp_split_env() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JMT_GEMM_PPSPLIT");
    v = e ? atoi(e) : 1;
  }
  return v;
}

static void plan(int dt, int M, int N, int K, int batch, int fixed_splits, int& cfg, int& splits) {
  const int bke = 128 / dtype_size(dt);
  // few 256 x 256 tiles over a long K (the weight gradients): the split-K ping-pong kernel,
  // one (tile, split) item per CU (gemm_persist.hip cfg 44)
  if (fixed_splits <= 0 && pp_split_env()) {
    const int s = pp_split_plan(dt, M, N, K, batch);
    if (s) {
      cfg = 44;
      splits = s;
      return;
    }
  }
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

// split-K workspace: the fp32 partial slabs
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
  JMT_CHECK_ARG(d->a_mode >= 0 && d->a_mode <= 3 && d->b_mode >= 0 && d->b_mode <= 3 &&
                    d->c_mode >= 0 && d->c_mode <= 1, "jmt_gemm: bad operand mode");
  if (d->a_mode == 2) JMT_CHECK_ARG(d->a_kseg % BKE == 0 && d->a_kseg * d->n_a >= d->K,
                                    "jmt_gemm: A K-concat segment must be a multiple of %d", BKE);
  if (d->b_mode == 2) JMT_CHECK_ARG(d->b_kseg % BKE == 0 && d->b_kseg * d->n_b >= d->K,
                                    "jmt_gemm: B K-concat segment must be a multiple of %d", BKE);
  // mode 3 (ABI 7): K-concat per batch entry, segment i of entry b0 at base[b0 * nseg + i]
  const int nseg_a = d->a_mode == 3 && d->a_kseg > 0 ? (d->K + d->a_kseg - 1) / d->a_kseg : 1;
  const int nseg_b = d->b_mode == 3 && d->b_kseg > 0 ? (d->K + d->b_kseg - 1) / d->b_kseg : 1;
  if (d->a_mode == 3) JMT_CHECK_ARG(d->a_kseg > 0 && d->a_kseg % BKE == 0 &&
                                        d->n_a >= batch0 * nseg_a && d->batch1 <= 1,
                                    "jmt_gemm: A per-batch K-concat needs kseg a multiple of %d, "
                                    "batch0 x ceil(K / kseg) pointers and batch1 = 1", BKE);
  if (d->b_mode == 3) JMT_CHECK_ARG(d->b_kseg > 0 && d->b_kseg % BKE == 0 &&
                                        d->n_b >= batch0 * nseg_b && d->batch1 <= 1,
                                    "jmt_gemm: B per-batch K-concat needs kseg a multiple of %d, "
                                    "batch0 x ceil(K / kseg) pointers and batch1 = 1", BKE);
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
  p.a_kseg = d->a_mode >= 2 ? d->a_kseg : 0;
  p.b_kseg = d->b_mode >= 2 ? d->b_kseg : 0;
  if (d->a_mode == 3) p.sA0 = nseg_a;                 // operand_base: segments per entry
  if (d->b_mode == 3) p.sB0 = nseg_b;
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
  // persistent path (gemm_persist.hip: eligibility and the default choice live there)
  {
    const int pc = persist_choice(d, p, splits, cfg);
    if (pc) {
      p.tiles_m = (d->M + 255) / 256;                 // cfg 45: the last row panel may be partial
      p.tiles_n = d->N / 256;
      const int W = p.tiles_m * p.tiles_n * batch0 * batch1;
      const int ncu = num_cus_persist();
      const int blocks = W < ncu ? W : ncu;
      launch_gemm_persist(p, dt, d->a_kmajor, d->b_kmajor, pc, blocks, as_stream(stream));
      JMT_LAUNCH_CHECK("jmt_gemm(persistent)");
      return JMT_OK;
    }
  }
  // split-K ping-pong (cfg 44): forced, or where the planner's split count came from it
  const bool pp_split = splits > 1 && pp_split_ok(dt, d->M, d->N, d->K, splits) &&
                        (cfg == 44 || (cfg == 0 && pp_split_env() &&
                                       pp_split_plan(dt, d->M, d->N, d->K, batch0 * batch1)));
  if (cfg == 44) cfg = 0;
  if (cfg == 40 || cfg == 43 || cfg == 45) cfg = 5;   // persistent configs not applicable
  if (dt == JMT_F32 && cfg >= 10) cfg = 1;   // occupancy / 160-row configs: 16-bit only
  if (cfg == 32 && !d->a_kmajor) cfg = 5;    // 160-row tile: K-major A only
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
  hipStream_t st = as_stream(stream);
  if (pp_split) {
    p.tiles_m = d->M / 256;
    p.tiles_n = d->N / 256;
    const int W = p.tiles_m * p.tiles_n * batch0 * batch1 * splits;
    const int ncu = num_cus_persist();
    launch_gemm_pp_split(p, dt, d->a_kmajor, d->b_kmajor, d->n_dbias > 0, W < ncu ? W : ncu, st);
    JMT_LAUNCH_CHECK("jmt_gemm(split-K ping-pong)");
  } else {
    int bm, bn;
    cfg_tile(cfg, bm, bn);
    p.tiles_m = (d->M + bm - 1) / bm;
    p.tiles_n = (d->N + bn - 1) / bn;
    dim3 grid(p.tiles_m * p.tiles_n, batch0 * batch1, splits);
    if (dt == JMT_F32) launch_t<float>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
    else if (dt == JMT_BF16) launch_t<__bf16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
    else launch_t<_Float16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
    JMT_LAUNCH_CHECK("jmt_gemm");
  }
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
