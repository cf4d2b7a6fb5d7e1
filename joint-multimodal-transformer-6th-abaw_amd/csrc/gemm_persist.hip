// Persistent form of the GEMM (jmt_gemm cfg 40): one block per CU walks whole output
// tiles with one continuous LDS-DMA pipeline (details at gemm_persist_kernel).
#include "gemm_tile.h"

namespace jmt {

// ------------------------------------------------------------------ persistent kernel
// One block per CU walks a list of whole output tiles with ONE continuous LDS-DMA pipeline over
// the K-tiles of all its tiles: the first K-tiles of tile i+1 are in flight while the last
// K-tiles of tile i compute, and tile i's epilogue stores are issued BEHIND those prefetches, so
// they drain under tile i+1's MFMAs instead of as one chip-wide write burst between rounds of a
// one-block-per-tile grid (2.3 us first K-tile + 7.9 us store burst per 256x256
// tile at K = 512).  The same structure as hipBLASLt's stream-K kernels on these shapes (225
// persistent workgroups x 2 tiles for 19200x512x512 b3, profiles/r04/pmc_gemm_vs_hipblaslt.txt).
//
// s_waitcnt vmcnt counts loads, LDS-DMA and stores together in issue order, so the wait for
// K-tile s counts exactly the VMEM operations issued after its DMA: the DMA of the younger
// K-tiles already issued (VMT each) and, for the S - 1 K-tiles whose DMA went out before the
// last epilogue, that epilogue's NST stores.  Every count is exact because the persistent path
// only takes full tiles (straight-line epilogue: TM * TN / 2 16-B stores per wave, no loads —
// the bias comes from LDS, staged once per launch).
// Preconditions (jmt_gemm, persist_ok): 16-bit A, B and C, M % BM == N % BN == 0, K % BKE == 0,
// C rows 16-B aligned, no split-K, no row sums, bias per column (tables of at most kPersistBias
// floats in all); beta * C and the ReLU mask are compile-time epilogue forms (EPI).

// s_waitcnt vmcnt(VMT * k + (st ? NST : 0)) for wave-uniform 0 <= k <= K
template <int VMT, int NST, int K>
__device__ __forceinline__ void wait_young(int k, bool st) {
  if constexpr (K >= 0) {
    if (k == K) {
      if (st) wait_vmcnt<VMT * K + NST>();
      else wait_vmcnt<VMT * K>();
    } else {
      wait_young<VMT, NST, K - 1>(k, st);
    }
  }
}

struct PItem {
  int m0, n0, b0, b1;
  int sp, kt0, len;             // split-K: split index, its first K-tile (64 deep) and count
};

// work item w (block w % G, G a multiple of 8: the hardware deals blocks to the XCDs round-robin)
// -> a logical tile, bijectively: the items of one XCD are a contiguous range of logical tiles
// (n fastest), so the N tiles of one A row panel run at the same time on one XCD's L2.
__device__ __forceinline__ PItem pitem(const GemmParams& p, int w, int W) {
  const int ntile = p.tiles_m * p.tiles_n;
  const int x = w & 7, q = W >> 3, r = W & 7;
  const int L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (w >> 3);
  const int b = L / ntile, t = L - b * ntile;
  PItem it;
  it.m0 = (t / p.tiles_n) * 256;
  it.n0 = (t % p.tiles_n) * 256;
  it.b0 = b / p.batch1;
  it.b1 = b - it.b0 * p.batch1;
  return it;
}

// pitem for w, w + G, w + 2 G, ... without divisions per item: G is a multiple of 8, so w's XCD
// slot x is fixed and the logical tile index L advances by G / 8 = dm * tiles_n + dn
// With split-K (p.splits = S > 1, the ping-pong kernel only) the split index is the fastest
// batch coordinate: the tiles of one (batch, split) — which share that K range's A and B panels —
// are consecutive logical items, so they run together on one XCD's L2.
struct PWalk {
  int mt, nt, b0, b1, sp;
  int dm, dn;
};
__device__ __forceinline__ PWalk pwalk_init(const GemmParams& p, int w, int W, int G) {
  const int ntile = p.tiles_m * p.tiles_n;
  const int x = w & 7, q = W >> 3, r = W & 7;
  const int L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (w >> 3);
  const int bs = L / ntile, t = L - bs * ntile;
  const int b = bs / p.splits;
  PWalk s;
  s.sp = bs - b * p.splits;
  s.mt = t / p.tiles_n;
  s.nt = t - s.mt * p.tiles_n;
  s.b0 = b / p.batch1;
  s.b1 = b - s.b0 * p.batch1;
  s.dm = (G >> 3) / p.tiles_n;
  s.dn = (G >> 3) - s.dm * p.tiles_n;
  return s;
}
__device__ __forceinline__ void pwalk_next(const GemmParams& p, PWalk& s) {
  s.nt += s.dn;
  s.mt += s.dm;
  if (s.nt >= p.tiles_n) {
    s.nt -= p.tiles_n;
    ++s.mt;
  }
  while (s.mt >= p.tiles_m) {
    s.mt -= p.tiles_m;
    if (++s.sp == p.splits) {
      s.sp = 0;
      if (++s.b1 == p.batch1) {
        s.b1 = 0;
        ++s.b0;
      }
    }
  }
}
__device__ __forceinline__ PItem pwalk_item(const GemmParams& p, const PWalk& s) {
  PItem it;
  it.m0 = s.mt * 256;
  it.n0 = s.nt * 256;
  it.b0 = s.b0;
  it.b1 = s.b1;
  it.sp = s.sp;
  const int nkt = p.K >> 6;                 // split sp: K-tiles [sp nkt / S, (sp + 1) nkt / S)
  if (p.splits == 1) {
    it.kt0 = 0;
    it.len = nkt;
  } else {
    it.kt0 = s.sp * nkt / p.splits;
    it.len = (s.sp + 1) * nkt / p.splits - it.kt0;
  }
  return it;
}

// two floats -> two 16-bit values in one dword (one v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32, RNE)
template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, t2));
}

// EPI: 0 plain, 1 beta * C, 2 ReLU mask (aux), 3 both, 4 plain + ReLU — compile-time, so that every load the
// epilogue issues is consumed on every path (a conditional load left hipcc unsure at the loop
// head and it waited vmcnt(4) there, draining the next K-tile's DMA every iteration)
// rows I0 .. I0 + NI - 1 of the wave's sub-tiles (the ping-pong kernel stores its two 64-row
// halves in two segments)
// part (cfg 45 only, M % 256 != 0): the item is the last row panel, rows >= M exist only in the
// tile — the beta * C / mask loads read row M - 1 instead and the stores go through a buffer
// resource that ends at row M, so the hardware drops them; the VMEM count stays the full tile's
// (the deadline counts above depend on it).
template <typename T, class C, int EPI, int I0 = 0, int NI = C::TM>
__device__ __forceinline__ void persist_epilogue(const GemmParams& p, const PItem& it,
                                                 f32x4 (&acc)[C::TM][C::TN],
                                                 const float* bias_lds, int lane, int wm, int wn,
                                                 bool nostore = false, bool part = false) {
  static_assert(C::TN % 2 == 0, "paired stores");
  T* cp;
  int64_t cbase;
  if (p.c_mode == 1) {
    cp = (T*)p.c_ptr[it.b0];
    cbase = (int64_t)it.b1 * p.sC1;
  } else {
    cp = (T*)p.c_ptr[0];
    cbase = (int64_t)it.b0 * p.sC0 + (int64_t)it.b1 * p.sC1;
  }
  const int g = lane >> 4, rl = lane & 15;
  float bias4[C::TN][4];
  if (p.bias_mode == 1 && bias_lds) {
    const float* bl = bias_lds + (p.n_bias > 0 ? it.b0 * p.N : 0);
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const f32x4 v = *(const f32x4*)(bl + it.n0 + wn * C::WTN + 16 * j + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) bias4[j][e] = v[e];
    }
  } else if (p.bias_mode == 1) {
    // scalar loads (SMEM, lgkmcnt): the wave's 16 columns of sub-tile j are uniform; lane group
    // g takes its four.  (A vector load here would make hipcc wait vmcnt(0) for it — behind the
    // LDS-DMA it cannot see.)
    typedef const __attribute__((address_space(4))) f32x4 cf4;
    const float* bp = p.n_bias > 0 ? p.bias_tab[it.b0] : p.bias;
    const int wnu = __builtin_amdgcn_readfirstlane(wn);
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      cf4* cb = (cf4*)(bp + it.n0 + wnu * C::WTN + 16 * j);
      const f32x4 v0 = cb[0], v1 = cb[1], v2 = cb[2], v3 = cb[3];
      const f32x4 v = g == 0 ? v0 : g == 1 ? v1 : g == 2 ? v2 : v3;
#pragma unroll
      for (int e = 0; e < 4; ++e) bias4[j][e] = v[e];
    }
  } else {
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) bias4[j][e] = 0.f;
  }
  const float alpha = p.alpha, beta = p.beta;
  // ReLU: compile-time for the plain forms (EPI 0 / 4), a runtime flag with beta * C / the mask
  const bool relu = EPI == 4 || ((EPI & 3) != 0 && p.relu != 0);
  const T* auxp = (const T*)p.aux;
  // beta * C and the ReLU-backward mask (aux > 0) of the one-block-per-tile epilogue, in its
  // order (+ beta C, ReLU, mask); their 8-B loads of row i + 1 are in flight while row i is
  // converted and stored.  hipcc waits for them by its own count (only its own loads and stores
  // follow them); the DMA it cannot see is older, issued a K-tile earlier.
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 cr[2][C::TN], ar[2][C::TN];
  constexpr bool ldc_ = (EPI & 1) != 0, lda_ = (EPI & 2) != 0;
  auto load_row = [&](int i, u32x2 (&c)[C::TN], u32x2 (&a)[C::TN]) {
    int m = it.m0 + wm * C::WTM + 16 * i + rl;
    if (part) m = min(m, p.M - 1);
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int n = it.n0 + wn * C::WTN + 16 * j + 4 * g;
      if constexpr (ldc_) c[j] = *(const u32x2*)(cp + cbase + (int64_t)m * p.ldc + n);
      if constexpr (lda_) a[j] = *(const u32x2*)(auxp + cbase + (int64_t)m * p.ldaux + n);
    }
  };
  if constexpr (ldc_ || lda_) load_row(I0, cr[I0 & 1], ar[I0 & 1]);
  // the lane's store address for sub-tile row 0, sub-tile pair 0: row rl, its 8-column chunk
  T* const cl = cp + cbase + (int64_t)(it.m0 + wm * C::WTM + rl) * p.ldc + it.n0 + wn * C::WTN +
                16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
  for (int i = I0; i < I0 + NI; ++i) {
    if constexpr (ldc_ || lda_)
      if (i + 1 < I0 + NI) load_row(i + 1, cr[(i + 1) & 1], ar[(i + 1) & 1]);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 vj[C::TN / 2];
#pragma unroll
    for (int jp = 0; jp < C::TN / 2; ++jp) {
      uint32_t pk[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * jp + h;
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = acc[i][j][e] * alpha + bias4[j][e];
        if constexpr (ldc_ || lda_) {
          const T* cv = (const T*)&cr[i & 1][j];
          const T* av = (const T*)&ar[i & 1][j];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (ldc_) x[e] += beta * to_f(cv[e]);
            if (relu) x[e] = fmaxf(x[e], 0.f);
            if constexpr (lda_)
              if (!(to_f(av[e]) > 0.f)) x[e] = 0.f;
          }
        } else if (EPI == 4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) pk[h][q] = pack2<T>(x[2 * q], x[2 * q + 1]);
      }
      const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      vj[jp] = u32x4{r0[0], r1[0], r0[1], r1[1]};
    }
    if (nostore) continue;
    if (part) {
      // byte offsets from the entry's C base; rows >= M lie past num_records
      const uint64_t ba = (uint64_t)(uintptr_t)(cp + cbase);
      const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)ba);
      const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)bhi << 32) | blo), 0, (int)((int64_t)p.M * p.ldc * (int64_t)sizeof(T)),
          0x00020000);
      const int row = it.m0 + wm * C::WTM + 16 * i + rl;
      const int col = it.n0 + wn * C::WTN + 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
      for (int jp = 0; jp < C::TN / 2; ++jp)
        __builtin_amdgcn_raw_buffer_store_b128(
            vj[jp], rsrc, (int)(((int64_t)row * p.ldc + col + 32 * jp) * (int64_t)sizeof(T)), 0, 0);
      continue;
    }
    T* const crow = cl + (int64_t)(16 * i) * p.ldc;
#pragma unroll
    for (int jp = 0; jp < C::TN / 2; ++jp) {
      JMT_DCHECK(it.m0 + wm * C::WTM + 16 * i + rl < p.M &&
                 it.n0 + wn * C::WTN + 32 * jp + 16 * (g & 1) + 8 * (g >> 1) + 8 <= p.N);
      __builtin_nontemporal_store(vj[jp], (u32x4*)(crow + 32 * jp));
    }
  }
}

// split-K form of the epilogue (ping-pong kernel, p.splits > 1): rows I0 .. I0 + NI - 1 of the
// wave's sub-tiles as raw fp32 partial sums into the item's slab, ws[(sp nb + b) M + m][n] (the
// layout splitk_reduce_kernel sums in split order): one 16-B store per sub-tile and lane
// (nontemporal; plain stores, which could leave the slabs in the last-level cache for the
// reduce, measured the same in the step: 4.067-4.082 vs 4.066-4.075 ms, profiles/r06/
// step_ab_slab_nt.txt)
template <class C, int I0, int NI>
__device__ __forceinline__ void pp_slab_epilogue(const GemmParams& p, const PItem& it,
                                                 const f32x4 (&acc)[C::TM][C::TN], int lane,
                                                 int wm, int wn) {
  const int g = lane >> 4, rl = lane & 15;
  const int nb = p.batch0 * p.batch1;
  const int b = it.b0 * p.batch1 + it.b1;
  float* const sl = p.ws + ((int64_t)it.sp * nb + b) * (int64_t)p.M * p.N +
                    (int64_t)(it.m0 + wm * C::WTM + rl) * p.N + it.n0 + wn * C::WTN + 4 * g;
#pragma unroll
  for (int i = I0; i < I0 + NI; ++i) {
    float* const row = sl + (int64_t)(16 * i) * p.N;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) __builtin_nontemporal_store(acc[i][j], (f32x4*)(row + 16 * j));
  }
}

// the A row sums of one 16-row sub-tile (lane group g = lane >> 4 holds k-slices of row
// lane & 15) into the item's split partial, dbias_ws[(sp nb + b) M + m]: ONE store instruction
// (lanes 0-15), issued on every path so the epilogue's VMEM count stays exact.  The N tiles of
// one row panel store the same sums (same fragments, same order): identical bits.
__device__ __forceinline__ void pp_rowsum_store(const GemmParams& p, const PItem& it, float v,
                                                int row0, int lane) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  const int nb = p.batch0 * p.batch1;
  const int b = it.b0 * p.batch1 + it.b1;
  float* const d = p.dbias_ws + ((int64_t)it.sp * nb + b) * p.M + it.m0 + row0 + (lane & 15);
  if (lane < 16) *d = v;
}

// ABL: development ablation (compute_tile MODE; dbg 64 -> 1, 128 -> 2), bf16 plain epilogue only
template <typename T, bool AK, bool BK, class C, int EPI, int ABL = 0>
__global__ __launch_bounds__(C::NT, C::OCC)
void gemm_persist_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(C::BM == 256 && C::BN == 256, "pitem deals 256x256 tiles");
  constexpr int BKE = C::KB / (int)sizeof(T);
  constexpr int IA = C::BM * C::KB;
  constexpr int NWV = C::NT / 64;
  constexpr int NIA = C::BM * C::KB / 1024 / NWV;
  constexpr int NIB = C::BN * C::KB / 1024 / NWV;
  static_assert(NIA * NWV * 1024 == C::BM * C::KB && NIB * NWV * 1024 == C::BN * C::KB,
                "even LDS-DMA split");
  constexpr int VMT = NIA + NIB;                       // DMA instructions per wave per K-tile
  constexpr int NST = C::TM * (C::TN / 2);             // 16-B stores per wave per epilogue
  constexpr int NR = C::KB / 64 * C::TM;               // MFMA rows per K-tile
  constexpr int P = C::S - 1;                          // K-tiles in flight
  constexpr int KY = C::S == 2 ? 1 : P - 1;           // younger K-tiles at a wait, at most
  static_assert(VMT * KY + NST < 64, "vmcnt range");
  float* bias_lds = (float*)(smem + C::S * C::STAGE);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int W = p.tiles_m * p.tiles_n * p.batch0 * p.batch1;
  const int G = gridDim.x;
  const int nm = (W - (int)blockIdx.x + G - 1) / G;
  const int nkt = p.K / BKE;
  const int total = nm * nkt;

  // per-column bias (tables) -> LDS, before any LDS-DMA is in flight
  if (p.bias_mode == 1) {
    const int nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
    for (int i = threadIdx.x; i < nb; i += C::NT) {
      const int b = i / p.N;
      bias_lds[i] = (p.n_bias > 0 ? p.bias_tab[b] : p.bias)[i - b * p.N];
    }
  }
  __syncthreads();

  uint32_t offa[NIA], offb[NIB];
  glds_offsets<T, AK, C::KB, C::BM, C::NT>(offa, p.lda, 1 << 30, 0);
  glds_offsets<T, BK, C::KB, C::BN, C::NT>(offb, p.ldb, 1 << 30, 0);
  // scalar source bases of K-tile kt of item `it`
  auto bases = [&](const PItem& it, int kt, const char*& sa, const char*& sb) {
    const int k0 = kt * BKE;
    int ka, kb;
    const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, it.b0, it.b1, p.a_kseg, k0, ka);
    const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, it.b0, it.b1, p.b_kseg, k0, kb);
    sa = (const char*)(AK ? A + (int64_t)it.m0 * p.lda + ka : A + (int64_t)ka * p.lda + it.m0);
    sb = (const char*)(BK ? B + (int64_t)it.n0 * p.ldb + kb : B + (int64_t)kb * p.ldb + it.n0);
  };
  // issue cursor: the next K-tile (stream index t) whose DMA goes out
  int iss_kt = 0, iss_k = 0;
  PWalk iss_w = pwalk_init(p, blockIdx.x, W, G);
  PItem iss = pwalk_item(p, iss_w);
  auto advance_issue = [&]() {
    if (++iss_kt == nkt) {
      iss_kt = 0;
      ++iss_k;
      if (iss_k < nm) {
        pwalk_next(p, iss_w);
        iss = pwalk_item(p, iss_w);
      }
    }
  };
#pragma unroll
  for (int t = 0; t < P; ++t) {
    if (t < total) {
      const char *sa, *sb;
      bases(iss, iss_kt, sa, sb);
      char* img = smem + t * C::STAGE;
#pragma unroll
      for (int i = 0; i < NIA; ++i) glds_slot<NIA>(img, sa, offa, i);
#pragma unroll
      for (int i = 0; i < NIB; ++i) glds_slot<NIB>(img + IA, sb, offb, i);
      advance_issue();
    }
  }

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  PWalk cur_w = pwalk_init(p, blockIdx.x, W, G);
  PItem cur = pwalk_item(p, cur_w);
  int cur_k = 0, cur_kt = 0;
  int last_ep = -(1 << 20);
  // dbg 32: wait for the stores as well (A/B of the overlap); dbg 2 issues no stores
  const bool count_stores = !(p.dbg & (32 | 2));

  for (int s = 0; s < total; ++s) {
    const char *sa = nullptr, *sb = nullptr;
    const bool go = s + P < total;                     // DMA of K-tile s + P this iteration
    if (go) bases(iss, iss_kt, sa, sb);
    char* nimg = smem + ((s + P) % C::S) * C::STAGE;
    if constexpr (C::S == 2) {
      // buffer (s + 1) & 1 was freed by the second barrier of iteration s - 1
      if (go) {
#pragma unroll
        for (int i = 0; i < NIA; ++i) glds_slot<NIA>(nimg, sa, offa, i);
#pragma unroll
        for (int i = 0; i < NIB; ++i) glds_slot<NIB>(nimg + IA, sb, offb, i);
      }
    }
    // VMEM operations issued after K-tile s's DMA: the younger K-tiles' DMA and, while s is
    // within P K-tiles of the last epilogue, that epilogue's stores
    wait_young<VMT, NST, KY>(min(KY, total - 1 - s), count_stores && s <= last_ep + P);
    __builtin_amdgcn_s_barrier();
    const char* img = smem + (s % C::S) * C::STAGE;
    if constexpr (C::S == 2) {
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C, NoIssue, ABL>(img, img + IA, wm, wn, acc);
      __builtin_amdgcn_s_barrier();                    // buffer s & 1 free for K-tile s + 2
    } else {
      // piece q of the next K-tile's NIA + NIB DMA instructions goes before MFMA row
      // q * NR / (NIA + NIB) (buffer (s - 1) % S: freed by this iteration's barrier)
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
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(img, img + IA, wm, wn, acc, issue);
      else issue(0);
    }
    if (go) advance_issue();
    if (++cur_kt == nkt) {                             // item done: stores behind the prefetch
      if (!(p.dbg & 2)) persist_epilogue<T, C, EPI>(p, cur, acc, bias_lds, lane, wm, wn);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      last_ep = s;
      cur_kt = 0;
      if (++cur_k < nm) {
        pwalk_next(p, cur_w);
        cur = pwalk_item(p, cur_w);
      }
    }
  }
}

// ------------------------------------------------------------------ ping-pong kernel (cfg 43)
// The persistent 256x256 tile with the DMA issue taken off the MFMA-issuing wave's critical
// path.  Measured on cfg 40 (profiles/r05/gemm_ablate_*.jsonl): its time is the sum of a
// DMA-only run and an MFMA-only run (NT b6 19200x1024x512: 64 + 70 -> 135 us without the
// epilogue) at every pipeline depth (2 or 4 stages): the waves that issue the next K-tile's
// LDS-DMA are the waves whose MFMAs then wait behind that issue, so no depth hides it.
// Here (cdna_hip_programming.md §5 "The 256² 8-phase template"): the two waves of each SIMD
// — group 0 = waves 0-3 (M rows 0-127 of the tile), group 1 = waves 4-7 (rows 128-255) — run
// the same phase sequence one barrier apart (group 1 starts with one extra s_barrier), so
// between any two barriers one group issues the next phase's LDS reads and its share of the
// LDS-DMA stream while the other group's 16 MFMAs run on the same SIMD.
//  * K-tile = 64 deep, staged as two k-halves (32 deep); a k-half slot holds A (256 x 64 B) and
//    B (256 x 64 B) images = 32 KiB; PP_NSLOT slots in a ring (k-half g in slot g % PP_NSLOT).
//  * Phases per K-tile (per wave): (ks, qm) = (0,0) (0,1) (1,0) (1,1): 4 row sub-tiles
//    (qm half of the wave's 128 rows) x 4 column sub-tiles x one 32-deep k-step = 16 MFMAs;
//    reads: 4 A fragments, + 4 B fragments when qm = 0 (B reused by qm = 1).
//  * DMA stream: piece P = 8 KiB (8 wave-instructions) = one half of one operand's k-half
//    image; interval I (between barriers I-1 and I; group I & 1 loads) issues piece I + PP_D,
//    2 instructions per wave of the loading group.  k-half g must be retired (counted vmcnt by
//    every issuing wave) before barrier 4g - 1 (group 0 reads it in interval 4g); its slot is
//    free after barrier 4g + 4 - 4 * PP_NSLOT: PP_D = 4 PP_NSLOT - 5 keeps both.
//  * Waits: the compiler never sees the DMA (inline asm); each wave counts its own VMEM issue
//    (DMA pairs, epilogue stores / loads) and waits vmcnt(issued since its last piece of g) at
//    the deadline; vmcnt counts in issue order, so rounding that count down (wait_vm_le) only
//    over-waits.
constexpr int PP_NSLOT = 4;
constexpr int PP_D = 4 * PP_NSLOT - 5;
static_assert(PP_D == 11, "pp_run's deadline counts (epilogue halves vs pieces per segment) are derived for PP_D = 11");
constexpr int PP_SLOT = 32768;
using CfgPP = TileCfg<256, 256, 2, 4, 64, 2, 1, 1, 0>;    // epilogue geometry (128 x 64 / wave)

// s_waitcnt vmcnt(m) for the largest m <= n among 0..16, 20, 24, ..., 60 (wave-uniform n)
__device__ __forceinline__ void wait_vm_le(int n) {
  if (n <= 16) {
    wait_vm(n);
    return;
  }
  switch (n >= 60 ? 15 : n >> 2) {
    case 4: wait_vmcnt<16>(); break;
    case 5: wait_vmcnt<20>(); break;
    case 6: wait_vmcnt<24>(); break;
    case 7: wait_vmcnt<28>(); break;
    case 8: wait_vmcnt<32>(); break;
    case 9: wait_vmcnt<36>(); break;
    case 10: wait_vmcnt<40>(); break;
    case 11: wait_vmcnt<44>(); break;
    case 12: wait_vmcnt<48>(); break;
    case 13: wait_vmcnt<52>(); break;
    case 14: wait_vmcnt<56>(); break;
    default: wait_vmcnt<60>(); break;
  }
}

// One group's whole schedule (GRP = 0: waves 0-3, 1: waves 4-7), everything that depends on
// the group compile-time: which pieces it issues, where its stream moves to the next K-tile,
// where its deadline waits go.  Per load segment the scalar work is a few adds: the wave's
// four DMA sources are per-lane pointers (VGPRs) advanced by one VALU add per K-tile; the
// item / K-concat bookkeeping runs once per K-tile of the stream.
// development: s_memtime stamps of one block's segments (dbg 8, bf16 EPI 0 only; read with
// jmt_gemm_pp_stamps_read): [wave][K-tile < PP_STK][phase][6]
constexpr int PP_STK = 24;
__device__ uint64_t g_pp_stamps[8 * PP_STK * 4 * 8];

template <typename T, bool AK, bool BK, int EPI, int GRP, int MODE = 0>
__device__ __forceinline__ void pp_run(const GemmParams& p, uint32_t lbase, const char* smem,
                                       const float* bias_lds, int nm, int W) {
  using C = CfgPP;
  typedef typename Frag16<T>::t F;
  // epilogue VMEM operations per wave: 16-B stores of paired 16-bit sub-tiles and the
  // beta * C / mask loads
  constexpr int NST = C::TM * (C::TN / 2);
  constexpr int NLD = ((EPI & 1) ? C::TM * C::TN : 0) + ((EPI & 2) ? C::TM * C::TN : 0);
  constexpr int SUB = (GRP + PP_D) & 1;                    // parity of this group's pieces
  // VMEM operations younger than the wave's last piece of k-half g at its deadline, away from
  // the stream's end: its pieces of the load intervals (4g + 2 + SUB - PP_D, 4g - 2 + GRP]
  constexpr int NSTEADY = 2 * ((PP_D - 4 + GRP - SUB) >> 1);
  constexpr int EPH = (NST + NLD) / 2;                      // VMEM operations per epilogue half
  constexpr int NSTEADY_EP1 = NSTEADY + EPH < 63 ? NSTEADY + EPH : 63;
  constexpr int NSTEADY_EP2 = NSTEADY + 2 * EPH < 63 ? NSTEADY + 2 * EPH : 63;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // SGPR: LDS addresses scalar
  const int wl = wid & 3;
  constexpr int wm = GRP;
  constexpr bool STAMP = MODE == 2;                        // MODE 1: ablations, 2: + stamps
  const int dbg = MODE ? p.dbg : 0;
  const int wn = wl;
  const int G = gridDim.x;
  const int nT = nm * (p.K >> 6);                          // K-tiles of this block's items
  const int npieces = 8 * nT;
  const int ins0 = SUB * 8 + 2 * wl;

  // per-lane byte offsets of this wave's instructions ins0, ins0 + 1 of each operand's k-half
  // image, relative to the operand's K-tile base
  int64_t offa[2], offb[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    int row, kk;
    chunk_src<T, AK, 64, 256>((ins0 + e) * 64 + lane, row, kk);
    offa[e] = (AK ? (int64_t)row * p.lda + kk : (int64_t)kk * p.lda + row) * (int64_t)sizeof(T);
    chunk_src<T, BK, 64, 256>((ins0 + e) * 64 + lane, row, kk);
    offb[e] = (BK ? (int64_t)row * p.ldb + kk : (int64_t)kk * p.ldb + row) * (int64_t)sizeof(T);
  }
  const int64_t da = (AK ? (int64_t)64 : (int64_t)64 * p.lda) * (int64_t)sizeof(T);   // K-tile
  const int64_t db = (BK ? (int64_t)64 : (int64_t)64 * p.ldb) * (int64_t)sizeof(T);
  const int64_t ha = da / 2, hb = db / 2;                                             // k-half
  const int sega = p.a_mode >= 2 ? p.a_kseg / 64 : 1 << 30;   // K-tiles per K-concat segment
  const int segb = p.b_mode >= 2 ? p.b_kseg / 64 : 1 << 30;

  // the issue stream: item iss_k, K-tile iss_kt of it, per-lane sources pa / pb of that K-tile
  PWalk iss_w = pwalk_init(p, blockIdx.x, W, G);
  PItem iss_it = pwalk_item(p, iss_w);
  int iss_k = 0, iss_kt = 0, lefta = 0, leftb = 0;
  const char* pa[2];
  const char* pb[2];
  auto set_stream = [&]() {
    const int k0 = (iss_it.kt0 + iss_kt) * 64;
    int ka, kb;
    const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, iss_it.b0, iss_it.b1,
                                 p.a_kseg, k0, ka);
    const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, iss_it.b0, iss_it.b1,
                                 p.b_kseg, k0, kb);
    const char* sa = (const char*)(AK ? A + (int64_t)iss_it.m0 * p.lda + ka
                                      : A + (int64_t)ka * p.lda + iss_it.m0);
    const char* sb = (const char*)(BK ? B + (int64_t)iss_it.n0 * p.ldb + kb
                                      : B + (int64_t)kb * p.ldb + iss_it.n0);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      pa[e] = sa + offa[e];
      pb[e] = sb + offb[e];
    }
    lefta = sega - (ka >> 6);                              // K-tiles left in A's segment
    leftb = segb - (kb >> 6);
  };
  auto next_ktile = [&]() {
    if (++iss_kt == iss_it.len) {
      iss_kt = 0;
      if (++iss_k < nm) {
        pwalk_next(p, iss_w);
        iss_it = pwalk_item(p, iss_w);
        set_stream();
      }
    } else if (--lefta == 0 || --leftb == 0) {
      set_stream();
    } else {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        pa[e] += da;
        pb[e] += db;
      }
    }
  };
  // this wave's two instructions of piece Q = (operand, half) of k-half g
  auto issue = [&](int g, int q) {
    const uint32_t dst = lbase + (g & (PP_NSLOT - 1)) * PP_SLOT + (q >= 2 ? 16384 : 0) + ins0 * 1024;
    const int h = g & 1;
    if (q < 2) {
      glds16_at(pa[0] + (h ? ha : 0), dst);
      glds16_at(pa[1] + (h ? ha : 0), dst + 1024);
    } else {
      glds16_at(pb[0] + (h ? hb : 0), dst);
      glds16_at(pb[1] + (h ? hb : 0), dst + 1024);
    }
  };
  // k-half g retired by this wave, at the barrier 4g - 1; i_now = this wave's latest load
  // interval (its piece issued).  Issued after its last piece of g: its pieces of the load
  // intervals in (i_last, i_now] (2 each, while pieces exist) and an epilogue of this K-tile.
  // neh: epilogue halves (EPH operations each) issued after the wave's last piece of g (the
  // caller knows them from the schedule: 0, 1 or 2)
  // steady: the caller's K-tile t has t + 3 <= nT, so i_now <= 8 t + 7 <= npieces - 1 - PP_D
  // and g < 2 nT (one flag per K-tile instead of two compares per deadline)
  auto deadline = [&](int g, int i_now, int neh, bool steady) {
    if (steady) {                                          // constant counts
      if (neh == 0) wait_vmcnt<NSTEADY>();
      else if (neh == 1) wait_vmcnt<NSTEADY_EP1>();
      else wait_vmcnt<NSTEADY_EP2>();
      return;
    }
    if (g >= 2 * nT) return;
    if (i_now <= npieces - 1 - PP_D) {
      if (neh == 0) wait_vmcnt<NSTEADY>();
      else if (neh == 1) wait_vmcnt<NSTEADY_EP1>();
      else wait_vmcnt<NSTEADY_EP2>();
      return;
    }
    const int i_last = 4 * g + 2 + SUB - PP_D;
    const int hi = min(i_now, npieces - 1 - PP_D);
    const int n = (hi > i_last ? 2 * ((hi - i_last) >> 1) : 0) + neh * EPH;
    wait_vm_le(n);
  };

  // prologue: this group's pieces among 0 .. PP_D-1, k-half 0 retired, one barrier for all
  set_stream();
#pragma unroll
  for (int P = SUB; P < PP_D; P += 2) {
    if (P >= 8 && P - 2 < 8) next_ktile();                 // (PP_D <= 16: K-tiles 0 and 1)
    if (P < npieces) issue(P >> 2, P & 3);
  }
  deadline(0, -1, 0, false);
  __builtin_amdgcn_s_barrier();
  if constexpr (GRP == 1) __builtin_amdgcn_s_barrier();    // group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  F fa[4] = {}, fb[4] = {};
  PWalk cur_w = pwalk_init(p, blockIdx.x, W, G);
  PItem cur = pwalk_item(p, cur_w);
  int cur_left = cur.len;
  // epilogue of an item in two halves: rows 0-63 of the wave (quadrant qm = 0, final after
  // phase 2 of the item's last K-tile) in that K-tile's phase-3 load segment, rows 64-127 in the
  // next K-tile's phase-0 load segment — half the store burst per segment
  bool epA = false, epB = false;

  // the stores of one epilogue half (h = 0: rows 0-63 of the wave, 1: rows 64-127) of item cur
  auto epilogue_half = [&](int h) {
    if (h == 0) persist_epilogue<T, C, EPI, 0, 4>(p, cur, acc, bias_lds, lane, wm, wn, dbg & 64);
    else persist_epilogue<T, C, EPI, 4, 4>(p, cur, acc, bias_lds, lane, wm, wn, dbg & 64);
  };

  const bool stamping = STAMP && blockIdx.x == 0 && lane == 0;
  for (int t = 0; t < nT; ++t) {
    const bool steady = t + 3 <= nT;
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int ks = pp >> 1, qm = pp & 1;
      const int I = 8 * t + 2 * pp + GRP;                  // this wave's load interval
      auto stamp = [&](int e) {
        if constexpr (STAMP) {
          if (stamping && t < PP_STK)
            g_pp_stamps[((wid * PP_STK + t) * 4 + pp) * 8 + e] = __builtin_amdgcn_s_memtime();
        }
      };
      stamp(0);
      // ---- load segment
      if (pp == 0) {
        epB = false;
        if (cur_left == 0) {                               // previous item done: rows 64-127
          if (!(dbg & 2)) epilogue_half(1);
          pwalk_next(p, cur_w);
          cur = pwalk_item(p, cur_w);
          cur_left = cur.len;
          epB = true;
        }
        --cur_left;
        epA = false;
      }
      if (pp == 3 && cur_left == 0 && t + 1 < nT) {        // the item's last K-tile: rows 0-63
        if (!(dbg & 2)) epilogue_half(0);
        epA = true;
      }
      // piece P = I + PP_D: K-tile t + (L >> 3), k-half 2 (t + (L >> 3)) + ((L >> 2) & 1),
      // quarter L & 3, L = 2 pp + GRP + PP_D (compile-time after unrolling).  The stream's K-tile
      // step comes before this segment's LDS reads: an item switch waits lgkmcnt(0) for its
      // scalar loads, which would otherwise also wait for the reads in flight
      stamp(6);
      const int L = 2 * pp + GRP + PP_D;
      const int Lp = 2 * pp - 2 + GRP + PP_D;
      if (pp > 0 ? ((L >> 3) != (Lp >> 3)) : ((L >> 3) != ((L + 6) >> 3) - 1))
        next_ktile();
      stamp(7);
      const char* slot = smem + ((2 * t + ks) & (PP_NSLOT - 1)) * PP_SLOT;
      if (!(dbg & 128)) {                                  // (ablation 128: no fragment reads)
        if (qm == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            fb[j] = read_frag16<T, BK, 64, 256>(slot + 16384, wn * C::WTN + 16 * j, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = read_frag16<T, AK, 64, 256>(slot, wm * C::WTM + 64 * qm + 16 * i, 0);
      }
      stamp(1);
      if (!(dbg & 4) && I + PP_D < npieces) issue(2 * (t + (L >> 3)) + ((L >> 2) & 1), L & 3);
      stamp(2);
      // epilogue halves younger than the wave's last piece of the k-half due (a segment issues
      // its epilogue half BEFORE its piece; counting one too many would under-wait): at phase 1
      // both halves of an epilogue that finished at this K-tile's start; at phase 3 this K-tile's
      // own first half, and for group 1 the second half of this K-tile's start (group 0's last
      // piece of k-half 2t + 2 went out after it, in the same phase-0 segment)
      const int neh = pp == 1 ? (epB ? 2 : 0)
                              : (GRP == 1 && epB ? 1 : 0) + (epA ? 1 : 0);
      if (GRP == 1 && (pp & 1) && !(dbg & 16)) deadline((I + 1) >> 2, I, neh, steady);
      stamp(3);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      stamp(4);
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
      if (!(dbg & 1)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 * qm + i][j] = mfma16(fb[j], fa[i], acc[4 * qm + i][j]);   // C^T sub-tiles
      }
      __builtin_amdgcn_s_setprio(0);
      // rows stored by this phase's load segment restart at 0, here behind the MFMAs that do not
      // touch them (rows 0-63 after phase 3's epilogue half, rows 64-127 after phase 0's)
      if (pp == 3 && epA) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (pp == 0 && epB) {
#pragma unroll
        for (int i = 4; i < C::TM; ++i)
#pragma unroll
          for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if (GRP == 0 && (pp & 1) && !(dbg & 16)) deadline((I + 2) >> 2, I, neh, steady);
      stamp(5);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (GRP == 0) __builtin_amdgcn_s_barrier();    // balance group 1's extra barrier
  if (!(dbg & 2)) {
    epilogue_half(0);
    epilogue_half(1);
  }
}

template <typename T, bool AK, bool BK, int EPI, int MODE = 0>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* bias_lds = (float*)(smem + PP_NSLOT * PP_SLOT);
  const int W = p.tiles_m * p.tiles_n * p.batch0 * p.batch1;
  const int G = gridDim.x;
  const int nm = (W - (int)blockIdx.x + G - 1) / G;
  if (p.bias_mode == 1) {
    const int nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
    for (int i = threadIdx.x; i < nb; i += 512) {
      const int b = i / p.N;
      bias_lds[i] = (p.n_bias > 0 ? p.bias_tab[b] : p.bias)[i - b * p.N];
    }
  }
  __syncthreads();
  if (nm <= 0 || p.K < 64) return;
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  if ((threadIdx.x >> 6) < 4) pp_run<T, AK, BK, EPI, 0, MODE>(p, lbase, smem, bias_lds, nm, W);
  else pp_run<T, AK, BK, EPI, 1, MODE>(p, lbase, smem, bias_lds, nm, W);
}

// ---------------------------------------------------------------- ping-pong, 32-MFMA phases
// cfg 45 (the default where the persistent path applies): the ping-pong schedule above with ONE
// phase per k-half — the whole 32-deep k-half over all 8 row sub-tiles of the wave, 12 fragment
// reads and 32 MFMAs — so a K-tile is 2 phases = 4 barrier intervals instead
// of 8 (the measured ≈ 250 cycles of barrier and bookkeeping per interval, halved per FLOP).
// DMA: interval I issues pieces 2 I + P2_D, 2 I + P2_D + 1 (P2_D = 10, the most the 4-slot ring
// allows: k-half g + 4 reuses g's slot, whose last reads retire in interval 2 g + 2); with P2_D
// even, group 0 (even intervals) always issues the B halves of k-half m + 2 at its phase m, group
// 1 the A halves of k-half m + 3.  Deadline of k-half g, before barrier 2 g - 1: group 0 in its
// MFMA segment of phase g - 1 (younger: its phase g - 1 pieces, 4 ops, and that load segment's
// epilogue), group 1 in its load segment of phase g - 1 after its pieces (younger: phases g - 2
// and g - 1, 8 ops, and their epilogues).  The epilogue of an item is whole, in each group's load
// segment of the next item's first phase (every phase writes all 8 row sub-tiles).
constexpr int P2_D = 10;
static_assert(P2_D % 2 == 0 && P2_D <= 10, "pp2 deadline counts are derived for an even P2_D <= 10");

// SPL: 0 the 16-bit C epilogue (persist_epilogue, EPI), 1 split-K fp32 slabs (pp_slab_epilogue),
// 2 slabs + the A row sums (dbias_ws)
template <typename T, bool AK, bool BK, int EPI, int GRP, int SPL = 0>
__device__ __forceinline__ void pp2_run(const GemmParams& p, uint32_t lbase, const char* smem,
                                        const float* bias_lds, int nm, int W) {
  using C = CfgPP;
  typedef typename Frag16<T>::t F;
  constexpr bool ISA = GRP == 1;                           // this group's operand: A (else B)
  constexpr bool KM = ISA ? AK : BK;
  constexpr int NST = SPL ? C::TM * C::TN + (SPL == 2 ? 2 : 0) : C::TM * (C::TN / 2);
  constexpr int NLD = SPL ? 0 : ((EPI & 1) ? C::TM * C::TN : 0) + ((EPI & 2) ? C::TM * C::TN : 0);
  constexpr int EPO = NST + NLD;                           // VMEM operations of one epilogue
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wl = wid & 3;
  constexpr int wm = GRP;
  const int wn = wl;
  const int G = gridDim.x;
  // K-tiles of this block's items (split-K items differ by one K-tile at most)
  int nT = nm * (p.K >> 6);
  if (SPL && p.splits > 1) {
    PWalk w = pwalk_init(p, blockIdx.x, W, G);
    nT = 0;
    for (int k = 0; k < nm; ++k) {
      if (k) pwalk_next(p, w);
      nT += pwalk_item(p, w).len;
    }
  }
  const int nh = 2 * nT;                                   // k-halves of the block's stream
  const int64_t ld = ISA ? p.lda : p.ldb;
  // per-lane byte offsets of this wave's instructions 2 wl, 2 wl + 1 of each half (h) of its
  // operand's k-half image, relative to the operand's K-tile base
  // (the A rows of a last, partial row panel (M % 256 != 0) are clamped to the last row — or the
  // last 8-row chunk, MN-major — in set_stream; their products are never stored)
  int rowv[2][2], kkv[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 2; ++e)
      chunk_src<T, KM, 64, 256>((8 * h + 2 * wl + e) * 64 + lane, rowv[h][e], kkv[h][e]);
  const int64_t dk = (KM ? (int64_t)64 : (int64_t)64 * ld) * (int64_t)sizeof(T);   // K-tile
  const int64_t hk = dk / 2;                                                          // k-half
  const int seg = (ISA ? p.a_mode : p.b_mode) >= 2 ? (ISA ? p.a_kseg : p.b_kseg) / 64 : 1 << 30;

  PWalk iss_w = pwalk_init(p, blockIdx.x, W, G);
  PItem iss_it = pwalk_item(p, iss_w);
  int iss_k = 0, iss_kt = 0, left = 0;
  const char* ps[2][2];
  auto set_stream = [&]() {
    const int k0 = (iss_it.kt0 + iss_kt) * 64;
    int kl;
    const T* X = ISA ? operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, iss_it.b0, iss_it.b1,
                                       p.a_kseg, k0, kl)
                     : operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, iss_it.b0, iss_it.b1,
                                       p.b_kseg, k0, kl);
    const int r0 = ISA ? iss_it.m0 : iss_it.n0;
    const char* sx = (const char*)(KM ? X + (int64_t)r0 * ld + kl : X + (int64_t)kl * ld + r0);
    const int rmax = ISA ? p.M - (KM ? 1 : 8) - r0 : 256;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int r = min(rowv[h][e], rmax);
        ps[h][e] = sx + (KM ? (int64_t)r * ld + kkv[h][e] : (int64_t)kkv[h][e] * ld + r) *
                            (int64_t)sizeof(T);
      }
    left = seg - (kl >> 6);
  };
  auto next_ktile = [&]() {
    if (++iss_kt == iss_it.len) {
      iss_kt = 0;
      if (++iss_k < nm) {
        pwalk_next(p, iss_w);
        iss_it = pwalk_item(p, iss_w);
        set_stream();
      }
    } else if (--left == 0) {
      set_stream();
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 2; ++e) ps[h][e] += dk;
    }
  };
  // this wave's 4 instructions of k-half g (its operand's two halves) from the current K-tile
  auto issue = [&](int g) {
    const uint32_t dst = lbase + (g & 3) * PP_SLOT + (ISA ? 0 : 16384) + 2 * wl * 1024;
    const int64_t kh = (g & 1) ? hk : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 2; ++e) glds16_at(ps[h][e] + kh, dst + (8 * h + e) * 1024);
  };
  // epilogues issued in this phase's / the previous phase's load segment (deadline counts)
  bool ep_cur = false, ep_prev = false;
  // k-half g retired by this wave (at phase g - 1); counts as in the header comment, rounded
  // down near the stream's end
  auto deadline = [&](int g) {
    if (g >= nh) return;
    const int m = g - 1;
    if constexpr (GRP == 0) {
      // younger: its piece of k-half m + 2 (phase m) and phase m's epilogue
      const int n = (m + 2 < nh ? 4 : 0) + (ep_cur ? EPO : 0);
      if (n == 4) wait_vmcnt<4>();
      else wait_vm_le(n);
    } else {
      // younger: its pieces of k-halves m + 2 (phase m - 1) and m + 3 (phase m)
      const int n = (m + 2 < nh ? 4 : 0) + (m + 3 < nh ? 4 : 0) +
                    ((ep_prev ? 1 : 0) + (ep_cur ? 1 : 0)) * EPO;
      if (n == 8) wait_vmcnt<8>();
      else wait_vm_le(n);
    }
  };

  // prologue: group 0 the B halves of k-halves 0, 1; group 1 the A halves of 0, 1, 2
  set_stream();
  if constexpr (GRP == 0) {
    issue(0);
    issue(1);
    wait_vmcnt<4>();                                       // k-half 0 retired
  } else {
    issue(0);
    if (nh > 1) issue(1);
    if (nh > 2) {
      next_ktile();
      issue(2);
    }
    wait_vm_le((nh > 1 ? 4 : 0) + (nh > 2 ? 4 : 0));
  }
  __builtin_amdgcn_s_barrier();
  if constexpr (GRP == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  F fa[8] = {}, fb[4] = {};
  PWalk cur_w = pwalk_init(p, blockIdx.x, W, G);
  PItem cur = pwalk_item(p, cur_w);
  int cur_left = cur.len;
  float rsum[2] = {0.f, 0.f};                              // SPL 2: row sums of sub-tiles wn, wn + 4
  auto epilogue = [&]() {
    if constexpr (SPL) {
      pp_slab_epilogue<C, 0, 8>(p, cur, acc, lane, wm, wn);
      if constexpr (SPL == 2) {
        pp_rowsum_store(p, cur, rsum[0], wm * C::WTM + 16 * wn, lane);
        pp_rowsum_store(p, cur, rsum[1], wm * C::WTM + 64 + 16 * wn, lane);
        rsum[0] = rsum[1] = 0.f;
      }
    } else {
      persist_epilogue<T, C, EPI>(p, cur, acc, bias_lds, lane, wm, wn, false,
                                  cur.m0 + 256 > p.M);
    }
  };
  for (int t = 0; t < nT; ++t) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int m = 2 * t + ks;
      // ---- load segment
      ep_prev = ep_cur;
      ep_cur = false;
      if (ks == 0) {
        if (cur_left == 0) {                               // previous item done: its epilogue
          epilogue();
          ep_cur = true;
#pragma unroll
          for (int i = 0; i < C::TM; ++i)
#pragma unroll
            for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          pwalk_next(p, cur_w);
          cur = pwalk_item(p, cur_w);
          cur_left = cur.len;
        }
        --cur_left;
      }
      // stream step: group 0 issues k-half m + 2 (K-tile t + 1), group 1 k-half m + 3
      if ((GRP == 0 && ks == 0) || (GRP == 1 && ks == 1)) next_ktile();
      const char* slot = smem + (m & 3) * PP_SLOT;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = read_frag16<T, BK, 64, 256>(slot + 16384, wn * C::WTN + 16 * j, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = read_frag16<T, AK, 64, 256>(slot, wm * C::WTM + 16 * i, 0);
      {
        const int g = m + (GRP == 0 ? 2 : 3);
        if (g < nh) issue(g);
      }
      if constexpr (GRP == 1) deadline(m + 1);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (SPL == 2) {                            // A row sums, sub-tiles wn and wn + 4
        if (wn == 0) { rsum[0] = rowsum8(fa[0], rsum[0]); rsum[1] = rowsum8(fa[4], rsum[1]); }
        else if (wn == 1) { rsum[0] = rowsum8(fa[1], rsum[0]); rsum[1] = rowsum8(fa[5], rsum[1]); }
        else if (wn == 2) { rsum[0] = rowsum8(fa[2], rsum[0]); rsum[1] = rowsum8(fa[6], rsum[1]); }
        else { rsum[0] = rowsum8(fa[3], rsum[0]); rsum[1] = rowsum8(fa[7], rsum[1]); }
      }
      if constexpr (GRP == 0) deadline(m + 1);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (GRP == 0) __builtin_amdgcn_s_barrier();
  epilogue();
}

template <typename T, bool AK, bool BK, int EPI>
__global__ __launch_bounds__(512) void gemm_pp2_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* bias_lds = (float*)(smem + PP_NSLOT * PP_SLOT);
  const int W = p.tiles_m * p.tiles_n * p.batch0 * p.batch1;
  const int G = gridDim.x;
  const int nm = (W - (int)blockIdx.x + G - 1) / G;
  if (p.bias_mode == 1) {
    const int nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
    for (int i = threadIdx.x; i < nb; i += 512) {
      const int b = i / p.N;
      bias_lds[i] = (p.n_bias > 0 ? p.bias_tab[b] : p.bias)[i - b * p.N];
    }
  }
  __syncthreads();
  if (nm <= 0 || p.K < 64) return;
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  if ((threadIdx.x >> 6) < 4) pp2_run<T, AK, BK, EPI, 0>(p, lbase, smem, bias_lds, nm, W);
  else pp2_run<T, AK, BK, EPI, 1>(p, lbase, smem, bias_lds, nm, W);
}

// split-K form (cfg 44, on the cfg 45 schedule): items are (tile, split) — the weight-gradient GEMMs (M, N = features,
// K = B x T rows: a few 256 x 256 tiles over a long K); fp32 partial slabs (+ the A row sums) for
// splitk_reduce_kernel, which jmt_gemm launches next
// (An in-launch reduction — the S blocks of a tile meeting at a per-tile counter, then each
// reducing its 256 / S rows over all S slabs — measured slower than the separate
// splitk_reduce_kernel launch on every weight-gradient shape, 5-10 %: the reduce loop of one
// 8-wave block per CU keeps too few slab loads in flight; profiles/r05/tn_fused_reduce_ab.txt.)

template <typename T, bool AK, bool BK, int SPL>
__global__ __launch_bounds__(512) void gemm_pp_split_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = p.tiles_m * p.tiles_n * p.batch0 * p.batch1 * p.splits;
  const int G = gridDim.x;
  const int nm = (W - (int)blockIdx.x + G - 1) / G;
  if (nm <= 0 || p.K < 64) return;
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  if ((threadIdx.x >> 6) < 4) pp2_run<T, AK, BK, 0, 0, SPL>(p, lbase, smem, nullptr, nm, W);
  else pp2_run<T, AK, BK, 0, 1, SPL>(p, lbase, smem, nullptr, nm, W);
}

// the persistent configuration (gemm_persist_kernel): cfg 40 = Cfg5's tile (128-B K-tiles, 2
// stages).  (Cfg20's 64-B K-tiles in 4 stages with interleaved DMA issue — "cfg 41" — and a
// three-deep A ring with the bias from scalar loads — "cfg 42" — measured slower on every step
// shape: profiles/r04/gemm_persist_vs_vendor_a.jsonl, gemm_persist_forced_ab.txt.)
using Cfg40 = Cfg5;

static int num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int v = 0;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    cache[dev] = v > 0 ? v : 256;
  }
  return cache[dev];
}

template <typename T, bool AK, bool BK, class C, int EPI>
static void launch_persist_epi(const GemmParams& p, int blocks, hipStream_t st) {
  void (*fn)(GemmParams) = gemm_persist_kernel<T, AK, BK, C, EPI>;
  if constexpr (EPI == 0 && sizeof(T) == 2) {
    if (p.dbg & 64) fn = gemm_persist_kernel<T, AK, BK, C, EPI, 1>;
    if (p.dbg & 128) fn = gemm_persist_kernel<T, AK, BK, C, EPI, 2>;
  }
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  int nb = 0;
  if (p.bias_mode == 1) nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
  const size_t lds = (size_t)C::S * C::STAGE + (size_t)nb * sizeof(float);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(C::NT), lds, st, p);
}

template <typename T, bool AK, bool BK, int EPI>
static void launch_pp_epi(const GemmParams& p, int blocks, hipStream_t st) {
  void (*fn)(GemmParams) = gemm_pp_kernel<T, AK, BK, EPI>;
  if constexpr (EPI == 0 && sizeof(T) == 2) {
    if (p.dbg & 8) fn = gemm_pp_kernel<T, AK, BK, EPI, 2>;
    else if (p.dbg & 215) fn = gemm_pp_kernel<T, AK, BK, EPI, 1>;
  }
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  int nb = 0;
  if (p.bias_mode == 1) nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
  const size_t lds = (size_t)PP_NSLOT * PP_SLOT + (size_t)nb * sizeof(float);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(512), lds, st, p);
}

template <typename T, bool AK, bool BK, int EPI>
static void launch_pp2_epi(const GemmParams& p, int blocks, hipStream_t st) {
  void (*fn)(GemmParams) = gemm_pp2_kernel<T, AK, BK, EPI>;
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  int nb = 0;
  if (p.bias_mode == 1) nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
  const size_t lds = (size_t)PP_NSLOT * PP_SLOT + (size_t)nb * sizeof(float);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(512), lds, st, p);
}

template <typename T, bool AK, bool BK, class C>
static void launch_persist_cfg(const GemmParams& p, int blocks, hipStream_t st, int cfg) {
  int epi = (p.beta != 0.f ? 1 : 0) | (p.aux != nullptr ? 2 : 0);
  if (epi == 0 && p.relu) epi = 4;
  if (cfg == 45) {
    switch (epi) {
      case 0: launch_pp2_epi<T, AK, BK, 0>(p, blocks, st); break;
      case 1: launch_pp2_epi<T, AK, BK, 1>(p, blocks, st); break;
      case 2: launch_pp2_epi<T, AK, BK, 2>(p, blocks, st); break;
      case 3: launch_pp2_epi<T, AK, BK, 3>(p, blocks, st); break;
      default: launch_pp2_epi<T, AK, BK, 4>(p, blocks, st); break;
    }
    return;
  }
  if (cfg == 43) {
    switch (epi) {
      case 0: launch_pp_epi<T, AK, BK, 0>(p, blocks, st); break;
      case 1: launch_pp_epi<T, AK, BK, 1>(p, blocks, st); break;
      case 2: launch_pp_epi<T, AK, BK, 2>(p, blocks, st); break;
      case 3: launch_pp_epi<T, AK, BK, 3>(p, blocks, st); break;
      default: launch_pp_epi<T, AK, BK, 4>(p, blocks, st); break;
    }
    return;
  }
  switch (epi) {
    case 0: launch_persist_epi<T, AK, BK, C, 0>(p, blocks, st); break;
    case 1: launch_persist_epi<T, AK, BK, C, 1>(p, blocks, st); break;
    case 2: launch_persist_epi<T, AK, BK, C, 2>(p, blocks, st); break;
    case 3: launch_persist_epi<T, AK, BK, C, 3>(p, blocks, st); break;
    default: launch_persist_epi<T, AK, BK, C, 4>(p, blocks, st); break;
  }
}

template <typename T, class C>
static void launch_persist_t(const GemmParams& p, int ak, int bk, int blocks, hipStream_t st,
                             int cfg) {
  if (ak && bk) launch_persist_cfg<T, true, true, C>(p, blocks, st, cfg);
  else if (ak) launch_persist_cfg<T, true, false, C>(p, blocks, st, cfg);
  else if (bk) launch_persist_cfg<T, false, true, C>(p, blocks, st, cfg);
  else launch_persist_cfg<T, false, false, C>(p, blocks, st, cfg);
}

int launch_gemm_persist(const GemmParams& p, int dt, int ak, int bk, int cfg, int blocks,
                        hipStream_t st) {
  if (dt == JMT_BF16) launch_persist_t<__bf16, Cfg40>(p, ak, bk, blocks, st, cfg);
  else launch_persist_t<_Float16, Cfg40>(p, ak, bk, blocks, st, cfg);
  return 0;
}

template <typename T, bool AK, bool BK>
static void launch_pp_split_t(const GemmParams& p, bool rs, int blocks, hipStream_t st) {
  void (*fn)(GemmParams) =
      rs ? gemm_pp_split_kernel<T, AK, BK, 2> : gemm_pp_split_kernel<T, AK, BK, 1>;
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(512), (size_t)PP_NSLOT * PP_SLOT, st, p);
}

template <typename T>
static void launch_pp_split_l(const GemmParams& p, int ak, int bk, bool rs, int blocks,
                              hipStream_t st) {
  if (ak && bk) launch_pp_split_t<T, true, true>(p, rs, blocks, st);
  else if (ak) launch_pp_split_t<T, true, false>(p, rs, blocks, st);
  else if (bk) launch_pp_split_t<T, false, true>(p, rs, blocks, st);
  else launch_pp_split_t<T, false, false>(p, rs, blocks, st);
}

// the split-K ping-pong launch (cfg 44): p.splits, p.tiles_m / tiles_n (256 x 256), p.ws and
// (row sums) p.dbias_ws set by the caller; the caller launches the slab reduction after it
void launch_gemm_pp_split(const GemmParams& p, int dt, int ak, int bk, bool rs, int blocks,
                          hipStream_t st) {
  if (dt == JMT_BF16) launch_pp_split_l<__bf16>(p, ak, bk, rs, blocks, st);
  else launch_pp_split_l<_Float16>(p, ak, bk, rs, blocks, st);
}

// cfg 44 eligibility (also the planner's split choice, pp_split_plan): 16-bit A / B, whole
// 256 x 256 tiles, whole 64-deep K-tiles, and at least 2 K-tiles per split
bool pp_split_ok(int dt, int M, int N, int K, int splits) {
  return dt != JMT_F32 && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && splits >= 2 &&
         (K / 64) / splits >= 2;
}

// the split count for cfg 44 on a launch of few tiles over a long K: enough (tile, split) items
// for every CU, at least 4 K-tiles each; 0 when the shape has tiles enough without splitting.
// Gate: the K-tiles each CU's item covers ((K / 64) x tiles / CUs, the work one 256 KiB fp32 slab
// pays for) >= 27 — round 5 gated on >= 24 tiles, which at K = 19,200 is the same bound (28.1
// K-tiles per CU at 24 tiles, 14 at the 12 of TN 512 x 512 b3: 62 vs 57 us on the 128 x 128 split
// plan; 1024 x 512 b3 / b6, 1536 x 512 b3, 1024 x 3072: 6-10 % faster, profiles/r05/
// tn_pp_split_ab.txt), but it also admits the 12-tile wgrads over K = 38,400 that the
// cross-attentions' two uses of each module form (per-batch K-concat, grouped.py) and keeps
// c4's 24 tiles over K = 16,384 (24 K-tiles per CU) off, where ADVICE r5 found cfg 44 slower.
int pp_split_plan(int dt, int M, int N, int K, int batch) {
  // long K only: at realdata's K = 1024 rows a split is a few K-tiles, its pipeline prologue and
  // slab epilogue dominate (realdata 1.00 -> 1.22 ms/step; profiles/r05/cfg_gemm_ab.txt)
  if (dt == JMT_F32 || M % 256 || N % 256 || K % 64 || K < 8192) return 0;
  const long tiles = (long)(M / 256) * (N / 256) * batch;
  const int ncu = num_cus_persist();
  static int min_kt = -1;                     // development: JMT_GEMM_PPSPLIT_MIN_KT
  if (min_kt < 0) {
    const char* e = getenv("JMT_GEMM_PPSPLIT_MIN_KT");
    min_kt = e ? atoi(e) : 27;
  }
  if (tiles * 2 > ncu || (long)(K / 64) * tiles < (long)min_kt * ncu) return 0;
  long s = ncu / tiles;
  const long smax = (K / 64) / 4;
  if (s > smax) s = smax;
  return s >= 2 ? (int)s : 0;
}

// persistent grid: a multiple of 8 blocks (pitem / pwalk deal items per XCD slot w % 8)
int num_cus_persist() {
  const int n = num_cus() & ~7;
  return n > 0 ? n : 8;
}

}  // namespace jmt

// development: copy the ping-pong kernel's segment stamps (jmt::g_pp_stamps, dbg 8) to the host
extern "C" int jmt_gemm_pp_stamps_read(uint64_t* host, int n) {
  const int cap = (int)(sizeof(jmt::g_pp_stamps) / sizeof(uint64_t));
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(host, HIP_SYMBOL(jmt::g_pp_stamps), sizeof(uint64_t) * n) != hipSuccess)
    return -1;
  return n;
}

namespace jmt {

// JMT_GEMM_PP_MPART=0: partial row panels (M % 256 != 0) off the ping-pong kernel by default
static int mpart_env() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JMT_GEMM_PP_MPART");
    v = e ? atoi(e) : 1;
  }
  return v;
}

int persist_choice(const jmt_gemm_desc* d, const GemmParams& p, int splits, int forced) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("JMT_GEMM_PERSIST");
    env = e ? atoi(e) : 1;
  }
  const int dt = d->ab_dtype;
  const int batch0 = d->batch0 < 1 ? 1 : d->batch0;
  const long nbias = p.bias_mode == 1 ? (long)(d->n_bias > 0 ? batch0 : 1) * d->N : 0;
  // (beta * C / the ReLU mask: 8-B loads of C / aux rows in the epilogue — c_vec4 covers aux)
  // M % 256 != 0 (c2's 9,600 rows): cfg 45 only — its last row panel clamps the A rows and stores
  // through a buffer resource ending at row M (32-bit byte offsets over the panel's rows)
  const bool mfull = d->M % 256 == 0;
  const int64_t mpad = (int64_t)(d->M + 256) * (int64_t)dtype_size(dt);
  const bool mpart = !mfull && d->M % 8 == 0 && mpad * d->ldc < (1LL << 31) &&
                     (d->aux == nullptr || mpad * d->ldaux < (1LL << 31));
  const bool ok = dt != JMT_F32 && d->c_dtype == dt && splits == 1 && d->n_dbias == 0 &&
                  (mfull || mpart) && d->N % 256 == 0 && d->K % 64 == 0 && d->K >= 128 &&
                  p.c_vec8 && p.c_vec4 && p.bias_mode != 2 && nbias <= kPersistBias;
  if (!ok) return 0;
  if (forced == 45 || (mfull && (forced == 40 || forced == 43))) return forced;
  if (forced != 0 || env == 0) return 0;
  if (env == 45 || (mfull && (env == 40 || env == 43))) return env;
  if (!mfull && !mpart_env()) return 0;
  // default: the ping-pong kernel (cfg 43) wherever the launch has at least 1.5 tiles per CU
  // (below that the 160x256 / split tiles of the one-block-per-tile kernel quantise better: NT
  // 19200x512x2048 53 vs 68 us).  cfg 40 beat the one-block-per-tile kernel on every batched
  // step shape by 9-20 % (profiles/r04/gemm_persist_vs_vendor_a.jsonl); cfg 43 beats cfg 40 by
  // 14-25 % on the same shapes (profiles/r05/step_ab_persist40_vs_pp43.txt), and cfg 45 (32-MFMA phases) beats cfg 43 in the step: 4.266 ->
  // 4.193 ms, NT 0.91 -> 0.87, NN 0.87 -> 0.81 ms/step (profiles/r05/step_ab_pp43_vs_pp45.txt)
  // Round 6: cfg 45 also wins below that on the single-batch B*T-row shapes the gate used to
  // leave on the 160x256 tile (NT 19200x512x2048 53.5 -> 47.8 us with 150 tiles, NT x1024x3072
  // 144 -> 138, NN x512x3072 83 -> 71, NN x1024x256 32 -> 28; profiles/r06/b1_cfg_sweep.jsonl):
  // the gate is now half a tile per CU (JMT_GEMM_PP_MINW2 = 2 W / CUs threshold, 3 before).
  static int minw2 = -1;
  if (minw2 < 0) {
    const char* e = getenv("JMT_GEMM_PP_MINW2");
    minw2 = e ? atoi(e) : 1;
  }
  const long W = (long)((d->M + 255) / 256) * (d->N / 256) * batch0 *
                 (d->batch1 < 1 ? 1 : d->batch1);
  return W * 2 >= (long)minw2 * num_cus() ? 45 : 0;
}

}  // namespace jmt
