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

// EPI: 0 plain, 1 beta * C, 2 ReLU mask (aux), 3 both — compile-time, so that every load the
// epilogue issues is consumed on every path (a conditional load left hipcc unsure at the loop
// head and it waited vmcnt(4) there, draining the next K-tile's DMA every iteration)
template <typename T, class C, int EPI>
__device__ __forceinline__ void persist_epilogue(const GemmParams& p, const PItem& it,
                                                 f32x4 (&acc)[C::TM][C::TN],
                                                 const float* bias_lds, int lane, int wm, int wn) {
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
  const bool relu = p.relu != 0;
  const T* auxp = (const T*)p.aux;
  // beta * C and the ReLU-backward mask (aux > 0) of the one-block-per-tile epilogue, in its
  // order (+ beta C, ReLU, mask); their 8-B loads of row i + 1 are in flight while row i is
  // converted and stored.  hipcc waits for them by its own count (only its own loads and stores
  // follow them); the DMA it cannot see is older, issued a K-tile earlier.
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 cr[2][C::TN], ar[2][C::TN];
  constexpr bool ldc_ = (EPI & 1) != 0, lda_ = (EPI & 2) != 0;
  auto load_row = [&](int i, u32x2 (&c)[C::TN], u32x2 (&a)[C::TN]) {
    const int m = it.m0 + wm * C::WTM + 16 * i + rl;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int n = it.n0 + wn * C::WTN + 16 * j + 4 * g;
      if constexpr (ldc_) c[j] = *(const u32x2*)(cp + cbase + (int64_t)m * p.ldc + n);
      if constexpr (lda_) a[j] = *(const u32x2*)(auxp + cbase + (int64_t)m * p.ldaux + n);
    }
  };
  if constexpr (ldc_ || lda_) load_row(0, cr[0], ar[0]);
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    const int m = it.m0 + wm * C::WTM + 16 * i + rl;
    const int64_t rowo = cbase + (int64_t)m * p.ldc;
    if constexpr (ldc_ || lda_)
      if (i + 1 < C::TM) load_row(i + 1, cr[(i + 1) & 1], ar[(i + 1) & 1]);
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
        } else if (relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          T hh[2] = {from_f<T>(x[2 * q]), from_f<T>(x[2 * q + 1])};
          pk[h][q] = *(const uint32_t*)hh;
        }
      }
      const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      const int n = it.n0 + wn * C::WTN + 16 * (2 * jp + (g & 1)) + 8 * (g >> 1);
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
      JMT_DCHECK(m < p.M && n + 8 <= p.N);
      __builtin_nontemporal_store(v, (u32x4*)(cp + rowo + n));
    }
  }
}

template <typename T, bool AK, bool BK, class C, int EPI>
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
  PItem iss = pitem(p, blockIdx.x, W);
  auto advance_issue = [&]() {
    if (++iss_kt == nkt) {
      iss_kt = 0;
      ++iss_k;
      if (iss_k < nm) iss = pitem(p, blockIdx.x + iss_k * G, W);
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
  PItem cur = pitem(p, blockIdx.x, W);
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
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, C>(img, img + IA, wm, wn, acc);
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
      if (++cur_k < nm) cur = pitem(p, blockIdx.x + cur_k * G, W);
    }
  }
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
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  int nb = 0;
  if (p.bias_mode == 1) nb = (p.n_bias > 0 ? p.batch0 : 1) * p.N;
  const size_t lds = (size_t)C::S * C::STAGE + (size_t)nb * sizeof(float);
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(C::NT), lds, st, p);
}

template <typename T, bool AK, bool BK, class C>
static void launch_persist_cfg(const GemmParams& p, int blocks, hipStream_t st) {
  const int epi = (p.beta != 0.f ? 1 : 0) | (p.aux != nullptr ? 2 : 0);
  switch (epi) {
    case 0: launch_persist_epi<T, AK, BK, C, 0>(p, blocks, st); break;
    case 1: launch_persist_epi<T, AK, BK, C, 1>(p, blocks, st); break;
    case 2: launch_persist_epi<T, AK, BK, C, 2>(p, blocks, st); break;
    default: launch_persist_epi<T, AK, BK, C, 3>(p, blocks, st); break;
  }
}

template <typename T, class C>
static void launch_persist_t(const GemmParams& p, int ak, int bk, int blocks, hipStream_t st) {
  if (ak && bk) launch_persist_cfg<T, true, true, C>(p, blocks, st);
  else if (ak) launch_persist_cfg<T, true, false, C>(p, blocks, st);
  else if (bk) launch_persist_cfg<T, false, true, C>(p, blocks, st);
  else launch_persist_cfg<T, false, false, C>(p, blocks, st);
}

int launch_gemm_persist(const GemmParams& p, int dt, int ak, int bk, int cfg, int blocks,
                        hipStream_t st) {
  (void)cfg;   // 40
  if (dt == JMT_BF16) launch_persist_t<__bf16, Cfg40>(p, ak, bk, blocks, st);
  else launch_persist_t<_Float16, Cfg40>(p, ak, bk, blocks, st);
  return 0;
}

int num_cus_persist() { return num_cus(); }

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
  const bool ok = dt != JMT_F32 && d->c_dtype == dt && splits == 1 && d->n_dbias == 0 &&
                  d->M % 256 == 0 && d->N % 256 == 0 && d->K % 64 == 0 && d->K >= 128 &&
                  p.c_vec8 && p.c_vec4 && p.bias_mode != 2 && nbias <= kPersistBias;
  if (!ok) return 0;
  if (forced == 40) return forced;
  if (forced != 0 || env == 0) return 0;
  if (env == 40) return env;
  // default: the 128-B-K-tile form wherever the launch has at least 1.5 tiles per CU (below
  // that the 160x256 / split tiles of the one-block-per-tile kernel quantise better: NT
  // 19200x512x2048 53 vs 68 us); it beat the one-block-per-tile kernel on every batched step
  // shape by 9-20 % and cfg 41 everywhere (profiles/r04/gemm_persist_vs_vendor_a.jsonl)
  const long W = (long)(d->M / 256) * (d->N / 256) * batch0 * (d->batch1 < 1 ? 1 : d->batch1);
  return W * 2 >= 3L * num_cus() ? 40 : 0;
}

}  // namespace jmt
