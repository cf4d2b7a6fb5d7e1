// Fused scaled-dot-product attention for the JMT path (gfx950, wave64), head_dim 512, per
// (batch n, head h):
//   forward:  O = softmax(scale Q K^T) V, + lse (natural log of the row sums, scaled scores)
//   backward: P = exp(scale Q K^T - lse) recomputed, dP = dO V^T, Delta = rowsum(dO o O),
//             dS = scale P o (dP - Delta), dQ = dS K;  P and dS written once (bf16/f16) for the
//             dK = dS^T Q / dV = P^T dO GEMMs
// Replaces the score GEMM -> softmax -> PV GEMM chain behind every nn.MultiheadAttention of the
// reference (F.multi_head_attention_forward, called from mm_multi_transformers.py:57,142-167,
// 191 and intra_modal_transformer_fusion.py) and its autograd backward.
//
// Geometry (both kernels): a block is 8 waves (512 threads, 2 waves per SIMD at one block per
// CU) owning 64 rows of the row operand (Q forward, Q / dO backward).  Wave w owns rows
// 16 (w & 3) .. +15 and HALF h = w >> 2 of the 512 head dims: its row-operand fragments
// (16 rows x 256 dims) and its accumulator (O or dQ: 16 rows x 256 dims, 64 registers) stay in
// registers.  The contraction over head dims of the score products (Q K^T, dO V^T) is split
// between the two waves of a pair (w, w ^ 4): each writes its 16 x KT fp32 partial into an LDS
// exchange slot, the pair adds them in one canonical order (half 0 + half 1, so both hold
// bitwise the same scores), and both run the same softmax; the update products (P V, dS K)
// need no exchange: each wave produces its own 256 output dims.  This halves the registers of
// the round-1 kernel (453 VGPRs, one wave per SIMD) so two waves per SIMD hide LDS / MFMA
// latency.
//
//  * MFMA operands swapped (stream operand first): an accumulator lane owns ONE row and 4
//    consecutive keys / dims, softmax row state is lane-local (2 shuffles per row reduction),
//    probabilities (or dS) feed the update MFMA straight from registers (their k-slot order is
//    mirrored in the transposed fragment reads of the stream image).
//  * K / V images: [rows][1024 B] with no padding, 16-B chunk c of row r stored at chunk
//    c ^ ((r & 7) << 1): the ds_read_b128 score fragments and the ds_read_b64_tr_b16 update
//    fragments are both conflict-free.  Filled by LDS-DMA (one 1-KiB wave-instruction per row,
//    the swizzle applied to the per-lane SOURCE address, the LDS side linear).
//  * Forward: 64-key tiles, K and V in one image each (K of tile j+1 lands during the P V of
//    tile j, V of tile j+1 during the scores of tile j+1); online softmax with LAZY rescaling
//    (the reference max is raised only when a row max exceeds it by > 8 in log2 units).
//    LDS: K 64 KiB + V 64 KiB + exchange 32 KiB = 160 KiB.
//  * Backward: 32-key tiles double-buffered (tile j+1's K and V land during tile j), scores and
//    dP exchanged together.  LDS: 2 x (K 32 KiB + V 32 KiB) + exchange 32 KiB = 160 KiB.
//  * Persistent grid (one block per CU, item_range): an item = (n, h, 64-row q-tile); the next
//    item's row fragments and K / V tile 0 are issued during the current item's last tile, and
//    the outputs (O, dQ) are stored straight from registers (16-B stores of paired accumulators),
//    so consecutive items overlap their loads and stores (3-7 % over one block per item).
//  * Waits: raw s_barrier after an explicit lgkmcnt(0); LDS-DMA retired by vmcnt before the
//    barrier that precedes the read (never __syncthreads, whose fence would drain the DMA).
//  * XCD-aware item order: the q-tiles of one (n, h) run on one XCD and share K / V in its L2.
#include "attn_common.h"

namespace jmt {

constexpr int AT_QT = 64;           // rows per block
constexpr int AF_KT = 64;           // forward keys per tile
constexpr int AB_KT = 32;           // backward keys per tile
constexpr int AT_XCH = 4096;        // exchange bytes per wave
constexpr int AF_LDS = 2 * AF_KT * AT_ROWB + 8 * AT_XCH;   // 160 KiB
constexpr int AB_LDS = 4 * AB_KT * AT_ROWB + 8 * AT_XCH;   // 160 KiB

struct AttnFwdArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  int64_t sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n;
  int Lq, Lk, H, nitems;
  float scale_log2;
  uint64_t* stamps;
};

// Phase stamps (diagnostic build only, STAMP = true): s_memtime at each phase boundary of every
// tile of one block in the middle of the grid, stored by every lane of waves 0 and 4 at a
// lane-indexed address (vector stores).
template <bool STAMP>
__device__ __forceinline__ void stamp(uint64_t* buf, int idx) {
  if constexpr (STAMP) {
    if (buf && blockIdx.x == gridDim.x / 2 && ((threadIdx.x >> 6) & 3) == 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      buf[((threadIdx.x >> 8) * 256 + idx) * 64 + (threadIdx.x & 63)] = t;
    }
  }
}

// OPT (compile-time schedule bits, ATTN_FWD_OPT below): 1 lane-group reductions by permlane swaps
// instead of ds_bpermute shuffles; 2 s_setprio(1) for the second-dispatched half (waves 4-7, the
// arbitration loser of every phase: MI355X_MICROARCH "Two waves per SIMD" item 4); 4 the next
// K tile's LDS-DMA issued in pieces between the P V MFMA batches instead of in one burst after
// the score barrier; 8 the exponentials of keys 32-63 issued between the first P V batches
// (which read only keys 0-31), VALU beside the MFMAs.
template <typename T, bool STAMP = false, int OPT = 0>
__global__ __launch_bounds__(512, 2) void attn_fwd_kernel(AttnFwdArgs p) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kimg = smem;
  char* vimg = smem + AF_KT * AT_ROWB;
  char* xch = smem + 2 * AF_KT * AT_ROWB;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, rg = w & 3, h = w >> 2;
  const int nqt = (p.Lq + AT_QT - 1) / AT_QT;
  const int nkt = (p.Lk + AF_KT - 1) / AF_KT;
  int item, iend, istride;
  item_range(p.nitems, item, iend, istride);
  if (item >= iend) return;
  if constexpr ((OPT & 2) != 0)
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);

  // item -> (n, head, first query row)
  int nh = item / nqt, n = nh / p.H, hd = nh % p.H, q0 = (item % nqt) * AT_QT;
  const T* kb = (const T*)p.k + (int64_t)n * p.sk_n + hd * AT_DH;
  const T* vb = (const T*)p.v + (int64_t)n * p.sv_n + hd * AT_DH;

  F qf[8];
  auto load_q = [&](int n_, int hd_, int q0_) {
    const T* qrow = (const T*)p.q + (int64_t)n_ * p.sq_n + hd_ * AT_DH +
                    (int64_t)min(q0_ + 16 * rg + li, p.Lq - 1) * p.sq_l + 256 * h + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const F*)(qrow + 32 * ks);
  };
  load_q(n, hd, q0);
  stage_rows<T, AF_KT, 8, true>(kimg, kb, p.sk_l, 0, p.Lk);
  stage_rows<T, AF_KT, 8, true>(vimg, vb, p.sv_l, 0, p.Lk);

  f32x4* xmine = (f32x4*)(xch + w * AT_XCH) + lane;
  const f32x4* xpart = (const f32x4*)(xch + (w ^ 4) * AT_XCH) + lane;
  int kb4[4], tb8[8];
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, h);
#pragma unroll
  for (int c = 0; c < 8; ++c) tb8[c] = tr_base(c, li, g, h);

  // Per item: Q (registers) and K / V tile 0 (LDS) were issued during the previous item's last
  // tile (K tile 0 and Q right after its score phase freed the K image and Q registers, V tile 0
  // after its P V phase), so an item's loads overlap the previous item's softmax, P V and output
  // stores instead of opening every block with a cold load.
  while (true) {
    const int qr = q0 + 16 * rg + li;
    const int nxt = item + istride;
    const bool more = nxt < iend;
    const int nh2 = nxt / nqt, n2 = nh2 / p.H, hd2 = nh2 % p.H, q02 = (nxt % nqt) * AT_QT;
    const T* kb2 = (const T*)p.k + (int64_t)n2 * p.sk_n + hd2 * AT_DH;
    const T* vb2 = (const T*)p.v + (int64_t)n2 * p.sv_n + hd2 * AT_DH;

    f32x4 o[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;

    wait_vmcnt<AF_KT / 8>();                        // Q and K tile 0 landed (V 0 in flight)
    lds_barrier();
    stamp<STAMP>(p.stamps, 255);
    for (int j = 0; j < nkt; ++j) {
      stamp<STAMP>(p.stamps, 8 * j);
      // ---- partial scores over this wave's 256 dims: s[kt][r] = <row qr, key 64j+16kt+4g+r>
      f32x4 s[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      {   // k-step batches of 4 fragments (key subtiles 0..3), double-buffered: the reads of
          // batch ks+1 are in flight while the 4 MFMAs of batch ks run (pinned by sched_barrier)
        F fa[4], fb[4];
        auto kbatch = [&](F* dst, int ks) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            dst[kt] = *(const F*)(kimg + kb4[ks & 3] + 256 * (ks >> 2) + 16384 * kt);
        };
        kbatch(fa, 0);
#pragma unroll
        for (int ks = 0; ks < 8; ks += 2) {
          kbatch(fb, ks + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) s[kt] = mfma16(fa[kt], qf[ks], s[kt]);
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 2 < 8) kbatch(fa, ks + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) s[kt] = mfma16(fb[kt], qf[ks + 1], s[kt]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      stamp<STAMP>(p.stamps, 8 * j + 1);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) xmine[64 * kt] = s[kt];
      wait_vmcnt<0>();                              // V tile j landed
      stamp<STAMP>(p.stamps, 8 * j + 2);
      lds_barrier();                                // partials visible; K image free
      stamp<STAMP>(p.stamps, 8 * j + 3);
      // the K image is free: K tile j+1 (or the next item's tile 0) is staged now, or in pieces
      // between the P V batches below (OPT & 4)
      const bool stage_k = j + 1 < nkt || more;
      const T* kb_next = j + 1 < nkt ? kb : kb2;
      const int k0_next = j + 1 < nkt ? AF_KT * (j + 1) : 0;
      if constexpr ((OPT & 4) == 0) {
        if (stage_k) stage_rows<T, AF_KT, 8, true>(kimg, kb_next, p.sk_l, k0_next, p.Lk);
      }
      if (j + 1 == nkt && more) load_q(n2, hd2, q02);   // next item's Q (registers free)
      const int kbase = AF_KT * j + 4 * g;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const f32x4 ps = xpart[64 * kt];
        const f32x4 full = h == 0 ? s[kt] + ps : ps + s[kt];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = (kbase + 16 * kt + r < p.Lk) ? full[r] * p.scale_log2 : -INFINITY;
          s[kt][r] = x;
          mx = fmaxf(mx, x);
        }
      }
      if constexpr ((OPT & 1) != 0) {
        mx = pl_pair_max(mx);
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      if (__any(mx > m_run + 8.f)) {                // lazy rescale (header)
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int t = 0; t < 16; ++t) o[t] *= alpha;
      }
      F pf[2];
      float ls = 0.f;
      auto exps = [&](int kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(s[kt][r] - m_run);
          ls += pv;
          pf[kt >> 1][(kt & 1) * 4 + r] = from_f<T>(pv);
        }
      };
      // OPT & 8: the probabilities of keys 32-63 (pf[1]) are exponentiated between the first
      // P V batches, which only read pf[0] (VALU beside the MFMAs); same summation order
      exps(0);
      exps(1);
      if constexpr ((OPT & 8) == 0) {
        exps(2);
        exps(3);
        l_run += ls;
      }
      stamp<STAMP>(p.stamps, 8 * j + 4);
      // ---- o[t] += sum_k P(k) V[k][256h + 16t + 4g + r]: transposed fragment reads of the V
      // image in double-buffered batches of 4 fragments (q = 4b + i: t = q % 16, u = q / 16)
      {
        F fa[4], fb[4];
        auto vbatch = [&](F* dst, int b) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = 4 * b + i, u = q >> 4, t = q & 15;
            const char* a = vimg + tb8[t & 7] + 256 * (t >> 3) + 32768 * u;
            const Hf lo = tr_read<Hf>(a);
            const Hf hi = tr_read<Hf>(a + 16384);
            dst[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        };
        vbatch(fa, 0);
#pragma unroll
        for (int b = 0; b < 8; b += 2) {
          vbatch(fb, b + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = 4 * b + i;
            o[q & 15] = mfma16(fa[i], pf[q >> 4], o[q & 15]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((OPT & 4) != 0) {           // 2 of the 8 K-tile pieces per batch pair
            constexpr int NP = AF_KT / 8;
            if (stage_k)
              stage_rows_part<T, AF_KT, 8, true>(kimg, kb_next, p.sk_l, k0_next, p.Lk, (b / 2) * NP / 4,
                                        (b / 2 + 1) * NP / 4);
            __builtin_amdgcn_sched_barrier(0);
          }
          if constexpr ((OPT & 8) != 0) {
            if (b < 4) exps(2 + b / 2);             // pf[1] before the batches that read it
            if (b == 2) l_run += ls;
            __builtin_amdgcn_sched_barrier(0);
          }
          if (b + 2 < 8) vbatch(fa, b + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = 4 * (b + 1) + i;
            o[q & 15] = mfma16(fb[i], pf[q >> 4], o[q & 15]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      stamp<STAMP>(p.stamps, 8 * j + 5);
      if (j + 1 < nkt) {
        wait_vmcnt<0>();                            // K tile j+1 landed
        stamp<STAMP>(p.stamps, 8 * j + 6);
        lds_barrier();                              // V image and exchange slots free
        stage_rows<T, AF_KT, 8, true>(vimg, vb, p.sv_l, AF_KT * (j + 1), p.Lk);
      }
    }
    stamp<STAMP>(p.stamps, 254);
    float lt = l_run;
    if constexpr ((OPT & 1) != 0) {
      lt = pl_pair_sum(lt);
    } else {
      lt += __shfl_xor(lt, 16, 64);
      lt += __shfl_xor(lt, 32, 64);
    }
    JMT_DCHECK(item < p.nitems && n * p.H + hd == nh);
    if (qr < p.Lq && g == 0 && h == 0 && p.lse)
      p.lse[(int64_t)nh * p.Lq + qr] = (m_run + __builtin_amdgcn_logf(lt)) * 0.69314718055994531f;
    store_acc_direct<T>(o, 1.f / lt,
                        (T*)p.o + (int64_t)n * p.so_n + hd * AT_DH + (int64_t)qr * p.so_l + 256 * h,
                        qr < p.Lq);
    if (!more) break;
    lds_barrier();                                  // every wave is done with the V image
    stage_rows<T, AF_KT, 8, true>(vimg, vb2, p.sv_l, 0, p.Lk);
    item = nxt; nh = nh2; n = n2; hd = hd2; q0 = q02; kb = kb2; vb = vb2;
  }
}


// (A software-pipelined form — each tile's P V deferred into the next tile's iteration and
// interleaved with its exponentials, the last P V of an item run in the next item's first
// iteration — measured 3-8 % slower than this kernel at N = 96-384: profiles/
// r02_attn_pipelined_fwd.txt.)
// (A 4-wave, one-wave-per-SIMD forward with v_mfma_f32_32x32x16, 32 rows x all 512 dims per wave
// and 128 rows per block — half the K/V bytes into LDS and half the LDS fragment bytes per FLOP —
// needs ~480 registers per wave (O 256 + Q 128 + working set) and spilled 256 VGPRs under hipcc:
// not kept.  Phase stamps of this 16x16 kernel: profiles/r02_attn_phase_stamps.txt.)


// OPT: as attn_fwd_kernel (1 permlane reductions of Delta, 2 s_setprio(1) for waves 4-7, 4 the
// next tile's K / V LDS-DMA issued in pieces between the score / dP MFMA batches); 16 each
// tile's P / dS row stores deferred to the start of the next tile: the end-of-tile
// vmcnt(0) that waits for the next tile's DMA otherwise also waits for the acknowledgement of
// the stores issued just before it (stores count in vmcnt, in issue order)
template <typename T, int OPT = 0>
__global__ __launch_bounds__(512, 2) void attn_bwd_kernel(AttnBwdArgs p) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int IMG = AB_KT * AT_ROWB;            // one K or V image
  char* xch = smem + 4 * IMG;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, rg = w & 3, h = w >> 2;
  const int nqt = (p.Lq + AT_QT - 1) / AT_QT;
  const int nkt = (p.Lk + AB_KT - 1) / AB_KT;
  int item, iend, istride;
  item_range(p.nitems, item, iend, istride);
  if (item >= iend) return;
  if constexpr ((OPT & 2) != 0)
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);

  int nh = item / nqt, n = nh / p.H, hd = nh % p.H, q0 = (item % nqt) * AT_QT;
  const T* kb = (const T*)p.k + (int64_t)n * p.sk_n + hd * AT_DH;
  const T* vb = (const T*)p.v + (int64_t)n * p.sv_n + hd * AT_DH;

  // row-operand fragments of an item: Q, dO (kept for the whole item) and O (Delta only)
  F qf[8], df[8], of[8];
  auto rows_off = [&](int q0_) { return (int64_t)min(q0_ + 16 * rg + li, p.Lq - 1); };
  auto load_qd = [&](int n_, int hd_, int q0_) {
    const int64_t qc_ = rows_off(q0_), coff = (int64_t)hd_ * AT_DH + 256 * h + 8 * g;
    const T* qrow = (const T*)p.q + (int64_t)n_ * p.sq_n + qc_ * p.sq_l + coff;
    const T* drow = (const T*)p.go + (int64_t)n_ * p.sgo_n + qc_ * p.sgo_l + coff;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = *(const F*)(qrow + 32 * ks);
      df[ks] = *(const F*)(drow + 32 * ks);
    }
  };
  auto load_o = [&](int n_, int hd_, int q0_) {
    const int64_t qc_ = rows_off(q0_), coff = (int64_t)hd_ * AT_DH + 256 * h + 8 * g;
    const T* orow = (const T*)p.o + (int64_t)n_ * p.so_n + qc_ * p.so_l + coff;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) of[ks] = *(const F*)(orow + 32 * ks);
  };
  load_qd(n, hd, q0);
  load_o(n, hd, q0);
  int buf = 0;                                    // buffer pair of the next tile to compute
  stage_rows<T, AB_KT>(smem, kb, p.sk_l, 0, p.Lk);
  stage_rows<T, AB_KT>(smem + IMG, vb, p.sv_l, 0, p.Lk);

  f32x4* xmine = (f32x4*)(xch + w * AT_XCH) + lane;
  const f32x4* xpart = (const f32x4*)(xch + (w ^ 4) * AT_XCH) + lane;
  int kb4[4], tb8[8];
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, h);
#pragma unroll
  for (int c = 0; c < 8; ++c) tb8[c] = tr_base(c, li, g, h);

  // Persistent items (item_range): the next item's Q / dO / O fragments are loaded right after
  // the last tile's score phase (their registers are free from there on) and its K / V tile 0
  // into the free buffer pair at the start of the last tile, so an item opens on landed data.
  while (true) {
    const int qr = q0 + 16 * rg + li;
    const int qc = min(qr, p.Lq - 1);
    const int64_t prow = (int64_t)nh * p.Lq + qc;
    const int nxt = item + istride;
    const bool more = nxt < iend;
    const int nh2 = nxt / nqt, n2 = nh2 / p.H, hd2 = nh2 % p.H, q02 = (nxt % nqt) * AT_QT;
    const T* kb2 = (const T*)p.k + (int64_t)n2 * p.sk_n + hd2 * AT_DH;
    const T* vb2 = (const T*)p.v + (int64_t)n2 * p.sv_n + hd2 * AT_DH;

    float delta;
    {
      float dp = 0.f;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) dp += (float)of[ks][e] * (float)df[ks][e];
      if constexpr ((OPT & 1) != 0) {
        dp = pl_pair_sum(dp);
      } else {
        dp += __shfl_xor(dp, 16, 64);
        dp += __shfl_xor(dp, 32, 64);
      }
      delta = dp;                                   // this half's part of rowsum(dO o O)
    }
    const float lse2 = p.lse[prow] * 1.4426950408889634f;
    ((float*)xch)[w * 64 + lane] = delta;

    f32x4 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    T* prow_p = (T*)p.pbuf + prow * p.ldp;
    T* prow_ds = (T*)p.dsbuf + prow * p.ldp;

    wait_vmcnt<0>();                                // tile 0 landed
    lds_barrier();                                  // ... and every Delta part written
    {
      const float part = ((const float*)xch)[(w ^ 4) * 64 + lane];
      delta = h == 0 ? delta + part : part + delta;
    }
    lds_barrier();                                  // Delta parts read: exchange slots free

    uint2 pend[2];                                  // OPT & 16: the previous tile's P / dS
    int pend_key[2] = {0, 0};
    bool pend_on = false;
    auto flush = [&]() {
      if (pend_on) {
        T* rowp = h == 0 ? prow_p : prow_ds;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
          if (qr < p.Lq && pend_key[kt] < p.ldp) *(uint2*)(rowp + pend_key[kt]) = pend[kt];
        pend_on = false;
      }
    };
    for (int j = 0; j < nkt; ++j) {
      const char* kimg = smem + buf * 2 * IMG;
      const char* vimg = kimg + IMG;
      if constexpr ((OPT & 16) != 0) flush();       // older than this tile's DMA
      char* nk = smem + (buf ^ 1) * 2 * IMG;        // tile j+1 (or the next item's tile 0)
      const bool stage_n = j + 1 < nkt || more;
      const T* kbn = j + 1 < nkt ? kb : kb2;
      const T* vbn = j + 1 < nkt ? vb : vb2;
      const int k0n = j + 1 < nkt ? AB_KT * (j + 1) : 0;
      if constexpr ((OPT & 4) == 0) {
        if (stage_n) {
          stage_rows<T, AB_KT>(nk, kbn, p.sk_l, k0n, p.Lk);
          stage_rows<T, AB_KT>(nk + IMG, vbn, p.sv_l, k0n, p.Lk);
        }
      }
      // ---- partial scores (K) and partial dP (V) over this wave's 256 dims
      f32x4 s[2], d[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        d[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      {   // k-step batches (K and V fragments of key subtiles 0, 1), double-buffered
        F fa[4], fb[4];
        auto batch = [&](F* dst, int ks) {
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            const int o = kb4[ks & 3] + 256 * (ks >> 2) + 16384 * kt;
            dst[kt] = *(const F*)(kimg + o);
            dst[2 + kt] = *(const F*)(vimg + o);
          }
        };
        batch(fa, 0);
#pragma unroll
        for (int ks = 0; ks < 8; ks += 2) {
          batch(fb, ks + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[kt] = mfma16(fa[kt], qf[ks], s[kt]);
            d[kt] = mfma16(fa[2 + kt], df[ks], d[kt]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 2 < 8) batch(fa, ks + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[kt] = mfma16(fb[kt], qf[ks + 1], s[kt]);
            d[kt] = mfma16(fb[2 + kt], df[ks + 1], d[kt]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr ((OPT & 4) != 0) {           // K then V pieces, 2 per batch pair
            constexpr int NP = AB_KT / 8;           // pieces per image per wave (4)
            if (stage_n) {
              if (ks < 4)
                stage_rows_part<T, AB_KT>(nk, kbn, p.sk_l, k0n, p.Lk, (ks / 2) * NP / 2,
                                          (ks / 2 + 1) * NP / 2);
              else
                stage_rows_part<T, AB_KT>(nk + IMG, vbn, p.sv_l, k0n, p.Lk,
                                          (ks / 2 - 2) * NP / 2, (ks / 2 - 1) * NP / 2);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      xmine[0] = s[0];
      xmine[64] = s[1];
      xmine[128] = d[0];
      xmine[192] = d[1];
      lds_barrier();                                // partials visible (tile j+1 DMA in flight)
      if (j + 1 == nkt && more) load_qd(n2, hd2, q02);     // next item's Q / dO fragments
      const int kbase = AB_KT * j + 4 * g;
      F dsf;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const f32x4 ps = xpart[64 * kt], pd = xpart[128 + 64 * kt];
        const f32x4 sf = h == 0 ? s[kt] + ps : ps + s[kt];
        const f32x4 dfull = h == 0 ? d[kt] + pd : pd + d[kt];
        T pv4[4], ds4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool in = kbase + 16 * kt + r < p.Lk;
          const float pv = in ? __builtin_amdgcn_exp2f(sf[r] * p.scale_log2 - lse2) : 0.f;
          const float ds = p.scale * pv * (dfull[r] - delta);
          pv4[r] = from_f<T>(pv);
          ds4[r] = from_f<T>(ds);
          dsf[kt * 4 + r] = ds4[r];
        }
        const int key = kbase + 16 * kt;
        JMT_DCHECK(qc >= 0 && qc < p.Lq && item < p.nitems);
        if constexpr ((OPT & 16) != 0) {
          pend[kt] = h == 0 ? *(const uint2*)pv4 : *(const uint2*)ds4;
          pend_key[kt] = key;
        } else if (qr < p.Lq && key < p.ldp) {
          if (h == 0) *(uint2*)(prow_p + key) = *(const uint2*)pv4;
          else *(uint2*)(prow_ds + key) = *(const uint2*)ds4;
        }
      }
      if constexpr ((OPT & 16) != 0) pend_on = true;
      // ---- acc[t] += sum_k dS(k) K[k][256h + 16t + 4g + r] (transposed K fragments in
      // double-buffered batches of 4)
      {
        F fa[4], fb[4];
        auto kbatch = [&](F* dst, int b) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int t = 4 * b + i;
            const char* a = kimg + tb8[t & 7] + 256 * (t >> 3);
            const Hf lo = tr_read<Hf>(a);
            const Hf hi = tr_read<Hf>(a + 16384);
            dst[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        };
        kbatch(fa, 0);
#pragma unroll
        for (int b = 0; b < 4; b += 2) {
          kbatch(fb, b + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[4 * b + i] = mfma16(fa[i], dsf, acc[4 * b + i]);
          __builtin_amdgcn_sched_barrier(0);
          if (b + 2 < 4) kbatch(fa, b + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[4 * b + 4 + i] = mfma16(fb[i], dsf, acc[4 * b + 4 + i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (j + 1 < nkt) {
        wait_vmcnt<0>();                            // tile j+1 landed (and P / dS stores issued)
        lds_barrier();                              // this buffer pair and the slots are free
      }
      buf ^= 1;
    }
    if constexpr ((OPT & 16) != 0) flush();         // the item's last tile
    store_acc_direct<T>(acc, 1.f,
                        (T*)p.dq + (int64_t)n * p.sdq_n + hd * AT_DH + (int64_t)qr * p.sdq_l +
                            256 * h,
                        qr < p.Lq);
    if (!more) break;
    load_o(n2, hd2, q02);                           // O of the next item (Delta), after acc is dead
    lds_barrier();                                  // every wave is done with the last tile's
                                                    // images and exchange slots
    item = nxt; nh = nh2; n = n2; hd = hd2; q0 = q02; kb = kb2; vb = vb2;
  }
}

// ------------------------------------------------------------------ P / dS only (round 6)
// The backward of the jmt_attn_dkdv path: P and dS for jmt_attn_dkdv, which computes dQ = dS K
// as its third product, so this kernel keeps no dQ accumulator.  The freed registers hold the
// WHOLE 512-dim Q and dO rows of a wave (16 fragments each, 128 VGPRs), so:
//  * a block is 8 waves x 16 rows = 128 query rows (the dQ kernel above: 64) — every K / V tile
//    staged into LDS feeds twice the rows, halving the L2 -> LDS fill per FLOP, which bounded it
//    (~64 KiB per 32-key tile per 64-row block at ~4 TB/s chip-wide);
//  * no exchange: each wave contracts all 512 dims itself (S and dP in one MFMA chain each), so
//    no partial-score slots, no pair barrier — one barrier per tile (the K / V buffer turnover);
//  * waves whose 16 rows all lie past Lq (the 44-row tail q-tile of L = 300) skip their MFMAs
//    and stores (wave-uniform), so the tail costs what its rows need.
// Per 32-key tile a wave reads the K and V tiles whole (64 KiB) and issues 64 MFMAs: the LDS
// array (256 B/clk/CU) and the MFMA pipes are both at 2048 cycles per tile at 2 waves/SIMD.
// P / dS leave by 16-B buffer stores, 64 contiguous bytes per row (range-checked rows: the count
// is fixed, so the end-of-tile wait leaves this tile's 2 stores in flight and waits only for the
// next tile's DMA).
// LDS: 2 x (K 32 KiB + V 32 KiB) = 128 KiB.
constexpr int AP_QT = 128;
constexpr int AP_KT = 32;
constexpr int AP_LDS = 4 * AP_KT * AT_ROWB;

// DBG (ablations, timing only, wrong results; JMT_ATTN_PDS_DBG in the diagnostic build): 1 no
// next-item row loads (stale Q / dO / O), 2 no MFMAs, 4 no softmax and no P / dS stores, 8 no
// K / V DMA, 16 softmax computed but not stored, 32 nontemporal stores; 64 phase stamps
// (s_memtime of block gridDim / 2, waves 0 and 4, into p.dq as a uint64 buffer of
// 2 x 256 x 64: phases 8 t + {0 tile start, 1 DMA issued, 2 MFMAs issued, 3 softmax + stores
// issued, 4 end wait, 5 barrier} of the block's first 31 tiles, 255 / 254 item start / end)
template <typename T, int DBG = 0>
__global__ __launch_bounds__(512, 2) void attn_bwd_pds_kernel(AttnBwdArgs p) {
  int tcount = 0;
  auto st = [&](int phase) {
    if constexpr ((DBG & 64) != 0) {
      if (tcount < 31) stamp<true>((uint64_t*)p.dq, 8 * tcount + phase);
    }
  };
  typedef typename Frag16<T>::t F;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int IMG = AP_KT * AT_ROWB;            // one K or V image (32 KiB)

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int nqt = (p.Lq + AP_QT - 1) / AP_QT;
  const int nkt = (p.Lk + AP_KT - 1) / AP_KT;
  int item, iend, istride;
  item_range(p.nitems, item, iend, istride);
  if (item >= iend) return;

  int nh = item / nqt, n = nh / p.H, hd = nh % p.H, q0 = (item % nqt) * AP_QT;
  const T* kb = (const T*)p.k + (int64_t)n * p.sk_n + hd * AT_DH;
  const T* vb = (const T*)p.v + (int64_t)n * p.sv_n + hd * AT_DH;

  // lane (li, g): row q0 + 16 w + li, dims 32 ks + 8 g .. +7 of fragment ks
  // The next item's Q / dO go out right after the last tile's MFMAs, its O (Delta only) after
  // the item's last softmax.
  F qf[16], df[16], of[16];
  auto load_qd = [&](int n_, int hd_, int q0_) {
    const int64_t qc_ = min(q0_ + 16 * w + li, p.Lq - 1), coff = (int64_t)hd_ * AT_DH + 8 * g;
    const T* qrow = (const T*)p.q + (int64_t)n_ * p.sq_n + qc_ * p.sq_l + coff;
    const T* drow = (const T*)p.go + (int64_t)n_ * p.sgo_n + qc_ * p.sgo_l + coff;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      qf[ks] = *(const F*)(qrow + 32 * ks);
      df[ks] = *(const F*)(drow + 32 * ks);
    }
  };
  auto load_o = [&](int n_, int hd_, int q0_) {
    const int64_t qc_ = min(q0_ + 16 * w + li, p.Lq - 1), coff = (int64_t)hd_ * AT_DH + 8 * g;
    const T* orow = (const T*)p.o + (int64_t)n_ * p.so_n + qc_ * p.so_l + coff;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) of[ks] = *(const F*)(orow + 32 * ks);
  };
  load_qd(n, hd, q0);
  load_o(n, hd, q0);
  int buf = 0;
  // K / V tile staging: wave w stages rows 4 w .. +3 of both images (one 1-KiB LDS-DMA row per
  // wave-instruction).  Row offsets in 32-bit byte arithmetic from the (n, h) base (the host
  // checks Lk rows fit) and the per-lane swizzled source offsets and LDS addresses computed once:
  // stage_rows' 64-bit row products cost ~25 scalar instructions per DMA on the CU's one scalar
  // unit (1-2.4k cycles of issue per tile, profiles/r06/pds_stamps*.txt)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  unsigned loff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) loff[i] = (unsigned)(lane ^ (((4 * wu + i) & 7) << 1)) << 4;
  const int ldk = (int)(p.sk_l * (int64_t)sizeof(T)), ldv = (int)(p.sv_l * (int64_t)sizeof(T));
  auto stage_tile = [&](int b, const T* kbase, const T* vbase, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * wu + i;
      const int src = min(k0 + r, p.Lk - 1);
      const uint32_t dst = lbase + b * 2 * IMG + r * AT_ROWB;
      glds16_at((const char*)kbase + (unsigned)(src * ldk) + loff[i], dst);
      glds16_at((const char*)vbase + (unsigned)(src * ldv) + loff[i], dst + IMG);
    }
  };
  stage_tile(0, kb, vb, 0);

  int kb4[4];                                     // ds_read_b128 lane bases (whole row)
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, 0);

  while (true) {
    const int qr = q0 + 16 * w + li;
    const int qc = min(qr, p.Lq - 1);
    // wave-uniform (scalar: the branches on it are s_cbranch, not EXEC masks): any row in range
    const bool wact = __builtin_amdgcn_readfirstlane(q0 + 16 * w) < p.Lq;
    const int nxt = item + istride;
    const bool more = nxt < iend;
    const int nh2 = nxt / nqt, n2 = nh2 / p.H, hd2 = nh2 % p.H, q02 = (nxt % nqt) * AP_QT;
    const T* kb2 = (const T*)p.k + (int64_t)n2 * p.sk_n + hd2 * AT_DH;
    const T* vb2 = (const T*)p.v + (int64_t)n2 * p.sv_n + hd2 * AT_DH;

    float delta;                                  // rowsum(dO o O) of row qr
    {
      float dp = 0.f;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) dp += (float)of[ks][e] * (float)df[ks][e];
      delta = pl_pair_sum(dp);
    }
    const float lse2 = p.lse[(int64_t)nh * p.Lq + qc] * 1.4426950408889634f;
    // P / dS of this (n, h), TILE-MAJOR: [key tile jt][query][32 keys] (64-B rows, ldp / 32
    // tiles), so one store instruction writes 16 consecutive rows = 1 KiB contiguous.  Buffer
    // resources over the (n, h) region; rows past Lq get an offset past its end and are dropped
    // by the range check, so every wave issues the same 2 stores per tile.
    const int64_t region = (int64_t)nh * p.Lq * p.ldp;
    const int nbytes = (int)((int64_t)p.Lq * p.ldp * (int64_t)sizeof(T));
    auto mk_rsrc = [&](void* base) {
      const uint64_t ba = (uint64_t)(uintptr_t)((T*)base + region);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ba);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
      return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                               __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
    };
    const auto rs_p = mk_rsrc(p.pbuf);
    const auto rs_ds = mk_rsrc(p.dsbuf);
    const int rowoff = qr * AP_KT;                // elements (used for rows below Lq only)

    wait_vmcnt<0>();                              // tile 0 and this item's rows landed
    lds_barrier();                                // ... for every wave; the previous item's
                                                  // buffers are free
    // One 32-key tile; the last one (LAST) is peeled out of the loop: the next item's Q / dO
    // loads issued inside the loop would be pending at its header for hipcc's wait insertion,
    // which then put a vmcnt(0) before every tile's first MFMA — waiting for the tile's own
    // freshly issued DMA (no load / compute overlap at all).
    auto tile = [&](int j, auto last_c) {
      constexpr bool LAST = decltype(last_c)::value;
      st(0);
      const char* kimg = smem + buf * 2 * IMG;
      const char* vimg = kimg + IMG;
      if ((DBG & 8) == 0 && (!LAST || more))
        stage_tile(buf ^ 1, LAST ? kb2 : kb, LAST ? vb2 : vb, LAST ? 0 : AP_KT * (j + 1));
      st(1);
      // ---- scores s[kt][r] = <row qr, key 32 j + 16 kt + 4 g + r> and dP over all 512 dims
      f32x4 s[2], d[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        d[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if ((DBG & 2) == 0 && wact) {   // k-step batches (K and V fragments of key subtiles 0, 1),
                                      // double-buffered
        F fa[4], fb[4];
        auto batch = [&](F* dst, int ks) {
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            const int o = kb4[ks & 3] + 256 * (ks >> 2) + 16384 * kt;
            dst[kt] = *(const F*)(kimg + o);
            dst[2 + kt] = *(const F*)(vimg + o);
          }
        };
        batch(fa, 0);
#pragma unroll
        for (int ks = 0; ks < 16; ks += 2) {
          batch(fb, ks + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[kt] = mfma16(fa[kt], qf[ks], s[kt]);
            d[kt] = mfma16(fa[2 + kt], df[ks], d[kt]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 2 < 16) batch(fa, ks + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[kt] = mfma16(fb[kt], qf[ks + 1], s[kt]);
            d[kt] = mfma16(fb[2 + kt], df[ks + 1], d[kt]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      st(2);
      if constexpr (LAST && (DBG & 1) == 0) {
        if (more) load_qd(n2, hd2, q02);          // registers free after the MFMAs
      }
      if ((DBG & 4) == 0 && wact) {
        const int kbase = AP_KT * j + 4 * g;
        uint32_t pk[2][2][2];                     // [P / dS][kt][dword]: 4 keys of subtile kt
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          T pv4[4], ds4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool in = kbase + 16 * kt + r < p.Lk;
            const float pv = in ? __builtin_amdgcn_exp2f(s[kt][r] * p.scale_log2 - lse2) : 0.f;
            pv4[r] = from_f<T>(pv);
            ds4[r] = from_f<T>(p.scale * pv * (d[kt][r] - delta));
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            pk[0][kt][q] = ((const uint32_t*)pv4)[q];
            pk[1][kt][q] = ((const uint32_t*)ds4)[q];
          }
        }
        // subtiles 0 / 1 paired by v_permlane16_swap (store_acc_direct's scheme): lane g then
        // holds the 8 consecutive keys 16 (g & 1) + 8 (g >> 1) .. +7 of the tile: 16 B per lane,
        // a whole 64-B tile row per 4 lanes, 16 rows contiguous (row-major [q][ldp] stores of
        // 32-B / 64-B row pieces took 3/4 of the kernel: 215 -> 57 us without stores,
        // profiles/r06/pds_ablate.txt)
        const int off = qr < p.Lq ? (rowoff + j * p.Lq * AP_KT + 16 * (g & 1) + 8 * (g >> 1)) *
                                        (int)sizeof(T)
                                  : 0x7ffffff0;
        JMT_DCHECK(AP_KT * j + AP_KT <= p.ldp);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const auto r0 = __builtin_amdgcn_permlane16_swap(pk[a][0][0], pk[a][1][0], false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(pk[a][0][1], pk[a][1][1], false, false);
          const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
          if constexpr ((DBG & 16) != 0) {
            asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(v, a == 0 ? rs_p : rs_ds, off, 0,
                                                   (DBG & 32) ? 2 : 0);
          }
        }
      }
      st(3);
      if constexpr (!LAST) {
        // tile j+1 landed: the 2 stores issued after its DMA may stay in flight
        if ((DBG & 20) == 0 && wact) wait_vmcnt<2>();
        else wait_vmcnt<0>();
        st(4);
        lds_barrier();                            // visible to every wave; buffer `buf` free
        st(5);
      }
      ++tcount;
      buf ^= 1;
    };
    for (int j = 0; j + 1 < nkt; ++j) tile(j, std::false_type{});
    tile(nkt - 1, std::true_type{});
    if (!more) break;
    // after the loop, not in its last iteration: loaded inside, O would be a loop-carried value
    // pinned over every tile (64 VGPRs: the kernel spilled, and each spill reload's vmcnt(0)
    // waited for the tile's DMA right after issuing it)
    if constexpr ((DBG & 1) == 0) load_o(n2, hd2, q02);
    item = nxt; nh = nh2; n = n2; hd = hd2; q0 = q02; kb = kb2; vb = vb2;
  }
}

template <typename K>
static void set_lds(K fn, int bytes) {
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

static int check_common(const char* name, int N, int H, int Lq, int Lk, const void* const* ptrs,
                        int nptr, const int64_t* strides, int nstr) {
  JMT_CHECK_ARG(N > 0 && H > 0 && Lq > 0 && Lk > 0 &&
                    (int64_t)N * H * ((Lq + AT_QT - 1) / AT_QT) < (1LL << 31),
                "%s: bad sizes", name);
  for (int i = 0; i < nptr; ++i)
    JMT_CHECK_ARG(ptrs[i] != nullptr && ((uintptr_t)ptrs[i] & 15) == 0,
                  "%s: operand %d null or not 16-B aligned", name, i);
  for (int i = 0; i < nstr; ++i)
    JMT_CHECK_ARG(strides[i] % 8 == 0, "%s: stride %d not a multiple of 8 elements", name, i);
  return JMT_OK;
}

}  // namespace jmt

using namespace jmt;

[[maybe_unused]] static void* g_stamps = nullptr;

// Schedule options of the bf16 / fp16 kernels (OPT bits, compile time; forward: 1 permlane
// reductions, 2 setprio for waves 4-7, 4 interleaved K-tile DMA, 8 split exponentials;
// backward: 1, 2, 4, 16 deferred P / dS stores).  The measured-fastest combination is the only
// one compiled (profiles/r03_attn_opt_ab.jsonl, interleaved A/B at the c3 launches: forward
// 1|2|8, backward 1|2|4).
constexpr int ATTN_FWD_OPT = 11;
constexpr int ATTN_BWD_OPT = 7;

template <int OPT>
static void launch_fwd_bf16(dim3 grid, hipStream_t st, const AttnFwdArgs& a) {
  static bool once = (set_lds(attn_fwd_kernel<__bf16, false, OPT>, AF_LDS), true);
  (void)once;
  hipLaunchKernelGGL((attn_fwd_kernel<__bf16, false, OPT>), grid, dim3(512), (size_t)AF_LDS, st,
                     a);
}
template <int OPT>
static void launch_bwd_bf16(dim3 grid, hipStream_t st, const AttnBwdArgs& a) {
  static bool once = (set_lds(attn_bwd_kernel<__bf16, OPT>, AB_LDS), true);
  (void)once;
  hipLaunchKernelGGL((attn_bwd_kernel<__bf16, OPT>), grid, dim3(512), (size_t)AB_LDS, st, a);
}

// one block per CU (the 160 KiB of LDS admit one), rounded down to a multiple of 8 (XCDs), when
// there are more items than CUs; otherwise one block per item
static unsigned persistent_grid(int nitems) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 8)
      v = 8;
    ncu = v / 8 * 8;
    const char* e = getenv("JMT_ATTN_PERSIST");   // dev A/B switch: 0 = one block per item
    if (e && e[0] == '0') ncu = 1 << 30;
  }
  return (unsigned)(nitems > ncu ? ncu : nitems);
}

// diagnostic: route jmt_attn_fwd (bf16) through the phase-stamped kernel, stamps into `buf`
// (2 x 256 x 64 uint64); NULL turns it off.  Only in the diagnostic build (make diag,
// -DJMT_DIAG=1); not part of include/jmt.h (dev tool).
extern "C" int jmt_attn_set_stamps(void* buf) {
#if JMT_DIAG
  g_stamps = buf;
  return JMT_OK;
#else
  return buf ? set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_set_stamps: diagnostic build only "
                                              "(make diag)") : JMT_OK;
#endif
}

extern "C" int jmt_attn_supported(int dt, int dh) {
  return (dt == JMT_BF16 || dt == JMT_F16) && dh == AT_DH;
}

extern "C" int jmt_attn_fwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* q,
                            int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n,
                            const void* v, int64_t sv_l, int64_t sv_n, void* o, int64_t so_l,
                            int64_t so_n, float scale, float* lse, void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_supported(dt, dh))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_fwd: dtype %d / head dim %d not supported",
                     dt, dh);
  const void* ptrs[] = {q, k, v, o};
  const int64_t strides[] = {sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n};
  int rc = check_common("jmt_attn_fwd", N, H, Lq, Lk, ptrs, 4, strides, 8);
  if (rc != JMT_OK) return rc;
  AttnFwdArgs a = {};
  a.q = q; a.k = k; a.v = v; a.o = o; a.lse = lse;
  a.sq_l = sq_l; a.sq_n = sq_n; a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n;
  a.so_l = so_l; a.so_n = so_n;
  a.Lq = Lq; a.Lk = Lk; a.H = H;
  a.scale_log2 = scale * 1.4426950408889634f;
  hipStream_t st = as_stream(stream);
  a.nitems = ((Lq + AT_QT - 1) / AT_QT) * N * H;
  const dim3 grid(persistent_grid(a.nitems));
#if JMT_DIAG
  if (g_stamps && dt == JMT_BF16) {   // diagnostic: phase stamps (jmt_attn_set_stamps)
    a.stamps = (uint64_t*)g_stamps;
    static bool once = (set_lds(attn_fwd_kernel<__bf16, true, ATTN_FWD_OPT>, AF_LDS), true);
    (void)once;
    hipLaunchKernelGGL((attn_fwd_kernel<__bf16, true, ATTN_FWD_OPT>), grid, dim3(512),
                       (size_t)AF_LDS, st, a);
    JMT_LAUNCH_CHECK("jmt_attn_fwd");
    return JMT_OK;
  }
#endif
  if (dt == JMT_BF16) {
    launch_fwd_bf16<ATTN_FWD_OPT>(grid, st, a);
  } else {
    static bool once = (set_lds(attn_fwd_kernel<_Float16, false, ATTN_FWD_OPT>, AF_LDS), true);
    (void)once;
    hipLaunchKernelGGL((attn_fwd_kernel<_Float16, false, ATTN_FWD_OPT>), grid, dim3(512),
                       (size_t)AF_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_fwd");
  return JMT_OK;
}

extern "C" int jmt_attn_bwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* go,
                            int64_t sgo_l, int64_t sgo_n, const void* o, int64_t so_l,
                            int64_t so_n, const void* q, int64_t sq_l, int64_t sq_n,
                            const void* k, int64_t sk_l, int64_t sk_n, const void* v,
                            int64_t sv_l, int64_t sv_n, const float* lse, void* p_out,
                            void* ds_out, int64_t ldp, void* dq, int64_t sdq_l, int64_t sdq_n,
                            float scale, void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_supported(dt, dh))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_bwd: dtype %d / head dim %d not supported",
                     dt, dh);
  const void* ptrs[] = {go, o, q, k, v, p_out, ds_out, dq};
  const int64_t strides[] = {sgo_l, sgo_n, so_l, so_n, sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, ldp,
                             sdq_l, sdq_n};
  const bool pds = dq == nullptr;                 // P / dS only: dQ left to jmt_attn_dkdv
  int rc = check_common("jmt_attn_bwd", N, H, Lq, Lk, ptrs, pds ? 7 : 8, strides, pds ? 11 : 13);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(lse && ldp >= Lk, "jmt_attn_bwd: lse missing or ldp < Lk");
  if (pds) {
    JMT_CHECK_ARG(ldp >= (int64_t)(Lk + AP_KT - 1) / AP_KT * AP_KT && ldp % AP_KT == 0 &&
                      (int64_t)(Lq + AP_QT) * ldp * 2 < (1LL << 30) &&
                      (int64_t)Lk * sk_l * 2 < (1LL << 31) && (int64_t)Lk * sv_l * 2 < (1LL << 31),
                  "jmt_attn_bwd (dq = NULL): ldp must be a multiple of 32 covering Lk, Lq rows "
                  "of ldp 16-bit values below 1 GiB and Lk K / V rows below 2 GiB");
    AttnBwdArgs a = {};
    a.go = go; a.o = o; a.q = q; a.k = k; a.v = v; a.lse = lse;
    a.pbuf = p_out; a.dsbuf = ds_out; a.dq = nullptr;
    a.sgo_l = sgo_l; a.sgo_n = sgo_n; a.so_l = so_l; a.so_n = so_n; a.sq_l = sq_l; a.sq_n = sq_n;
    a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n;
    a.ldp = ldp;
    a.Lq = Lq; a.Lk = Lk; a.H = H;
    a.scale = scale;
    a.scale_log2 = scale * 1.4426950408889634f;
    a.nitems = ((Lq + AP_QT - 1) / AP_QT) * N * H;
    const dim3 grid(persistent_grid(a.nitems));
    hipStream_t st = as_stream(stream);
#if JMT_DIAG
    static const int dbg = getenv("JMT_ATTN_PDS_DBG") ? atoi(getenv("JMT_ATTN_PDS_DBG")) : 0;
    if (dbg && dt == JMT_BF16) {
      if (dbg & 64) a.dq = g_stamps;              // the stamps buffer (jmt_attn_set_stamps)
#define JMT_PDS_DBG(D)                                                                       \
  case D: {                                                                                  \
    static bool once = (set_lds(attn_bwd_pds_kernel<__bf16, D>, AP_LDS), true);             \
    (void)once;                                                                              \
    hipLaunchKernelGGL((attn_bwd_pds_kernel<__bf16, D>), grid, dim3(512), (size_t)AP_LDS, st, \
                       a);                                                                   \
  } break;
      switch (dbg) {
        JMT_PDS_DBG(1) JMT_PDS_DBG(2) JMT_PDS_DBG(3) JMT_PDS_DBG(4) JMT_PDS_DBG(6)
        JMT_PDS_DBG(7) JMT_PDS_DBG(8) JMT_PDS_DBG(15) JMT_PDS_DBG(16) JMT_PDS_DBG(32)
        JMT_PDS_DBG(17) JMT_PDS_DBG(18) JMT_PDS_DBG(64)
        default: return set_error(JMT_ERR_ARG, "JMT_ATTN_PDS_DBG=%d not built", dbg);
      }
#undef JMT_PDS_DBG
      JMT_LAUNCH_CHECK("jmt_attn_bwd");
      return JMT_OK;
    }
#endif
    if (dt == JMT_BF16) {
      static bool once = (set_lds(attn_bwd_pds_kernel<__bf16>, AP_LDS), true);
      (void)once;
      hipLaunchKernelGGL((attn_bwd_pds_kernel<__bf16>), grid, dim3(512), (size_t)AP_LDS, st, a);
    } else {
      static bool once = (set_lds(attn_bwd_pds_kernel<_Float16>, AP_LDS), true);
      (void)once;
      hipLaunchKernelGGL((attn_bwd_pds_kernel<_Float16>), grid, dim3(512), (size_t)AP_LDS, st,
                         a);
    }
    JMT_LAUNCH_CHECK("jmt_attn_bwd");
    return JMT_OK;
  }
  AttnBwdArgs a = {};
  a.go = go; a.o = o; a.q = q; a.k = k; a.v = v; a.lse = lse;
  a.pbuf = p_out; a.dsbuf = ds_out; a.dq = dq;
  a.sgo_l = sgo_l; a.sgo_n = sgo_n; a.so_l = so_l; a.so_n = so_n; a.sq_l = sq_l; a.sq_n = sq_n;
  a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n; a.sdq_l = sdq_l; a.sdq_n = sdq_n;
  a.ldp = ldp;
  a.Lq = Lq; a.Lk = Lk; a.H = H;
  a.scale = scale;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.nitems = ((Lq + AT_QT - 1) / AT_QT) * N * H;
  const dim3 grid(persistent_grid(a.nitems));
  hipStream_t st = as_stream(stream);
  if (dt == JMT_BF16) {
    launch_bwd_bf16<ATTN_BWD_OPT>(grid, st, a);
  } else {
    static bool once = (set_lds(attn_bwd_kernel<_Float16, ATTN_BWD_OPT>, AB_LDS), true);
    (void)once;
    hipLaunchKernelGGL((attn_bwd_kernel<_Float16, ATTN_BWD_OPT>), grid, dim3(512),
                       (size_t)AB_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_bwd");
  return JMT_OK;
}

