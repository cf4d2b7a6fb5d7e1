// Long-sequence attention backward with 32 query rows per wave (gfx950, wave64), head dim 512:
// the same products and outputs as attn.hip's attn_bwd_kernel —
//   P = exp(scale Q K^T - lse) recomputed, dP = dO V^T, Delta = rowsum(dO o O),
//   dS = scale P o (dP - Delta), dQ = dS K;  P and dS written once for jmt_attn_dkdv
// — in a 4-wave block (one wave per SIMD) instead of 8.  VERDICT r3 next #3: the 8-wave kernel
// gives a wave 16 query rows, so every K / V fragment it reads from LDS feeds one MFMA per row
// group, and the LDS traffic per tile (8 waves x 48 KiB of K / V fragments + the score exchange,
// ~450 KiB per 32-key tile) is about twice the MFMA time of the tile.  Here wave w owns query
// rows 32 (w & 1) .. +31 (two 16-row groups) and HALF h = w >> 1 of the head dims: each K / V
// fragment read feeds both row groups, so a tile reads ~256 KiB.  The price is registers: Q, dO
// (and O for Delta) fragments and the dQ accumulator of 32 x 256 per wave, ~340 VGPRs, which only
// one wave per SIMD can hold (the accumulators in AGPRs).
// Reference: autograd's backward of F.multi_head_attention_forward behind every
// nn.MultiheadAttention of mm_multi_transformers.py:57,142-167.
//
// Geometry otherwise as attn_bwd_kernel: 64 query rows per block (an item = (n, h, 64-row
// q-tile), persistent over items with XCD-contiguous ranges), 32-key K / V tiles double-buffered
// by LDS-DMA (the next tile lands during the current one, the next item's tile 0 during the last),
// the pair (w, w ^ 2) exchanges its score / dP partials through LDS and sums them in one canonical
// order (half 0 + half 1), dQ stored straight from registers.  LDS: 2 x (K 32 KiB + V 32 KiB) +
// 4 x 8 KiB exchange = 160 KiB.
#include "attn_common.h"

namespace jmt {

constexpr int B2_QT = 64;                        // query rows per block
constexpr int B2_KT = 32;                        // keys per tile
constexpr int B2_XCH = 8192;                     // exchange bytes per wave (2 row groups)
constexpr int B2_IMG = B2_KT * AT_ROWB;          // one K or V image
constexpr int B2_LDS = 4 * B2_IMG + 4 * B2_XCH;  // 160 KiB

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd_rg2_kernel(AttnBwdArgs p) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xch = smem + 4 * B2_IMG;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, rp = w & 1, h = w >> 1;
  const int nqt = (p.Lq + B2_QT - 1) / B2_QT;
  const int nkt = (p.Lk + B2_KT - 1) / B2_KT;
  int item, iend, istride;
  item_range(p.nitems, item, iend, istride);
  if (item >= iend) return;

  int nh = item / nqt, n = nh / p.H, hd = nh % p.H, q0 = (item % nqt) * B2_QT;
  const T* kb = (const T*)p.k + (int64_t)n * p.sk_n + hd * AT_DH;
  const T* vb = (const T*)p.v + (int64_t)n * p.sv_n + hd * AT_DH;

  // row-operand fragments of an item: Q, dO (kept for the whole item) and O (Delta only)
  F qf[2][8], df[2][8], of[2][8];
  auto rows_off = [&](int q0_, int i) {
    return (int64_t)min(q0_ + 32 * rp + 16 * i + li, p.Lq - 1);
  };
  auto load_qd = [&](int n_, int hd_, int q0_) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t qc_ = rows_off(q0_, i), coff = (int64_t)hd_ * AT_DH + 256 * h + 8 * g;
      const T* qrow = (const T*)p.q + (int64_t)n_ * p.sq_n + qc_ * p.sq_l + coff;
      const T* drow = (const T*)p.go + (int64_t)n_ * p.sgo_n + qc_ * p.sgo_l + coff;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        qf[i][ks] = *(const F*)(qrow + 32 * ks);
        df[i][ks] = *(const F*)(drow + 32 * ks);
      }
    }
  };
  auto load_o = [&](int n_, int hd_, int q0_) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t qc_ = rows_off(q0_, i), coff = (int64_t)hd_ * AT_DH + 256 * h + 8 * g;
      const T* orow = (const T*)p.o + (int64_t)n_ * p.so_n + qc_ * p.so_l + coff;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) of[i][ks] = *(const F*)(orow + 32 * ks);
    }
  };
  load_qd(n, hd, q0);
  load_o(n, hd, q0);
  int buf = 0;                                    // buffer pair of the next tile to compute
  stage_rows<T, B2_KT, 4>(smem, kb, p.sk_l, 0, p.Lk);
  stage_rows<T, B2_KT, 4>(smem + B2_IMG, vb, p.sv_l, 0, p.Lk);

  f32x4* xmine = (f32x4*)(xch + w * B2_XCH) + lane;
  const f32x4* xpart = (const f32x4*)(xch + (w ^ 2) * B2_XCH) + lane;
  int kb4[4], tb8[8];
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, h);
#pragma unroll
  for (int c = 0; c < 8; ++c) tb8[c] = tr_base(c, li, g, h);

  while (true) {
    int qr[2];
    int64_t prow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      qr[i] = q0 + 32 * rp + 16 * i + li;
      prow[i] = (int64_t)nh * p.Lq + min(qr[i], p.Lq - 1);
    }
    const int nxt = item + istride;
    const bool more = nxt < iend;
    const int nh2 = nxt / nqt, n2 = nh2 / p.H, hd2 = nh2 % p.H, q02 = (nxt % nqt) * B2_QT;
    const T* kb2 = (const T*)p.k + (int64_t)n2 * p.sk_n + hd2 * AT_DH;
    const T* vb2 = (const T*)p.v + (int64_t)n2 * p.sv_n + hd2 * AT_DH;

    float delta[2], lse2[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float dp = 0.f;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) dp += (float)of[i][ks][e] * (float)df[i][ks][e];
      delta[i] = pl_pair_sum(dp);                 // this half's part of rowsum(dO o O)
      lse2[i] = p.lse[prow[i]] * 1.4426950408889634f;
      ((float*)xch)[w * 128 + 64 * i + lane] = delta[i];
    }

    f32x4 acc[2][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    T* rowp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) rowp[i] = (T*)(h == 0 ? p.pbuf : p.dsbuf) + prow[i] * p.ldp;

    wait_vmcnt<0>();                              // tile 0 landed
    lds_barrier();                                // ... and every Delta part written
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float part = ((const float*)xch)[(w ^ 2) * 128 + 64 * i + lane];
      delta[i] = h == 0 ? delta[i] + part : part + delta[i];
    }
    lds_barrier();                                // Delta parts read: exchange slots free

    for (int j = 0; j < nkt; ++j) {
      const char* kimg = smem + buf * 2 * B2_IMG;
      const char* vimg = kimg + B2_IMG;
      char* nk = smem + (buf ^ 1) * 2 * B2_IMG;   // tile j+1 (or the next item's tile 0)
      if (j + 1 < nkt || more) {
        const T* kbn = j + 1 < nkt ? kb : kb2;
        const T* vbn = j + 1 < nkt ? vb : vb2;
        const int k0n = j + 1 < nkt ? B2_KT * (j + 1) : 0;
        stage_rows<T, B2_KT, 4>(nk, kbn, p.sk_l, k0n, p.Lk);
        stage_rows<T, B2_KT, 4>(nk + B2_IMG, vbn, p.sv_l, k0n, p.Lk);
      }
      // ---- partial scores (K) and partial dP (V) over this wave's 256 dims, both row groups
      f32x4 s[2][2], d[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[i][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
          d[i][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      {   // K and V fragments of key subtiles 0, 1 per k-step, double-buffered; each feeds both
          // row groups
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
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
              s[i][kt] = mfma16(fa[kt], qf[i][ks], s[i][kt]);
              d[i][kt] = mfma16(fa[2 + kt], df[i][ks], d[i][kt]);
            }
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 2 < 8) batch(fa, ks + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
              s[i][kt] = mfma16(fb[kt], qf[i][ks + 1], s[i][kt]);
              d[i][kt] = mfma16(fb[2 + kt], df[i][ks + 1], d[i][kt]);
            }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          xmine[64 * (2 * i + kt)] = s[i][kt];
          xmine[64 * (4 + 2 * i + kt)] = d[i][kt];
        }
      lds_barrier();                              // partials visible (tile j+1 DMA in flight)
      if (j + 1 == nkt && more) load_qd(n2, hd2, q02);     // next item's Q / dO fragments
      const int kbase = B2_KT * j + 4 * g;
      F dsf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const f32x4 ps = xpart[64 * (2 * i + kt)], pd = xpart[64 * (4 + 2 * i + kt)];
          const f32x4 sf = h == 0 ? s[i][kt] + ps : ps + s[i][kt];
          const f32x4 dfull = h == 0 ? d[i][kt] + pd : pd + d[i][kt];
          T pv4[4], ds4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool in = kbase + 16 * kt + r < p.Lk;
            const float pv = in ? __builtin_amdgcn_exp2f(sf[r] * p.scale_log2 - lse2[i]) : 0.f;
            const float ds = p.scale * pv * (dfull[r] - delta[i]);
            pv4[r] = from_f<T>(pv);
            ds4[r] = from_f<T>(ds);
            dsf[i][kt * 4 + r] = ds4[r];
          }
          const int key = kbase + 16 * kt;
          JMT_DCHECK(prow[i] >= 0 && item < p.nitems);
          if (qr[i] < p.Lq && key < p.ldp)
            *(uint2*)(rowp[i] + key) = h == 0 ? *(const uint2*)pv4 : *(const uint2*)ds4;
        }
      }
      // ---- acc[i][t] += sum_k dS(k) K[k][256h + 16t + 4g + r] (transposed K fragments in
      // double-buffered batches of 4, each feeding both row groups)
      {
        F fa[4], fb[4];
        auto kbatch = [&](F* dst, int b) {
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const int t = 4 * b + x;
            const char* a = kimg + tb8[t & 7] + 256 * (t >> 3);
            const Hf lo = tr_read<Hf>(a);
            const Hf hi = tr_read<Hf>(a + 16384);
            dst[x] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        };
        kbatch(fa, 0);
#pragma unroll
        for (int b = 0; b < 4; b += 2) {
          kbatch(fb, b + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int i = 0; i < 2; ++i) acc[i][4 * b + x] = mfma16(fa[x], dsf[i], acc[i][4 * b + x]);
          __builtin_amdgcn_sched_barrier(0);
          if (b + 2 < 4) kbatch(fa, b + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int i = 0; i < 2; ++i)
              acc[i][4 * b + 4 + x] = mfma16(fb[x], dsf[i], acc[i][4 * b + 4 + x]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (j + 1 < nkt) {
        wait_vmcnt<0>();                          // tile j+1 landed (and P / dS stores issued)
        lds_barrier();                            // this buffer pair and the slots are free
      }
      buf ^= 1;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      store_acc_direct<T>(acc[i], 1.f,
                          (T*)p.dq + (int64_t)n * p.sdq_n + hd * AT_DH +
                              (int64_t)qr[i] * p.sdq_l + 256 * h,
                          qr[i] < p.Lq);
    if (!more) break;
    load_o(n2, hd2, q02);                         // O of the next item (Delta), after acc is dead
    lds_barrier();                                // every wave is done with the last tile's
                                                  // images and exchange slots
    item = nxt; nh = nh2; n = n2; hd = hd2; q0 = q02; kb = kb2; vb = vb2;
  }
}

void launch_attn_bwd_rg2(int dt, dim3 grid, hipStream_t st, const AttnBwdArgs& a) {
  if (dt == JMT_BF16) {
    static bool once = ((void)hipFuncSetAttribute((const void*)attn_bwd_rg2_kernel<__bf16>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  B2_LDS), true);
    (void)once;
    hipLaunchKernelGGL((attn_bwd_rg2_kernel<__bf16>), grid, dim3(256), (size_t)B2_LDS, st, a);
  } else {
    static bool once = ((void)hipFuncSetAttribute((const void*)attn_bwd_rg2_kernel<_Float16>,
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  B2_LDS), true);
    (void)once;
    hipLaunchKernelGGL((attn_bwd_rg2_kernel<_Float16>), grid, dim3(256), (size_t)B2_LDS, st, a);
  }
}

}  // namespace jmt
