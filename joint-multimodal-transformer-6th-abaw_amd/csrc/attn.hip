// Fused scaled-dot-product attention for the JMT path (gfx950, wave64), forward and the dQ half
// of the backward, per (batch n, head h):
//   forward:  O = softmax(scale Q K^T) V,  + lse and (training) the probabilities P
//   backward: dP = dO V^T,  dS = scale * P o (dP - rowsum(dO o O)),  dQ = dS K   (+ P, dS out)
// Replaces the score GEMM -> softmax -> PV GEMM chain behind every nn.MultiheadAttention of the
// reference (F.multi_head_attention_forward, called from mm_multi_transformers.py:57,142-167,
// 191 and intra_modal_transformer_fusion.py) and the dP GEMM + softmax
// backward + dQ GEMM of its autograd backward; dK = dS^T Q and dV = P^T dO stay GEMMs.
//
// Both passes are the same kernel shape (MODE): a block of 4 waves owns 64 rows of the "row
// operand" (Q forward, dO backward); wave w owns rows 16w..16w+15: their fragments stay in
// registers, a 16 x DH fp32 accumulator (O / dQ) in registers.  Key tiles of 64 stream through
// two LDS images: the SCORE stream (K forward, V backward) is read as ds_read_b128 fragments for
// the 16x64 score tile, the ACCUMULATE stream (V forward, K backward) through
// ds_read_b64_tr_b16 for the 16 x DH update.  Stream 2 of tile j lands during the score phase,
// stream 1 of tile j+1 during the update phase.
//
//  * Both products run with the MFMA operands swapped (stream operand first), so an accumulator
//    lane owns ONE row and 4 consecutive keys / head columns: softmax row state is lane-local
//    (2 shuffles per row reduction), the probabilities (or dS) feed the update MFMA straight from
//    registers (their k-slot order is mirrored in the transposed fragment reads), and output
//    rows are stored as 8-B column groups.
//  * Forward softmax is online with LAZY rescaling: probabilities are taken against a reference
//    max that is raised (O and the row sum rescaled) only when a row max exceeds it by > 8
//    (log2 units).  With P output on, the unnormalised tile values and each tile's reference max
//    are written; the backward kernel normalises them with the lse and writes the exact P back
//    for the dV GEMM.
//  * Images: [key][DH] rows at a 32-B padded pitch (AttnGeo) -> conflict-free fragment reads with
//    immediate offsets.  XCD-aware block order: the q-tile blocks of one (n, h) share an L2.
#include "common.h"

namespace jmt {

// A block is NW waves owning 16 NW rows; every block streams the whole K/V of its (n, h) through
// LDS (attn_waves() picks NW).
constexpr int AT_KT = 64;       // keys per tile
constexpr int AT_FWD = 0, AT_DQ = 1;

struct AttnParams {
  const void* a;        // row operand: Q (fwd) / dO (dq)
  const void* s1;       // score stream: K (fwd) / V (dq)
  const void* s2;       // accumulate stream: V (fwd) / K (dq)
  void* out;            // O (fwd) / dQ (dq)
  const void* o_in;     // dq: forward output O (for rowsum(dO o O))
  void* pbuf;           // fwd: unnormalised P out (nullable); dq: in, normalised P written back
  void* dsbuf;          // dq: dS out
  float* lse;           // fwd: out (nullable); dq: in
  float* mt;            // per (row, key tile) reference max (fwd out, dq in) when pbuf is used
  int64_t sa_l, sa_n, s1_l, s1_n, s2_l, s2_n, so_l, so_n, soi_l, soi_n, ldp;
  int Lq, Lk, H;
  float scale, scale_log2;
};

template <int DH> struct AttnGeo {
  static constexpr int RB = DH * 2;
  static constexpr int PITCH = RB + 32;
  static constexpr int IMG = AT_KT * PITCH;
};

// stage one tile of AT_KT key rows (row r <- source row min(k0 + r, Lk - 1)): one 1-KiB
// LDS-DMA wave-instruction per row (DH = 512)
template <typename T, int DH, int NW>
__device__ __forceinline__ void stage_kv(char* img, const T* base, int64_t ld, int k0, int Lk) {
  typedef AttnGeo<DH> G;
  static_assert(G::RB == 1024, "one LDS-DMA instruction per key row");
  constexpr int NI = AT_KT / NW;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = w * NI;
  char* dst = img + r0 * G::PITCH;
  if (k0 + AT_KT <= Lk) {          // whole tile in range: rows r0.. at a constant stride
    const T* src = base + (int64_t)(k0 + r0) * ld + lane * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(src + i * ld, dst + i * G::PITCH);
  } else {                         // last tile: rows past Lk repeat row Lk-1 (masked later)
    const T* src = base + lane * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      glds16(src + (int64_t)min(k0 + r0 + i, Lk - 1) * ld, dst + i * G::PITCH);
  }
}

template <typename T, int DH, int MODE, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_kernel(AttnParams p) {
  constexpr int AT_QT = 16 * NW;                  // rows per block
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  typedef AttnGeo<DH> G;
  constexpr int KS = DH / 32;                     // k-steps of the score product
  constexpr int TD = DH / 16;                     // 16-column tiles of the accumulator
  constexpr int NI = AT_KT / NW;                  // LDS-DMA instructions per wave per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img1 = smem;
  char* img2 = smem + G::IMG;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware bijective remap: the q-tile blocks of one (n, h) share K/V through one XCD's L2
  const int nqt = (p.Lq + AT_QT - 1) / AT_QT;
  const int nwg = gridDim.x;
  int wg = blockIdx.x;
  if (nwg >= 16) {
    const int qd = nwg / 8, rm = nwg % 8, x = blockIdx.x % 8;
    wg = (x < rm ? x * (qd + 1) : rm * (qd + 1) + (x - rm) * qd) + blockIdx.x / 8;
  }
  const int nh = wg / nqt;
  const int n = nh / p.H, h = nh % p.H;
  const int q0 = (wg % nqt) * AT_QT;
  const T* ab = (const T*)p.a + (int64_t)n * p.sa_n + h * DH;
  const T* s1b = (const T*)p.s1 + (int64_t)n * p.s1_n + h * DH;
  const T* s2b = (const T*)p.s2 + (int64_t)n * p.s2_n + h * DH;
  const int nkt = (p.Lk + AT_KT - 1) / AT_KT;

  // this lane's row and its row-operand fragments (rows past Lq read row Lq-1, never stored)
  const int qr = q0 + 16 * w + li;
  const int qc = min(qr, p.Lq - 1);
  F qf[KS];
  {
    const T* arow = ab + (int64_t)qc * p.sa_l;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const F*)(arow + 32 * ks + 8 * g);
  }
  const int64_t prow = ((int64_t)nh * p.Lq + qc);          // row index into P / dS / lse / mt
  float delta = 0.f, lse2 = 0.f;
  F of[MODE == AT_DQ ? KS : 1];
  if constexpr (MODE == AT_DQ) {
    const T* orow = (const T*)p.o_in + (int64_t)qc * p.soi_l + (int64_t)n * p.soi_n + h * DH;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) of[ks] = *(const F*)(orow + 32 * ks + 8 * g);
    lse2 = p.lse[prow] * 1.4426950408889634f;
  }
  // tile-0 DMA is issued behind the row loads (vmcnt retires in issue order)
  stage_kv<T, DH, NW>(img1, s1b, p.s1_l, 0, p.Lk);
  stage_kv<T, DH, NW>(img2, s2b, p.s2_l, 0, p.Lk);
  if constexpr (MODE == AT_DQ) {
    // Delta = rowsum(dO o O) = rowsum(P o dP)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) delta += (float)of[ks][e] * (float)qf[ks][e];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
  }

  f32x4 o[TD];
#pragma unroll
  for (int t = 0; t < TD; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  // per-lane fragment bases: stream-1 rows 16kt + li, chunk 4ks + g; stream-2 transpose-read
  // rows 32u + 4g + (li>>2) (+16 for the upper k-slots), columns 16t + 4(li&3)
  const char* s1l = img1 + li * G::PITCH + g * 16;
  const char* s2l = img2 + (4 * g + (li >> 2)) * G::PITCH + 8 * (li & 3);
  T* prow_p = (T*)p.pbuf + prow * p.ldp;
  T* prow_ds = (T*)p.dsbuf + prow * p.ldp;
  uint2 pin[4];                                   // dq: this tile's unnormalised P (4 x 4 keys)
  float mref = 0.f;                               // dq: this tile's reference max
  auto load_p = [&](int j) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const int key = AT_KT * j + 16 * kt + 4 * g;
      pin[kt] = key < p.ldp ? *(const uint2*)(prow_p + key) : make_uint2(0u, 0u);
    }
    mref = p.mt[prow * nkt + j];
  };
  if constexpr (MODE == AT_DQ) load_p(0);

  wait_vmcnt<NI>();                               // stream-1 tile 0 landed (tile-0 stream 2 in flight)
  __syncthreads();
  for (int j = 0; j < nkt; ++j) {
    // ---- score tile: s[kt][r] = <row qr, key 64j + 16kt + 4g + r>
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {   // score fragments double-buffered: k-step ks+1's reads issue before k-step ks's MFMAs
      F kf[2][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) kf[0][kt] = *(const F*)(s1l + kt * 16 * G::PITCH);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
            kf[(ks + 1) & 1][kt] = *(const F*)(s1l + kt * 16 * G::PITCH + (ks + 1) * 64);
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[kt] = mfma16(kf[ks & 1][kt], qf[ks], s[kt]);
      }
    }
    const int kbase = AT_KT * j + 4 * g;
    F pf[2];
    if constexpr (MODE == AT_FWD) {
      // ---- online softmax (log2 domain); keys >= Lk masked
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = (kbase + 16 * kt + r < p.Lk) ? s[kt][r] * p.scale_log2 : -INFINITY;
          s[kt][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (__any(mx > m_run + 8.f)) {              // lazy rescale (see header)
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int t = 0; t < TD; ++t) o[t] *= alpha;
      }
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(s[kt][r] - m_run);
          ls += pv;
          pf[kt >> 1][(kt & 1) * 4 + r] = from_f<T>(pv);
        }
      l_run += ls;
      if (p.pbuf && qr < p.Lq) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const int key = kbase + 16 * kt;
          if (key < p.ldp) {
            T v4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v4[r] = pf[kt >> 1][(kt & 1) * 4 + r];
            *(uint2*)(prow_p + key) = *(const uint2*)v4;
          }
        }
        if (g == 0) p.mt[prow * nkt + j] = m_run;
      }
    } else {
      // ---- dS = scale * P o (dP - Delta), P = Ptilde * 2^(mref - lse); P written back exact
      const float f = __builtin_amdgcn_exp2f(mref - lse2);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const T* pt = (const T*)&pin[kt];
        T pn[4], dsv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = (float)pt[r] * f;
          pn[r] = from_f<T>(pv);
          const float ds = p.scale * pv * (s[kt][r] - delta);
          dsv[r] = from_f<T>(ds);
          pf[kt >> 1][(kt & 1) * 4 + r] = dsv[r];
        }
        const int key = kbase + 16 * kt;
        if (qr < p.Lq && key < p.ldp) {
          *(uint2*)(prow_p + key) = *(const uint2*)pn;
          *(uint2*)(prow_ds + key) = *(const uint2*)dsv;
        }
      }
    }

    wait_vmcnt<0>();                              // stream-2 tile j landed
    __syncthreads();                              // ... for all waves; stream-1 image free
    if (j + 1 < nkt) {
      stage_kv<T, DH, NW>(img1, s1b, p.s1_l, AT_KT * (j + 1), p.Lk);
      if constexpr (MODE == AT_DQ) load_p(j + 1);
    }

    // ---- accumulate: acc[t] += sum_k pf(k) * stream2[k][16t + 4g + r]
    // fragment reads run PD MFMAs ahead (a ring of PD fragments): the transposed LDS reads of
    // fragment q+PD are in flight while MFMA q executes, instead of one read->wait->MFMA chain
    {
      constexpr int NQ = 2 * TD, PD = 4;
      auto vread = [&](int q) -> F {
        const int u = q / TD, t = q % TD;
        const Hf lo = tr_read<Hf>(s2l + 32 * u * G::PITCH + 32 * t);
        const Hf hi = tr_read<Hf>(s2l + (32 * u + 16) * G::PITCH + 32 * t);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      F ring[PD];
#pragma unroll
      for (int q = 0; q < PD; ++q) ring[q] = vread(q);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const F vf = ring[q % PD];
        if (q + PD < NQ) ring[q % PD] = vread(q + PD);
        o[q % TD] = mfma16(vf, pf[q / TD], o[q % TD]);
      }
    }
    if (j + 1 < nkt) {
      wait_vmcnt<0>();                            // stream-1 tile j+1 landed
      __syncthreads();                            // ... for all waves; stream-2 image free
      stage_kv<T, DH, NW>(img2, s2b, p.s2_l, AT_KT * (j + 1), p.Lk);
    }
  }

  // ---- store: lane owns row qr, columns 16t + 4g .. +3
  float inv = 1.f;
  if constexpr (MODE == AT_FWD) {
    float lt = l_run;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    inv = 1.f / lt;
    if (qr < p.Lq && g == 0 && p.lse)
      p.lse[prow] = (m_run + __builtin_amdgcn_logf(lt)) * 0.69314718055994531f;
  }
  if (qr < p.Lq) {
    T* orow = (T*)p.out + (int64_t)qr * p.so_l + (int64_t)n * p.so_n + h * DH;
#pragma unroll
    for (int t = 0; t < TD; ++t) {
      T v4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v4[r] = from_f<T>(o[t][r] * inv);
      *(uint2*)(orow + 16 * t + 4 * g) = *(const uint2*)v4;
    }
  }
}

// waves per block: 4.  8-wave blocks (half the K/V staging per FLOP) measured 3-33% SLOWER at
// T = 300 (fwd 290 vs 280 us, dQ 400 vs 352 us for the 6 cross-attention pairs at B = 64), so the
// kernel is not K/V-load-bound there; NW stays a template parameter for other shapes.
static int attn_waves(int) { return 4; }

template <typename T, int DH, int MODE, int NW>
static void launch_nw(const AttnParams& p, int N, hipStream_t st) {
  constexpr int LDS = 2 * AttnGeo<DH>::IMG;
  auto fn = attn_kernel<T, DH, MODE, NW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  dim3 grid((unsigned)(((p.Lq + 16 * NW - 1) / (16 * NW)) * N * p.H));
  hipLaunchKernelGGL(fn, grid, dim3(64 * NW), (size_t)LDS, st, p);
}

template <typename T, int DH, int MODE>
static void launch(const AttnParams& p, int N, hipStream_t st) {
  (void)attn_waves(p.Lq);
  launch_nw<T, DH, MODE, 4>(p, N, st);
}

static int check_common(const char* name, int N, int H, int Lq, int Lk, const void* const* ptrs,
                        int nptr, const int64_t* strides, int nstr) {
  JMT_CHECK_ARG(N > 0 && H > 0 && Lq > 0 && Lk > 0 &&
                    (int64_t)N * H * ((Lq + 63) / 64) < (1LL << 31),
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

extern "C" int jmt_attn_supported(int dt, int dh) {
  return (dt == JMT_BF16 || dt == JMT_F16) && dh == 512;
}

extern "C" int jmt_attn_mt_floats(int N, int H, int Lq, int Lk) {
  return N * H * Lq * ((Lk + AT_KT - 1) / AT_KT);
}

extern "C" int jmt_attn_fwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* q,
                            int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n,
                            const void* v, int64_t sv_l, int64_t sv_n, void* o, int64_t so_l,
                            int64_t so_n, float scale, float* lse, void* p_out, int64_t ldp,
                            float* mt, void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_supported(dt, dh))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_fwd: dtype %d / head dim %d not supported",
                     dt, dh);
  const void* ptrs[] = {q, k, v, o};
  const int64_t strides[] = {sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n};
  int rc = check_common("jmt_attn_fwd", N, H, Lq, Lk, ptrs, 4, strides, 8);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(!p_out || (mt && ldp >= Lk && ldp % 8 == 0 && ((uintptr_t)p_out & 15) == 0),
                "jmt_attn_fwd: P output needs mt, ldp >= Lk, ldp %% 8 == 0, 16-B alignment");
  AttnParams p = {};
  p.a = q; p.s1 = k; p.s2 = v; p.out = o; p.lse = lse; p.pbuf = p_out; p.mt = mt;
  p.sa_l = sq_l; p.sa_n = sq_n; p.s1_l = sk_l; p.s1_n = sk_n; p.s2_l = sv_l; p.s2_n = sv_n;
  p.so_l = so_l; p.so_n = so_n; p.ldp = ldp;
  p.Lq = Lq; p.Lk = Lk; p.H = H;
  p.scale = scale;
  p.scale_log2 = scale * 1.4426950408889634f;
  hipStream_t st = as_stream(stream);
  if (dt == JMT_BF16) launch<__bf16, 512, AT_FWD>(p, N, st);
  else launch<_Float16, 512, AT_FWD>(p, N, st);
  JMT_LAUNCH_CHECK("jmt_attn_fwd");
  return JMT_OK;
}

extern "C" int jmt_attn_bwd_dq(int dt, int N, int H, int Lq, int Lk, int dh, const void* go,
                               int64_t sgo_l, int64_t sgo_n, const void* o, int64_t so_l,
                               int64_t so_n, const void* k, int64_t sk_l, int64_t sk_n,
                               const void* v, int64_t sv_l, int64_t sv_n, const float* lse,
                               void* p_buf, const float* mt, int64_t ldp, void* ds, void* dq,
                               int64_t sdq_l, int64_t sdq_n, float scale, void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_supported(dt, dh))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_bwd_dq: dtype %d / head dim %d not supported",
                     dt, dh);
  const void* ptrs[] = {go, o, k, v, p_buf, ds, dq};
  const int64_t strides[] = {sgo_l, sgo_n, so_l, so_n, sk_l, sk_n, sv_l, sv_n, sdq_l, sdq_n, ldp};
  int rc = check_common("jmt_attn_bwd_dq", N, H, Lq, Lk, ptrs, 7, strides, 11);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(lse && mt && ldp >= Lk, "jmt_attn_bwd_dq: lse / mt missing or ldp < Lk");
  AttnParams p = {};
  p.a = go; p.s1 = v; p.s2 = k; p.out = dq; p.o_in = o; p.pbuf = p_buf; p.dsbuf = ds;
  p.lse = const_cast<float*>(lse); p.mt = const_cast<float*>(mt);
  p.sa_l = sgo_l; p.sa_n = sgo_n; p.s1_l = sv_l; p.s1_n = sv_n; p.s2_l = sk_l; p.s2_n = sk_n;
  p.so_l = sdq_l; p.so_n = sdq_n; p.soi_l = so_l; p.soi_n = so_n; p.ldp = ldp;
  p.Lq = Lq; p.Lk = Lk; p.H = H;
  p.scale = scale;
  p.scale_log2 = scale * 1.4426950408889634f;
  hipStream_t st = as_stream(stream);
  if (dt == JMT_BF16) launch<__bf16, 512, AT_DQ>(p, N, st);
  else launch<_Float16, 512, AT_DQ>(p, N, st);
  JMT_LAUNCH_CHECK("jmt_attn_bwd_dq");
  return JMT_OK;
}
