// Fused attention over SHORT sequences (Lq, Lk <= 32), head dim 512, gfx950 wave64: the forward
// and the WHOLE backward — dQ, dK AND dV — each in one kernel, one block per (sequence n, head h).
//
// Where it runs: nn.MultiheadAttention over the batch axis of MultimodalTransformer_wo_JR
// (mm_transformers.py:119-146, bench config c2: a length-B = 32 sequence per time step) and every
// attention of the shipped real-data configuration (config_file.json: T = 16 clips per window,
// mm_multi_transformers.py:57,142-167).  The long-sequence kernels (attn.hip) tile 64 query rows
// and hand P and dS to two TN GEMMs for dK / dV; at L <= 32 that leaves >= 3/4 of every tile idle
// and spends two extra launches of M = K = L GEMMs per attention.  Here the
// whole key range fits one tile, so the key-side products run in the same block:
//
//  * 4 waves: wave w owns query rows 16 (w & 1) .. +15 and HALF h = w >> 1 of the 512 head dims
//    (the attn.hip geometry with one 32-key tile): the score / dP partials over each half are
//    exchanged through LDS and summed in one canonical order (half 0 + half 1), so both halves
//    hold bitwise the same probabilities; the forward is bit-identical to attn_fwd_kernel.
//  * backward: P recomputed from the forward's lse, Delta = rowsum(dO o O), dS = scale P o
//    (dP - Delta); dQ = dS K from registers (as attn_bwd_kernel); P^T and dS^T (16-bit, the same
//    rounded values the long path writes to HBM) go to a 5 KiB LDS image instead, and the same
//    block computes dV^T = dO^T P and dK^T = Q^T dS (wave w: keys 16 (w & 1) .. +15, half h) from
//    transposed fragment reads of the dO / Q row images.  No P / dS in HBM, no dK / dV launches.
//  * every output stored straight from registers (16-B stores of paired accumulators).
// HBM bytes per sequence: forward (Lq + 2 Lk) reads + Lq writes of 1 KiB rows; backward
// (3 Lq + 2 Lk) reads (q, o, dO, k, v) + (Lq + 2 Lk) writes — the kernels are latency / HBM
// bound, the MFMA work (a 32 x 32 tile) is small.
#include "attn_common.h"

namespace jmt {

constexpr int AS_L = 32;                           // image rows: queries / keys padded to 32
constexpr int AS_IMG = AS_L * AT_ROWB;             // one 32-row image (32 KiB)
constexpr int AS_XF = 2 * 64 * 16;                 // fwd exchange per wave: S partial, 2 slots
constexpr int AS_XB = 4 * 64 * 16;                 // bwd exchange per wave: S and dP partials
constexpr int AS_TLD = 40;                         // P^T / dS^T row stride (16-bit elements)
constexpr int AS_T = AS_L * AS_TLD * 2;            // one P^T / dS^T image (2.5 KiB)
constexpr int ASF_LDS = 2 * AS_IMG + 4 * AS_XF;                       // 72 KiB: 2 blocks / CU
constexpr int ASB_LDS = 4 * AS_IMG + 4 * AS_XB + 4 * 64 * 4 + 2 * AS_T;  // 150 KiB

struct AttnShortArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* o;      // backward: the forward's output (Delta)
  const void* go;     // backward: dO
  void* out;          // forward: o
  float* lse;         // forward: written; backward: read
  void* dq;
  void* dk;
  void* dv;
  int64_t sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n, sgo_l, sgo_n;
  int64_t sdq_l, sdq_n, sdk_l, sdk_n, sdv_l, sdv_n;
  int Lq, Lk, H;
  float scale, scale_log2;
};

template <typename T>
__global__ __launch_bounds__(256, 2) void attn_short_fwd_kernel(AttnShortArgs p) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kimg = smem;
  char* vimg = smem + AS_IMG;
  char* xch = smem + 2 * AS_IMG;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, h = w >> 1;
  const int nh = blockIdx.x, n = nh / p.H, hd = nh % p.H;
  const int qr = 16 * (w & 1) + li;
  stage_rows<T, AS_L, 4>(kimg, (const T*)p.k + (int64_t)n * p.sk_n + hd * AT_DH, p.sk_l, 0, p.Lk);
  stage_rows<T, AS_L, 4>(vimg, (const T*)p.v + (int64_t)n * p.sv_n + hd * AT_DH, p.sv_l, 0, p.Lk);
  F qf[8];
  {
    const T* qrow = (const T*)p.q + (int64_t)n * p.sq_n + hd * AT_DH +
                    (int64_t)min(qr, p.Lq - 1) * p.sq_l + 256 * h + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const F*)(qrow + 32 * ks);
  }
  int kb4[4], tb8[8];
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, h);
#pragma unroll
  for (int c = 0; c < 8; ++c) tb8[c] = tr_base(c, li, g, h);
  wait_vmcnt<0>();
  lds_barrier();                                  // K / V images landed (every wave's DMA)

  // partial scores over this wave's 256 dims: s[kt][r] = <row qr, key 16 kt + 4 g + r>
  f32x4 s[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
      s[kt] = mfma16(*(const F*)(kimg + kb4[ks & 3] + 256 * (ks >> 2) + 16384 * kt), qf[ks], s[kt]);
  f32x4* xmine = (f32x4*)(xch + w * AS_XF) + lane;
  const f32x4* xpart = (const f32x4*)(xch + (w ^ 2) * AS_XF) + lane;
  xmine[0] = s[0];
  xmine[64] = s[1];
  lds_barrier();
  float x[2][4], mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const f32x4 ps = xpart[64 * kt];
    const f32x4 full = h == 0 ? s[kt] + ps : ps + s[kt];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[kt][r] = (16 * kt + 4 * g + r < p.Lk) ? full[r] * p.scale_log2 : -INFINITY;
      mx = fmaxf(mx, x[kt][r]);
    }
  }
  mx = pl_pair_max(mx);
  F pf;
  float ls = 0.f;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = __builtin_amdgcn_exp2f(x[kt][r] - mx);
      ls += pv;
      pf[kt * 4 + r] = from_f<T>(pv);
    }
  ls = pl_pair_sum(ls);
  if (qr < p.Lq && g == 0 && h == 0 && p.lse)
    p.lse[(int64_t)nh * p.Lq + qr] = (mx + __builtin_amdgcn_logf(ls)) * 0.69314718055994531f;
  // o[t] = sum_k P(k) V[k][256 h + 16 t + 4 g + r] (transposed V fragments, one 32-key step)
  f32x4 o[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const char* a = vimg + tb8[t & 7] + 256 * (t >> 3);
    const Hf lo = tr_read<Hf>(a);
    const Hf hi = tr_read<Hf>(a + 16384);
    o[t] = mfma16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), pf,
                  f32x4{0.f, 0.f, 0.f, 0.f});
  }
  JMT_DCHECK(nh < gridDim.x);
  store_acc_direct<T>(o, 1.f / ls,
                      (T*)p.out + (int64_t)n * p.so_n + hd * AT_DH + (int64_t)qr * p.so_l + 256 * h,
                      qr < p.Lq);
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_short_bwd_kernel(AttnShortArgs p) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* qimg = smem;
  char* kimg = smem + AS_IMG;
  char* vimg = smem + 2 * AS_IMG;
  char* dimg = smem + 3 * AS_IMG;
  char* xch = smem + 4 * AS_IMG;
  float* dlt = (float*)(xch + 4 * AS_XB);
  T* pt = (T*)(dlt + 4 * 64);                     // P^T  [key][query], row stride AS_TLD
  T* dst = pt + AS_L * AS_TLD;                    // dS^T [key][query]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15, h = w >> 1, rb = 16 * (w & 1);
  const int nh = blockIdx.x, n = nh / p.H, hd = nh % p.H;
  const int qr = rb + li, qc = min(qr, p.Lq - 1);
  const int64_t hoff = (int64_t)hd * AT_DH;
  stage_rows<T, AS_L, 4>(qimg, (const T*)p.q + (int64_t)n * p.sq_n + hoff, p.sq_l, 0, p.Lq);
  stage_rows<T, AS_L, 4>(kimg, (const T*)p.k + (int64_t)n * p.sk_n + hoff, p.sk_l, 0, p.Lk);
  stage_rows<T, AS_L, 4>(vimg, (const T*)p.v + (int64_t)n * p.sv_n + hoff, p.sv_l, 0, p.Lk);
  stage_rows<T, AS_L, 4>(dimg, (const T*)p.go + (int64_t)n * p.sgo_n + hoff, p.sgo_l, 0, p.Lq);
  F of[8];
  {
    const T* orow = (const T*)p.o + (int64_t)n * p.so_n + hoff + (int64_t)qc * p.so_l + 256 * h +
                    8 * g;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) of[ks] = *(const F*)(orow + 32 * ks);
  }
  const float lse2 = p.lse[(int64_t)nh * p.Lq + qc] * 1.4426950408889634f;
  int kb4[4], tb8[8];
#pragma unroll
  for (int m = 0; m < 4; ++m) kb4[m] = row_base(m, li, g, h);
#pragma unroll
  for (int c = 0; c < 8; ++c) tb8[c] = tr_base(c, li, g, h);
  wait_vmcnt<0>();
  lds_barrier();                                  // the four images landed

  // row-operand fragments of rows qr (Q, dO) from the images; this half's part of Delta
  F qf[8], df[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int off = kb4[ks & 3] + 256 * (ks >> 2) + 1024 * rb;
    qf[ks] = *(const F*)(qimg + off);
    df[ks] = *(const F*)(dimg + off);
  }
  float dpart = 0.f;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) dpart += (float)of[ks][e] * (float)df[ks][e];
  dpart = pl_pair_sum(dpart);
  // partial scores (K) and dP (V) over this wave's 256 dims
  f32x4 s[2], d[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    d[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int o_ = kb4[ks & 3] + 256 * (ks >> 2) + 16384 * kt;
      s[kt] = mfma16(*(const F*)(kimg + o_), qf[ks], s[kt]);
      d[kt] = mfma16(*(const F*)(vimg + o_), df[ks], d[kt]);
    }
  f32x4* xmine = (f32x4*)(xch + w * AS_XB) + lane;
  const f32x4* xpart = (const f32x4*)(xch + (w ^ 2) * AS_XB) + lane;
  xmine[0] = s[0];
  xmine[64] = s[1];
  xmine[128] = d[0];
  xmine[192] = d[1];
  dlt[w * 64 + lane] = dpart;
  lds_barrier();
  float delta;
  {
    const float part = dlt[(w ^ 2) * 64 + lane];
    delta = h == 0 ? dpart + part : part + dpart;
  }
  F dsf;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const f32x4 ps = xpart[64 * kt], pd = xpart[128 + 64 * kt];
    const f32x4 sf = h == 0 ? s[kt] + ps : ps + s[kt];
    const f32x4 dfull = h == 0 ? d[kt] + pd : pd + d[kt];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * kt + 4 * g + r;
      const bool in = key < p.Lk && qr < p.Lq;
      const float pv = in ? __builtin_amdgcn_exp2f(sf[r] * p.scale_log2 - lse2) : 0.f;
      const T ds = from_f<T>(p.scale * pv * (dfull[r] - delta));
      dsf[kt * 4 + r] = ds;
      // both halves hold the same values: half 0 writes P^T, half 1 dS^T
      if (h == 0) pt[key * AS_TLD + qr] = from_f<T>(pv);
      else dst[key * AS_TLD + qr] = ds;
    }
  }
  // dQ[qr][256 h + 16 t + 4 g + r] = sum_k dS(k) K[k][.] (transposed K fragments)
  {
    f32x4 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const char* a = kimg + tb8[t & 7] + 256 * (t >> 3);
      const Hf lo = tr_read<Hf>(a);
      const Hf hi = tr_read<Hf>(a + 16384);
      acc[t] = mfma16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), dsf,
                      f32x4{0.f, 0.f, 0.f, 0.f});
    }
    store_acc_direct<T>(acc, 1.f,
                        (T*)p.dq + (int64_t)n * p.sdq_n + hoff + (int64_t)qr * p.sdq_l + 256 * h,
                        qr < p.Lq);
  }
  lds_barrier();                                  // P^T / dS^T complete
  // key side: rows kr = keys; B fragments = P^T / dS^T rows, query slots in the transposed
  // fragments' k order (16 (e >> 2) + 4 g + (e & 3))
  const int kr = rb + li;
  F ptf, dstf;
  {
    const Hf a0 = *(const Hf*)(pt + kr * AS_TLD + 4 * g);
    const Hf a1 = *(const Hf*)(pt + kr * AS_TLD + 16 + 4 * g);
    const Hf b0 = *(const Hf*)(dst + kr * AS_TLD + 4 * g);
    const Hf b1 = *(const Hf*)(dst + kr * AS_TLD + 16 + 4 * g);
    ptf = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
    dstf = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  {   // dV[kr][.] = sum_q P(q, kr) dO[q][.]
    f32x4 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const char* a = dimg + tb8[t & 7] + 256 * (t >> 3);
      const Hf lo = tr_read<Hf>(a);
      const Hf hi = tr_read<Hf>(a + 16384);
      acc[t] = mfma16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), ptf,
                      f32x4{0.f, 0.f, 0.f, 0.f});
    }
    store_acc_direct<T>(acc, 1.f,
                        (T*)p.dv + (int64_t)n * p.sdv_n + hoff + (int64_t)kr * p.sdv_l + 256 * h,
                        kr < p.Lk);
  }
  {   // dK[kr][.] = sum_q dS(q, kr) Q[q][.]
    f32x4 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const char* a = qimg + tb8[t & 7] + 256 * (t >> 3);
      const Hf lo = tr_read<Hf>(a);
      const Hf hi = tr_read<Hf>(a + 16384);
      acc[t] = mfma16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), dstf,
                      f32x4{0.f, 0.f, 0.f, 0.f});
    }
    JMT_DCHECK(nh < gridDim.x);
    store_acc_direct<T>(acc, 1.f,
                        (T*)p.dk + (int64_t)n * p.sdk_n + hoff + (int64_t)kr * p.sdk_l + 256 * h,
                        kr < p.Lk);
  }
}

template <typename K>
static void as_set_lds(K fn, int bytes) {
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

static int as_check(const char* name, int N, int H, int Lq, int Lk, const void* const* ptrs,
                    int nptr, const int64_t* strides, int nstr) {
  JMT_CHECK_ARG(N > 0 && H > 0 && Lq >= 1 && Lq <= AS_L && Lk >= 1 && Lk <= AS_L &&
                    (int64_t)N * H < (1LL << 31),
                "%s: bad sizes (N %d H %d Lq %d Lk %d)", name, N, H, Lq, Lk);
  for (int i = 0; i < nptr; ++i)
    JMT_CHECK_ARG(ptrs[i] != nullptr && ((uintptr_t)ptrs[i] & 15) == 0,
                  "%s: operand %d null or not 16-B aligned", name, i);
  for (int i = 0; i < nstr; ++i)
    JMT_CHECK_ARG(strides[i] % 8 == 0, "%s: stride %d not a multiple of 8 elements", name, i);
  return JMT_OK;
}

}  // namespace jmt

using namespace jmt;

extern "C" int jmt_attn_short_supported(int dt, int dh, int Lq, int Lk) {
  return (dt == JMT_BF16 || dt == JMT_F16) && dh == AT_DH && Lq >= 1 && Lq <= AS_L && Lk >= 1 &&
         Lk <= AS_L;
}

extern "C" int jmt_attn_short_fwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* q,
                                  int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l,
                                  int64_t sk_n, const void* v, int64_t sv_l, int64_t sv_n, void* o,
                                  int64_t so_l, int64_t so_n, float scale, float* lse,
                                  void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_short_supported(dt, dh, Lq, Lk))
    return set_error(JMT_ERR_UNSUPPORTED,
                     "jmt_attn_short_fwd: dtype %d / head dim %d / Lq %d / Lk %d not supported",
                     dt, dh, Lq, Lk);
  const void* ptrs[] = {q, k, v, o};
  const int64_t strides[] = {sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n};
  int rc = as_check("jmt_attn_short_fwd", N, H, Lq, Lk, ptrs, 4, strides, 8);
  if (rc != JMT_OK) return rc;
  AttnShortArgs a = {};
  a.q = q; a.k = k; a.v = v; a.out = o; a.lse = lse;
  a.sq_l = sq_l; a.sq_n = sq_n; a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n;
  a.so_l = so_l; a.so_n = so_n;
  a.Lq = Lq; a.Lk = Lk; a.H = H;
  a.scale = scale;
  a.scale_log2 = scale * 1.4426950408889634f;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(N * H));
  if (dt == JMT_BF16) {
    static bool once = (as_set_lds(attn_short_fwd_kernel<__bf16>, ASF_LDS), true);
    (void)once;
    hipLaunchKernelGGL(attn_short_fwd_kernel<__bf16>, grid, dim3(256), (size_t)ASF_LDS, st, a);
  } else {
    static bool once = (as_set_lds(attn_short_fwd_kernel<_Float16>, ASF_LDS), true);
    (void)once;
    hipLaunchKernelGGL(attn_short_fwd_kernel<_Float16>, grid, dim3(256), (size_t)ASF_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_short_fwd");
  return JMT_OK;
}

extern "C" int jmt_attn_short_bwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* go,
                                  int64_t sgo_l, int64_t sgo_n, const void* o, int64_t so_l,
                                  int64_t so_n, const void* q, int64_t sq_l, int64_t sq_n,
                                  const void* k, int64_t sk_l, int64_t sk_n, const void* v,
                                  int64_t sv_l, int64_t sv_n, const float* lse, void* dq,
                                  int64_t sdq_l, int64_t sdq_n, void* dk, int64_t sdk_l,
                                  int64_t sdk_n, void* dv, int64_t sdv_l, int64_t sdv_n,
                                  float scale, void* stream) {
  if (N == 0 || Lq == 0) return JMT_OK;
  if (!jmt_attn_short_supported(dt, dh, Lq, Lk))
    return set_error(JMT_ERR_UNSUPPORTED,
                     "jmt_attn_short_bwd: dtype %d / head dim %d / Lq %d / Lk %d not supported",
                     dt, dh, Lq, Lk);
  const void* ptrs[] = {go, o, q, k, v, dq, dk, dv};
  const int64_t strides[] = {sgo_l, sgo_n, so_l, so_n, sq_l, sq_n, sk_l, sk_n, sv_l, sv_n,
                             sdq_l, sdq_n, sdk_l, sdk_n, sdv_l, sdv_n};
  int rc = as_check("jmt_attn_short_bwd", N, H, Lq, Lk, ptrs, 8, strides, 16);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(lse != nullptr, "jmt_attn_short_bwd: lse missing");
  AttnShortArgs a = {};
  a.q = q; a.k = k; a.v = v; a.o = o; a.go = go; a.lse = (float*)lse;
  a.dq = dq; a.dk = dk; a.dv = dv;
  a.sq_l = sq_l; a.sq_n = sq_n; a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n;
  a.so_l = so_l; a.so_n = so_n; a.sgo_l = sgo_l; a.sgo_n = sgo_n;
  a.sdq_l = sdq_l; a.sdq_n = sdq_n; a.sdk_l = sdk_l; a.sdk_n = sdk_n; a.sdv_l = sdv_l;
  a.sdv_n = sdv_n;
  a.Lq = Lq; a.Lk = Lk; a.H = H;
  a.scale = scale;
  a.scale_log2 = scale * 1.4426950408889634f;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(N * H));
  if (dt == JMT_BF16) {
    static bool once = (as_set_lds(attn_short_bwd_kernel<__bf16>, ASB_LDS), true);
    (void)once;
    hipLaunchKernelGGL(attn_short_bwd_kernel<__bf16>, grid, dim3(256), (size_t)ASB_LDS, st, a);
  } else {
    static bool once = (as_set_lds(attn_short_bwd_kernel<_Float16>, ASB_LDS), true);
    (void)once;
    hipLaunchKernelGGL(attn_short_bwd_kernel<_Float16>, grid, dim3(256), (size_t)ASB_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_short_bwd");
  return JMT_OK;
}
