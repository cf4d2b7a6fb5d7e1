// Attention over very short sequences (Lk <= 8), head width E = 512 split into H heads:
//   forward  O_i = sum_j P_ij V_j,  P_i = softmax_j(scale Q_i . K_j)      (P kept, fp32)
//   backward dV_j = sum_i P_ij dO_i, dP_ij = dO_i . V_j, dS_ij = scale P_ij (dP_ij - sum_j P dP),
//            dQ_i = sum_j dS_ij K_j, dK_j = sum_i dS_ij Q_i
// The SELF_ATTEN head of MultimodalTransformer_w_JR attends over the 6 cross-attention outputs of
// every (window, clip) pair — 6-token sequences, batch B*T (mm_multi_transformers.py:169-199) —
// and Intra_modal_transformer_fusion over 2 backbone features (intra_modal_transformer_fusion.py:
// 93-108).  With 64-row tiles (attn.hip) such sequences waste >90 % of every MFMA and stage a
// 64-key K / V tile per sequence; here the work is HBM-bound by construction:
//  * one wave per sequence, lane l owns head dims 8 l .. 8 l + 7 of the 512 (head h = the lanes
//    l * 8 / dh == h): every Q / K / V / O row is ONE coalesced 1 KiB wave load / store;
//  * the Lq x Lk dot products accumulate in fp32 per lane and are reduced over the head's lane
//    group with xor shuffles; softmax in fp32 on every lane (no P rounding);
//  * P (fp32, N * H * Lq * Lk) is saved for the backward, which needs no score recompute.
// Bytes per sequence (forward): (Lq + 2 Lk + Lq) * E * |T| — the kernel's roofline is HBM.
#include "common.h"

namespace jmt {

constexpr int SA_E = 512;
constexpr int SA_WPB = 4;          // waves (sequences) per block

struct SmallAttnArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* go;
  void* o;
  void* dq;
  void* dk;
  void* dv;
  float* p;
  int64_t sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n;
  int64_t sdq_l, sdq_n, sdk_l, sdk_n, sdv_l, sdv_n;
  int N, H, Lq;
  float scale;
};

// 8 consecutive elements of a row as floats
template <typename T>
__device__ __forceinline__ void load8(const T* src, float (&x)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    const uint4 u = *(const uint4*)src;
    const T* h = (const T*)&u;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (float)h[e];
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* dst, const float (&x)[8]) {
  if constexpr (sizeof(T) == 4) {
    *(float4*)dst = make_float4(x[0], x[1], x[2], x[3]);
    *(float4*)(dst + 4) = make_float4(x[4], x[5], x[6], x[7]);
  } else {
    T h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = from_f<T>(x[e]);
    *(uint4*)dst = *(const uint4*)h;
  }
}

// sum over the G = dh / 8 lanes of one head (G a power of two, 1 .. 64)
__device__ __forceinline__ float group_sum(float x, int G) {
  for (int off = G >> 1; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

template <typename T, int LK>
__global__ __launch_bounds__(64 * SA_WPB) void small_attn_fwd_kernel(SmallAttnArgs p) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * SA_WPB + (threadIdx.x >> 6);
  if (n >= p.N) return;                                   // whole waves
  const int G = SA_E / 8 / p.H;                           // lanes per head
  const int hd = lane / G;
  const int c = 8 * lane;
  float k[LK][8], v[LK][8];
#pragma unroll
  for (int j = 0; j < LK; ++j) {
    load8((const T*)p.k + (int64_t)n * p.sk_n + (int64_t)j * p.sk_l + c, k[j]);
    load8((const T*)p.v + (int64_t)n * p.sv_n + (int64_t)j * p.sv_l + c, v[j]);
  }
  for (int i = 0; i < p.Lq; ++i) {
    float q[8];
    load8((const T*)p.q + (int64_t)n * p.sq_n + (int64_t)i * p.sq_l + c, q);
    float s[LK], mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(q[e], k[j][e], d);
      s[j] = group_sum(d, G) * p.scale;
      mx = fmaxf(mx, s[j]);
    }
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      s[j] = __expf(s[j] - mx);
      l += s[j];
    }
    const float inv = 1.f / l;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      s[j] *= inv;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(s[j], v[j][e], o[e]);
    }
    store8((T*)p.o + (int64_t)n * p.so_n + (int64_t)i * p.so_l + c, o);
    if (p.p && (lane % G) == 0) {
      float* pr = p.p + (((int64_t)n * p.H + hd) * p.Lq + i) * LK;
#pragma unroll
      for (int j = 0; j < LK; ++j) pr[j] = s[j];
    }
  }
}

template <typename T, int LK>
__global__ __launch_bounds__(64 * SA_WPB) void small_attn_bwd_kernel(SmallAttnArgs p) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * SA_WPB + (threadIdx.x >> 6);
  if (n >= p.N) return;
  const int G = SA_E / 8 / p.H;
  const int hd = lane / G;
  const int c = 8 * lane;
  float k[LK][8], v[LK][8], dk[LK][8], dv[LK][8];
#pragma unroll
  for (int j = 0; j < LK; ++j) {
    load8((const T*)p.k + (int64_t)n * p.sk_n + (int64_t)j * p.sk_l + c, k[j]);
    load8((const T*)p.v + (int64_t)n * p.sv_n + (int64_t)j * p.sv_l + c, v[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) { dk[j][e] = 0.f; dv[j][e] = 0.f; }
  }
  for (int i = 0; i < p.Lq; ++i) {
    float q[8], go[8];
    load8((const T*)p.q + (int64_t)n * p.sq_n + (int64_t)i * p.sq_l + c, q);
    load8((const T*)p.go + (int64_t)n * p.so_n + (int64_t)i * p.so_l + c, go);
    const float* pr = p.p + (((int64_t)n * p.H + hd) * p.Lq + i) * LK;
    float pij[LK], dp[LK], dsum = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      pij[j] = pr[j];
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(go[e], v[j][e], d);
      dp[j] = group_sum(d, G);
      dsum = fmaf(pij[j], dp[j], dsum);
    }
    float dq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dq[e] = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      const float ds = p.scale * pij[j] * (dp[j] - dsum);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dq[e] = fmaf(ds, k[j][e], dq[e]);
        dk[j][e] = fmaf(ds, q[e], dk[j][e]);
        dv[j][e] = fmaf(pij[j], go[e], dv[j][e]);
      }
    }
    store8((T*)p.dq + (int64_t)n * p.sdq_n + (int64_t)i * p.sdq_l + c, dq);
  }
#pragma unroll
  for (int j = 0; j < LK; ++j) {
    store8((T*)p.dk + (int64_t)n * p.sdk_n + (int64_t)j * p.sdk_l + c, dk[j]);
    store8((T*)p.dv + (int64_t)n * p.sdv_n + (int64_t)j * p.sdv_l + c, dv[j]);
  }
}

template <typename T, int LK, bool BWD>
static bool launch_static(int Lq, const SmallAttnArgs& a, hipStream_t st);

template <int LK, bool BWD>
static void launch_lk(int dt, const SmallAttnArgs& a, hipStream_t st) {
  if (dt == JMT_BF16 && launch_static<__bf16, LK, BWD>(a.Lq, a, st)) return;
  if (dt == JMT_F16 && launch_static<_Float16, LK, BWD>(a.Lq, a, st)) return;
  const dim3 grid((unsigned)((a.N + SA_WPB - 1) / SA_WPB)), block(64 * SA_WPB);
#define JMT_SA(T)                                                                           \
  if (BWD) hipLaunchKernelGGL((small_attn_bwd_kernel<T, LK>), grid, block, 0, st, a);       \
  else hipLaunchKernelGGL((small_attn_fwd_kernel<T, LK>), grid, block, 0, st, a);
  if (dt == JMT_F32) { JMT_SA(float) }
  else if (dt == JMT_BF16) { JMT_SA(__bf16) }
  else { JMT_SA(_Float16) }
#undef JMT_SA
}

// ---- 16-bit, Lq fixed at compile time (Lq == Lk: self-attention; Lq == 1: last-token query):
// every row load and P read of a sequence is issued before the first use, so a wave pays ONE
// memory latency per sequence instead of one per query row (the runtime-Lq kernels above walk
// the query rows in a loop whose loads wait on each other's iteration).  Rows stay packed
// (one 16-B register quad each) until used.
template <typename T>
__device__ __forceinline__ void unpack8(const uint4& u, float (&x)[8]) {
  const T* h = (const T*)&u;
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (float)h[e];
}

template <typename T, int LK, int LQ>
__global__ __launch_bounds__(64 * SA_WPB) void small_attn_fwd_static(SmallAttnArgs p) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * SA_WPB + (threadIdx.x >> 6);
  if (n >= p.N) return;
  const int G = SA_E / 8 / p.H;
  const int hd = lane / G;
  const int c = 8 * lane;
  uint4 kr[LK], vr[LK], qr[LQ];
#pragma unroll
  for (int j = 0; j < LK; ++j) {
    kr[j] = *(const uint4*)((const T*)p.k + (int64_t)n * p.sk_n + (int64_t)j * p.sk_l + c);
    vr[j] = *(const uint4*)((const T*)p.v + (int64_t)n * p.sv_n + (int64_t)j * p.sv_l + c);
  }
#pragma unroll
  for (int i = 0; i < LQ; ++i)
    qr[i] = *(const uint4*)((const T*)p.q + (int64_t)n * p.sq_n + (int64_t)i * p.sq_l + c);
#pragma unroll
  for (int i = 0; i < LQ; ++i) {
    float q[8];
    unpack8<T>(qr[i], q);
    float s[LK], mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      float kk[8];
      unpack8<T>(kr[j], kk);
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(q[e], kk[e], d);
      s[j] = group_sum(d, G) * p.scale;
      mx = fmaxf(mx, s[j]);
    }
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      s[j] = __expf(s[j] - mx);
      l += s[j];
    }
    const float inv = 1.f / l;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      s[j] *= inv;
      float vv[8];
      unpack8<T>(vr[j], vv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(s[j], vv[e], o[e]);
    }
    store8((T*)p.o + (int64_t)n * p.so_n + (int64_t)i * p.so_l + c, o);
    if (p.p && (lane % G) == 0) {
      float* pr = p.p + (((int64_t)n * p.H + hd) * LQ + i) * LK;
#pragma unroll
      for (int j = 0; j < LK; ++j) pr[j] = s[j];
    }
  }
}

template <typename T, int LK, int LQ>
__global__ __launch_bounds__(64 * SA_WPB) void small_attn_bwd_static(SmallAttnArgs p) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * SA_WPB + (threadIdx.x >> 6);
  if (n >= p.N) return;
  const int G = SA_E / 8 / p.H;
  const int hd = lane / G;
  const int c = 8 * lane;
  uint4 kr[LK], vr[LK], qr[LQ], gr[LQ];
  float P[LQ][LK];
#pragma unroll
  for (int j = 0; j < LK; ++j) {
    kr[j] = *(const uint4*)((const T*)p.k + (int64_t)n * p.sk_n + (int64_t)j * p.sk_l + c);
    vr[j] = *(const uint4*)((const T*)p.v + (int64_t)n * p.sv_n + (int64_t)j * p.sv_l + c);
  }
  const float* pb = p.p + ((int64_t)n * p.H + hd) * LQ * LK;
#pragma unroll
  for (int i = 0; i < LQ; ++i) {
    qr[i] = *(const uint4*)((const T*)p.q + (int64_t)n * p.sq_n + (int64_t)i * p.sq_l + c);
    gr[i] = *(const uint4*)((const T*)p.go + (int64_t)n * p.so_n + (int64_t)i * p.so_l + c);
#pragma unroll
    for (int j = 0; j < LK; ++j) P[i][j] = pb[i * LK + j];
  }
  // dS = scale P o (dP - rowsum(P o dP)),  dP_ij = dO_i . V_j
  float dS[LQ][LK];
#pragma unroll
  for (int i = 0; i < LQ; ++i) {
    float g[8];
    unpack8<T>(gr[i], g);
    float dsum = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      float vv[8];
      unpack8<T>(vr[j], vv);
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(g[e], vv[e], d);
      dS[i][j] = group_sum(d, G);
      dsum = fmaf(P[i][j], dS[i][j], dsum);
    }
#pragma unroll
    for (int j = 0; j < LK; ++j) dS[i][j] = p.scale * P[i][j] * (dS[i][j] - dsum);
  }
#pragma unroll
  for (int i = 0; i < LQ; ++i) {                               // dQ_i = sum_j dS_ij K_j
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int j = 0; j < LK; ++j) {
      float kk[8];
      unpack8<T>(kr[j], kk);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(dS[i][j], kk[e], acc[e]);
    }
    store8((T*)p.dq + (int64_t)n * p.sdq_n + (int64_t)i * p.sdq_l + c, acc);
  }
#pragma unroll
  for (int j = 0; j < LK; ++j) {                               // dK_j, dV_j
    float ak[8], av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { ak[e] = 0.f; av[e] = 0.f; }
#pragma unroll
    for (int i = 0; i < LQ; ++i) {
      float qq[8], gg[8];
      unpack8<T>(qr[i], qq);
      unpack8<T>(gr[i], gg);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ak[e] = fmaf(dS[i][j], qq[e], ak[e]);
        av[e] = fmaf(P[i][j], gg[e], av[e]);
      }
    }
    store8((T*)p.dk + (int64_t)n * p.sdk_n + (int64_t)j * p.sdk_l + c, ak);
    store8((T*)p.dv + (int64_t)n * p.sdv_n + (int64_t)j * p.sdv_l + c, av);
  }
}

template <typename T, int LK, bool BWD>
static bool launch_static(int Lq, const SmallAttnArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.N + SA_WPB - 1) / SA_WPB)), block(64 * SA_WPB);
  if (Lq == LK) {
    if (BWD) hipLaunchKernelGGL((small_attn_bwd_static<T, LK, LK>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((small_attn_fwd_static<T, LK, LK>), grid, block, 0, st, a);
    return true;
  }
  if (Lq == 1) {
    if (BWD) hipLaunchKernelGGL((small_attn_bwd_static<T, LK, 1>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((small_attn_fwd_static<T, LK, 1>), grid, block, 0, st, a);
    return true;
  }
  return false;
}

template <bool BWD>
static void launch(int dt, int Lk, const SmallAttnArgs& a, hipStream_t st) {
  switch (Lk) {
    case 1: launch_lk<1, BWD>(dt, a, st); break;
    case 2: launch_lk<2, BWD>(dt, a, st); break;
    case 3: launch_lk<3, BWD>(dt, a, st); break;
    case 4: launch_lk<4, BWD>(dt, a, st); break;
    case 5: launch_lk<5, BWD>(dt, a, st); break;
    case 6: launch_lk<6, BWD>(dt, a, st); break;
    case 7: launch_lk<7, BWD>(dt, a, st); break;
    default: launch_lk<8, BWD>(dt, a, st); break;
  }
}

static int check(const char* name, int dt, int N, int H, int Lq, int Lk, int E,
                 const void* const* ptrs, int nptr, const int64_t* strides, int nstr) {
  JMT_CHECK_ARG(dt == JMT_F32 || dt == JMT_BF16 || dt == JMT_F16, "%s: dtype %d", name, dt);
  JMT_CHECK_ARG(E == SA_E && H >= 1 && H <= 64 && (SA_E / 8) % H == 0 &&
                    (((SA_E / 8 / H) & (SA_E / 8 / H - 1)) == 0),
                "%s: E must be %d and E / 8 / H a power of two (E %d, H %d)", name, SA_E, E, H);
  JMT_CHECK_ARG(N > 0 && Lq >= 1 && Lq <= 8 && Lk >= 1 && Lk <= 8, "%s: sizes (Lq %d, Lk %d)",
                name, Lq, Lk);
  const int align = dt == JMT_F32 ? 32 : 16;
  for (int i = 0; i < nptr; ++i)
    JMT_CHECK_ARG(ptrs[i] && ((uintptr_t)ptrs[i] % align) == 0,
                  "%s: operand %d null or not %d-B aligned", name, i, align);
  for (int i = 0; i < nstr; ++i)
    JMT_CHECK_ARG(strides[i] % 8 == 0, "%s: stride %d not a multiple of 8", name, i);
  return JMT_OK;
}

}  // namespace jmt

using namespace jmt;

extern "C" int jmt_small_attn_fwd(int dt, int N, int H, int Lq, int Lk, int E, const void* q,
                                  int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l,
                                  int64_t sk_n, const void* v, int64_t sv_l, int64_t sv_n,
                                  void* o, int64_t so_l, int64_t so_n, float scale, float* p_out,
                                  void* stream) {
  if (N == 0) return JMT_OK;
  const void* ptrs[] = {q, k, v, o};
  const int64_t st[] = {sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, so_l, so_n};
  int rc = check("jmt_small_attn_fwd", dt, N, H, Lq, Lk, E, ptrs, 4, st, 8);
  if (rc != JMT_OK) return rc;
  SmallAttnArgs a = {};
  a.q = q; a.k = k; a.v = v; a.o = o; a.p = p_out;
  a.sq_l = sq_l; a.sq_n = sq_n; a.sk_l = sk_l; a.sk_n = sk_n; a.sv_l = sv_l; a.sv_n = sv_n;
  a.so_l = so_l; a.so_n = so_n;
  a.N = N; a.H = H; a.Lq = Lq; a.scale = scale;
  launch<false>(dt, Lk, a, as_stream(stream));
  JMT_LAUNCH_CHECK("jmt_small_attn_fwd");
  return JMT_OK;
}

extern "C" int jmt_small_attn_bwd(int dt, int N, int H, int Lq, int Lk, int E, const void* go,
                                  int64_t sgo_l, int64_t sgo_n, const void* q, int64_t sq_l,
                                  int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n,
                                  const void* v, int64_t sv_l, int64_t sv_n, const float* p,
                                  void* dq, int64_t sdq_l, int64_t sdq_n, void* dk,
                                  int64_t sdk_l, int64_t sdk_n, void* dv, int64_t sdv_l,
                                  int64_t sdv_n, float scale, void* stream) {
  if (N == 0) return JMT_OK;
  const void* ptrs[] = {go, q, k, v, dq, dk, dv};
  const int64_t st[] = {sgo_l, sgo_n, sq_l, sq_n, sk_l, sk_n, sv_l, sv_n, sdq_l, sdq_n,
                        sdk_l, sdk_n, sdv_l, sdv_n};
  int rc = check("jmt_small_attn_bwd", dt, N, H, Lq, Lk, E, ptrs, 7, st, 14);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(p != nullptr, "jmt_small_attn_bwd: P (the forward's probabilities) missing");
  SmallAttnArgs a = {};
  a.go = go; a.q = q; a.k = k; a.v = v; a.dq = dq; a.dk = dk; a.dv = dv;
  a.p = const_cast<float*>(p);
  a.so_l = sgo_l; a.so_n = sgo_n; a.sq_l = sq_l; a.sq_n = sq_n; a.sk_l = sk_l; a.sk_n = sk_n;
  a.sv_l = sv_l; a.sv_n = sv_n; a.sdq_l = sdq_l; a.sdq_n = sdq_n; a.sdk_l = sdk_l;
  a.sdk_n = sdk_n; a.sdv_l = sdv_l; a.sdv_n = sdv_n;
  a.N = N; a.H = H; a.Lq = Lq; a.scale = scale;
  launch<true>(dt, Lk, a, as_stream(stream));
  JMT_LAUNCH_CHECK("jmt_small_attn_bwd");
  return JMT_OK;
}
