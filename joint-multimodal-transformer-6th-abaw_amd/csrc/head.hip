// Output layer of the V / A regressor pair (two_transformers.py:104-114: Linear(dim, 128) ->
// ReLU -> Dropout(0) -> Linear(128, k), applied to the same input by `vregressor` and
// `aregressor`, :125-126) as two small row kernels instead of three GEMM launches.
//
// The two heads read the halves of ONE hidden buffer h = [h_0 | h_1] (rows x 2*128, row stride
// ldh, 16-bit; the first layers' grouped GEMM writes it, ReLU applied):
//   forward : y_g[r][o]  = sum_j h_g[r][j] W2_g[o][j] + b2_g[o]          (fp32 accumulation)
//   backward: dh_g[r][j] = [h_g[r][j] > 0] sum_o gy_g[r][o] W2_g[o][j]     (16-bit out)
//             dW2_g[o][j] += sum_r gy_g[r][o] h_g[r][j],  db2_g[o] += sum_r gy_g[r][o]
// k = nout <= 24 (1 for the V / A regressors, 20 for configs[4]'s expression-style head).
//
// A wave owns one row at a time: lanes 0-31 head 0, lanes 32-63 head 1, each lane 4 consecutive
// hidden units, so a row of h is one 512-B coalesced access; the k dot products reduce over the
// head's 32 lanes with xor shuffles.  The weight / bias gradients are sums over all B*T rows:
// per-lane fp32 accumulators, summed over the block's waves in LDS in a fixed order, one fp32
// slab per block, and a fixed-order reduce over the blocks (deterministic; the graph replay is
// bit-identical to eager).  The weight gradient is an exact fp32 sum of fp32 gy x (16-bit h as
// fp32), as the GEMM path's fp32 route did (functional.MLPFn: these sums nearly cancel for the
// CCC loss, so a 16-bit rounded copy of gy is avoided).
//
// Replaces, per step (B=64, T=300): the N = 1 forward GEMM (10 us), the K = 1 masked dgrad GEMM
// (16 us), the M = 1 fp32 weight-gradient GEMM with its 256-way split-K (36 us) and the bias
// column sum; HBM-bound: the kernels read h once (9.8 MB) and write dh once.
#include "common.h"

namespace jmt {

constexpr int HD_HID = 128;        // hidden width of the regressors (two_transformers.py:104)
constexpr int HD_KMAX = 24;        // largest k of the fused path
constexpr int HD_RPW = 16;         // rows per wave per block

template <typename T> struct V4l;   // 4 consecutive 16-bit values <-> 8-B accesses
template <> struct V4l<__bf16> {
  static __device__ __forceinline__ void ld(const __bf16* p, float* v) {
    const uint2 u = *(const uint2*)p;
    const __bf16* e = (const __bf16*)&u;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)e[i];
  }
  static __device__ __forceinline__ void st(__bf16* p, const float* v) {
    __bf16 e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = (__bf16)v[i];
    *(uint2*)p = *(const uint2*)e;
  }
};
template <> struct V4l<_Float16> {
  static __device__ __forceinline__ void ld(const _Float16* p, float* v) {
    const uint2 u = *(const uint2*)p;
    const _Float16* e = (const _Float16*)&u;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)e[i];
  }
  static __device__ __forceinline__ void st(_Float16* p, const float* v) {
    _Float16 e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = (_Float16)v[i];
    *(uint2*)p = *(const uint2*)e;
  }
};

// sum over the 32 lanes of this lane's half-wave
__device__ __forceinline__ float half_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

struct HeadArgs {
  const void* h;
  int64_t ldh;
  const void* w2[2];     // (k, 128) each, compute dtype
  const float* b2[2];
  void* y[2];            // forward outputs (rows, k) at row stride ldy
  int64_t ldy;
  const void* gy[2];     // backward: incoming gradients (rows, k) at row stride ldgy
  int64_t ldgy;
  void* dh;              // backward: (rows, 256) at row stride lddh
  int64_t lddh;
  float* partials;       // backward: per block 2 * k * (128 + 1) floats
  float* dw2[2];
  float* db2[2];
  int64_t rows;
  int k;
};

template <typename TH, typename TY, int K>
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 5, c = 4 * (lane & 31);
  const int k = K == 1 ? 1 : a.k;
  float wv[K][4];
  const TH* W = (const TH*)a.w2[g];
#pragma unroll
  for (int o = 0; o < K; ++o)
    if (o < k) V4l<TH>::ld(W + o * HD_HID + c, wv[o]);
  const float* bp = a.b2[g];
  TY* yp = (TY*)a.y[g];
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + w) * HD_RPW;
  for (int i = 0; i < HD_RPW; ++i) {
    const int64_t r = r0 + i;
    if (r >= a.rows) break;
    float hv[4];
    V4l<TH>::ld((const TH*)a.h + r * a.ldh + g * HD_HID + c, hv);
#pragma unroll
    for (int o = 0; o < K; ++o) {
      if (o < k) {            // (no break: the loop must unroll to keep wv in registers)
        float s = hv[0] * wv[o][0] + hv[1] * wv[o][1] + hv[2] * wv[o][2] + hv[3] * wv[o][3];
        s = half_sum(s);
        if ((lane & 31) == 0) yp[r * a.ldy + o] = from_f<TY>(s + (bp ? bp[o] : 0.f));
      }
    }
  }
}

template <typename TH, typename TG, int K>
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadArgs a) {
  __shared__ float red[2][HD_KMAX * HD_HID + HD_KMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 5, c = 4 * (lane & 31);
  const int k = K == 1 ? 1 : a.k;
  float wv[K][4], aw[K][4], ab[K];
  const TH* W = (const TH*)a.w2[g];
#pragma unroll
  for (int o = 0; o < K; ++o) {
    if (o < k) V4l<TH>::ld(W + o * HD_HID + c, wv[o]);
    ab[o] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) aw[o][e] = 0.f;
  }
  const TG* gp = (const TG*)a.gy[g];
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + w) * HD_RPW;
  for (int i = 0; i < HD_RPW; ++i) {
    const int64_t r = r0 + i;
    if (r >= a.rows) break;
    float hv[4], d[4] = {0.f, 0.f, 0.f, 0.f};
    V4l<TH>::ld((const TH*)a.h + r * a.ldh + g * HD_HID + c, hv);
#pragma unroll
    for (int o = 0; o < K; ++o) {
      if (o < k) {
        const float gy = to_f(gp[r * a.ldgy + o]);
        ab[o] += gy;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d[e] += gy * wv[o][e];
          aw[o][e] += gy * hv[e];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = hv[e] > 0.f ? d[e] : 0.f;
    V4l<TH>::st((TH*)a.dh + r * a.lddh + g * HD_HID + c, d);
  }
  // block sum of the weight / bias gradient partials, waves added in a fixed order
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int o = 0; o < K; ++o) {
        if (o < k) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float& t = red[g][o * HD_HID + c + e];
            t = ww == 0 ? aw[o][e] : t + aw[o][e];
          }
          if ((lane & 31) == 0) {
            float& t = red[g][HD_KMAX * HD_HID + o];
            t = ww == 0 ? ab[o] : t + ab[o];
          }
        }
      }
    }
    __syncthreads();
  }
  // compact slab of this block: per head k*128 weight sums then k bias sums
  const int SK = k * (HD_HID + 1);
  float* slab = a.partials + (int64_t)blockIdx.x * 2 * SK;
  for (int i = threadIdx.x; i < 2 * SK; i += blockDim.x) {
    const int gg = i / SK, j = i % SK;
    slab[i] = j < k * HD_HID ? red[gg][j] : red[gg][HD_KMAX * HD_HID + (j - k * HD_HID)];
  }
}

// fixed-order sum of the blocks' slabs into the gradient buffers (+=): one wave per output
// (wave-uniform index), lane l adds slabs l, l + 64, ... in order, then a fixed xor butterfly;
// lane 0 stores.  (One thread per output walking all ~300 slabs serially was a 74 us chain of
// dependent L2 loads per step: profiles/r03_p1_kernel_stats.csv.)
__global__ __launch_bounds__(256) void head_reduce_kernel(HeadArgs a, int nblk) {
  const int SK = a.k * (HD_HID + 1);
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= 2 * SK) return;
  const int g = i / SK, j = i % SK;
  const bool isw = j < a.k * HD_HID;
  float* dst = isw ? a.dw2[g] : a.db2[g];
  if (!dst) return;
  float s = 0.f;
  for (int b = lane; b < nblk; b += 64) s += a.partials[(int64_t)b * 2 * SK + i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) dst[isw ? j : j - a.k * HD_HID] += s;
}

static int head_blocks(int64_t rows) { return (int)((rows + 4 * HD_RPW - 1) / (4 * HD_RPW)); }

}  // namespace jmt

using namespace jmt;

extern "C" size_t jmt_head_bwd_workspace_bytes(int64_t rows) {
  return (size_t)head_blocks(rows) * 2 * (HD_KMAX * HD_HID + HD_KMAX) * sizeof(float);
}

static int head_check(const char* name, int h_dt, int64_t rows, int hid, int k, const void* h,
                      int64_t ldh, const void* w0, const void* w1) {
  JMT_CHECK_ARG(h_dt == JMT_BF16 || h_dt == JMT_F16, "%s: h must be bf16 / f16", name);
  JMT_CHECK_ARG(hid == HD_HID, "%s: hidden width %d (128 supported)", name, hid);
  JMT_CHECK_ARG(k >= 1 && k <= HD_KMAX, "%s: k = %d (1..%d supported)", name, k, HD_KMAX);
  JMT_CHECK_ARG(rows >= 0 && h && w0 && w1, "%s: null pointer", name);
  JMT_CHECK_ARG(ldh % 4 == 0 && ((uintptr_t)h & 7) == 0 && ((uintptr_t)w0 & 7) == 0 &&
                    ((uintptr_t)w1 & 7) == 0, "%s: h / W2 not 8-B aligned", name);
  return JMT_OK;
}

extern "C" int jmt_head_fwd(int h_dt, int y_dt, int64_t rows, int hid, int k, const void* h,
                            int64_t ldh, const void* w2_0, const void* w2_1, const float* b2_0,
                            const float* b2_1, void* y_0, void* y_1, int64_t ldy, void* stream) {
  int rc = head_check("jmt_head_fwd", h_dt, rows, hid, k, h, ldh, w2_0, w2_1);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(y_dt == JMT_F32 || y_dt == h_dt, "jmt_head_fwd: y dtype");
  JMT_CHECK_ARG(y_0 && y_1 && ldy >= k, "jmt_head_fwd: outputs");
  if (rows == 0) return JMT_OK;
  HeadArgs a = {};
  a.h = h; a.ldh = ldh; a.w2[0] = w2_0; a.w2[1] = w2_1; a.b2[0] = b2_0; a.b2[1] = b2_1;
  a.y[0] = y_0; a.y[1] = y_1; a.ldy = ldy; a.rows = rows; a.k = k;
  const dim3 grid(head_blocks(rows));
  hipStream_t st = as_stream(stream);
#define HFWD(TH, TY)                                                                     \
  {                                                                                      \
    if (k == 1) hipLaunchKernelGGL((head_fwd_kernel<TH, TY, 1>), grid, dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((head_fwd_kernel<TH, TY, HD_KMAX>), grid, dim3(256), 0, st, a); \
  }
  if (h_dt == JMT_BF16) {
    if (y_dt == JMT_F32) HFWD(__bf16, float) else HFWD(__bf16, __bf16)
  } else {
    if (y_dt == JMT_F32) HFWD(_Float16, float) else HFWD(_Float16, _Float16)
  }
#undef HFWD
  JMT_LAUNCH_CHECK("jmt_head_fwd");
  return JMT_OK;
}

extern "C" int jmt_head_bwd(int h_dt, int gy_dt, int64_t rows, int hid, int k, const void* h,
                            int64_t ldh, const void* w2_0, const void* w2_1, const void* gy_0,
                            const void* gy_1, int64_t ldgy, void* dh, int64_t lddh, float* dw2_0,
                            float* dw2_1, float* db2_0, float* db2_1, float* partials,
                            void* stream) {
  int rc = head_check("jmt_head_bwd", h_dt, rows, hid, k, h, ldh, w2_0, w2_1);
  if (rc != JMT_OK) return rc;
  JMT_CHECK_ARG(gy_dt == JMT_F32 || gy_dt == h_dt, "jmt_head_bwd: gy dtype");
  JMT_CHECK_ARG(gy_0 && gy_1 && dh && partials && ldgy >= k && lddh % 4 == 0 &&
                    ((uintptr_t)dh & 7) == 0, "jmt_head_bwd: bad gradient buffers");
  if (rows == 0) return JMT_OK;
  HeadArgs a = {};
  a.h = h; a.ldh = ldh; a.w2[0] = w2_0; a.w2[1] = w2_1;
  a.gy[0] = gy_0; a.gy[1] = gy_1; a.ldgy = ldgy; a.dh = dh; a.lddh = lddh;
  a.partials = partials; a.dw2[0] = dw2_0; a.dw2[1] = dw2_1; a.db2[0] = db2_0; a.db2[1] = db2_1;
  a.rows = rows; a.k = k;
  const int nblk = head_blocks(rows);
  hipStream_t st = as_stream(stream);
#define HBWD(TH, TG)                                                                          \
  {                                                                                           \
    if (k == 1) hipLaunchKernelGGL((head_bwd_kernel<TH, TG, 1>), dim3(nblk), dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((head_bwd_kernel<TH, TG, HD_KMAX>), dim3(nblk), dim3(256), 0, st, a); \
  }
  if (h_dt == JMT_BF16) {
    if (gy_dt == JMT_F32) HBWD(__bf16, float) else HBWD(__bf16, __bf16)
  } else {
    if (gy_dt == JMT_F32) HBWD(_Float16, float) else HBWD(_Float16, _Float16)
  }
#undef HBWD
  JMT_LAUNCH_CHECK("jmt_head_bwd");
  if (dw2_0 || dw2_1 || db2_0 || db2_1) {
    const int SK = k * (HD_HID + 1);
    hipLaunchKernelGGL(head_reduce_kernel, dim3((2 * SK + 3) / 4), dim3(256), 0, st, a, nblk);
    JMT_LAUNCH_CHECK("jmt_head_bwd(reduce)");
  }
  return JMT_OK;
}
