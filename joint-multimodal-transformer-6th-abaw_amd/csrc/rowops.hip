// Row-wise / reduction kernels of the JMT path (gfx950, wave64): L2 normalize, residual+LayerNorm,
// attention softmax, bias-gradient column sums, strided copies.  All HBM-bound: one wave owns a
// row, lanes stride the row so every wave-instruction is a coalesced 256-B (f32) / 128-B (16-bit)
// access; statistics in fp32 with two passes (torch's numerics class), cross-row reductions as
// fp32 partial slabs + a second pass (deterministic, no atomics).
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace jmt {

constexpr int RB = 256;   // threads per block (4 waves)

template <typename TI>
__device__ __forceinline__ float ldr(const TI* p, int64_t i) { return to_f(p[i]); }

// ------------------------------------------------------------------ L2 normalize
template <typename TX, typename TY>
__global__ __launch_bounds__(RB) void l2norm_fwd_kernel(int64_t rows, int D, const TX* x,
                                                        int64_t ldx, TY* y, int64_t ldy,
                                                        float* inv_norm, float eps) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const TX* xr = x + r * ldx;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float v = to_f(xr[c]);
    s += v * v;
  }
  s = wave_sum(s);
  const float inv = 1.f / fmaxf(sqrtf(s), eps);
  TY* yr = y + r * ldy;
  for (int c = lane; c < D; c += 64) yr[c] = from_f<TY>(to_f(xr[c]) * inv);
  if (lane == 0) inv_norm[r] = inv;
}

// single-pass form (D = 256 NV, rows 4-aligned): the row stays in registers between the norm
// and the scaled write, so x is read once (the loop form above reads it twice)
template <typename TX, typename TY, int NV>
__global__ __launch_bounds__(RB) void l2norm_fwd_vec_kernel(int64_t rows, const TX* x,
                                                            int64_t ldx, TY* y, int64_t ldy,
                                                            float* inv_norm, float eps);

template <typename TX, typename TG, typename TD>
__global__ __launch_bounds__(RB) void l2norm_bwd_kernel(int64_t rows, int D, const TX* x,
                                                        int64_t ldx, const TG* dy, int64_t lddy,
                                                        const float* inv_norm, float eps, TD* dx,
                                                        int64_t lddx) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const TX* xr = x + r * ldx;
  const TG* gr = dy + r * lddy;
  const float inv = inv_norm[r];
  // ||x|| > eps  <=>  inv < 1/eps ; clamp_min's gradient is zero on the clamped side
  const bool clamped = !(inv < 1.f / eps);
  float dot = 0.f;
  for (int c = lane; c < D; c += 64) dot += to_f(xr[c]) * inv * to_f(gr[c]);
  dot = wave_sum(dot);
  TD* dr = dx + r * lddx;
  for (int c = lane; c < D; c += 64) {
    const float yv = to_f(xr[c]) * inv;
    const float g = to_f(gr[c]);
    dr[c] = from_f<TD>(clamped ? g * inv : (g - yv * dot) * inv);
  }
}

// ------------------------------------------------------------------ residual + LayerNorm
template <typename TI, typename TO>
__global__ __launch_bounds__(RB) void ln_fwd_kernel(int64_t rows, int D, const TI* x, int64_t ldx,
                                                    const TI* rr, int64_t ldr, const float* gamma,
                                                    const float* beta, float eps, TO* y,
                                                    int64_t ldy, float* mean, float* rstd) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const TI* xr = x + r * ldx;
  const TI* res = rr ? rr + r * ldr : nullptr;
  constexpr int MAXC = 32;   // D <= 2048
  float v[MAXC];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    float t = 0.f;
    if (c < D) {
      t = to_f(xr[c]);
      if (res) t += to_f(res[c]);
    }
    v[j] = t;
    s += t;
  }
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < D) {
      const float d = v[j] - mu;
      q += d * d;
    }
  }
  const float var = wave_sum(q) / (float)D;
  const float rs = rsqrtf(var + eps);
  TO* yr = y + r * ldy;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < D) yr[c] = from_f<TO>((v[j] - mu) * rs * gamma[c] + beta[c]);
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// LayerNorm backward rows per block (partials: ceil(rows / 16) blocks).  Each block writes NS*D
// fp32 partials, so the grouped launch (G x more blocks) takes 32 rows per block: half the
// partial traffic (37 % of the row bytes at D = 512) — 57.6 -> 54.4 us at G = 3, 129.5 ->
// 123.4 at G = 6; one group alone keeps 16 (1200 blocks; 32 measured 69 -> 80 us for three
// separate launches): profiles/r03_rowops.jsonl, r03_rowops_ln32.jsonl
constexpr int LN_ROWS_PER_BLOCK = 16;
constexpr int LN_ROWS_PER_BLOCK_GROUPED = 32;

// 4-element vector loads/stores (8 B for 16-bit types, 16 B for f32); rows are 4-aligned
template <typename T> struct V4;
template <> struct V4<float> {
  static __device__ __forceinline__ void ld(const float* p, float (&v)[4]) {
    const float4 t = *(const float4*)p;
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&v)[4]) {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <typename H> struct V4h {
  static __device__ __forceinline__ void ld(const H* p, float (&v)[4]) {
    const uint2 t = *(const uint2*)p;
    const H* h = (const H*)&t;
    v[0] = (float)h[0]; v[1] = (float)h[1]; v[2] = (float)h[2]; v[3] = (float)h[3];
  }
  static __device__ __forceinline__ void st(H* p, const float (&v)[4]) {
    H h[4] = {(H)v[0], (H)v[1], (H)v[2], (H)v[3]};
    *(uint2*)p = *(const uint2*)h;
  }
};
template <> struct V4<__bf16> : V4h<__bf16> {};
template <> struct V4<_Float16> : V4h<_Float16> {};

// 8 consecutive 16-bit values <-> one 16-B access, as two 4-element halves
template <typename H>
__device__ __forceinline__ void ld8(const H* p, float (&a)[4], float (&b)[4]) {
  const uint4 t = *(const uint4*)p;
  const H* h = (const H*)&t;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = (float)h[e];
    b[e] = (float)h[4 + e];
  }
}
template <typename H>
__device__ __forceinline__ void st8(H* p, const float (&a)[4], const float (&b)[4]) {
  H h[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (H)a[e];
    h[4 + e] = (H)b[e];
  }
  *(uint4*)p = *(const uint4*)h;
}

template <typename TX, typename TY, int NV>
__global__ __launch_bounds__(RB) void l2norm_fwd_vec_kernel(int64_t rows, const TX* x,
                                                            int64_t ldx, TY* y, int64_t ldy,
                                                            float* inv_norm, float eps) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float v[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) V4<TX>::ld(x + r * ldx + 4 * (lane + 64 * j), v[j]);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[j][e] * v[j][e];
  s = wave_sum(s);
  const float inv = 1.f / fmaxf(sqrtf(s), eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = v[j][e] * inv;
    V4<TY>::st(y + r * ldy + 4 * (lane + 64 * j), o);
  }
  if (lane == 0) inv_norm[r] = inv;
}

// single-pass backward (D = 256 NV, 4-element aligned rows): x and dy are read once, 8-B / 16-B
// per lane, and kept in registers between the row dot product and the write (the loop form above
// reads both twice with 2-B lane loads)
template <typename TX, typename TG, typename TD, int NV>
__global__ __launch_bounds__(RB) void l2norm_bwd_vec_kernel(int64_t rows, const TX* x,
                                                            int64_t ldx, const TG* dy,
                                                            int64_t lddy, const float* inv_norm,
                                                            float eps, TD* dx, int64_t lddx) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float inv = inv_norm[r];
  const bool clamped = !(inv < 1.f / eps);
  float xv[NV][4], gv[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    V4<TX>::ld(x + r * ldx + 4 * (lane + 64 * j), xv[j]);
    V4<TG>::ld(dy + r * lddy + 4 * (lane + 64 * j), gv[j]);
  }
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) dot += xv[j][e] * inv * gv[j][e];
  dot = wave_sum(dot);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = clamped ? gv[j][e] * inv : (gv[j][e] - xv[j][e] * inv * dot) * inv;
    V4<TD>::st(dx + r * lddx + 4 * (lane + 64 * j), o);
  }
}

// Grouped LayerNorm (round 3): G same-shaped LayerNorms (the grouped encoders' LN1 / LN2, one per
// stream, jmt/grouped.py) in one launch, group g = blockIdx.y: its rows at x + g*sx (residual
// r + g*sr, output / input gradient + g*sy, dy + g*sdy), statistics at mean / rstd + g*rows,
// parameters from the tables.  gridDim.y == 1 is the plain form.
struct LnGrp {
  int64_t sx, sr, sy, sdy;
  const float* gamma[8];
  const float* beta[8];
};

// Vector forward (D = 256 NV, 4-aligned rows): lane owns elements 4*(lane + 64 j) .. +3; each
// wave normalises LNF_RPW rows, issuing all of a row's x / residual loads before its reductions.
constexpr int LNF_RPW = 4;
template <typename TI, typename TO, int NV>
__global__ __launch_bounds__(RB) void ln_fwd_vec_kernel(int64_t rows, const TI* x, int64_t ldx,
                                                        const TI* rr, int64_t ldr,
                                                        const float* gamma, const float* beta,
                                                        float eps, TO* y, int64_t ldy,
                                                        float* mean, float* rstd,
                                                        LnGrp grp = LnGrp{}) {
  constexpr int D = NV * 256;
  JMT_DCHECK(ldx >= D && ldy >= D && (!rr || ldr >= D));
  if (gridDim.y > 1) {
    const int gi = blockIdx.y;
    x += gi * grp.sx;
    if (rr) rr += gi * grp.sr;
    y += gi * grp.sy;
    mean += gi * rows;
    rstd += gi * rows;
    gamma = grp.gamma[gi];
    beta = grp.beta[gi];
  }
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * LNF_RPW;
  float gm[NV][4], bt[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    V4<float>::ld(gamma + 4 * (lane + 64 * j), gm[j]);
    V4<float>::ld(beta + 4 * (lane + 64 * j), bt[j]);
  }
  for (int i = 0; i < LNF_RPW; ++i) {
    const int64_t r = r0 + i;
    if (r >= rows) return;
    float v[NV][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) V4<TI>::ld(x + r * ldx + 4 * (lane + 64 * j), v[j]);
    if (rr) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        float t[4];
        V4<TI>::ld(rr + r * ldr + 4 * (lane + 64 * j), t);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] += t[e];
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += v[j][e];
    const float mu = wave_sum(s) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mu;
        q += d * d;
      }
    const float rs = rsqrtf(wave_sum(q) * (1.f / D) + eps);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mu) * rs * gm[j][e] + bt[j][e];
      V4<TO>::st(y + r * ldy + 4 * (lane + 64 * j), o);
    }
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
}

// NV = D / 256: lane owns elements 4*(lane + 64 j) .. +3, j < NV.  C8 (D = 512, 16-bit x / r /
// dy / dx with 16-B aligned rows): lane owns the 8 consecutive elements 8 lane .. +7 instead, one
// 16-B access per row and operand (half the load / store instructions of the 8-B form)
template <typename TI, typename TG, typename TD, int NV, bool DS = false,
          int RPB = LN_ROWS_PER_BLOCK, int U = 1, bool C8 = false>
__global__ __launch_bounds__(RB) void ln_bwd_vec_kernel(int64_t rows, const TI* x, int64_t ldx,
                                                        const TI* rr, int64_t ldr, const TG* dy,
                                                        int64_t lddy, const float* mean,
                                                        const float* rstd, const float* gamma,
                                                        TD* dx, int64_t lddx, float* partials,
                                                        LnGrp grp = LnGrp{}) {
  constexpr int D = NV * 256;
  constexpr int NS = DS ? 3 : 2;                 // slabs: dgamma, dbeta (+ column sums of dx)
  __shared__ float red[4][NS][D];
  if (gridDim.y > 1) {
    const int gi = blockIdx.y;
    x += gi * grp.sx;
    if (rr) rr += gi * grp.sr;
    dy += gi * grp.sdy;
    dx += gi * grp.sy;
    mean += gi * rows;
    rstd += gi * rows;
    gamma = grp.gamma[gi];
    partials += (int64_t)gi * gridDim.x * NS * D;
  }
  static_assert(!C8 || (NV == 2 && sizeof(TI) == 2 && sizeof(TG) == 2 && sizeof(TD) == 2),
                "C8: D = 512, 16-bit operands");
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  // first element of the lane's j-th group of 4
  auto col = [&](int j) { return C8 ? 8 * lane + 4 * j : 4 * (lane + 64 * j); };
  float pg[NV][4], pb[NV][4], gm[NV][4], ps[NV][4];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float4 g4 = *(const float4*)(gamma + col(j));
    gm[j][0] = g4.x; gm[j][1] = g4.y; gm[j][2] = g4.z; gm[j][3] = g4.w;
#pragma unroll
    for (int e = 0; e < 4; ++e) pg[j][e] = pb[j][e] = ps[j][e] = 0.f;
  }
  const int64_t rbeg = (int64_t)blockIdx.x * RPB;
  // U rows per wave per iteration, all their loads issued before any is reduced (rows past the
  // end are clamped for the loads and skipped for the math: wave-uniform).  U = 2 for the
  // grouped launch (53.6 vs 57.6 us at G = 3); one group alone keeps U = 1 (2 measured 24 -> 28)
  for (int i0 = w; i0 < RPB; i0 += 4 * U) {
    float xv[U][NV][4], gv[U][NV][4], mu[U], rs[U];
    int64_t rw[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = rbeg + i0 + 4 * u;
      ok[u] = r < rows;
      const int64_t rc = ok[u] ? r : rows - 1;
      rw[u] = rc;
      mu[u] = mean[rc];
      rs[u] = rstd[rc];
      if constexpr (C8) {
        const int c = 8 * lane;
        ld8(x + rc * ldx + c, xv[u][0], xv[u][1]);
        if (rr) {
          float r0[4], r1[4];
          ld8(rr + rc * ldr + c, r0, r1);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            xv[u][0][e] += r0[e];
            xv[u][1][e] += r1[e];
          }
        }
        ld8(dy + rc * lddy + c, gv[u][0], gv[u][1]);
        continue;
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c = 4 * (lane + 64 * j);
        V4<TI>::ld(x + rc * ldx + c, xv[u][j]);
        if (rr) {
          float rv[4];
          V4<TI>::ld(rr + rc * ldr + c, rv);
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[u][j][e] += rv[e];
        }
        V4<TG>::ld(dy + rc * lddy + c, gv[u][j]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const int64_t r = rw[u];
      float xh[NV][4], gd[NV][4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[j][e] = (xv[u][j][e] - mu[u]) * rs[u];
          pg[j][e] += gv[u][j][e] * xh[j][e];
          pb[j][e] += gv[u][j][e];
          gd[j][e] = gv[u][j][e] * gm[j][e];
          s1 += gd[j][e];
          s2 += gd[j][e] * xh[j][e];
        }
      }
      s1 = wave_sum(s1) * (1.f / D);
      s2 = wave_sum(s2) * (1.f / D);
      float o[NV][4];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[j][e] = rs[u] * (gd[j][e] - s1 - xh[j][e] * s2);
        if constexpr (!C8) V4<TD>::st(dx + r * lddx + 4 * (lane + 64 * j), o[j]);
        if constexpr (DS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) ps[j][e] += o[j][e];
        }
      }
      if constexpr (C8) st8(dx + r * lddx + 8 * lane, o[0], o[1]);
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[w][0][col(j) + e] = pg[j][e];
      red[w][1][col(j) + e] = pb[j][e];
      if constexpr (DS) red[w][2][col(j) + e] = ps[j][e];
    }
  __syncthreads();
  float* out = partials + (int64_t)blockIdx.x * NS * D;
  for (int c = threadIdx.x; c < NS * D; c += RB) {
    const int h = c / D, cc = c - h * D;
    out[c] = red[0][h][cc] + red[1][h][cc] + red[2][h][cc] + red[3][h][cc];
  }
}

// generic fallback (any D <= 2048): one element per lane-stride
template <typename TI, typename TG, typename TD>
__global__ __launch_bounds__(RB) void ln_bwd_kernel(int64_t rows, int D, const TI* x, int64_t ldx,
                                                    const TI* rr, int64_t ldr, const TG* dy,
                                                    int64_t lddy, const float* mean,
                                                    const float* rstd, const float* gamma, TD* dx,
                                                    int64_t lddx, float* partials) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  __shared__ float red[4][64];
  const int64_t rbeg = (int64_t)blockIdx.x * LN_ROWS_PER_BLOCK;
  for (int i = w; i < LN_ROWS_PER_BLOCK; i += 4) {
    const int64_t r = rbeg + i;
    if (r >= rows) break;
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
    for (int c = lane; c < D; c += 64) {
      float t = to_f(x[r * ldx + c]);
      if (rr) t += to_f(rr[r * ldr + c]);
      const float xh = (t - mu) * rs;
      const float gd = to_f(dy[r * lddy + c]) * gamma[c];
      s1 += gd;
      s2 += gd * xh;
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
    for (int c = lane; c < D; c += 64) {
      float t = to_f(x[r * ldx + c]);
      if (rr) t += to_f(rr[r * ldr + c]);
      const float xh = (t - mu) * rs;
      const float gd = to_f(dy[r * lddy + c]) * gamma[c];
      dx[r * lddx + c] = from_f<TD>(rs * (gd - s1 - xh * s2));
    }
  }
  // column partials: each wave sums its columns over the block's rows
  float* out = partials + (int64_t)blockIdx.x * 2 * D;
  for (int c0 = 0; c0 < D; c0 += 64) {
    const int c = c0 + lane;
    float pg = 0.f, pb = 0.f;
    if (c < D) {
      for (int i = w; i < LN_ROWS_PER_BLOCK; i += 4) {
        const int64_t r = rbeg + i;
        if (r >= rows) break;
        float t = to_f(x[r * ldx + c]);
        if (rr) t += to_f(rr[r * ldr + c]);
        const float g = to_f(dy[r * lddy + c]);
        pg += g * (t - mean[r]) * rstd[r];
        pb += g;
      }
    }
    red[w][lane] = pg;
    __syncthreads();
    if (w == 0 && c < D) out[c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    __syncthreads();
    red[w][lane] = pb;
    __syncthreads();
    if (w == 0 && c < D) out[D + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    __syncthreads();
  }
}

// sum partial slabs: for c < W, v = sum_b partials[b*stride + c];  c < split -> out0[c],
// else out1[c - split]  ((+)= with beta_acc).  Block = 4 column quads (16 columns) x 64 slab
// groups: each thread streams ~nblk/64 float4 loads with 4 independent accumulators, then a
// fixed-order two-level LDS reduction (deterministic).  W % 4 == 0, stride % 4 == 0.
constexpr int SR_G = 64;
struct OutTab { float* p[8]; };
__global__ __launch_bounds__(RB) void slab_reduce_kernel(int nblk, int W, const float* partials,
                                                         int64_t stride, int split, float* out0,
                                                         float* out1, int beta_acc,
                                                         OutTab tab = OutTab{}, int grouped = 0,
                                                         float* out2 = nullptr,
                                                         OutTab tab1 = OutTab{},
                                                         OutTab tab2 = OutTab{}) {
  if (grouped) {   // group g = blockIdx.y: slabs at partials + g*nblk*stride, output tab.p[g]
    partials += (int64_t)blockIdx.y * nblk * stride;
    out0 = out1 = tab.p[blockIdx.y];
    if (grouped == 2) {   // grouped LayerNorm: dgamma / dbeta / (dsum) tables
      out1 = tab1.p[blockIdx.y];
      out2 = tab2.p[blockIdx.y];
    }
  }
  __shared__ float4 red[SR_G][4];
  __shared__ float4 red2[16][4];
  const int q = threadIdx.x & 3, g = threadIdx.x >> 2;
  const int c = blockIdx.x * 16 + 4 * q;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  if (c < W) {
    const float* base = partials + c;
    int b = g;
    for (; b + 3 * SR_G < nblk; b += 4 * SR_G) {
      const float4 v0 = *(const float4*)(base + (int64_t)b * stride);
      const float4 v1 = *(const float4*)(base + (int64_t)(b + SR_G) * stride);
      const float4 v2 = *(const float4*)(base + (int64_t)(b + 2 * SR_G) * stride);
      const float4 v3 = *(const float4*)(base + (int64_t)(b + 3 * SR_G) * stride);
      a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
      a1.x += v1.x; a1.y += v1.y; a1.z += v1.z; a1.w += v1.w;
      a2.x += v2.x; a2.y += v2.y; a2.z += v2.z; a2.w += v2.w;
      a3.x += v3.x; a3.y += v3.y; a3.z += v3.z; a3.w += v3.w;
    }
    for (; b < nblk; b += SR_G) {
      const float4 v0 = *(const float4*)(base + (int64_t)b * stride);
      a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
    }
  }
  red[g][q] = make_float4(a0.x + a1.x + a2.x + a3.x, a0.y + a1.y + a2.y + a3.y,
                          a0.z + a1.z + a2.z + a3.z, a0.w + a1.w + a2.w + a3.w);
  __syncthreads();
  if (threadIdx.x < 64) {   // 16 partial groups x 4 quads: each sums 4 of the 64 slab groups
    const int qq = threadIdx.x & 3, gg = threadIdx.x >> 2;
    float4 t = red[4 * gg][qq];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const float4 u = red[4 * gg + i][qq];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    red2[gg][qq] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4 && blockIdx.x * 16 + 4 * threadIdx.x < W) {
    float4 t = red2[0][threadIdx.x];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      const float4 u = red2[i][threadIdx.x];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const int cc = blockIdx.x * 16 + 4 * threadIdx.x;
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = cc + e;
      float* o = col < split ? out0 + col
                 : (out2 && col >= 2 * split) ? out2 + (col - 2 * split) : out1 + (col - split);
      *o = beta_acc ? *o + tv[e] : tv[e];
    }
  }
}

// scalar fallback (W or stride not a multiple of 4)
__global__ __launch_bounds__(RB) void slab_reduce_scalar_kernel(int nblk, int W,
                                                                const float* partials,
                                                                int64_t stride, int split,
                                                                float* out0, float* out1,
                                                                int beta_acc) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f;
  if (c < W)
    for (int b = g; b < nblk; b += 4) s0 += partials[(int64_t)b * stride + c];
  red[g][lane] = s0;
  __syncthreads();
  if (g == 0 && c < W) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    float* o = c < split ? out0 + c : out1 + (c - split);
    *o = beta_acc ? *o + t : t;
  }
}

static void launch_slab_reduce(int nblk, int W, const float* partials, int64_t stride, int split,
                               float* out0, float* out1, int beta_acc, hipStream_t st) {
  if (W % 4 == 0 && stride % 4 == 0 && ((uintptr_t)partials & 15) == 0)
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((W + 15) / 16), dim3(RB), 0, st, nblk, W,
                       partials, stride, split, out0, out1, beta_acc);
  else
    hipLaunchKernelGGL(slab_reduce_scalar_kernel, dim3((W + 63) / 64), dim3(RB), 0, st, nblk, W,
                       partials, stride, split, out0, out1, beta_acc);
}

// ------------------------------------------------------------------ softmax
template <typename TP>
__global__ __launch_bounds__(RB) void softmax_fwd_kernel(int64_t rows, int n, const float* s,
                                                         int64_t lds, float scale, TP* p,
                                                         int64_t ldp) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* sr = s + r * lds;
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, sr[c] * scale);
  m = wave_max(m);
  float z = 0.f;
  for (int c = lane; c < n; c += 64) z += __expf(sr[c] * scale - m);
  z = wave_sum(z);
  const float iz = 1.f / z;
  TP* pr = p + r * ldp;
  for (int c = lane; c < ldp; c += 64)
    pr[c] = from_f<TP>(c < n ? __expf(sr[c] * scale - m) * iz : 0.f);
}

template <typename TP, typename TS>
__global__ __launch_bounds__(RB) void softmax_bwd_kernel(int64_t rows, int n, const TP* p,
                                                         int64_t ldp, const float* dp,
                                                         int64_t lddp, float scale, TS* ds,
                                                         int64_t ldds) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const TP* pr = p + r * ldp;
  const float* gr = dp + r * lddp;
  float dot = 0.f;
  for (int c = lane; c < n; c += 64) dot += to_f(pr[c]) * gr[c];
  dot = wave_sum(dot);
  TS* dr = ds + r * ldds;
  for (int c = lane; c < ldds; c += 64)
    dr[c] = from_f<TS>(c < n ? scale * to_f(pr[c]) * (gr[c] - dot) : 0.f);
}

// ------------------------------------------------------------------ column sums (bias grad)
constexpr int CS_ROWS = 256;

// 16-B aligned rows: block = 8 column chunks of VE = 16/sizeof(T) elements (8*VE columns) x 32
// row lanes over CS_ROWS rows; each thread issues CS_ROWS/32 independent 16-B loads.
template <typename T>
__global__ __launch_bounds__(RB) void colsum_vec_kernel(int64_t rows, int N, const T* dy,
                                                        int64_t ld, float* partials,
                                                        int64_t sdy = 0) {
  dy += (int64_t)blockIdx.z * sdy;                              // group g = blockIdx.z
  partials += (int64_t)blockIdx.z * gridDim.x * N;
  constexpr int VE = 16 / sizeof(T);
  constexpr int NC = 8 * VE;                // columns per block
  __shared__ float red[32][NC + 1];
  const int q = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.y * NC + q * VE;
  const int64_t r0 = (int64_t)blockIdx.x * CS_ROWS;
  float acc[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) acc[e] = 0.f;
  if (c < N) {
#pragma unroll
    for (int i = 0; i < CS_ROWS / 32; ++i) {
      const int64_t r = r0 + rl + 32 * i;
      if (r < rows) {
        const uint4 u = *(const uint4*)(dy + r * ld + c);
        const T* v = (const T*)&u;
#pragma unroll
        for (int e = 0; e < VE; ++e) acc[e] += to_f(v[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VE; ++e) red[rl][q * VE + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < NC) {
    const int cc = blockIdx.y * NC + threadIdx.x;
    float s = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) s += red[i][threadIdx.x];
    if (cc < N) partials[(int64_t)blockIdx.x * N + cc] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(RB) void colsum_kernel(int64_t rows, int N, const T* dy, int64_t ld,
                                                    float* partials) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= N) return;
  const int64_t r0 = (int64_t)blockIdx.x * CS_ROWS;
  const int64_t r1 = min(rows, r0 + CS_ROWS);
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += to_f(dy[r * ld + c]);
  partials[(int64_t)blockIdx.x * N + c] = s;
}

// Narrow column sums (N <= 64, e.g. the 1-wide regressor output bias): NP = N rounded up to a
// power of two columns x RB/NP row lanes per block, fixed-order LDS tree over the row lanes.
template <typename T>
__global__ __launch_bounds__(RB) void colsum_small_kernel(int64_t rows, int N, int NP,
                                                          const T* dy, int64_t ld,
                                                          float* partials) {
  __shared__ float red[RB];
  const int c = threadIdx.x % NP, ro = threadIdx.x / NP, rs = RB / NP;
  const int64_t r0 = (int64_t)blockIdx.x * CS_ROWS;
  const int64_t r1 = min(rows, r0 + CS_ROWS);
  float s = 0.f;
  if (c < N)
    for (int64_t r = r0 + ro; r < r1; r += rs) s += to_f(dy[r * ld + c]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = rs / 2; h > 0; h >>= 1) {
    if (ro < h) red[threadIdx.x] += red[threadIdx.x + h * NP];
    __syncthreads();
  }
  if (ro == 0 && c < N) partials[(int64_t)blockIdx.x * N + c] = red[threadIdx.x];
}

// ------------------------------------------------------------------ strided copy
// Row-contiguous copy / cast (both column strides 1, cols % 8 == 0, 16-B aligned rows when the
// element is 16-bit; 8 elements per thread per step: 16-B loads of 16-bit, 2x16-B of f32).
template <typename TS, typename TD>
__global__ __launch_bounds__(RB) void copy_rows_vec_kernel(int64_t rows, int64_t cols,
                                                           const TS* src, int64_t srs, TD* dst,
                                                           int64_t drs) {
  const int64_t c8 = cols / 8;
  const int64_t total = rows * c8;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / c8, c = (e - r * c8) * 8;
    const TS* sp = src + r * srs + c;
    TD* dp = dst + r * drs + c;
    float v[8];
    if constexpr (sizeof(TS) == 4) {
      const float4 a = *(const float4*)sp, b = *(const float4*)(sp + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 u = *(const uint4*)sp;
      const TS* h = (const TS*)&u;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = to_f(h[i]);
    }
    if constexpr (sizeof(TD) == 4) {
      *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(dp + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      TD h[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) h[i] = from_f<TD>(v[i]);
      *(uint4*)dp = *(const uint4*)h;
    }
  }
}

__global__ __launch_bounds__(RB) void copy2d_kernel(int sdt, int ddt, int64_t rows, int64_t cols,
                                                    const void* src, int64_t srs, int64_t scs,
                                                    void* dst, int64_t drs, int64_t dcs, int acc) {
  const int64_t total = rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols, c = e - r * cols;
    float v = ld_dyn(src, r * srs + c * scs, sdt);
    const int64_t o = r * drs + c * dcs;
    if (acc) v += ld_dyn(dst, o, ddt);
    st_dyn(dst, o, ddt, v);
  }
}

static inline unsigned row_blocks(int64_t rows) { return (unsigned)((rows + 3) / 4); }

}  // namespace jmt

using namespace jmt;

// dtype dispatch helpers --------------------------------------------------------------------
#define JMT_DISPATCH1(dt, T, ...)                        \
  switch (dt) {                                          \
    case JMT_F32: { typedef float T; __VA_ARGS__; } break;     \
    case JMT_BF16: { typedef __bf16 T; __VA_ARGS__; } break;   \
    case JMT_F16: { typedef _Float16 T; __VA_ARGS__; } break;  \
    default: return set_error(JMT_ERR_ARG, "bad dtype %d", (int)dt); \
  }

extern "C" int jmt_l2norm_fwd(int x_dt, int y_dt, int64_t rows, int D, const void* x, int64_t ldx,
                              void* y, int64_t ldy, float* inv_norm, float eps, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(D > 0 && x && y && inv_norm, "jmt_l2norm_fwd: bad args");
  hipStream_t st = as_stream(stream);
  const bool vec = (D == 512 || D == 1024 || D == 2048) && ldx % 4 == 0 && ldy % 4 == 0 &&
                   ((uintptr_t)x % (4 * dtype_size(x_dt))) == 0 &&
                   ((uintptr_t)y % (4 * dtype_size(y_dt))) == 0;
#define JMT_L2V(NV)                                                                          \
  hipLaunchKernelGGL((l2norm_fwd_vec_kernel<TX, TY, NV>), dim3(row_blocks(rows)), dim3(RB), 0, \
                     st, rows, (const TX*)x, ldx, (TY*)y, ldy, inv_norm, eps)
  JMT_DISPATCH1(x_dt, TX, JMT_DISPATCH1(y_dt, TY,
      if (vec && D == 512) { JMT_L2V(2); }
      else if (vec && D == 1024) { JMT_L2V(4); }
      else if (vec && D == 2048) { JMT_L2V(8); }
      else {
        hipLaunchKernelGGL((l2norm_fwd_kernel<TX, TY>), dim3(row_blocks(rows)), dim3(RB), 0, st,
                           rows, D, (const TX*)x, ldx, (TY*)y, ldy, inv_norm, eps);
      }));
#undef JMT_L2V
  JMT_LAUNCH_CHECK("jmt_l2norm_fwd");
  return JMT_OK;
}

extern "C" int jmt_l2norm_bwd(int x_dt, int dy_dt, int dx_dt, int64_t rows, int D, const void* x,
                              int64_t ldx, const void* dy, int64_t lddy, const float* inv_norm,
                              float eps, void* dx, int64_t lddx, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(D > 0 && x && dy && dx && inv_norm, "jmt_l2norm_bwd: bad args");
  hipStream_t st = as_stream(stream);
  const bool vec = (D == 512 || D == 1024 || D == 2048) && ldx % 4 == 0 && lddy % 4 == 0 &&
                   lddx % 4 == 0 && ((uintptr_t)x % (4 * dtype_size(x_dt))) == 0 &&
                   ((uintptr_t)dy % (4 * dtype_size(dy_dt))) == 0 &&
                   ((uintptr_t)dx % (4 * dtype_size(dx_dt))) == 0;
#define JMT_L2BV(NV)                                                                          \
  hipLaunchKernelGGL((l2norm_bwd_vec_kernel<TX, TG, TD, NV>), dim3(row_blocks(rows)), dim3(RB), \
                     0, st, rows, (const TX*)x, ldx, (const TG*)dy, lddy, inv_norm, eps,       \
                     (TD*)dx, lddx)
  JMT_DISPATCH1(x_dt, TX, JMT_DISPATCH1(dy_dt, TG, JMT_DISPATCH1(dx_dt, TD,
      if (vec && D == 512) { JMT_L2BV(2); }
      else if (vec && D == 1024) { JMT_L2BV(4); }
      else if (vec && D == 2048) { JMT_L2BV(8); }
      else {
        hipLaunchKernelGGL((l2norm_bwd_kernel<TX, TG, TD>), dim3(row_blocks(rows)), dim3(RB), 0,
                           st, rows, D, (const TX*)x, ldx, (const TG*)dy, lddy, inv_norm, eps,
                           (TD*)dx, lddx);
      })));
#undef JMT_L2BV
  JMT_LAUNCH_CHECK("jmt_l2norm_bwd");
  return JMT_OK;
}

extern "C" int jmt_layernorm_fwd(int dt_in, int dt_out, int64_t rows, int D, const void* x,
                                 int64_t ldx, const void* r, int64_t ldr, const float* gamma,
                                 const float* beta, float eps, void* y, int64_t ldy, float* mean,
                                 float* rstd, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(D > 0 && D <= 2048, "jmt_layernorm_fwd: D=%d unsupported (<=2048)", D);
  JMT_CHECK_ARG(x && y && gamma && beta && mean && rstd, "jmt_layernorm_fwd: null pointer");
  hipStream_t st = as_stream(stream);
  const uintptr_t ai = 4 * dtype_size(dt_in), ao = 4 * dtype_size(dt_out);
  const bool vec = (D % 256 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) && (!r || ldr % 4 == 0) &&
                   ((uintptr_t)gamma % 16 == 0) && ((uintptr_t)beta % 16 == 0) &&
                   ((uintptr_t)x % ai == 0) && ((uintptr_t)r % ai == 0) && ((uintptr_t)y % ao == 0);
  const unsigned vblocks = (unsigned)((rows + 4 * LNF_RPW - 1) / (4 * LNF_RPW));
#define JMT_LNF_VEC(NV)                                                                     \
  hipLaunchKernelGGL((ln_fwd_vec_kernel<TI, TO, NV>), dim3(vblocks), dim3(RB), 0, st, rows, \
                     (const TI*)x, ldx, (const TI*)r, ldr, gamma, beta, eps, (TO*)y, ldy, mean, \
                     rstd)
  JMT_DISPATCH1(dt_in, TI, JMT_DISPATCH1(dt_out, TO,
      if (vec && D == 512) { JMT_LNF_VEC(2); }
      else if (vec && D == 768) { JMT_LNF_VEC(3); }
      else if (vec && D == 1024) { JMT_LNF_VEC(4); }
      else {
        hipLaunchKernelGGL((ln_fwd_kernel<TI, TO>), dim3(row_blocks(rows)), dim3(RB), 0, st, rows,
                           D, (const TI*)x, ldx, (const TI*)r, ldr, gamma, beta, eps, (TO*)y, ldy,
                           mean, rstd);
      }));
#undef JMT_LNF_VEC
  JMT_LAUNCH_CHECK("jmt_layernorm_fwd");
  return JMT_OK;
}

extern "C" int jmt_layernorm_bwd_blocks(int64_t rows) {
  return (int)((rows + LN_ROWS_PER_BLOCK - 1) / LN_ROWS_PER_BLOCK);
}

extern "C" int jmt_layernorm_bwd_grouped_blocks(int64_t rows) {
  return (int)((rows + LN_ROWS_PER_BLOCK_GROUPED - 1) / LN_ROWS_PER_BLOCK_GROUPED);
}

// JMT_LN_C8=0: the LayerNorm backward keeps the 8-B element mapping (A/B switch)
static bool ln_c8_off() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JMT_LN_C8");
    v = e ? atoi(e) : 1;
  }
  return v == 0;
}

// the C8 form of ln_bwd_vec_kernel applies: D = 512, 16-bit x / r / dy / dx of one type, 16-B
// aligned bases, row (and group) strides multiples of 8 elements
static bool ln_c8_ok(int dt_in, int dt_dy, int dt_dx, int D, const void* x, int64_t ldx,
                     const void* r, int64_t ldr, const void* dy, int64_t lddy, const void* dx,
                     int64_t lddx, int64_t sx = 0, int64_t sr = 0, int64_t sdy = 0,
                     int64_t sdx = 0) {
  return D == 512 && dt_in != JMT_F32 && dt_in == dt_dy && dt_in == dt_dx && !ln_c8_off() &&
         ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0 &&
         ldx % 8 == 0 && lddy % 8 == 0 && lddx % 8 == 0 && sx % 8 == 0 && sdy % 8 == 0 &&
         sdx % 8 == 0 && (!r || (((uintptr_t)r & 15) == 0 && ldr % 8 == 0 && sr % 8 == 0));
}

extern "C" int jmt_layernorm_bwd(int dt_in, int dt_dy, int dt_dx, int64_t rows, int D,
                                 const void* x, int64_t ldx, const void* r, int64_t ldr,
                                 const void* dy, int64_t lddy, const float* mean,
                                 const float* rstd, const float* gamma, void* dx, int64_t lddx,
                                 float* dgamma, float* dbeta, int beta_acc, float* partials,
                                 void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(D > 0 && D <= 2048, "jmt_layernorm_bwd: D=%d unsupported (<=2048)", D);
  JMT_CHECK_ARG(x && dy && dx && mean && rstd && gamma && partials && dgamma && dbeta,
                "jmt_layernorm_bwd: null pointer");
  hipStream_t st = as_stream(stream);
  const int nblk = jmt_layernorm_bwd_blocks(rows);
  const bool vec = (D % 256 == 0) && (ldx % 4 == 0) && (lddy % 4 == 0) && (lddx % 4 == 0) &&
                   (!r || ldr % 4 == 0) && ((uintptr_t)gamma % 16 == 0) &&
                   ((uintptr_t)x % (4 * dtype_size(dt_in)) == 0) &&
                   ((uintptr_t)r % (4 * dtype_size(dt_in)) == 0) &&
                   ((uintptr_t)dy % (4 * dtype_size(dt_dy)) == 0) &&
                   ((uintptr_t)dx % (4 * dtype_size(dt_dx)) == 0);
#define JMT_LNB_VEC(NV)                                                                     \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, NV>), dim3(nblk), dim3(RB), 0, st, rows, \
                     (const TI*)x, ldx, (const TI*)r, ldr, (const TG*)dy, lddy, mean, rstd, \
                     gamma, (TD*)dx, lddx, partials)
  const bool c8 = vec && ln_c8_ok(dt_in, dt_dy, dt_dx, D, x, ldx, r, ldr, dy, lddy, dx, lddx);
  JMT_DISPATCH1(dt_in, TI, JMT_DISPATCH1(dt_dy, TG, JMT_DISPATCH1(dt_dx, TD,
      constexpr bool same = sizeof(TI) == 2 && std::is_same<TI, TG>::value &&
                            std::is_same<TI, TD>::value;
      if constexpr (same) {
        if (c8) {
          hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, 2, false, LN_ROWS_PER_BLOCK, 1, true>),
                             dim3(nblk), dim3(RB), 0, st, rows, (const TI*)x, ldx, (const TI*)r,
                             ldr, (const TG*)dy, lddy, mean, rstd, gamma, (TD*)dx, lddx, partials);
          break;
        }
      }
      if (vec && D == 512) { JMT_LNB_VEC(2); }
      else if (vec && D == 768) { JMT_LNB_VEC(3); }
      else if (vec && D == 1024) { JMT_LNB_VEC(4); }
      else {
        hipLaunchKernelGGL((ln_bwd_kernel<TI, TG, TD>), dim3(nblk), dim3(RB), 0, st, rows, D,
                           (const TI*)x, ldx, (const TI*)r, ldr, (const TG*)dy, lddy, mean, rstd,
                           gamma, (TD*)dx, lddx, partials);
      })));
#undef JMT_LNB_VEC
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd");
  launch_slab_reduce(nblk, 2 * D, partials, (int64_t)2 * D, D, dgamma, dbeta, beta_acc, st);
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd(reduce)");
  return JMT_OK;
}

extern "C" int jmt_layernorm_bwd_dsum(int dt_in, int dt_dy, int dt_dx, int64_t rows, int D,
                                      const void* x, int64_t ldx, const void* r, int64_t ldr,
                                      const void* dy, int64_t lddy, const float* mean,
                                      const float* rstd, const float* gamma, void* dx,
                                      int64_t lddx, float* dgamma, float* dbeta, float* dsum,
                                      int beta_acc, float* partials, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(x && dy && dx && mean && rstd && gamma && partials && dgamma && dbeta && dsum,
                "jmt_layernorm_bwd_dsum: null pointer");
  const bool vec = (D == 512 || D == 768 || D == 1024) && (ldx % 4 == 0) && (lddy % 4 == 0) &&
                   (lddx % 4 == 0) && (!r || ldr % 4 == 0) && ((uintptr_t)gamma % 16 == 0) &&
                   ((uintptr_t)x % (4 * dtype_size(dt_in)) == 0) &&
                   ((uintptr_t)r % (4 * dtype_size(dt_in)) == 0) &&
                   ((uintptr_t)dy % (4 * dtype_size(dt_dy)) == 0) &&
                   ((uintptr_t)dx % (4 * dtype_size(dt_dx)) == 0) &&
                   ((uintptr_t)partials % 16 == 0);
  if (!vec)
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_layernorm_bwd_dsum: D=%d / layout not covered", D);
  hipStream_t st = as_stream(stream);
  const int nblk = jmt_layernorm_bwd_blocks(rows);
#define JMT_LNB_DS(NV)                                                                          \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, NV, true>), dim3(nblk), dim3(RB), 0, st, rows, \
                     (const TI*)x, ldx, (const TI*)r, ldr, (const TG*)dy, lddy, mean, rstd,    \
                     gamma, (TD*)dx, lddx, partials)
  const bool c8 = ln_c8_ok(dt_in, dt_dy, dt_dx, D, x, ldx, r, ldr, dy, lddy, dx, lddx);
  JMT_DISPATCH1(dt_in, TI, JMT_DISPATCH1(dt_dy, TG, JMT_DISPATCH1(dt_dx, TD,
      constexpr bool same = sizeof(TI) == 2 && std::is_same<TI, TG>::value &&
                            std::is_same<TI, TD>::value;
      if constexpr (same) {
        if (c8) {
          hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, 2, true, LN_ROWS_PER_BLOCK, 1, true>),
                             dim3(nblk), dim3(RB), 0, st, rows, (const TI*)x, ldx, (const TI*)r,
                             ldr, (const TG*)dy, lddy, mean, rstd, gamma, (TD*)dx, lddx, partials);
          break;
        }
      }
      if (D == 512) { JMT_LNB_DS(2); }
      else if (D == 768) { JMT_LNB_DS(3); }
      else { JMT_LNB_DS(4); })));
#undef JMT_LNB_DS
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd_dsum");
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((3 * D + 15) / 16), dim3(RB), 0, st, nblk, 3 * D,
                     partials, (int64_t)3 * D, D, dgamma, dbeta, beta_acc, OutTab{}, 0, dsum);
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd_dsum(reduce)");
  return JMT_OK;
}

extern "C" int jmt_softmax_fwd(int p_dt, int64_t rows, int n, const float* s, int64_t lds,
                               float scale, void* p, int64_t ldp, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(n > 0 && ldp >= n && s && p, "jmt_softmax_fwd: bad args");
  hipStream_t st = as_stream(stream);
  JMT_DISPATCH1(p_dt, TP,
      hipLaunchKernelGGL((softmax_fwd_kernel<TP>), dim3(row_blocks(rows)), dim3(RB), 0, st, rows,
                         n, s, lds, scale, (TP*)p, ldp));
  JMT_LAUNCH_CHECK("jmt_softmax_fwd");
  return JMT_OK;
}

extern "C" int jmt_softmax_bwd(int p_dt, int ds_dt, int64_t rows, int n, const void* p,
                               int64_t ldp, const float* dp, int64_t lddp, float scale, void* ds,
                               int64_t ldds, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(n > 0 && ldds >= n && p && dp && ds, "jmt_softmax_bwd: bad args");
  hipStream_t st = as_stream(stream);
  JMT_DISPATCH1(p_dt, TP, JMT_DISPATCH1(ds_dt, TS,
      hipLaunchKernelGGL((softmax_bwd_kernel<TP, TS>), dim3(row_blocks(rows)), dim3(RB), 0, st,
                         rows, n, (const TP*)p, ldp, dp, lddp, scale, (TS*)ds, ldds)));
  JMT_LAUNCH_CHECK("jmt_softmax_bwd");
  return JMT_OK;
}

static int next_pow2(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

extern "C" int jmt_colsum_blocks(int64_t rows) { return (int)((rows + CS_ROWS - 1) / CS_ROWS); }

extern "C" int jmt_colsum(int dt, int64_t rows, int N, const void* dy, int64_t ld, float* db,
                          int beta_acc, float* partials, void* stream) {
  JMT_CHECK_ARG(N > 0 && db && partials, "jmt_colsum: bad args");
  hipStream_t st = as_stream(stream);
  const int nblk = jmt_colsum_blocks(rows);
  if (nblk == 0) {
    if (!beta_acc) (void)hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return JMT_OK;
  }
  const int ve = 16 / dtype_size(dt);
  const bool vec = (N % ve == 0) && (ld % ve == 0) && ((uintptr_t)dy % 16 == 0);
  JMT_DISPATCH1(dt, T,
      if (vec)
        hipLaunchKernelGGL((colsum_vec_kernel<T>), dim3(nblk, (N + 8 * ve - 1) / (8 * ve)),
                           dim3(RB), 0, st, rows, N, (const T*)dy, ld, partials);
      else if (N <= 64)
        hipLaunchKernelGGL((colsum_small_kernel<T>), dim3(nblk), dim3(RB), 0, st, rows, N,
                           next_pow2(N), (const T*)dy, ld, partials);
      else
        hipLaunchKernelGGL((colsum_kernel<T>), dim3(nblk, (N + RB - 1) / RB), dim3(RB), 0, st,
                           rows, N, (const T*)dy, ld, partials));
  launch_slab_reduce(nblk, N, partials, (int64_t)N, N, db, db, beta_acc, st);
  JMT_LAUNCH_CHECK("jmt_colsum");
  return JMT_OK;
}

extern "C" int jmt_colsum_grouped(int dt, int G, int64_t rows, int N, const void* dy, int64_t ld,
                                  int64_t sdy, float* const* db_tab, int beta_acc,
                                  float* partials, void* stream) {
  JMT_CHECK_ARG(G >= 1 && G <= 8 && N > 0 && db_tab && partials && dy,
                "jmt_colsum_grouped: bad args");
  const int ve = 16 / dtype_size(dt);
  JMT_CHECK_ARG((N % ve == 0) && (ld % ve == 0) && (sdy % ve == 0) && ((uintptr_t)dy % 16 == 0),
                "jmt_colsum_grouped: N, ld, sdy must be multiples of %d and dy 16-B aligned", ve);
  OutTab tab{};
  for (int g = 0; g < G; ++g) {
    JMT_CHECK_ARG(db_tab[g] != nullptr, "jmt_colsum_grouped: null output %d", g);
    tab.p[g] = db_tab[g];
  }
  hipStream_t st = as_stream(stream);
  const int nblk = jmt_colsum_blocks(rows);
  if (nblk == 0) {
    if (!beta_acc)
      for (int g = 0; g < G; ++g) (void)hipMemsetAsync(db_tab[g], 0, sizeof(float) * N, st);
    return JMT_OK;
  }
  JMT_DISPATCH1(dt, T,
      hipLaunchKernelGGL((colsum_vec_kernel<T>), dim3(nblk, (N + 8 * ve - 1) / (8 * ve), G),
                         dim3(RB), 0, st, rows, N, (const T*)dy, ld, partials, sdy));
  JMT_LAUNCH_CHECK("jmt_colsum_grouped");
  JMT_CHECK_ARG(N % 4 == 0, "jmt_colsum_grouped: N %% 4");
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((N + 15) / 16, G), dim3(RB), 0, st, nblk, N,
                     (const float*)partials, (int64_t)N, N, (float*)nullptr, (float*)nullptr,
                     beta_acc, tab, 1);
  JMT_LAUNCH_CHECK("jmt_colsum_grouped(reduce)");
  return JMT_OK;
}

extern "C" int jmt_copy2d(int src_dt, int dst_dt, int64_t rows, int64_t cols, const void* src,
                          int64_t src_rs, int64_t src_cs, void* dst, int64_t dst_rs,
                          int64_t dst_cs, int accumulate, void* stream) {
  if (rows == 0 || cols == 0) return JMT_OK;
  JMT_CHECK_ARG(src && dst, "jmt_copy2d: null pointer");
  JMT_CHECK_ARG(src_dt >= 0 && src_dt <= 2 && dst_dt >= 0 && dst_dt <= 2, "jmt_copy2d: dtype");
  const int64_t total = rows * cols;
  const bool vec = !accumulate && src_cs == 1 && dst_cs == 1 && cols % 8 == 0 &&
                   src_rs % 8 == 0 && dst_rs % 8 == 0 && ((uintptr_t)src % 16) == 0 &&
                   ((uintptr_t)dst % 16) == 0;
  if (vec) {
    int64_t vb = (total / 8 + RB - 1) / RB;
    const unsigned blocks = (unsigned)(vb > 16384 ? 16384 : (vb < 1 ? 1 : vb));
    JMT_DISPATCH1(src_dt, TS, JMT_DISPATCH1(dst_dt, TD,
        hipLaunchKernelGGL((copy_rows_vec_kernel<TS, TD>), dim3(blocks), dim3(RB), 0,
                           as_stream(stream), rows, cols, (const TS*)src, src_rs, (TD*)dst,
                           dst_rs)));
    JMT_LAUNCH_CHECK("jmt_copy2d(vec)");
    return JMT_OK;
  }
  int blocks = (int)((total + RB - 1) / RB);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(copy2d_kernel, dim3(blocks), dim3(RB), 0, as_stream(stream), src_dt, dst_dt,
                     rows, cols, src, src_rs, src_cs, dst, dst_rs, dst_cs, accumulate);
  JMT_LAUNCH_CHECK("jmt_copy2d");
  return JMT_OK;
}

// ------------------------------------------------------------------------------------ no-op
// One empty 64-thread block: the event-pair overhead probe of bench.py's per-launch timing
// (the time between two HIP events around a launch that does no work).
__global__ void noop_kernel() {}

extern "C" int jmt_noop(void* stream) {
  hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, as_stream(stream));
  JMT_LAUNCH_CHECK("jmt_noop");
  return JMT_OK;
}

// ------------------------------------------------------------------ grouped LayerNorm
// G (<= 8) same-shaped LayerNorms in one launch (+ one reduce launch in the backward): the
// grouped encoders' LN1 / LN2 (mm_multi_transformers.py:61-70 for each stream, jmt/grouped.py).
// Vector layouts only (D = 512 / 768 / 1024, 4-element-aligned rows); otherwise
// JMT_ERR_UNSUPPORTED and the caller runs the groups one by one.
static bool ln_grp_vec(int D, int64_t ld0, int64_t ld1, int64_t ld2, int64_t s0, int64_t s1,
                       int64_t s2, const void* p0, const void* p1, const void* p2) {
  return (D == 512 || D == 768 || D == 1024) && ld0 % 4 == 0 && ld1 % 4 == 0 && ld2 % 4 == 0 &&
         s0 % 4 == 0 && s1 % 4 == 0 && s2 % 4 == 0 && ((uintptr_t)p0 & 15) == 0 &&
         ((uintptr_t)p1 & 15) == 0 && ((uintptr_t)p2 & 15) == 0;
}

extern "C" int jmt_layernorm_fwd_grouped(int dt_in, int dt_out, int G, int64_t rows, int D,
                                         const void* x, int64_t ldx, int64_t sx, const void* r,
                                         int64_t ldr, int64_t sr, const float* const* gamma,
                                         const float* const* beta, float eps, void* y,
                                         int64_t ldy, int64_t sy, float* mean, float* rstd,
                                         void* stream) {
  if (rows == 0 || G == 0) return JMT_OK;
  JMT_CHECK_ARG(G >= 1 && G <= 8 && gamma && beta && x && y && mean && rstd,
                "jmt_layernorm_fwd_grouped: bad arguments");
  if (!ln_grp_vec(D, ldx, r ? ldr : 4, ldy, sx, r ? sr : 4, sy, x, r, y))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_layernorm_fwd_grouped: D=%d / layout", D);
  LnGrp grp = {};
  grp.sx = sx; grp.sr = sr; grp.sy = sy;
  for (int g = 0; g < G; ++g) {
    JMT_CHECK_ARG(gamma[g] && beta[g] && ((uintptr_t)gamma[g] & 15) == 0 &&
                      ((uintptr_t)beta[g] & 15) == 0, "jmt_layernorm_fwd_grouped: gamma/beta %d", g);
    grp.gamma[g] = gamma[g];
    grp.beta[g] = beta[g];
  }
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)((rows + 4 * LNF_RPW - 1) / (4 * LNF_RPW)), (unsigned)G);
#define JMT_LNFG(NV)                                                                            \
  hipLaunchKernelGGL((ln_fwd_vec_kernel<TI, TO, NV>), grid, dim3(RB), 0, st, rows, (const TI*)x, \
                     ldx, (const TI*)r, ldr, grp.gamma[0], grp.beta[0], eps, (TO*)y, ldy, mean,  \
                     rstd, grp)
  JMT_DISPATCH1(dt_in, TI, JMT_DISPATCH1(dt_out, TO,
      if (D == 512) { JMT_LNFG(2); }
      else if (D == 768) { JMT_LNFG(3); }
      else { JMT_LNFG(4); }));
#undef JMT_LNFG
  JMT_LAUNCH_CHECK("jmt_layernorm_fwd_grouped");
  return JMT_OK;
}

extern "C" int jmt_layernorm_bwd_grouped(int dt_in, int dt_dy, int dt_dx, int G, int64_t rows,
                                         int D, const void* x, int64_t ldx, int64_t sx,
                                         const void* r, int64_t ldr, int64_t sr, const void* dy,
                                         int64_t lddy, int64_t sdy, const float* mean,
                                         const float* rstd, const float* const* gamma, void* dx,
                                         int64_t lddx, int64_t sdx, float* const* dgamma,
                                         float* const* dbeta, float* const* dsum, int beta_acc,
                                         float* partials, void* stream) {
  if (rows == 0 || G == 0) return JMT_OK;
  JMT_CHECK_ARG(G >= 1 && G <= 8 && gamma && dgamma && dbeta && x && dy && dx && mean && rstd &&
                    partials && ((uintptr_t)partials & 15) == 0,
                "jmt_layernorm_bwd_grouped: bad arguments");
  if (!ln_grp_vec(D, ldx, lddy, lddx, sx, sdy, sdx, x, dy, dx) ||
      (r && (ldr % 4 != 0 || sr % 4 != 0 || ((uintptr_t)r & 15) != 0)))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_layernorm_bwd_grouped: D=%d / layout", D);
  LnGrp grp = {};
  grp.sx = sx; grp.sr = sr; grp.sy = sdx; grp.sdy = sdy;
  OutTab t0 = {}, t1 = {}, t2 = {};
  for (int g = 0; g < G; ++g) {
    JMT_CHECK_ARG(gamma[g] && ((uintptr_t)gamma[g] & 15) == 0 && dgamma[g] && dbeta[g] &&
                      (!dsum || dsum[g]), "jmt_layernorm_bwd_grouped: group %d pointers", g);
    grp.gamma[g] = gamma[g];
    t0.p[g] = dgamma[g];
    t1.p[g] = dbeta[g];
    t2.p[g] = dsum ? dsum[g] : nullptr;
  }
  hipStream_t st = as_stream(stream);
  const int nblk = jmt_layernorm_bwd_grouped_blocks(rows);
  const dim3 grid((unsigned)nblk, (unsigned)G);
  // (4 rows in flight per wave measured slower in isolation and equal in the step:
  // profiles/r03_ln_bwd_u_ab.jsonl; 2 is the only form compiled)
#define JMT_LNBG_U(NV, DS, U)                                                                    \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, NV, DS, LN_ROWS_PER_BLOCK_GROUPED, U>), grid, \
                     dim3(RB), 0, st, rows,                                                     \
                     (const TI*)x, ldx, (const TI*)r, ldr, (const TG*)dy, lddy, mean, rstd,     \
                     grp.gamma[0], (TD*)dx, lddx, partials, grp)
  // 16-B rows for the C8 form (D = 512): every base 16-B aligned, every stride a multiple of 8
  const bool c8 = ln_c8_ok(dt_in, dt_dy, dt_dx, D, x, ldx, r, ldr, dy, lddy, dx, lddx, sx, sr,
                           sdy, sdx);
#define JMT_LNBG_C8(DS)                                                                          \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<TI, TG, TD, 2, DS, LN_ROWS_PER_BLOCK_GROUPED, 2,         \
                                        true>), grid, dim3(RB), 0, st, rows, (const TI*)x, ldx,  \
                     (const TI*)r, ldr, (const TG*)dy, lddy, mean, rstd, grp.gamma[0], (TD*)dx,  \
                     lddx, partials, grp)
#define JMT_LNBG(NV, DS) JMT_LNBG_U(NV, DS, 2)
  JMT_DISPATCH1(dt_in, TI, JMT_DISPATCH1(dt_dy, TG, JMT_DISPATCH1(dt_dx, TD,
      constexpr bool same = sizeof(TI) == 2 && std::is_same<TI, TG>::value &&
                            std::is_same<TI, TD>::value;
      (void)same;
      if constexpr (same) {
        if (c8) {
          if (dsum) { JMT_LNBG_C8(true); } else { JMT_LNBG_C8(false); }
          break;
        }
      }
      if (dsum) {
        if (D == 512) { JMT_LNBG(2, true); }
        else if (D == 768) { JMT_LNBG(3, true); }
        else { JMT_LNBG(4, true); }
      } else {
        if (D == 512) { JMT_LNBG(2, false); }
        else if (D == 768) { JMT_LNBG(3, false); }
        else { JMT_LNBG(4, false); }
      })));
#undef JMT_LNBG_C8
#undef JMT_LNBG
#undef JMT_LNBG_U
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd_grouped");
  const int NS = dsum ? 3 : 2;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((NS * D + 15) / 16, G), dim3(RB), 0, st, nblk,
                     NS * D, partials, (int64_t)NS * D, D, (float*)nullptr, (float*)nullptr,
                     beta_acc, t0, 2, (float*)nullptr, t1, t2);
  JMT_LAUNCH_CHECK("jmt_layernorm_bwd_grouped(reduce)");
  return JMT_OK;
}
