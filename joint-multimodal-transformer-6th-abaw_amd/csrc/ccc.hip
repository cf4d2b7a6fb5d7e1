// Concordance-correlation-coefficient losses of the JMT path (losses/loss.py:8-32 and
// losses/CCCLoss.py:4-43), forward + analytic backward, with rank-local sufficient statistics
// that combine exactly across data-parallel ranks (Chan et al. pairwise update) so the loss stays
// a GLOBAL-batch statistic as it is under the reference's DataParallel gather.
//
// Statistics are accumulated in double (one 1024-thread block; n = B*T elements per rank, a few
// 10^4) — the kernel is latency-bound, never bandwidth-bound: one memory pass, register-cached.
#include "common.h"

namespace jmt {

constexpr int CT = 1024;
constexpr int MAXK = 64;   // digitize_num bins

// numpy.linspace(lo, hi, k)[c] in float64, then cast to float32 (loss.py:14-16)
__device__ __forceinline__ float bin_value(int c, int k, float lo, float hi) {
  if (k == 1) return lo;
  const double step = ((double)hi - (double)lo) / (double)(k - 1);
  double v = (double)lo + (double)c * step;
  if (c == k - 1) v = hi;
  return (float)v;
}

// prediction value of element i: the raw prediction (k == 1) or sum_c softmax(z_i)_c * bins_c
template <typename T>
__device__ __forceinline__ float pred_value(const T* pred, int64_t i, int k, float lo, float hi) {
  if (k == 1) return to_f(pred[i]);
  const T* z = pred + i * k;
  float m = -INFINITY;
  for (int c = 0; c < k; ++c) m = fmaxf(m, to_f(z[c]));
  float s = 0.f, e = 0.f;
  for (int c = 0; c < k; ++c) {
    const float p = __expf(to_f(z[c]) - m);
    s += p;
    e += p * bin_value(c, k, lo, hi);
  }
  return e / s;
}

// three block sums at once (one LDS round trip)
__device__ __forceinline__ void block_sum3_d(double& a, double& b, double& c, double* red) {
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  c = wave_sum_d(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[3 * w] = a;
    red[3 * w + 1] = b;
    red[3 * w + 2] = c;
  }
  __syncthreads();
  a = b = c = 0.0;
  for (int i = 0; i < CT / 64; ++i) {
    a += red[3 * i];
    b += red[3 * i + 1];
    c += red[3 * i + 2];
  }
  __syncthreads();
}

// Two-pass (mean, then centred sums) statistics.  A thread's first RC elements are kept in
// registers from pass 1 (all their loads issued together), so for n <= RC * CT (the JMT batches:
// B*T = 19,200) pass 2 reads no memory; beyond that the rest is re-read.
constexpr int RC = 24;
template <typename T>
__global__ __launch_bounds__(CT) void ccc_stats_kernel(int kind, int64_t n, int k, const T* pred,
                                                       const float* label, float ignore, float lo,
                                                       float hi, double* stats) {
  __shared__ double red[3 * (CT / 64)];
  float xs[RC], ys[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int64_t i = threadIdx.x + (int64_t)r * CT;
    const bool in = i < n;
    ys[r] = in ? label[i] : ignore;
    xs[r] = in ? pred_value(pred, i, k, lo, hi) : 0.f;
  }
  double c = 0, sx = 0, sy = 0;
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int64_t i = threadIdx.x + (int64_t)r * CT;
    if (i >= n || (kind == 1 && ys[r] == ignore)) continue;
    c += 1.0;
    sx += xs[r];
    sy += ys[r];
  }
  for (int64_t i = threadIdx.x + (int64_t)RC * CT; i < n; i += CT) {
    const float y = label[i];
    if (kind == 1 && y == ignore) continue;
    c += 1.0;
    sx += pred_value(pred, i, k, lo, hi);
    sy += y;
  }
  block_sum3_d(c, sx, sy, red);
  const double mx = c > 0 ? sx / c : 0.0, my = c > 0 ? sy / c : 0.0;
  double xx = 0, yy = 0, xy = 0;
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int64_t i = threadIdx.x + (int64_t)r * CT;
    if (i >= n || (kind == 1 && ys[r] == ignore)) continue;
    const double dx = (double)xs[r] - mx, dy = (double)ys[r] - my;
    xx += dx * dx;
    yy += dy * dy;
    xy += dx * dy;
  }
  for (int64_t i = threadIdx.x + (int64_t)RC * CT; i < n; i += CT) {
    const float y = label[i];
    if (kind == 1 && y == ignore) continue;
    const double dx = (double)pred_value(pred, i, k, lo, hi) - mx, dy = (double)y - my;
    xx += dx * dx;
    yy += dy * dy;
    xy += dx * dy;
  }
  block_sum3_d(xx, yy, xy, red);
  if (threadIdx.x == 0) {
    stats[0] = c; stats[1] = mx; stats[2] = my;
    stats[3] = xx; stats[4] = yy; stats[5] = xy;
    stats[6] = (double)n;                         // pre-mask element count (global bs, below)
    stats[7] = 0;
  }
}

// Combine rank statistics in fixed rank order, then loss + gradient coefficients.
//   coef = {c0, c1, c2, mean_x, mean_y, valid, 0, 0};  dL/dx_i = c0 + c1 (x_i - mx) + c2 (y_i - my)
// bs (kind 1, CCCLoss.py:17 `y_pred.size(0)` before masking): bs >= 1 is used as given (the
// (1, B*T) view of train.py:303-307: size(0) is 1 on every rank and after the gather); bs < 0
// means "1-D predictions": size(0) of the GATHERED batch = the sum of the ranks' pre-mask counts.
// `add` (may be NULL): the loss written is *add + this loss, rounded once as torch's fp32
// `l1 + l2` of train.py:311 (the two criteria of a step summed without a separate add kernel)
__global__ void ccc_finish_kernel(int kind, int world, const double* st, int64_t bs_in, float eps,
                                  const float* add, float* loss, double* coef) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  auto put = [&](float v) { *loss = add ? *add + v : v; };
  double n = st[0], mx = st[1], my = st[2], Sxx = st[3], Syy = st[4], Sxy = st[5];
  double bsd = (double)bs_in;
  if (bs_in < 0) {
    bsd = 0.0;
    for (int r = 0; r < world; ++r) bsd += st[8 * r + 6];
  }
  for (int r = 1; r < world; ++r) {
    const double* s = st + 8 * r;
    const double nb = s[0];
    if (nb <= 0) continue;
    if (n <= 0) { n = nb; mx = s[1]; my = s[2]; Sxx = s[3]; Syy = s[4]; Sxy = s[5]; continue; }
    const double nt = n + nb, dx = s[1] - mx, dy = s[2] - my, f = n * nb / nt;
    Sxx += s[3] + dx * dx * f;
    Syy += s[4] + dy * dy * f;
    Sxy += s[5] + dx * dy * f;
    mx += dx * nb / nt;
    my += dy * nb / nt;
    n = nt;
  }
  for (int i = 0; i < 8; ++i) coef[i] = 0.0;
  coef[3] = mx;
  coef[4] = my;
  if (kind == 0) {
    // losses/loss.py:23-32 in fp32 op order (rho with eps, unbiased std, no eps in the ccc)
    const float fn = (float)n;
    const float sxx = (float)Sxx, syy = (float)Syy, sxy = (float)Sxy;
    const float a = sqrtf(sxx), b = sqrtf(syy);
    const float q = a * b + eps;
    const float rho = sxy / q;
    const float xs = sqrtf(sxx / (fn - 1.f)), ys = sqrtf(syy / (fn - 1.f));
    const float dmean = (float)mx - (float)my;
    const float den = xs * xs + ys * ys + dmean * dmean;
    const float ccc = 2.f * rho * xs * ys / den;
    put(1.f - ccc);
    // analytic gradient in double
    const double nm1 = n - 1.0;
    const double A = sqrt(Sxx), Bv = sqrt(Syy), Q = A * Bv + (double)eps;
    const double num = 2.0 * Sxy * A * Bv / (nm1 * Q);
    const double D = (Sxx + Syy) / nm1 + (mx - my) * (mx - my);
    const double dnum_dSxy = 2.0 * A * Bv / (nm1 * Q);
    const double dnum_dSxx = A > 0 ? Sxy * Bv * (double)eps / (nm1 * Q * Q * A) : 0.0;
    const double dccc_dSxy = dnum_dSxy / D;
    const double dccc_dSxx = dnum_dSxx / D - num / (D * D) / nm1;
    const double dccc_dmx = -num / (D * D) * 2.0 * (mx - my);
    coef[0] = -dccc_dmx / n;
    coef[1] = -2.0 * dccc_dSxx;
    coef[2] = -dccc_dSxy;
    coef[5] = 1.0;
  } else {
    // losses/CCCLoss.py:24-43: masked compaction, <=1 element -> 0; std names swapped;
    // ccc = 2 s_xy / ((std(t)^2 + std(p)^2 + (mp - mt)^2 + 1e-8) * bs)
    if (n <= 1.0) {
      put(0.f);
      return;
    }
    const float fn = (float)n;
    const float x_std = sqrtf((float)Syy / (fn - 1.f));   // std(y_true)
    const float y_std = sqrtf((float)Sxx / (fn - 1.f));   // std(y_pred)
    const float dm = (float)mx - (float)my;
    const float den = x_std * x_std + y_std * y_std + dm * dm + 1e-8f;
    const float ccc = 2.f * (float)Sxy / (den * (float)bsd);
    put(1.f - ccc);
    const double nm1 = n - 1.0;
    const double D = Syy / nm1 + Sxx / nm1 + (mx - my) * (mx - my) + 1e-8;
    const double dccc_dSxy = 2.0 / (D * bsd);
    const double g = -2.0 * Sxy / (D * D * bsd);
    const double dccc_dSxx = g / nm1;
    const double dccc_dmx = g * 2.0 * (mx - my);
    coef[0] = -dccc_dmx / n;
    coef[1] = -2.0 * dccc_dSxx;
    coef[2] = -dccc_dSxy;
    coef[5] = 1.0;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ccc_bwd_kernel(int kind, int64_t n, int k, const T* pred,
                                                      const float* label, float ignore, float lo,
                                                      float hi, const double* coef,
                                                      const float* grad_loss, T* dpred) {
  const double c0 = coef[0], c1 = coef[1], c2 = coef[2], mx = coef[3], my = coef[4];
  const bool valid = coef[5] != 0.0;
  const float g = grad_loss ? *grad_loss : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float y = label[i];
    const bool masked = !valid || (kind == 1 && y == ignore);
    if (k == 1) {
      float d = 0.f;
      if (!masked) {
        const double x = to_f(pred[i]);
        d = (float)((c0 + c1 * (x - mx) + c2 * ((double)y - my)) * (double)g);
      }
      dpred[i] = from_f<T>(d);
    } else {
      const T* z = pred + i * k;
      T* dz = dpred + i * k;
      if (masked) {
        for (int c = 0; c < k; ++c) dz[c] = from_f<T>(0.f);
        continue;
      }
      float m = -INFINITY;
      for (int c = 0; c < k; ++c) m = fmaxf(m, to_f(z[c]));
      float s = 0.f, e = 0.f;
      float pv[MAXK];
      for (int c = 0; c < k; ++c) {
        pv[c] = __expf(to_f(z[c]) - m);
        s += pv[c];
        e += pv[c] * bin_value(c, k, lo, hi);
      }
      const float x = e / s;
      const float dx = (float)((c0 + c1 * ((double)x - mx) + c2 * ((double)y - my)) * (double)g);
      for (int c = 0; c < k; ++c) dz[c] = from_f<T>(dx * (pv[c] / s) * (bin_value(c, k, lo, hi) - x));
    }
  }
}

// ordered stream compaction of (label != ignore) with one block
__global__ __launch_bounds__(CT) void mask_indices_kernel(int64_t n, const float* label,
                                                          float ignore, int64_t* idx,
                                                          int64_t* count) {
  __shared__ int wsum[CT / 64];
  __shared__ int64_t base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t off = 0; off < n; off += CT) {
    const int64_t i = off + threadIdx.x;
    const bool keep = i < n && label[i] != ignore;
    const unsigned long long bal = __ballot(keep);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int wbase = 0;
    for (int j = 0; j < w; ++j) wbase += wsum[j];
    if (keep) idx[base + wbase + before] = i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int j = 0; j < CT / 64; ++j) t += wsum[j];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

// ---- CELoss (losses/loss.py:34-51): labels digitized on the device -----------------------------
// np.digitize(y, linspace(lo, hi, k + 1)) - 1 with the top bin clamped (loss.py:44-48): the bin
// is (number of edges <= y) - 1, edges in float64 as numpy builds them (i * step + lo, the last
// = hi); NaN -> k - 1 (numpy gives len(edges)).  A label below lo gives bin -1, on which the
// reference's F.cross_entropy raises: here it is counted (stats[2]), the loss is NaN and the
// host side raises on the count (jmt/functional.py _ce_label_check).
__device__ __forceinline__ int ce_bin(float yf, int k, float lo, float hi) {
  if (yf != yf) return k - 1;
  const double y = (double)yf, step = ((double)hi - (double)lo) / (double)k;
  int c = 0;
  for (int j = 0; j <= k; ++j) {
    const double e = j == k ? (double)hi : (double)j * step + (double)lo;
    c += e <= y;
  }
  c -= 1;
  return c == k ? k - 1 : c;
}

// one block: per row nll = logsumexp(x_i) - x_i[c_i], weight w[c_i] (1 without weights);
// stats = (sum w nll, sum w, invalid labels, 0) in double, rows in a fixed order per thread
template <typename T>
__global__ __launch_bounds__(CT) void ce_stats_kernel(int64_t n, int k, const T* x,
                                                      const float* label, float lo, float hi,
                                                      const float* wts, double* stats) {
  __shared__ double red[3 * (CT / 64)];
  double sl = 0, sw = 0, bad = 0;
  for (int64_t i = threadIdx.x; i < n; i += CT) {
    const int c = ce_bin(label[i], k, lo, hi);
    if (c < 0) {
      bad += 1.0;
      continue;
    }
    const T* z = x + i * k;
    float m = -INFINITY;
    for (int j = 0; j < k; ++j) m = fmaxf(m, to_f(z[j]));
    float s = 0.f;
    for (int j = 0; j < k; ++j) s += __expf(to_f(z[j]) - m);
    const double nll = (double)(m + __logf(s) - to_f(z[c]));
    const double w = wts ? (double)wts[c] : 1.0;
    sl += w * nll;
    sw += w;
  }
  block_sum3_d(sl, sw, bad, red);
  if (threadIdx.x == 0) {
    stats[0] = sl;
    stats[1] = sw;
    stats[2] = bad;
    stats[3] = 0.0;
  }
}

// world ranks' stats (rank order) -> loss = sum w nll / sum w (NaN on an invalid label) and
// coef[0] = 1 / sum w for the backward
__global__ void ce_finish_kernel(int world, const double* stats_all, float* loss, double* coef) {
  if (threadIdx.x != 0) return;
  double sl = 0, sw = 0, bad = 0;
  for (int r = 0; r < world; ++r) {
    sl += stats_all[4 * r];
    sw += stats_all[4 * r + 1];
    bad += stats_all[4 * r + 2];
  }
  *loss = bad > 0 ? __builtin_nanf("") : (float)(sl / sw);
  coef[0] = bad > 0 ? __builtin_nan("") : 1.0 / sw;
}

// dx_ij = grad_loss * w[c_i] / sum w * (softmax(x_i)_j - [j == c_i])
template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(int64_t n, int k, const T* x,
                                                     const float* label, float lo, float hi,
                                                     const float* wts, const double* coef,
                                                     const float* grad_loss, T* dx) {
  const double inv = coef[0];
  const float g = grad_loss ? *grad_loss : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = ce_bin(label[i], k, lo, hi);
    const T* z = x + i * k;
    T* dz = dx + i * k;
    const float sc = c < 0 ? __builtin_nanf("")
                           : (float)((wts ? (double)wts[c] : 1.0) * inv * (double)g);
    float m = -INFINITY;
    for (int j = 0; j < k; ++j) m = fmaxf(m, to_f(z[j]));
    float s = 0.f;
    float pv[MAXK];
    for (int j = 0; j < k; ++j) {
      pv[j] = __expf(to_f(z[j]) - m);
      s += pv[j];
    }
    const float is = 1.f / s;
    for (int j = 0; j < k; ++j) dz[j] = from_f<T>(sc * (pv[j] * is - (j == c ? 1.f : 0.f)));
  }
}

// the digitized labels themselves (int64, as the reference's torch.cuda.LongTensor(y_dig))
__global__ void ce_labels_kernel(int64_t n, int k, const float* label, float lo, float hi,
                                 int64_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ce_bin(label[i], k, lo, hi);
}

}  // namespace jmt

using namespace jmt;

#define JMT_CE_DISPATCH(name, KER, GRID, BLK, ...)                                         \
  switch (x_dt) {                                                                          \
    case JMT_F32: hipLaunchKernelGGL((KER<float>), GRID, BLK, 0, st, __VA_ARGS__(float)); break; \
    case JMT_BF16: hipLaunchKernelGGL((KER<__bf16>), GRID, BLK, 0, st, __VA_ARGS__(__bf16)); break; \
    case JMT_F16: hipLaunchKernelGGL((KER<_Float16>), GRID, BLK, 0, st, __VA_ARGS__(_Float16)); break; \
    default: return set_error(JMT_ERR_ARG, name ": dtype");                                 \
  }

extern "C" int jmt_ce_stats(int x_dt, int64_t n, int k, const void* x, const float* label,
                            float lo, float hi, const float* weights, double* stats,
                            void* stream) {
  JMT_CHECK_ARG(k >= 2 && k <= MAXK, "jmt_ce_stats: digitize_num %d unsupported", k);
  JMT_CHECK_ARG(stats && (n == 0 || (x && label)), "jmt_ce_stats: null pointer");
  hipStream_t st = as_stream(stream);
#define ARGS(T) n, k, (const T*)x, label, lo, hi, weights, stats
  JMT_CE_DISPATCH("jmt_ce_stats", ce_stats_kernel, dim3(1), dim3(CT), ARGS)
#undef ARGS
  JMT_LAUNCH_CHECK("jmt_ce_stats");
  return JMT_OK;
}

extern "C" int jmt_ce_finish(int world, const double* stats_all, float* loss, double* coef,
                             void* stream) {
  JMT_CHECK_ARG(world >= 1 && stats_all && loss && coef, "jmt_ce_finish: bad args");
  hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(64), 0, as_stream(stream), world,
                     stats_all, loss, coef);
  JMT_LAUNCH_CHECK("jmt_ce_finish");
  return JMT_OK;
}

extern "C" int jmt_ce_bwd(int x_dt, int64_t n, int k, const void* x, const float* label,
                          float lo, float hi, const float* weights, const double* coef,
                          const float* grad_loss, void* dx, void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(k >= 2 && k <= MAXK && x && label && coef && dx, "jmt_ce_bwd: bad args");
  hipStream_t st = as_stream(stream);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
#define ARGS(T) n, k, (const T*)x, label, lo, hi, weights, coef, grad_loss, (T*)dx
  JMT_CE_DISPATCH("jmt_ce_bwd", ce_bwd_kernel, dim3(blocks), dim3(256), ARGS)
#undef ARGS
  JMT_LAUNCH_CHECK("jmt_ce_bwd");
  return JMT_OK;
}

extern "C" int jmt_ce_labels(int64_t n, int k, const float* label, float lo, float hi,
                             int64_t* out, void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(k >= 2 && k <= MAXK && label && out, "jmt_ce_labels: bad args");
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(ce_labels_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), n, k,
                     label, lo, hi, out);
  JMT_LAUNCH_CHECK("jmt_ce_labels");
  return JMT_OK;
}

extern "C" int jmt_ccc_stats(int kind, int pred_dt, int64_t n, int k, const void* pred,
                             const float* label, float ignore, float lo, float hi, double* stats,
                             void* stream) {
  JMT_CHECK_ARG(kind == 0 || kind == 1, "jmt_ccc_stats: kind");
  JMT_CHECK_ARG(k >= 1 && k <= MAXK, "jmt_ccc_stats: digitize_num %d unsupported", k);
  JMT_CHECK_ARG(stats && (n == 0 || (pred && label)), "jmt_ccc_stats: null pointer");
  hipStream_t st = as_stream(stream);
  switch (pred_dt) {
    case JMT_F32: hipLaunchKernelGGL((ccc_stats_kernel<float>), dim3(1), dim3(CT), 0, st, kind, n, k, (const float*)pred, label, ignore, lo, hi, stats); break;
    case JMT_BF16: hipLaunchKernelGGL((ccc_stats_kernel<__bf16>), dim3(1), dim3(CT), 0, st, kind, n, k, (const __bf16*)pred, label, ignore, lo, hi, stats); break;
    case JMT_F16: hipLaunchKernelGGL((ccc_stats_kernel<_Float16>), dim3(1), dim3(CT), 0, st, kind, n, k, (const _Float16*)pred, label, ignore, lo, hi, stats); break;
    default: return set_error(JMT_ERR_ARG, "jmt_ccc_stats: dtype");
  }
  JMT_LAUNCH_CHECK("jmt_ccc_stats");
  return JMT_OK;
}

extern "C" int jmt_ccc_finish(int kind, int world, const double* stats_all, int64_t bs, float eps,
                              float* loss, double* coef, void* stream) {
  return jmt_ccc_finish_add(kind, world, stats_all, bs, eps, nullptr, loss, coef, stream);
}

extern "C" int jmt_ccc_finish_add(int kind, int world, const double* stats_all, int64_t bs,
                                  float eps, const float* add, float* loss, double* coef,
                                  void* stream) {
  JMT_CHECK_ARG(world >= 1 && stats_all && loss && coef, "jmt_ccc_finish: bad args");
  hipLaunchKernelGGL(ccc_finish_kernel, dim3(1), dim3(64), 0, as_stream(stream), kind, world,
                     stats_all, bs, eps, add, loss, coef);
  JMT_LAUNCH_CHECK("jmt_ccc_finish");
  return JMT_OK;
}

extern "C" int jmt_ccc_bwd(int kind, int pred_dt, int64_t n, int k, const void* pred,
                           const float* label, float ignore, float lo, float hi,
                           const double* coef, const float* grad_loss, void* dpred,
                           void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(k >= 1 && k <= MAXK && pred && label && coef && dpred, "jmt_ccc_bwd: bad args");
  hipStream_t st = as_stream(stream);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  switch (pred_dt) {
    case JMT_F32: hipLaunchKernelGGL((ccc_bwd_kernel<float>), dim3(blocks), dim3(256), 0, st, kind, n, k, (const float*)pred, label, ignore, lo, hi, coef, grad_loss, (float*)dpred); break;
    case JMT_BF16: hipLaunchKernelGGL((ccc_bwd_kernel<__bf16>), dim3(blocks), dim3(256), 0, st, kind, n, k, (const __bf16*)pred, label, ignore, lo, hi, coef, grad_loss, (__bf16*)dpred); break;
    case JMT_F16: hipLaunchKernelGGL((ccc_bwd_kernel<_Float16>), dim3(blocks), dim3(256), 0, st, kind, n, k, (const _Float16*)pred, label, ignore, lo, hi, coef, grad_loss, (_Float16*)dpred); break;
    default: return set_error(JMT_ERR_ARG, "jmt_ccc_bwd: dtype");
  }
  JMT_LAUNCH_CHECK("jmt_ccc_bwd");
  return JMT_OK;
}

extern "C" int jmt_mask_indices(int64_t n, const float* label, float ignore, int64_t* idx,
                                int64_t* count, void* stream) {
  JMT_CHECK_ARG(idx && count && (n == 0 || label), "jmt_mask_indices: null pointer");
  hipLaunchKernelGGL(mask_indices_kernel, dim3(1), dim3(CT), 0, as_stream(stream), n, label,
                     ignore, idx, count);
  JMT_LAUNCH_CHECK("jmt_mask_indices");
  return JMT_OK;
}
