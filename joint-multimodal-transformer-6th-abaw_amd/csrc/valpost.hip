// Validation post-processing of the JMT path on the GPU, replacing the
// per-frame Python loop of val.py:313-357, the numpy/scipy tail of val.py:359-382 and
// EvaluationMetrics/cccmetric.py:4-21:
//   scatter   per-frame predictions / labels into per-video arrays (frames with a -5.0 label are
//             skipped; a later (frame, video) hit overwrites an earlier one, as the Python loop's
//             iteration order does),
//   smooth    clip to [-1, 1] + scipy.ndimage.uniform_filter1d(size, mode='constant', cval=0)
//             per video,
//   ccc       Lin's CCC of the concatenated (smoothed prediction, label) arrays.
// Everything in float64 (the reference's numpy arrays are float64 whenever a frame stayed at the
// integer 0 it was initialised with).  Integer work (slot indices, the last-writer rule) is exact.
#include "common.h"

namespace jmt {

constexpr int VT = 256;

// flat slot of element i, or -1 when the reference skips it (val.py:335-352): label -5.0,
// frameid > length; index frameid-1 with Python's negative-index rule (frameid 0 -> last
// element); an index outside the video's array (an IndexError in the reference) is skipped.
__device__ __forceinline__ int64_t vp_slot(int64_t i, const int* fid, const int* len,
                                           const int* vid, const int64_t* off, const int* seglen,
                                           const float* lv, const float* la, float ignore) {
  if (la[i] == ignore || lv[i] == ignore) return -1;
  const int f = fid[i];
  if (f > len[i]) return -1;
  const int v = vid[i];
  const int L = seglen[v];
  int64_t idx = (int64_t)f - 1;
  if (idx < 0) idx += L;
  if (idx < 0 || idx >= L) return -1;
  return off[v] + idx;
}

// winner[slot] = max(seq0 + i + 1) over the elements hitting the slot: the LAST writer in the
// reference's iteration order (sequence numbers grow across update calls, so earlier batches lose)
__global__ __launch_bounds__(VT) void vp_claim_kernel(int64_t n, const int* fid, const int* len,
                                                      const int* vid, const int64_t* off,
                                                      const int* seglen, const float* lv,
                                                      const float* la, float ignore, int64_t seq0,
                                                      unsigned long long* winner) {
  for (int64_t i = blockIdx.x * (int64_t)VT + threadIdx.x; i < n; i += (int64_t)gridDim.x * VT) {
    const int64_t s = vp_slot(i, fid, len, vid, off, seglen, lv, la, ignore);
    if (s >= 0) atomicMax(winner + s, (unsigned long long)(seq0 + i + 1));
  }
}

__global__ __launch_bounds__(VT) void vp_write_kernel(int64_t n, const int* fid, const int* len,
                                                      const int* vid, const int64_t* off,
                                                      const int* seglen, const float* pv,
                                                      const float* pa, const float* lv,
                                                      const float* la, float ignore, int64_t seq0,
                                                      const unsigned long long* winner,
                                                      double* PV, double* PA, double* LV,
                                                      double* LA) {
  for (int64_t i = blockIdx.x * (int64_t)VT + threadIdx.x; i < n; i += (int64_t)gridDim.x * VT) {
    const int64_t s = vp_slot(i, fid, len, vid, off, seglen, lv, la, ignore);
    if (s >= 0 && winner[s] == (unsigned long long)(seq0 + i + 1)) {
      PV[s] = (double)pv[i];
      PA[s] = (double)pa[i];
      LV[s] = (double)lv[i];
      LA[s] = (double)la[i];
    }
  }
}

// y[i] = mean of clip(x, -1, 1) over [i - size/2, i - size/2 + size) inside i's video, zero
// outside (uniform_filter1d, mode='constant', origin 0: window offset size//2 to the left)
__global__ __launch_bounds__(VT) void vp_smooth_kernel(int64_t total, int nseg, const int64_t* off,
                                                       const int* seglen, const double* x,
                                                       int size, double* y) {
  for (int64_t i = blockIdx.x * (int64_t)VT + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * VT) {
    int lo = 0, hi = nseg - 1;                 // last segment with off <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int64_t o = off[lo];
    const int64_t L = seglen[lo];
    const int64_t j = i - o;
    const int64_t w0 = j - size / 2;
    double s = 0.0;
    for (int k = 0; k < size; ++k) {
      const int64_t t = w0 + k;
      if (t >= 0 && t < L) s += fmin(fmax(x[o + t], -1.0), 1.0);
    }
    y[i] = s / (double)size;
  }
}

__device__ __forceinline__ double vp_block_sum(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < 1024 / 64; ++i) s += red[i];
  __syncthreads();
  return s;
}

// cccmetric.py:4-21 in float64; block b handles pair b (valence, arousal).  Deterministic: fixed
// per-thread striding and a fixed-order block reduction.
__global__ __launch_bounds__(1024) void vp_ccc_kernel(int64_t n, const double* x0, const double* y0,
                                                      const double* x1, const double* y1,
                                                      double* out) {
  __shared__ double red[1024 / 64];
  const double* x = blockIdx.x == 0 ? x0 : x1;
  const double* y = blockIdx.x == 0 ? y0 : y1;
  double sx = 0.0, sy = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    sx += x[i];
    sy += y[i];
  }
  const double mx = vp_block_sum(sx, red) / (double)n;
  const double my = vp_block_sum(sy, red) / (double)n;
  double xx = 0.0, yy = 0.0, xy = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const double dx = x[i] - mx, dy = y[i] - my;
    xx += dx * dx;
    yy += dy * dy;
    xy += dx * dy;
  }
  xx = vp_block_sum(xx, red);
  yy = vp_block_sum(yy, red);
  xy = vp_block_sum(xy, red);
  if (threadIdx.x == 0) {
    const double rho = xy / (sqrt(xx) * sqrt(yy));
    const double xs = sqrt(xx / (double)n), ys = sqrt(yy / (double)n);
    out[blockIdx.x] = 2.0 * rho * xs * ys / (xs * xs + ys * ys + (mx - my) * (mx - my));
  }
}

static unsigned vp_blocks(int64_t n) {
  const int64_t b = (n + VT - 1) / VT;
  return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace jmt

using namespace jmt;

extern "C" int jmt_vp_scatter(int64_t n, const int* fid, const int* len, const int* vid,
                              const int64_t* off, const int* seglen, const float* pv,
                              const float* pa, const float* lv, const float* la, float ignore,
                              int64_t seq0, uint64_t* winner, double* PV, double* PA, double* LV,
                              double* LA, void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(n > 0 && seq0 >= 0 && fid && len && vid && off && seglen && pv && pa && lv && la &&
                    winner && PV && PA && LV && LA,
                "jmt_vp_scatter: bad args");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(vp_claim_kernel, dim3(vp_blocks(n)), dim3(VT), 0, st, n, fid, len, vid, off,
                     seglen, lv, la, ignore, seq0, (unsigned long long*)winner);
  JMT_LAUNCH_CHECK("jmt_vp_scatter(claim)");
  hipLaunchKernelGGL(vp_write_kernel, dim3(vp_blocks(n)), dim3(VT), 0, st, n, fid, len, vid, off,
                     seglen, pv, pa, lv, la, ignore, seq0, (const unsigned long long*)winner, PV,
                     PA, LV, LA);
  JMT_LAUNCH_CHECK("jmt_vp_scatter(write)");
  return JMT_OK;
}

extern "C" int jmt_vp_smooth(int64_t total, int nseg, const int64_t* off, const int* seglen,
                             const double* x, int size, double* y, void* stream) {
  if (total == 0) return JMT_OK;
  JMT_CHECK_ARG(total > 0 && nseg > 0 && size > 0 && off && seglen && x && y,
                "jmt_vp_smooth: bad args");
  hipLaunchKernelGGL(vp_smooth_kernel, dim3(vp_blocks(total)), dim3(VT), 0, as_stream(stream),
                     total, nseg, off, seglen, x, size, y);
  JMT_LAUNCH_CHECK("jmt_vp_smooth");
  return JMT_OK;
}

extern "C" int jmt_vp_ccc(int64_t n, const double* x0, const double* y0, const double* x1,
                          const double* y1, double* out2, void* stream) {
  JMT_CHECK_ARG(n > 1, "jmt_vp_ccc: needs at least 2 frames (cccmetric.py:9-11 exits)");
  JMT_CHECK_ARG(x0 && y0 && x1 && y1 && out2, "jmt_vp_ccc: null pointer");
  hipLaunchKernelGGL(vp_ccc_kernel, dim3(2), dim3(1024), 0, as_stream(stream), n, x0, y0, x1, y1,
                     out2);
  JMT_LAUNCH_CHECK("jmt_vp_ccc");
  return JMT_OK;
}
