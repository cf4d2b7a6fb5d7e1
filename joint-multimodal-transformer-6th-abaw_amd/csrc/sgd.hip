// Fused SGD (momentum, dampening, weight decay, nesterov) over one flat fp32 parameter buffer,
// torch.optim.SGD semantics as configured by instantiator.py:32-38 / config_file.json:73-80.
// One launch for all parameters (the reference's per-tensor foreach kernels become one stream of
// 16-B vector accesses), optional unscale of the gradient (GradScaler) and an optional bf16/f16
// shadow copy of the updated weights for the next step's MFMA GEMMs.
#include "common.h"

namespace jmt {

// ZG: the gradient is read and then zeroed in the same pass (the next step's zero_grad folded in:
// no separate 53.6 MB fill launch per step)
template <typename TS, bool ZG>
__global__ __launch_bounds__(256) void sgd_kernel(int64_t n, float* __restrict__ p,
                                                  float* __restrict__ g,
                                                  float* __restrict__ buf, float lr, float mom,
                                                  float damp, float wd, int nesterov, int first,
                                                  float gs, TS* __restrict__ shadow) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float w = p[i];
    float d = g[i] * gs;
    if constexpr (ZG) g[i] = 0.f;
    if (wd != 0.f) d += wd * w;
    if (mom != 0.f) {
      float b = first ? d : buf[i] * mom + (1.f - damp) * d;
      buf[i] = b;
      d = nesterov ? d + mom * b : b;
    }
    const float nw = w - lr * d;
    p[i] = nw;
    if (shadow) shadow[i] = from_f<TS>(nw);
  }
}

}  // namespace jmt

using namespace jmt;

static int sgd_launch(int64_t n, float* param, float* grad, float* momentum_buf, float lr,
                      float momentum, float dampening, float weight_decay, int nesterov,
                      int first_step, float grad_scale, void* shadow, int shadow_dt, bool zg,
                      void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(param && grad, "jmt_sgd_step: null pointer");
  JMT_CHECK_ARG(momentum == 0.f || momentum_buf, "jmt_sgd_step: momentum needs a buffer");
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = as_stream(stream);
#define JMT_SGD(TS, ZG)                                                                         \
  hipLaunchKernelGGL((sgd_kernel<TS, ZG>), dim3(blocks), dim3(256), 0, st, n, param, grad,       \
                     momentum_buf, lr, momentum, dampening, weight_decay, nesterov, first_step,  \
                     grad_scale, (TS*)shadow)
  const bool f16 = shadow && shadow_dt == JMT_F16;
  if (f16 && zg) JMT_SGD(_Float16, true);
  else if (f16) JMT_SGD(_Float16, false);
  else if (zg) JMT_SGD(__bf16, true);
  else JMT_SGD(__bf16, false);
#undef JMT_SGD
  JMT_LAUNCH_CHECK("jmt_sgd_step");
  return JMT_OK;
}

extern "C" int jmt_sgd_step(int64_t n, float* param, const float* grad, float* momentum_buf,
                            float lr, float momentum, float dampening, float weight_decay,
                            int nesterov, int first_step, float grad_scale, void* shadow,
                            int shadow_dt, void* stream) {
  return sgd_launch(n, param, const_cast<float*>(grad), momentum_buf, lr, momentum, dampening,
                    weight_decay, nesterov, first_step, grad_scale, shadow, shadow_dt, false,
                    stream);
}

extern "C" int jmt_sgd_step_zero(int64_t n, float* param, float* grad, float* momentum_buf,
                                 float lr, float momentum, float dampening, float weight_decay,
                                 int nesterov, int first_step, float grad_scale, void* shadow,
                                 int shadow_dt, void* stream) {
  return sgd_launch(n, param, grad, momentum_buf, lr, momentum, dampening, weight_decay,
                    nesterov, first_step, grad_scale, shadow, shadow_dt, true, stream);
}

// ------------------------------------------------------------------ GradScaler (train.py:89,
// 314-316: scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()) with all state
// on the device, so a training step with loss scaling needs no host synchronisation and captures
// into a hipGraph.  amp[5] (fp32): scale, inv_scale, found_inf, growth_tracker, steps_taken.
namespace jmt {

__global__ __launch_bounds__(256) void amp_check_kernel(int64_t n, const float* __restrict__ g,
                                                        float* amp) {
  const float inv = amp[1];
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i] * inv);
  if (__any(bad) && (threadIdx.x & 63) == 0) amp[2] = 1.f;   // same value from every writer
}

// torch.optim.SGD step on the unscaled gradient, skipped when found_inf (torch's scaler.step
// skips optimizer.step()); the momentum buffer's first-step rule follows the device step count.
template <typename TS, bool ZG>
__global__ __launch_bounds__(256) void sgd_amp_kernel(int64_t n, float* __restrict__ p,
                                                      float* __restrict__ g,
                                                      float* __restrict__ buf, float lr, float mom,
                                                      float damp, float wd, int nesterov,
                                                      int allow_first, const float* amp,
                                                      TS* __restrict__ shadow) {
  const bool skip = amp[2] != 0.f;            // found_inf: no update (the grads still zeroed)
  if (skip && !ZG) return;
  const float gs = amp[1];
  const int first = allow_first && amp[4] == 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (skip) {
      g[i] = 0.f;
      continue;
    }
    const float w = p[i];
    float d = g[i] * gs;
    if constexpr (ZG) g[i] = 0.f;
    if (wd != 0.f) d += wd * w;
    if (mom != 0.f) {
      float b = first ? d : buf[i] * mom + (1.f - damp) * d;
      buf[i] = b;
      d = nesterov ? d + mom * b : b;
    }
    const float nw = w - lr * d;
    p[i] = nw;
    if (shadow) shadow[i] = from_f<TS>(nw);
  }
}

// torch's _amp_update_scale_: backoff on overflow, growth after growth_interval clean steps
__global__ void amp_update_kernel(float* amp, float growth, float backoff, int interval) {
  if (threadIdx.x != 0) return;
  float scale = amp[0];
  if (amp[2] != 0.f) {
    scale *= backoff;
    amp[3] = 0.f;
  } else {
    amp[4] += 1.f;
    const float t = amp[3] + 1.f;
    if (t >= (float)interval) {
      const float ns = scale * growth;
      if (isfinite(ns)) scale = ns;
      amp[3] = 0.f;
    } else {
      amp[3] = t;
    }
  }
  amp[0] = scale;
  amp[1] = (float)(1.0 / (double)scale);   // unscale_: scale.double().reciprocal().float()
  amp[2] = 0.f;
}

}  // namespace jmt

extern "C" int jmt_amp_check(int64_t n, const float* grad, float* amp, void* stream) {
  JMT_CHECK_ARG(grad && amp && n >= 0, "jmt_amp_check: bad args");
  if (n == 0) return JMT_OK;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(amp_check_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), n, grad,
                     amp);
  JMT_LAUNCH_CHECK("jmt_amp_check");
  return JMT_OK;
}

static int sgd_amp_launch(int64_t n, float* param, float* grad, float* momentum_buf, float lr,
                          float momentum, float dampening, float weight_decay, int nesterov,
                          int allow_first, const float* amp, void* shadow, int shadow_dt, bool zg,
                          void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(param && grad && amp, "jmt_sgd_step_amp: null pointer");
  JMT_CHECK_ARG(momentum == 0.f || momentum_buf, "jmt_sgd_step_amp: momentum needs a buffer");
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = as_stream(stream);
#define JMT_SGDA(TS, ZG)                                                                        \
  hipLaunchKernelGGL((sgd_amp_kernel<TS, ZG>), dim3(blocks), dim3(256), 0, st, n, param, grad,   \
                     momentum_buf, lr, momentum, dampening, weight_decay, nesterov, allow_first, \
                     amp, (TS*)shadow)
  const bool f16 = shadow && shadow_dt == JMT_F16;
  if (f16 && zg) JMT_SGDA(_Float16, true);
  else if (f16) JMT_SGDA(_Float16, false);
  else if (zg) JMT_SGDA(__bf16, true);
  else JMT_SGDA(__bf16, false);
#undef JMT_SGDA
  JMT_LAUNCH_CHECK("jmt_sgd_step_amp");
  return JMT_OK;
}

extern "C" int jmt_sgd_step_amp(int64_t n, float* param, const float* grad, float* momentum_buf,
                                float lr, float momentum, float dampening, float weight_decay,
                                int nesterov, int allow_first, const float* amp, void* shadow,
                                int shadow_dt, void* stream) {
  return sgd_amp_launch(n, param, const_cast<float*>(grad), momentum_buf, lr, momentum,
                        dampening, weight_decay, nesterov, allow_first, amp, shadow, shadow_dt,
                        false, stream);
}

extern "C" int jmt_sgd_step_amp_zero(int64_t n, float* param, float* grad, float* momentum_buf,
                                     float lr, float momentum, float dampening,
                                     float weight_decay, int nesterov, int allow_first,
                                     const float* amp, void* shadow, int shadow_dt,
                                     void* stream) {
  return sgd_amp_launch(n, param, grad, momentum_buf, lr, momentum, dampening, weight_decay,
                        nesterov, allow_first, amp, shadow, shadow_dt, true, stream);
}

extern "C" int jmt_amp_update(float* amp, float growth_factor, float backoff_factor,
                              int growth_interval, void* stream) {
  JMT_CHECK_ARG(amp && growth_interval >= 1, "jmt_amp_update: bad args");
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, as_stream(stream), amp,
                     growth_factor, backoff_factor, growth_interval);
  JMT_LAUNCH_CHECK("jmt_amp_update");
  return JMT_OK;
}
