// Fused SGD (momentum, dampening, weight decay, nesterov) over one flat fp32 parameter buffer,
// torch.optim.SGD semantics as configured by instantiator.py:32-38 / config_file.json:73-80.
// One launch for all parameters (the reference's per-tensor foreach kernels become one stream of
// 16-B vector accesses), optional unscale of the gradient (GradScaler) and an optional bf16/f16
// shadow copy of the updated weights for the next step's MFMA GEMMs.
#include "common.h"

namespace jmt {

template <typename TS>
__global__ __launch_bounds__(256) void sgd_kernel(int64_t n, float* __restrict__ p,
                                                  const float* __restrict__ g,
                                                  float* __restrict__ buf, float lr, float mom,
                                                  float damp, float wd, int nesterov, int first,
                                                  float gs, TS* __restrict__ shadow) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float w = p[i];
    float d = g[i] * gs;
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

extern "C" int jmt_sgd_step(int64_t n, float* param, const float* grad, float* momentum_buf,
                            float lr, float momentum, float dampening, float weight_decay,
                            int nesterov, int first_step, float grad_scale, void* shadow,
                            int shadow_dt, void* stream) {
  if (n == 0) return JMT_OK;
  JMT_CHECK_ARG(param && grad, "jmt_sgd_step: null pointer");
  JMT_CHECK_ARG(momentum == 0.f || momentum_buf, "jmt_sgd_step: momentum needs a buffer");
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = as_stream(stream);
  if (shadow && shadow_dt == JMT_F16)
    hipLaunchKernelGGL((sgd_kernel<_Float16>), dim3(blocks), dim3(256), 0, st, n, param, grad,
                       momentum_buf, lr, momentum, dampening, weight_decay, nesterov, first_step,
                       grad_scale, (_Float16*)shadow);
  else
    hipLaunchKernelGGL((sgd_kernel<__bf16>), dim3(blocks), dim3(256), 0, st, n, param, grad,
                       momentum_buf, lr, momentum, dampening, weight_decay, nesterov, first_step,
                       grad_scale, (__bf16*)shadow);
  JMT_LAUNCH_CHECK("jmt_sgd_step");
  return JMT_OK;
}
