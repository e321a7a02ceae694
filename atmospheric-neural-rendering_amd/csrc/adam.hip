// K10: fused Adam / AdamW over one flat f32 parameter buffer.
//
// Replaces torch.optim.AdamW at src/atmonr/pipelines/instant_ngp.py:120-126 (two param
// groups: hash tables wd=0, MLPs wd=1e-2; stepped at src/atmonr/trainer.py:105) and
// torch.optim.Adam at src/atmonr/pipelines/nerf.py:70. Per element, following torch's
// single-tensor algorithm:
//   AdamW: p *= 1 - lr*wd            Adam(L2): g += wd*p
//   m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
// One HBM pass: reads p, g, m, v; writes p, m, v, optionally the f16 shadow of p used by
// the next forward, and optionally zeroes g (optimizer.zero_grad fused in).

#pragma clang fp contract(off)

#include "anr_common.h"

#include <cmath>

namespace anr {

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   __half* __restrict__ p16, int64_t n,
                                                   float lr, float b1, float b2, float eps,
                                                   float wd, float decay, int decoupled,
                                                   float step_size, float bc2_sqrt,
                                                   int zero_grad) {
  const float w1 = 1.0f - b1;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float pi = p[i];
    float gi = g[i];
    if (wd != 0.0f) {
      if (decoupled)
        pi = pi * decay;  // param.mul_(1 - lr * weight_decay), scalar in double
      else
        gi = gi + wd * pi;
    }
    float mi = m[i];
    // torch.lerp(self, end, weight)
    mi = w1 < 0.5f ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.0f - w1);
    float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + (-step_size) * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (p16) p16[i] = __float2half_rn(pi);
    if (zero_grad) g[i] = 0.0f;
  }
}

}  // namespace anr

extern "C" int anr_adam_step(float* params, float* grad, float* exp_avg, float* exp_avg_sq,
                             void* params_f16, int64_t n, float lr, float beta1, float beta2,
                             float eps, float weight_decay, int32_t decoupled, int64_t step,
                             int32_t zero_grad, anr_stream_t stream) {
  using namespace anr;
  if (n == 0) return ANR_OK;
  ANR_CHECK_ARG(params && grad && exp_avg && exp_avg_sq, "anr_adam_step: null argument");
  ANR_CHECK_ARG(n >= 0 && step >= 1, "anr_adam_step: bad size/step");
  if (n == 0) return ANR_OK;
  // Python-double bias corrections, as torch computes them for a non-capturable step.
  const double bc1 = 1.0 - std::pow(static_cast<double>(beta1), static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(static_cast<double>(beta2), static_cast<double>(step));
  const float step_size = static_cast<float>(static_cast<double>(lr) / bc1);
  const float bc2_sqrt = static_cast<float>(std::sqrt(bc2));
  const float decay =
      static_cast<float>(1.0 - static_cast<double>(lr) * static_cast<double>(weight_decay));
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     as_stream(stream), params, grad, exp_avg, exp_avg_sq,
                     static_cast<__half*>(params_f16), n, lr, beta1, beta2, eps, weight_decay,
                     decay, decoupled, step_size, bc2_sqrt, zero_grad);
  ANR_CHECK_LAUNCH("anr_adam_step");
  return ANR_OK;
}
