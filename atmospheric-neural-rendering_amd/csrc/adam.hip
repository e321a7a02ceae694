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
// anr_adam_step_multi updates every tensor of a step in one launch (FusedAdam's default).

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

// Multi-tensor form: every tensor of an optimizer step in ONE launch. The per-tensor
// descriptors travel by value in the kernel arguments (no device memory of the library's
// own); tensor t owns blocks [first[t], first[t + 1]) of the grid, each block 1,024
// consecutive elements (4 per thread, strided by 256 for coalescing). Same per-element
// arithmetic as adam_kernel.
struct AdamTensors {
  float* p[ANR_ADAM_MAX_TENSORS];
  float* g[ANR_ADAM_MAX_TENSORS];
  float* m[ANR_ADAM_MAX_TENSORS];
  float* v[ANR_ADAM_MAX_TENSORS];
  __half* p16[ANR_ADAM_MAX_TENSORS];
  int64_t n[ANR_ADAM_MAX_TENSORS];
  float wd[ANR_ADAM_MAX_TENSORS], decay[ANR_ADAM_MAX_TENSORS];
  float step_size[ANR_ADAM_MAX_TENSORS], bc2_sqrt[ANR_ADAM_MAX_TENSORS];
  float gq[ANR_ADAM_MAX_TENSORS];  // grad_quant (0: none)
  int first[ANR_ADAM_MAX_TENSORS + 1];
  int count;
};

// anr_grad_quantize_f16's rounding on the update's read of g
__device__ __forceinline__ float quant_f16(float g, float s) {
  const float h1 = __half2float(__float2half_rn(g * s));
  return __half2float(__float2half_rn(h1 * (1.0f / s)));
}

__global__ void __launch_bounds__(256) adam_multi_kernel(AdamTensors a, float b1, float b2,
                                                         float eps, int decoupled,
                                                         int zero_grad) {
  int t = 0;  // block-uniform
  while (t + 1 < a.count && static_cast<int>(blockIdx.x) >= a.first[t + 1]) ++t;
  float* __restrict__ p = a.p[t];
  float* __restrict__ g = a.g[t];
  float* __restrict__ m = a.m[t];
  float* __restrict__ v = a.v[t];
  __half* __restrict__ p16 = a.p16[t];
  const int64_t n = a.n[t];
  const float wd = a.wd[t], decay = a.decay[t], step_size = a.step_size[t],
              bc2_sqrt = a.bc2_sqrt[t], gq = a.gq[t];
  const float w1 = 1.0f - b1;
  const int64_t base = static_cast<int64_t>(static_cast<int>(blockIdx.x) - a.first[t]) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i >= n) break;
    float pi = p[i];
    float gi = g[i];
    if (gq != 0.0f) gi = quant_f16(gi, gq);
    if (wd != 0.0f) {
      if (decoupled)
        pi = pi * decay;
      else
        gi = gi + wd * pi;
    }
    float mi = m[i];
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

// Device-step form (hipGraph capture): the step count and every tensor's lr live in
// caller-owned device memory, so one captured launch pair serves every replay. The tick
// kernel advances the step and forms each tensor's scalars in double, as adam_scalars
// does on the host; the update kernel reads them (block-uniform scalar loads) and runs
// adam_multi_kernel's per-element arithmetic.
struct AdamWd {
  float v[ANR_ADAM_DEV_MAX_TENSORS];
};

__global__ void adam_tick_kernel(int64_t* __restrict__ d_step, const float* __restrict__ d_lr,
                                 AdamWd wd, float beta1, float beta2, int n,
                                 float* __restrict__ scal) {
  const int t = threadIdx.x;
  const int64_t step = *d_step + 1;
  __syncthreads();  // every thread has read the old count before thread 0 writes
  if (t == 0) *d_step = step;
  if (t >= n) return;
  const double lr = static_cast<double>(d_lr[t]);
  const double bc1 = 1.0 - pow(static_cast<double>(beta1), static_cast<double>(step));
  const double bc2 = 1.0 - pow(static_cast<double>(beta2), static_cast<double>(step));
  scal[3 * t + 0] = static_cast<float>(lr / bc1);
  scal[3 * t + 1] = static_cast<float>(sqrt(bc2));
  scal[3 * t + 2] = static_cast<float>(1.0 - lr * static_cast<double>(wd.v[t]));
}

struct AdamTensorsDev {
  float* p[ANR_ADAM_MAX_TENSORS];
  float* g[ANR_ADAM_MAX_TENSORS];
  float* m[ANR_ADAM_MAX_TENSORS];
  float* v[ANR_ADAM_MAX_TENSORS];
  __half* p16[ANR_ADAM_MAX_TENSORS];
  int64_t n[ANR_ADAM_MAX_TENSORS];
  float wd[ANR_ADAM_MAX_TENSORS];
  int idx[ANR_ADAM_MAX_TENSORS];  // the tensor's index in the caller's array (its scalars)
  float gq[ANR_ADAM_MAX_TENSORS];  // grad_quant (0: none)
  int first[ANR_ADAM_MAX_TENSORS + 1];
  int count;
};

__global__ void __launch_bounds__(256) adam_multi_dev_kernel(AdamTensorsDev a,
                                                             const float* __restrict__ scal,
                                                             float b1, float b2, float eps,
                                                             int decoupled, int zero_grad) {
  int t = 0;  // block-uniform
  while (t + 1 < a.count && static_cast<int>(blockIdx.x) >= a.first[t + 1]) ++t;
  float* __restrict__ p = a.p[t];
  float* __restrict__ g = a.g[t];
  float* __restrict__ m = a.m[t];
  float* __restrict__ v = a.v[t];
  __half* __restrict__ p16 = a.p16[t];
  const int64_t n = a.n[t];
  const float wd = a.wd[t], gq = a.gq[t];
  const float step_size = scal[3 * a.idx[t] + 0], bc2_sqrt = scal[3 * a.idx[t] + 1],
              decay = scal[3 * a.idx[t] + 2];
  const float w1 = 1.0f - b1;
  const int64_t base = static_cast<int64_t>(static_cast<int>(blockIdx.x) - a.first[t]) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i >= n) break;
    float pi = p[i];
    float gi = g[i];
    if (gq != 0.0f) gi = quant_f16(gi, gq);
    if (wd != 0.0f) {
      if (decoupled)
        pi = pi * decay;
      else
        gi = gi + wd * pi;
    }
    float mi = m[i];
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

// torch's bias corrections and decoupled decay factor, in Python double
static void adam_scalars(float lr, float beta1, float beta2, float weight_decay, int64_t step,
                         float* step_size, float* bc2_sqrt, float* decay) {
  const double bc1 = 1.0 - std::pow(static_cast<double>(beta1), static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(static_cast<double>(beta2), static_cast<double>(step));
  *step_size = static_cast<float>(static_cast<double>(lr) / bc1);
  *bc2_sqrt = static_cast<float>(std::sqrt(bc2));
  *decay = static_cast<float>(1.0 - static_cast<double>(lr) * static_cast<double>(weight_decay));
}

}  // namespace anr

extern "C" int anr_adam_step_multi(const anr_adam_tensor* tensors, int32_t n_tensors,
                                   float beta1, float beta2, float eps, int32_t decoupled,
                                   int32_t zero_grad, anr_stream_t stream) {
  using namespace anr;
  ANR_CHECK_ARG(n_tensors >= 0 && (n_tensors == 0 || tensors), "anr_adam_step_multi: bad tensors");
  // every descriptor is checked before the first launch: a bad tensor after the first
  // ANR_ADAM_MAX_TENSORS must not leave the earlier ones updated (a partial step)
  for (int32_t i = 0; i < n_tensors; ++i) {
    const anr_adam_tensor& d = tensors[i];
    ANR_CHECK_ARG(d.n >= 0 && d.step >= 1, "anr_adam_step_multi: tensor %d: bad size/step", i);
    ANR_CHECK_ARG(d.n == 0 || (d.params && d.grad && d.exp_avg && d.exp_avg_sq),
                  "anr_adam_step_multi: tensor %d: null pointer", i);
    ANR_CHECK_ARG(d.grad_quant >= 0.0f && d.grad_quant < 65504.0f,
                  "anr_adam_step_multi: tensor %d: bad grad_quant", i);
  }
  int32_t t = 0;  // next tensor to place (empty tensors take no slot)
  while (t < n_tensors) {
    AdamTensors a;
    memset(&a, 0, sizeof(a));
    int64_t blocks = 0;
    for (; t < n_tensors && a.count < ANR_ADAM_MAX_TENSORS; ++t) {
      const anr_adam_tensor& d = tensors[t];
      ANR_CHECK_ARG(d.n >= 0 && d.step >= 1, "anr_adam_step_multi: tensor %d: bad size/step", t);
      if (d.n == 0) continue;
      ANR_CHECK_ARG(d.params && d.grad && d.exp_avg && d.exp_avg_sq,
                    "anr_adam_step_multi: tensor %d: null pointer", t);
      const int c = a.count++;
      a.p[c] = d.params;
      a.g[c] = d.grad;
      a.m[c] = d.exp_avg;
      a.v[c] = d.exp_avg_sq;
      a.p16[c] = static_cast<__half*>(d.params_f16);
      a.n[c] = d.n;
      a.wd[c] = d.weight_decay;
      a.gq[c] = d.grad_quant;
      adam_scalars(d.lr, beta1, beta2, d.weight_decay, d.step, &a.step_size[c], &a.bc2_sqrt[c],
                   &a.decay[c]);
      a.first[c] = static_cast<int>(blocks);
      blocks += ceil_div(d.n, 1024);
      ANR_CHECK_ARG(blocks < (int64_t(1) << 31), "anr_adam_step_multi: too many elements");
    }
    if (a.count == 0) continue;
    a.first[a.count] = static_cast<int>(blocks);
    hipLaunchKernelGGL(adam_multi_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       as_stream(stream), a, beta1, beta2, eps, decoupled, zero_grad);
    ANR_CHECK_LAUNCH("anr_adam_step_multi");
  }
  return ANR_OK;
}

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
  float step_size, bc2_sqrt, decay;
  adam_scalars(lr, beta1, beta2, weight_decay, step, &step_size, &bc2_sqrt, &decay);
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     as_stream(stream), params, grad, exp_avg, exp_avg_sq,
                     static_cast<__half*>(params_f16), n, lr, beta1, beta2, eps, weight_decay,
                     decay, decoupled, step_size, bc2_sqrt, zero_grad);
  ANR_CHECK_LAUNCH("anr_adam_step");
  return ANR_OK;
}

extern "C" int anr_adam_step_multi_dev(const anr_adam_tensor* tensors, int32_t n_tensors,
                                       float beta1, float beta2, float eps, int32_t decoupled,
                                       int32_t zero_grad, int64_t* d_step, const float* d_lr,
                                       float* d_scratch, anr_stream_t stream) {
  using namespace anr;
  ANR_CHECK_ARG(n_tensors >= 0 && n_tensors <= ANR_ADAM_DEV_MAX_TENSORS &&
                    (n_tensors == 0 || tensors),
                "anr_adam_step_multi_dev: 0..%d tensors", ANR_ADAM_DEV_MAX_TENSORS);
  ANR_CHECK_ARG(d_step && d_lr && d_scratch, "anr_adam_step_multi_dev: null device state");
  for (int32_t i = 0; i < n_tensors; ++i) {
    const anr_adam_tensor& d = tensors[i];
    ANR_CHECK_ARG(d.n >= 0, "anr_adam_step_multi_dev: tensor %d: bad size", i);
    ANR_CHECK_ARG(d.n == 0 || (d.params && d.grad && d.exp_avg && d.exp_avg_sq),
                  "anr_adam_step_multi_dev: tensor %d: null pointer", i);
    ANR_CHECK_ARG(d.grad_quant >= 0.0f && d.grad_quant < 65504.0f,
                  "anr_adam_step_multi_dev: tensor %d: bad grad_quant", i);
  }
  AdamWd wd;
  memset(&wd, 0, sizeof(wd));
  for (int32_t i = 0; i < n_tensors; ++i) wd.v[i] = tensors[i].weight_decay;
  hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(ANR_ADAM_DEV_MAX_TENSORS), 0,
                     as_stream(stream), d_step, d_lr, wd, beta1, beta2, n_tensors, d_scratch);
  ANR_CHECK_LAUNCH("anr_adam_step_multi_dev (tick)");
  int32_t t = 0;
  while (t < n_tensors) {
    AdamTensorsDev a;
    memset(&a, 0, sizeof(a));
    int64_t blocks = 0;
    for (; t < n_tensors && a.count < ANR_ADAM_MAX_TENSORS; ++t) {
      const anr_adam_tensor& d = tensors[t];
      if (d.n == 0) continue;
      const int c = a.count++;
      a.p[c] = d.params;
      a.g[c] = d.grad;
      a.m[c] = d.exp_avg;
      a.v[c] = d.exp_avg_sq;
      a.p16[c] = static_cast<__half*>(d.params_f16);
      a.n[c] = d.n;
      a.wd[c] = d.weight_decay;
      a.gq[c] = d.grad_quant;
      a.idx[c] = t;
      a.first[c] = static_cast<int>(blocks);
      blocks += ceil_div(d.n, 1024);
      ANR_CHECK_ARG(blocks < (int64_t(1) << 31), "anr_adam_step_multi_dev: too many elements");
    }
    if (a.count == 0) continue;
    a.first[a.count] = static_cast<int>(blocks);
    hipLaunchKernelGGL(adam_multi_dev_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       as_stream(stream), a, d_scratch, beta1, beta2, eps, decoupled,
                       zero_grad);
    ANR_CHECK_LAUNCH("anr_adam_step_multi_dev");
  }
  return ANR_OK;
}
