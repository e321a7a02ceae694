// K9: losses of src/atmonr/losses.py:5-33 applied as in
// src/atmonr/pipelines/instant_ngp.py:249-263:
//   pred = take_along_dim(color_map, irgb_idx[:, None], 1)[:, 0];  gt = rad.to(pred.dtype)
//   mse_plus_hdr = mean((p/m - g/m)^2) + 0.2 * mean((log(g + 1e-3 m) - log(p + 1e-3 m))^2)
// The loss is a batch mean, so dL/dpred of each ray depends only on that ray: the kernel
// writes the gradient and per-block partial sums in one pass; a 1-block finalize sums the
// partials (deterministic order) into the scalar loss.

#include "anr_common.h"

namespace anr {

struct LossTerms {
  float t1, t2, g;  // first term, hdr term (before the mean), dL/dp (before the 1/B)
};

__device__ __forceinline__ LossTerms loss_terms(int type, float p, float g, float m) {
  const float eps = 1e-3f * m;
  LossTerms r{0.0f, 0.0f, 0.0f};
  auto hdr = [&](float& t, float& gr) {
    const float lg = logf(g + eps), lp = logf(p + eps);
    t = (lg - lp) * (lg - lp);
    gr = 2.0f * (lp - lg) / (p + eps);
  };
  switch (type) {
    case ANR_LOSS_DARK: {  // ((p - g) / (p.detach() + eps))^2
      const float den = p + eps;
      const float q = (p - g) / den;
      r.t1 = q * q;
      r.g = 2.0f * q / den;
      break;
    }
    case ANR_LOSS_HDR: {
      float gr;
      hdr(r.t1, gr);
      r.g = gr;
      break;
    }
    case ANR_LOSS_L1:
    case ANR_LOSS_L1_PLUS_HDR: {
      const float d = p / m - g / m;
      r.t1 = fabsf(d);
      r.g = (d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f)) / m;
      if (type == ANR_LOSS_L1_PLUS_HDR) {
        float gr;
        hdr(r.t2, gr);
        r.g += 0.2f * gr;
      }
      break;
    }
    default: {  // MSE, MSE_PLUS_HDR
      const float d = p / m - g / m;
      r.t1 = d * d;
      r.g = 2.0f * d / m;
      if (type == ANR_LOSS_MSE_PLUS_HDR) {
        float gr;
        hdr(r.t2, gr);
        r.g += 0.2f * gr;
      }
      break;
    }
  }
  return r;
}

__global__ void __launch_bounds__(256) loss_kernel(int type, const void* cmap, int pdt, int C,
                                                   const int64_t* __restrict__ idx,
                                                   const float* __restrict__ gt, int64_t B,
                                                   float m, float grad_scale, void* grad,
                                                   float* __restrict__ partial) {
  __shared__ float s1[4], s2[4];
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float t1 = 0.0f, t2 = 0.0f;
  if (b < B) {
    const int64_t k = idx[b];
    const float p = load_dyn(cmap, pdt, b * C + k);
    float g = gt[b];
    if (pdt == ANR_F16) g = __half2float(__float2half_rn(g));  // rad.to(pred.dtype)
    const LossTerms r = loss_terms(type, p, g, m);
    t1 = r.t1;
    t2 = r.t2;
    if (grad) {
      const float gb = r.g * grad_scale / static_cast<float>(B);
      for (int c = 0; c < C; ++c) store_dyn(grad, pdt, b * C + c, c == k ? gb : 0.0f);
    }
  }
  t1 = wave_sum(t1);
  t2 = wave_sum(t2);
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    s1[w] = t1;
    s2[w] = t2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a1 = 0.0f, a2 = 0.0f;
    for (int i = 0; i < static_cast<int>(blockDim.x / 64); ++i) {
      a1 += s1[i];
      a2 += s2[i];
    }
    partial[2 * blockIdx.x] = a1;
    partial[2 * blockIdx.x + 1] = a2;
  }
}

__global__ void __launch_bounds__(256) loss_finalize_kernel(int type, const float* partial,
                                                            int nblk, int64_t B,
                                                            float* loss) {
  __shared__ float s1[4], s2[4];
  float a1 = 0.0f, a2 = 0.0f;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    a1 += partial[2 * i];
    a2 += partial[2 * i + 1];
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if ((threadIdx.x & 63) == 0) {
    s1[threadIdx.x / 64] = a1;
    s2[threadIdx.x / 64] = a2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t1 = (s1[0] + s1[1] + s1[2] + s1[3]) / static_cast<float>(B);
    const float t2 = (s2[0] + s2[1] + s2[2] + s2[3]) / static_cast<float>(B);
    const bool has_hdr2 = type == ANR_LOSS_L1_PLUS_HDR || type == ANR_LOSS_MSE_PLUS_HDR;
    *loss = has_hdr2 ? t1 + 0.2f * t2 : t1;
  }
}

}  // namespace anr

extern "C" int64_t anr_loss_workspace_bytes(int64_t B) {
  return 2 * sizeof(float) * anr::ceil_div(B > 0 ? B : 1, 256);
}

extern "C" int anr_loss_fwd_bwd(int32_t loss_type, const void* color_map, int32_t pred_dtype,
                                int32_t C, const int64_t* irgb_idx, const float* gt,
                                int64_t B, float max_i, float grad_scale, float* loss_out,
                                void* grad_out, void* workspace, anr_stream_t stream) {
  using namespace anr;
  ANR_CHECK_ARG(color_map && irgb_idx && gt && loss_out && workspace,
                "anr_loss_fwd_bwd: null argument");
  ANR_CHECK_ARG(loss_type >= ANR_LOSS_DARK && loss_type <= ANR_LOSS_MSE_PLUS_HDR,
                "anr_loss_fwd_bwd: unknown loss %d", loss_type);
  ANR_CHECK_ARG(B >= 1 && C >= 1, "anr_loss_fwd_bwd: bad shape");
  ANR_CHECK_ARG(pred_dtype == ANR_F16 || pred_dtype == ANR_F32, "anr_loss_fwd_bwd: bad dtype");
  const int nblk = static_cast<int>(ceil_div(B, 256));
  float* partial = static_cast<float*>(workspace);
  hipLaunchKernelGGL(loss_kernel, dim3(nblk), dim3(256), 0, as_stream(stream), loss_type,
                     color_map, pred_dtype, C, irgb_idx, gt, B, max_i, grad_scale, grad_out,
                     partial);
  ANR_CHECK_LAUNCH("anr_loss_fwd_bwd");
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, as_stream(stream),
                     loss_type, partial, nblk, B, loss_out);
  ANR_CHECK_LAUNCH("anr_loss_fwd_bwd(finalize)");
  return ANR_OK;
}
