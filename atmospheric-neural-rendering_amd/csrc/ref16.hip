// Reference-numerics mode: the reference's f16 composite and loss, and tcnn's loss-scaled
// f16 parameter gradients, reproduced op by op on the GPU.
//
// In the reference's Instant-NGP path every tinycudann module returns f16, so
// render_with_surface (src/atmonr/graphics_utils.py:6-77) and the loss
// (src/atmonr/pipelines/instant_ngp.py:259-263, src/atmonr/losses.py:5-33) are chains of
// torch f16 ops, differentiated by autograd with more f16 ops. Each op computes in f32 and
// stores f16 (round to nearest even); the accumulating ops follow torch's CUDA kernels:
// cumprod and the reversed cumsum of its backward keep an f16 accumulator (ATen
// ScanUtils.cuh, outer-dimension scan), sum and prod accumulate in f32. The restatement
// these kernels follow, with every rounding point, is oracle/ref_f16.py
// (tests/test_ref16_gpu.py holds them bit-exact to it).
//
// The default build (composite.hip, loss.hip) keeps the composite and the loss in f32;
// these kernels are the opt-in "reference numerics" of InstantNGPPipeline
// (numerics="reference"), used to show PSNR parity with the reference's own f16 path.
// One wavefront per ray: the per-sample ops run across lanes, the sequential f16 / f32
// accumulations (which have no parallel form that rounds the same way) as serial scans
// of one lane over LDS.
#pragma clang fp contract(off)

#include "anr_common.h"

namespace anr {
namespace ref16 {

constexpr int kMaxC = 8;

__device__ __forceinline__ float h(float x) { return __half2float(__float2half_rn(x)); }

// f64 -> f16 with ONE rounding (round to odd into f32, then nearest-even into f16: the
// f32 intermediate has 13 more bits than f16, so the double rounding is exact)
__device__ __forceinline__ float h64(double d) {
  float f = static_cast<float>(d);
  if (static_cast<double>(f) != d && f != 0.0f && isfinite(f)) {
    uint32_t u = __float_as_uint(f);
    if (fabs(static_cast<double>(f)) > fabs(d)) u -= 1;  // rounded away from zero: truncate
    f = __uint_as_float(u | 1u);
  }
  return h(f);
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i) { return to_f32<T>(p[i]); }

// z_vals (f32) * scale -> f16 (graphics_utils.py:28)
__device__ __forceinline__ float zh(const float* zr, float zs, int i) { return h(zr[i] * zs); }

// delta_i = diff([0, (z_0 + z_1) / 2, ..., (z_{N-2} + z_{N-1}) / 2, z_{N-1}])_i in f16
// (graphics_utils.py:31-35)
__device__ __forceinline__ float delta_ref(const float* zr, float zs, int i, int N) {
  const float zi = zh(zr, zs, i);
  const float lo = i == 0 ? h(zi * 0.0f) : h(h(zh(zr, zs, i - 1) + zi) * 0.5f);
  const float hi = i == N - 1 ? zi : h(h(zi + zh(zr, zs, i + 1)) * 0.5f);
  return h(hi - lo);
}

struct Sample {
  float delta, e, alpha, q2;  // q2 = 1 - alpha + 1e-10 (= om = 1 - alpha in f16)
};

__device__ __forceinline__ Sample sample(float sig, float dl) {
  Sample s;
  s.delta = dl;
  const float x = h(-sig * dl);                       // -sigma * delta   (:38)
  s.e = h64(exp(static_cast<double>(x)));             // exp
  s.alpha = h(1.0f - s.e);                            // 1 - exp
  s.q2 = h(h(1.0f - s.alpha) + 1e-10f);               // 1 - alpha + 1e-10 (:45)
  return s;
}

// One wavefront per ray (block = 64 threads), samples in segments of kSeg. Each segment
// splits into lane-parallel phases (the per-sample f16 ops: delta, exp, alpha, weights,
// the colour products) and serial scans run by one lane over LDS (the f16 cumprod, the
// f32 product and sums, the f16 reversed cumsum of the backward) -- exactly the
// accumulations that have no parallel form rounding the same way. Every value is formed
// by the same expression as in the one-thread-per-ray r03 kernels, so the outputs are
// unchanged bit for bit; r03 ran everything serially from HBM, one ray per thread
// (1.5 ms forward / 3.3 ms backward at 8,192 x 1,024, latency-bound).
constexpr int kSeg = 256;  // samples per segment: 4 per lane

// Every staged value is an f16 value (the outputs of h()), so LDS holds them as f16. The
// serial cumprod / reversed cumsum steps run in native f16 arithmetic: the f32 product of
// two f16 values is exact, and their f32 sum rounds only where the smaller operand is
// below a quarter f16 ulp of the larger (both forms then return the larger), so one IEEE
// f16 multiply / add rounds exactly as h(a * b) / h(a + b) -- one dependent instruction
// per step of the chain instead of three.
struct FwdLds {
  // padded past a segment's n samples with the chain's neutral elements, so the serial
  // scans run in whole 8-sample (16-B) LDS vectors: q2 = 1 (cp * 1, pr * 1 exact), t = -0
  // (x + -0 == x for every x, signed zeros included)
  __attribute__((aligned(16))) _Float16 q2[kSeg];
  __attribute__((aligned(16))) _Float16 alpha[kSeg];
  __attribute__((aligned(16))) _Float16 T[kSeg];
  __attribute__((aligned(16))) _Float16 t[kMaxC][kSeg];  // f16(f16(color) * w) per band
};
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
constexpr float kNegZero = -0.0f;

template <typename T>
__global__ void __launch_bounds__(64) fwd_kernel(const float* __restrict__ z, float zs,
                                                 const T* __restrict__ color,
                                                 const T* __restrict__ sigma,
                                                 const T* __restrict__ cs, int64_t B, int N,
                                                 int C, __half* cmap, __half* atmo_out,
                                                 __half* surf_out, __half* weights,
                                                 __half* alpha_out, __half* color16,
                                                 __half* sigma16) {
  __shared__ FwdLds L;
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const float* zr = z + b * N;
  _Float16 cp = 1.0f;  // cumprod output, f16 accumulator (cuda scan); lane 0
  float pr = 1.0f;     // prod over samples, f32 accumulator; lane 0
  float acc = 0.0f;    // lane c < C: band c's sum over samples, f32 accumulator
  for (int s0 = 0; s0 < N; s0 += kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    for (int li = lane; li < nv; li += 64) {
      if (li < n) {
        const float sg = h(ld(sigma, b * N + s0 + li));
        if (sigma16) sigma16[b * N + s0 + li] = __float2half_rn(sg);
        const Sample sm = sample(sg, delta_ref(zr, zs, s0 + li, N));
        L.q2[li] = static_cast<_Float16>(sm.q2);
        L.alpha[li] = static_cast<_Float16>(sm.alpha);
      } else {
        L.q2[li] = static_cast<_Float16>(1.0f);
      }
    }
    __syncthreads();
    if (lane == 0) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v q = *reinterpret_cast<const h8v*>(&L.q2[l8]);
        h8v tv;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          tv[k] = cp;                                   // cumprod(...)[:, :-1]
          cp = cp * q[k];                               // = h(cp * q2)
          pr = pr * static_cast<float>(q[k]);           // (1 - alpha).prod   (:75)
        }
        *reinterpret_cast<h8v*>(&L.T[l8]) = tv;
      }
    }
    __syncthreads();
    for (int li = lane; li < nv; li += 64) {
      if (li < n) {
        const int64_t i = b * N + s0 + li;
        const float al = static_cast<float>(L.alpha[li]);
        const float w = h(al * static_cast<float>(L.T[li]));   // alpha * T    (:43-46)
        for (int c = 0; c < C; ++c) {
          const float col = h(ld(color, i * C + c));
          if (color16) color16[i * C + c] = __float2half_rn(col);
          L.t[c][li] = static_cast<_Float16>(h(col * w));  // (:48)
        }
        if (weights) weights[i] = __float2half_rn(w);
        if (alpha_out) alpha_out[i] = __float2half_rn(al);
      } else {
        for (int c = 0; c < C; ++c) L.t[c][li] = static_cast<_Float16>(kNegZero);
      }
    }
    __syncthreads();
    if (lane < C) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v tv = *reinterpret_cast<const h8v*>(&L.t[lane][l8]);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = acc + static_cast<float>(tv[k]);
      }
    }
    __syncthreads();
  }
  pr = h(__shfl(pr, 0));
  if (lane < C) {
    const int c = lane;
    const float atmo = h(acc);
    const float surf = cs ? h(pr * h(ld(cs, b * C + c))) : 0.0f;
    cmap[b * C + c] = __float2half_rn(cs ? h(atmo + surf) : atmo);          // (:76)
    if (atmo_out) atmo_out[b * C + c] = __float2half_rn(atmo);
    if (surf_out && cs) surf_out[b * C + c] = __float2half_rn(surf);
  }
}

// Autograd of fwd_kernel for dL/dcolor_map (oracle/ref_f16.py render_bwd). d_sigma
// (one value per sample) doubles as the scratch holding the forward's cumprod outputs T_i,
// read back in the reverse pass before the gradient overwrites them. Same wave-per-ray
// phases as fwd_kernel: pass 1 replays the cumprod; pass 2 walks the segments from the
// last, with the reversed cumsum (rc) as the one serial scan.
struct BwdLds {
  // padded as FwdLds: q2 = 1, u = -0 past a segment's n samples
  __attribute__((aligned(16))) _Float16 q2[kSeg];
  __attribute__((aligned(16))) _Float16 u[kSeg];    // pass 1: T_k; pass 2: f16(T_k * dL/dT_k)
  __attribute__((aligned(16))) _Float16 rin[kSeg];  // rc before sample k's term
};

template <typename T, typename G>
__global__ void __launch_bounds__(64) bwd_kernel(const float* __restrict__ z, float zs,
                                                 const T* __restrict__ color,
                                                 const T* __restrict__ sigma,
                                                 const T* __restrict__ cs, int64_t B, int N,
                                                 int C, const __half* __restrict__ g_cm,
                                                 G* d_color, G* d_sigma, G* d_cs,
                                                 int* zero_rays) {
  __shared__ BwdLds L;
  constexpr int J = kSeg / 64;
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const float* zr = z + b * N;
  float g[kMaxC], csv[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    g[c] = c < C ? __half2float(g_cm[b * C + c]) : 0.0f;
    csv[c] = (c < C && cs) ? h(ld(cs, b * C + c)) : 0.0f;
  }
  // pass 1: the forward's cumprod outputs (scratch) and the surface product
  _Float16 cp = 1.0f;
  float pr = 1.0f;
  bool zero = false;
  for (int s0 = 0; s0 < N; s0 += kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    for (int li = lane; li < nv; li += 64) {
      if (li < n) {
        const Sample sm = sample(h(ld(sigma, b * N + s0 + li)), delta_ref(zr, zs, s0 + li, N));
        L.q2[li] = static_cast<_Float16>(sm.q2);
        zero = zero || sm.q2 == 0.0f;
      } else {
        L.q2[li] = static_cast<_Float16>(1.0f);
      }
    }
    __syncthreads();
    if (lane == 0) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v q = *reinterpret_cast<const h8v*>(&L.q2[l8]);
        h8v tv;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          tv[k] = cp;  // T_i, staged for the coalesced scratch store below
          cp = cp * q[k];  // = h(cp * q2)
          pr = pr * static_cast<float>(q[k]);
        }
        *reinterpret_cast<h8v*>(&L.u[l8]) = tv;
      }
    }
    __syncthreads();
    for (int li = lane; li < n; li += 64)
      d_sigma[b * N + s0 + li] = static_cast<G>(static_cast<float>(L.u[li]));
    __syncthreads();
  }
  pr = h(__shfl(pr, 0));
  zero = __any(zero);
  // surface term: surf = pr * cs -> dL/dpr (sum over bands), dL/dcs
  float g_pr = 0.0f;
  if (cs) {
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
      if (c < C) {
        g_pr = g_pr + h(g[c] * csv[c]);
        if (d_cs && lane == 0) d_cs[b * C + c] = static_cast<G>(h(g[c] * pr));
      }
    g_pr = h(g_pr);
  }
  if (zero) {
    // alpha rounded to 1 in f16 (sigma * delta > ~9): torch takes its zero-input backward
    // branches (prod_safe_zeros_backward, cumprod's first-zero formula) -- not restated
    // rounding for rounding; flagged to the caller, gradients of this ray set to 0
    if (lane == 0) atomicAdd(zero_rays, 1);
    for (int i = lane; i < N; i += 64) {
      d_sigma[b * N + i] = static_cast<G>(0.0f);
      for (int c = 0; c < C; ++c) d_color[(b * N + i) * C + c] = static_cast<G>(0.0f);
    }
    return;
  }
  // pass 2, reverse: reversed cumsum of cp * dL/dcp with an f16 accumulator
  // (cumprod_backward), then each sample's gradients in autograd's order
  _Float16 rc = 0.0f;  // reversed cumsum at j = N: cp_N * 0 (lane 0)
  for (int s0 = ((N - 1) / kSeg) * kSeg; s0 >= 0; s0 -= kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    float e_[J], dl_[J], q2_[J], gab_[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int li = lane + 64 * j;
      if (li >= n) {
        if (li < nv) L.u[li] = static_cast<_Float16>(kNegZero);
        continue;
      }
      const int64_t k = b * N + s0 + li;
      const float sig = h(ld(sigma, k));
      const Sample sm = sample(sig, delta_ref(zr, zs, s0 + li, N));
      const float Tk = static_cast<float>(d_sigma[k]);
      const float w = h(sm.alpha * Tk);
      float gw = 0.0f;
      for (int c = 0; c < C; ++c) {
        const float col = h(ld(color, k * C + c));
        gw = gw + h(g[c] * col);                                  // sum_to_size over bands
        d_color[k * C + c] = static_cast<G>(h(g[c] * w));         // color * w -> color
      }
      gw = h(gw);
      gab_[j] = h(gw * Tk);                                       // alpha * T -> alpha
      const float g_T = h(gw * sm.alpha);                         // -> T
      L.u[li] = static_cast<_Float16>(h(Tk * g_T));               // cp_k * dL/dcp_k
      e_[j] = sm.e;
      dl_[j] = sm.delta;
      q2_[j] = sm.q2;
    }
    __syncthreads();
    if (lane == 0) {
      for (int l8 = nv - 8; l8 >= 0; l8 -= 8) {
        const h8v uv = *reinterpret_cast<const h8v*>(&L.u[l8]);
        h8v rv;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
          rv[k] = rc;
          rc = rc + uv[k];  // = h(rc + u)
        }
        *reinterpret_cast<h8v*>(&L.rin[l8]) = rv;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int li = lane + 64 * j;
      if (li >= n) continue;
      const float g_cpin = h(static_cast<float>(L.rin[li]) / q2_[j]);  // cumprod bwd at k+1
      const float g_alpha_c = -g_cpin;                            // 1 - alpha + 1e-10
      float g_alpha;
      if (cs) {
        const float g_om = h(g_pr * h(pr / q2_[j]));              // prod backward
        g_alpha = h(h(-g_om + gab_[j]) + g_alpha_c);
      } else {
        g_alpha = h(gab_[j] + g_alpha_c);
      }
      const float g_x = h(-g_alpha * e_[j]);                      // 1 - exp(x)
      d_sigma[b * N + s0 + li] = static_cast<G>(-h(g_x * dl_[j]));   // -sigma * delta
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ losses (f16 ops)
struct LossOut {
  float t1, t2, g;  // per-ray terms of the two means (f16 values), dL/dpred (f16 value)
};

// losses.py:5-33 for one ray, f16 semantics of oracle/ref_f16.py loss_f16 (acc="cuda")
__device__ LossOut loss_ray(int type, float p, float gt, float inv, float eps, float norm,
                            float inv_n) {
  LossOut r{0.0f, 0.0f, 0.0f};
  const float c02 = h(0.2f);
  auto mse = [&](float a, float b, float gout, float& t, float& ga) {
    const float d = h(a - b);
    t = h(d * d);
    ga = h(h(norm * d) * gout);
  };
  auto l1 = [&](float a, float b, float gout, float& t, float& ga) {
    const float d = h(a - b);
    t = fabsf(d);
    const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
    ga = h(h(sg * gout) * h(inv_n));
  };
  auto hdr = [&](float gout, float& t, float& gp) {
    const float xg = h(gt + eps), xp = h(p + eps);
    const float la = h64(log(static_cast<double>(xg))), lb = h64(log(static_cast<double>(xp)));
    const float d = h(la - lb);
    t = h(d * d);
    const float g_lb = h(h(norm * h(lb - la)) * gout);
    gp = h(g_lb / xp);
  };
  switch (type) {
    case ANR_LOSS_MSE:
    case ANR_LOSS_L1: {
      const float a = h(p * inv), b = h(gt * inv);
      float ga;
      if (type == ANR_LOSS_MSE) mse(a, b, 1.0f, r.t1, ga); else l1(a, b, 1.0f, r.t1, ga);
      r.g = h(ga * inv);
      break;
    }
    case ANR_LOSS_HDR:
      hdr(1.0f, r.t1, r.g);
      break;
    case ANR_LOSS_MSE_PLUS_HDR:
    case ANR_LOSS_L1_PLUS_HDR: {
      const float a = h(p * inv), b = h(gt * inv);
      float ga, gp2;
      if (type == ANR_LOSS_MSE_PLUS_HDR) mse(a, b, 1.0f, r.t1, ga); else l1(a, b, 1.0f, r.t1, ga);
      hdr(c02, r.t2, gp2);
      r.g = h(h(ga * inv) + gp2);
      break;
    }
    default: {  // DARK: (((p - g) / (p.detach() + eps)) ** 2).mean()
      const float den = h(p + eps);
      const float q = h(h(p - gt) / den);
      r.t1 = h(q * q);
      r.g = h(h(h(2.0f * q) * h(inv_n)) / den);
      break;
    }
  }
  return r;
}

__global__ void __launch_bounds__(256) loss_kernel(int type, const __half* __restrict__ cmap,
                                                   int C, const int64_t* __restrict__ idx,
                                                   const float* __restrict__ gt, int64_t B,
                                                   float inv, float eps, float norm, float inv_n,
                                                   __half* grad, float* __restrict__ partial) {
  __shared__ float s1[4], s2[4];
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float t1 = 0.0f, t2 = 0.0f;
  if (b < B) {
    const int64_t k = idx[b];
    const float p = __half2float(cmap[b * C + k]);
    const float g = h(gt[b]);  // rad.to(pred.dtype)  (instant_ngp.py:262)
    const LossOut r = loss_ray(type, p, g, inv, eps, norm, inv_n);
    t1 = r.t1;
    t2 = r.t2;
    if (grad)
      for (int c = 0; c < C; ++c) grad[b * C + c] = __float2half_rn(c == k ? r.g : 0.0f);
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
    partial[2 * blockIdx.x] = s1[0] + s1[1] + s1[2] + s1[3];
    partial[2 * blockIdx.x + 1] = s2[0] + s2[1] + s2[2] + s2[3];
  }
}

__global__ void __launch_bounds__(64) loss_finalize_kernel(int type, const float* partial,
                                                           int nblk, int64_t B, float* loss) {
  float a1 = 0.0f, a2 = 0.0f;
  for (int i = threadIdx.x; i < nblk; i += 64) {
    a1 += partial[2 * i];
    a2 += partial[2 * i + 1];
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if (threadIdx.x == 0) {
    // means in f32 then f16; the two-term losses as v1 + f16(0.2 * v2) in f16
    const float v1 = h(a1 / static_cast<float>(B)), v2 = h(a2 / static_cast<float>(B));
    const bool two = type == ANR_LOSS_L1_PLUS_HDR || type == ANR_LOSS_MSE_PLUS_HDR;
    *loss = two ? h(v1 + h(v2 * 0.2f)) : v1;
  }
}

// tcnn's parameter gradient: f16(f16(g * s) / s) -- the module's f16 gradient at loss scale
// s, divided by s in f16 (tinycudann/modules.py, _module_function_backward)
__global__ void __launch_bounds__(256) quantize_kernel(float* __restrict__ g, int64_t n,
                                                       float s, float inv_s) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += stride)
    g[i] = h(h(g[i] * s) * inv_s);
}

}  // namespace ref16
}  // namespace anr

using namespace anr;

extern "C" int anr_composite_ref16_fwd(const float* z, float z_scale, const void* color,
                                       const void* sigma, const void* color_surf,
                                       int32_t in_dtype, int64_t B, int32_t N, int32_t C,
                                       void* color_map, void* color_map_atmo,
                                       void* color_map_surf, void* weights, void* alpha,
                                       void* color16, void* sigma16, anr_stream_t stream) {
  ANR_CHECK_ARG(z && color && sigma && color_map, "anr_composite_ref16_fwd: null argument");
  ANR_CHECK_ARG(B >= 0 && N >= 1 && C >= 1 && C <= ref16::kMaxC,
                "anr_composite_ref16_fwd: bad shape B=%lld N=%d C=%d", (long long)B, N, C);
  ANR_CHECK_ARG(in_dtype == ANR_F16 || in_dtype == ANR_F32, "anr_composite_ref16_fwd: bad dtype");
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(B < (1LL << 31), "anr_composite_ref16_fwd: B=%lld too large", (long long)B);
  const dim3 grid(static_cast<unsigned>(B)), block(64);
#define ANR_R16F(T)                                                                           \
  hipLaunchKernelGGL(ref16::fwd_kernel<T>, grid, block, 0, as_stream(stream), z, z_scale,    \
                     static_cast<const T*>(color), static_cast<const T*>(sigma),               \
                     static_cast<const T*>(color_surf), B, N, C,                              \
                     static_cast<__half*>(color_map), static_cast<__half*>(color_map_atmo),  \
                     static_cast<__half*>(color_map_surf), static_cast<__half*>(weights),     \
                     static_cast<__half*>(alpha), static_cast<__half*>(color16),              \
                     static_cast<__half*>(sigma16))
  if (in_dtype == ANR_F16) ANR_R16F(__half); else ANR_R16F(float);
#undef ANR_R16F
  ANR_CHECK_LAUNCH("anr_composite_ref16_fwd");
  return ANR_OK;
}

extern "C" int anr_composite_ref16_bwd(const float* z, float z_scale, const void* color,
                                       const void* sigma, const void* color_surf,
                                       int32_t in_dtype, int64_t B, int32_t N, int32_t C,
                                       const void* d_color_map, void* d_color, void* d_sigma,
                                       void* d_color_surf, int32_t out_dtype, int32_t* zero_rays,
                                       anr_stream_t stream) {
  ANR_CHECK_ARG(z && color && sigma && d_color_map && d_color && d_sigma && zero_rays,
                "anr_composite_ref16_bwd: null argument");
  ANR_CHECK_ARG(B >= 0 && N >= 1 && C >= 1 && C <= ref16::kMaxC,
                "anr_composite_ref16_bwd: bad shape");
  ANR_CHECK_ARG(in_dtype == ANR_F16 || in_dtype == ANR_F32, "anr_composite_ref16_bwd: bad dtype");
  ANR_CHECK_ARG(out_dtype == ANR_F16 || out_dtype == ANR_F32,
                "anr_composite_ref16_bwd: bad output dtype");
  ANR_CHECK_ARG(d_color_surf == nullptr || color_surf != nullptr,
                "anr_composite_ref16_bwd: d_color_surf without color_surf");
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(B < (1LL << 31), "anr_composite_ref16_bwd: B=%lld too large", (long long)B);
  const dim3 grid(static_cast<unsigned>(B)), block(64);
#define ANR_R16B(T, G)                                                                        \
  hipLaunchKernelGGL((ref16::bwd_kernel<T, G>), grid, block, 0, as_stream(stream), z, z_scale, \
                     static_cast<const T*>(color), static_cast<const T*>(sigma),               \
                     static_cast<const T*>(color_surf), B, N, C,                              \
                     static_cast<const __half*>(d_color_map), static_cast<G*>(d_color),       \
                     static_cast<G*>(d_sigma), static_cast<G*>(d_color_surf), zero_rays)
  if (in_dtype == ANR_F16) {
    if (out_dtype == ANR_F16) ANR_R16B(__half, __half); else ANR_R16B(__half, float);
  } else {
    if (out_dtype == ANR_F16) ANR_R16B(float, __half); else ANR_R16B(float, float);
  }
#undef ANR_R16B
  ANR_CHECK_LAUNCH("anr_composite_ref16_bwd");
  return ANR_OK;
}

extern "C" int anr_loss_ref16_fwd_bwd(int32_t loss_type, const void* color_map, int32_t C,
                                      const int64_t* irgb_idx, const float* gt, int64_t B,
                                      float max_i, float* loss_out, void* grad_out,
                                      void* workspace, anr_stream_t stream) {
  ANR_CHECK_ARG(color_map && irgb_idx && gt && loss_out && workspace,
                "anr_loss_ref16_fwd_bwd: null argument");
  ANR_CHECK_ARG(loss_type >= ANR_LOSS_DARK && loss_type <= ANR_LOSS_MSE_PLUS_HDR,
                "anr_loss_ref16_fwd_bwd: unknown loss %d", loss_type);
  ANR_CHECK_ARG(B >= 1 && C >= 1, "anr_loss_ref16_fwd_bwd: bad shape");
  const int nblk = static_cast<int>(ceil_div(B, 256));
  // scalars as torch forms them: x / max_i = x * (1 / max_i) in f32, the Python scalar
  // 1e-3 * max_i in f32, mse_loss's 2 / numel and mean's 1 / numel as f16
  const float inv = 1.0f / max_i;
  const float eps = static_cast<float>(1e-3 * static_cast<double>(max_i));
  const float norm = __half2float(__float2half_rn(static_cast<float>(2.0 / static_cast<double>(B))));
  const float inv_n = static_cast<float>(1.0 / static_cast<double>(B));
  hipLaunchKernelGGL(ref16::loss_kernel, dim3(nblk), dim3(256), 0, as_stream(stream), loss_type,
                     static_cast<const __half*>(color_map), C, irgb_idx, gt, B, inv, eps, norm,
                     inv_n, static_cast<__half*>(grad_out), static_cast<float*>(workspace));
  ANR_CHECK_LAUNCH("anr_loss_ref16_fwd_bwd");
  hipLaunchKernelGGL(ref16::loss_finalize_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                     loss_type, static_cast<const float*>(workspace), nblk, B, loss_out);
  ANR_CHECK_LAUNCH("anr_loss_ref16_fwd_bwd(finalize)");
  return ANR_OK;
}

extern "C" int anr_grad_quantize_f16(float* grad, int64_t n, float loss_scale,
                                     anr_stream_t stream) {
  ANR_CHECK_ARG(grad != nullptr || n == 0, "anr_grad_quantize_f16: null argument");
  ANR_CHECK_ARG(n >= 0 && loss_scale > 0.0f, "anr_grad_quantize_f16: bad argument");
  if (n == 0) return ANR_OK;
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(ref16::quantize_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     as_stream(stream), grad, n, loss_scale, 1.0f / loss_scale);
  ANR_CHECK_LAUNCH("anr_grad_quantize_f16");
  return ANR_OK;
}
