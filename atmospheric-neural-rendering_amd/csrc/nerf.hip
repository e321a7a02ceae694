// NeRF path (configs/nerf.json): positional encoding and the
// hierarchical (pdf) sampler, forward and backward.
//
//   positional_encoding  src/atmonr/encoders.py:4-28
//   sample_pdf           src/atmonr/samplers.py:50-103
//
// Both follow the reference's f32 operation order (no FMA contraction) so that values
// match it to rounding; sample_pdf's cdf accumulates in f64 and rounds each entry to f32,
// which is what the reference's torch.cumsum does on the CPU the golden vectors come from
// (SURVEY §8 a14), so searchsorted indices match it.

#pragma clang fp contract(off)

#include "anr_common.h"

namespace anr {
namespace nerf {

constexpr float kPiF = 3.14159265358979323846f;  // torch.pi as an f32 tensor factor

struct PE {
  int n_dims, interleaved, width;
  int L[ANR_POSENC_MAX_DIMS];
  int col0[ANR_POSENC_MAX_DIMS];  // first output column of each input coordinate
};

static bool make_pe(const anr_posenc_desc* d, PE* p) {
  if (d->n_dims < 1 || d->n_dims > ANR_POSENC_MAX_DIMS) return false;
  p->n_dims = d->n_dims;
  p->interleaved = d->interleaved ? 1 : 0;
  int w = 0;
  for (int i = 0; i < d->n_dims; ++i) {
    const int L = d->interleaved ? d->L[0] : d->L[i];
    if (L < 1 || L > 30) return false;
    p->L[i] = L;
    p->col0[i] = w;
    w += 2 * L;
  }
  p->width = w;
  return true;
}

// output column -> (coordinate i, frequency l, cos?)
__device__ __forceinline__ void pe_col(const PE& p, int col, int* i, int* l, bool* is_cos) {
  int k = 0;
#pragma unroll 1
  while (k + 1 < p.n_dims && col >= p.col0[k + 1]) ++k;
  const int r = col - p.col0[k];
  *i = k;
  if (p.interleaved) {  // [sin f0, cos f0, sin f1, cos f1, ...]   (encoders.py:13-19)
    *l = r >> 1;
    *is_cos = r & 1;
  } else {              // [sin f0 .. f(L-1), cos f0 .. f(L-1)]    (encoders.py:20-26)
    *l = r < p.L[k] ? r : r - p.L[k];
    *is_cos = r >= p.L[k];
  }
}

// (2^l * pi) in f32 times x in f32, as `(2**l_ls * torch.pi) * pts`
__device__ __forceinline__ float pe_arg(int l, float x) { return ldexpf(kPiF, l) * x; }

__global__ void __launch_bounds__(256) posenc_fwd_kernel(PE p, const float* __restrict__ x,
                                                         int64_t rows_per_x, int64_t P,
                                                         float* __restrict__ out,
                                                         int64_t out_stride) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= P * p.width) return;
  const int64_t row = idx / p.width;
  const int col = static_cast<int>(idx - row * p.width);
  int i, l;
  bool c;
  pe_col(p, col, &i, &l, &c);
  const float a = pe_arg(l, x[(row / rows_per_x) * p.n_dims + i]);
  out[row * out_stride + col] = c ? cosf(a) : sinf(a);
}

// dx_i = sum_l f_l * (cos(f_l x_i) * g_sin - sin(f_l x_i) * g_cos)
__global__ void __launch_bounds__(256) posenc_bwd_kernel(PE p, const float* __restrict__ x,
                                                         int64_t P, const float* __restrict__ dout,
                                                         int64_t dout_stride,
                                                         float* __restrict__ dx) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= P * p.n_dims) return;
  const int64_t row = idx / p.n_dims;
  const int i = static_cast<int>(idx - row * p.n_dims);
  const float xv = x[idx];
  const float* g = dout + row * dout_stride + p.col0[i];
  float acc = 0.0f;
  for (int l = 0; l < p.L[i]; ++l) {
    const float f = ldexpf(kPiF, l);
    const float a = f * xv;
    const float gs = p.interleaved ? g[2 * l] : g[l];
    const float gc = p.interleaved ? g[2 * l + 1] : g[p.L[i] + l];
    acc += f * (cosf(a) * gs) - f * (sinf(a) * gc);
  }
  dx[idx] = acc;
}

// --------------------------------------------------------------------------------
// sample_pdf: one wavefront per ray
// --------------------------------------------------------------------------------
struct PdfArgs {
  const float* w;   // (B, Nc, S): weights of the coarse render; channel 0 used
  int64_t w_ray;    // elements between rays
  int32_t w_samp;   // elements between samples
  const float* zc;  // (B, Nc)
  const float* u;   // (B, Nf)
  const float* origin;
  const float* dir;
  int64_t B;
  int32_t Nc, Nf;
  float* z;       // (B, Nc+Nf) sorted
  float* pts;     // (B, Nc+Nf, 3) nullable
  int32_t* src;   // (B, Nc+Nf): source of each sorted value (< Nc coarse, else Nc + k)
  int32_t* inds;  // (B, Nf): searchsorted(cdf, u, right=True)
  float* cdf;     // (B, Nc-1)
  // backward
  const float* dz;    // (B, Nc+Nf) nullable
  const float* dpts;  // (B, Nc+Nf, 3) nullable
  float* dw;          // (B, Nc, S) channel 0 written, others untouched
};

constexpr int kMaxNc = 64, kMaxNf = 256;

// Sum of p[0..n) in the order torch's CPU float sum uses for one contiguous row
// (ATen/native/cpu/SumKernel.cpp: vectorized_inner_sum over Vectorized<float> of 8 lanes,
// row_sum with ILP 4; the multi-level cascade only starts at 16·4 vectors, above kMaxNc).
// Every lane returns the same f32 value. Pinned against torch on 2000 random rows of
// 62/63/127/190 elements and the golden sample_pdf rays.
__device__ inline float torch_cpu_row_sum(const float* p, int n, int lane) {
  const int nv = n / 8, si = nv / 4;
  float col = 0.0f;
  if (lane < 8) {
    float q0 = 0.0f, q1 = 0.0f, q2 = 0.0f, q3 = 0.0f;
    for (int r = 0; r < si; ++r) {
      q0 += p[(4 * r + 0) * 8 + lane];
      q1 += p[(4 * r + 1) * 8 + lane];
      q2 += p[(4 * r + 2) * 8 + lane];
      q3 += p[(4 * r + 3) * 8 + lane];
    }
    for (int v = 4 * si; v < nv; ++v) q0 += p[v * 8 + lane];
    col = ((q0 + q1) + q2) + q3;
  }
  float s = 0.0f;
  for (int k = 8 * nv; k < n; ++k) s += p[k];
  for (int l = 0; l < 8; ++l) s += __shfl(col, l);
  return s;
}

__global__ void __launch_bounds__(64) sample_pdf_fwd_kernel(PdfArgs a) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int Nc = a.Nc, Nf = a.Nf, Nt = Nc + Nf, Ncdf = Nc - 1;
  __shared__ float cdf[kMaxNc], mid[kMaxNc], vals[kMaxNc + kMaxNf], pl[kMaxNc];
  const float* w = a.w + b * a.w_ray;
  // pdf = (w[1:-1] + 1e-8) / sum(w[1:-1] + 1e-8)   (samplers.py:71-74)
  const int np = Nc - 2;
  if (lane < np) pl[lane] = w[static_cast<int64_t>(lane + 1) * a.w_samp] + 1e-8f;
  __syncthreads();
  const float S = torch_cpu_row_sum(pl, np, lane);
  if (lane < np) pl[lane] = pl[lane] / S;
  __syncthreads();
  // cdf = cat([0], cumsum(pdf)): torch's CPU cumsum accumulates floats sequentially in
  // double and rounds each prefix to f32
  if (lane == 0) cdf[0] = 0.0f;
  if (lane < np) {
    double c = 0.0;
    for (int j = 0; j <= lane; ++j) c += static_cast<double>(pl[j]);
    cdf[lane + 1] = static_cast<float>(c);
  }
  // bin midpoints 0.5 * (z[1:] + z[:-1])   (samplers.py:85)
  const float* zc = a.zc + b * Nc;
  if (lane < Nc - 1) mid[lane] = 0.5f * (zc[lane + 1] + zc[lane]);
  if (lane < Nc) vals[lane] = zc[lane];
  __syncthreads();
  if (lane < Ncdf) a.cdf[b * Ncdf + lane] = cdf[lane];
  for (int k = lane; k < Nf; k += 64) {
    const float u = a.u[b * Nf + k];
    // searchsorted(cdf, u, right=True): number of entries <= u
    int lo = 0, hi = Ncdf;
    while (lo < hi) {
      const int md = (lo + hi) >> 1;
      if (cdf[md] <= u) lo = md + 1;
      else hi = md;
    }
    const int ind = lo;
    a.inds[b * Nf + k] = ind;
    const int below = ind - 1 > 0 ? ind - 1 : 0;
    const int above = ind < Ncdf - 1 ? ind : Ncdf - 1;
    const float c0 = cdf[below], c1 = cdf[above];
    float den = c1 - c0;
    if (den < 1e-8f) den = 1.0f;
    const float t = (u - c0) / den;
    const float b0 = mid[below], b1 = mid[above];
    vals[Nc + k] = b0 + t * (b1 - b0);
  }
  __syncthreads();
  // sort(cat(z_c, samples)): rank of each value (ties by index -> stable)
  const float* o = a.origin + b * 3;
  const float* d = a.dir + b * 3;
  for (int i = lane; i < Nt; i += 64) {
    const float v = vals[i];
    int r = 0;
    for (int j = 0; j < Nt; ++j) {
      const float x = vals[j];
      r += (x < v) || (x == v && j < i);
    }
    a.z[b * Nt + r] = v;
    a.src[b * Nt + r] = i;
    if (a.pts) {
      float* q = a.pts + (b * Nt + r) * 3;
      q[0] = o[0] + d[0] * v;
      q[1] = o[1] + d[1] * v;
      q[2] = o[2] + d[2] * v;
    }
  }
}

// Gradient of the samples w.r.t. the coarse weights, through t_in_bin (samplers.py:92-96;
// the bin width is detached, the coarse z values carry no gradient).
__global__ void __launch_bounds__(64) sample_pdf_bwd_kernel(PdfArgs a) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int Nc = a.Nc, Nf = a.Nf, Nt = Nc + Nf, Ncdf = Nc - 1, np = Nc - 2;
  __shared__ float gs[kMaxNf], mid[kMaxNc], cdf[kMaxNc];
  __shared__ double dc[kMaxNc];
  const float* zc = a.zc + b * Nc;
  if (lane < Nc - 1) mid[lane] = 0.5f * (zc[lane + 1] + zc[lane]);
  if (lane < Ncdf) cdf[lane] = a.cdf[b * Ncdf + lane];
  const float* d = a.dir + b * 3;
  // d z (sorted) incl. pts = o + d * z  ->  gradient of each sample (sort backward)
  for (int i = lane; i < Nt; i += 64) {
    float g = a.dz ? a.dz[b * Nt + i] : 0.0f;
    if (a.dpts) {
      const float* q = a.dpts + (b * Nt + i) * 3;
      g += (q[0] * d[0] + q[1] * d[1]) + q[2] * d[2];
    }
    const int s = a.src[b * Nt + i];
    if (s >= Nc) gs[s - Nc] = g;
  }
  __syncthreads();
  // dL/dcdf[j]: every sample whose below / above bin is j (deterministic order)
  if (lane < Ncdf) {
    double acc = 0.0;
    for (int k = 0; k < Nf; ++k) {
      const int ind = a.inds[b * Nf + k];
      const int below = ind - 1 > 0 ? ind - 1 : 0;
      const int above = ind < Ncdf - 1 ? ind : Ncdf - 1;
      if (below != lane && above != lane) continue;
      const float u = a.u[b * Nf + k];
      const float c0 = cdf[below], c1 = cdf[above];
      const float den_raw = c1 - c0;
      const bool ok = !(den_raw < 1e-8f);
      const double den = ok ? den_raw : 1.0;
      const double t = (static_cast<double>(u) - c0) / den;
      const double dt = static_cast<double>(gs[k]) * (mid[above] - mid[below]);
      if (below == lane) acc += ok ? dt * (t - 1.0) / den : -dt;
      if (above == lane && ok) acc += -dt * t / den;
    }
    dc[lane] = acc;
  }
  __syncthreads();
  // cumsum backward: dpdf_i = sum_{j > i} dcdf_j ; pdf = p / S backward ; dw[1 + i] = dp_i
  const float* w = a.w + b * a.w_ray;
  __shared__ float pl[kMaxNc];
  double dpdf = 0.0, p = 0.0;
  if (lane < np) {
    for (int j = lane + 1; j < Ncdf; ++j) dpdf += dc[j];
    pl[lane] = w[static_cast<int64_t>(lane + 1) * a.w_samp] + 1e-8f;
    p = static_cast<double>(pl[lane]);
  }
  __syncthreads();
  const double S = torch_cpu_row_sum(pl, np, lane);  // the forward's f32 normaliser
  double dot = dpdf * p;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) dot += __shfl_xor(dot, m);
  float* dw = a.dw + b * a.w_ray;
  if (lane < np) dw[static_cast<int64_t>(lane + 1) * a.w_samp] = static_cast<float>(dpdf / S - dot / (S * S));
  if (lane == 0) {
    dw[0] = 0.0f;
    dw[static_cast<int64_t>(Nc - 1) * a.w_samp] = 0.0f;
  }
}


// AtmoNeRF Linear+ReLU backward (models/nerf.py:48-93 under autograd): g' = g where the
// saved output y > 0, else 0 (torch's threshold_backward, exact), and the bias gradient
// sum_r g'[r, :] as per-block column partial sums in a fixed order (the caller adds the
// P partial rows), so g' is not read a second time by a separate reduction. Threads:
// C/4 column quads x (256 / (C/4)) row lanes; block b owns rows [b*R, (b+1)*R).
__global__ void __launch_bounds__(256) relu_bwd_colsum_kernel(const float* __restrict__ g,
                                                              const float* __restrict__ y,
                                                              int64_t M, int C, int64_t R,
                                                              float* __restrict__ gout,
                                                              float* __restrict__ partial) {
  __shared__ float4 red[256];
  const int nq = C >> 2;
  const int lanes = blockDim.x / nq;
  const int q = threadIdx.x % nq, rl = threadIdx.x / nq;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int64_t r1 = r0 + R < M ? r0 + R : M;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rl < lanes) {
    for (int64_t r = r0 + rl; r < r1; r += lanes) {
      const int64_t o = r * C + 4 * q;
      const float4 gv = *reinterpret_cast<const float4*>(g + o);
      const float4 yv = *reinterpret_cast<const float4*>(y + o);
      float4 v;
      v.x = yv.x > 0.f ? gv.x : 0.f;
      v.y = yv.y > 0.f ? gv.y : 0.f;
      v.z = yv.z > 0.f ? gv.z : 0.f;
      v.w = yv.w > 0.f ? gv.w : 0.f;
      *reinterpret_cast<float4*>(gout + o) = v;
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rl == 0) {
    for (int k = 1; k < lanes; ++k) {
      const float4 t = red[k * nq + q];
      acc.x += t.x;
      acc.y += t.y;
      acc.z += t.z;
      acc.w += t.w;
    }
    *reinterpret_cast<float4*>(partial + static_cast<int64_t>(blockIdx.x) * C + 4 * q) = acc;
  }
}

}  // namespace nerf
}  // namespace anr

using namespace anr::nerf;

extern "C" int32_t anr_posenc_width(const anr_posenc_desc* d) {
  PE p;
  return make_pe(d, &p) ? p.width : -1;
}

extern "C" int anr_posenc_fwd(const anr_posenc_desc* d, const float* x, int64_t rows_per_x,
                              int64_t P, float* out, int64_t out_stride, anr_stream_t stream) {
  PE p;
  ANR_CHECK_ARG(d && make_pe(d, &p), "anr_posenc_fwd: bad descriptor");
  ANR_CHECK_ARG(P >= 0 && rows_per_x >= 1, "anr_posenc_fwd: bad sizes");
  if (P == 0) return ANR_OK;
  ANR_CHECK_ARG(x && out && out_stride >= p.width, "anr_posenc_fwd: null pointer / stride");
  const int64_t n = P * p.width;
  hipLaunchKernelGGL(posenc_fwd_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256),
                     0, reinterpret_cast<hipStream_t>(stream), p, x, rows_per_x, P, out, out_stride);
  ANR_CHECK_LAUNCH("anr_posenc_fwd");
  return ANR_OK;
}

extern "C" int anr_posenc_bwd(const anr_posenc_desc* d, const float* x, int64_t P,
                              const float* dout, int64_t dout_stride, float* dx,
                              anr_stream_t stream) {
  PE p;
  ANR_CHECK_ARG(d && make_pe(d, &p), "anr_posenc_bwd: bad descriptor");
  ANR_CHECK_ARG(P >= 0, "anr_posenc_bwd: bad sizes");
  if (P == 0) return ANR_OK;
  ANR_CHECK_ARG(x && dout && dx && dout_stride >= p.width, "anr_posenc_bwd: null pointer / stride");
  const int64_t n = P * p.n_dims;
  hipLaunchKernelGGL(posenc_bwd_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256),
                     0, reinterpret_cast<hipStream_t>(stream), p, x, P, dout, dout_stride, dx);
  ANR_CHECK_LAUNCH("anr_posenc_bwd");
  return ANR_OK;
}

extern "C" int anr_sample_pdf_fwd(const float* weights, int64_t w_ray_stride,
                                  int32_t w_sample_stride, const float* z_coarse,
                                  const float* u, const float* origin, const float* dir,
                                  int64_t B, int32_t Nc, int32_t Nf, float* z, float* pts,
                                  int32_t* src, int32_t* inds, float* cdf, anr_stream_t stream) {
  ANR_CHECK_ARG(B >= 0 && Nc >= 3 && Nc <= kMaxNc && Nf >= 1 && Nf <= kMaxNf,
                "anr_sample_pdf_fwd: need 3 <= Nc <= 64, 1 <= Nf <= 256");
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(weights && z_coarse && u && origin && dir && z && src && inds && cdf,
                "anr_sample_pdf_fwd: null pointer");
  PdfArgs a{};
  a.w = weights;
  a.w_ray = w_ray_stride;
  a.w_samp = w_sample_stride;
  a.zc = z_coarse;
  a.u = u;
  a.origin = origin;
  a.dir = dir;
  a.B = B;
  a.Nc = Nc;
  a.Nf = Nf;
  a.z = z;
  a.pts = pts;
  a.src = src;
  a.inds = inds;
  a.cdf = cdf;
  hipLaunchKernelGGL(sample_pdf_fwd_kernel, dim3(static_cast<unsigned>(B)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  ANR_CHECK_LAUNCH("anr_sample_pdf_fwd");
  return ANR_OK;
}

extern "C" int anr_sample_pdf_bwd(const float* weights, int64_t w_ray_stride,
                                  int32_t w_sample_stride, const float* z_coarse,
                                  const float* u, const float* dir, const int32_t* src,
                                  const int32_t* inds, const float* cdf, int64_t B, int32_t Nc,
                                  int32_t Nf, const float* d_z, const float* d_pts,
                                  float* d_weights, anr_stream_t stream) {
  ANR_CHECK_ARG(B >= 0 && Nc >= 3 && Nc <= kMaxNc && Nf >= 1 && Nf <= kMaxNf,
                "anr_sample_pdf_bwd: need 3 <= Nc <= 64, 1 <= Nf <= 256");
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(weights && z_coarse && u && dir && src && inds && cdf && d_weights,
                "anr_sample_pdf_bwd: null pointer");
  PdfArgs a{};
  a.w = weights;
  a.w_ray = w_ray_stride;
  a.w_samp = w_sample_stride;
  a.zc = z_coarse;
  a.u = u;
  a.dir = dir;
  a.B = B;
  a.Nc = Nc;
  a.Nf = Nf;
  a.src = const_cast<int32_t*>(src);
  a.inds = const_cast<int32_t*>(inds);
  a.cdf = const_cast<float*>(cdf);
  a.dz = d_z;
  a.dpts = d_pts;
  a.dw = d_weights;
  hipLaunchKernelGGL(sample_pdf_bwd_kernel, dim3(static_cast<unsigned>(B)), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  ANR_CHECK_LAUNCH("anr_sample_pdf_bwd");
  return ANR_OK;
}

extern "C" int anr_relu_bwd_colsum(const float* g, const float* y, int64_t M, int32_t C,
                                   float* g_out, float* partial, int32_t n_parts,
                                   anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && C >= 4 && C <= 1024 && C % 4 == 0 && n_parts >= 1,
                "anr_relu_bwd_colsum: need M >= 0, C a multiple of 4 in [4, 1024], n_parts >= 1");
  ANR_CHECK_ARG(partial && (M == 0 || (g && y && g_out)), "anr_relu_bwd_colsum: null pointer");
  ANR_CHECK_ARG(((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y) |
                  reinterpret_cast<uintptr_t>(g_out) | reinterpret_cast<uintptr_t>(partial)) & 15) == 0,
                "anr_relu_bwd_colsum: pointers must be 16-byte aligned");
  const int64_t R = M > 0 ? (M + n_parts - 1) / n_parts : 1;
  // every partial row is written (blocks past the last row write zeros)
  hipLaunchKernelGGL(anr::nerf::relu_bwd_colsum_kernel, dim3(static_cast<unsigned>(n_parts)),
                     dim3(256), 0, reinterpret_cast<hipStream_t>(stream), g, y, M, C, R, g_out,
                     partial);
  ANR_CHECK_LAUNCH("anr_relu_bwd_colsum");
  return ANR_OK;
}
