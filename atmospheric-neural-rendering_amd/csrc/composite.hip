// K8: transmittance / alpha-composite integrator, forward and backward.
//
// Replaces render() and render_with_surface() at src/atmonr/graphics_utils.py:6-77
// (called at src/atmonr/pipelines/instant_ngp.py:187-192 with z_vals*(scale/1000) and
// at pipelines/nerf.py:156). Reference math per ray (graphics_utils.py:28-48, 75-76):
//   mid   = [0, (z_i + z_{i+1})/2 ..., z_{N-1}]        delta_i = mid_{i+1} - mid_i
//   alpha = 1 - exp(-sigma * delta)                    t_i = 1 - alpha_i + 1e-10
//   T_i   = prod_{j<i} t_j (cumprod)                   w_i = alpha_i * T_i
//   C_atmo = sum_i w_i * c_i      C_surf = prod_i (1 - alpha_i) * c_surf
//   C = C_atmo + C_surf
// One wavefront per ray; lane l owns the contiguous samples [l*spl, (l+1)*spl). The
// cumprod is a lane-local product followed by a 64-lane shuffle exclusive scan; sums
// and the full product are shuffle reductions. The backward (autograd of the above)
// needs two suffix quantities, computed with reverse shuffle scans:
//   dL/dalpha_i = T_i (q_i - U_i) - r * prod_{k!=i}(1 - alpha_k) + dL/dalpha_i(direct)
//   U_i = sum_{j>i} q_j alpha_j prod_{i<k<j} t_k   (affine suffix scan; no division)
// with q_i = dL/dw_i and r = dL/dC_surf-product, so it stays exact when alpha -> 1.
// Arithmetic is f32 regardless of the storage dtype.
#pragma clang fp contract(off)

#include "anr_common.h"

namespace anr {

constexpr int kMaxCh = 8;

// 1: always use the generic (LDS-staged) kernels; test hook (anr_composite_force_generic).
static int g_composite_generic = 0;

template <typename T>
__device__ __forceinline__ float ldv(const T* p, int64_t i) { return to_f32<T>(p[i]); }
// alpha = 1 - exp(-x) (graphics_utils.py:38) as -expm1(-x): accurate to an ulp of alpha
// itself. Evaluated as 1 - expf(-x), f32 loses log2(1/x) bits to cancellation, and at
// BASELINE configs[2]'s 1,024 samples per ray x = sigma * delta is ~1e-6 at
// initialisation: dL/dcolor = w * dL/dC then carries 2e-2 relative error and the GPU
// exp's rounding bias accumulates in the dir-MLP gradient (tools/composite_diag.py).
__device__ __forceinline__ float alpha_of(float x) { return -expm1f(-x); }

// Exclusive multiplicative scan across the wave (lane 0 gets 1).
__device__ __forceinline__ float wave_excl_prod(float v, int lane) {
  float incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float o = shfl_up(incl, d);
    if (lane >= d) incl *= o;
  }
  const float ex = shfl_up(incl, 1);
  return lane == 0 ? 1.0f : ex;
}
// Exclusive multiplicative suffix scan (lane 63 gets 1).
__device__ __forceinline__ float wave_excl_suffix_prod(float v, int lane) {
  float incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float o = shfl_down(incl, d);
    if (lane + d < 64) incl *= o;
  }
  const float ex = shfl_down(incl, 1);
  return lane == 63 ? 1.0f : ex;
}
__device__ __forceinline__ float wave_prod(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v *= shfl_xor(v, m);
  return v;
}
// Reverse affine scan: lane holds map x -> A*x + B for its block; returns the value
// entering the lane's block from the right, i.e. (composition of lanes > l)(0).
__device__ __forceinline__ float wave_affine_suffix(float A, float B, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float Ao = shfl_down(A, d);
    const float Bo = shfl_down(B, d);
    if (lane + d < 64) {
      B = A * Bo + B;
      A = A * Ao;
    }
  }
  const float nxt = shfl_down(B, 1);
  return lane == 63 ? 0.0f : nxt;
}

struct CompArgs {
  const float* z;
  float z_scale;
  const void* color;
  const void* sigma;
  const void* color_surf;
  int64_t B;
  int N, C, S;
  // forward outputs
  void *color_map, *atmo, *surf, *weights, *alpha;
  // backward inputs / outputs
  const void *d_color_map, *d_atmo, *d_surf, *d_weights, *d_alpha;
  void *d_color, *d_sigma, *d_color_surf;
  float* d_z;
};

// delta_i for sample i of a ray (graphics_utils.py:30-34), z already in the ray's row.
__device__ __forceinline__ float delta_at(const float* zr, float zs, int i, int N) {
  const float zi = zr[i] * zs;
  const float lo = i == 0 ? zr[0] * zs * 0.0f : (zr[i - 1] * zs + zi) / 2.0f;
  const float hi = i == N - 1 ? zi : (zi + zr[i + 1] * zs) / 2.0f;
  return hi - lo;
}

template <typename T>
__global__ void __launch_bounds__(256) composite_fwd_kernel(CompArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64;
  if (b >= a.B) return;
  const int N = a.N, C = a.C, S = a.S;
  const int spl = (N + 63) / 64;
  const int i0 = lane * spl;
  const int i1 = min(i0 + spl, N);
  const float* zr = a.z + b * N;
  const T* sig = static_cast<const T*>(a.sigma) + b * N * S;
  const T* col = static_cast<const T*>(a.color) + b * N * C;

  // pass 1: lane products of t and (1 - alpha)
  float pt[kMaxCh], pom[kMaxCh];
#pragma unroll
  for (int s = 0; s < kMaxCh; ++s) pt[s] = pom[s] = 1.0f;
  for (int i = i0; i < i1; ++i) {
    const float dl = delta_at(zr, a.z_scale, i, N);
#pragma unroll
    for (int s = 0; s < kMaxCh; ++s) {
      if (s < S) {
        const float al = alpha_of(ldv(sig, i * S + s) * dl);
        pt[s] *= (1.0f - al) + 1e-10f;
        pom[s] *= 1.0f - al;
      }
    }
  }
  float T_in[kMaxCh], Stot[kMaxCh];
#pragma unroll
  for (int s = 0; s < kMaxCh; ++s) {
    if (s < S) {
      T_in[s] = wave_excl_prod(pt[s], lane);
      Stot[s] = wave_prod(pom[s]);
    }
  }
  // pass 2: weights and the atmospheric sum
  float cm[kMaxCh];
#pragma unroll
  for (int c = 0; c < kMaxCh; ++c) cm[c] = 0.0f;
  for (int i = i0; i < i1; ++i) {
    const float dl = delta_at(zr, a.z_scale, i, N);
    float w[kMaxCh];
#pragma unroll
    for (int s = 0; s < kMaxCh; ++s) {
      if (s < S) {
        const float al = alpha_of(ldv(sig, i * S + s) * dl);
        w[s] = al * T_in[s];
        T_in[s] *= (1.0f - al) + 1e-10f;
        const int64_t o = (b * N + i) * S + s;
        if (a.weights) static_cast<T*>(a.weights)[o] = from_f32<T>(w[s]);
        if (a.alpha) static_cast<T*>(a.alpha)[o] = from_f32<T>(al);
      }
    }
#pragma unroll
    for (int c = 0; c < kMaxCh; ++c)
      if (c < C) cm[c] += ldv(col, i * C + c) * w[S == 1 ? 0 : c];
  }
#pragma unroll
  for (int c = 0; c < kMaxCh; ++c) {
    if (c < C) {
      const float atmo = wave_sum(cm[c]);
      float surf = 0.0f;
      if (a.color_surf)
        surf = Stot[S == 1 ? 0 : c] * ldv(static_cast<const T*>(a.color_surf), b * C + c);
      if (lane == 0) {
        static_cast<T*>(a.color_map)[b * C + c] = from_f32<T>(atmo + surf);
        if (a.atmo) static_cast<T*>(a.atmo)[b * C + c] = from_f32<T>(atmo);
        if (a.surf) static_cast<T*>(a.surf)[b * C + c] = from_f32<T>(surf);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) composite_bwd_kernel(CompArgs a) {
  // Per wave LDS: lane-local prefix products Tloc, Ploc (N*S each) and dL/d(delta) (N).
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x / 64;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * (blockDim.x / 64) + wv;
  const bool active = b < a.B;
  const int N = a.N, C = a.C, S = a.S;
  float* Tloc = lds + static_cast<int64_t>(wv) * (2 * S + 1) * N;
  float* Ploc = Tloc + N * S;
  float* dD = Ploc + N * S;
  const int spl = (N + 63) / 64;
  const int i0 = lane * spl;
  const int i1 = min(i0 + spl, N);
  const int64_t bb = active ? b : 0;
  const T* sig = static_cast<const T*>(a.sigma) + bb * N * S;
  const T* col = static_cast<const T*>(a.color) + bb * N * C;
  const float* zr = a.z + bb * N;

  // per-ray upstream gradients: g_atmo = dC + dC_atmo, g_surf = dC + dC_surf
  float ga[kMaxCh], gs[kMaxCh];
#pragma unroll
  for (int c = 0; c < kMaxCh; ++c) {
    ga[c] = gs[c] = 0.0f;
    if (c < C && active) {
      const float dc = a.d_color_map ? ldv(static_cast<const T*>(a.d_color_map), bb * C + c) : 0.0f;
      ga[c] = dc + (a.d_atmo ? ldv(static_cast<const T*>(a.d_atmo), bb * C + c) : 0.0f);
      gs[c] = dc + (a.d_surf ? ldv(static_cast<const T*>(a.d_surf), bb * C + c) : 0.0f);
    }
  }

  // pass 1 (forward over the lane's block): lane products of t and 1-alpha, local
  // prefixes to LDS, and the block's reverse affine map of V_i = q_i*alpha_i + t_i*V_{i+1}
  // accumulated left-to-right as (A, B) <- (A*t_i, B + A*q_i*alpha_i).
  float pt[kMaxCh], pom[kMaxCh], A[kMaxCh], Bv[kMaxCh];
#pragma unroll
  for (int s = 0; s < kMaxCh; ++s) { pt[s] = pom[s] = A[s] = 1.0f; Bv[s] = 0.0f; }
  if (active) {
    for (int i = i0; i < i1; ++i) {
      const float dl = delta_at(zr, a.z_scale, i, N);
      float q[kMaxCh];
#pragma unroll
      for (int s = 0; s < kMaxCh; ++s) q[s] = 0.0f;
#pragma unroll
      for (int c = 0; c < kMaxCh; ++c)
        if (c < C) q[S == 1 ? 0 : c] += ldv(col, i * C + c) * ga[c];
#pragma unroll
      for (int s = 0; s < kMaxCh; ++s)
        if (s < S) {
          if (a.d_weights) q[s] += ldv(static_cast<const T*>(a.d_weights), (bb * N + i) * S + s);
          const float al = alpha_of(ldv(sig, i * S + s) * dl);
          const float t = (1.0f - al) + 1e-10f;
          Tloc[i * S + s] = pt[s];
          Ploc[i * S + s] = pom[s];
          pt[s] *= t;
          pom[s] *= 1.0f - al;
          Bv[s] = Bv[s] + A[s] * q[s] * al;
          A[s] = A[s] * t;
        }
    }
  }
  float T_in[kMaxCh], P_in[kMaxCh], Q[kMaxCh], V[kMaxCh], Stot[kMaxCh], r[kMaxCh];
#pragma unroll
  for (int s = 0; s < kMaxCh; ++s) {
    r[s] = 0.0f;
    if (s < S) {
      T_in[s] = wave_excl_prod(pt[s], lane);
      P_in[s] = wave_excl_prod(pom[s], lane);
      Q[s] = wave_excl_suffix_prod(pom[s], lane);
      Stot[s] = wave_prod(pom[s]);
      V[s] = wave_affine_suffix(A[s], Bv[s], lane);
    }
  }
  if (a.color_surf && active) {
#pragma unroll
    for (int c = 0; c < kMaxCh; ++c)
      if (c < C) r[S == 1 ? 0 : c] += ldv(static_cast<const T*>(a.color_surf), bb * C + c) * gs[c];
  }

  // pass 2 (reverse over the lane's block): per-sample gradients.
  if (active) {
    for (int i = i1 - 1; i >= i0; --i) {
      const float dl = delta_at(zr, a.z_scale, i, N);
      float q[kMaxCh];
#pragma unroll
      for (int s = 0; s < kMaxCh; ++s) q[s] = 0.0f;
#pragma unroll
      for (int c = 0; c < kMaxCh; ++c)
        if (c < C) q[S == 1 ? 0 : c] += ldv(col, i * C + c) * ga[c];
      float dd = 0.0f;  // dL/d(delta_i), summed over density channels
#pragma unroll
      for (int s = 0; s < kMaxCh; ++s)
        if (s < S) {
          const int64_t o = (bb * N + i) * S + s;
          if (a.d_weights) q[s] += ldv(static_cast<const T*>(a.d_weights), o);
          const float sg = ldv(sig, i * S + s);
          const float al = alpha_of(sg * dl);
          const float e = expf(-(sg * dl));  // d alpha / dx, accurate where alpha -> 1
          const float t = (1.0f - al) + 1e-10f;
          const float Ti = T_in[s] * Tloc[i * S + s];
          const float Pi = P_in[s] * Ploc[i * S + s];
          const float w = al * Ti;
#pragma unroll
          for (int c = 0; c < kMaxCh; ++c)
            if (c < C && (S == 1 || c == s) && a.d_color)
              static_cast<T*>(a.d_color)[(bb * N + i) * C + c] = from_f32<T>(w * ga[c]);
          float dal = Ti * (q[s] - V[s]) - r[s] * Pi * Q[s];
          if (a.d_alpha) dal += ldv(static_cast<const T*>(a.d_alpha), o);
          // alpha = 1 - exp(-sigma*delta): d/dsigma = delta*e, d/ddelta = sigma*e
          if (a.d_sigma) static_cast<T*>(a.d_sigma)[o] = from_f32<T>(dal * e * dl);
          dd += dal * e * sg;
          V[s] = q[s] * al + t * V[s];
          Q[s] *= 1.0f - al;
        }
      if (a.d_z) dD[i] = dd;
    }
  }
  if (a.d_color_surf && active && lane == 0) {
#pragma unroll
    for (int c = 0; c < kMaxCh; ++c)
      if (c < C)
        static_cast<T*>(a.d_color_surf)[bb * C + c] = from_f32<T>(Stot[S == 1 ? 0 : c] * gs[c]);
  }
  if (a.d_z) {
    __syncthreads();
    if (active) {
      // delta_i = mid_{i+1} - mid_i, mid_j = (zs_{j-1} + zs_j)/2 for 1 <= j <= N-1,
      // mid_0 = 0, mid_N = zs_{N-1}; zs = z * z_scale.
      for (int j = i0; j < i1; ++j) {
        float g = 0.0f;
        if (j >= 1) g += 0.5f * (dD[j - 1] - dD[j]);
        if (j + 1 <= N - 1) g += 0.5f * (dD[j] - dD[j + 1]);
        if (j == N - 1) g += dD[N - 1];
        a.d_z[bb * N + j] = g * a.z_scale;
      }
    }
  }
}


// ---------------------------------------------------------------------------------------
// Register-blocked kernels (SPL = samples per lane known at compile time, C = 4 bands,
// S in {1, 4}): each lane loads its contiguous block of z / sigma / color ONCE with vector
// loads into registers; neighbour z values at the block edges come from the adjacent
// lanes by shuffles. Same math and rounding order per sample as the kernels above.
namespace rb {

template <typename T>
__device__ __forceinline__ void load_block(const T* p, int n, float* dst) {
#pragma unroll
  for (int i = 0; i < n; ++i) dst[i] = to_f32<T>(p[i]);
}
template <>
__device__ __forceinline__ void load_block<float>(const float* p, int n, float* dst) {
  if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) {
#pragma unroll
    for (int i = 0; i < n; i += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + i);
      dst[i] = v.x; dst[i + 1] = v.y; dst[i + 2] = v.z; dst[i + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < n; ++i) dst[i] = p[i];
  }
}

// delta for the lane's SPL samples (graphics_utils.py:30-34); zs = z * z_scale. The
// neighbours across a lane boundary come from the adjacent lane; across a wave boundary
// (several waves per ray) they are read from the row.
template <int SPL>
__device__ __forceinline__ void deltas(const float* zrow, float zscale, int i0, int nvalid,
                                       int N, int lane, float* dl) {
  const float* zr = zrow + i0;
  float zs[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) zs[j] = j < nvalid ? zr[j] * zscale : 0.0f;
  float prev = shfl_up(zs[SPL - 1], 1);  // last sample of lane-1
  float next = shfl_down(zs[0], 1);      // first sample of lane+1
  if (lane == 0 && i0 > 0) prev = zrow[i0 - 1] * zscale;
  if (lane == 63 && i0 + SPL < N) next = zrow[i0 + SPL] * zscale;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int i = i0 + j;
    const float zi = zs[j];
    const float zprev = j == 0 ? prev : zs[j - 1];
    const float znext = j == SPL - 1 ? next : zs[j + 1];
    const float lo = i == 0 ? zi * 0.0f : (zprev + zi) / 2.0f;
    const float hi = i == N - 1 ? zi : (zi + znext) / 2.0f;
    dl[j] = hi - lo;
  }
}

// Wave-level reverse affine scan returning, for lane l, the composed map of the lanes
// > l (identity for lane 63) and the wave's total map (lane 0's inclusive composition).
__device__ __forceinline__ void wave_affine_suffix_maps(float A, float B, int lane, float* Aex,
                                                        float* Bex, float* Atot, float* Btot) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float Ao = shfl_down(A, d);
    const float Bo = shfl_down(B, d);
    if (lane + d < 64) {
      B = A * Bo + B;
      A = A * Ao;
    }
  }
  const float An = shfl_down(A, 1), Bn = shfl_down(B, 1);
  *Aex = lane == 63 ? 1.0f : An;
  *Bex = lane == 63 ? 0.0f : Bn;
  *Atot = __shfl(A, 0);
  *Btot = __shfl(B, 0);
}

// W waves per ray. W = 1: one wavefront per ray, 4 rays per 256-thread block, all scans
// are shuffles. W = 4: one block per ray (SPL = N/256 per lane, a quarter of the
// registers, four times the waves in flight); each scan is a wave scan plus the totals
// of the other waves through LDS (one barrier per group of scans).
template <typename T, int SPL, int S, int W>
__global__ void __launch_bounds__(256) fwd_kernel(CompArgs a) {
  constexpr int C = 4;
  constexpr int RPB = 4 / W;
  __shared__ float sh_t[RPB][2][4][S];
  __shared__ float sh_c[RPB][4][C];
  const int lane = threadIdx.x & 63;
  const int wid = static_cast<int>(threadIdx.x >> 6);
  const int part = wid % W, rib = wid / W;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * RPB + rib;
  if (b >= a.B) return;  // uniform per ray (per block when W > 1)
  const int N = a.N;
  const int i0 = (part * 64 + lane) * SPL;
  const int nvalid = max(0, min(SPL, N - i0));
  float dl[SPL], sg[SPL * S], col[SPL * C];
  deltas<SPL>(a.z + b * N, a.z_scale, i0, nvalid, N, lane, dl);
  if (nvalid == SPL) {
    load_block<T>(static_cast<const T*>(a.sigma) + (b * N + i0) * S, SPL * S, sg);
    load_block<T>(static_cast<const T*>(a.color) + (b * N + i0) * C, SPL * C, col);
  } else {
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
#pragma unroll
      for (int s = 0; s < S; ++s)
        sg[j * S + s] = j < nvalid ? ldv(static_cast<const T*>(a.sigma), (b * N + i0 + j) * S + s) : 0.0f;
#pragma unroll
      for (int c = 0; c < C; ++c)
        col[j * C + c] = j < nvalid ? ldv(static_cast<const T*>(a.color), (b * N + i0 + j) * C + c) : 0.0f;
    }
  }
  float al[SPL * S], pt[S], pom[S];
#pragma unroll
  for (int s = 0; s < S; ++s) pt[s] = pom[s] = 1.0f;
#pragma unroll
  for (int j = 0; j < SPL; ++j)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float x = alpha_of(sg[j * S + s] * dl[j]);
      al[j * S + s] = j < nvalid ? x : 0.0f;
      pt[s] *= (1.0f - al[j * S + s]) + (j < nvalid ? 1e-10f : 0.0f);
      pom[s] *= 1.0f - al[j * S + s];
    }
  float Tin[S], Stot[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    Tin[s] = wave_excl_prod(pt[s], lane);
    Stot[s] = wave_prod(pom[s]);
  }
  if constexpr (W > 1) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float tot = wave_prod(pt[s]);
      if (lane == 0) {
        sh_t[rib][0][part][s] = tot;
        sh_t[rib][1][part][s] = Stot[s];
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float pre = 1.0f, all = 1.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        if (w < part) pre *= sh_t[rib][0][w][s];
        all *= sh_t[rib][1][w][s];
      }
      Tin[s] *= pre;
      Stot[s] = all;
    }
  }
  float cm[C] = {0.0f, 0.0f, 0.0f, 0.0f};
  T* wout = a.weights ? static_cast<T*>(a.weights) + (b * N + i0) * S : nullptr;
  T* aout = a.alpha ? static_cast<T*>(a.alpha) + (b * N + i0) * S : nullptr;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    float w[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      w[s] = al[j * S + s] * Tin[s];
      Tin[s] *= (1.0f - al[j * S + s]) + 1e-10f;
      if (j < nvalid) {
        if (wout) wout[j * S + s] = from_f32<T>(w[s]);
        if (aout) aout[j * S + s] = from_f32<T>(al[j * S + s]);
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) cm[c] += col[j * C + c] * w[S == 1 ? 0 : c];
  }
  float atmo[C];
#pragma unroll
  for (int c = 0; c < C; ++c) atmo[c] = wave_sum(cm[c]);
  if constexpr (W > 1) {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) sh_c[rib][part][c] = atmo[c];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float t = 0.0f;
#pragma unroll
      for (int w = 0; w < W; ++w) t += sh_c[rib][w][c];
      atmo[c] = t;
    }
  }
  if (part == 0 && lane == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float surf = 0.0f;
      if (a.color_surf) surf = Stot[S == 1 ? 0 : c] * ldv(static_cast<const T*>(a.color_surf), b * C + c);
      static_cast<T*>(a.color_map)[b * C + c] = from_f32<T>(atmo[c] + surf);
      if (a.atmo) static_cast<T*>(a.atmo)[b * C + c] = from_f32<T>(atmo[c]);
      if (a.surf) static_cast<T*>(a.surf)[b * C + c] = from_f32<T>(surf);
    }
  }
}

template <typename T, int SPL, int S, int W>
__global__ void __launch_bounds__(256) bwd_kernel(CompArgs a) {
  constexpr int C = 4;
  constexpr int RPB = 4 / W;
  // per wave: totals of pt, pom and the wave's affine map (A, B); boundary dD values
  __shared__ float sh_t[RPB][4][4][S];
  __shared__ float sh_d[RPB][4][2];
  const int lane = threadIdx.x & 63;
  const int wid = static_cast<int>(threadIdx.x >> 6);
  const int part = wid % W, rib = wid / W;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * RPB + rib;
  if (b >= a.B) return;  // uniform per ray (per block when W > 1)
  const int N = a.N;
  const int i0 = (part * 64 + lane) * SPL;
  const int nvalid = max(0, min(SPL, N - i0));
  float dl[SPL], sg[SPL * S], col[SPL * C];
  deltas<SPL>(a.z + b * N, a.z_scale, i0, nvalid, N, lane, dl);
  if (nvalid == SPL) {
    load_block<T>(static_cast<const T*>(a.sigma) + (b * N + i0) * S, SPL * S, sg);
    load_block<T>(static_cast<const T*>(a.color) + (b * N + i0) * C, SPL * C, col);
  } else {
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
#pragma unroll
      for (int s = 0; s < S; ++s)
        sg[j * S + s] = j < nvalid ? ldv(static_cast<const T*>(a.sigma), (b * N + i0 + j) * S + s) : 0.0f;
#pragma unroll
      for (int c = 0; c < C; ++c)
        col[j * C + c] = j < nvalid ? ldv(static_cast<const T*>(a.color), (b * N + i0 + j) * C + c) : 0.0f;
    }
  }
  float ga[C], gs[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float dc = a.d_color_map ? ldv(static_cast<const T*>(a.d_color_map), b * C + c) : 0.0f;
    ga[c] = dc + (a.d_atmo ? ldv(static_cast<const T*>(a.d_atmo), b * C + c) : 0.0f);
    gs[c] = dc + (a.d_surf ? ldv(static_cast<const T*>(a.d_surf), b * C + c) : 0.0f);
  }
  // forward over the block: e = exp(-sigma*delta), alpha, local prefixes, lane aggregates
  float e[SPL * S], al[SPL * S], Tl[SPL * S], Pl[SPL * S], q[SPL * S];
  float pt[S], pom[S], A[S], Bv[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { pt[s] = pom[s] = A[s] = 1.0f; Bv[s] = 0.0f; }
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    float qq[S];
#pragma unroll
    for (int s = 0; s < S; ++s) qq[s] = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) qq[S == 1 ? 0 : c] += col[j * C + c] * ga[c];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int o = j * S + s;
      if (a.d_weights && j < nvalid) qq[s] += ldv(static_cast<const T*>(a.d_weights), (b * N + i0 + j) * S + s);
      const float ao = alpha_of(sg[o] * dl[j]);
      // d alpha / dx = exp(-x) on its own: 1 - alpha cancels once alpha nears 1 (x > ~8)
      const float ee = expf(-(sg[o] * dl[j]));
      e[o] = ee;
      al[o] = j < nvalid ? ao : 0.0f;
      q[o] = j < nvalid ? qq[s] : 0.0f;
      const float t = (1.0f - al[o]) + (j < nvalid ? 1e-10f : 0.0f);
      Tl[o] = pt[s];
      Pl[o] = pom[s];
      pt[s] *= t;
      pom[s] *= 1.0f - al[o];
      Bv[s] = Bv[s] + A[s] * q[o] * al[o];
      A[s] = A[s] * t;
    }
  }
  float Tin[S], Pin[S], Q[S], V[S], Stot[S], r[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    Tin[s] = wave_excl_prod(pt[s], lane);
    Pin[s] = wave_excl_prod(pom[s], lane);
    Q[s] = wave_excl_suffix_prod(pom[s], lane);
    Stot[s] = wave_prod(pom[s]);
    r[s] = 0.0f;
  }
  float Aex[S], Bex[S], Atot[S], Btot[S];
#pragma unroll
  for (int s = 0; s < S; ++s)
    wave_affine_suffix_maps(A[s], Bv[s], lane, &Aex[s], &Bex[s], &Atot[s], &Btot[s]);
  if constexpr (W > 1) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float tpt = wave_prod(pt[s]);
      if (lane == 0) {
        sh_t[rib][0][part][s] = tpt;
        sh_t[rib][1][part][s] = Stot[s];
        sh_t[rib][2][part][s] = Atot[s];
        sh_t[rib][3][part][s] = Btot[s];
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float pre_t = 1.0f, pre_p = 1.0f, suf_p = 1.0f, all = 1.0f, xin = 0.0f;
#pragma unroll
      for (int w = W - 1; w >= 0; --w) {
        const float wt = sh_t[rib][0][w][s], wp = sh_t[rib][1][w][s];
        if (w < part) {
          pre_t *= wt;
          pre_p *= wp;
        }
        if (w > part) {
          suf_p *= wp;
          xin = sh_t[rib][2][w][s] * xin + sh_t[rib][3][w][s];
        }
        all *= wp;
      }
      Tin[s] *= pre_t;
      Pin[s] *= pre_p;
      Q[s] *= suf_p;
      Stot[s] = all;
      V[s] = Aex[s] * xin + Bex[s];
    }
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) V[s] = Bex[s];
  }
  if (a.color_surf) {
#pragma unroll
    for (int c = 0; c < C; ++c)
      r[S == 1 ? 0 : c] += ldv(static_cast<const T*>(a.color_surf), b * C + c) * gs[c];
  }
  float dD[SPL];
  T* dcol = a.d_color ? static_cast<T*>(a.d_color) + (b * N + i0) * C : nullptr;
  T* dsig = a.d_sigma ? static_cast<T*>(a.d_sigma) + (b * N + i0) * S : nullptr;
#pragma unroll
  for (int j = SPL - 1; j >= 0; --j) {
    float dd = 0.0f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int o = j * S + s;
      const float Ti = Tin[s] * Tl[o];
      const float Pi = Pin[s] * Pl[o];
      const float w = al[o] * Ti;
      if (dcol && j < nvalid) {
#pragma unroll
        for (int c = 0; c < C; ++c)
          if (S == 1 || c == s) {
            dcol[j * C + c] = from_f32<T>(w * ga[c]);
          }
      }
      float dal = Ti * (q[o] - V[s]) - r[s] * Pi * Q[s];
      if (a.d_alpha && j < nvalid) dal += ldv(static_cast<const T*>(a.d_alpha), (b * N + i0 + j) * S + s);
      if (dsig && j < nvalid) {
        dsig[j * S + s] = from_f32<T>(dal * e[o] * dl[j]);
      }
      dd += dal * e[o] * sg[o];
      const float t = (1.0f - al[o]) + (j < nvalid ? 1e-10f : 0.0f);
      V[s] = q[o] * al[o] + t * V[s];
      Q[s] *= 1.0f - al[o];
    }
    dD[j] = j < nvalid ? dd : 0.0f;
  }
  if (a.d_color_surf && part == 0 && lane == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c)
      static_cast<T*>(a.d_color_surf)[b * C + c] = from_f32<T>(Stot[S == 1 ? 0 : c] * gs[c]);
  }
  if (a.d_z) {
    float dprev = shfl_up(dD[SPL - 1], 1);
    float dnext = shfl_down(dD[0], 1);
    if constexpr (W > 1) {
      if (lane == 0) sh_d[rib][part][0] = dD[0];
      if (lane == 63) sh_d[rib][part][1] = dD[SPL - 1];
      __syncthreads();
      if (lane == 0 && part > 0) dprev = sh_d[rib][part - 1][1];
      if (lane == 63 && part < W - 1) dnext = sh_d[rib][part + 1][0];
    }
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int i = i0 + j;
      if (j >= nvalid) break;
      const float dm1 = j == 0 ? dprev : dD[j - 1];
      const float dp1 = j == SPL - 1 ? dnext : dD[j + 1];
      float g = 0.0f;
      if (i >= 1) g += 0.5f * (dm1 - dD[j]);
      if (i + 1 <= N - 1) g += 0.5f * (dD[j] - dp1);
      if (i == N - 1) g += dD[j];
      a.d_z[b * N + i] = g * a.z_scale;
    }
  }
}

}  // namespace rb

// Launch a register-blocked kernel if (C, S, N) is covered; returns false otherwise.
// Rays of up to 256 samples: one wavefront each; longer rays (N <= 4096): one 4-wave
// block each.
template <typename T>
static bool launch_rb(bool bwd, const CompArgs& a, hipStream_t st) {
  if (a.C != 4 || !(a.S == 1 || a.S == 4)) return false;
#define ANR_RB(SPL, S, W)                                                                    \
  do {                                                                                       \
    const dim3 grid(static_cast<unsigned>(ceil_div(a.B, 4 / (W)))), block(256);              \
    if (bwd)                                                                                 \
      hipLaunchKernelGGL((rb::bwd_kernel<T, SPL, S, W>), grid, block, 0, st, a);             \
    else                                                                                     \
      hipLaunchKernelGGL((rb::fwd_kernel<T, SPL, S, W>), grid, block, 0, st, a);             \
  } while (0)
#define ANR_RB_S(SPL, W) \
  if (a.S == 1) ANR_RB(SPL, 1, W); else ANR_RB(SPL, 4, W); return true;
  if (a.N <= 256) {
    switch ((a.N + 63) / 64) {
      case 1: ANR_RB_S(1, 1)
      case 2: ANR_RB_S(2, 1)
      case 3: ANR_RB_S(3, 1)
      case 4: ANR_RB_S(4, 1)
      default: return false;
    }
  }
  switch ((a.N + 255) / 256) {
    case 2: ANR_RB_S(2, 4)
    case 3: ANR_RB_S(3, 4)
    case 4: ANR_RB_S(4, 4)
    case 8: ANR_RB_S(8, 4)
    case 16: ANR_RB_S(16, 4)
    default: return false;
  }
#undef ANR_RB_S
#undef ANR_RB
}
}  // namespace anr

extern "C" int anr_composite_force_generic(int32_t on) {
  const int prev = anr::g_composite_generic;
  anr::g_composite_generic = on ? 1 : 0;
  return prev;
}

extern "C" int anr_composite_fwd(const float* z, float z_scale, const void* color,
                                 const void* sigma, const void* color_surf, int32_t io_dtype,
                                 int64_t B, int32_t N, int32_t C, int32_t S, void* color_map,
                                 void* color_map_atmo, void* color_map_surf, void* weights,
                                 void* alpha, anr_stream_t stream) {
  using namespace anr;
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(z && color && sigma && color_map, "anr_composite_fwd: null argument");
  ANR_CHECK_ARG(B >= 0 && N >= 1 && C >= 1 && C <= kMaxCh && (S == 1 || S == C),
                "anr_composite_fwd: bad shape B=%lld N=%d C=%d S=%d", (long long)B, N, C, S);
  ANR_CHECK_ARG(io_dtype == ANR_F16 || io_dtype == ANR_F32, "anr_composite_fwd: bad dtype");
  if (B == 0) return ANR_OK;
  CompArgs a{};
  a.z = z; a.z_scale = z_scale; a.color = color; a.sigma = sigma; a.color_surf = color_surf;
  a.B = B; a.N = N; a.C = C; a.S = S;
  a.color_map = color_map; a.atmo = color_map_atmo; a.surf = color_map_surf;
  a.weights = weights; a.alpha = alpha;
  if (!g_composite_generic &&
      (io_dtype == ANR_F16 ? launch_rb<__half>(false, a, as_stream(stream))
                           : launch_rb<float>(false, a, as_stream(stream)))) {
    ANR_CHECK_LAUNCH("anr_composite_fwd(rb)");
    return ANR_OK;
  }
  const dim3 grid(static_cast<unsigned>(ceil_div(B, 4))), block(256);
  if (io_dtype == ANR_F16)
    hipLaunchKernelGGL(composite_fwd_kernel<__half>, grid, block, 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(composite_fwd_kernel<float>, grid, block, 0, as_stream(stream), a);
  ANR_CHECK_LAUNCH("anr_composite_fwd");
  return ANR_OK;
}

extern "C" int anr_composite_bwd(const float* z, float z_scale, const void* color,
                                 const void* sigma, const void* color_surf, int32_t io_dtype,
                                 int64_t B, int32_t N, int32_t C, int32_t S,
                                 const void* d_color_map, const void* d_atmo,
                                 const void* d_surf, const void* d_weights,
                                 const void* d_alpha, void* d_color, void* d_sigma,
                                 void* d_color_surf, float* d_z, anr_stream_t stream) {
  using namespace anr;
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(z && color && sigma, "anr_composite_bwd: null argument");
  ANR_CHECK_ARG(B >= 0 && N >= 1 && C >= 1 && C <= kMaxCh && (S == 1 || S == C),
                "anr_composite_bwd: bad shape");
  ANR_CHECK_ARG(io_dtype == ANR_F16 || io_dtype == ANR_F32, "anr_composite_bwd: bad dtype");
  ANR_CHECK_ARG(d_color_surf == nullptr || color_surf != nullptr,
                "anr_composite_bwd: d_color_surf without color_surf");
  if (B == 0) return ANR_OK;
  CompArgs a{};
  a.z = z; a.z_scale = z_scale; a.color = color; a.sigma = sigma; a.color_surf = color_surf;
  a.B = B; a.N = N; a.C = C; a.S = S;
  a.d_color_map = d_color_map; a.d_atmo = d_atmo; a.d_surf = d_surf;
  a.d_weights = d_weights; a.d_alpha = d_alpha;
  a.d_color = d_color; a.d_sigma = d_sigma; a.d_color_surf = d_color_surf; a.d_z = d_z;
  if (!g_composite_generic &&
      (io_dtype == ANR_F16 ? launch_rb<__half>(true, a, as_stream(stream))
                           : launch_rb<float>(true, a, as_stream(stream)))) {
    ANR_CHECK_LAUNCH("anr_composite_bwd(rb)");
    return ANR_OK;
  }
  const size_t per_wave = static_cast<size_t>(2 * S + 1) * N * sizeof(float);
  int waves = 4;
  while (waves > 1 && waves * per_wave > 64 * 1024) --waves;
  const size_t lds = waves * per_wave;
  ANR_CHECK_ARG(lds <= 64 * 1024, "anr_composite_bwd: N*S too large (%d*%d)", N, S);
  const dim3 grid(static_cast<unsigned>(ceil_div(B, waves))), block(64 * waves);
  if (io_dtype == ANR_F16)
    hipLaunchKernelGGL(composite_bwd_kernel<__half>, grid, block, lds, as_stream(stream), a);
  else
    hipLaunchKernelGGL(composite_bwd_kernel<float>, grid, block, lds, as_stream(stream), a);
  ANR_CHECK_LAUNCH("anr_composite_bwd");
  return ANR_OK;
}
