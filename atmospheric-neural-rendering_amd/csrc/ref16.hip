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

#include <stdlib.h>

#include "anr_common.h"

namespace anr {
namespace ref16 {

constexpr int kMaxC = 8;
constexpr int kSeg = 64;   // samples per ray and segment: one per lane

// Round an f32 VALUE to f16. The asm barrier makes the f32 rounding of the expression that
// produced x happen first: without it the backend fuses h(a * b) and h(a + b) into one
// v_fma_mixlo_f16, which rounds the EXACT product / sum to f16 once, where torch's f16 ops
// round to f32 (opmath) and then to f16. The two differ when the f32 result lands on an f16
// tie (z_vals * scale -> f16 km, x * (1 / max_i), norm * d, gt + eps): measured on the
// PSNR test's first step, 6 of 65,536 dL/dsigma moved between neighbouring samples (an f16
// z one ulp off shifts a mid-point, i.e. swaps two deltas) -- the r04 N = 1,024 PSNR drift
// (tools/r5/composite_ref16_diag.py).
__device__ __forceinline__ float h(float x) {
  asm("" : "+v"(x));
  return __half2float(__float2half_rn(x));
}

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

// delta_i = diff([0, (z_0 + z_1) / 2, ..., (z_{N-2} + z_{N-1}) / 2, z_{N-1}])_i in f16
// (graphics_utils.py:31-35), z_vals (f32) * scale -> f16 first (graphics_utils.py:28); from
// the raw f32 z values at i - 1, i, i + 1 (zm / zp unused at the ends)
__device__ __forceinline__ float delta_z(float zm, float z0, float zp, float zs, int i, int N) {
  const float zi = h(z0 * zs);
  const float lo = i == 0 ? h(zi * 0.0f) : h(h(h(zm * zs) + zi) * 0.5f);
  const float hi = i == N - 1 ? zi : h(h(zi + h(zp * zs)) * 0.5f);
  return h(hi - lo);
}

// A wavefront is the whole workgroup here: LDS written by one lane and read by another
// needs only program order (LDS executes a wave's instructions in issue order) and a
// compiler barrier. __syncthreads() would also wait for every global load and store in
// flight (its workgroup-scope release), which is what kept these kernels latency-bound.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One segment's global inputs for the R rays of a wave, one sample per lane, loaded a
// segment ahead so the loads are in flight during the current segment's scans.
template <int R, bool COLOR, bool SIGMA>
struct SegIn {
  float zm[R], z0[R], zp[R], sg[R], col[R][kMaxC];

  template <typename T>
  __device__ __forceinline__ void fetch(const float* z, const T* sigma, const T* color,
                                        int64_t b0, int nr, int s0, int N, int C, int lane) {
    const int i = s0 + lane;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nr && lane < N - s0 && lane < kSeg) {
        const int64_t b = b0 + r;
        const float* zr = z + b * N;
        z0[r] = zr[i];
        zm[r] = i > 0 ? zr[i - 1] : 0.0f;
        zp[r] = i < N - 1 ? zr[i + 1] : 0.0f;
        if (SIGMA) sg[r] = ld(sigma, b * N + i);
        if (COLOR) {
#pragma unroll
          for (int c = 0; c < kMaxC; ++c)
            if (c < C) col[r][c] = ld(color, (b * N + i) * C + c);
        }
      }
    }
  }
};

struct Sample {
  float delta, e, alpha, q2;  // q2 = 1 - alpha + 1e-10 (= om = 1 - alpha in f16)
};

__device__ __forceinline__ Sample from_e(float e, float dl) {
  Sample s;
  s.delta = dl;
  s.e = e;
  s.alpha = h(1.0f - s.e);                            // 1 - exp
  s.q2 = h(h(1.0f - s.alpha) + 1e-10f);               // 1 - alpha + 1e-10 (:45)
  return s;
}

__device__ __forceinline__ Sample sample(float sig, float dl) {
  const float x = h(-sig * dl);                       // -sigma * delta   (:38)
  return from_e(h64(exp(static_cast<double>(x))), dl);  // exp
}

// R rays per wavefront (block = 64 threads), samples in segments of kSeg = 64 per ray. A
// segment splits into lane-parallel phases (the per-sample f16 ops: delta, exp, alpha,
// weights, the colour products), run as R passes of one ray's 64 samples across the
// lanes, and serial scans over LDS (the f16 cumprod, the f32 product and band sums, the
// f16 reversed cumsum of the backward) -- exactly the accumulations that have no parallel
// form rounding the same way. A scan runs on lane r for ray r (the band sums on lane
// r * C + c), so one scan instruction advances R rays: at R = 1 (r04's first form, one
// wave per ray) the scans left 63 of 64 lanes idle and were ~3/4 of the kernels' VALU
// issue. Every value is formed by the same expression as in the one-thread-per-ray r03
// kernels, so the outputs are unchanged bit for bit.
constexpr int kPad = 72;   // LDS row stride in halves: 144 B = 36 banks, rows on distinct banks

// Every staged value is an f16 value (the outputs of h()), so LDS holds them as f16. The
// serial cumprod / reversed cumsum steps run in native f16 arithmetic: the f32 product of
// two f16 values is exact, and their f32 sum rounds only where the smaller operand is
// below a quarter f16 ulp of the larger (both forms then return the larger), so one IEEE
// f16 multiply / add rounds exactly as h(a * b) / h(a + b) -- one dependent instruction
// per step of the chain instead of three.
template <int R>
struct __attribute__((aligned(16))) FwdLds {
  // padded past a segment's n samples with the chain's neutral elements, so the serial
  // scans run in whole 8-sample (16-B) LDS vectors: q2 = 1 (cp * 1, pr * 1 exact), t = -0
  // (x + -0 == x for every x, signed zeros included)
  _Float16 q2[R][kPad];
  _Float16 alpha[R][kPad];
  _Float16 T[R][kPad];
  _Float16 t[kMaxC][R][kPad];  // f16(f16(color) * w) per band
};
typedef _Float16 h8v __attribute__((ext_vector_type(8)));

// f32 x f16 and f32 + f16 with one rounding, as the f32 ops on the converted f16 value:
// fma(a, q, +0) = round(a * q) (a * q >= 0 here, so no -0 case) and fma(x, 1, acc) =
// round(acc + x); one v_fma_mix_f32 each instead of a conversion and the op -- the serial
// scans are most of these kernels' VALU issue
__device__ __forceinline__ float mul_h(float a, _Float16 q) {
  return __builtin_fmaf(a, static_cast<float>(q), 0.0f);
}
__device__ __forceinline__ float add_h(float acc, _Float16 x) {
  return __builtin_fmaf(static_cast<float>(x), 1.0f, acc);
}
constexpr float kNegZero = -0.0f;

template <int R, typename T>
__global__ void __launch_bounds__(64) fwd_kernel(const float* __restrict__ z, float zs,
                                                 const T* __restrict__ color,
                                                 const T* __restrict__ sigma,
                                                 const T* __restrict__ cs, int64_t B, int N,
                                                 int C, __half* cmap, __half* atmo_out,
                                                 __half* surf_out, __half* weights,
                                                 __half* alpha_out, __half* color16,
                                                 __half* sigma16) {
  __shared__ FwdLds<R> L;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = B - b0 < R ? static_cast<int>(B - b0) : R;  // rays of this wave
  const int lane = threadIdx.x;
  const int sr = lane / C, sc = lane - sr * C;  // band-sum lane: ray sr, band sc
  _Float16 cp = 1.0f;  // lane r < nr: ray r's cumprod output, f16 accumulator (cuda scan)
  float pr = 1.0f;     // lane r < nr: ray r's prod over samples, f32 accumulator
  float acc = 0.0f;    // lane sr < nr: ray sr's band sc sum over samples, f32 accumulator
  SegIn<R, true, true> nxt;
  nxt.fetch(z, sigma, color, b0, nr, 0, N, C, lane);
  for (int s0 = 0; s0 < N; s0 += kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    const SegIn<R, true, true> cur = nxt;
    if (s0 + kSeg < N) nxt.fetch(z, sigma, color, b0, nr, s0 + kSeg, N, C, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nr && lane < n) {
        const int64_t b = b0 + r;
        const float sg = h(cur.sg[r]);
        if (sigma16) sigma16[b * N + s0 + lane] = __float2half_rn(sg);
        const Sample sm = sample(sg, delta_z(cur.zm[r], cur.z0[r], cur.zp[r], zs, s0 + lane, N));
        L.q2[r][lane] = static_cast<_Float16>(sm.q2);
        L.alpha[r][lane] = static_cast<_Float16>(sm.alpha);
      } else if (lane < nv) {
        L.q2[r][lane] = static_cast<_Float16>(1.0f);
      }
    }
    wave_sync();
    if (lane < nr) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v q = *reinterpret_cast<const h8v*>(&L.q2[lane][l8]);
        h8v tv;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          tv[k] = cp;                                   // cumprod(...)[:, :-1]
          cp = cp * q[k];                               // = h(cp * q2)
          pr = mul_h(pr, q[k]);                         // (1 - alpha).prod   (:75)
        }
        *reinterpret_cast<h8v*>(&L.T[lane][l8]) = tv;
      }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nr && lane < n) {
        const int64_t i = (b0 + r) * N + s0 + lane;
        const float al = static_cast<float>(L.alpha[r][lane]);
        const float w = h(al * static_cast<float>(L.T[r][lane]));   // alpha * T    (:43-46)
#pragma unroll
        for (int c = 0; c < kMaxC; ++c) {
          if (c >= C) break;
          const float col = h(cur.col[r][c]);
          if (color16) color16[i * C + c] = __float2half_rn(col);
          L.t[c][r][lane] = static_cast<_Float16>(h(col * w));  // (:48)
        }
        if (weights) weights[i] = __float2half_rn(w);
        if (alpha_out) alpha_out[i] = __float2half_rn(al);
      } else if (lane < nv) {
        for (int c = 0; c < C; ++c) L.t[c][r][lane] = static_cast<_Float16>(kNegZero);
      }
    }
    wave_sync();
    if (sr < nr) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v tv = *reinterpret_cast<const h8v*>(&L.t[sc][sr][l8]);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = add_h(acc, tv[k]);
      }
    }
    wave_sync();
  }
  const float prr = h(__shfl(pr, sr < R ? sr : 0));
  if (sr < nr) {
    const int64_t b = b0 + sr;
    const int c = sc;
    const float atmo = h(acc);
    const float surf = cs ? h(prr * h(ld(cs, b * C + c))) : 0.0f;
    cmap[b * C + c] = __float2half_rn(cs ? h(atmo + surf) : atmo);          // (:76)
    if (atmo_out) atmo_out[b * C + c] = __float2half_rn(atmo);
    if (surf_out && cs) surf_out[b * C + c] = __float2half_rn(surf);
  }
}

// Autograd of fwd_kernel for dL/dcolor_map (oracle/ref_f16.py render_bwd). d_sigma
// (one value per sample) doubles as the scratch holding the forward's cumprod outputs T_i,
// and d_color's first band as the one holding exp(-sigma * delta), both read back in the
// reverse pass before the gradients overwrite them. Same R-rays-per-wave
// phases as fwd_kernel: pass 1 replays the cumprod; pass 2 walks the segments from the
// last, with the reversed cumsum (rc) as the one serial scan.
template <int R>
struct __attribute__((aligned(16))) BwdLds {
  // padded as FwdLds: q2 = 1, u = -0 past a segment's n samples
  _Float16 q2[R][kPad];
  _Float16 u[R][kPad];    // pass 1: T_k; pass 2: f16(T_k * dL/dT_k)
  _Float16 rin[R][kPad];  // rc before sample k's term
  float g[R][kMaxC];      // dL/dcolor_map per ray and band
  float g_pr[R];          // dL/d(surface product) per ray
  float pr[R];            // the surface product per ray (f16 value)
};

template <int R, typename T, typename G>
__global__ void __launch_bounds__(64) bwd_kernel(const float* __restrict__ z, float zs,
                                                 const T* __restrict__ color,
                                                 const T* __restrict__ sigma,
                                                 const T* __restrict__ cs, int64_t B, int N,
                                                 int C, const __half* __restrict__ g_cm,
                                                 G* d_color, G* d_sigma, G* d_cs,
                                                 int* zero_rays) {
  __shared__ BwdLds<R> L;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = B - b0 < R ? static_cast<int>(B - b0) : R;
  const int lane = threadIdx.x;
  const int sr = lane / C, sc = lane - sr * C;
  float gl = 0.0f;  // lane sr < nr: ray sr's band sc
  if (sr < nr) {
    gl = __half2float(g_cm[(b0 + sr) * C + sc]);
    L.g[sr][sc] = gl;
  }
  // pass 1: the forward's cumprod outputs (scratch) and the surface product
  _Float16 cp = 1.0f;
  float pr = 1.0f;
  uint32_t zmask = 0;  // bit r: ray r has an f16 alpha of 1 (uniform)
  SegIn<R, false, true> nxt;
  nxt.fetch(z, sigma, color, b0, nr, 0, N, C, lane);
  for (int s0 = 0; s0 < N; s0 += kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    const SegIn<R, false, true> cur = nxt;
    if (s0 + kSeg < N) nxt.fetch(z, sigma, color, b0, nr, s0 + kSeg, N, C, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool zr = false;
      if (r < nr && lane < n) {
        const int64_t b = b0 + r;
        const Sample sm = sample(h(cur.sg[r]),
                                 delta_z(cur.zm[r], cur.z0[r], cur.zp[r], zs, s0 + lane, N));
        L.q2[r][lane] = static_cast<_Float16>(sm.q2);
        // exp(-sigma * delta) (an f16 value) parked in the sample's first d_color slot until
        // pass 2 reads it back before writing that slot: one f64 exp per sample
        d_color[(b * N + s0 + lane) * C] = static_cast<G>(sm.e);
        zr = sm.q2 == 0.0f;
      } else if (lane < nv) {
        L.q2[r][lane] = static_cast<_Float16>(1.0f);
      }
      if (__any(zr)) zmask |= 1u << r;
    }
    wave_sync();
    if (lane < nr) {
      for (int l8 = 0; l8 < nv; l8 += 8) {
        const h8v q = *reinterpret_cast<const h8v*>(&L.q2[lane][l8]);
        h8v tv;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          tv[k] = cp;  // T_i, staged for the coalesced scratch store below
          cp = cp * q[k];  // = h(cp * q2)
          pr = mul_h(pr, q[k]);
        }
        *reinterpret_cast<h8v*>(&L.u[lane][l8]) = tv;
      }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r < nr && lane < n)
        d_sigma[(b0 + r) * N + s0 + lane] = static_cast<G>(static_cast<float>(L.u[r][lane]));
    wave_sync();
  }
  // surface term: surf = pr * cs -> dL/dpr (sum over bands), dL/dcs
  const float prr = h(__shfl(pr, sr < R ? sr : 0));
  if (lane < nr) L.pr[lane] = h(pr);
  if (cs && sr < nr) {
    if (d_cs) d_cs[(b0 + sr) * C + sc] = static_cast<G>(h(gl * prr));
  }
  if (lane < nr) {
    float g_pr = 0.0f;
    if (cs) {
      for (int c = 0; c < C; ++c) {
        const float csv = h(ld(cs, (b0 + lane) * C + c));
        g_pr = g_pr + h(L.g[lane][c] * csv);
      }
      g_pr = h(g_pr);
    }
    L.g_pr[lane] = g_pr;
  }
  // alpha rounded to 1 in f16 (sigma * delta > ~9): torch takes its zero-input backward
  // branches (prod_safe_zeros_backward, cumprod's first-zero formula) -- not restated
  // rounding for rounding; flagged to the caller, gradients of such a ray set to 0
  if (zmask && lane == 0) atomicAdd(zero_rays, __popc(zmask));
  wave_sync();
  // pass 2, reverse: reversed cumsum of cp * dL/dcp with an f16 accumulator
  // (cumprod_backward), then each sample's gradients in autograd's order
  _Float16 rc = 0.0f;  // lane r < nr: ray r's reversed cumsum, at j = N: cp_N * 0
  // a segment's inputs, fetched one segment ahead: z, colour, and the parked T and exp
  float zm_[R], z0_[R], zp_[R], ee_[R], tt_[R], col_[R][kMaxC];
  auto fetch2 = [&](int s0) {
    const int i = s0 + lane;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nr && lane < N - s0) {
        const int64_t k = (b0 + r) * N + i;
        const float* zr = z + (b0 + r) * N;
        z0_[r] = zr[i];
        zm_[r] = i > 0 ? zr[i - 1] : 0.0f;
        zp_[r] = i < N - 1 ? zr[i + 1] : 0.0f;
        ee_[r] = static_cast<float>(d_color[k * C]);
        tt_[r] = static_cast<float>(d_sigma[k]);
#pragma unroll
        for (int c = 0; c < kMaxC; ++c)
          if (c < C) col_[r][c] = ld(color, k * C + c);
      }
    }
  };
  fetch2(((N - 1) / kSeg) * kSeg);
  wave_sync();
  for (int s0 = ((N - 1) / kSeg) * kSeg; s0 >= 0; s0 -= kSeg) {
    const int n = N - s0 < kSeg ? N - s0 : kSeg;
    const int nv = (n + 7) & ~7;
    float czm[R], cz0[R], czp[R], cee[R], ctt[R], ccol[R][kMaxC];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      czm[r] = zm_[r]; cz0[r] = z0_[r]; czp[r] = zp_[r]; cee[r] = ee_[r]; ctt[r] = tt_[r];
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) ccol[r][c] = col_[r][c];
    }
    if (s0 > 0) fetch2(s0 - kSeg);
    float e_[R], dl_[R], q2_[R], gab_[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      e_[r] = dl_[r] = q2_[r] = gab_[r] = 0.0f;
      if (!(r < nr && lane < n)) {
        if (lane < nv) L.u[r][lane] = static_cast<_Float16>(kNegZero);
        continue;
      }
      const int64_t k = (b0 + r) * N + s0 + lane;
      if (zmask & (1u << r)) {
        L.u[r][lane] = static_cast<_Float16>(kNegZero);
        for (int c = 0; c < C; ++c) d_color[k * C + c] = static_cast<G>(0.0f);
        continue;
      }
      const Sample sm = from_e(cee[r], delta_z(czm[r], cz0[r], czp[r], zs, s0 + lane, N));
      const float Tk = ctt[r];
      const float w = h(sm.alpha * Tk);
      float gw = 0.0f;
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        if (c >= C) break;
        const float gc = L.g[r][c];
        const float col = h(ccol[r][c]);
        gw = gw + h(gc * col);                                    // sum_to_size over bands
        d_color[k * C + c] = static_cast<G>(h(gc * w));           // color * w -> color
      }
      gw = h(gw);
      gab_[r] = h(gw * Tk);                                       // alpha * T -> alpha
      const float g_T = h(gw * sm.alpha);                         // -> T
      L.u[r][lane] = static_cast<_Float16>(h(Tk * g_T));          // cp_k * dL/dcp_k
      e_[r] = sm.e;
      dl_[r] = sm.delta;
      q2_[r] = sm.q2;
    }
    wave_sync();
    if (lane < nr) {
      for (int l8 = nv - 8; l8 >= 0; l8 -= 8) {
        const h8v uv = *reinterpret_cast<const h8v*>(&L.u[lane][l8]);
        h8v rv;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
          rv[k] = rc;
          rc = rc + uv[k];  // = h(rc + u)
        }
        *reinterpret_cast<h8v*>(&L.rin[lane][l8]) = rv;
      }
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!(r < nr && lane < n)) continue;
      const int64_t k = (b0 + r) * N + s0 + lane;
      if (zmask & (1u << r)) {
        d_sigma[k] = static_cast<G>(0.0f);
        continue;
      }
      const float g_cpin = h(static_cast<float>(L.rin[r][lane]) / q2_[r]);  // cumprod bwd at k+1
      const float g_alpha_c = -g_cpin;                            // 1 - alpha + 1e-10
      float g_alpha;
      if (cs) {
        const float g_om = h(L.g_pr[r] * h(L.pr[r] / q2_[r]));    // prod backward
        g_alpha = h(h(-g_om + gab_[r]) + g_alpha_c);
      } else {
        g_alpha = h(gab_[r] + g_alpha_c);
      }
      const float g_x = h(-g_alpha * e_[r]);                      // 1 - exp(x)
      d_sigma[k] = static_cast<G>(-h(g_x * dl_[r]));              // -sigma * delta
    }
    wave_sync();
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

// Rays per wavefront: 2 from 8,192 rays up, 1 below (fewer rays leave SIMDs idle, and
// then one ray per wave's extra waves beat the shared scans); ANR_REF16_R = 1 / 2 / 4 / 8
// or anr_composite_ref16_set_rays overrides (r04 sweep in DESIGN.md §10). Halved until
// the band-sum lanes R * C fit the wave.
static int g_rays = 0;
static int rays_per_wave(int C, int64_t B) {
  static const int env = [] {
    const char* s = getenv("ANR_REF16_R");
    const int v = s ? atoi(s) : 0;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 0;
  }();
  int R = g_rays ? g_rays : (env ? env : (B >= 8192 ? 2 : 1));
  while (R > 1 && R * C > 64) R /= 2;
  return R;
}

}  // namespace ref16
}  // namespace anr

using namespace anr;

extern "C" int anr_composite_ref16_set_rays(int32_t rays_per_wave) {
  ANR_CHECK_ARG(rays_per_wave == 0 || rays_per_wave == 1 || rays_per_wave == 2 ||
                    rays_per_wave == 4 || rays_per_wave == 8,
                "anr_composite_ref16_set_rays: %d (0 = default, 1 / 2 / 4 / 8)", rays_per_wave);
  ref16::g_rays = rays_per_wave;
  return ANR_OK;
}

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
  const int R = ref16::rays_per_wave(C, B);
#define ANR_R16F(RR, T)                                                                        \
  hipLaunchKernelGGL((ref16::fwd_kernel<RR, T>), dim3(static_cast<unsigned>(ceil_div(B, RR))), \
                     dim3(64), 0, as_stream(stream), z, z_scale,                               \
                     static_cast<const T*>(color), static_cast<const T*>(sigma),               \
                     static_cast<const T*>(color_surf), B, N, C,                              \
                     static_cast<__half*>(color_map), static_cast<__half*>(color_map_atmo),  \
                     static_cast<__half*>(color_map_surf), static_cast<__half*>(weights),     \
                     static_cast<__half*>(alpha), static_cast<__half*>(color16),              \
                     static_cast<__half*>(sigma16))
#define ANR_R16F_T(T)                                                                         \
  switch (R) {                                                                                \
    case 1: ANR_R16F(1, T); break;                                                            \
    case 2: ANR_R16F(2, T); break;                                                            \
    case 4: ANR_R16F(4, T); break;                                                            \
    default: ANR_R16F(8, T); break;                                                           \
  }
  if (in_dtype == ANR_F16) { ANR_R16F_T(__half) } else { ANR_R16F_T(float) }
#undef ANR_R16F_T
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
  const int R = ref16::rays_per_wave(C, B);
#define ANR_R16B(RR, T, G)                                                                     \
  hipLaunchKernelGGL((ref16::bwd_kernel<RR, T, G>),                                           \
                     dim3(static_cast<unsigned>(ceil_div(B, RR))), dim3(64), 0,               \
                     as_stream(stream), z, z_scale,                                           \
                     static_cast<const T*>(color), static_cast<const T*>(sigma),               \
                     static_cast<const T*>(color_surf), B, N, C,                              \
                     static_cast<const __half*>(d_color_map), static_cast<G*>(d_color),       \
                     static_cast<G*>(d_sigma), static_cast<G*>(d_color_surf), zero_rays)
#define ANR_R16B_TG(T, G)                                                                     \
  switch (R) {                                                                                \
    case 1: ANR_R16B(1, T, G); break;                                                         \
    case 2: ANR_R16B(2, T, G); break;                                                         \
    case 4: ANR_R16B(4, T, G); break;                                                         \
    default: ANR_R16B(8, T, G); break;                                                        \
  }
  if (in_dtype == ANR_F16) {
    if (out_dtype == ANR_F16) { ANR_R16B_TG(__half, __half) } else { ANR_R16B_TG(__half, float) }
  } else {
    if (out_dtype == ANR_F16) { ANR_R16B_TG(float, __half) } else { ANR_R16B_TG(float, float) }
  }
#undef ANR_R16B_TG
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
