// K1 + K2: stratified ray sampler fused with the HARP2 "horizontal" preprocessor.
//
// Reference semantics (file:line relative to nasa/atmospheric-neural-rendering):
//   sample_uniform_bins   src/atmonr/samplers.py:8-47
//   preprocess_coords     src/atmonr/datasets/harp2.py:372-386
//   cartesian_to_horizontal (Bowring)  src/atmonr/geospatial/wgs_84.py:56-97
//   Instant-NGP remap     src/atmonr/pipelines/instant_ngp.py:149,160
//
// One thread per sample. The reference runs ~30 separate fp64 elementwise passes over
// (B,N,3); here each sample is read once (ray data is shared through L1/L2 by the 1024
// samples of a ray) and the three outputs are written once. Each arithmetic step keeps
// the reference's operation order and rounding points: f32 where torch computes in f32,
// f64 where the fp64 `offset` promotes (harp2.py:376). FMA contraction is disabled so
// the f32 parts (z, pts) are bit-identical to torch's for identical draws u.
#pragma clang fp contract(off)

#include "anr_common.h"

namespace anr {

// WGS-84 constants, wgs_84.py:16-20 (Python doubles).
constexpr double kA = 6378137.0;
constexpr double kB = 6356752.314245;
constexpr double kE = (kA * kA - kB * kB) / (kA * kA);
constexpr double kE2 = (kA * kA - kB * kB) / (kB * kB);
constexpr double kPi = 3.141592653589793;  // torch.pi

struct PrepDev {
  int mode, shift_lon, ngp_remap;
  float scale_f;  // (float)scale: torch multiplies an f32 tensor by a Python float in f32
  double scale_d;
  double offset[3];
  double lat_min, lat_range, lon_min, lon_range, h;
  double k_lat, k_lon, k_h;  // 2 / lat_range, 2 / lon_range, 2 / h (host-computed)
  float alt_compress;
};

// Python-style modulus (torch.remainder for doubles): a - floor(a/b)*b.
__device__ __forceinline__ double py_mod(double a, double b) {
  double r = fmod(a, b);
  if (r != 0.0 && ((r < 0.0) != (b < 0.0))) r += b;
  return r;
}


// preprocess_coords for one point p (normalized scene frame) -> coords (f32).
// T = float: the training path (f32 points; the result is cast to f32 before the clip and
// the NGP remap, harp2.py:384-385). T = double: the extract path (extract.py:206 feeds
// f64 points, so clip and remap stay in f64 and only the final value is rounded — tcnn
// casts the encoder input to f32). kClip=false stops before clip(-1, 1) (the backward's
// clamp mask needs the raw value).
template <typename T = float, bool kClip = true>
__device__ __forceinline__ void preprocess_point(const PrepDev& P, T px, T py, T pz,
                                                 float* out) {
  T cx = px, cy = py, cz = pz;
  if (P.mode == 1) {
    // coords_xyz * scale + offset (f64), harp2.py:376; an f32 tensor times a Python float
    // is computed in f32 first
    double x, y, z;
    if constexpr (sizeof(T) == 4) {
      x = static_cast<double>(px * P.scale_f) + P.offset[0];
      y = static_cast<double>(py * P.scale_f) + P.offset[1];
      z = static_cast<double>(pz * P.scale_f) + P.offset[2];
    } else {
      x = px * P.scale_d + P.offset[0];
      y = py * P.scale_d + P.offset[1];
      z = pz * P.scale_d + P.offset[2];
    }
    // cartesian_to_horizontal, wgs_84.py:83-97. The sines and cosines of the angles the
    // reference builds with atan2 are formed from the atan2 arguments instead
    // (sin(atan2(p, q)) = p / hypot, cos = q / hypot; cos(lon) = x / D), and every f64
    // division but five is a multiplication by a reciprocal formed once (alt = x / (cos lat
    // cos lon) = D rl / X; the degree and range scalings multiply by host-computed
    // constants): each value moves by an f64 ulp or two, 2^-29 of the f32 rounding of the
    // outputs, at about half of the f64 instructions (this kernel is f64-issue-bound).
    // Only lon and lat themselves need atan2.
    const double lon = atan2(y, x);
    const double D = sqrt(x * x + y * y);
    const double iD = 1.0 / D;
    const double t = z * iD, k = kA / kB;
    const double ru = sqrt(t * t + k * k);
    const double iru = 1.0 / ru;
    const double su = t * iru, cu = k * iru;
    const double Y = z + (kE2 * kB) * (su * su * su);
    const double X = D - (kE * kA) * (cu * cu * cu);
    const double lat = atan2(Y, X);
    const double rl = sqrt(X * X + Y * Y);
    const double sl = Y / rl;
    const double Nr = kA / sqrt(1.0 - kE * (sl * sl));
    // x / (cos(lat) cos(lon)) (wgs_84.py:96) with cos(lon) = x / D and cos(lat) = X / rl.
    // Deliberate deviation at x = 0 (lon = +-90 deg): the reference divides 0 by cos(lon)
    // ~ 6e-17 (a finite value that depends on atan2's last ulp, or inf / NaN), this form
    // stays finite; no HARP2 scene here reaches it (scenes centred on lon = +-90 deg would)
    const double alt = (D * rl) / X - Nr;
    constexpr double kDeg = 180.0 / kPi;
    double lat_d = lat * kDeg;
    double lon_d = lon * kDeg;
    if (P.shift_lon) lon_d = py_mod(lon_d, 360.0) - 180.0;  // harp2.py:379-380
    // harp2.py:381-383
    const double a = (lat_d - P.lat_min) * P.k_lat - 1.0;
    const double b = (lon_d - P.lon_min) * P.k_lon - 1.0;
    const double c = alt * P.k_h - 1.0;
    // .to(input dtype) then clip(-1, 1), harp2.py:384-385
    cx = static_cast<T>(a);
    cy = static_cast<T>(b);
    cz = static_cast<T>(c);
    if (kClip) {
      cx = cx < T(-1) ? T(-1) : (cx > T(1) ? T(1) : cx);  // NaN propagates, as torch.clip
      cy = cy < T(-1) ? T(-1) : (cy > T(1) ? T(1) : cy);
      cz = cz < T(-1) ? T(-1) : (cz > T(1) ? T(1) : cz);
    }
  }
  if (P.ngp_remap) {
    // pts = (pts + 1) / 2 ; pts[..., 2] /= alt_compress_factor (instant_ngp.py:149,160)
    cx = (cx + T(1)) / T(2);
    cy = (cy + T(1)) / T(2);
    cz = (cz + T(1)) / T(2);
    cz = cz / static_cast<T>(P.alt_compress);
  }
  out[0] = static_cast<float>(cx);
  out[1] = static_cast<float>(cy);
  out[2] = static_cast<float>(cz);
}

// ---- backward of preprocess_point (NeRF back-propagates into the sample points through
// the fp64 preprocessor, harp2.py:372-386): forward-mode dual numbers over (px, py, pz).
struct D3 {
  double v, d[3];
};
__device__ __forceinline__ D3 dc(double v) { return D3{v, {0.0, 0.0, 0.0}}; }
__device__ __forceinline__ D3 operator+(D3 a, D3 b) {
  return D3{a.v + b.v, {a.d[0] + b.d[0], a.d[1] + b.d[1], a.d[2] + b.d[2]}};
}
__device__ __forceinline__ D3 operator-(D3 a, D3 b) {
  return D3{a.v - b.v, {a.d[0] - b.d[0], a.d[1] - b.d[1], a.d[2] - b.d[2]}};
}
__device__ __forceinline__ D3 operator*(D3 a, D3 b) {
  return D3{a.v * b.v, {a.d[0] * b.v + a.v * b.d[0], a.d[1] * b.v + a.v * b.d[1],
                        a.d[2] * b.v + a.v * b.d[2]}};
}
__device__ __forceinline__ D3 operator/(D3 a, D3 b) {
  const double q = a.v / b.v, ib = 1.0 / b.v;
  return D3{q, {(a.d[0] - q * b.d[0]) * ib, (a.d[1] - q * b.d[1]) * ib, (a.d[2] - q * b.d[2]) * ib}};
}
__device__ __forceinline__ D3 scale(D3 a, double k) {
  return D3{a.v * k, {a.d[0] * k, a.d[1] * k, a.d[2] * k}};
}
__device__ __forceinline__ D3 dsin(D3 a) {
  const double c = cos(a.v);
  return D3{sin(a.v), {c * a.d[0], c * a.d[1], c * a.d[2]}};
}
__device__ __forceinline__ D3 dcos(D3 a) {
  const double s = -sin(a.v);
  return D3{cos(a.v), {s * a.d[0], s * a.d[1], s * a.d[2]}};
}
__device__ __forceinline__ D3 dsqrt(D3 a) {
  const double r = sqrt(a.v), k = 0.5 / r;
  return D3{r, {k * a.d[0], k * a.d[1], k * a.d[2]}};
}
__device__ __forceinline__ D3 datan2(D3 y, D3 x) {
  const double den = x.v * x.v + y.v * y.v;
  D3 r{atan2(y.v, x.v), {}};
  for (int k = 0; k < 3; ++k) r.d[k] = (x.v * y.d[k] - y.v * x.d[k]) / den;
  return r;
}

// d out_j / d p_k of preprocess_point (values follow the forward; the f32 cast passes the
// gradient through, clip(-1, 1) passes it where -1 <= value <= 1, as torch.clamp does).
__device__ void preprocess_jacobian(const PrepDev& P, float px, float py, float pz,
                                    double J[3][3]) {
  for (int j = 0; j < 3; ++j)
    for (int k = 0; k < 3; ++k) J[j][k] = j == k ? 1.0 : 0.0;
  if (P.mode == 1) {
    const double sf = static_cast<double>(P.scale_f);
    const D3 x{static_cast<double>(px * P.scale_f) + P.offset[0], {sf, 0.0, 0.0}};
    const D3 y{static_cast<double>(py * P.scale_f) + P.offset[1], {0.0, sf, 0.0}};
    const D3 z{static_cast<double>(pz * P.scale_f) + P.offset[2], {0.0, 0.0, sf}};
    const D3 lon = datan2(y, x);
    const D3 D = dsqrt(x * x + y * y);
    const D3 u = datan2(z / D, dc(0.0 + kA / kB));
    const D3 su = dsin(u), cu = dcos(u);
    const D3 lat = datan2(z + scale(su * su * su, kE2 * kB), D - scale(cu * cu * cu, kE * kA));
    const D3 sl = dsin(lat);
    const D3 Nr = dc(kA) / dsqrt(dc(1.0) - scale(sl * sl, kE));
    const D3 alt = x / (dcos(lat) * dcos(lon)) - Nr;
    const D3 o[3] = {scale(scale(lat, 180.0 / kPi), 2.0 / P.lat_range),
                     scale(scale(lon, 180.0 / kPi), 2.0 / P.lon_range),
                     scale(alt, 2.0 / P.h)};
    float val[3];  // f32 values before clip and NGP remap: torch.clamp's gradient mask
    PrepDev Q = P;
    Q.ngp_remap = 0;
    preprocess_point<float, false>(Q, px, py, pz, val);
    for (int j = 0; j < 3; ++j) {
      const bool pass = val[j] >= -1.0f && val[j] <= 1.0f;
      for (int k = 0; k < 3; ++k) J[j][k] = pass ? o[j].d[k] : 0.0;
    }
  }
  if (P.ngp_remap) {
    for (int k = 0; k < 3; ++k) {
      J[0][k] *= 0.5;
      J[1][k] *= 0.5;
      J[2][k] = J[2][k] * 0.5 / static_cast<double>(P.alt_compress);
    }
  }
}

__global__ void __launch_bounds__(256) preprocess_points_bwd_kernel(
    const float* __restrict__ pts, int64_t P_n, PrepDev P, const float* __restrict__ dcoords,
    float* __restrict__ dpts) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= P_n) return;
  double J[3][3];
  preprocess_jacobian(P, pts[idx * 3 + 0], pts[idx * 3 + 1], pts[idx * 3 + 2], J);
  const double g[3] = {dcoords[idx * 3 + 0], dcoords[idx * 3 + 1], dcoords[idx * 3 + 2]};
  for (int k = 0; k < 3; ++k)
    dpts[idx * 3 + k] = static_cast<float>(g[0] * J[0][k] + g[1] * J[1][k] + g[2] * J[2][k]);
}

__global__ void __launch_bounds__(256) sample_uniform_bins_kernel(
    const float* __restrict__ origin, const float* __restrict__ dir,
    const float* __restrict__ len, const float* __restrict__ u,
    const float* __restrict__ bins, int64_t B, int32_t N, float* __restrict__ pts,
    float* __restrict__ zout, PrepDev P, int do_prep, float* __restrict__ coords) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= B * N) return;
  const int64_t b = idx / N;
  const int32_t i = static_cast<int32_t>(idx - b * N);
  // samplers.py:42 — z = (bins[:-1] + t_in_bin / n_bins) * len
  const float t = u ? u[idx] : 0.5f;
  const float z = (bins[i] + t / static_cast<float>(N)) * len[b];
  // samplers.py:45 — pts = origin + dir * z
  const float px = origin[b * 3 + 0] + dir[b * 3 + 0] * z;
  const float py = origin[b * 3 + 1] + dir[b * 3 + 1] * z;
  const float pz = origin[b * 3 + 2] + dir[b * 3 + 2] * z;
  if (zout) zout[idx] = z;
  if (pts) {
    pts[idx * 3 + 0] = px;
    pts[idx * 3 + 1] = py;
    pts[idx * 3 + 2] = pz;
  }
  if (do_prep) {
    float c[3];
    preprocess_point(P, px, py, pz, c);
    coords[idx * 3 + 0] = c[0];
    coords[idx * 3 + 1] = c[1];
    coords[idx * 3 + 2] = c[2];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) preprocess_points_kernel(
    const T* __restrict__ pts, int64_t P_n, PrepDev P, float* __restrict__ coords) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= P_n) return;
  float c[3];
  preprocess_point<T>(P, pts[idx * 3 + 0], pts[idx * 3 + 1], pts[idx * 3 + 2], c);
  coords[idx * 3 + 0] = c[0];
  coords[idx * 3 + 1] = c[1];
  coords[idx * 3 + 2] = c[2];
}

static PrepDev make_prep(const anr_prep_params* p) {
  PrepDev d{};
  d.mode = p->mode;
  d.shift_lon = p->shift_lon;
  d.ngp_remap = p->ngp_remap;
  d.scale_f = static_cast<float>(p->scale);
  d.scale_d = p->scale;
  for (int k = 0; k < 3; ++k) d.offset[k] = p->offset[k];
  d.lat_min = p->lat_min;
  d.lat_range = p->lat_range;
  d.lon_min = p->lon_min;
  d.lon_range = p->lon_range;
  d.h = p->ray_origin_height;
  d.k_lat = 2.0 / p->lat_range;
  d.k_lon = 2.0 / p->lon_range;
  d.k_h = 2.0 / p->ray_origin_height;
  d.alt_compress = p->alt_compress;
  return d;
}

}  // namespace anr

extern "C" int anr_sample_uniform_bins(const float* origin, const float* dir,
                                       const float* len, const float* u,
                                       const float* bins, int64_t B, int32_t N,
                                       float* pts, float* z, const anr_prep_params* prep,
                                       float* coords, anr_stream_t stream) {
  using namespace anr;
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(origin && dir && len && bins, "anr_sample_uniform_bins: null ray input");
  ANR_CHECK_ARG(B >= 0 && N > 0, "anr_sample_uniform_bins: bad shape B=%lld N=%d",
                (long long)B, N);
  ANR_CHECK_ARG((coords == nullptr) == (prep == nullptr),
                "anr_sample_uniform_bins: coords and prep must be given together");
  if (B == 0) return ANR_OK;
  PrepDev P{};
  if (prep) {
    ANR_CHECK_ARG(prep->mode == 0 || prep->mode == 1, "anr_sample_uniform_bins: bad mode");
    ANR_CHECK_ARG(prep->mode == 0 || (prep->lat_range != 0.0 && prep->lon_range != 0.0 &&
                                      prep->ray_origin_height != 0.0),
                  "anr_sample_uniform_bins: degenerate preprocessor ranges");
    P = make_prep(prep);
  }
  const int64_t total = B * N;
  const int threads = 256;
  hipLaunchKernelGGL(sample_uniform_bins_kernel, dim3(ceil_div(total, threads)),
                     dim3(threads), 0, as_stream(stream), origin, dir, len, u, bins, B, N,
                     pts, z, P, prep ? 1 : 0, coords);
  ANR_CHECK_LAUNCH("anr_sample_uniform_bins");
  return ANR_OK;
}

extern "C" int anr_preprocess_points(const float* pts, int64_t P_n,
                                     const anr_prep_params* prep, float* coords,
                                     anr_stream_t stream) {
  using namespace anr;
  if (P_n == 0) return ANR_OK;
  ANR_CHECK_ARG(pts && prep && coords, "anr_preprocess_points: null argument");
  ANR_CHECK_ARG(P_n >= 0, "anr_preprocess_points: negative size");
  ANR_CHECK_ARG(prep->mode == 0 || prep->mode == 1, "anr_preprocess_points: bad mode");
  if (P_n == 0) return ANR_OK;
  PrepDev P = make_prep(prep);
  hipLaunchKernelGGL(preprocess_points_kernel<float>, dim3(ceil_div(P_n, 256)), dim3(256), 0,
                     as_stream(stream), pts, P_n, P, coords);
  ANR_CHECK_LAUNCH("anr_preprocess_points");
  return ANR_OK;
}

extern "C" int anr_preprocess_points_f64(const double* pts, int64_t P_n,
                                         const anr_prep_params* prep, float* coords,
                                         anr_stream_t stream) {
  using namespace anr;
  if (P_n == 0) return ANR_OK;
  ANR_CHECK_ARG(pts && prep && coords, "anr_preprocess_points_f64: null argument");
  ANR_CHECK_ARG(P_n >= 0, "anr_preprocess_points_f64: negative size");
  ANR_CHECK_ARG(prep->mode == 0 || prep->mode == 1, "anr_preprocess_points_f64: bad mode");
  PrepDev P = make_prep(prep);
  hipLaunchKernelGGL(preprocess_points_kernel<double>, dim3(ceil_div(P_n, 256)), dim3(256), 0,
                     as_stream(stream), pts, P_n, P, coords);
  ANR_CHECK_LAUNCH("anr_preprocess_points_f64");
  return ANR_OK;
}

extern "C" int anr_preprocess_points_bwd(const float* pts, int64_t P, const anr_prep_params* prep,
                                         const float* d_coords, float* d_pts,
                                         anr_stream_t stream) {
  ANR_CHECK_ARG(prep != nullptr && P >= 0, "anr_preprocess_points_bwd: bad arguments");
  if (P == 0) return ANR_OK;
  ANR_CHECK_ARG(pts && d_coords && d_pts, "anr_preprocess_points_bwd: null pointer");
  const anr::PrepDev d = anr::make_prep(prep);
  hipLaunchKernelGGL(anr::preprocess_points_bwd_kernel, dim3(static_cast<unsigned>((P + 255) / 256)),
                     dim3(256), 0, reinterpret_cast<hipStream_t>(stream), pts, P, d, d_coords, d_pts);
  ANR_CHECK_LAUNCH("anr_preprocess_points_bwd");
  return ANR_OK;
}
