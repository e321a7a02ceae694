// K5: SphericalHarmonics, Identity and constant-padding encodings — the members of the
// tinycudann "Composite" encodings at src/atmonr/pipelines/instant_ngp.py:69-72 (dir
// encoder: SH degree 2 on the ray direction + Identity on pos_mlp features, called at
// :165-169) and :78-80 (surface encoder: 2-D HashGrid + SH degree 2, called at :173).
// tcnn semantics (unpinned in the reference): SH inputs in [0,1] are
// remapped to 2x-1; degree d yields d*d real SH terms in the standard order; encodings
// are padded with 1.0 up to the network's input width.

#include "anr_common.h"

#include <stdarg.h>

namespace anr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// SH basis up to degree 4 (16 terms), input already in [-1, 1].
__device__ __forceinline__ void sh_eval(int degree, float x, float y, float z, float* o) {
  const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
  o[0] = 0.28209479177387814f;
  if (degree <= 1) return;
  o[1] = -0.48860251190291987f * y;
  o[2] = 0.48860251190291987f * z;
  o[3] = -0.48860251190291987f * x;
  if (degree <= 2) return;
  o[4] = 1.0925484305920792f * xy;
  o[5] = -1.0925484305920792f * yz;
  o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
  o[7] = -1.0925484305920792f * xz;
  o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
  if (degree <= 3) return;
  o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
  o[10] = 2.8906114426405538f * xy * z;
  o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
  o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
  o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
  o[14] = 1.4453057213202769f * z * (x2 - y2);
  o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

// d o[k] / d(x, y, z) for the same basis.
__device__ __forceinline__ void sh_grad(int degree, float x, float y, float z,
                                        float (*g)[3]) {
  for (int k = 0; k < 16; ++k) g[k][0] = g[k][1] = g[k][2] = 0.0f;
  if (degree <= 1) return;
  const float c1 = 0.48860251190291987f;
  g[1][1] = -c1;
  g[2][2] = c1;
  g[3][0] = -c1;
  if (degree <= 2) return;
  const float c2 = 1.0925484305920792f, c3 = 0.94617469575755997f, c5 = 0.54627421529603959f;
  g[4][0] = c2 * y; g[4][1] = c2 * x;
  g[5][1] = -c2 * z; g[5][2] = -c2 * y;
  g[6][2] = 2.0f * c3 * z;
  g[7][0] = -c2 * z; g[7][2] = -c2 * x;
  g[8][0] = 2.0f * c5 * x; g[8][1] = -2.0f * c5 * y;
  if (degree <= 3) return;
  const float a = 0.59004358992664352f, b = 2.8906114426405538f, c = 0.45704579946446572f,
              d = 0.3731763325901154f, e = 1.4453057213202769f;
  const float x2 = x * x, y2 = y * y, z2 = z * z;
  g[9][0] = -6.0f * a * x * y; g[9][1] = a * (3.0f * y2 - 3.0f * x2);
  g[10][0] = b * y * z; g[10][1] = b * x * z; g[10][2] = b * x * y;
  g[11][1] = c * (1.0f - 5.0f * z2); g[11][2] = -10.0f * c * y * z;
  g[12][2] = d * (15.0f * z2 - 3.0f);
  g[13][0] = c * (1.0f - 5.0f * z2); g[13][2] = -10.0f * c * x * z;
  g[14][0] = 2.0f * e * x * z; g[14][1] = -2.0f * e * y * z; g[14][2] = e * (x2 - y2);
  g[15][0] = a * (3.0f * y2 - 3.0f * x2); g[15][1] = 6.0f * a * x * y;
}

__global__ void __launch_bounds__(256) sh_fwd_kernel(int degree, const float* __restrict__ x,
                                                     int64_t x_stride, int64_t M, void* out,
                                                     int32_t odt, int64_t out_stride) {
  const int64_t m = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float o[16];
  sh_eval(degree, x[m * x_stride + 0] * 2.0f - 1.0f, x[m * x_stride + 1] * 2.0f - 1.0f,
          x[m * x_stride + 2] * 2.0f - 1.0f, o);
  const int n = degree * degree;
  for (int k = 0; k < n; ++k) store_dyn(out, odt, m * out_stride + k, o[k]);
}

__global__ void __launch_bounds__(256) sh_bwd_kernel(int degree, const float* __restrict__ x,
                                                     int64_t x_stride, int64_t M,
                                                     const void* dout, int32_t gdt,
                                                     int64_t dout_stride, float* dx,
                                                     int64_t dx_stride) {
  const int64_t m = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float g[16][3];
  sh_grad(degree, x[m * x_stride + 0] * 2.0f - 1.0f, x[m * x_stride + 1] * 2.0f - 1.0f,
          x[m * x_stride + 2] * 2.0f - 1.0f, g);
  float acc[3] = {0.0f, 0.0f, 0.0f};
  const int n = degree * degree;
  for (int k = 0; k < n; ++k) {
    const float go = load_dyn(dout, gdt, m * dout_stride + k);
    acc[0] += go * g[k][0];
    acc[1] += go * g[k][1];
    acc[2] += go * g[k][2];
  }
  // chain rule through the 2x-1 remap
  dx[m * dx_stride + 0] += 2.0f * acc[0];
  dx[m * dx_stride + 1] += 2.0f * acc[1];
  dx[m * dx_stride + 2] += 2.0f * acc[2];
}

__global__ void __launch_bounds__(256) identity_kernel(const void* x, int32_t xdt,
                                                       int64_t x_stride, int64_t M, int32_t n,
                                                       void* out, int32_t odt,
                                                       int64_t out_stride) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= M * n) return;
  const int64_t m = t / n;
  const int32_t j = static_cast<int32_t>(t - m * n);
  store_dyn(out, odt, m * out_stride + j, load_dyn(x, xdt, m * x_stride + j));
}

__global__ void __launch_bounds__(256) fill_cols_kernel(void* out, int32_t odt,
                                                        int64_t out_stride, int64_t M,
                                                        int32_t n, float value) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= M * n) return;
  const int64_t m = t / n;
  const int32_t j = static_cast<int32_t>(t - m * n);
  store_dyn(out, odt, m * out_stride + j, value);
}

}  // namespace anr

extern "C" int anr_abi_version(void) { return ANR_ABI_VERSION; }
extern "C" const char* anr_last_error(void) { return anr::g_err; }

extern "C" int anr_sh_fwd(int32_t degree, const float* x, int64_t x_stride, int64_t M,
                          void* out, int32_t out_dtype, int64_t out_stride,
                          anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(x && out, "anr_sh_fwd: null argument");
  ANR_CHECK_ARG(degree >= 1 && degree <= 4, "anr_sh_fwd: degree %d not in [1,4]", degree);
  ANR_CHECK_ARG(x_stride >= 3 && out_stride >= degree * degree && M >= 0,
                "anr_sh_fwd: bad shape/stride");
  ANR_CHECK_ARG(out_dtype == ANR_F16 || out_dtype == ANR_F32, "anr_sh_fwd: bad dtype");
  if (M == 0) return ANR_OK;
  hipLaunchKernelGGL(sh_fwd_kernel, dim3(ceil_div(M, 256)), dim3(256), 0, as_stream(stream),
                     degree, x, x_stride, M, out, out_dtype, out_stride);
  ANR_CHECK_LAUNCH("anr_sh_fwd");
  return ANR_OK;
}

extern "C" int anr_sh_bwd(int32_t degree, const float* x, int64_t x_stride, int64_t M,
                          const void* dout, int32_t dout_dtype, int64_t dout_stride,
                          float* dx, int64_t dx_stride, anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(x && dout && dx, "anr_sh_bwd: null argument");
  ANR_CHECK_ARG(degree >= 1 && degree <= 4, "anr_sh_bwd: degree %d not in [1,4]", degree);
  ANR_CHECK_ARG(x_stride >= 3 && dx_stride >= 3 && dout_stride >= degree * degree && M >= 0,
                "anr_sh_bwd: bad shape/stride");
  ANR_CHECK_ARG(dout_dtype == ANR_F16 || dout_dtype == ANR_F32, "anr_sh_bwd: bad dtype");
  if (M == 0) return ANR_OK;
  hipLaunchKernelGGL(sh_bwd_kernel, dim3(ceil_div(M, 256)), dim3(256), 0, as_stream(stream),
                     degree, x, x_stride, M, dout, dout_dtype, dout_stride, dx, dx_stride);
  ANR_CHECK_LAUNCH("anr_sh_bwd");
  return ANR_OK;
}

extern "C" int anr_identity(const void* x, int32_t x_dtype, int64_t x_stride, int64_t M,
                            int32_t n, void* out, int32_t out_dtype, int64_t out_stride,
                            anr_stream_t stream) {
  using namespace anr;
  if (M == 0 || n == 0) return ANR_OK;
  ANR_CHECK_ARG(x && out, "anr_identity: null argument");
  ANR_CHECK_ARG(n >= 0 && M >= 0 && x_stride >= n && out_stride >= n,
                "anr_identity: bad shape/stride");
  ANR_CHECK_ARG((x_dtype == ANR_F16 || x_dtype == ANR_F32) &&
                    (out_dtype == ANR_F16 || out_dtype == ANR_F32),
                "anr_identity: bad dtype");
  if (M == 0 || n == 0) return ANR_OK;
  hipLaunchKernelGGL(identity_kernel, dim3(ceil_div(M * n, 256)), dim3(256), 0,
                     as_stream(stream), x, x_dtype, x_stride, M, n, out, out_dtype,
                     out_stride);
  ANR_CHECK_LAUNCH("anr_identity");
  return ANR_OK;
}

extern "C" int anr_fill_cols(void* out, int32_t out_dtype, int64_t out_stride, int64_t M,
                             int32_t n, float value, anr_stream_t stream) {
  using namespace anr;
  if (M == 0 || n == 0) return ANR_OK;
  ANR_CHECK_ARG(out, "anr_fill_cols: null argument");
  ANR_CHECK_ARG(n >= 0 && M >= 0 && out_stride >= n, "anr_fill_cols: bad shape/stride");
  ANR_CHECK_ARG(out_dtype == ANR_F16 || out_dtype == ANR_F32, "anr_fill_cols: bad dtype");
  if (M == 0 || n == 0) return ANR_OK;
  hipLaunchKernelGGL(fill_cols_kernel, dim3(ceil_div(M * n, 256)), dim3(256), 0,
                     as_stream(stream), out, out_dtype, out_stride, M, n, value);
  ANR_CHECK_LAUNCH("anr_fill_cols");
  return ANR_OK;
}
