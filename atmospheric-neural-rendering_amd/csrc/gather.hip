// Ray-batch gather and the Instant-NGP surface input: the per-step glue in front of K1.
//
// anr_gather_rows replaces the per-field indexing of HARP2Dataset.__getitem__ /
// __getbatch__ (src/atmonr/datasets/harp2.py:392-420; one torch index kernel per ray
// field) with one
// launch that copies every field of the selected rays. anr_ingp_surface_input replaces
// the four elementwise passes and the cat of InstantNGPPipeline.forward
// (src/atmonr/pipelines/instant_ngp.py:143,150,173): pts_surf = (o + d * len + 1) / 2,
// surf_in = [pts_surf[:, :2] | d], rounded exactly as torch rounds those f32 ops.

#pragma clang fp contract(off)

#include "anr_common.h"

namespace anr {

struct GatherCols {
  anr_gather_col c[ANR_GATHER_MAX_COLS];
  int32_t n;
};

// One thread per (row, 4-byte word of one column's row); columns are looped so a
// thread handles the same word index of every column (rows are 4-byte multiples).
__global__ void __launch_bounds__(256) gather_rows_kernel(const int64_t* __restrict__ idx,
                                                          int64_t B, GatherCols cols,
                                                          int32_t max_words) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t row = t / max_words;
  const int32_t w = static_cast<int32_t>(t - row * max_words);
  if (row >= B) return;
  const int64_t src_row = idx[row];
  for (int k = 0; k < cols.n; ++k) {
    const int32_t words = static_cast<int32_t>(cols.c[k].row_bytes >> 2);
    if (w < words) {
      const uint32_t* s = static_cast<const uint32_t*>(cols.c[k].src);
      uint32_t* d = static_cast<uint32_t*>(cols.c[k].dst);
      d[row * words + w] = s[src_row * words + w];
    }
  }
}

__global__ void __launch_bounds__(256) surface_input_kernel(const float* __restrict__ origin,
                                                            const float* __restrict__ dir,
                                                            const float* __restrict__ len,
                                                            int64_t B, float* __restrict__ out) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float l = len[b];
  float d[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) d[k] = dir[b * 3 + k];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float p = origin[b * 3 + k] + d[k] * l;  // o + d * len[:, None]
    out[b * 5 + k] = (p + 1.0f) / 2.0f;             // (pts_surf + 1) / 2
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) out[b * 5 + 2 + k] = d[k];
}

}  // namespace anr

extern "C" int anr_gather_rows(const int64_t* idx, int64_t B, int32_t n_cols,
                               const anr_gather_col* cols, anr_stream_t stream) {
  using namespace anr;
  if (B == 0 || n_cols == 0) return ANR_OK;
  ANR_CHECK_ARG(idx && cols && B > 0, "anr_gather_rows: null argument");
  ANR_CHECK_ARG(n_cols > 0 && n_cols <= ANR_GATHER_MAX_COLS, "anr_gather_rows: %d columns",
                n_cols);
  GatherCols gc{};
  gc.n = n_cols;
  int32_t max_words = 1;
  for (int k = 0; k < n_cols; ++k) {
    ANR_CHECK_ARG(cols[k].src && cols[k].dst, "anr_gather_rows: null column %d", k);
    ANR_CHECK_ARG(cols[k].row_bytes > 0 && cols[k].row_bytes % 4 == 0 &&
                      cols[k].row_bytes <= 4096,
                  "anr_gather_rows: column %d row_bytes %lld", k,
                  static_cast<long long>(cols[k].row_bytes));
    gc.c[k] = cols[k];
    const int32_t w = static_cast<int32_t>(cols[k].row_bytes >> 2);
    if (w > max_words) max_words = w;
  }
  const int64_t threads = B * max_words;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(static_cast<unsigned>(ceil_div(threads, 256))),
                     dim3(256), 0, as_stream(stream), idx, B, gc, max_words);
  ANR_CHECK_LAUNCH("anr_gather_rows");
  return ANR_OK;
}

extern "C" int anr_ingp_surface_input(const float* origin, const float* dir, const float* len,
                                      int64_t B, float* out, anr_stream_t stream) {
  using namespace anr;
  if (B == 0) return ANR_OK;
  ANR_CHECK_ARG(origin && dir && len && out && B > 0, "anr_ingp_surface_input: null argument");
  hipLaunchKernelGGL(surface_input_kernel, dim3(static_cast<unsigned>(ceil_div(B, 256))),
                     dim3(256), 0, as_stream(stream), origin, dir, len, B, out);
  ANR_CHECK_LAUNCH("anr_ingp_surface_input");
  return ANR_OK;
}
