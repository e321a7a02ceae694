// Occupancy-grid sample culling for the Instant-NGP path (beyond the reference, which
// samples every ray uniformly at instant_ngp.py:145; BASELINE.json configs[4]).
//
// A grid of gx x gy x gz cells over the hash-grid domain [0,1] x [0,1] x [0, 1/alt] holds
// one occupancy byte per cell. The sampler's coordinates (ray-major, B x N) are culled
// to the samples whose cell is occupied, in two launches with an exclusive scan between
// them (done by the caller): count per block, then compact. Compaction keeps the sample
// order inside a block and blocks in order, so the kept samples stay ray-major (the hash
// walkers rely on consecutive samples sharing cells) and the result is deterministic.
// Culled samples keep sigma = 0 (their alpha is exactly 0 in the composite).

#include "anr_common.h"

namespace anr {

constexpr int kOccThreads = 256;
constexpr int kOccItems = 4;  // samples per thread
constexpr int kOccBlock = kOccThreads * kOccItems;

struct OccGrid {
  const uint8_t* occ;
  int32_t gx, gy, gz;
  float zmul;  // z in the hash domain * zmul -> [0, 1] (the Instant-NGP alt compression)
};

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

__device__ __forceinline__ bool occupied(const OccGrid& g, const float* p) {
  const int ix = clampi(static_cast<int>(floorf(p[0] * g.gx)), g.gx - 1);
  const int iy = clampi(static_cast<int>(floorf(p[1] * g.gy)), g.gy - 1);
  const int iz = clampi(static_cast<int>(floorf(p[2] * g.zmul * g.gz)), g.gz - 1);
  return g.occ[(static_cast<int64_t>(iz) * g.gy + iy) * g.gx + ix] != 0;
}

// Block-wide exclusive scan of one small count per thread (4 waves).
__device__ __forceinline__ int block_excl_scan(int v, int* total) {
  __shared__ int wsum[kOccThreads / kWave];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kOccThreads / kWave; ++w) {
    if (w < wave) base += wsum[w];
    tot += wsum[w];
  }
  *total = tot;
  return base + x - v;
}

__global__ void __launch_bounds__(kOccThreads) occ_count_kernel(const float* __restrict__ x,
                                                                int64_t M, OccGrid g,
                                                                int32_t* __restrict__ counts) {
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * kOccBlock + threadIdx.x * kOccItems;
  int c = 0;
#pragma unroll
  for (int i = 0; i < kOccItems; ++i)
    if (m0 + i < M && occupied(g, x + (m0 + i) * 3)) ++c;
  int total;
  block_excl_scan(c, &total);
  if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kOccThreads) occ_compact_kernel(
    const float* __restrict__ x, int64_t M, OccGrid g, const int64_t* __restrict__ offsets,
    int32_t* __restrict__ rows, float* __restrict__ xc) {
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * kOccBlock + threadIdx.x * kOccItems;
  bool keep[kOccItems];
  int c = 0;
#pragma unroll
  for (int i = 0; i < kOccItems; ++i) {
    keep[i] = m0 + i < M && occupied(g, x + (m0 + i) * 3);
    c += keep[i] ? 1 : 0;
  }
  int total;
  int64_t o = offsets[blockIdx.x] + block_excl_scan(c, &total);
#pragma unroll
  for (int i = 0; i < kOccItems; ++i) {
    if (keep[i]) {
      const int64_t m = m0 + i;
      rows[o] = static_cast<int32_t>(m);
#pragma unroll
      for (int d = 0; d < 3; ++d) xc[o * 3 + d] = x[m * 3 + d];
      ++o;
    }
  }
}

static int make_grid(const uint8_t* occ, int32_t gx, int32_t gy, int32_t gz, float zmul,
                     OccGrid* g) {
  if (!occ || gx < 1 || gy < 1 || gz < 1 || !(zmul > 0.0f)) return 1;
  *g = OccGrid{occ, gx, gy, gz, zmul};
  return 0;
}

}  // namespace anr

extern "C" int64_t anr_occupancy_n_blocks(int64_t M) {
  return M <= 0 ? 0 : anr::ceil_div(M, anr::kOccBlock);
}

extern "C" int anr_occupancy_count(const float* coords, int64_t M, const uint8_t* occ,
                                   int32_t gx, int32_t gy, int32_t gz, float zmul,
                                   int32_t* counts, anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  OccGrid g;
  ANR_CHECK_ARG(M > 0 && M < (1LL << 31) && coords && counts &&
                    make_grid(occ, gx, gy, gz, zmul, &g) == 0,
                "anr_occupancy_count: bad argument");
  hipLaunchKernelGGL(occ_count_kernel, dim3(static_cast<unsigned>(ceil_div(M, kOccBlock))),
                     dim3(kOccThreads), 0, as_stream(stream), coords, M, g, counts);
  ANR_CHECK_LAUNCH("anr_occupancy_count");
  return ANR_OK;
}

extern "C" int anr_occupancy_compact(const float* coords, int64_t M, const uint8_t* occ,
                                     int32_t gx, int32_t gy, int32_t gz, float zmul,
                                     const int64_t* offsets, int32_t* rows, float* coords_out,
                                     anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  OccGrid g;
  ANR_CHECK_ARG(M > 0 && M < (1LL << 31) && coords && offsets && rows && coords_out &&
                    make_grid(occ, gx, gy, gz, zmul, &g) == 0,
                "anr_occupancy_compact: bad argument");
  hipLaunchKernelGGL(occ_compact_kernel, dim3(static_cast<unsigned>(ceil_div(M, kOccBlock))),
                     dim3(kOccThreads), 0, as_stream(stream), coords, M, g, offsets, rows,
                     coords_out);
  ANR_CHECK_LAUNCH("anr_occupancy_compact");
  return ANR_OK;
}
