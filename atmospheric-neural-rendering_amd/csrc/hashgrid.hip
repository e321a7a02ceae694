// K3 / K4: multi-resolution hash-grid encoding, forward and backward.
//
// Replaces tinycudann.Encoding(n, {"otype": "HashGrid", ...}) at
// src/atmonr/pipelines/instant_ngp.py:60-63 (3-D positions, called at :163/:236) and the
// 2-D surface grid nested in the surface Composite (:78-80, called at :173).
// Semantics (tiny-cuda-nn GridEncoding; the reference pins no version — see DESIGN.md):
//   scale_l = 2^(l * log2(per_level_scale)) * base_resolution - 1     (f32)
//   res_l   = ceil(scale_l) + 1
//   pos     = fma(scale_l, x, 0.5); cell = floor(pos); w = pos - cell (linear)
//   index   = dense stride index while stride <= T_l, else XOR prime hash; % T_l
//   out[l*F + f] = sum over 2^D corners of prod(w or 1-w) * table[(off_l + index)*F + f]
//
// Work decomposition (MI355X-specific): one thread owns one LEVEL of a CHUNK of K
// consecutive samples. Samples are ray-major, so consecutive samples of a ray usually
// stay in the same cell of a level (always on the coarse levels, ~4 samples per cell on
// the finest). The forward keeps the 2^D corner features of the current cell in
// registers and re-gathers only when the cell changes; the backward accumulates the
// corner gradients of the current cell in registers and issues the f32 atomics only
// when the cell changes. Lanes of a wavefront are the levels of one chunk (16 levels ->
// 4 chunks per wave): the per-sample coordinate load is a broadcast and the per-sample
// feature row (L*F values) is read/written contiguously.

#include "anr_common.h"
#include "hash_levels.h"

// Profiling ablation (tools): 1 = backward without its atomics. 0 in product builds.
#ifndef HASH_BS
// samples per prefetch batch of the v2 backward walker. 6 rather than 8: the batch's
// scalar coordinates (two batches of 3 x BS SGPRs) spilled 40 SGPRs at 8, 3 at 6; on the
// settled reference-numerics step's own inputs 0.717 -> 0.690 ms (with the max-ILP
// scheduler 0.689; profiles/r05_hash_bwd_variants.log). The tile path keeps 8.
#define HASH_BS 6
#endif
#ifndef HASH_FBS
#define HASH_FBS 4  // samples per coordinate prefetch batch of the forward walker
#endif
#ifndef HASH_EXP
#define HASH_EXP 0
#endif


#include <cmath>
#include <type_traits>
#include <cstdlib>

namespace anr {

// Corner addressing for the v2 walkers, where a lane owns the x-offset b and the NC =
// 2^(D-1) corners over dims 1..D-1. The per-dimension components of the cell are formed
// once per cell; corner c then costs an xor (hashed) or add (dense) with compile-time
// component choice after unrolling, and the hashed / dense choice is a select on the
// level's flag, not a branch. The dense wrap (only for points outside [0, 1]) is one
// rarely-taken branch for all corners.
template <int D>
struct LaneCorners {
  static constexpr int NC = 1 << (D - 1);
  __device__ static void indices(const LevelIdx<D>& li, const uint32_t* cell, int b,
                                 uint32_t* idx) {
    const uint32_t cx = (cell[0] + static_cast<uint32_t>(b)) * li.mul[0];
    uint32_t c1[2], c2[2] = {0u, 0u};
    c1[0] = cell[1] * li.mul[1];
    c1[1] = c1[0] + li.mul[1];
    if constexpr (D == 3) {
      c2[0] = cell[2] * li.mul[2];
      c2[1] = c2[0] + li.mul[2];
    }
    uint32_t sum[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      uint32_t hx = cx ^ c1[c & 1];
      sum[c] = cx + c1[c & 1];
      if constexpr (D == 3) {
        hx ^= c2[c >> 1];
        sum[c] += c2[c >> 1];
      }
      idx[c] = li.hashed ? (hx & (li.T - 1u)) : sum[c];
    }
    // a dense corner sum can reach T only with a corner on the far face or outside the
    // grid: below that every sum is <= res^D - 1 < T (one test per cell, not per corner;
    // the unsigned max also catches negative cell coordinates). A branch-free form (selects
    // on every flush, the modulo behind one wave-uniform test) measured slower: hash bwd
    // 0.39-0.41 -> 0.45-0.47 ms (profiles/r06_hash_dense_wrap_ab.log)
    uint32_t gm = cell[0] + static_cast<uint32_t>(b);
#pragma unroll
    for (int d = 1; d < D; ++d) gm = gm > cell[d] ? gm : cell[d];
    if (!li.hashed && gm >= li.res1) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (!li.hashed && sum[c] >= li.T) {
          const uint32_t s1 = sum[c] - li.T;
          idx[c] = s1 < li.T ? s1 : sum[c] % li.T;
        }
    }
  }
  // A corner with offset o along a dim keeps its lattice point in the new cell iff
  // n = o + (old - new) is 0 or 1; it then becomes corner n there.
  __device__ static bool leaves(int c, const int* dl) {
    // bitwise, not short-circuit: || became a divergent branch (exec save / restore) per
    // corner in the walk's flush
    bool out = static_cast<unsigned>((c & 1) + dl[1]) > 1u;
    if constexpr (D == 3) out = out | (static_cast<unsigned>((c >> 1) + dl[2]) > 1u);
    return out;
  }
  // Carry accumulators onto the new cell's corners, one dimension at a time with
  // compile-time corner structure (dl = old - new per dim; all leave if x moved).
  __device__ static void carry(const float* a, const int* dl, bool keepx, float* n) {
    const int dy = dl[1];
    const bool y0 = dy == 0, ym = dy == -1, yp = dy == 1;
    float t[NC];
#pragma unroll
    for (int z = 0; z < NC / 2; ++z) {
      const float a0 = a[2 * z], a1 = a[2 * z + 1];
      t[2 * z] = y0 ? a0 : (ym ? a1 : 0.0f);
      t[2 * z + 1] = y0 ? a1 : (yp ? a0 : 0.0f);
    }
    if constexpr (D == 3) {
      const int dz = dl[2];
      const bool z0 = dz == 0, zm = dz == -1, zp = dz == 1;
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        n[y] = z0 ? t[y] : (zm ? t[y + 2] : 0.0f);
        n[y + 2] = z0 ? t[y + 2] : (zp ? t[y] : 0.0f);
      }
    } else {
      n[0] = t[0];
      n[1] = t[1];
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) n[c] = keepx ? n[c] : 0.0f;
  }
};

template <typename T, int F>
struct Vec;
template <>
struct Vec<__half, 2> {
  __device__ static void load(const __half* p, float* v) {
    const __half2 h = *reinterpret_cast<const __half2*>(p);
    const float2 f = __half22float2(h);
    v[0] = f.x;
    v[1] = f.y;
  }
};
template <>
struct Vec<float, 2> {
  __device__ static void load(const float* p, float* v) {
    const float2 f = *reinterpret_cast<const float2*>(p);
    v[0] = f.x;
    v[1] = f.y;
  }
};
template <typename T>
struct Vec<T, 1> {
  __device__ static void load(const T* p, float* v) { v[0] = to_f32<T>(p[0]); }
};
template <typename T>
struct Vec<T, 4> {
  __device__ static void load(const T* p, float* v) {
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] = to_f32<T>(p[f]);
  }
};
template <typename T>
struct Vec<T, 8> {
  __device__ static void load(const T* p, float* v) {
#pragma unroll
    for (int f = 0; f < 8; ++f) v[f] = to_f32<T>(p[f]);
  }
};

template <typename TO, int F>
__device__ __forceinline__ void store_feat(TO* p, const float* v) {
#pragma unroll
  for (int f = 0; f < F; ++f) p[f] = from_f32<TO>(v[f]);
}
template <>
__device__ __forceinline__ void store_feat<__half, 2>(__half* p, const float* v) {
  *reinterpret_cast<__half2*>(p) = __floats2half2_rn(v[0], v[1]);
}

// A wavefront serves lpw consecutive levels (lane % lpw) of 64/lpw chunks (lane / lpw);
// wavefronts cycle through the n_groups level groups of a block of chunks. Grouping few
// levels per wave keeps the divergent gather path to the waves whose levels actually
// change cell (fine levels: often; coarse levels: almost never).
template <int D, int F, typename TT, typename TO>
__global__ void __launch_bounds__(256) hashgrid_fwd_kernel(
    GridLevels G, int n_levels, int lpw, int n_groups, const float* __restrict__ x,
    int64_t x_stride, int64_t M, int64_t K, const TT* __restrict__ table,
    TO* __restrict__ out, int64_t out_stride) {
  // level group = block index mod n_groups: consecutive blocks go to different XCDs
  // (round-robin dispatch), so with n_groups = 8 each XCD's L2 serves the table slice of
  // its own levels only (speed only; any block placement gives the same result)
  const int lane = static_cast<int>(threadIdx.x & 63);
  const int lg = static_cast<int>(blockIdx.x % n_groups);
  const int64_t wave_in = (static_cast<int64_t>(blockIdx.x / n_groups) * blockDim.x + threadIdx.x) >> 6;
  const int64_t chunk = wave_in * (64 / lpw) + lane / lpw;
  const int level = lg * lpw + lane % lpw;
  const int64_t m0 = chunk * K;
  if (level >= n_levels || m0 >= M) return;
  const int64_t m1 = m0 + K < M ? m0 + K : M;

  const float scale = G.scale[level];
  const uint32_t res = G.res[level];
  const uint32_t T = G.size[level];
  const TT* __restrict__ grid = table + static_cast<int64_t>(G.offset[level]) * F;
  LevelIdx<D> li;
  li.init(T, res);

  uint32_t cell[D];
  bool have = false;
#pragma unroll
  for (int d = 0; d < D; ++d) cell[d] = 0u;
  float val[1 << D][F];

  // All 2^D corners are gathered together on a cell change: one divergent region, so
  // the waits for the gathers do not also wait for the younger coordinate prefetches
  // (per-corner conditional gathers, tried, cost more than the loads they save).
  auto step = [&](int64_t m, const float* xv) {
    float w[D];
    uint32_t g[D];
    bool same = have;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float p = fmaf(scale, xv[d], 0.5f);
      const float fl = floorf(p);
      g[d] = static_cast<uint32_t>(static_cast<int>(fl));
      w[d] = p - fl;
      same = same & (g[d] == cell[d]);
    }
    if (!same) {
      have = true;
      uint32_t comp[D][2];
      li.dims(g, comp);
#pragma unroll
      for (int c = 0; c < (1 << D); ++c)
        Vec<TT, F>::load(grid + static_cast<int64_t>(li.corner(comp, c)) * F, val[c]);
#pragma unroll
      for (int d = 0; d < D; ++d) cell[d] = g[d];
    }
    float acc[F];
#pragma unroll
    for (int f = 0; f < F; ++f) acc[f] = 0.0f;
#pragma unroll
    for (int c = 0; c < (1 << D); ++c) {
      float wt = 1.0f;
#pragma unroll
      for (int d = 0; d < D; ++d) wt *= ((c >> d) & 1) ? w[d] : 1.0f - w[d];
#pragma unroll
      for (int f = 0; f < F; ++f) acc[f] = fmaf(wt, val[c][f], acc[f]);
    }
    if constexpr ((HASH_EXP & 2) == 0) store_feat<TO, F>(out + m * out_stride + level * F, acc);
    else if (acc[0] == 12345.0f) out[0] = from_f32<TO>(acc[F - 1]);  // keep the work alive
  };

  // coordinates prefetched one batch ahead (indices clamped to the chunk: no branch)
  constexpr int BS = HASH_FBS;
  float xb[BS][D], xn[BS][D];
  auto load_batch = [&](int64_t mb, float (*xo)[D]) {
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      const int64_t m = mb + j < m1 ? mb + j : m1 - 1;
#pragma unroll
      for (int d = 0; d < D; ++d) xo[j][d] = x[m * x_stride + d];
    }
  };
  load_batch(m0, xb);
  for (int64_t mb = m0; mb < m1; mb += BS) {
    load_batch(mb + BS, xn);
#pragma unroll
    for (int j = 0; j < BS; ++j)
      if (mb + j < m1) step(mb + j, xb[j]);
#pragma unroll
    for (int j = 0; j < BS; ++j)
#pragma unroll
      for (int d = 0; d < D; ++d) xb[j][d] = xn[j][d];
  }
}

template <typename TG>
__device__ __forceinline__ float load_grad(const TG* p) {
  return to_f32<TG>(*p);
}

template <int D, int F, typename TG>
__global__ void __launch_bounds__(256) hashgrid_bwd_kernel(
    GridLevels G, int n_levels, int lanes_per_chunk, const float* __restrict__ x,
    int64_t x_stride, int64_t M, int64_t K, const TG* __restrict__ dout,
    int64_t dout_stride, float* __restrict__ dtable) {
  const int64_t gtid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t chunk = gtid / lanes_per_chunk;
  const int level = static_cast<int>(gtid % lanes_per_chunk);
  const int64_t m0 = chunk * K;
  if (level >= n_levels || m0 >= M) return;
  const int64_t m1 = m0 + K < M ? m0 + K : M;

  const float scale = G.scale[level];
  const uint32_t res = G.res[level];
  const uint32_t T = G.size[level];
  float* __restrict__ grad = dtable + static_cast<int64_t>(G.offset[level]) * F;

  uint32_t cell[D];
  bool have = false;
  float acc[1 << D][F];
#pragma unroll
  for (int d = 0; d < D; ++d) cell[d] = 0u;
#pragma unroll
  for (int c = 0; c < (1 << D); ++c)
#pragma unroll
    for (int f = 0; f < F; ++f) acc[c][f] = 0.0f;

  auto flush = [&]() {
#pragma unroll
    for (int c = 0; c < (1 << D); ++c) {
      bool any = false;
#pragma unroll
      for (int f = 0; f < F; ++f) any = any || (acc[c][f] != 0.0f);
      if (any) {
        uint32_t gc[D];
#pragma unroll
        for (int d = 0; d < D; ++d) gc[d] = cell[d] + ((c >> d) & 1);
        const uint32_t idx = grid_index<D>(T, res, gc);
        float* dst = grad + static_cast<int64_t>(idx) * F;
#pragma unroll
        for (int f = 0; f < F; ++f) {
          if (acc[c][f] != 0.0f) atomicAdd(dst + f, acc[c][f]);
          acc[c][f] = 0.0f;
        }
      }
    }
  };

  for (int64_t m = m0; m < m1; ++m) {
    float w[D];
    uint32_t g[D];
    bool same = have;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float p = fmaf(scale, x[m * x_stride + d], 0.5f);
      const float fl = floorf(p);
      g[d] = static_cast<uint32_t>(static_cast<int>(fl));
      w[d] = p - fl;
      same = same & (g[d] == cell[d]);
    }
    if (!same) {
      if (have) flush();
      have = true;
#pragma unroll
      for (int d = 0; d < D; ++d) cell[d] = g[d];
    }
    float gv[F];
#pragma unroll
    for (int f = 0; f < F; ++f) gv[f] = load_grad<TG>(dout + m * dout_stride + level * F + f);
#pragma unroll
    for (int c = 0; c < (1 << D); ++c) {
      float wt = 1.0f;
#pragma unroll
      for (int d = 0; d < D; ++d) wt *= ((c >> d) & 1) ? w[d] : 1.0f - w[d];
#pragma unroll
      for (int f = 0; f < F; ++f) acc[c][f] = fmaf(wt, gv[f], acc[c][f]);
    }
  }
  if (have) flush();
}


// ---------------------------------------------------------------------------------------
// v2 (F = 2, L <= 16): 4 lanes per level, one chunk of K consecutive samples per wave.
// lane = 4*level + 2*b + f owns feature f of the 2^(D-1) corners whose x-offset is b.
// The 4 lanes of a level touch entries (x, x+1) x features (0, 1): adjacent addresses on
// dense levels (and on hashed levels when x is even, since the first hash prime is 1),
// so one wave instruction issues one memory request per level instead of four. When
// the sample moves to a neighbouring cell with the same x, corners shared by the two
// cells keep their accumulated gradient (bwd) / gathered feature (fwd).
template <int D>
struct Corners {
  static constexpr int NC = 1 << (D - 1);
  // lattice offset bit of corner c (0..NC-1) along dim d >= 1
  __device__ static int bit(int c, int d) { return (c >> (d - 1)) & 1; }
};

// ---------------------------------------------------------------------------------------
// Forward v6 (F = 2, L <= 16): v1's decomposition (lane = one level of one of the 4
// chunks a wavefront walks side by side) with the per-sample instruction stream rebuilt.
// A wavefront takes the gather path whenever any of its 64 lanes changes cell (~99 % of
// samples on the bench geometry), and its lanes mix dense and hashed levels, so in v1
// every per-corner branch (hashed / dense / dense wrap) ran both ways on nearly every
// sample, next to 64-bit clamped coordinate indices. Here:
//   * corner indices are branch-free (hashed and dense forms, one select per corner); the
//     dense wrap (a corner sum reaching T) is one rarely-taken branch per cell, entered
//     only when a corner can reach the far face (cell coordinate >= res - 1 or outside the
//     grid: below that every corner sum is <= res^D - 1 < T);
//   * memory goes through buffer descriptors with 32-bit offsets: reads past the end of x
//     return 0 and writes past the last row are dropped by the hardware range check, so
//     the walk has no per-sample bounds checks and a wave-uniform trip count;
//   * f16 corner features are interpolated straight from the packed pair (v_fma_mix_f32
//     reads the f16 operand in place: no conversions).
// Same corner order, weights and fma chain as v1: results are bit-identical to it. The
// default forward since r02 (0.667 -> 0.648 ms at bench size).
template <typename TO>
__device__ __forceinline__ void store2(__amdgpu_buffer_rsrc_t r, uint32_t off, float a0, float a1);
template <>
__device__ __forceinline__ void store2<__half>(__amdgpu_buffer_rsrc_t r, uint32_t off, float a0,
                                               float a1) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, __floats2half2_rn(a0, a1)),
                                        r, off, 0, 0);
}
template <>
__device__ __forceinline__ void store2<float>(__amdgpu_buffer_rsrc_t r, uint32_t off, float a0,
                                              float a1) {
  using v2 = uint32_t __attribute__((vector_size(8)));
  const v2 v = {__float_as_uint(a0), __float_as_uint(a1)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 0);
}

// One lane's walk of v6: level ``level`` over the K samples of the chunk starting at m0,
// writing each sample's 2 features at oo, oo + ostep, ... of the output buffer.
template <int D, typename TT, typename TO>
__device__ __forceinline__ void fwd_walk_v6(const GridLevels& G, int level, int64_t m0, int K,
                                            __amdgpu_buffer_rsrc_t rx, uint32_t xs4,
                                            __amdgpu_buffer_rsrc_t rt, __amdgpu_buffer_rsrc_t ro,
                                            uint32_t oo, uint32_t ostep) {
  using R = Raw2<TT>;
  const float scale = G.scale[level];
  const uint32_t res = G.res[level];
  const uint32_t T = G.size[level];
  const uint32_t base = G.offset[level] * R::bytes;
  LevelIdx<D> li;
  li.init(T, res);
  const uint32_t hmask = T - 1u;

  uint32_t xo = static_cast<uint32_t>(m0) * xs4;

  uint32_t cell[D];
  bool have = false;
#pragma unroll
  for (int d = 0; d < D; ++d) cell[d] = 0u;
  typename R::type val[1 << D];
#pragma unroll
  for (int c = 0; c < (1 << D); ++c) val[c] = {};

  auto step = [&](const float* xv) {
    float w[D];
    uint32_t g[D];
    bool same = have;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float p = fmaf(scale, xv[d], 0.5f);
      const float fl = floorf(p);
      g[d] = static_cast<uint32_t>(static_cast<int>(fl));
      w[d] = p - fl;
      same = same & (g[d] == cell[d]);
    }
    if (!same) {
      uint32_t comp[D][2];
      li.dims(g, comp);
      uint32_t idx[1 << D], sum[1 << D];
#pragma unroll
      for (int c = 0; c < (1 << D); ++c) {
        uint32_t hx = 0u, sm = 0u;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          hx ^= comp[d][(c >> d) & 1];
          sm += comp[d][(c >> d) & 1];
        }
        sum[c] = sm;
        idx[c] = li.hashed ? (hx & hmask) : sm;
      }
      uint32_t gmax = g[0];
#pragma unroll
      for (int d = 1; d < D; ++d) gmax = gmax > g[d] ? gmax : g[d];
      if (!li.hashed && gmax >= res - 1u) {
#pragma unroll
        for (int c = 0; c < (1 << D); ++c)
          if (sum[c] >= T) {
            const uint32_t s1 = sum[c] - T;
            idx[c] = s1 < T ? s1 : sum[c] % T;
          }
      }
      if constexpr ((HASH_EXP & 4) != 0 && std::is_same<TT, __half>::value) {
        // ceiling probe (wrong values): one 8-B load per x-pair at the aligned pair of x0
#pragma unroll
        for (int c = 0; c < (1 << D); c += 2) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(rt, base + (idx[c] & ~1u) * 4u, 0, 0);
          val[c] = v[0];
          val[c + 1] = v[1];
        }
      } else if constexpr ((HASH_EXP & 8) != 0 && std::is_same<TT, __half>::value) {
#pragma unroll
        for (int c = 0; c < (1 << D); ++c) val[c] = idx[c];  // no gathers (probe, wrong values)
      } else {
#pragma unroll
        for (int c = 0; c < (1 << D); ++c) val[c] = R::load(rt, base + idx[c] * R::bytes);
      }
#pragma unroll
      for (int d = 0; d < D; ++d) cell[d] = g[d];
      have = true;
    }
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
    for (int c = 0; c < (1 << D); ++c) {
      float wt = 1.0f;
#pragma unroll
      for (int d = 0; d < D; ++d) wt *= ((c >> d) & 1) ? w[d] : 1.0f - w[d];
      R::fma2(wt, val[c], a0, a1);
    }
    store2<TO>(ro, oo, a0, a1);
    oo += ostep;
  };

  // coordinates prefetched one batch ahead; past the end of x the loads return 0
  constexpr int BS = HASH_FBS;
  float xb[BS][D], xn[BS][D];
  auto load_batch = [&](float (*xo_)[D]) {
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      if constexpr (D == 3) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rx, xo, 0, 0);
        xo_[j][0] = __uint_as_float(v[0]);
        xo_[j][1] = __uint_as_float(v[1]);
        xo_[j][2] = __uint_as_float(v[2]);
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rx, xo, 0, 0);
        xo_[j][0] = __uint_as_float(v[0]);
        xo_[j][1] = __uint_as_float(v[1]);
      }
      xo += xs4;
    }
  };
  load_batch(xb);
  for (int jb = 0; jb < K; jb += BS) {  // wave-uniform trip count
    load_batch(xn);
#pragma unroll
    for (int j = 0; j < BS; ++j)
      if (jb + j < K) step(xb[j]);
#pragma unroll
    for (int j = 0; j < BS; ++j)
#pragma unroll
      for (int d = 0; d < D; ++d) xb[j][d] = xn[j][d];
  }
}

template <int D, typename TT, typename TO>
__global__ void __launch_bounds__(256) hashgrid_fwd_v6_kernel(
    GridLevels G, int n_levels, const float* __restrict__ x, uint32_t x_bytes, uint32_t xs4,
    int64_t M, int K, const TT* __restrict__ table, uint32_t table_bytes,
    TO* __restrict__ out, uint32_t out_bytes, uint32_t os_bytes) {
  const int level = static_cast<int>(threadIdx.x & 15);
  const int64_t chunk = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
  const int64_t m0 = chunk * K;
  if (level >= n_levels || m0 >= M) return;
  fwd_walk_v6<D, TT, TO>(
      G, level, m0, K, wave_rsrc(x, x_bytes), xs4, wave_rsrc(table, table_bytes),
      wave_rsrc(out, out_bytes),
      static_cast<uint32_t>(m0) * os_bytes + static_cast<uint32_t>(level) * 2u * sizeof(TO),
      os_bytes);
}

// ---------------------------------------------------------------------------------------
// Forward v9 "quad planes" (F = 2, f16 output): one lane per SAMPLE, every level, output
// in level-quad planes -- plane q holds levels 4q..4q+3 of every row, 16 B per row
// (level l feature f of row m at out[(l / 4) * plane + 8 m + 2 (l % 4) + f]). The walkers
// (v1 / v6) keep a lane on one level of one chunk and re-gather only on a cell change,
// but their wavefronts touch 4-16 chunks far apart, so each gather instruction lands on as
// many unrelated lines. Here a wavefront's 64 lanes are 64 consecutive samples of one
// ray: a corner gather's addresses coincide wherever neighbouring samples share a cell
// (all of them on the coarse levels, ~4 per cell on the finest), the coordinate load is
// one contiguous 768 B, and each quad's store is one contiguous 1 KiB (a level-major row
// layout written lane by lane leaves partial lines: 1.57 ms measured, against 0.47 for
// the planes). Every sample gathers its 8 corners per level (no cell reuse inside a
// lane). Same corner order, weights and fma chain as v6: bit-identical values. Measured
// on the bench coordinates (profiles/r05_hash_fwd_planes.log): v6 0.634 ms, v9 0.47-0.50
// ms; pinning level pairs to XCDs (block b -> XCD b % 8) made it slower (0.77 / 1.13 ms:
// every XCD then reads every coordinate).
template <int D, typename TT, int DEDUP>
__global__ void __launch_bounds__(256) hashgrid_fwd_planes_kernel(
    GridLevels G, int n_levels, const float* __restrict__ x, uint32_t x_bytes, uint32_t xs4,
    int64_t M, const TT* __restrict__ table, uint32_t table_bytes, __half* __restrict__ out,
    uint32_t out_bytes, uint32_t plane_bytes) {
  const int64_t m = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const __amdgpu_buffer_rsrc_t rx = wave_rsrc(x, x_bytes);
  const __amdgpu_buffer_rsrc_t rt = wave_rsrc(table, table_bytes);
  const __amdgpu_buffer_rsrc_t ro = wave_rsrc(out, out_bytes);
  const uint32_t xo = static_cast<uint32_t>(m) * xs4;  // past the end: loads return 0
  float xv[D];
  if constexpr (D == 3) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rx, xo, 0, 0);
    xv[0] = __uint_as_float(v[0]);
    xv[1] = __uint_as_float(v[1]);
    xv[2] = __uint_as_float(v[2]);
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rx, xo, 0, 0);
    xv[0] = __uint_as_float(v[0]);
    xv[1] = __uint_as_float(v[1]);
  }
  // rows past M: the stores are dropped by the range check (offset >= out_bytes)
  const uint32_t orow = m < M ? static_cast<uint32_t>(m) * 16u : 0x80000000u;
  const int n_quads = (n_levels + 3) >> 2;
  for (int q = 0; q < n_quads; ++q) {
    uint32_t packed[4];
    plane_quad<D, TT, DEDUP>(G, n_levels, q, xv, rt, packed);
    typedef uint32_t u4q __attribute__((vector_size(16)));
    const u4q v = {packed[0], packed[1], packed[2], packed[3]};
    __builtin_amdgcn_raw_buffer_store_b128(v, ro, static_cast<uint32_t>(q) * plane_bytes + orow,
                                           0, 0);
  }
}

// XS / DS: compile-time coordinate and dL/dy row strides (0 = the run-time x_stride /
// dout_stride). With both known (the fused field's (M,3) coordinates and (M,32) dL/denc)
// every prefetch address is a per-batch scalar base plus immediate offsets: the walk
// issues no per-sample address arithmetic (r01 spent ~25 scalar instructions per sample
// on 64-bit clamped indices), and only a chunk's last two batches clamp.
// Distinct 64-B segments among the active lanes' addresses: the memory-side requests one
// wave-level float atomic instruction makes (MI355X_MICROARCH.md "Global float atomics").
// Called in divergent code: the count is returned to the instruction's first active lane
// only (0 elsewhere), so per-lane sums add every instruction exactly once.
__device__ __forceinline__ uint32_t distinct_segments(bool active, uint64_t seg) {
  uint64_t mask = __ballot(active);
  const uint64_t execm = __ballot(true);
  const bool first = (__lane_id() == __ffsll(static_cast<unsigned long long>(execm)) - 1);
  uint32_t n = 0;
  while (mask) {
    const int l = __ffsll(static_cast<unsigned long long>(mask)) - 1;
    const uint32_t lo = __shfl(static_cast<uint32_t>(seg), l);
    const uint32_t hi = __shfl(static_cast<uint32_t>(seg >> 32), l);
    const uint64_t s = (static_cast<uint64_t>(hi) << 32) | lo;
    mask &= ~__ballot(active && seg == s);
    ++n;
  }
  return first ? n : 0;
}

// COUNT: the request-count instrument (anr_hashgrid_bwd_count_requests): the same walk,
// but every flush instruction adds its number of distinct 64-B segments to *count
// instead of issuing the atomics (dtable is not written)
// SPARSE: anr_hashgrid_bwd_rows: row_nz holds one bit per dL/dy row (32 rows per word,
// written by anr_ingp_field_bwd_ref16_rows), and only the rows whose bit is set are loaded
// and walked (16 levels: every lane takes part in the chunk's compaction)
template <int D, typename TG, int XS, int DS, bool COUNT = false, int BSZ = HASH_BS,
          bool SPARSE = false>
__global__ void __launch_bounds__(256) hashgrid_bwd_v2_kernel(
    GridLevels G, int n_levels, const float* __restrict__ x, int64_t x_stride_rt, int64_t M,
    int64_t K, const TG* __restrict__ dout, int64_t dout_stride_rt, float* __restrict__ dtable,
    int skip_zero, unsigned long long* __restrict__ count = nullptr,
    const uint8_t* __restrict__ tile_nz = nullptr, const uint32_t* __restrict__ row_nz = nullptr) {
  constexpr int NC = Corners<D>::NC;
  const int64_t x_stride = XS > 0 ? XS : x_stride_rt;
  const int64_t dout_stride = DS > 0 ? DS : dout_stride_rt;
  const int lane = threadIdx.x & 63;
  const int level = lane >> 2, b = (lane >> 1) & 1, f = lane & 1;
  const int64_t chunk = __builtin_amdgcn_readfirstlane(
      static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6));
  const int64_t m0 = chunk * K;
  // chunk bounds are wave-uniform: kept in scalar registers
  const int64_t m1 = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(
      static_cast<int>(m0 + K < M ? K : M - m0))) + m0;
  if (m0 >= M || level >= n_levels) return;
  const float scale = G.scale[level];
  const uint32_t res = G.res[level];
  const uint32_t T = G.size[level];
  float* __restrict__ grad = dtable + static_cast<int64_t>(G.offset[level]) * 2 + f;
  LevelIdx<D> li;
  li.init(T, res);
  // The flushes are buffer atomics whose non-flushing lanes get an offset past the
  // table: the hardware range check drops them, so a flush is one select and one atomic
  // instruction, not a divergent branch (exec save / test / restore: scalar instructions,
  // which bounded this walk — SQ counters, profiles/r04_sq_close.md)
  const uint32_t table_bytes = (G.offset[n_levels - 1] + G.size[n_levels - 1]) * 8u;
  const __amdgpu_buffer_rsrc_t rg = wave_rsrc(dtable, table_bytes);
  const uint32_t gbase = (G.offset[level] * 2u + static_cast<uint32_t>(f)) * 4u;
  constexpr uint32_t kDrop = 0x80000000u;  // >= table_bytes (ABI: tables < 2 GB)

  uint32_t cell[D];
  bool have = false;
#pragma unroll
  for (int d = 0; d < D; ++d) cell[d] = 0u;
  float acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.0f;
  uint32_t n_req = 0;  // COUNT only (wave-uniform)
  auto flush = [&](bool out, uint32_t e, float v) {
    if constexpr (COUNT) {
      n_req += distinct_segments(
          out, reinterpret_cast<uintptr_t>(grad + static_cast<int64_t>(e) * 2) >> 6);
    } else if constexpr ((HASH_EXP & 1) == 0) {
      __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rg, out ? gbase + e * 8u : kDrop, 0, 0);
    }
  };

  auto step = [&](const float* xv, float gv) {
    float w[D];
    uint32_t g[D];
    bool same = have;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float p = fmaf(scale, xv[d], 0.5f);
      const float fl = floorf(p);
      g[d] = static_cast<uint32_t>(static_cast<int>(fl));
      w[d] = p - fl;
      same = same & (g[d] == cell[d]);
    }
    if (!same) {
      if (have) {
        uint32_t idx[NC];
        LaneCorners<D>::indices(li, cell, b, idx);
        const bool keepx = g[0] == cell[0];
        int dl[D];
        dl[0] = 0;
#pragma unroll
        for (int d = 1; d < D; ++d) dl[d] = static_cast<int>(cell[d] - g[d]);
        float nacc[NC];
        LaneCorners<D>::carry(acc, dl, keepx, nacc);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          // skip_zero: a leaving corner whose sum is exactly zero issues no request
          // (reference numerics: tcnn's x128 f16 backward rounds most dL/denc to zero);
          // without skip_zero only the leaving test applies
          const bool out = ((!keepx) | LaneCorners<D>::leaves(c, dl)) &
                           ((skip_zero == 0) | (acc[c] != 0.0f));
          flush(out, idx[c], acc[c]);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] = nacc[c];
      }
#pragma unroll
      for (int d = 0; d < D; ++d) cell[d] = g[d];
      have = true;
    }
    const float wx = b ? w[0] : 1.0f - w[0];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float wt = wx;
#pragma unroll
      for (int d = 1; d < D; ++d) wt *= Corners<D>::bit(c, d) ? w[d] : 1.0f - w[d];
      acc[c] = fmaf(wt, gv, acc[c]);
    }
  };

  // Batches of BS samples: the next batch's coordinates and gradients are loaded while
  // this one is processed (indices clamped to the chunk, so the loads need no branch).
  constexpr int BS = BSZ;
  float xb[BS][D], xn[BS][D];
  TG gb[BS], gn[BS];
  const int col = level * 2 + f;
  auto load_batch = [&](int64_t mb, float (*xo)[D], TG* go) {
    if ((XS > 0 && DS > 0) && mb + BS <= m1) {  // wave-uniform: a full batch, no clamp
      // the batch's coordinates are the same for every lane: scalar loads through the
      // constant address space (24 dwords: one s_load_dwordx16 + one x8) instead of 24
      // vector loads of one broadcast dword each (hash bwd live 1.18 -> 1.06 ms, bench
      // profiles/r04_hash_bwd_scalar_x_ab.log)
      typedef __attribute__((address_space(4))) const float cf32;
      const cf32* __restrict__ xp = (const cf32*)(x + mb * XS);
      const TG* __restrict__ dp = dout + mb * DS;
#pragma unroll
      for (int j = 0; j < BS; ++j)
#pragma unroll
        for (int d = 0; d < D; ++d) xo[j][d] = xp[j * XS + d];
#pragma unroll
      for (int j = 0; j < BS; ++j) go[j] = dp[j * DS + col];
    } else {
#pragma unroll
      for (int j = 0; j < BS; ++j) {
        const int64_t m = mb + j < m1 ? mb + j : m1 - 1;
#pragma unroll
        for (int d = 0; d < D; ++d) xo[j][d] = x[m * x_stride + d];
        go[j] = dout[m * dout_stride + col];
      }
    }
  };
  // A batch whose dL/dy is zero in every lane (all 16 levels x 2 features of its BS
  // samples: the reference numerics' f16 underflow leaves half of the 8-sample batches so
  // at the bench state) adds nothing and is skipped with one test. skip_zero 2 (default)
  // also skips single all-zero samples inside a batch and keeps the pending cell across
  // the skipped ones; skip_zero 1 (the r04 form, A/B) walks every sample of a batch with
  // any nonzero value and flushes at an all-zero batch as at a chunk end. Either way the
  // same contributions reach the same entries (a pending sum may arrive in two atomics
  // instead of one: f32 order, as any run). With skip_zero 0 (A/B) every batch is walked.
  auto flush_all = [&]() {
    if (have) {
      uint32_t idx[NC];
      LaneCorners<D>::indices(li, cell, b, idx);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        flush(acc[c] != 0.0f, idx[c], acc[c]);
        acc[c] = 0.0f;
      }
      have = false;
    }
  };
  auto do_batch = [&](int64_t mb) {
    bool nzb = false;
#pragma unroll
    for (int j = 0; j < BS; ++j) nzb = nzb || (mb + j < m1 && to_f32<TG>(gb[j]) != 0.0f);
    if (!skip_zero || __any(nzb)) {
#pragma unroll
      for (int j = 0; j < BS; ++j) {
        const float gv = to_f32<TG>(gb[j]);
        // skip_zero 2: a SAMPLE whose dL/dy row is zero in every lane (all levels and
        // features) is not walked at all: it adds nothing, and the walk stays exact
        // because the next walked sample's cell test / carry handles any jump (every
        // corner leaves when a coordinate moves by more than one cell)
        if (mb + j < m1 && (skip_zero < 2 || __any(gv != 0.0f))) step(xb[j], gv);
      }
    } else if (skip_zero == 1) {
      flush_all();
    }
  };
  auto advance = [&]() {
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      gb[j] = gn[j];
#pragma unroll
      for (int d = 0; d < D; ++d) xb[j][d] = xn[j][d];
    }
  };
  if constexpr (SPARSE) {
    static_assert(XS == 3 && DS == 32 && !COUNT, "row-mask walk: fused-field layout only");
    // The chunk's set rows, compacted in order into this wave's LDS slot (K <= 256, a
    // multiple of 32; 64 rows per round: lane l tests row r0 + l), then walked in batches of
    // BS with the next batch's coordinates (scalar loads) and gradients prefetched. Every
    // loaded row is nonzero in some lane, so no per-sample test remains; the rows whose bit
    // is clear are exactly those the dense walk's per-sample skip passes over, so the same
    // corner sums reach the same entries.
    constexpr int BS = BSZ;
    static_assert(BS % 2 == 0, "row indices are read in pairs");
    // K <= 256 rows, then 2 BS copies of the last set row: a batch (and the prefetch past
    // the end) reads its BS indices in pairs with no clamp
    __shared__ __attribute__((aligned(16))) uint32_t sidx[4][256 + 2 * BS];
    uint32_t* my = sidx[threadIdx.x >> 6];
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    int n = 0;
    for (int64_t r0 = m0; r0 < m1; r0 += 64) {
      const cu32* mp = (const cu32*)(row_nz + (r0 >> 5));
      const uint32_t lo = mp[0];
      const uint32_t hi = r0 + 32 < m1 ? mp[1] : 0u;
      uint64_t bits = (static_cast<uint64_t>(hi) << 32) | lo;
      const int64_t span = m1 - r0;
      if (span < 64) bits &= (1ull << span) - 1ull;
      const int below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bits >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bits), 0u));
      if ((bits >> lane) & 1ull) my[n + below] = static_cast<uint32_t>(r0 - m0 + lane);
      n += __popcll(bits);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n > 0) {
      const uint32_t last = my[n - 1];
      if (lane < 2 * BS) my[n + lane] = last;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    typedef __attribute__((address_space(4))) const float cf32;
    // chunk-relative bases: a row's addresses are 32-bit scalar offsets from them
    const float* __restrict__ xc = x + m0 * 3;
    const TG* __restrict__ dc = dout + m0 * 32 + col;
    auto load_rows = [&](int bb, float (*xo)[D], TG* go) {
      uint32_t r[BS];
#pragma unroll
      for (int j = 0; j < BS; j += 2) {
        const uint2 q = *reinterpret_cast<const uint2*>(my + bb + j);
        r[j] = q.x;
        r[j + 1] = q.y;
      }
#pragma unroll
      for (int j = 0; j < BS; ++j) {
        const uint32_t i = __builtin_amdgcn_readfirstlane(r[j]);
        const cf32* xp = (const cf32*)(xc + i * 3u);
#pragma unroll
        for (int d = 0; d < D; ++d) xo[j][d] = xp[d];
        go[j] = dc[i * 32u];
      }
    };
    if (n > 0) {
      load_rows(0, xb, gb);
      for (int bb = 0; bb < n; bb += BS) {
        load_rows(bb + BS, xn, gn);
#pragma unroll
        for (int j = 0; j < BS; ++j)
          if (bb + j < n) step(xb[j], to_f32<TG>(gb[j]));
        advance();
      }
    }
  } else if (BSZ != 8 || tile_nz == nullptr) {  // the tile mask below is laid out for BS = 8
    load_batch(m0, xb, gb);
    for (int64_t mb = m0; mb < m1; mb += BS) {
      load_batch(mb + BS, xn, gn);
      do_batch(mb);
      advance();
    }
  } else {
    // anr_hashgrid_bwd_tiles: the field backward marked the 32-row tiles whose dL/dy is
    // zero in every row (it skipped them); their batches are neither loaded nor walked.
    // A chunk (K <= 256 rows, a multiple of 32, tile-aligned) is <= 32 batches of 8: one
    // wave-uniform bit mask, walked in order with the next set batch prefetched.
    const int nbatch = static_cast<int>((m1 - m0 + BS - 1) / BS);
    const int ntile = static_cast<int>((m1 - m0 + 31) >> 5);
    const uint8_t* tf = tile_nz + (m0 >> 5);
    uint32_t bm = 0;
    for (int t = 0; t < ntile; ++t)
      if (tf[t]) bm |= 0xFu << (4 * t);
    if (nbatch < 32) bm &= (1u << nbatch) - 1u;
    if (bm) {
      int j = __builtin_ctz(bm);
      bm &= bm - 1u;
      load_batch(m0 + static_cast<int64_t>(j) * BS, xb, gb);
      while (true) {
        const bool more = bm != 0u;
        const int jn = more ? __builtin_ctz(bm) : j;  // no further batch: reload j (unused)
        load_batch(m0 + static_cast<int64_t>(jn) * BS, xn, gn);
        do_batch(m0 + static_cast<int64_t>(j) * BS);
        if (!more) break;
        advance();
        j = jn;
        bm &= bm - 1u;
      }
    }
  }
  flush_all();
  if constexpr (COUNT) {
    // per lane (lanes above n_levels have returned; an instrument, not the hot path)
    if (n_req) atomicAdd(count, static_cast<unsigned long long>(n_req));
  }
}

// v2: one chunk per wave. Every chunk ends with a flush of all its held corners, so a
// chunk should be long (requests per sample on the bench coordinates, tools/
// hash_bwd_requests.py: K = 32 / 64 / 128 / 256 / 512 -> 4.42 / 3.33 / 2.79 / 2.51 / 2.37),
// but the grid still needs waves to hide the walk's latency. Measured (r04 sweep,
// profiles/r04_hash_bwd_ksweep.md): at 1,024 rays x 1,024 samples K = 256 (4,096 waves)
// takes 0.176 ms against 0.295 ms at the r03 rule's K = 32 and 0.244 ms at K = 512; at
// 8,192 rays K = 256 / 512 / 1024 take 1.219 / 1.200 / 1.287 ms -- but in the bench step
// K = 512 makes the STEP slower (3.227 / 3.228 ms at 256 vs 3.270 / 3.267 at 512, alternating
// runs on one box, hash bwd 1.139 vs 1.129 ms: profiles/r04_hash_bwd_k_step_ab.log). Rule:
// 256 samples per chunk down to 4,096 chunks, shorter below that.
static int64_t env_k(const char* name) {
  const char* e = getenv(name);  // profiling override of the chunk length
  return e ? atoll(e) : 0;
}
// run-leader gathers in the planes forward (plane_quad): ANR_HASH_DEDUP = the largest
// number of cell changes per wavefront at which a level gathers at the run leaders only
// (0 = off, 16 / 32 / 48 / 64; A/B hook, default HASH_DEDUP = 64: every level. Measured on
// the settled bench step, hash fwd 0.478 ms off, 0.435 / 0.439 / 0.433 / 0.421 ms at
// 32 / 16 / 48 / 64: profiles/r06_hash_fwd_dedup_sweep.log)
static int plane_dedup() {
  static const int v = [] {
    const char* e = getenv("ANR_HASH_DEDUP");
    return e ? atoi(e) : HASH_DEDUP;
  }();
  return v;
}
static int64_t pick_chunk_v2(int64_t M) {
  static const int64_t over = env_k("ANR_HASH_KB");
  if (over > 0) return over;
  int64_t K = M / 4096;
  if (K < 1) K = 1;
  if (K > 256) K = 256;
  return K;
}

// Kernel generation per direction. Mode 0 (default): forward v6, backward v2 (measured
// fastest on the ray-coherent bench workload; v6 falls back to v1 above 16 levels or
// past 32-bit buffer offsets); 1: both v1 (the generic kernels every shape falls back
// to); 6: forward v1, backward v2 (the r01 default); 7: as 0 with the backward's run-time-
// stride instantiation (A/B of the compile-time strides). ANR_HASHGRID_MODE or
// anr_hashgrid_force_v1() selects it (test hook). The r02 forward experiments v2-v5
// (x-pair lanes, batched gathers, one thread per sample, LDS-compacted gathers) measured
// slower than v6 and were removed in r04 (profiles/r02_hash_fwd_v6_v7_ab.log). On the
// bench coordinates the forward spends ~0.35 of its ~0.65 ms on the corner gathers' memory
// traffic (0.29 ms with no gathers at all) and is not issue-bound.
static bool valid_mode(int m) { return m == 0 || m == 1 || m == 6 || m == 7; }
static int g_hashgrid_mode = [] {
  const char* e = getenv("ANR_HASHGRID_MODE");
  return (e && e[0] >= '0' && e[0] <= '9' && valid_mode(e[0] - '0')) ? e[0] - '0' : 0;
}();
static bool fwd_v6() { return g_hashgrid_mode == 0 || g_hashgrid_mode == 7; }
static bool bwd_v2() { return g_hashgrid_mode != 1; }

// Levels per wavefront of the forward walker (1, 2, 4, 8, 16, 32 or 64).
static int fwd_lpw() {
  static const int v = [] {
    const char* e = getenv("ANR_HASH_LPW");  // profiling override
    const int k = e ? atoi(e) : 0;
    return (k >= 1 && k <= 64 && (64 % k) == 0) ? k : 16;
  }();
  return v;
}

// Samples per chunk: long chunks amortise the per-cell gathers/atomics, but the grid
// must still fill 256 CUs. Aim for >= 64K chunks (bench size: 128 samples per chunk,
// forward 0.656 -> 0.646 ms against 64).
// run > 0: the points come in runs of `run` neighbours (anr_hashgrid_fwd_runs), and a
// chunk is one run (up to 256 points), so no chunk straddles two runs. On the extract grid
// (81-point columns, 250 m apart in altitude) the default M / 65,536 = 40-point chunks
// ended or began mid-column every time: 0.782 ms per 2.65 M points against 0.412 ms with
// 81-point chunks (profiles/r04_extract_chunk_sweep.log).
static int64_t pick_chunk(int64_t M, int64_t run = 0) {
  static const int64_t over = env_k("ANR_HASH_KF");
  if (over > 0) return over;
  if (run > 0 && run <= 256) return run;
  int64_t K = M / 65536;
  if (K < 1) K = 1;
  if (K > 128) K = 128;
  return K;
}

template <int D, int F>
static int launch_fwd(const GridLevels& G, const anr_hashgrid_desc* d, const float* x,
                      int64_t x_stride, int64_t M, const void* table, int32_t tdt,
                      void* out, int32_t odt, int64_t out_stride, hipStream_t s,
                      int64_t run = 0) {
  if (F == 2 && d->n_levels <= 16 && fwd_v6()) {
    // 32-bit buffer offsets: every byte range must stay below 2^31
    const int64_t esz_t = tdt == ANR_F16 ? 2 : 4, esz_o = odt == ANR_F16 ? 2 : 4;
    const int64_t x_bytes = ((M - 1) * x_stride + D) * 4;
    const int64_t t_bytes = static_cast<int64_t>(G.offset[d->n_levels - 1] + G.size[d->n_levels - 1]) * 2 * esz_t;
    const int64_t o_bytes = ((M - 1) * out_stride + d->n_levels * 2) * esz_o;
    const int64_t K = pick_chunk(M, run);
    const int64_t lim = int64_t(1) << 31;
    if (x_bytes < lim && t_bytes < lim && o_bytes < lim && (M + K) * x_stride * 4 < lim &&
        (M + K) * out_stride * esz_o < lim) {
      const int64_t chunks = ceil_div(M, K);
      const dim3 grid(static_cast<unsigned>(ceil_div(chunks, 16))), block(256);
#define ANR_HG_FWD6(TT, TO)                                                                    \
  hipLaunchKernelGGL((hashgrid_fwd_v6_kernel<D, TT, TO>), grid, block, 0, s, G, d->n_levels,   \
                     x, static_cast<uint32_t>(x_bytes), static_cast<uint32_t>(x_stride * 4), M, \
                     static_cast<int>(K), static_cast<const TT*>(table),                       \
                     static_cast<uint32_t>(t_bytes), static_cast<TO*>(out),                    \
                     static_cast<uint32_t>(o_bytes), static_cast<uint32_t>(out_stride * esz_o))
      if (tdt == ANR_F16 && odt == ANR_F16) ANR_HG_FWD6(__half, __half);
      else if (tdt == ANR_F16 && odt == ANR_F32) ANR_HG_FWD6(__half, float);
      else if (tdt == ANR_F32 && odt == ANR_F16) ANR_HG_FWD6(float, __half);
      else ANR_HG_FWD6(float, float);
#undef ANR_HG_FWD6
      ANR_CHECK_LAUNCH("anr_hashgrid_fwd(v6)");
      return ANR_OK;
    }
  }
  const int lpw = fwd_lpw();
  const int n_groups = static_cast<int>(ceil_div(d->n_levels, lpw));
  const int64_t K = pick_chunk(M, run);
  const int64_t chunks = ceil_div(M, K);
  const int64_t blocks_per_group = ceil_div(ceil_div(chunks, 64 / lpw), 4);
  const dim3 grid(static_cast<unsigned>(blocks_per_group * n_groups)), block(256);
#define ANR_HG_FWD(TT, TO)                                                                  \
  hipLaunchKernelGGL((hashgrid_fwd_kernel<D, F, TT, TO>), grid, block, 0, s, G,             \
                     d->n_levels, lpw, n_groups, x, x_stride, M, K,                          \
                     static_cast<const TT*>(table), static_cast<TO*>(out), out_stride)
  if (tdt == ANR_F16 && odt == ANR_F16) ANR_HG_FWD(__half, __half);
  else if (tdt == ANR_F16 && odt == ANR_F32) ANR_HG_FWD(__half, float);
  else if (tdt == ANR_F32 && odt == ANR_F16) ANR_HG_FWD(float, __half);
  else ANR_HG_FWD(float, float);
#undef ANR_HG_FWD
  ANR_CHECK_LAUNCH("anr_hashgrid_fwd");
  return ANR_OK;
}

// Cell-move flushes skip corners whose sum is exactly zero (the chunk-end flush always
// did). Under build numerics such sums are rare and the test is pure cost; under the
// reference numerics most samples' f16 dL/denc underflow to zero (tcnn's x128 loss scale
// rounds them away), and the memory-side request count at the chunk ends alone fell from
// 20.8 M to 18.7 M per launch after the first step (profiles/r04_close PMC).
// ANR_HASH_SKIP0 = 0 / 1 / 2 overrides (A/B hook); default 2 (per-sample skip of
// all-zero dL/dy rows, r05).
static int bwd_skip_zero() {
  static const int v = [] {
    const char* e = getenv("ANR_HASH_SKIP0");
    const int k = e ? atoi(e) : 2;
    return k < 0 ? 0 : (k > 2 ? 2 : k);
  }();
  return v;
}

template <int D, int F>
static int launch_bwd(const GridLevels& G, const anr_hashgrid_desc* d, const float* x,
                      int64_t x_stride, int64_t M, const void* dout, int32_t gdt,
                      int64_t dout_stride, float* dtable, hipStream_t s) {
  // v2 addresses the gradient table through a buffer descriptor (32-bit byte offsets, the
  // drop offset at 2 GB): larger tables (2^24 entries x 16 levels) take the v1 walker
  const uint64_t grad_bytes =
      (static_cast<uint64_t>(G.offset[d->n_levels - 1]) + G.size[d->n_levels - 1]) * F * 4u;
  if (F == 2 && d->n_levels <= 16 && grad_bytes < 0x80000000ull && bwd_v2()) {
    const int64_t K = pick_chunk_v2(M);
    const int64_t waves = ceil_div(M, K);
    const dim3 grid(static_cast<unsigned>(ceil_div(waves, 4))), block(256);
    // compile-time strides for the fused field's layout ((M,3) coordinates, (M,32) dL/denc)
    const bool fixed = D == 3 && x_stride == 3 && dout_stride == 32 && g_hashgrid_mode != 7;
#define ANR_HG_BWD2(TG, XS_, DS_)                                                          \
  hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<D, TG, XS_, DS_>), grid, block, 0, s, G,        \
                     d->n_levels, x, x_stride, M, K, static_cast<const TG*>(dout),          \
                     dout_stride, dtable, bwd_skip_zero())
    if (gdt == ANR_F16) {
      if (fixed) ANR_HG_BWD2(__half, 3, 32);
      else ANR_HG_BWD2(__half, 0, 0);
    } else {
      if (fixed) ANR_HG_BWD2(float, 3, 32);
      else ANR_HG_BWD2(float, 0, 0);
    }
#undef ANR_HG_BWD2
    ANR_CHECK_LAUNCH("anr_hashgrid_bwd(v2)");
    return ANR_OK;
  }
  const int lpc = d->n_levels <= 16 ? 16 : 32;
  const int64_t K = pick_chunk(M);
  const int64_t chunks = ceil_div(M, K);
  const int64_t threads = chunks * lpc;
  const dim3 grid(static_cast<unsigned>(ceil_div(threads, 256))), block(256);
  if (gdt == ANR_F16)
    hipLaunchKernelGGL((hashgrid_bwd_kernel<D, F, __half>), grid, block, 0, s, G,
                       d->n_levels, lpc, x, x_stride, M, K,
                       static_cast<const __half*>(dout), dout_stride, dtable);
  else
    hipLaunchKernelGGL((hashgrid_bwd_kernel<D, F, float>), grid, block, 0, s, G,
                       d->n_levels, lpc, x, x_stride, M, K,
                       static_cast<const float*>(dout), dout_stride, dtable);
  ANR_CHECK_LAUNCH("anr_hashgrid_bwd");
  return ANR_OK;
}

}  // namespace anr

extern "C" int anr_hashgrid_force_v1(int32_t mode) {
  ANR_CHECK_ARG(anr::valid_mode(mode), "anr_hashgrid_force_v1: mode %d is not 0, 1, 6 or 7",
                mode);
  const int prev = anr::g_hashgrid_mode;
  anr::g_hashgrid_mode = mode;
  return prev;
}

extern "C" int anr_hashgrid_init(anr_hashgrid_desc* d, int32_t n_dims, int32_t n_levels,
                                 int32_t n_features, int32_t base_resolution,
                                 float per_level_scale, int32_t log2_hashmap_size) {
  using namespace anr;
  ANR_CHECK_ARG(d, "anr_hashgrid_init: null desc");
  ANR_CHECK_ARG(n_dims == 2 || n_dims == 3, "anr_hashgrid_init: n_dims must be 2 or 3");
  ANR_CHECK_ARG(n_levels >= 1 && n_levels <= ANR_MAX_LEVELS,
                "anr_hashgrid_init: n_levels must be in [1, %d]", ANR_MAX_LEVELS);
  ANR_CHECK_ARG(n_features == 1 || n_features == 2 || n_features == 4 || n_features == 8,
                "anr_hashgrid_init: n_features must be 1, 2, 4 or 8");
  ANR_CHECK_ARG(log2_hashmap_size >= 4 && log2_hashmap_size <= 30,
                "anr_hashgrid_init: log2_hashmap_size out of range");
  ANR_CHECK_ARG(base_resolution >= 1 && per_level_scale >= 1.0f,
                "anr_hashgrid_init: bad resolution parameters");
  memset(d, 0, sizeof(*d));
  d->n_dims = n_dims;
  d->n_levels = n_levels;
  d->n_features = n_features;
  d->base_resolution = base_resolution;
  d->per_level_scale = per_level_scale;
  d->log2_hashmap_size = log2_hashmap_size;
  const float log2_pls = std::log2(per_level_scale);
  const uint32_t max_params = 0xffffffffu / 2;
  uint64_t offset = 0;
  for (int l = 0; l < n_levels; ++l) {
    const float scale =
        std::exp2(static_cast<float>(l) * log2_pls) * static_cast<float>(base_resolution) -
        1.0f;
    const uint32_t res = static_cast<uint32_t>(std::ceil(scale)) + 1u;
    uint64_t params_in_level;
    if (std::pow(static_cast<float>(res), static_cast<float>(n_dims)) >
        static_cast<float>(max_params)) {
      params_in_level = max_params;
    } else {
      params_in_level = 1;
      for (int k = 0; k < n_dims; ++k) params_in_level *= res;
    }
    params_in_level = (params_in_level + 7) / 8 * 8;
    const uint64_t T = 1ull << log2_hashmap_size;
    if (params_in_level > T) params_in_level = T;
    d->scales[l] = scale;
    d->resolutions[l] = res;
    d->offsets[l] = static_cast<uint32_t>(offset);
    offset += params_in_level;
    ANR_CHECK_ARG(offset < (1ull << 32), "anr_hashgrid_init: table too large");
  }
  d->offsets[n_levels] = static_cast<uint32_t>(offset);
  d->n_params = static_cast<int64_t>(offset) * n_features;
  return ANR_OK;
}

#define ANR_HG_DISPATCH(FN, ...)                                                   \
  switch (d->n_dims * 16 + d->n_features) {                                        \
    case 2 * 16 + 1: return FN<2, 1>(__VA_ARGS__);                                 \
    case 2 * 16 + 2: return FN<2, 2>(__VA_ARGS__);                                 \
    case 2 * 16 + 4: return FN<2, 4>(__VA_ARGS__);                                 \
    case 2 * 16 + 8: return FN<2, 8>(__VA_ARGS__);                                 \
    case 3 * 16 + 1: return FN<3, 1>(__VA_ARGS__);                                 \
    case 3 * 16 + 2: return FN<3, 2>(__VA_ARGS__);                                 \
    case 3 * 16 + 4: return FN<3, 4>(__VA_ARGS__);                                 \
    case 3 * 16 + 8: return FN<3, 8>(__VA_ARGS__);                                 \
    default:                                                                       \
      ::anr::set_error("hashgrid: unsupported n_dims=%d n_features=%d", d->n_dims, \
                       d->n_features);                                             \
      return ANR_E_UNSUPPORTED;                                                    \
  }

extern "C" int anr_hashgrid_bwd_count_requests(const anr_hashgrid_desc* d, const float* x,
                                               int64_t x_stride, int64_t M, const void* dout,
                                               int32_t dout_dtype, int64_t dout_stride,
                                               const float* dtable, unsigned long long* count,
                                               anr_stream_t stream) {
  using namespace anr;
  ANR_CHECK_ARG(d && x && dout && dtable && count, "anr_hashgrid_bwd_count_requests: null argument");
  ANR_CHECK_ARG(M >= 0 && x_stride >= d->n_dims && dout_stride >= (int64_t)d->n_levels * d->n_features,
                "anr_hashgrid_bwd_count_requests: bad shape/stride");
  ANR_CHECK_ARG(dout_dtype == ANR_F16 || dout_dtype == ANR_F32,
                "anr_hashgrid_bwd_count_requests: bad dtype");
  if (!(d->n_dims == 3 && d->n_features == 2 && d->n_levels <= 16 && bwd_v2())) {
    set_error("anr_hashgrid_bwd_count_requests: only the v2 backward (3-D, 2 features, <= 16 "
              "levels) is instrumented");
    return ANR_E_UNSUPPORTED;
  }
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_bwd_count_requests: descriptor not initialised");
  // the same gate as launch_bwd: gradient tables of 2 GB or more take the v1 walker there,
  // whose requests this v2 instrument does not model
  const uint64_t grad_bytes =
      (static_cast<uint64_t>(G.offset[d->n_levels - 1]) + G.size[d->n_levels - 1]) * 2u * 4u;
  if (grad_bytes >= 0x80000000ull) {
    set_error("anr_hashgrid_bwd_count_requests: gradient table of 2 GB or more (the backward "
              "runs the uninstrumented v1 walker there)");
    return ANR_E_UNSUPPORTED;
  }
  if (M == 0) return ANR_OK;
  const int64_t K = pick_chunk_v2(M);
  const dim3 grid(static_cast<unsigned>(ceil_div(ceil_div(M, K), 4))), block(256);
  float* tab = const_cast<float*>(dtable);  // not written in COUNT mode
  if (dout_dtype == ANR_F16)
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, __half, 0, 0, true>), grid, block, 0,
                       as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const __half*>(dout), dout_stride, tab, bwd_skip_zero(), count);
  else
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, float, 0, 0, true>), grid, block, 0,
                       as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const float*>(dout), dout_stride, tab, bwd_skip_zero(), count);
  ANR_CHECK_LAUNCH("anr_hashgrid_bwd_count_requests");
  return ANR_OK;
}

extern "C" int64_t anr_hashgrid_bwd_chunk(int64_t M) {
  return M > 0 ? anr::pick_chunk_v2(M) : 0;
}

extern "C" int anr_hashgrid_fwd_runs(const anr_hashgrid_desc* d, const float* x,
                                     int64_t x_stride, int64_t M, int64_t run_length,
                                     const void* table, int32_t table_dtype, void* out,
                                     int32_t out_dtype, int64_t out_stride,
                                     anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && x && table && out, "anr_hashgrid_fwd: null argument");
  ANR_CHECK_ARG(run_length >= 0, "anr_hashgrid_fwd_runs: run_length %lld < 0",
                (long long)run_length);
  ANR_CHECK_ARG(M >= 0 && x_stride >= d->n_dims &&
                    out_stride >= (int64_t)d->n_levels * d->n_features,
                "anr_hashgrid_fwd: bad shape/stride");
  ANR_CHECK_ARG((table_dtype == ANR_F16 || table_dtype == ANR_F32) &&
                    (out_dtype == ANR_F16 || out_dtype == ANR_F32),
                "anr_hashgrid_fwd: bad dtype");
  if (M == 0) return ANR_OK;
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_fwd: descriptor not initialised");
  ANR_HG_DISPATCH(launch_fwd, G, d, x, x_stride, M, table, table_dtype, out, out_dtype,
                  out_stride, as_stream(stream), run_length);
}

extern "C" int anr_hashgrid_fwd(const anr_hashgrid_desc* d, const float* x,
                                int64_t x_stride, int64_t M, const void* table,
                                int32_t table_dtype, void* out, int32_t out_dtype,
                                int64_t out_stride, anr_stream_t stream) {
  return anr_hashgrid_fwd_runs(d, x, x_stride, M, 0, table, table_dtype, out, out_dtype,
                               out_stride, stream);
}

extern "C" int anr_hashgrid_fwd_planes(const anr_hashgrid_desc* d, const float* x,
                                       int64_t x_stride, int64_t M, const void* table,
                                       int32_t table_dtype, void* out, int64_t plane_stride,
                                       anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && x && table && out, "anr_hashgrid_fwd_planes: null argument");
  ANR_CHECK_ARG(M > 0 && x_stride >= d->n_dims && plane_stride >= 8 * M,
                "anr_hashgrid_fwd_planes: bad shape/stride (plane_stride >= 8 M)");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0 && (plane_stride & 7) == 0,
                "anr_hashgrid_fwd_planes: out and plane_stride must be 16-byte aligned");
  ANR_CHECK_ARG(table_dtype == ANR_F16 || table_dtype == ANR_F32,
                "anr_hashgrid_fwd_planes: bad dtype");
  ANR_CHECK_ARG(d->n_features == 2 && d->n_levels <= 16 && (d->n_dims == 2 || d->n_dims == 3),
                "anr_hashgrid_fwd_planes: 2 features, <= 16 levels, 2-D or 3-D");
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_fwd_planes: descriptor not initialised");
  const int64_t esz_t = table_dtype == ANR_F16 ? 2 : 4;
  const int64_t n_quads = (d->n_levels + 3) / 4;
  const int64_t x_bytes = ((M - 1) * x_stride + d->n_dims) * 4;
  const int64_t t_bytes =
      static_cast<int64_t>(G.offset[d->n_levels - 1] + G.size[d->n_levels - 1]) * 2 * esz_t;
  const int64_t o_bytes = ((n_quads - 1) * plane_stride + 8 * M) * 2;
  const int64_t lim = int64_t(1) << 31;
  ANR_CHECK_ARG(x_bytes < lim && t_bytes < lim && o_bytes < lim &&
                    (M + 256) * x_stride * 4 < lim && plane_stride * 2 < lim,
                "anr_hashgrid_fwd_planes: byte ranges must stay below 2^31");
  const dim3 grid(static_cast<unsigned>(ceil_div(M, 256))), block(256);
  const int dd = plane_dedup();
#define ANR_HG_PL(D_, TT)                                                                    \
  do {                                                                                       \
    switch (dd) {                                                                            \
      case 0: ANR_HG_PL1(D_, TT, 0); break;                                                  \
      case 16: ANR_HG_PL1(D_, TT, 16); break;                                                \
      case 48: ANR_HG_PL1(D_, TT, 48); break;                                                \
      case 32: ANR_HG_PL1(D_, TT, 32); break;                                                \
      default: ANR_HG_PL1(D_, TT, HASH_DEDUP); break;                                        \
    }                                                                                        \
  } while (0)
#define ANR_HG_PL1(D_, TT, DD)                                                               \
  hipLaunchKernelGGL((hashgrid_fwd_planes_kernel<D_, TT, DD>), grid, block, 0, as_stream(stream), \
                     G, d->n_levels, x, static_cast<uint32_t>(x_bytes),                      \
                     static_cast<uint32_t>(x_stride * 4), M, static_cast<const TT*>(table),  \
                     static_cast<uint32_t>(t_bytes), static_cast<__half*>(out),              \
                     static_cast<uint32_t>(o_bytes), static_cast<uint32_t>(plane_stride * 2))
  if (d->n_dims == 3) {
    if (table_dtype == ANR_F16) ANR_HG_PL(3, __half);
    else ANR_HG_PL(3, float);
  } else {
    if (table_dtype == ANR_F16) ANR_HG_PL(2, __half);
    else ANR_HG_PL(2, float);
  }
#undef ANR_HG_PL
#undef ANR_HG_PL1
  ANR_CHECK_LAUNCH("anr_hashgrid_fwd_planes");
  return ANR_OK;
}

extern "C" int anr_hashgrid_bwd_tiles(const anr_hashgrid_desc* d, const float* x,
                                      int64_t x_stride, int64_t M, const void* dout,
                                      int32_t dout_dtype, int64_t dout_stride, float* dtable,
                                      const uint8_t* tile_nz, anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && x && dout && dtable && tile_nz, "anr_hashgrid_bwd_tiles: null argument");
  ANR_CHECK_ARG(M > 0 && x_stride >= d->n_dims &&
                    dout_stride >= (int64_t)d->n_levels * d->n_features,
                "anr_hashgrid_bwd_tiles: bad shape/stride");
  ANR_CHECK_ARG(dout_dtype == ANR_F16 || dout_dtype == ANR_F32, "anr_hashgrid_bwd_tiles: bad dtype");
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_bwd_tiles: descriptor not initialised");
  const uint64_t grad_bytes =
      (static_cast<uint64_t>(G.offset[d->n_levels - 1]) + G.size[d->n_levels - 1]) * 2u * 4u;
  const int64_t K = pick_chunk_v2(M);
  if (!(d->n_dims == 3 && d->n_features == 2 && d->n_levels <= 16 && bwd_v2() &&
        grad_bytes < 0x80000000ull && K % 32 == 0 && x_stride == 3 && dout_stride == 32)) {
    // outside the tiled walker's shapes: the flags are an optimisation only
    return anr_hashgrid_bwd(d, x, x_stride, M, dout, dout_dtype, dout_stride, dtable, stream);
  }
  const dim3 grid(static_cast<unsigned>(ceil_div(ceil_div(M, K), 4))), block(256);
  if (dout_dtype == ANR_F16)
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, __half, 3, 32, false, 8>), grid, block, 0,
                       as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const __half*>(dout), dout_stride, dtable, bwd_skip_zero(),
                       nullptr, tile_nz);
  else
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, float, 3, 32, false, 8>), grid, block, 0,
                       as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const float*>(dout), dout_stride, dtable, bwd_skip_zero(),
                       nullptr, tile_nz);
  ANR_CHECK_LAUNCH("anr_hashgrid_bwd_tiles");
  return ANR_OK;
}

namespace anr {
// rows whose bit is clear -> 0 (anr_hashgrid_bwd_rows outside its walker: the dense walker
// reads every row, and a clear row need not have been written)
template <typename TG>
__global__ void zero_clear_rows_kernel(TG* __restrict__ dout, int64_t stride, int64_t M, int ncol,
                                       const uint32_t* __restrict__ row_nz) {
  const int64_t n = M * ncol;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t m = e / ncol;
    if (((row_nz[m >> 5] >> (m & 31)) & 1u) == 0u) dout[m * stride + e % ncol] = TG(0.0f);
  }
}
}  // namespace anr

extern "C" int anr_hashgrid_bwd_rows(const anr_hashgrid_desc* d, const float* x,
                                     int64_t x_stride, int64_t M, void* dout,
                                     int32_t dout_dtype, int64_t dout_stride, float* dtable,
                                     const uint32_t* row_nz, anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && x && dout && dtable && row_nz, "anr_hashgrid_bwd_rows: null argument");
  ANR_CHECK_ARG(M > 0 && x_stride >= d->n_dims &&
                    dout_stride >= (int64_t)d->n_levels * d->n_features,
                "anr_hashgrid_bwd_rows: bad shape/stride");
  ANR_CHECK_ARG(dout_dtype == ANR_F16 || dout_dtype == ANR_F32, "anr_hashgrid_bwd_rows: bad dtype");
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_bwd_rows: descriptor not initialised");
  const uint64_t grad_bytes =
      (static_cast<uint64_t>(G.offset[d->n_levels - 1]) + G.size[d->n_levels - 1]) * 2u * 4u;
  // chunks of whole 32-row words (the rule's length rounded down, at least one word)
  int64_t K = pick_chunk_v2(M) / 32 * 32;
  if (K < 32) K = 32;
  if (K > 256) K = 256;
  if (!(d->n_dims == 3 && d->n_features == 2 && d->n_levels == 16 && bwd_v2() &&
        grad_bytes < 0x80000000ull && x_stride == 3 && dout_stride == 32 &&
        M < (int64_t{1} << 31))) {
    // outside the row-mask walker's shapes: the clear rows are zeroed in place, then the
    // dense walker reads every row
    const int ncol = d->n_levels * d->n_features;
    const int64_t nb = ceil_div(M * ncol, 256), blocks = nb < 4096 ? nb : 4096;
    if (dout_dtype == ANR_F16)
      hipLaunchKernelGGL(zero_clear_rows_kernel<__half>, dim3(static_cast<unsigned>(blocks)),
                         dim3(256), 0, as_stream(stream), static_cast<__half*>(dout), dout_stride,
                         M, ncol, row_nz);
    else
      hipLaunchKernelGGL(zero_clear_rows_kernel<float>, dim3(static_cast<unsigned>(blocks)),
                         dim3(256), 0, as_stream(stream), static_cast<float*>(dout), dout_stride,
                         M, ncol, row_nz);
    ANR_CHECK_LAUNCH("anr_hashgrid_bwd_rows(zero)");
    return anr_hashgrid_bwd(d, x, x_stride, M, dout, dout_dtype, dout_stride, dtable, stream);
  }
  const dim3 grid(static_cast<unsigned>(ceil_div(ceil_div(M, K), 4))), block(256);
  if (dout_dtype == ANR_F16)
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, __half, 3, 32, false, HASH_BS, true>), grid,
                       block, 0, as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const __half*>(dout), dout_stride, dtable, 2, nullptr,
                       nullptr, row_nz);
  else
    hipLaunchKernelGGL((hashgrid_bwd_v2_kernel<3, float, 3, 32, false, HASH_BS, true>), grid,
                       block, 0, as_stream(stream), G, d->n_levels, x, x_stride, M, K,
                       static_cast<const float*>(dout), dout_stride, dtable, 2, nullptr,
                       nullptr, row_nz);
  ANR_CHECK_LAUNCH("anr_hashgrid_bwd_rows");
  return ANR_OK;
}

extern "C" int anr_hashgrid_bwd(const anr_hashgrid_desc* d, const float* x,
                                int64_t x_stride, int64_t M, const void* dout,
                                int32_t dout_dtype, int64_t dout_stride, float* dtable,
                                anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && x && dout && dtable, "anr_hashgrid_bwd: null argument");
  ANR_CHECK_ARG(M >= 0 && x_stride >= d->n_dims &&
                    dout_stride >= (int64_t)d->n_levels * d->n_features,
                "anr_hashgrid_bwd: bad shape/stride");
  ANR_CHECK_ARG(dout_dtype == ANR_F16 || dout_dtype == ANR_F32, "anr_hashgrid_bwd: bad dtype");
  if (M == 0) return ANR_OK;
  GridLevels G;
  ANR_CHECK_ARG(make_levels(d, &G), "anr_hashgrid_bwd: descriptor not initialised");
  ANR_HG_DISPATCH(launch_bwd, G, d, x, x_stride, M, dout, dout_dtype, dout_stride, dtable,
                  as_stream(stream));
}
