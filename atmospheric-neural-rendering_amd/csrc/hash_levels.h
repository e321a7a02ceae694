// Hash-grid level tables and the per-sample level-quad evaluation shared by the hash-grid
// kernels (hashgrid.hip) and the fused hash-grid + field forward (field_fused.hip).
// tiny-cuda-nn GridEncoding semantics: see hashgrid.hip's header.
#pragma once

#include "anr_common.h"

#ifndef HASH_DEDUP
// plane_quad: levels whose cells change at no more than this many of a wavefront's lanes
// gather at the run leaders only (see there); 0 = every lane gathers, 64 = every level
#define HASH_DEDUP 64
#endif
#ifndef HASH_FMA_MIX
// Raw2<__half>::fma2 as v_fma_mix_f32 (1) or f16 -> f32 conversions + f32 FMAs (0)
#define HASH_FMA_MIX 1
#endif

namespace anr {

struct GridLevels {
  uint32_t offset[ANR_MAX_LEVELS];
  uint32_t size[ANR_MAX_LEVELS];  // hashmap size T_l (entries)
  uint32_t res[ANR_MAX_LEVELS];
  float scale[ANR_MAX_LEVELS];
};

template <int D>
__device__ __forceinline__ uint32_t grid_index(uint32_t T, uint32_t res, const uint32_t* g) {
  uint32_t stride = 1, index = 0;
#pragma unroll
  for (int d = 0; d < D && stride <= T; ++d) {
    index += g[d] * stride;
    stride *= res;
  }
  if (T < stride) {
    constexpr uint32_t primes[3] = {1u, 2654435761u, 805459861u};
    index = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) index ^= g[d] * primes[d];
    // hashed levels have T = 2^log2_hashmap_size (checked by make_levels): % T == & (T-1)
    return index & (T - 1u);
  }
  // dense levels: index < T except at the far faces (a corner at res) or for coordinates
  // outside [0, 1]; the division is only paid there
  return index < T ? index : index % T;
}

// Per-level corner indexing with the per-cell work hoisted: the 2^D corner indices of a
// cell are built from 2 values per dimension (coordinate and coordinate+1, each times the
// dense stride or the hash prime) with one 3-input add (dense) or xor (hashed) per
// corner. Same result as grid_index for every corner, dense wrap (far faces, coordinates
// outside [0,1]) included; branch-free apart from the rare full modulo.
template <int D>
struct LevelIdx {
  uint32_t T, mul[D], res1;  // res1 = res - 1
  bool hashed;
  __device__ void init(uint32_t T_, uint32_t res) {
    constexpr uint32_t primes[3] = {1u, 2654435761u, 805459861u};
    T = T_;
    res1 = res - 1u;
    uint64_t st = 1;
    uint32_t stride[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      stride[d] = static_cast<uint32_t>(st);
      st *= res;
    }
    hashed = st > T;  // res^D > T, as grid_index decides
#pragma unroll
    for (int d = 0; d < D; ++d) mul[d] = hashed ? primes[d] : stride[d];
  }
  // comp[d][o] = (cell[d] + o) * mul[d]  (uint32 wrap, as tcnn)
  __device__ void dims(const uint32_t* cell, uint32_t (*comp)[2]) const {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      comp[d][0] = cell[d] * mul[d];
      comp[d][1] = comp[d][0] + mul[d];
    }
  }
  // corner c: bit d = offset along dimension d
  __device__ uint32_t corner(const uint32_t (*comp)[2], int c) const {
    uint32_t hx = 0u, sum = 0u;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      hx ^= comp[d][(c >> d) & 1];
      sum += comp[d][(c >> d) & 1];
    }
    if (hashed) return hx & (T - 1u);
    if (sum < T) return sum;
    const uint32_t s1 = sum - T;
    return s1 < T ? s1 : sum % T;
  }
};

template <typename TT>
struct Raw2;
template <>
struct Raw2<__half> {
  using type = uint32_t;  // the two f16 features of one entry
  static constexpr uint32_t bytes = 4;
  __device__ static type load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  }
  // voff per lane, soff wave-uniform (the level's base: the instruction's SGPR offset)
  __device__ static type load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
  }
  // the value of lane src (ds_bpermute)
  __device__ static type from_lane(type v, int src) {
    return static_cast<type>(__builtin_amdgcn_ds_bpermute(src << 2, static_cast<int>(v)));
  }
  // a0 += wt * f32(lo), a1 += wt * f32(hi): the f16 -> f32 conversion is exact, so one
  // mixed-precision FMA per feature is the same single-rounded result as the conversion
  // plus an f32 FMA (hipcc emits the two: it forms v_fma_mix only when f32 denormals are
  // flushed; these products are far above the f32 denormal range)
  __device__ static void fma2(float wt, type v, float& a0, float& a1) {
#if HASH_FMA_MIX
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(a0) : "v"(wt), "v"(v));
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(a1) : "v"(wt), "v"(v));
#else
    const __half2 h = __builtin_bit_cast(__half2, v);
    a0 = fmaf(wt, __low2float(h), a0);
    a1 = fmaf(wt, __high2float(h), a1);
#endif
  }
};
template <>
struct Raw2<float> {
  using type = uint32_t __attribute__((vector_size(8)));
  static constexpr uint32_t bytes = 8;
  __device__ static type load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  }
  __device__ static type load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  }
  __device__ static type from_lane(type v, int src) {
    type o;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      o[k] = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src << 2, static_cast<int>(v[k])));
    return o;
  }
  __device__ static void fma2(float wt, type v, float& a0, float& a1) {
    a0 = fmaf(wt, __uint_as_float(v[0]), a0);
    a1 = fmaf(wt, __uint_as_float(v[1]), a1);
  }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, uint32_t bytes) {
  // descriptor words provably wave-uniform (kernel arguments), so no waterfall loops
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes),
                                           0x00020000);
}


// Level quad q (levels 4q..4q+3, 2 features each, f16 pairs packed in four u32; a partial
// last quad is zero-filled) of the sample at coordinates xv: the forward v9 arithmetic
// (one lane per sample, every corner gathered through the table descriptor rt; same corner
// order, weights and fma chain as the walkers, bit-identical to them).
template <int D, typename TT, int DEDUP = HASH_DEDUP>
__device__ __forceinline__ void plane_quad(const GridLevels& G, int n_levels, int q,
                                           const float* xv, __amdgpu_buffer_rsrc_t rt,
                                           uint32_t (&packed)[4]) {
  using R = Raw2<TT>;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int level = 4 * q + j;
    packed[j] = 0u;
    if (level >= n_levels) continue;  // wave-uniform
    const float scale = G.scale[level];
    const uint32_t res = G.res[level];
    const uint32_t T = G.size[level];
    const uint32_t base = G.offset[level] * R::bytes;
    LevelIdx<D> li;
    li.init(T, res);
    const uint32_t hmask = T - 1u;
    float w[D];
    uint32_t g[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float p = fmaf(scale, xv[d], 0.5f);
      const float fl = floorf(p);
      g[d] = static_cast<uint32_t>(static_cast<int>(fl));
      w[d] = p - fl;
    }
    // idx: the corners' byte offsets within the level (its base goes to the loads' SGPR
    // offset). Hashed levels (wave-uniform branch) hash byte-scaled components: R::bytes is
    // a power of two, so (a*k ^ b*k ^ c*k) & (T-1)*k == ((a ^ b ^ c) & (T-1)) * k, bits
    // lost past 2^32 included (they are above the mask); dense levels scale after the wrap
    uint32_t idx[1 << D];
    if (li.hashed) {
      uint32_t comp[D][2];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const uint32_t m = li.mul[d] * R::bytes;
        comp[d][0] = g[d] * m;
        comp[d][1] = comp[d][0] + m;
      }
      const uint32_t hmb = hmask * R::bytes;
#pragma unroll
      for (int c = 0; c < (1 << D); ++c) {
        uint32_t hx = 0u;
#pragma unroll
        for (int d = 0; d < D; ++d) hx ^= comp[d][(c >> d) & 1];
        idx[c] = hx & hmb;
      }
    } else {
      uint32_t comp[D][2];
      li.dims(g, comp);
      uint32_t sum[1 << D];
#pragma unroll
      for (int c = 0; c < (1 << D); ++c) {
        uint32_t sm = 0u;
#pragma unroll
        for (int d = 0; d < D; ++d) sm += comp[d][(c >> d) & 1];
        sum[c] = sm;
        idx[c] = sm;
      }
      uint32_t gmax = g[0];
#pragma unroll
      for (int d = 1; d < D; ++d) gmax = gmax > g[d] ? gmax : g[d];
      if (gmax >= res - 1u) {
#pragma unroll
        for (int c = 0; c < (1 << D); ++c)
          if (sum[c] >= T) {
            const uint32_t s1 = sum[c] - T;
            idx[c] = s1 < T ? s1 : sum[c] % T;
          }
      }
#pragma unroll
      for (int c = 0; c < (1 << D); ++c) idx[c] *= R::bytes;
    }
    typename R::type val[1 << D];
    bool plain = true;
    if constexpr (DEDUP > 0) {
      // Lanes are consecutive samples of a ray, so runs of lanes share a cell (one run per
      // wavefront on the coarse levels, every few samples on the finest). The gathers'
      // cost is address processing per active lane (profiles/r06_ta_probe.log: masked
      // lanes are skipped), so only the first lane of each run gathers and the run's other
      // lanes take its corner values through ds_bpermute (the LDS crossbar, not the
      // texture path). Levels whose cells change at more than DEDUP lanes gather
      // plainly. The same entries reach every lane: bit-identical.
      const int lane = __lane_id();
      bool lead = lane == 0;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        // the previous lane's cell (DPP wave_shr:1; lane 0 reads 0 and leads anyway)
        const uint32_t pg = static_cast<uint32_t>(
            __builtin_amdgcn_update_dpp(0, static_cast<int>(g[d]), 0x138, 0xf, 0xf, false));
        lead = lead || pg != g[d];
      }
      const uint64_t lm = __ballot(lead);
      if (__popcll(lm) <= DEDUP) {  // wave-uniform
        plain = false;
        // this lane's run leader: the highest leading lane at or below it
        const uint64_t below = lm & ((2ull << lane) - 1ull);
        const int src = 63 - static_cast<int>(__clzll(static_cast<long long>(below)));
        if (lead) {
#pragma unroll
          for (int c = 0; c < (1 << D); ++c) val[c] = R::load(rt, idx[c], base);
        }
#pragma unroll
        for (int c = 0; c < (1 << D); ++c) val[c] = R::from_lane(val[c], src);
      }
    }
    if (plain) {
#pragma unroll
      for (int c = 0; c < (1 << D); ++c) val[c] = R::load(rt, idx[c], base);
    }
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
    for (int c = 0; c < (1 << D); ++c) {
      float wt = 1.0f;
#pragma unroll
      for (int d = 0; d < D; ++d) wt *= ((c >> d) & 1) ? w[d] : 1.0f - w[d];
      R::fma2(wt, val[c], a0, a1);
    }
    packed[j] = __builtin_bit_cast(uint32_t, __floats2half2_rn(a0, a1));
  }
}

// host: the level tables of a descriptor (false: not initialised / invalid)
inline bool make_levels(const anr_hashgrid_desc* d, GridLevels* G) {
  if (d->n_levels < 1 || d->n_levels > ANR_MAX_LEVELS) return false;
  for (int l = 0; l < d->n_levels; ++l) {
    G->offset[l] = d->offsets[l];
    G->size[l] = d->offsets[l + 1] - d->offsets[l];
    G->res[l] = d->resolutions[l];
    G->scale[l] = d->scales[l];
    if (G->size[l] == 0) return false;
    // grid_index: a level too large for a dense table is hashed, and its size must be a
    // power of two there (always true for tcnn's min(next_mult(res^D, 8), 2^log2T))
    uint64_t dense = 1;
    for (int k = 0; k < d->n_dims && dense <= G->size[l]; ++k) dense *= G->res[l];
    if (dense > G->size[l] && (G->size[l] & (G->size[l] - 1)) != 0) return false;
  }
  return true;
}

}  // namespace anr
