// K6+K7 fused: the whole per-sample Instant-NGP radiance field after the hash encoding,
// forward and backward, in one kernel each (f16 MFMA, f32 accumulation).
//
//   pos_out = pos_mlp(enc)                       32 -> W -> 16     (instant_ngp.py:163-164)
//   sigma   = relu(pos_out[:, 0])                                  (:178,184)
//   x_dir   = [SH2(dir) | pos_out[:, 1:16] | 1.0 ...]              (:165-169)
//   color   = relu(dir_mlp(x_dir))               32 -> W (x NHD) -> 16  (:170-171,183)
//
// Layers are evaluated in transposed form on v_mfma_f32_16x16x32_f16, out^T = W · in^T,
// with 16 samples as the MFMA's N dimension. The C tile of one layer (lane = sample
// l&15, units 4(l>>4)+i of each 16-unit block) is, after ReLU and f16 conversion, the B
// operand of the next layer once that layer's weight columns are permuted the same way
// (perm32 below) — so no activation of the forward chain, and no gradient of the
// backward dAct chain, goes through LDS. The packed weight buffer (anr_ingp_field_pack)
// stores every weight matrix directly in MFMA A-fragment order, lane-linear, with those
// permutations (and the dir-input column order) applied.
//
// Backward: per 32-sample tile the forward is recomputed; each layer's input and output
// gradient tiles are written to LDS once, row-major, and read back transposed with
// ds_read_b64_tr_b16 as the operands of dW += G^T · X (contraction over the 32 samples),
// which accumulates in registers across all tiles of a wavefront and is flushed with
// one f32 atomic per element at the end. Gradients are scaled in f16 by one power of two
// per wavefront (pre-pass over |dL/dcolor| and |dL/dsigma|) and unscaled in f32.
// dL/dpos_out never leaves the registers; the kernel writes only dL/denc (f32).

#include "anr_common.h"

namespace anr {
namespace field {

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

__device__ __forceinline__ f4 mma32(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mma16(h4 a, h4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}

// B-operand slot k' (0..31) of a 32-wide K block -> unit index when the operand is the
// concatenation of two C tiles' lane values (4 from block 2kb, 4 from block 2kb+1).
__host__ __device__ constexpr int perm32(int k) {
  return ((k & 4) ? 16 : 0) + 4 * (k >> 3) + (k & 3);
}
// Dir-MLP input slot k' -> tcnn input column. Lane group g holds pos_out[4g..4g+3] in
// slots 8g..8g+3 (pos_out[p] is column p+3; slot 0 carries a 1.0 padding column instead
// of pos_out[0] = density), and SH2 (g = 0) or more 1.0 padding (g > 0) in 8g+4..8g+7.
__host__ __device__ constexpr int dir_col(int k) {
  const int g = k >> 3, j = k & 7;
  return j < 4 ? ((g == 0 && j == 0) ? 19 : 4 * g + j + 3) : (g == 0 ? j - 4 : 20 + 4 * (g - 1) + (j - 4));
}

template <int W, int NHD>
struct Net {
  static_assert(W == 32 || W == 64, "width 32 or 64");
  static_assert(NHD == 1 || NHD == 2, "1 or 2 dir hidden layers");
  static constexpr int NT = W / 16, KB = W / 32;
  static constexpr int F32 = 512, F16 = 256;  // halves per 16x16x32 / 16x16x16 A fragment
  // parameter offsets (tcnn order, each layer row-major [out][in])
  static constexpr int P0 = 0, P1 = 32 * W, NPOS = 32 * W + 16 * W;
  static constexpr int D0 = 0, D1 = 32 * W, D2 = 32 * W + (NHD - 1) * W * W;
  static constexpr int NDIR = D2 + 16 * W;
  // packed fragment offsets (halves): forward A = W, backward A = W^T
  static constexpr int oFP0 = 0;                                  // [NT]
  static constexpr int oFP1 = oFP0 + NT * F32;                    // [KB]
  static constexpr int oFD0 = oFP1 + KB * F32;                    // [NT]
  static constexpr int oFD1 = oFD0 + NT * F32;                    // [NT][KB] (NHD == 2)
  static constexpr int oFD2 = oFD1 + (NHD - 1) * NT * KB * F32;   // [KB]
  static constexpr int n_fwd = oFD2 + KB * F32;
  static constexpr int oBD2 = n_fwd;                              // [NT] 16x16x16
  static constexpr int oBD1 = oBD2 + NT * F16;                    // [NT][KB] (NHD == 2)
  static constexpr int oBD0 = oBD1 + (NHD - 1) * NT * KB * F32;   // [KB]
  static constexpr int oBP1 = oBD0 + KB * F32;                    // [NT] 16x16x16
  static constexpr int oBP0 = oBP1 + NT * F16;                    // [2][KB]
  static constexpr int n_packed = oBP0 + 2 * KB * F32;
  static constexpr int n_bwd = n_packed - n_fwd;
  // backward per-wave LDS tiles (32 samples, row-major, +8 halves of padding per row)
  static constexpr int LX = 40, LH = W + 8;
  static constexpr int oXpe = 0;                  // enc            [32][LX]
  static constexpr int oXph = oXpe + 32 * LX;     // pos hidden     [32][LH]
  static constexpr int oXde = oXph + 32 * LH;     // dir input (k') [32][LX]
  static constexpr int oXd0 = oXde + 32 * LX;     // dir hidden 0   [32][LH]
  static constexpr int oXd1 = oXd0 + 32 * LH;     // dir hidden 1   [32][LH] (NHD == 2)
  static constexpr int oGa = oXd1 + (NHD - 1) * 32 * LH;
  static constexpr int oGb = oGa + 32 * LH;
  static constexpr int wave_lds = oGb + 32 * LH;
};

// ---------------------------------------------------------------------------------
// weight packing (f32 master params -> f16 fragments)
// ---------------------------------------------------------------------------------
template <int W, int NHD>
__global__ void pack_kernel(const float* __restrict__ pp, const float* __restrict__ pd,
                            _Float16* __restrict__ out) {
  using N = Net<W, NHD>;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N::n_packed) return;
  int f, r, k;
  auto frag32 = [&](int base) {
    const int o = e - base;
    f = o / N::F32;
    const int w = o - f * N::F32, lane = w >> 3;
    r = lane & 15;
    k = 8 * (lane >> 4) + (w & 7);
  };
  auto frag16 = [&](int base) {
    const int o = e - base;
    f = o / N::F16;
    const int w = o - f * N::F16, lane = w >> 2;
    r = lane & 15;
    k = 4 * (lane >> 4) + (w & 3);
  };
  constexpr int W_ = W;
  float v;
  if (e < N::oFP1) {
    frag32(N::oFP0);
    v = pp[N::P0 + (16 * f + r) * 32 + k];
  } else if (e < N::oFD0) {
    frag32(N::oFP1);
    v = pp[N::P1 + r * W_ + 32 * f + perm32(k)];
  } else if (e < N::oFD1) {
    frag32(N::oFD0);
    v = pd[N::D0 + (16 * f + r) * 32 + dir_col(k)];
  } else if (e < N::oFD2) {
    frag32(N::oFD1);
    const int nt = f / N::KB, kb = f - nt * N::KB;
    v = pd[N::D1 + (16 * nt + r) * W_ + 32 * kb + perm32(k)];
  } else if (e < N::oBD2) {
    frag32(N::oFD2);
    v = pd[N::D2 + r * W_ + 32 * f + perm32(k)];
  } else if (e < N::oBD1) {
    frag16(N::oBD2);
    v = pd[N::D2 + k * W_ + 16 * f + r];
  } else if (e < N::oBD0) {
    frag32(N::oBD1);
    const int kt = f / N::KB, kb = f - kt * N::KB;
    v = pd[N::D1 + (32 * kb + perm32(k)) * W_ + 16 * kt + r];
  } else if (e < N::oBP1) {
    frag32(N::oBD0);
    v = r == 0 ? 0.0f : pd[N::D0 + (32 * f + perm32(k)) * 32 + r + 3];
  } else if (e < N::oBP0) {
    frag16(N::oBP1);
    v = pp[N::P1 + k * W_ + 16 * f + r];
  } else {
    frag32(N::oBP0);
    const int kt = f / N::KB, kb = f - kt * N::KB;
    v = pp[N::P0 + (32 * kb + perm32(k)) * 32 + 16 * kt + r];
  }
  out[e] = static_cast<_Float16>(v);
}

struct Args {
  const _Float16* packed;
  const _Float16* enc;
  int64_t enc_stride;
  const float* dirs;
  uint32_t n_per_ray;
  int64_t M;
  int n_out;
  float* sigma;
  float* color;
  int64_t color_stride;
  const float* d_sigma;
  const float* d_color;
  int64_t d_color_stride;
  float* d_enc;
  int64_t d_enc_stride;
  float* g_pos;
  float* g_dir;
};

__device__ __forceinline__ h8 cat(h4 a, h4 b) {
  return h8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}
__device__ __forceinline__ h4 relu_h4(f4 v) {
  return h4{static_cast<_Float16>(fmaxf(v[0], 0.0f)), static_cast<_Float16>(fmaxf(v[1], 0.0f)),
            static_cast<_Float16>(fmaxf(v[2], 0.0f)), static_cast<_Float16>(fmaxf(v[3], 0.0f))};
}
__device__ __forceinline__ h4 to_h4(f4 v) {
  return h4{static_cast<_Float16>(v[0]), static_cast<_Float16>(v[1]),
            static_cast<_Float16>(v[2]), static_cast<_Float16>(v[3])};
}
// zero where the forward activation was not positive (ReLU derivative)
__device__ __forceinline__ h4 mask_h4(f4 g, h4 act) {
  return h4{static_cast<_Float16>(act.x > static_cast<_Float16>(0) ? g[0] : 0.0f),
            static_cast<_Float16>(act.y > static_cast<_Float16>(0) ? g[1] : 0.0f),
            static_cast<_Float16>(act.z > static_cast<_Float16>(0) ? g[2] : 0.0f),
            static_cast<_Float16>(act.w > static_cast<_Float16>(0) ? g[3] : 0.0f)};
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Input row of the dir MLP for the sample in this lane (B-operand slots 8g..8g+7).
__device__ __forceinline__ h8 dir_input(const Args& a, int64_t row, int g, f4 po) {
  if (row >= a.M) return h8{};
  h8 x;
  if (g == 0) {
    const uint32_t ray = static_cast<uint32_t>(row) / a.n_per_ray;
    const float* d = a.dirs + static_cast<int64_t>(ray) * 3;
    const float dx = d[0] * 2.0f - 1.0f, dy = d[1] * 2.0f - 1.0f, dz = d[2] * 2.0f - 1.0f;
    x = h8{static_cast<_Float16>(1.0f), static_cast<_Float16>(po[1]),
           static_cast<_Float16>(po[2]), static_cast<_Float16>(po[3]),
           static_cast<_Float16>(0.28209479177387814f),
           static_cast<_Float16>(-0.48860251190291987f * dy),
           static_cast<_Float16>(0.48860251190291987f * dz),
           static_cast<_Float16>(-0.48860251190291987f * dx)};
  } else {
    const _Float16 one = static_cast<_Float16>(1.0f);
    x = h8{static_cast<_Float16>(po[0]), static_cast<_Float16>(po[1]),
           static_cast<_Float16>(po[2]), static_cast<_Float16>(po[3]), one, one, one, one};
  }
  return x;
}

template <int W, int NHD>
struct FwdWeights {
  using N = Net<W, NHD>;
  h8 p0[N::NT], p1[N::KB], d0[N::NT], d1[NHD == 2 ? N::NT * N::KB : 1], d2[N::KB];
  __device__ void load(const _Float16* pk, int lane) {
    auto ld = [&](int off) { return *reinterpret_cast<const h8*>(pk + off + lane * 8); };
#pragma unroll
    for (int i = 0; i < N::NT; ++i) p0[i] = ld(N::oFP0 + i * N::F32);
#pragma unroll
    for (int i = 0; i < N::KB; ++i) p1[i] = ld(N::oFP1 + i * N::F32);
#pragma unroll
    for (int i = 0; i < N::NT; ++i) d0[i] = ld(N::oFD0 + i * N::F32);
    if constexpr (NHD == 2) {
#pragma unroll
      for (int i = 0; i < N::NT * N::KB; ++i) d1[i] = ld(N::oFD1 + i * N::F32);
    }
#pragma unroll
    for (int i = 0; i < N::KB; ++i) d2[i] = ld(N::oFD2 + i * N::F32);
  }
};

// Forward of one 16-sample tile; every intermediate the backward needs is returned.
template <int W, int NHD>
struct Tile {
  using N = Net<W, NHD>;
  h8 xe, xd;
  h4 hp[N::NT], hd0[N::NT], hd1[NHD == 2 ? N::NT : 1];
  f4 po, col;
};

template <int W, int NHD>
__device__ __forceinline__ void tile_forward(const Args& a, const FwdWeights<W, NHD>& fw,
                                             int64_t row, int g, Tile<W, NHD>& t) {
  using N = Net<W, NHD>;
  t.xe = h8{};
  if (row < a.M) t.xe = *reinterpret_cast<const h8*>(a.enc + row * a.enc_stride + 8 * g);
#pragma unroll
  for (int nt = 0; nt < N::NT; ++nt)
    t.hp[nt] = relu_h4(mma32(fw.p0[nt], t.xe, f4{0.0f, 0.0f, 0.0f, 0.0f}));
  t.po = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int kb = 0; kb < N::KB; ++kb) t.po = mma32(fw.p1[kb], cat(t.hp[2 * kb], t.hp[2 * kb + 1]), t.po);
  t.xd = dir_input(a, row, g, t.po);
#pragma unroll
  for (int nt = 0; nt < N::NT; ++nt)
    t.hd0[nt] = relu_h4(mma32(fw.d0[nt], t.xd, f4{0.0f, 0.0f, 0.0f, 0.0f}));
  const h4* last = t.hd0;
  if constexpr (NHD == 2) {
#pragma unroll
    for (int nt = 0; nt < N::NT; ++nt) {
      f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kb = 0; kb < N::KB; ++kb)
        acc = mma32(fw.d1[nt * N::KB + kb], cat(t.hd0[2 * kb], t.hd0[2 * kb + 1]), acc);
      t.hd1[nt] = relu_h4(acc);
    }
    last = t.hd1;
  }
  t.col = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int kb = 0; kb < N::KB; ++kb) t.col = mma32(fw.d2[kb], cat(last[2 * kb], last[2 * kb + 1]), t.col);
}

template <int W, int NHD>
__global__ void __launch_bounds__(256) fwd_kernel(Args a) {
  using N = Net<W, NHD>;
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int waves = blockDim.x >> 6, wave = threadIdx.x >> 6;
  FwdWeights<W, NHD> fw;
  fw.load(a.packed, lane);
  const int64_t n_tiles = (a.M + 15) / 16;
  for (int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave; tile < n_tiles;
       tile += static_cast<int64_t>(gridDim.x) * waves) {
    const int64_t row = tile * 16 + (lane & 15);
    Tile<W, NHD> t;
    tile_forward<W, NHD>(a, fw, row, g, t);
    if (row < a.M) {
      if (g == 0) a.sigma[row] = fmaxf(t.po[0], 0.0f);
      const int c0 = 4 * g;
      if (c0 + 3 < a.n_out && (a.color_stride & 3) == 0) {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(t.col[i], 0.0f);
        *reinterpret_cast<f4*>(a.color + row * a.color_stride + c0) = v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (c0 + i < a.n_out) a.color[row * a.color_stride + c0 + i] = fmaxf(t.col[i], 0.0f);
      }
    }
  }
}

// lane (column c = l&15 of a 16-column block at col0) receives rows 8g..8g+7 of that
// column of a row-major LDS tile: two 4x16 hardware-transposed reads
__device__ __forceinline__ h8 tr_read(const _Float16* base, int ld, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const _Float16* p0 = base + (8 * g + (li >> 2)) * ld + col0 + 4 * (li & 3);
  const _Float16* p1 = p0 + 4 * ld;
  const s4v v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p0));
  const s4v v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p1));
  return cat(__builtin_bit_cast(h4, v0), __builtin_bit_cast(h4, v1));
}

// C-layout (sample l&15, units 4g..4g+3) store into row `mrow` of a row-major tile
__device__ __forceinline__ void st4(_Float16* base, int ld, int mrow, int col, h4 v) {
  *reinterpret_cast<h4*>(base + mrow * ld + col) = v;
}

template <int W, int NHD>
__global__ void __launch_bounds__(256) bwd_kernel(Args a, float target) {
  using N = Net<W, NHD>;
  constexpr int NT = N::NT, KB = N::KB, LX = N::LX, LH = N::LH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  _Float16* wb = reinterpret_cast<_Float16*>(smem);  // backward fragments, N::n_bwd halves
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int waves = blockDim.x >> 6, wave = threadIdx.x >> 6;
  for (int e = threadIdx.x * 8; e < N::n_bwd; e += blockDim.x * 8)
    *reinterpret_cast<h8*>(wb + e) = *reinterpret_cast<const h8*>(a.packed + N::n_fwd + e);
  _Float16* L = wb + N::n_bwd + wave * N::wave_lds;
  _Float16* Xpe = L + N::oXpe;
  _Float16* Xph = L + N::oXph;
  _Float16* Xde = L + N::oXde;
  _Float16* Xd0 = L + N::oXd0;
  _Float16* Xd1 = L + N::oXd1;
  _Float16* Ga = L + N::oGa;
  _Float16* Gb = L + N::oGb;
  _Float16* Xlast = NHD == 2 ? Xd1 : Xd0;
  FwdWeights<W, NHD> fw;
  fw.load(a.packed, lane);
  __syncthreads();
  auto bfrag32 = [&](int off) { return *reinterpret_cast<const h8*>(wb + (off - N::n_fwd) + lane * 8); };
  auto bfrag16 = [&](int off) { return *reinterpret_cast<const h4*>(wb + (off - N::n_fwd) + lane * 4); };

  const int64_t n_tiles = (a.M + 31) / 32;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * waves + wave;
  const int64_t tstride = static_cast<int64_t>(gridDim.x) * waves;

  // per-wavefront gradient scale: max(|dL/dcolor|, |dL/dsigma|) over this wave's rows -> target
  float s = 1.0f, inv_s = 1.0f;
  {
    float gmax = 0.0f;
    for (int64_t tile = t0; tile < n_tiles; tile += tstride) {
      const int64_t row = tile * 32 + (lane & 31);
      if (row < a.M) {
        const int half = lane >> 5;  // two lanes per row: columns split
        for (int c = half; c < a.n_out; c += 2)
          gmax = fmaxf(gmax, fabsf(a.d_color[row * a.d_color_stride + c]));
        if (half == 0 && a.d_sigma) gmax = fmaxf(gmax, fabsf(a.d_sigma[row]));
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) gmax = fmaxf(gmax, __shfl_xor(gmax, m));
    if (gmax > 0.0f) {
      int e2 = static_cast<int>(floorf(log2f(target / gmax)));
      e2 = e2 < -60 ? -60 : (e2 > 100 ? 100 : e2);
      s = ldexpf(1.0f, e2);
      inv_s = ldexpf(1.0f, -e2);
    }
  }

  f4 dD2[NT], dD1[NHD == 2 ? NT * NT : 1], dD0[NT * 2], dP1[NT], dP0[NT * 2];
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < NT; ++i) dD2[i] = dP1[i] = z4;
#pragma unroll
  for (int i = 0; i < NT * 2; ++i) dD0[i] = dP0[i] = z4;
  if constexpr (NHD == 2) {
#pragma unroll
    for (int i = 0; i < NT * NT; ++i) dD1[i] = z4;
  }

  for (int64_t tile = t0; tile < n_tiles; tile += tstride) {
    Tile<W, NHD> t[2];
    h4 gc[2];
    bool dens[2];
    // ---- recompute the forward for both 16-sample halves, write layer inputs to LDS
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int64_t row = tile * 32 + mt * 16 + li;
      const int m = mt * 16 + li;
      tile_forward<W, NHD>(a, fw, row, g, t[mt]);
      *reinterpret_cast<h8*>(Xpe + m * LX + 8 * g) = t[mt].xe;
      *reinterpret_cast<h8*>(Xde + m * LX + 8 * g) = t[mt].xd;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        st4(Xph, LH, m, 16 * nt + 4 * g, t[mt].hp[nt]);
        st4(Xd0, LH, m, 16 * nt + 4 * g, t[mt].hd0[nt]);
        if constexpr (NHD == 2) st4(Xd1, LH, m, 16 * nt + 4 * g, t[mt].hd1[nt]);
      }
      dens[mt] = t[mt].po[0] > 0.0f;
      // dL/d(color pre-activation), scaled
      f4 gv = z4;
      if (row < a.M) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 4 * g + i;
          if (c < a.n_out && t[mt].col[i] > 0.0f) gv[i] = a.d_color[row * a.d_color_stride + c] * s;
        }
      }
      gc[mt] = to_h4(gv);
      st4(Ga, LH, m, 4 * g, gc[mt]);
    }
    wave_sync();
    // ---- dir output layer: dW_D2 (16 x W) += gc^T · X_last ; dX_last = D2^T gc
    {
      const h8 ga = tr_read(Ga, LH, 0, lane);
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) dD2[kt] = mma32(ga, tr_read(Xlast, LH, 16 * kt, lane), dD2[kt]);
    }
    h4 dl[2][NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const h4 wf = bfrag16(N::oBD2 + kt * N::F16);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f4 acc = mma16(wf, gc[mt], z4);
        dl[mt][kt] = mask_h4(acc, NHD == 2 ? t[mt].hd1[kt] : t[mt].hd0[kt]);
        st4(Gb, LH, mt * 16 + li, 16 * kt + 4 * g, dl[mt][kt]);
      }
    }
    wave_sync();
    // ---- dir hidden layer 1 (NHD == 2): dW_D1 (W x W) += dl^T · X_d0 ; dh0 = D1^T dl
    h4 dh0[2][NT];
    _Float16* Gdh0 = Gb;
    if constexpr (NHD == 2) {
      h8 xb[NT];
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) xb[kt] = tr_read(Xd0, LH, 16 * kt, lane);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const h8 ga = tr_read(Gb, LH, 16 * nt, lane);
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) dD1[nt * NT + kt] = mma32(ga, xb[kt], dD1[nt * NT + kt]);
      }
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        f4 acc[2] = {z4, z4};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          const h8 wf = bfrag32(N::oBD1 + (kt * KB + kb) * N::F32);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) acc[mt] = mma32(wf, cat(dl[mt][2 * kb], dl[mt][2 * kb + 1]), acc[mt]);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          dh0[mt][kt] = mask_h4(acc[mt], t[mt].hd0[kt]);
          st4(Ga, LH, mt * 16 + li, 16 * kt + 4 * g, dh0[mt][kt]);
        }
      }
      Gdh0 = Ga;
      wave_sync();
    } else {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) dh0[mt][kt] = dl[mt][kt];
    }
    _Float16* Gfree = Gdh0 == Ga ? Gb : Ga;
    // ---- dir input layer: dW_D0 (W x 32, k' order) += dh0^T · X_de ; dpos = D0^T dh0
    {
      const h8 x0 = tr_read(Xde, LX, 0, lane), x1 = tr_read(Xde, LX, 16, lane);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const h8 ga = tr_read(Gdh0, LH, 16 * nt, lane);
        dD0[nt * 2] = mma32(ga, x0, dD0[nt * 2]);
        dD0[nt * 2 + 1] = mma32(ga, x1, dD0[nt * 2 + 1]);
      }
    }
    h4 dpo[2];
    {
      f4 acc[2] = {z4, z4};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const h8 wf = bfrag32(N::oBD0 + kb * N::F32);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt] = mma32(wf, cat(dh0[mt][2 * kb], dh0[mt][2 * kb + 1]), acc[mt]);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int64_t row = tile * 32 + mt * 16 + li;
        if (g == 0) {  // pos_out[:, 0] is the density: its gradient is dL/dsigma through the ReLU
          const float ds = (a.d_sigma && row < a.M && dens[mt]) ? a.d_sigma[row] * s : 0.0f;
          acc[mt][0] = ds;
        }
        dpo[mt] = to_h4(acc[mt]);
        st4(Gfree, LH, mt * 16 + li, 4 * g, dpo[mt]);
      }
    }
    wave_sync();
    // ---- pos output layer: dW_P1 (16 x W) += dpo^T · X_ph ; dhp = P1^T dpo
    {
      const h8 ga = tr_read(Gfree, LH, 0, lane);
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) dP1[kt] = mma32(ga, tr_read(Xph, LH, 16 * kt, lane), dP1[kt]);
    }
    h4 dhp[2][NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      const h4 wf = bfrag16(N::oBP1 + kt * N::F16);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        dhp[mt][kt] = mask_h4(mma16(wf, dpo[mt], z4), t[mt].hp[kt]);
        st4(Gdh0, LH, mt * 16 + li, 16 * kt + 4 * g, dhp[mt][kt]);
      }
    }
    wave_sync();
    // ---- pos input layer: dW_P0 (W x 32) += dhp^T · X_pe ; d_enc = P0^T dhp
    {
      const h8 x0 = tr_read(Xpe, LX, 0, lane), x1 = tr_read(Xpe, LX, 16, lane);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const h8 ga = tr_read(Gdh0, LH, 16 * nt, lane);
        dP0[nt * 2] = mma32(ga, x0, dP0[nt * 2]);
        dP0[nt * 2 + 1] = mma32(ga, x1, dP0[nt * 2 + 1]);
      }
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f4 acc[2] = {z4, z4};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const h8 wf = bfrag32(N::oBP0 + (kt * KB + kb) * N::F32);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt] = mma32(wf, cat(dhp[mt][2 * kb], dhp[mt][2 * kb + 1]), acc[mt]);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int64_t row = tile * 32 + mt * 16 + li;
        if (row < a.M) {
          const f4 v = acc[mt] * inv_s;
          *reinterpret_cast<f4*>(a.d_enc + row * a.d_enc_stride + 16 * kt + 4 * g) = v;
        }
      }
    }
    wave_sync();
  }

  // ---- flush: lane holds dW[n = 16·ntile + 4g + i][k = 16·ktile + li]
  auto flush = [&](float* dst, int ld, const f4& d, int n0, int k) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (d[i] != 0.0f) atomicAdd(dst + (n0 + 4 * g + i) * ld + k, d[i] * inv_s);
  };
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    flush(a.g_dir + N::D2, W, dD2[kt], 0, 16 * kt + li);
    flush(a.g_pos + N::P1, W, dP1[kt], 0, 16 * kt + li);
  }
  if constexpr (NHD == 2) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) flush(a.g_dir + N::D1, W, dD1[nt * NT + kt], 16 * nt, 16 * kt + li);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      flush(a.g_dir + N::D0, 32, dD0[nt * 2 + kt], 16 * nt, dir_col(16 * kt + li));
      flush(a.g_pos + N::P0, 32, dP0[nt * 2 + kt], 16 * nt, 16 * kt + li);
    }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
static int g_target_log2 = 6;  // f16 gradient scale: max |dL/dout| of a wavefront -> 2^6

template <int W, int NHD>
static int run(int op, const Args& a, hipStream_t st) {
  using N = Net<W, NHD>;
  const int waves = 4;
  const int64_t tile_rows = op == 1 ? 16 : 32;
  const int64_t tiles = (a.M + tile_rows - 1) / tile_rows;
  const void* fn = op == 1 ? reinterpret_cast<const void*>(&fwd_kernel<W, NHD>)
                           : reinterpret_cast<const void*>(&bwd_kernel<W, NHD>);
  const size_t lds = op == 1 ? 0 : (static_cast<size_t>(N::n_bwd) + waves * N::wave_lds) * 2;
  if (lds > 160 * 1024) return 1;
  if (lds) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  static int per_cu[3] = {0, 0, 0};
  int& pc = per_cu[op];
  if (pc == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * waves, lds) != hipSuccess || nb < 1) nb = 1;
    pc = nb;
  }
  int64_t blocks = (tiles + waves - 1) / waves;
  const int64_t cap = 256LL * pc;  // persistent: one resident wave per slot
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (op == 1)
    hipLaunchKernelGGL((fwd_kernel<W, NHD>), dim3(blocks), dim3(64 * waves), 0, st, a);
  else
    hipLaunchKernelGGL((bwd_kernel<W, NHD>), dim3(blocks), dim3(64 * waves), lds, st, a,
                       ldexpf(1.0f, g_target_log2));
  return 0;
}

template <int W, int NHD>
static void launch_pack(const float* pp, const float* pd, _Float16* out, hipStream_t st) {
  using N = Net<W, NHD>;
  hipLaunchKernelGGL((pack_kernel<W, NHD>), dim3((N::n_packed + 255) / 256), dim3(256), 0, st, pp, pd, out);
}

// (W, NHD) of a supported pos/dir pair, or 0
static int variant(const anr_mlp_desc* pos, const anr_mlp_desc* dir) {
  if (!pos || !dir) return 0;
  if (pos->n_input != 32 || pos->n_input_padded != 32 || pos->n_output != 16 ||
      pos->n_output_padded != 16 || pos->n_hidden_layers != 1 ||
      pos->output_activation != ANR_ACT_NONE)
    return 0;
  if (dir->n_input != 19 || dir->n_input_padded != 32 || dir->n_output < 1 || dir->n_output > 16 ||
      dir->n_output_padded != 16 || dir->width != pos->width ||
      (dir->n_hidden_layers != 1 && dir->n_hidden_layers != 2))
    return 0;
  if (pos->width != 32 && pos->width != 64) return 0;
  return pos->width * 10 + dir->n_hidden_layers;
}

static int dispatch(int v, int op, const Args& a, hipStream_t st) {
  switch (v) {
    case 321: return run<32, 1>(op, a, st);
    case 322: return run<32, 2>(op, a, st);
    case 641: return run<64, 1>(op, a, st);
    case 642: return run<64, 2>(op, a, st);
  }
  return 1;
}

}  // namespace field
}  // namespace anr

using namespace anr::field;

extern "C" int anr_ingp_field_supported(const anr_mlp_desc* pos, const anr_mlp_desc* dir) {
  return variant(pos, dir) != 0;
}

extern "C" int64_t anr_ingp_field_packed_size(const anr_mlp_desc* pos, const anr_mlp_desc* dir) {
  switch (variant(pos, dir)) {
    case 321: return Net<32, 1>::n_packed;
    case 322: return Net<32, 2>::n_packed;
    case 641: return Net<64, 1>::n_packed;
    case 642: return Net<64, 2>::n_packed;
  }
  return 0;
}

extern "C" int anr_ingp_field_set_grad_scale(int32_t log2_target) {
  const int prev = g_target_log2;
  g_target_log2 = log2_target;
  return prev;
}

extern "C" int anr_ingp_field_pack(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                   const float* pos_params, const float* dir_params,
                                   void* packed, anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_pack: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(pos_params && dir_params && packed, "anr_ingp_field_pack: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  _Float16* out = static_cast<_Float16*>(packed);
  switch (v) {
    case 321: launch_pack<32, 1>(pos_params, dir_params, out, st); break;
    case 322: launch_pack<32, 2>(pos_params, dir_params, out, st); break;
    case 641: launch_pack<64, 1>(pos_params, dir_params, out, st); break;
    case 642: launch_pack<64, 2>(pos_params, dir_params, out, st); break;
  }
  ANR_CHECK_LAUNCH("anr_ingp_field_pack");
  return ANR_OK;
}

extern "C" int anr_ingp_field_fwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                  const void* packed, const void* enc, int64_t enc_stride,
                                  const float* dirs, int64_t n_per_ray, int64_t M, float* sigma,
                                  float* color, int64_t color_stride, anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_fwd: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(M >= 0 && M < (1LL << 31), "anr_ingp_field_fwd: bad M");
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(packed && enc && dirs && sigma && color, "anr_ingp_field_fwd: null pointer");
  ANR_CHECK_ARG(n_per_ray >= 1 && n_per_ray < (1LL << 31) && enc_stride >= 32 &&
                    enc_stride % 8 == 0 && color_stride >= dir->n_output,
                "anr_ingp_field_fwd: bad shape/stride");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0,
                "anr_ingp_field_fwd: enc/packed must be 16-byte aligned");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  a.enc = static_cast<const _Float16*>(enc);
  a.enc_stride = enc_stride;
  a.dirs = dirs;
  a.n_per_ray = static_cast<uint32_t>(n_per_ray);
  a.M = M;
  a.n_out = dir->n_output;
  a.sigma = sigma;
  a.color = color;
  a.color_stride = color_stride;
  ANR_CHECK_ARG(dispatch(v, 1, a, reinterpret_cast<hipStream_t>(stream)) == 0,
                "anr_ingp_field_fwd: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_field_fwd");
  return ANR_OK;
}

extern "C" int anr_ingp_field_bwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                  const void* packed, const void* enc, int64_t enc_stride,
                                  const float* dirs, int64_t n_per_ray, int64_t M,
                                  const float* d_sigma, const float* d_color,
                                  int64_t d_color_stride, float* d_enc, int64_t d_enc_stride,
                                  float* g_pos, float* g_dir, anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_bwd: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(M >= 0 && M < (1LL << 31), "anr_ingp_field_bwd: bad M");
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(packed && enc && dirs && d_color && d_enc && g_pos && g_dir,
                "anr_ingp_field_bwd: null pointer");
  ANR_CHECK_ARG(n_per_ray >= 1 && n_per_ray < (1LL << 31) && enc_stride >= 32 &&
                    enc_stride % 8 == 0 && d_color_stride >= dir->n_output &&
                    d_enc_stride >= 32 && d_enc_stride % 4 == 0,
                "anr_ingp_field_bwd: bad shape/stride");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(d_enc) & 15) == 0,
                "anr_ingp_field_bwd: enc/packed/d_enc must be 16-byte aligned");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  a.enc = static_cast<const _Float16*>(enc);
  a.enc_stride = enc_stride;
  a.dirs = dirs;
  a.n_per_ray = static_cast<uint32_t>(n_per_ray);
  a.M = M;
  a.n_out = dir->n_output;
  a.d_sigma = d_sigma;
  a.d_color = d_color;
  a.d_color_stride = d_color_stride;
  a.d_enc = d_enc;
  a.d_enc_stride = d_enc_stride;
  a.g_pos = g_pos;
  a.g_dir = g_dir;
  ANR_CHECK_ARG(dispatch(v, 2, a, reinterpret_cast<hipStream_t>(stream)) == 0,
                "anr_ingp_field_bwd: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_field_bwd");
  return ANR_OK;
}
