// K6 / K7 (specialised): fully-fused MLP for compile-time shapes.
//
// Same semantics as mlp.hip (tinycudann FullyFusedMLP, bias-free, ReLU hidden, 1.0
// input padding, output padding) for the shapes AtmoNR uses: width 32/64, padded input
// 16/32/48, padded output 16, 1-2 hidden layers (pos_mlp 32->64->16, dir_mlp
// 32->64->64->16, surf_mlp 48->64->64->16 at instant_ngp.py:64-85). Everything is
// unrolled at compile time, which is what makes the backward fast:
//
// * Layers are computed in transposed form, out^T (N x rows) = W (N x K) · act^T: the A
//   operand is a row of W and the B operand a row of the row-major activation tile, and
//   the C tile (4 consecutive output units of one row per lane) is written back to the
//   row-major LDS tile with ONE 8-byte store per lane (f16).
// * dW = gᵀ·act needs both tiles column-wise; gfx950's ds_read_b64_tr_b16 delivers the
//   4x16 block transposed, so the operands come from the same row-major tiles.
// * dW accumulates in registers (f32) across every row tile a wavefront processes and
//   is flushed once per wavefront with coalesced f32 atomics (16 lanes = 64 contiguous
//   bytes). The generic kernel instead did one LDS atomic per dW element per tile.
// * f16 gradients are scaled by one power of two per wavefront (max |dL/dout| over the
//   wave's rows -> 256, found by a pre-pass over dout) and unscaled exactly in f32 when
//   dW is flushed and when dL/din is written.

#include "anr_common.h"

namespace anr {
namespace fused {

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

template <typename TC>
struct Ops;

template <>
struct Ops<_Float16> {
  static constexpr int KS = 16;
  using frag = h4;
  // lane (row l&15) reads 4 consecutive elements at column 4(l>>4)
  __device__ static frag rows(const _Float16* b, int ld, int lane) {
    return *reinterpret_cast<const frag*>(b + (lane & 15) * ld + 4 * (lane >> 4));
  }
  // lane (column l&15) receives rows 4(l>>4) .. +3 of that column (hardware transpose)
  __device__ static frag cols(const _Float16* b, int ld, int lane) {
    const int li = lane & 15;
    const _Float16* addr = b + (4 * (lane >> 4) + (li >> 2)) * ld + 4 * (li & 3);
    // generic -> LDS address-space cast (addr always points into the dynamic LDS)
    const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(addr));
    return __builtin_bit_cast(frag, v);
  }
  __device__ static f4 mma(frag a, frag b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  }
  // C (m = 4(l>>4)+i, n = l&15) stored as dst[n][m]: one 8-byte store
  __device__ static void store_t(_Float16* dst, int ld, f4 c, int lane) {
    h4 v;
    v.x = static_cast<_Float16>(c[0]);
    v.y = static_cast<_Float16>(c[1]);
    v.z = static_cast<_Float16>(c[2]);
    v.w = static_cast<_Float16>(c[3]);
    *reinterpret_cast<h4*>(dst + (lane & 15) * ld + 4 * (lane >> 4)) = v;
  }
  __device__ static f4 load_t(const _Float16* src, int ld, int lane) {
    const h4 v = *reinterpret_cast<const h4*>(src + (lane & 15) * ld + 4 * (lane >> 4));
    return f4{static_cast<float>(v.x), static_cast<float>(v.y), static_cast<float>(v.z),
              static_cast<float>(v.w)};
  }
};

template <>
struct Ops<float> {
  static constexpr int KS = 4;
  using frag = float;
  __device__ static frag rows(const float* b, int ld, int lane) {
    return b[(lane & 15) * ld + (lane >> 4)];
  }
  __device__ static frag cols(const float* b, int ld, int lane) {
    return b[(lane >> 4) * ld + (lane & 15)];
  }
  __device__ static f4 mma(frag a, frag b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static void store_t(float* dst, int ld, f4 c, int lane) {
    *reinterpret_cast<f4*>(dst + (lane & 15) * ld + 4 * (lane >> 4)) = c;
  }
  __device__ static f4 load_t(const float* src, int ld, int lane) {
    return *reinterpret_cast<const f4*>(src + (lane & 15) * ld + 4 * (lane >> 4));
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct Args {
  int n_in, n_out, out_relu;
  int64_t M;
  const void* params;  // compute precision (f16 or f32), tcnn layer order
  const void* in;
  int in_dt;
  int64_t in_stride;
  const void* dout;
  int dout_dt;
  int64_t dout_stride;
  void* out;  // fwd: output ; bwd: din (nullable)
  int out_dt;
  int64_t out_stride;
  float* dparams;
  // MODE 1 (Instant-NGP dir MLP, instant_ngp.py:165-171): the input row is
  // [SH2(dir of its ray) | pos_out[r, 1:16] | 1.0 ...] built on the fly; the backward
  // writes dL/dpos_out (col 0 = dL/dsigma * [pos_out[r,0] > 0], cols 1.. from dIn).
  const float* pos_out;
  int64_t pos_stride;
  const float* dirs;
  int64_t n_per_ray;
  const float* d_sigma;
  // bwd (nullable): one n_params row of f32 per wavefront; each wavefront stores its dW
  // there instead of adding it with atomics, and slab_reduce_kernel sums the rows into
  // dparams (small batches: the atomics would pile onto the same few KB)
  float* slab;
  int64_t slab_floats;
  // > 0 (f16, MODE 0): reference numerics (anr_mlp_bwd_ref16): tcnn's fixed loss scale
  // instead of the per-wavefront one, and dL/dinput written as f16(f16(g_scaled) / scale)
  float loss_scale;
};

// dparams[p] += sum over the nw slab rows of slab[w * n + p]. Block = 64 params x 16 row
// groups: group y sums rows y, y+16, ... and the 16 partials are added in a fixed order
// (deterministic; 16 independent load streams per column instead of one serial walk).
__global__ void __launch_bounds__(1024) slab_reduce_kernel(const float* __restrict__ slab,
                                                           int64_t nw, int64_t n,
                                                           float* __restrict__ dparams) {
  __shared__ float part[16][64];
  const int x = threadIdx.x & 63, y = threadIdx.x >> 6;
  const int64_t p = static_cast<int64_t>(blockIdx.x) * 64 + x;
  float acc = 0.0f;
  if (p < n)
    for (int64_t w = y; w < nw; w += 16) acc += slab[w * n + p];
  part[y][x] = acc;
  __syncthreads();
  if (y == 0 && p < n) {
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += part[j][x];
    dparams[p] += s;
  }
}

// Compile-time network shape.
template <int W, int NIP, int NOP, int NH>
struct Shape {
  static constexpr int NL = NH + 1;
  __host__ __device__ static constexpr int K(int k) { return k == 0 ? NIP : W; }
  __host__ __device__ static constexpr int N(int k) { return k == NL - 1 ? NOP : W; }
  __host__ __device__ static constexpr int woff(int k) {  // element offset in params
    int o = 0;
    for (int j = 0; j < k; ++j) o += K(j) * N(j);
    return o;
  }
  static constexpr int n_params = woff(NL);
  // LDS leading dimensions (+8 halves: keeps 16-byte alignment, staggers banks)
  __host__ __device__ static constexpr int ldw(int k) { return K(k) + 8; }
  __host__ __device__ static constexpr int ldwt(int k) { return N(k) + 8; }
  __host__ __device__ static constexpr int lws(int k) {  // W tile offset in LDS
    int o = 0;
    for (int j = 0; j < k; ++j) o += N(j) * ldw(j);
    return o;
  }
  __host__ __device__ static constexpr int lwts(int k) {
    int o = 0;
    for (int j = 0; j < k; ++j) o += K(j) * ldwt(j);
    return o;
  }
  static constexpr int w_lds = lws(NL);
  static constexpr int wt_lds = lwts(NL);
  static constexpr int lda(int k) { return K(k) + 8; }
  static constexpr int GMAX = W > NOP ? W : NOP;
  static constexpr int ldg = GMAX + 8;
  static constexpr int ldo = NOP + 8;
  // per-wave activation tiles act_0..act_{NL-1} (16 rows each)
  __host__ __device__ static constexpr int acts(int k) {
    int o = 0;
    for (int j = 0; j < k; ++j) o += 16 * lda(j);
    return o;
  }
  static constexpr int act_total = acts(NL);
  static constexpr int wave_fwd = 16 * lda(0) + 2 * 16 * (W + 8);          // elements
  static constexpr int wave_bwd = act_total + 16 * ldo + 2 * 16 * ldg;      // elements
  __host__ __device__ static constexpr int tiles(int k) { return (N(k) / 16) * (K(k) / 16); }
  __host__ __device__ static constexpr int tile_off(int k) {
    int o = 0;
    for (int j = 0; j < k; ++j) o += tiles(j);
    return o;
  }
  static constexpr int n_tiles = tile_off(NL);
};

template <typename TC, typename S>
__device__ void stage_weights(const Args& a, TC* w, TC* wt) {
  const TC* p = static_cast<const TC*>(a.params);
#pragma unroll
  for (int k = 0; k < S::NL; ++k) {
    constexpr int dummy = 0;
    (void)dummy;
    const int K = S::K(k), N = S::N(k);
    for (int e = threadIdx.x; e < K * N; e += blockDim.x) {
      const int n = e / K, kk = e - n * K;
      const TC v = p[S::woff(k) + e];
      w[S::lws(k) + n * S::ldw(k) + kk] = v;
      if (wt) wt[S::lwts(k) + kk * S::ldwt(k) + n] = v;
    }
  }
}

// SH degree 2 of a direction remapped from [0,1] coordinates (tcnn convention: the raw
// direction is fed as if in [0,1], i.e. 2d-1; instant_ngp.py:165-169).
__device__ __forceinline__ float sh2(int c, float x, float y, float z) {
  x = x * 2.0f - 1.0f;
  y = y * 2.0f - 1.0f;
  z = z * 2.0f - 1.0f;
  return c == 0 ? 0.28209479177387814f
                : (c == 1 ? -0.48860251190291987f * y
                          : (c == 2 ? 0.48860251190291987f * z : -0.48860251190291987f * x));
}

// Load a 16-row input tile into act0 (ld = lda(0)); pad columns with 1.0.
template <typename TC, typename S, int MODE>
__device__ void load_input(const Args& a, int64_t r0, TC* act0, int lane) {
  constexpr int NIP = S::K(0);
  constexpr int ld = S::lda(0);
  if constexpr (MODE == 1) {
    // [SH2(dir) (4) | pos_out[:, 1:16] (15) | 1.0 (13)], NIP == 32: lane = (row, 8-column
    // part); one 32-bit division per row, pos_out read as float4s.
    static_assert(NIP == 32, "dir mode expects 19 inputs padded to 32");
    const int r = lane & 15, part = lane >> 4;
    const int64_t row = r0 + r;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.0f;
    if (row < a.M) {
      const float* po = a.pos_out + row * a.pos_stride;
      if (part == 0) {
        const uint32_t ray = static_cast<uint32_t>(row) / static_cast<uint32_t>(a.n_per_ray);
        const float* d = a.dirs + static_cast<int64_t>(ray) * 3;
        const float x = d[0] * 2.0f - 1.0f, y = d[1] * 2.0f - 1.0f, z = d[2] * 2.0f - 1.0f;
        v[0] = 0.28209479177387814f;
        v[1] = -0.48860251190291987f * y;
        v[2] = 0.48860251190291987f * z;
        v[3] = -0.48860251190291987f * x;
        const float4 p1 = *reinterpret_cast<const float4*>(po);      // cols 0..3
        const float4 p2 = *reinterpret_cast<const float4*>(po + 4);  // cols 4..7
        v[4] = p1.y; v[5] = p1.z; v[6] = p1.w; v[7] = p2.x;
      } else if (part == 1) {
        const float4 p2 = *reinterpret_cast<const float4*>(po + 4);
        const float4 p3 = *reinterpret_cast<const float4*>(po + 8);
        const float4 p4 = *reinterpret_cast<const float4*>(po + 12);
        v[0] = p2.y; v[1] = p2.z; v[2] = p2.w; v[3] = p3.x;
        v[4] = p3.y; v[5] = p3.z; v[6] = p3.w; v[7] = p4.x;
      } else if (part == 2) {
        const float4 p4 = *reinterpret_cast<const float4*>(po + 12);
        v[0] = p4.y; v[1] = p4.z; v[2] = p4.w;
#pragma unroll
        for (int i = 3; i < 8; ++i) v[i] = 1.0f;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 1.0f;
      }
    }
    TC* dst = act0 + r * ld + part * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i] = static_cast<TC>(v[i]);
    return;
  }
  if constexpr (sizeof(TC) == 2) {
    if (a.in_dt == ANR_F16 && a.n_in == NIP && (a.in_stride % 8) == 0) {
      // 16 rows x NIP halves, 16 bytes per lane per chunk
      constexpr int chunks = 16 * NIP / 8;
      const __half* in = static_cast<const __half*>(a.in);
#pragma unroll
      for (int c = lane; c < chunks; c += 64) {
        const int r = c / (NIP / 8), cc = (c - r * (NIP / 8)) * 8;
        const int64_t row = r0 + r;
        h8 v = {};
        if (row < a.M) v = *reinterpret_cast<const h8*>(in + row * a.in_stride + cc);
        *reinterpret_cast<h8*>(act0 + r * ld + cc) = v;
      }
      return;
    }
  }
  for (int e = lane; e < 16 * NIP; e += 64) {
    const int r = e / NIP, c = e - r * NIP;
    const int64_t row = r0 + r;
    float v = 0.0f;
    if (row < a.M) v = c < a.n_in ? load_dyn(a.in, a.in_dt, row * a.in_stride + c) : 1.0f;
    act0[r * ld + c] = static_cast<TC>(v);
  }
}

// One hidden layer in transposed form: dst (16 x N, row-major) = relu(src · Wᵀ).
template <typename TC, typename S, int k>
__device__ __forceinline__ void hidden_layer(const TC* w, const TC* src, TC* dst, int ldd,
                                             int lane) {
  using O = Ops<TC>;
  constexpr int K = S::K(k), N = S::N(k);
#pragma unroll
  for (int nt = 0; nt < N / 16; ++nt) {
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ks = 0; ks < K; ks += O::KS)
      acc = O::mma(O::rows(w + S::lws(k) + nt * 16 * S::ldw(k) + ks, S::ldw(k), lane),
                   O::rows(src + ks, S::lda(k), lane), acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = fmaxf(acc[i], 0.0f);
    O::store_t(dst + nt * 16, ldd, acc, lane);
  }
}

template <typename TC, int W, int NIP, int NOP, int NH, int MODE>
__global__ void __launch_bounds__(256) fwd_kernel(Args a) {
  using S = Shape<W, NIP, NOP, NH>;
  using O = Ops<TC>;
  constexpr int NL = S::NL;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  TC* w = reinterpret_cast<TC*>(smem);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int waves = blockDim.x >> 6;
  TC* act0 = w + S::w_lds + wave * S::wave_fwd;
  TC* hA = act0 + 16 * S::lda(0);
  TC* hB = hA + 16 * (W + 8);
  stage_weights<TC, S>(a, w, nullptr);
  __syncthreads();
  const int64_t n_tiles = (a.M + 15) / 16;
  for (int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave; tile < n_tiles;
       tile += static_cast<int64_t>(gridDim.x) * waves) {
    const int64_t r0 = tile * 16;
    load_input<TC, S, MODE>(a, r0, act0, lane);
    wave_sync();
    hidden_layer<TC, S, 0>(w, act0, hA, W + 8, lane);
    wave_sync();
    const TC* last_in = hA;
    if constexpr (NH >= 2) {
      hidden_layer<TC, S, 1>(w, hA, hB, W + 8, lane);
      wave_sync();
      last_in = hB;
    }
    if constexpr (NH >= 3) {
      hidden_layer<TC, S, 2>(w, hB, hA, W + 8, lane);
      wave_sync();
      last_in = hA;
    }
    // output layer straight from the accumulators: lane holds out[r0 + (l&15)][n0 + 4(l>>4) + i]
    constexpr int k = NL - 1;
#pragma unroll
    for (int nt = 0; nt < NOP / 16; ++nt) {
      if (nt * 16 >= a.n_out) break;
      f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < W; ks += O::KS)
        acc = O::mma(O::rows(w + S::lws(k) + nt * 16 * S::ldw(k) + ks, S::ldw(k), lane),
                     O::rows(last_in + ks, W + 8, lane), acc);
      const int64_t row = r0 + (lane & 15);
      const int c0 = nt * 16 + 4 * (lane >> 4);
      if (row < a.M) {
        if (a.out_dt == ANR_F32 && c0 + 3 < a.n_out && (a.out_stride % 4) == 0) {
          f4 v = acc;
          if (a.out_relu)
            for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.0f);
          *reinterpret_cast<f4*>(static_cast<float*>(a.out) + row * a.out_stride + c0) = v;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = acc[i];
            if (a.out_relu) v = fmaxf(v, 0.0f);
            if (c0 + i < a.n_out) store_dyn(a.out, a.out_dt, row * a.out_stride + c0 + i, v);
          }
        }
      }
    }
    wave_sync();
  }
}

template <typename TC, int W, int NIP, int NOP, int NH, int MODE>
__global__ void __launch_bounds__(256) bwd_kernel(Args a) {
  using S = Shape<W, NIP, NOP, NH>;
  using O = Ops<TC>;
  constexpr int NL = S::NL;
  constexpr bool half = sizeof(TC) == 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  TC* w = reinterpret_cast<TC*>(smem);
  TC* wt = w + S::w_lds;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int waves = blockDim.x >> 6;
  TC* base = wt + S::wt_lds + wave * S::wave_bwd;
  TC* outb = base + S::act_total;
  TC* g0 = outb + 16 * S::ldo;
  TC* g1 = g0 + 16 * S::ldg;
  stage_weights<TC, S>(a, w, wt);
  __syncthreads();

  f4 dw[S::n_tiles];
#pragma unroll
  for (int t = 0; t < S::n_tiles; ++t) dw[t] = f4{0.0f, 0.0f, 0.0f, 0.0f};

  const int64_t n_tiles = (a.M + 15) / 16;
  // f16: one power-of-two gradient scale per wavefront (max |dL/dout| over all its rows
  // -> 256), so dW accumulates directly in the MFMA accumulators and is unscaled once.
  float s = 1.0f, inv_s = 1.0f;
  const bool ref = half && a.loss_scale > 0.0f;
  if (ref) {
    s = a.loss_scale;
    inv_s = 1.0f / a.loss_scale;
  } else if constexpr (half) {
    float gmax = 0.0f;
    for (int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave; tile < n_tiles;
         tile += static_cast<int64_t>(gridDim.x) * waves) {
      for (int e = lane; e < 16 * a.n_out; e += 64) {
        const int r = e / a.n_out, c = e - r * a.n_out;
        const int64_t row = tile * 16 + r;
        if (row < a.M) gmax = fmaxf(gmax, fabsf(load_dyn(a.dout, a.dout_dt, row * a.dout_stride + c)));
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) gmax = fmaxf(gmax, shfl_xor(gmax, m));
    if (gmax > 0.0f) {
      int e2 = static_cast<int>(floorf(log2f(256.0f / gmax)));
      e2 = e2 < -60 ? -60 : (e2 > 100 ? 100 : e2);
      s = ldexpf(1.0f, e2);
      inv_s = ldexpf(1.0f, -e2);
    }
  }
  TC* const w_base = w;
  TC* const wt_base = wt;
  for (int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave; tile < n_tiles;
       tile += static_cast<int64_t>(gridDim.x) * waves) {
    const int64_t r0 = tile * 16;
    // Re-read weight fragments from LDS every tile instead of letting the compiler hoist
    // them into ~110 VGPRs: with the register-resident dW that would cap the kernel at one
    // wavefront per SIMD. An opaque zero offset keeps the LDS base (ds_read addressing).
    int zoff = 0;
    asm volatile("" : "+v"(zoff));
    w = w_base + zoff;
    wt = wt_base + zoff;
    // ---- recompute the forward, keeping each layer's input tile
    load_input<TC, S, MODE>(a, r0, base + S::acts(0), lane);
    wave_sync();
    hidden_layer<TC, S, 0>(w, base + S::acts(0), base + S::acts(1), S::lda(1), lane);
    wave_sync();
    if constexpr (NH >= 2) {
      hidden_layer<TC, S, 1>(w, base + S::acts(1), base + S::acts(2), S::lda(2), lane);
      wave_sync();
    }
    if constexpr (NH >= 3) {
      hidden_layer<TC, S, 2>(w, base + S::acts(2), base + S::acts(3), S::lda(3), lane);
      wave_sync();
    }
    if (a.out_relu) {  // activated output, needed only for the output-ReLU mask
      constexpr int k = NL - 1;
#pragma unroll
      for (int nt = 0; nt < NOP / 16; ++nt) {
        f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < W; ks += O::KS)
          acc = O::mma(O::rows(w + S::lws(k) + nt * 16 * S::ldw(k) + ks, S::ldw(k), lane),
                       O::rows(base + S::acts(k) + ks, S::lda(k), lane), acc);
        O::store_t(outb + nt * 16, S::ldo, acc, lane);
      }
      wave_sync();
    }
    // ---- output gradient tile g = dL/d(pre-activation output), scaled for f16
    float gv[NOP / 4];
    {
      const int r = lane & 15;
      const int64_t row = r0 + r;
#pragma unroll
      for (int j = 0; j < NOP / 4; ++j) {
        // lane covers columns 4*(lane>>4) + 16*(j/4) + (j%4) of row r
        const int c = 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
        float v = 0.0f;
        if (row < a.M && c < a.n_out) v = load_dyn(a.dout, a.dout_dt, row * a.dout_stride + c);
        if (a.out_relu && !(static_cast<float>(outb[r * S::ldo + c]) > 0.0f)) v = 0.0f;
        gv[j] = v;
      }
    }
#pragma unroll
    for (int q = 0; q < NOP / 16; ++q) {
      f4 v = {gv[4 * q] * s, gv[4 * q + 1] * s, gv[4 * q + 2] * s, gv[4 * q + 3] * s};
      O::store_t(g0 + 16 * q, S::ldg, v, lane);
    }
    wave_sync();
    // ---- backward through the layers (unrolled)
    TC* g = g0;
    TC* gn = g1;
#pragma unroll
    for (int k = NL - 1; k >= 0; --k) {
      const int K = S::K(k), N = S::N(k);
      const TC* act = base + S::acts(k);
      const int lda = S::lda(k);
      // dW_k (N x K) += gᵀ · act over the 16 rows
#pragma unroll
      for (int mt = 0; mt < N / 16; ++mt) {
#pragma unroll
        for (int nt = 0; nt < K / 16; ++nt) {
          f4& d = dw[S::tile_off(k) + mt * (K / 16) + nt];
#pragma unroll
          for (int ks = 0; ks < 16; ks += O::KS)
            d = O::mma(O::cols(g + ks * S::ldg + mt * 16, S::ldg, lane),
                       O::cols(act + ks * lda + nt * 16, lda, lane), d);
        }
      }
      // dAct_k^T (K x 16) = W_kᵀ · gᵀ
      if (k > 0 || a.out != nullptr) {
#pragma unroll
        for (int nt = 0; nt < K / 16; ++nt) {
          f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < N; ks += O::KS)
            acc = O::mma(O::rows(wt + S::lwts(k) + nt * 16 * S::ldwt(k) + ks, S::ldwt(k), lane),
                         O::rows(g + ks, S::ldg, lane), acc);
          if (k > 0) {
            const f4 av = O::load_t(act + nt * 16, lda, lane);  // relu mask from act_k
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = av[i] > 0.0f ? acc[i] : 0.0f;
            O::store_t(gn + nt * 16, S::ldg, acc, lane);
          } else if constexpr (MODE == 1) {
            // dIn columns 4..18 are dL/dpos_out[:, 1..15]; column 0 of dL/dpos_out is
            // dL/dsigma through the density ReLU (instant_ngp.py:178,184).
            const int64_t row = r0 + (lane & 15);
            const int c0 = nt * 16 + 4 * (lane >> 4);
            if (row < a.M) {
              float* dp = static_cast<float*>(a.out) + row * a.out_stride;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int c = c0 + i;
                if (c >= 4 && c < 19) dp[c - 3] = acc[i] * inv_s;
              }
              if (c0 == 0) {
                const float ds = a.d_sigma ? a.d_sigma[row] : 0.0f;
                dp[0] = a.pos_out[row * a.pos_stride] > 0.0f ? ds : 0.0f;
              }
            }
          } else {
            const int64_t row = r0 + (lane & 15);
            const int c0 = nt * 16 + 4 * (lane >> 4);
            if (row < a.M) {
              if (ref) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  acc[i] = static_cast<float>(static_cast<_Float16>(acc[i]));
              }
              if (a.out_dt == ANR_F32 && c0 + 3 < a.n_in && (a.out_stride % 4) == 0) {
                f4 v = {acc[0] * inv_s, acc[1] * inv_s, acc[2] * inv_s, acc[3] * inv_s};
                if (ref) {
#pragma unroll
                  for (int i = 0; i < 4; ++i) v[i] = static_cast<float>(static_cast<_Float16>(v[i]));
                }
                *reinterpret_cast<f4*>(static_cast<float*>(a.out) + row * a.out_stride + c0) = v;
              } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  if (c0 + i < a.n_in)
                    store_dyn(a.out, a.out_dt, row * a.out_stride + c0 + i,
                              ref ? static_cast<float>(static_cast<_Float16>(acc[i] * inv_s))
                                  : acc[i] * inv_s);
              }
            }
          }
        }
      }
      wave_sync();
      TC* tmp = g; g = gn; gn = tmp;
    }
  }
  // ---- flush this wavefront's dW: lane holds dW[mt*16 + 4(l>>4) + i][nt*16 + (l&15)]
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int K = S::K(k), N = S::N(k);
#pragma unroll
    for (int mt = 0; mt < N / 16; ++mt)
#pragma unroll
      for (int nt = 0; nt < K / 16; ++nt) {
        const f4 d = dw[S::tile_off(k) + mt * (K / 16) + nt];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = mt * 16 + 4 * (lane >> 4) + i, col = nt * 16 + (lane & 15);
          if (a.slab) {
            const int64_t w_id = static_cast<int64_t>(blockIdx.x) * waves + wave;
            a.slab[w_id * S::n_params + S::woff(k) + row * K + col] = d[i] * inv_s;
          } else if (d[i] != 0.0f) {
            atomicAdd(a.dparams + S::woff(k) + row * K + col, d[i] * inv_s);
          }
        }
      }
  }
}

template <typename TC, int W, int NIP, int NOP, int NH, int MODE>
static int launch(bool bwd, const Args& a, hipStream_t st) {
  using S = Shape<W, NIP, NOP, NH>;
  const size_t es = sizeof(TC);
  const int waves = 4;
  size_t lds;
  const void* fn;
  if (bwd) {
    lds = (static_cast<size_t>(S::w_lds) + S::wt_lds + waves * S::wave_bwd) * es;
    fn = reinterpret_cast<const void*>(&bwd_kernel<TC, W, NIP, NOP, NH, MODE>);
  } else {
    lds = (static_cast<size_t>(S::w_lds) + waves * S::wave_fwd) * es;
    fn = reinterpret_cast<const void*>(&fwd_kernel<TC, W, NIP, NOP, NH, MODE>);
  }
  if (lds > 160 * 1024) return 1;  // does not fit: caller falls back to the generic kernel
  const int64_t tiles = (a.M + 15) / 16;
  int64_t blocks = (tiles + waves - 1) / waves;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  // bwd: one resident wave per slot, each folding many tiles into its register dW (so
  // the flush atomics stay few); size the grid to what is co-resident (once per kernel)
  static int per_cu[2] = {0, 0};
  int& pc = per_cu[bwd ? 1 : 0];
  if (pc == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * waves, lds) != hipSuccess || nb < 1)
      nb = 1;
    pc = nb;
  }
  const int64_t cap = bwd ? 256LL * pc : 2048;
  if (blocks > cap) blocks = cap;
  if (bwd) {
    // Minimum tiles per wave (profiling override ANR_MLP_BWD_MIN_TILES). On the per-ray
    // surface network (8192 rows) 8 tiles per wave (64 waves, 64 flush adds per weight
    // instead of 512) measured 0.104 ms against 0.057 ms with one tile per wave: the
    // serial tile walk costs more than the contended flush saves, so the default is 1.
    static const int64_t min_tiles = [] {
      const char* e = getenv("ANR_MLP_BWD_MIN_TILES");
      const long long v = e ? atoll(e) : 0;
      return v > 0 ? static_cast<int64_t>(v) : static_cast<int64_t>(1);
    }();
    const int64_t by_tiles = (tiles + waves * min_tiles - 1) / (waves * min_tiles);
    if (blocks > by_tiles) blocks = by_tiles > 0 ? by_tiles : 1;
  }
  if (bwd) {
    Args b = a;
    if (a.slab && blocks * waves * static_cast<int64_t>(S::n_params) > a.slab_floats)
      b.slab = nullptr;  // workspace too small for this grid: atomics
    hipLaunchKernelGGL((bwd_kernel<TC, W, NIP, NOP, NH, MODE>), dim3(blocks), dim3(64 * waves),
                       lds, st, b);
    if (b.slab)
      hipLaunchKernelGGL(slab_reduce_kernel, dim3(static_cast<unsigned>((S::n_params + 63) / 64)),
                         dim3(1024), 0, st, b.slab, blocks * waves,
                         static_cast<int64_t>(S::n_params), a.dparams);
  }
  else
    hipLaunchKernelGGL((fwd_kernel<TC, W, NIP, NOP, NH, MODE>), dim3(blocks), dim3(64 * waves),
                       lds, st, a);
  return 0;
}

template <typename TC>
static int dispatch_tc(const anr_mlp_desc* d, bool bwd, const Args& a, hipStream_t st) {
  if (d->n_output_padded != 16) return 1;
  const int key = d->width * 10000 + d->n_input_padded * 10 + d->n_hidden_layers;
  switch (key) {
#define ANR_CASE(W, NIP, NH) \
  case W * 10000 + NIP * 10 + NH: return launch<TC, W, NIP, 16, NH, 0>(bwd, a, st);
    ANR_CASE(32, 16, 1) ANR_CASE(32, 32, 1) ANR_CASE(32, 48, 1)
    ANR_CASE(32, 16, 2) ANR_CASE(32, 32, 2) ANR_CASE(32, 48, 2)
    ANR_CASE(64, 16, 1) ANR_CASE(64, 32, 1) ANR_CASE(64, 48, 1)
    ANR_CASE(64, 16, 2) ANR_CASE(64, 32, 2) ANR_CASE(64, 48, 2)
#undef ANR_CASE
    default: return 1;
  }
}

template <typename TC>
static int dispatch_dir(const anr_mlp_desc* d, bool bwd, const Args& a, hipStream_t st) {
  if (d->n_output_padded != 16 || d->n_input != 19 || d->n_input_padded != 32) return 1;
  if (d->width == 64 && d->n_hidden_layers == 2) return launch<TC, 64, 32, 16, 2, 1>(bwd, a, st);
  if (d->width == 32 && d->n_hidden_layers == 2) return launch<TC, 32, 32, 16, 2, 1>(bwd, a, st);
  if (d->width == 64 && d->n_hidden_layers == 1) return launch<TC, 64, 32, 16, 1, 1>(bwd, a, st);
  if (d->width == 32 && d->n_hidden_layers == 1) return launch<TC, 32, 32, 16, 1, 1>(bwd, a, st);
  return 1;
}

}  // namespace fused

// True if dispatch_tc has a specialised kernel for this shape (the plain MLP entry points).
bool mlp_fused_has(const anr_mlp_desc* d) {
  return d->n_output_padded == 16 && (d->width == 32 || d->width == 64) &&
         (d->n_hidden_layers == 1 || d->n_hidden_layers == 2) &&
         (d->n_input_padded == 16 || d->n_input_padded == 32 || d->n_input_padded == 48);
}

// Returns 0 if a specialised kernel was launched, 1 if the caller must use the generic
// kernel. The weights must already be in compute precision.
int mlp_fused_try(const anr_mlp_desc* d, int32_t precision, bool bwd, const void* params,
                  const void* in, int32_t in_dt, int64_t in_stride, int64_t M,
                  const void* dout, int32_t dout_dt, int64_t dout_stride, void* out,
                  int32_t out_dt, int64_t out_stride, float* dparams, hipStream_t st,
                  float* slab, int64_t slab_floats, float loss_scale) {
  fused::Args a{};
  a.loss_scale = loss_scale;
  a.slab = slab;
  a.slab_floats = slab_floats;
  a.n_in = d->n_input;
  a.n_out = d->n_output;
  a.out_relu = d->output_activation == ANR_ACT_RELU;
  a.M = M;
  a.params = params;
  a.in = in;
  a.in_dt = in_dt;
  a.in_stride = in_stride;
  a.dout = dout;
  a.dout_dt = dout_dt;
  a.dout_stride = dout_stride;
  a.out = out;
  a.out_dt = out_dt;
  a.out_stride = out_stride;
  a.dparams = dparams;
  if (precision == ANR_F16) return fused::dispatch_tc<_Float16>(d, bwd, a, st);
  return fused::dispatch_tc<float>(d, bwd, a, st);
}

}  // namespace anr

// ---------------------------------------------------------------------------------------
// Instant-NGP dir MLP with the dir encoding fused into its input (instant_ngp.py:165-171).
extern "C" int anr_ingp_dir_mlp_fwd(const anr_mlp_desc* d, int32_t precision,
                                    const void* params, const float* pos_out,
                                    int64_t pos_stride, const float* dirs, int64_t n_per_ray,
                                    int64_t M, void* color, int32_t out_dtype,
                                    int64_t out_stride, anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && params && pos_out && dirs && color, "anr_ingp_dir_mlp_fwd: null argument");
  ANR_CHECK_ARG(precision == ANR_F16 || precision == ANR_F32, "anr_ingp_dir_mlp_fwd: precision");
  ANR_CHECK_ARG(n_per_ray >= 1 && pos_stride >= 16 && pos_stride % 4 == 0 &&
                    out_stride >= d->n_output && M < (1LL << 31),
                "anr_ingp_dir_mlp_fwd: bad shape/stride");
  fused::Args a{};
  a.n_in = d->n_input;
  a.n_out = d->n_output;
  a.out_relu = d->output_activation == ANR_ACT_RELU;
  a.M = M;
  a.params = params;
  a.out = color;
  a.out_dt = out_dtype;
  a.out_stride = out_stride;
  a.pos_out = pos_out;
  a.pos_stride = pos_stride;
  a.dirs = dirs;
  a.n_per_ray = n_per_ray;
  const int rc = precision == ANR_F16 ? fused::dispatch_dir<_Float16>(d, false, a, as_stream(stream))
                                      : fused::dispatch_dir<float>(d, false, a, as_stream(stream));
  if (rc != 0) {
    set_error("anr_ingp_dir_mlp_fwd: unsupported network shape (width %d, hidden %d, in %d)",
              d->width, d->n_hidden_layers, d->n_input);
    return ANR_E_UNSUPPORTED;
  }
  ANR_CHECK_LAUNCH("anr_ingp_dir_mlp_fwd");
  return ANR_OK;
}

extern "C" int anr_ingp_dir_mlp_bwd(const anr_mlp_desc* d, int32_t precision,
                                    const void* params, const float* pos_out,
                                    int64_t pos_stride, const float* dirs, int64_t n_per_ray,
                                    int64_t M, const float* d_color, int64_t d_color_stride,
                                    const float* d_sigma, float* d_pos_out,
                                    int64_t d_pos_stride, float* dparams,
                                    anr_stream_t stream) {
  using namespace anr;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(d && params && pos_out && dirs && d_color && d_pos_out && dparams,
                "anr_ingp_dir_mlp_bwd: null argument");
  ANR_CHECK_ARG(precision == ANR_F16 || precision == ANR_F32, "anr_ingp_dir_mlp_bwd: precision");
  ANR_CHECK_ARG(n_per_ray >= 1 && pos_stride >= 16 && pos_stride % 4 == 0 &&
                    d_pos_stride >= 16 && d_color_stride >= d->n_output && M < (1LL << 31),
                "anr_ingp_dir_mlp_bwd: bad shape/stride");
  fused::Args a{};
  a.n_in = d->n_input;
  a.n_out = d->n_output;
  a.out_relu = d->output_activation == ANR_ACT_RELU;
  a.M = M;
  a.params = params;
  a.dout = d_color;
  a.dout_dt = ANR_F32;
  a.dout_stride = d_color_stride;
  a.out = d_pos_out;
  a.out_dt = ANR_F32;
  a.out_stride = d_pos_stride;
  a.dparams = dparams;
  a.pos_out = pos_out;
  a.pos_stride = pos_stride;
  a.dirs = dirs;
  a.n_per_ray = n_per_ray;
  a.d_sigma = d_sigma;
  const int rc = precision == ANR_F16 ? fused::dispatch_dir<_Float16>(d, true, a, as_stream(stream))
                                      : fused::dispatch_dir<float>(d, true, a, as_stream(stream));
  if (rc != 0) {
    set_error("anr_ingp_dir_mlp_bwd: unsupported network shape (width %d, hidden %d, in %d)",
              d->width, d->n_hidden_layers, d->n_input);
    return ANR_E_UNSUPPORTED;
  }
  ANR_CHECK_LAUNCH("anr_ingp_dir_mlp_bwd");
  return ANR_OK;
}
