// K6 / K7: fully-fused tiny MLP, forward and backward, on MFMA.
//
// Replaces tinycudann.Network(n_in, n_out, {"otype": "FullyFusedMLP", ...}) at
// src/atmonr/pipelines/instant_ngp.py:64-68 (pos_mlp, called :164/:237), :73-77 (dir_mlp,
// :170) and :81-85 (surf_mlp, :174). tcnn semantics (unpinned): bias-free
// linear layers, ReLU hidden activations, input padded to a multiple of 16 with 1.0,
// output padded to a multiple of 16 and sliced.
//
// Design: each wavefront owns 16-row tiles (grid-stride). All layer weights of the
// network are staged once per workgroup in LDS (compute precision). A tile's
// activations never leave LDS: layer k reads its input tile as MFMA A fragments and the
// weights as B fragments (v_mfma_f32_16x16x16_f16 with f32 accumulation, or the exact
// f32 v_mfma_f32_16x16x4_f32), applies ReLU on the accumulators and writes the next
// tile. The backward recomputes the forward of its tile on chip (no activation
// round-trip through HBM), then walks the layers backwards: dIn = g·W and
// dW += gᵀ·act, with dW summed per workgroup in LDS (ds_add_f32) and flushed to the
// global f32 gradient once per workgroup. In f16 precision the tile's output gradient
// is rescaled by a per-tile power of two before rounding to f16 (dynamic loss scaling
// per tile), and every product is unscaled exactly in f32.

#include "anr_common.h"

#include <algorithm>
#include <cstdlib>

namespace anr {

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename TC>
struct MF;

template <>
struct MF<_Float16> {
  static constexpr int KS = 16;  // k per MFMA
  using frag = h4;
  // A[m][k] from a row-major [m][ld] matrix: lane holds row (l&15), k = 4(l>>4)+j.
  __device__ static frag ld_rows(const _Float16* base, int ld, int lane) {
    // ld and the tile base are multiples of 4 halves: one 8-byte LDS read.
    return *reinterpret_cast<const frag*>(base + (lane & 15) * ld + 4 * (lane >> 4));
  }
  // Fragment whose k index runs down the rows of a row-major [k][ld] matrix:
  // lane holds column (l&15), k = 4(l>>4)+j.
  __device__ static frag ld_cols(const _Float16* base, int ld, int lane) {
    const _Float16* p = base + (4 * (lane >> 4)) * ld + (lane & 15);
    frag f;
    f.x = p[0]; f.y = p[ld]; f.z = p[2 * ld]; f.w = p[3 * ld];
    return f;
  }
  __device__ static f4 mma(frag a, frag b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  }
};

template <>
struct MF<float> {
  static constexpr int KS = 4;
  using frag = float;
  __device__ static frag ld_rows(const float* base, int ld, int lane) {
    return base[(lane & 15) * ld + (lane >> 4)];
  }
  __device__ static frag ld_cols(const float* base, int ld, int lane) {
    return base[(lane >> 4) * ld + (lane & 15)];
  }
  __device__ static f4 mma(frag a, frag b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// Make LDS writes of this wave visible to its other lanes (no cross-wave sync).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct MlpArgs {
  int nip, n_in, nop, n_out, width, nl;  // nl = n_hidden_layers + 1
  int out_relu;
  int64_t M;
  const void* params;  // f32 (precision f32) or f16 (precision f16)
  const void* in;
  int in_dt;
  int64_t in_stride;
  const void* dout;
  int dout_dt;
  int64_t dout_stride;
  void* out;  // forward: out ; backward: din
  int out_dt;
  int64_t out_stride;
  float* dparams;
  int waves;
  int64_t n_params;
  int dw_in_lds;
};

__device__ __forceinline__ int layer_in(const MlpArgs& a, int k) { return k == 0 ? a.nip : a.width; }
__device__ __forceinline__ int layer_out(const MlpArgs& a, int k) {
  return k == a.nl - 1 ? a.nop : a.width;
}

// Stage all weights into LDS in compute precision.
template <typename TC>
__device__ void stage_weights(const MlpArgs& a, TC* w) {
  for (int64_t i = threadIdx.x; i < a.n_params; i += blockDim.x) {
    const float v = sizeof(TC) == 2 ? __half2float(static_cast<const __half*>(a.params)[i])
                                    : static_cast<const float*>(a.params)[i];
    w[i] = static_cast<TC>(v);
  }
}

// Load a 16-row input tile (cols >= n_in read as 1.0, rows >= M as 0).
template <typename TC>
__device__ void load_input_tile(const MlpArgs& a, int64_t r0, TC* dst, int ld, int lane) {
  const int n = 16 * a.nip;
  for (int e = lane; e < n; e += kWave) {
    const int r = e / a.nip, c = e - r * a.nip;
    const int64_t row = r0 + r;
    float v = 0.0f;
    if (row < a.M) v = c < a.n_in ? load_dyn(a.in, a.in_dt, row * a.in_stride + c) : 1.0f;
    dst[r * ld + c] = static_cast<TC>(v);
  }
}

// One dense layer on a 16-row tile: dst = act(src · Wᵀ); returns nothing, writes LDS or,
// for the last layer, optionally global output.
template <typename TC>
__device__ void layer_fwd(const TC* src, int lds, const TC* W, int K, int N, TC* dst, int ldd,
                          bool relu, int lane) {
  using F = MF<TC>;
  for (int nt = 0; nt < N / 16; ++nt) {
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int ks = 0; ks < K; ks += F::KS) {
      const typename F::frag av = F::ld_rows(src + ks, lds, lane);
      const typename F::frag bv = F::ld_rows(W + static_cast<int64_t>(nt) * 16 * K + ks, K, lane);
      acc = F::mma(av, bv, acc);
    }
    const int col = nt * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * (lane >> 4) + i;
      float v = acc[i];
      if (relu) v = fmaxf(v, 0.0f);
      dst[row * ldd + col] = static_cast<TC>(v);
    }
  }
}

template <typename TC>
__global__ void __launch_bounds__(256) mlp_fwd_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  TC* w = reinterpret_cast<TC*>(smem);
  const int64_t wP = (a.n_params + 7) / 8 * 8;
  const int ldmax = (a.nip > a.width ? a.nip : a.width) > a.nop
                        ? (a.nip > a.width ? a.nip : a.width)
                        : a.nop;
  const int ld = ldmax + 4;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  TC* buf0 = w + wP + static_cast<int64_t>(wave) * 2 * 16 * ld;
  TC* buf1 = buf0 + 16 * ld;
  stage_weights<TC>(a, w);
  __syncthreads();

  const int64_t n_tiles = (a.M + 15) / 16;
  for (int64_t tile = static_cast<int64_t>(blockIdx.x) * a.waves + wave; tile < n_tiles;
       tile += static_cast<int64_t>(gridDim.x) * a.waves) {
    const int64_t r0 = tile * 16;
    load_input_tile<TC>(a, r0, buf0, ld, lane);
    wave_sync();
    TC* src = buf0;
    TC* dst = buf1;
    int64_t woff = 0;
    for (int k = 0; k < a.nl - 1; ++k) {
      const int K = layer_in(a, k), N = layer_out(a, k);
      layer_fwd<TC>(src, ld, w + woff, K, N, dst, ld, true, lane);
      wave_sync();
      woff += static_cast<int64_t>(K) * N;
      TC* t = src; src = dst; dst = t;
    }
    // last layer: straight from the f32 accumulators to global (real columns only)
    {
      using F = MF<TC>;
      const int K = layer_in(a, a.nl - 1);
      const TC* W = w + woff;
      for (int nt = 0; nt < a.nop / 16; ++nt) {
        if (nt * 16 >= a.n_out) break;
        f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int ks = 0; ks < K; ks += F::KS) {
          const typename F::frag av = F::ld_rows(src + ks, ld, lane);
          const typename F::frag bv =
              F::ld_rows(W + static_cast<int64_t>(nt) * 16 * K + ks, K, lane);
          acc = F::mma(av, bv, acc);
        }
        const int col = nt * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = r0 + 4 * (lane >> 4) + i;
          float v = acc[i];
          if (a.out_relu) v = fmaxf(v, 0.0f);
          if (row < a.M && col < a.n_out) store_dyn(a.out, a.out_dt, row * a.out_stride + col, v);
        }
      }
    }
    wave_sync();
  }
}

template <typename TC>
__global__ void __launch_bounds__(256) mlp_bwd_kernel(MlpArgs a) {
  using F = MF<TC>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  TC* w = reinterpret_cast<TC*>(smem);
  const int64_t wP = (a.n_params + 7) / 8 * 8;
  float* dw = reinterpret_cast<float*>(w + wP);
  const int64_t dwP = a.dw_in_lds ? wP : 0;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  const int ldin = a.nip + 4, ldh = a.width + 4, ldo = a.nop + 4;
  const int gmax = a.width > a.nop ? a.width : a.nop;
  const int ldg = gmax + 4;
  const int64_t per_wave = 16 * (ldin + (a.nl - 1) * ldh + ldo + 2 * ldg);
  TC* base = reinterpret_cast<TC*>(dw + dwP) + static_cast<int64_t>(wave) * per_wave;
  TC* act0 = base;                          // 16 x nip
  TC* acth = act0 + 16 * ldin;              // (nl-1) x 16 x width
  TC* outb = acth + (a.nl - 1) * 16 * ldh;  // 16 x nop (activated output)
  TC* g0 = outb + 16 * ldo;
  TC* g1 = g0 + 16 * ldg;

  stage_weights<TC>(a, w);
  if (a.dw_in_lds)
    for (int64_t i = threadIdx.x; i < a.n_params; i += blockDim.x) dw[i] = 0.0f;
  __syncthreads();

  auto act_ptr = [&](int k) -> TC* { return k == 0 ? act0 : acth + (k - 1) * 16 * ldh; };
  auto act_ld = [&](int k) -> int { return k == 0 ? ldin : ldh; };

  const int64_t n_tiles = (a.M + 15) / 16;
  for (int64_t tile = static_cast<int64_t>(blockIdx.x) * a.waves + wave; tile < n_tiles;
       tile += static_cast<int64_t>(gridDim.x) * a.waves) {
    const int64_t r0 = tile * 16;
    // ---- recompute forward, keeping every layer's input tile
    load_input_tile<TC>(a, r0, act0, ldin, lane);
    wave_sync();
    int64_t woff = 0;
    for (int k = 0; k < a.nl; ++k) {
      const int K = layer_in(a, k), N = layer_out(a, k);
      const bool last = k == a.nl - 1;
      TC* dst = last ? outb : act_ptr(k + 1);
      const int ldd = last ? ldo : ldh;
      layer_fwd<TC>(act_ptr(k), act_ld(k), w + woff, K, N, dst, ldd,
                    last ? a.out_relu != 0 : true, lane);
      wave_sync();
      woff += static_cast<int64_t>(K) * N;
    }
    // ---- output gradient tile (masked by the output ReLU), scaled for f16
    float gmaxabs = 0.0f;
    for (int e = lane; e < 16 * a.nop; e += kWave) {
      const int r = e / a.nop, c = e - r * a.nop;
      const int64_t row = r0 + r;
      float v = 0.0f;
      if (row < a.M && c < a.n_out) v = load_dyn(a.dout, a.dout_dt, row * a.dout_stride + c);
      if (a.out_relu && !(static_cast<float>(outb[r * ldo + c]) > 0.0f)) v = 0.0f;
      gmaxabs = fmaxf(gmaxabs, fabsf(v));
    }
    float s = 1.0f, inv_s = 1.0f;
    if (sizeof(TC) == 2) {
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) gmaxabs = fmaxf(gmaxabs, shfl_xor(gmaxabs, m));
      if (gmaxabs > 0.0f) {
        int e2 = static_cast<int>(floorf(log2f(256.0f / gmaxabs)));
        e2 = e2 < -60 ? -60 : (e2 > 100 ? 100 : e2);
        s = ldexpf(1.0f, e2);
        inv_s = ldexpf(1.0f, -e2);
      }
    }
    for (int e = lane; e < 16 * a.nop; e += kWave) {
      const int r = e / a.nop, c = e - r * a.nop;
      const int64_t row = r0 + r;
      float v = 0.0f;
      if (row < a.M && c < a.n_out) v = load_dyn(a.dout, a.dout_dt, row * a.dout_stride + c);
      if (a.out_relu && !(static_cast<float>(outb[r * ldo + c]) > 0.0f)) v = 0.0f;
      g0[r * ldg + c] = static_cast<TC>(v * s);
    }
    wave_sync();
    // ---- backward through the layers
    TC* g = g0;
    TC* gn = g1;
    for (int k = a.nl - 1; k >= 0; --k) {
      const int K = layer_in(a, k), N = layer_out(a, k);
      woff -= static_cast<int64_t>(K) * N;
      const TC* Wk = w + woff;
      const TC* act = act_ptr(k);
      const int lda = act_ld(k);
      // dW_k (N x K) += gᵀ (N x 16) · act (16 x K)
      for (int mt = 0; mt < N / 16; ++mt) {
        for (int nt = 0; nt < K / 16; ++nt) {
          f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < 16; ks += F::KS) {
            const typename F::frag av = F::ld_cols(g + ks * ldg + mt * 16, ldg, lane);
            const typename F::frag bv = F::ld_cols(act + ks * lda + nt * 16, lda, lane);
            acc = F::mma(av, bv, acc);
          }
          const int col = nt * 16 + (lane & 15);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = mt * 16 + 4 * (lane >> 4) + i;
            const float v = acc[i] * inv_s;
            const int64_t o = woff + static_cast<int64_t>(row) * K + col;
            if (v != 0.0f) {
              if (a.dw_in_lds)
                atomicAdd(dw + o, v);
              else
                atomicAdd(a.dparams + o, v);
            }
          }
        }
      }
      // dAct_k (16 x K) = g (16 x N) · W_k (N x K)
      if (k > 0 || a.out != nullptr) {
        for (int nt = 0; nt < K / 16; ++nt) {
          f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
          for (int ks = 0; ks < N; ks += F::KS) {
            const typename F::frag av = F::ld_rows(g + ks, ldg, lane);
            const typename F::frag bv = F::ld_cols(Wk + static_cast<int64_t>(ks) * K + nt * 16, K, lane);
            acc = F::mma(av, bv, acc);
          }
          const int col = nt * 16 + (lane & 15);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 4 * (lane >> 4) + i;
            if (k > 0) {
              // ReLU': act_k = relu(pre_{k-1}) > 0
              const bool on = static_cast<float>(act[row * lda + col]) > 0.0f;
              gn[row * ldg + col] = static_cast<TC>(on ? acc[i] : 0.0f);
            } else {
              const int64_t grow = r0 + row;
              if (grow < a.M && col < a.n_in)
                store_dyn(a.out, a.out_dt, grow * a.out_stride + col, acc[i] * inv_s);
            }
          }
        }
      }
      wave_sync();
      TC* t = g; g = gn; gn = t;
    }
  }
  if (a.dw_in_lds) {
    __syncthreads();
    for (int64_t i = threadIdx.x; i < a.n_params; i += blockDim.x) {
      const float v = dw[i];
      if (v != 0.0f) atomicAdd(a.dparams + i, v);
    }
  }
}

static int64_t n_params_of(const anr_mlp_desc* d) {
  int64_t n = static_cast<int64_t>(d->width) * d->n_input_padded;
  n += static_cast<int64_t>(d->n_hidden_layers - 1) * d->width * d->width;
  n += static_cast<int64_t>(d->n_output_padded) * d->width;
  return n;
}

static int check_desc(const anr_mlp_desc* d) {
  ANR_CHECK_ARG(d, "mlp: null desc");
  ANR_CHECK_ARG(d->width == 16 || d->width == 32 || d->width == 64 || d->width == 128,
                "mlp: width %d not in {16,32,64,128}", d->width);
  ANR_CHECK_ARG(d->n_hidden_layers >= 1 && d->n_hidden_layers <= 8, "mlp: n_hidden_layers");
  ANR_CHECK_ARG(d->n_input >= 1 && d->n_input_padded % 16 == 0 &&
                    d->n_input_padded >= d->n_input && d->n_input_padded <= 256,
                "mlp: bad input padding %d/%d", d->n_input, d->n_input_padded);
  ANR_CHECK_ARG(d->n_output >= 1 && d->n_output_padded % 16 == 0 &&
                    d->n_output_padded >= d->n_output && d->n_output_padded <= 256,
                "mlp: bad output padding %d/%d", d->n_output, d->n_output_padded);
  ANR_CHECK_ARG(d->activation == ANR_ACT_RELU, "mlp: only ReLU hidden activation");
  ANR_CHECK_ARG(d->output_activation == ANR_ACT_NONE || d->output_activation == ANR_ACT_RELU,
                "mlp: output activation must be None or ReLU");
  return ANR_OK;
}

static MlpArgs base_args(const anr_mlp_desc* d, int64_t M) {
  MlpArgs a{};
  a.nip = d->n_input_padded;
  a.n_in = d->n_input;
  a.nop = d->n_output_padded;
  a.n_out = d->n_output;
  a.width = d->width;
  a.nl = d->n_hidden_layers + 1;
  a.out_relu = d->output_activation == ANR_ACT_RELU;
  a.M = M;
  a.n_params = n_params_of(d);
  return a;
}

static int grid_for(int64_t M, int waves, int max_blocks) {
  int64_t tiles = (M + 15) / 16;
  int64_t blocks = (tiles + waves - 1) / waves;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  return static_cast<int>(blocks);
}

constexpr size_t kLdsBudget = 160 * 1024;

int mlp_fused_try(const anr_mlp_desc* d, int32_t precision, bool bwd, const void* params,
                  const void* in, int32_t in_dt, int64_t in_stride, int64_t M,
                  const void* dout, int32_t dout_dt, int64_t dout_stride, void* out,
                  int32_t out_dt, int64_t out_stride, float* dparams, hipStream_t st,
                  float* slab = nullptr, int64_t slab_floats = 0, float loss_scale = 0.0f);
bool mlp_fused_has(const anr_mlp_desc* d);

// ANR_MLP_GENERIC=1 (or anr_mlp_force_generic) forces the generic kernels.
static int g_force_generic = [] {
  const char* e = getenv("ANR_MLP_GENERIC");
  return (e && e[0] == '1') ? 1 : 0;
}();
static bool force_generic() { return g_force_generic != 0; }

}  // namespace anr

extern "C" int anr_mlp_force_generic(int32_t on) {
  const int prev = anr::g_force_generic;
  anr::g_force_generic = on ? 1 : 0;
  return prev;
}

extern "C" int64_t anr_mlp_n_params(const anr_mlp_desc* d) {
  if (anr::check_desc(d) != ANR_OK) return -1;
  return anr::n_params_of(d);
}

extern "C" int anr_mlp_fwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                           const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                           void* out, int32_t out_dtype, int64_t out_stride,
                           anr_stream_t stream) {
  using namespace anr;
  if (int rc = check_desc(d)) return rc;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(params && in && out, "anr_mlp_fwd: null argument");
  ANR_CHECK_ARG(precision == ANR_F16 || precision == ANR_F32, "anr_mlp_fwd: bad precision");
  ANR_CHECK_ARG(M >= 0 && in_stride >= d->n_input && out_stride >= d->n_output,
                "anr_mlp_fwd: bad shape/stride");
  if (M == 0) return ANR_OK;
  if (!force_generic() &&
      mlp_fused_try(d, precision, false, params, in, in_dtype, in_stride, M, nullptr, 0, 0,
                    out, out_dtype, out_stride, nullptr, as_stream(stream)) == 0) {
    ANR_CHECK_LAUNCH("anr_mlp_fwd(fused)");
    return ANR_OK;
  }
  MlpArgs a = base_args(d, M);
  a.params = params;
  a.in = in;
  a.in_dt = in_dtype;
  a.in_stride = in_stride;
  a.out = out;
  a.out_dt = out_dtype;
  a.out_stride = out_stride;
  const size_t es = precision == ANR_F16 ? 2 : 4;
  const int ldmax = std::max(std::max(a.nip, a.width), a.nop) + 4;
  const size_t wbytes = static_cast<size_t>((a.n_params + 7) / 8 * 8) * es;
  int waves = 4;
  while (waves > 1 && wbytes + static_cast<size_t>(waves) * 2 * 16 * ldmax * es > kLdsBudget / 2)
    --waves;
  const size_t lds = wbytes + static_cast<size_t>(waves) * 2 * 16 * ldmax * es;
  ANR_CHECK_ARG(lds <= kLdsBudget, "anr_mlp_fwd: network too large for LDS (%zu bytes)", lds);
  a.waves = waves;
  const dim3 grid(grid_for(M, waves, 2048)), block(64 * waves);
  if (precision == ANR_F16) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fwd_kernel<_Float16>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(mlp_fwd_kernel<_Float16>, grid, block, lds, as_stream(stream), a);
  } else {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fwd_kernel<float>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(mlp_fwd_kernel<float>, grid, block, lds, as_stream(stream), a);
  }
  ANR_CHECK_LAUNCH("anr_mlp_fwd");
  return ANR_OK;
}

// Batches up to this many rows may use the slab (per-wavefront dW rows + one reduction)
// instead of atomics in the specialised backward: with one 16-row tile per wavefront the
// atomics pile onto the same few KB of dW (the per-ray surface network, 8192 rows).
constexpr int64_t kSlabMaxRows = 1 << 16;

extern "C" int64_t anr_mlp_bwd_workspace_bytes(const anr_mlp_desc* d, int64_t M) {
  using namespace anr;
  if (check_desc(d) != ANR_OK || M <= 0 || M > kSlabMaxRows || !mlp_fused_has(d)) return 0;
  const int64_t waves = (M + 15) / 16 + 3;  // one 16-row tile per wavefront, 4 per block
  return waves * n_params_of(d) * static_cast<int64_t>(sizeof(float));
}

static int mlp_bwd_impl(const anr_mlp_desc* d, int32_t precision, const void* params,
                        const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                        const void* dout, int32_t dout_dtype, int64_t dout_stride, void* din,
                        int32_t din_dtype, int64_t din_stride, float* dparams,
                        void* workspace, int64_t workspace_bytes, anr_stream_t stream,
                        float loss_scale = 0.0f) {
  using namespace anr;
  if (int rc = check_desc(d)) return rc;
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(loss_scale == 0.0f || (loss_scale > 0.0f && precision == ANR_F16),
                "anr_mlp_bwd: reference numerics (loss_scale) need f16");
  ANR_CHECK_ARG(params && in && dout && dparams, "anr_mlp_bwd: null argument");
  ANR_CHECK_ARG(precision == ANR_F16 || precision == ANR_F32, "anr_mlp_bwd: bad precision");
  ANR_CHECK_ARG(M >= 0 && in_stride >= d->n_input && dout_stride >= d->n_output &&
                    (din == nullptr || din_stride >= d->n_input),
                "anr_mlp_bwd: bad shape/stride");
  if (M == 0) return ANR_OK;
  if (!force_generic() &&
      mlp_fused_try(d, precision, true, params, in, in_dtype, in_stride, M, dout, dout_dtype,
                    dout_stride, din, din_dtype, din_stride, dparams, as_stream(stream),
                    M <= kSlabMaxRows ? static_cast<float*>(workspace) : nullptr,
                    workspace_bytes / static_cast<int64_t>(sizeof(float)), loss_scale) == 0) {
    ANR_CHECK_LAUNCH("anr_mlp_bwd(fused)");
    return ANR_OK;
  }
  ANR_CHECK_ARG(loss_scale == 0.0f,
                "anr_mlp_bwd_ref16: no specialised kernel for this shape (reference numerics "
                "run on the fused MLP kernels only)");
  MlpArgs a = base_args(d, M);
  a.params = params;
  a.in = in;
  a.in_dt = in_dtype;
  a.in_stride = in_stride;
  a.dout = dout;
  a.dout_dt = dout_dtype;
  a.dout_stride = dout_stride;
  a.out = din;
  a.out_dt = din_dtype;
  a.out_stride = din_stride;
  a.dparams = dparams;
  const size_t es = precision == ANR_F16 ? 2 : 4;
  const size_t wP = static_cast<size_t>((a.n_params + 7) / 8 * 8);
  const int gmax = std::max(a.width, a.nop);
  const size_t per_wave =
      16 * static_cast<size_t>((a.nip + 4) + (a.nl - 1) * (a.width + 4) + (a.nop + 4) +
                               2 * (gmax + 4)) * es;
  int dw_in_lds = 1;
  size_t fixed = wP * es + wP * 4;
  if (fixed + per_wave > kLdsBudget) {
    dw_in_lds = 0;
    fixed = wP * es;
  }
  int waves = 4;
  while (waves > 1 && fixed + waves * per_wave > kLdsBudget) --waves;
  const size_t lds = fixed + waves * per_wave;
  ANR_CHECK_ARG(lds <= kLdsBudget, "anr_mlp_bwd: network too large for LDS (%zu bytes)", lds);
  a.waves = waves;
  a.dw_in_lds = dw_in_lds;
  const dim3 grid(grid_for(M, waves, 1024)), block(64 * waves);
  if (precision == ANR_F16) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_bwd_kernel<_Float16>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(mlp_bwd_kernel<_Float16>, grid, block, lds, as_stream(stream), a);
  } else {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_bwd_kernel<float>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(mlp_bwd_kernel<float>, grid, block, lds, as_stream(stream), a);
  }
  ANR_CHECK_LAUNCH("anr_mlp_bwd");
  return ANR_OK;
}

extern "C" int anr_mlp_bwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                           const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                           const void* dout, int32_t dout_dtype, int64_t dout_stride,
                           void* din, int32_t din_dtype, int64_t din_stride, float* dparams,
                           anr_stream_t stream) {
  return mlp_bwd_impl(d, precision, params, in, in_dtype, in_stride, M, dout, dout_dtype,
                      dout_stride, din, din_dtype, din_stride, dparams, nullptr, 0, stream);
}

extern "C" int anr_mlp_bwd_ws(const anr_mlp_desc* d, int32_t precision, const void* params,
                              const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                              const void* dout, int32_t dout_dtype, int64_t dout_stride,
                              void* din, int32_t din_dtype, int64_t din_stride, float* dparams,
                              void* workspace, int64_t workspace_bytes, anr_stream_t stream) {
  return mlp_bwd_impl(d, precision, params, in, in_dtype, in_stride, M, dout, dout_dtype,
                      dout_stride, din, din_dtype, din_stride, dparams, workspace,
                      workspace_bytes, stream);
}

extern "C" int anr_mlp_bwd_ref16(const anr_mlp_desc* d, const void* params, const void* in,
                                 int32_t in_dtype, int64_t in_stride, int64_t M,
                                 const void* dout, int32_t dout_dtype, int64_t dout_stride,
                                 void* din, int32_t din_dtype, int64_t din_stride,
                                 float* dparams, void* workspace, int64_t workspace_bytes,
                                 float loss_scale, anr_stream_t stream) {
  ANR_CHECK_ARG(loss_scale > 0.0f, "anr_mlp_bwd_ref16: loss_scale must be > 0");
  return mlp_bwd_impl(d, ANR_F16, params, in, in_dtype, in_stride, M, dout, dout_dtype,
                      dout_stride, din, din_dtype, din_stride, dparams, workspace,
                      workspace_bytes, stream, loss_scale);
}
