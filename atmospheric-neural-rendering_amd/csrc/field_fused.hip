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

#include <type_traits>

#include "anr_common.h"
#include "hash_levels.h"

// Profiling ablations (tools/field_ablate.sh); 0 in every product build. Bits:
// 1 no dW MFMAs, 2 no layer-input stores, 4 no gradient-tile stores, 8 no mask reads.
#ifndef FIELD_EXP
#define FIELD_EXP 0
#endif
// Stage barrier of the backward: which instruction classes may be scheduled across the
// point where a stage's LDS reads have been issued (sched_barrier mask: 0x1 ALU, 0x2
// VALU, 0x4 SALU, 0x8 MFMA; memory instructions never cross).
#ifndef FIELD_STAGE_MASK
#define FIELD_STAGE_MASK 0
#endif

namespace anr {
namespace field {

#ifdef FIELD_STAMP
// per-stage cycle totals of wavefront 0 of the backward (s_memtime), debug builds only
__device__ unsigned long long g_stamp[16];
#define STAMP(k)                                                             \
  do {                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                       \
    unsigned long long t_;                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));        \
    __builtin_amdgcn_sched_barrier(0);                                       \
    if (stamp_on) { st_acc[k] += t_ - st_last; }                             \
    st_last = t_;                                                            \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

// 16-bit operand carriers. With BF = false they hold f16 values; with BF = true
// (BASELINE configs[4]: bf16 MFMA MLP over the f16 hash features) the same vectors carry
// bf16 bit patterns: only the MFMA opcodes, the f32 -> 16-bit conversions, the ReLU and
// the constants differ, everything in between (LDS tiles, transposed reads, ReLU masks
// on the bits) is type-blind.
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((vector_size(8)));
typedef short s4e __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

template <bool BF>
__device__ __forceinline__ f4 mma32(h8 a, h8 b, f4 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a),
                                                   __builtin_bit_cast(b8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// dW accumulation: the accumulator lives in AGPRs for the whole kernel (the rest of the
// kernel's MFMAs write VGPRs). The compiler does not see these as MFMAs, so every VALU
// access to an accumulator goes through agpr_fence() + agpr_pin() first (result-latency
// wait states); volatile keeps them in program order with the fence.
template <bool BF>
__device__ __forceinline__ void mma32_acc(f4& acc, h8 a, h8 b) {
  if constexpr ((FIELD_EXP & 1) != 0) return;
  if constexpr (BF)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// the same with operands fresh from VALU (the register-transposed backward): two wait
// states between a VALU write of an operand and the MFMA reading it (hipcc pads nothing
// inside an asm statement). Volatile, so these stay in program order with agpr_fence():
// the register allocator may copy the accumulators between AGPRs at a loop exit
// (v_accvgpr_mov / _read, measured in the bf16 W=64 instantiation), and such a copy must
// not read an accumulator that an MFMA is still writing — every tile ends with a fence.
template <bool BF>
__device__ __forceinline__ void mma32_acc_v(f4& acc, h8 a, h8 b) {
  if constexpr ((FIELD_EXP & 1) != 0) return;
  if constexpr (BF)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void agpr_fence() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}
// After agpr_fence(): an empty volatile asm that "rewrites" each accumulator, so no read
// or copy of it (v_accvgpr_read / _mov are register-only, which a "memory" clobber does
// not order) can be scheduled above the fence.
template <int N>
__device__ __forceinline__ void agpr_pin(f4 (&acc)[N]) {
  if constexpr ((FIELD_EXP & 1) != 0) return;
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+a"(acc[i]));
}
template <bool BF>
__device__ __forceinline__ f4 mma16(h4 a, h4 b, f4 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4e, a),
                                                     __builtin_bit_cast(s4e, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
// one f32 -> the 16-bit operand type (round to nearest even), as bits in a _Float16
template <bool BF>
__device__ __forceinline__ _Float16 cvt1(float v) {
  if constexpr (BF)
    return __builtin_bit_cast(_Float16, static_cast<__bf16>(v));
  else
    return static_cast<_Float16>(v);
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
  static constexpr int wave_x = oXd1 + (NHD - 1) * 32 * LH;  // layer-input tiles
  static constexpr int oGa = 0, oGb = 32 * LH, wave_g = 2 * 32 * LH;  // gradient tiles
  static constexpr int wave_lds = wave_x + wave_g;
};

// ---------------------------------------------------------------------------------
// weight packing (f32 master params -> f16 fragments)
// ---------------------------------------------------------------------------------
template <int W, int NHD, bool BF>
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
  out[e] = cvt1<BF>(v);
}

struct Args {
  const _Float16* packed;
  const _Float16* enc;
  // row r, levels 4g..4g+3 (one lane's 8 values) at enc + r * enc_stride + g * enc_gstride:
  // row layout (M, >= 32): gstride 8; level-quad planes (anr_hashgrid_fwd_planes,
  // enc_stride = -plane at the ABI): enc_stride 8, gstride = plane
  int64_t enc_stride;
  int64_t enc_gstride;
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
  // occupancy-compacted samples (nullable): row r of enc / d_enc is sample rows[r] of the
  // dense (ray-major) arrays sigma, color, d_sigma, d_color; its ray is rows[r] / n_per_ray
  const int32_t* rows;
  // > 0: reference numerics (tcnn's loss-scaled f16 backward, anr_ingp_field_bwd_ref16):
  // fixed gradient scale, f16 module-boundary gradients; 0: per-wavefront dynamic scale
  float loss_scale;
  // nullable: per 32-row tile, 1 if the tile's incoming gradients had a nonzero value (the
  // tile was walked), 0 if it was skipped (dL/denc rows zero) -- the hash-grid backward
  // then skips those rows without loading them (anr_hashgrid_bwd_tiles)
  uint8_t* tile_nz;
  // anr_ingp_field_bwd_ref16_rows: dL/denc as f16 rows (instead of d_enc) and per 32-row
  // tile a word of row bits, bit i set when row 32 t + i has a nonzero value
  _Float16* d_enc_h;
  uint32_t* row_nz;
  // its pos / list passes (workspace): the tiles with a nonzero dL/dcolor and their count
  int32_t* tile_list;
  uint32_t* tile_count;
};

// ROWS is a compile-time choice: a run-time test on a.rows in the prefetch paths put a
// branch join (and with it a wait for the in-flight loads) in front of the MFMAs
template <bool ROWS>
__device__ __forceinline__ int64_t dense_row(const Args& a, int64_t row) {
  if constexpr (ROWS) return static_cast<int64_t>(a.rows[row]);
  return row;
}

__device__ __forceinline__ h8 cat(h4 a, h4 b) {
  return h8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}
// f32 accumulators -> 16-bit (round to nearest even, v_cvt_pk_{f16,bf16}_f32)
template <bool BF>
__device__ __forceinline__ h4 to_h4(f4 v) {
  if constexpr (BF)
    return __builtin_bit_cast(h4, __builtin_convertvector(v, b4));
  else
    return __builtin_convertvector(v, h4);
}
// -> ReLU: f16 after the conversion (v_pk_max_f16), bf16 before it (v_max_f32)
template <bool BF>
__device__ __forceinline__ h4 relu_h4(f4 v) {
  if constexpr (BF) {
    return to_h4<true>(__builtin_elementwise_max(v, f4{0.0f, 0.0f, 0.0f, 0.0f}));
  } else {
    const h4 x = __builtin_convertvector(v, h4);
    return __builtin_elementwise_max(x, h4{0, 0, 0, 0});
  }
}
// the f16 hash features as MFMA operands (bf16: f16 -> f32 -> bf16, round to nearest)
template <bool BF>
__device__ __forceinline__ h8 enc_in(h8 e) {
  if constexpr (BF) {
    const h4 lo = {e[0], e[1], e[2], e[3]}, hi = {e[4], e[5], e[6], e[7]};
    const h4 a = to_h4<true>(__builtin_convertvector(lo, f4));
    const h4 b = to_h4<true>(__builtin_convertvector(hi, f4));
    return h8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  } else {
    return e;
  }
}
// ReLU derivative: keep g where the forward activation (>= 0, f16) is nonzero. On the bits:
// v_pk_min_u16(act, 1) is 0 or 1 per half and v_pk_mul_lo_u16 by it keeps or clears g
// (two instructions per pair; written as asm because the compiler expands it to compares
// and selects). The result feeds MFMAs, and hipcc pads nothing for a VALU write inside an
// asm statement: the two wait states a VALU-written MFMA operand needs end the string.
template <bool BF>
__device__ __forceinline__ h4 mask_h4(f4 g, h4 act) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  const u2 gb = __builtin_bit_cast(u2, to_h4<BF>(g)), ab = __builtin_bit_cast(u2, act);
  uint32_t m0, m1;
  asm("v_pk_min_u16 %0, %2, 1 op_sel_hi:[1,0]\n\t"
      "v_pk_min_u16 %1, %3, 1 op_sel_hi:[1,0]\n\t"
      "v_pk_mul_lo_u16 %0, %4, %0\n\t"
      "v_pk_mul_lo_u16 %1, %5, %1\n\t"
      "s_nop 1"
      : "=&v"(m0), "=&v"(m1)
      : "v"(ab.x), "v"(ab.y), "v"(gb.x), "v"(gb.y));
  return __builtin_bit_cast(h4, u2{m0, m1});
}

// Reference numerics: the gradient tiles hold tcnn's loss-scaled f16 values, many of them
// deep in f16's subnormal range, and v_mfma_f32_16x16x32_f16 sums products of deeply
// subnormal f16 operands inexactly (a single product is exact; 64-term sums of operands
// ~2^-20 come out 28,844 f32 ulps rms from the exact sum against 62 for an f32 loop, with
// a bias toward zero: tools/r5/mfma_precision.py, profiles/r05_mfma_precision.log). The
// input-gradient products therefore take the subnormal part of the gradient operand
// separately, scaled by 2^10 into the normal range (exact: a power of two, and every
// subnormal times 2^10 stays below 1/16): W g = W g_normal + 2^-10 W (2^10 g_subnormal).
// The split is exact and the two f32 partial sums are added once. (The dW products keep
// the plain operand: their sums are dominated by the normal-range gradients.)
#ifndef ANR_REF_SPLIT
#define ANR_REF_SPLIT 0
#endif
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split_sub(h4 g, h4& gn, h4& gs) {
  const u16x4 b = __builtin_bit_cast(u16x4, g);
  const u16x4 z = {0, 0, 0, 0};
  const u16x4 sub = (b & u16x4{0x7C00, 0x7C00, 0x7C00, 0x7C00}) == z ? b : z;  // exp field 0
  gn = __builtin_bit_cast(h4, b ^ sub);
  const _Float16 k = static_cast<_Float16>(1024.0f);
  gs = __builtin_bit_cast(h4, sub) * h4{k, k, k, k};
}

// Global inputs of one 16-sample half-tile for this lane, loaded a tile ahead.
struct Rows {
  h8 xe;          // enc[row][8g .. 8g+7]
  float dx, dy, dz;  // direction of the row's ray, remapped 2d-1 (g == 0 lanes)
  f4 dc;          // dL/dcolor[row][4g .. 4g+3] (backward)
  float ds;       // dL/dsigma[row] (backward, g == 0 lanes)
};

template <bool ROWS>
__device__ __forceinline__ void load_rows(const Args& a, int64_t row, int g, bool bwd, Rows& in) {
  in.xe = h8{};
  in.dx = in.dy = in.dz = 0.0f;
  in.dc = f4{0.0f, 0.0f, 0.0f, 0.0f};
  in.ds = 0.0f;
  if (row >= a.M) return;
  in.xe = *reinterpret_cast<const h8*>(a.enc + row * a.enc_stride + g * a.enc_gstride);
  const int64_t drow = dense_row<ROWS>(a, row);
  if (g == 0) {
    const uint32_t ray = static_cast<uint32_t>(drow) / a.n_per_ray;
    const float* d = a.dirs + static_cast<int64_t>(ray) * 3;
    in.dx = d[0] * 2.0f - 1.0f;
    in.dy = d[1] * 2.0f - 1.0f;
    in.dz = d[2] * 2.0f - 1.0f;
    if (bwd && a.d_sigma) in.ds = a.d_sigma[drow];
  }
  if (bwd) {
    const int c0 = 4 * g;
    const float* dcp = a.d_color + drow * a.d_color_stride + c0;
    if (c0 + 3 < a.n_out && (a.d_color_stride & 3) == 0) {
      in.dc = *reinterpret_cast<const f4*>(dcp);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (c0 + i < a.n_out) in.dc[i] = dcp[i];
    }
  }
}

// Input row of the dir MLP for the sample in this lane (B-operand slots 8g..8g+7).
// Branch-free (per-lane selects): a divergent branch here gives the compiler a place to
// merge other g == 0 code into, including uses of the backward's prefetched loads, which
// then wait for those loads at once.
template <bool BF>
__device__ __forceinline__ h8 dir_input(const Rows& in, bool valid, int g, f4 po) {
  const _Float16 one = cvt1<BF>(1.0f);
  const h8 lead = {one, cvt1<BF>(po[1]), cvt1<BF>(po[2]), cvt1<BF>(po[3]),
                   cvt1<BF>(0.28209479177387814f), cvt1<BF>(-0.48860251190291987f * in.dy),
                   cvt1<BF>(0.48860251190291987f * in.dz), cvt1<BF>(-0.48860251190291987f * in.dx)};
  const h8 rest = {cvt1<BF>(po[0]), cvt1<BF>(po[1]), cvt1<BF>(po[2]), cvt1<BF>(po[3]), one, one,
                   one, one};
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const u4 l = __builtin_bit_cast(u4, lead), r = __builtin_bit_cast(u4, rest);
  const bool g0 = g == 0;
  u4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = valid ? (g0 ? l[i] : r[i]) : 0u;
  return __builtin_bit_cast(h8, v);
}

template <int W, int NHD>
struct FwdWeights {
  using N = Net<W, NHD>;
  h8 p0[N::NT], p1[N::KB], d0[N::NT], d1[NHD == 2 ? N::NT * N::KB : 1], d2[N::KB];
  // dir = false: the pos network's fragments only (tile_forward without the dir network)
  __device__ void load(const _Float16* pk, int lane, bool dir = true) {
    auto ld = [&](int off) { return *reinterpret_cast<const h8*>(pk + off + lane * 8); };
#pragma unroll
    for (int i = 0; i < N::NT; ++i) p0[i] = ld(N::oFP0 + i * N::F32);
#pragma unroll
    for (int i = 0; i < N::KB; ++i) p1[i] = ld(N::oFP1 + i * N::F32);
    if (!dir) return;
#pragma unroll
    for (int i = 0; i < N::NT; ++i) d0[i] = ld(N::oFD0 + i * N::F32);
    if constexpr (NHD == 2) {
#pragma unroll
      for (int i = 0; i < N::NT * N::KB; ++i) d1[i] = ld(N::oFD1 + i * N::F32);
    }
#pragma unroll
    for (int i = 0; i < N::KB; ++i) d2[i] = ld(N::oFD2 + i * N::F32);
  }
  __device__ h8 P0(int i) const { return p0[i]; }
  __device__ h8 P1(int i) const { return p1[i]; }
  __device__ h8 D0(int i) const { return d0[i]; }
  __device__ h8 D1(int i) const { return d1[i]; }
  __device__ h8 D2(int i) const { return d2[i]; }
};

// The same fragments read from a packed copy in LDS (backward kernel).
template <int W, int NHD>
struct LdsWeights {
  using N = Net<W, NHD>;
  const _Float16* base;
  int lane;
  __device__ h8 frag(int off) const { return *reinterpret_cast<const h8*>(base + off + lane * 8); }
  __device__ h8 P0(int i) const { return frag(N::oFP0 + i * N::F32); }
  __device__ h8 P1(int i) const { return frag(N::oFP1 + i * N::F32); }
  __device__ h8 D0(int i) const { return frag(N::oFD0 + i * N::F32); }
  __device__ h8 D1(int i) const { return frag(N::oFD1 + i * N::F32); }
  __device__ h8 D2(int i) const { return frag(N::oFD2 + i * N::F32); }
};

// Forward of NM 16-sample tiles, layer by layer across the tiles (independent MFMAs back
// to back, so no result is consumed right after the instruction that produces it).
template <int W, int NHD>
struct Tile {
  using N = Net<W, NHD>;
  h8 xe, xd;
  h4 hp[N::NT], hd0[N::NT], hd1[NHD == 2 ? N::NT : 1];
  f4 po, col;
};

struct NoSink {
  __device__ void xe(int, h8) const {}
  __device__ void xd(int, h8) const {}
  __device__ void hp(int, int, h4) const {}
  __device__ void hd0(int, int, h4) const {}
  __device__ void hd1(int, int, h4) const {}
};

// sink: receives every layer input as soon as it is computed (the backward writes them
// to LDS there, so they need not stay live in registers)
// dir = false (wave-uniform): the pos network only; col = 0 (the backward of a tile whose
// dL/dcolor is zero in every row needs nothing of the dir network)
template <int W, int NHD, int NM, bool BF, typename WS, typename SK>
__device__ __forceinline__ void tile_forward(const WS& fw, const Rows* in, const bool* valid,
                                             int g, Tile<W, NHD>* t, const SK& sink,
                                             bool dir = true) {
  using N = Net<W, NHD>;
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    t[mt].xe = enc_in<BF>(in[mt].xe);
    sink.xe(mt, t[mt].xe);
  }
#pragma unroll
  for (int nt = 0; nt < N::NT; ++nt) {
    const h8 w = fw.P0(nt);
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      t[mt].hp[nt] = relu_h4<BF>(mma32<BF>(w, t[mt].xe, z4));
      sink.hp(mt, nt, t[mt].hp[nt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) t[mt].po = z4;
#pragma unroll
  for (int kb = 0; kb < N::KB; ++kb) {
    const h8 w = fw.P1(kb);
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) t[mt].po = mma32<BF>(w, cat(t[mt].hp[2 * kb], t[mt].hp[2 * kb + 1]), t[mt].po);
  }
  if (!dir) {
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) t[mt].col = z4;
    return;
  }
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    t[mt].xd = dir_input<BF>(in[mt], valid[mt], g, t[mt].po);
    sink.xd(mt, t[mt].xd);
  }
#pragma unroll
  for (int nt = 0; nt < N::NT; ++nt) {
    const h8 w = fw.D0(nt);
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      t[mt].hd0[nt] = relu_h4<BF>(mma32<BF>(w, t[mt].xd, z4));
      sink.hd0(mt, nt, t[mt].hd0[nt]);
    }
  }
  if constexpr (NHD == 2) {
#pragma unroll
    for (int nt = 0; nt < N::NT; ++nt) {
      f4 acc[NM];
#pragma unroll
      for (int mt = 0; mt < NM; ++mt) acc[mt] = z4;
#pragma unroll
      for (int kb = 0; kb < N::KB; ++kb) {
        const h8 w = fw.D1(nt * N::KB + kb);
#pragma unroll
        for (int mt = 0; mt < NM; ++mt)
          acc[mt] = mma32<BF>(w, cat(t[mt].hd0[2 * kb], t[mt].hd0[2 * kb + 1]), acc[mt]);
      }
#pragma unroll
      for (int mt = 0; mt < NM; ++mt) {
        t[mt].hd1[nt] = relu_h4<BF>(acc[mt]);
        sink.hd1(mt, nt, t[mt].hd1[nt]);
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) t[mt].col = z4;
#pragma unroll
  for (int kb = 0; kb < N::KB; ++kb) {
    const h8 w = fw.D2(kb);
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      const h4* last = NHD == 2 ? t[mt].hd1 : t[mt].hd0;
      t[mt].col = mma32<BF>(w, cat(last[2 * kb], last[2 * kb + 1]), t[mt].col);
    }
  }
}

// Raw inputs of one 16-sample tile of the forward, prefetched a tile ahead for tiles with
// all rows in range: every lane loads its row's encoding slice and its ray's direction
// (the four lane groups read the same direction: one cache line), nothing is computed on
// them until the next iteration, so no wait for these loads is placed in front of the
// current tile's MFMAs.
struct FwdRaw {
  h8 xe;
  float d0, d1, d2;
};

template <bool ROWS>
__device__ __forceinline__ void load_fwd_raw(const Args& a, int64_t row, int g, FwdRaw& r) {
  r.xe = *reinterpret_cast<const h8*>(a.enc + row * a.enc_stride + g * a.enc_gstride);
  const uint32_t ray = static_cast<uint32_t>(dense_row<ROWS>(a, row)) / a.n_per_ray;
  const float* d = a.dirs + static_cast<int64_t>(ray) * 3;
  r.d0 = d[0];
  r.d1 = d[1];
  r.d2 = d[2];
}

__device__ __forceinline__ void fwd_raw_to_rows(const FwdRaw& r, Rows& in) {
  in.xe = r.xe;
  in.dx = r.d0 * 2.0f - 1.0f;
  in.dy = r.d1 * 2.0f - 1.0f;
  in.dz = r.d2 * 2.0f - 1.0f;
  in.dc = f4{0.0f, 0.0f, 0.0f, 0.0f};
  in.ds = 0.0f;
}

// Uniform-tile forward (UT): dense rows, n_per_ray a multiple of 16, 4 colour outputs,
// 16-byte aligned colour rows, byte offsets below 2^31 — the bench and training shape.
// A 16-row tile is then one ray's samples, so its direction is one scalar load (scalar
// cache and lgkmcnt, not the vector-memory queue), and the outputs go out as raw buffer
// stores, one sigma and one 4-wide colour store per lane with no branch (lanes with
// nothing to write get an out-of-range offset, which the hardware drops). Every tile then
// issues the same vector-memory instructions (one input load, two stores), so the wait
// for the next tile's prefetched encodings is vmcnt(2) and leaves this tile's stores in
// flight. In the general form the per-lane guarded stores and the branch-sunk direction
// remap made the compiler wait with vmcnt(0) twice per tile: one store round trip and
// one prefetch round trip per tile.
typedef uint32_t u4v __attribute__((vector_size(16)));
typedef __attribute__((address_space(4))) const float const_f32;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes),
                                           0x00020000);
}

// Four waves per SIMD: at the compiler's free choice the W = 64 forward took 136 VGPRs
// (3 waves); capped at 128 it fits in 126 without spills, and the fourth wave hides more
// of the per-tile prefetch latency (field fwd 0.204 -> 0.201 ms, step -0.02 ms;
// profiles/r03_field_fwd_occ.log). The grid is sized from the same occupancy query.
template <int W, int NHD, bool ROWS, bool BF, bool UT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) fwd_kernel(Args a) {
  static_assert(!(UT && ROWS), "the uniform-tile form needs dense rows");
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  // wave index through readfirstlane: the tile loop then runs on scalar registers
  const int waves = blockDim.x >> 6, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  FwdWeights<W, NHD> fw;
  fw.load(a.packed, lane);
  const int64_t n_tiles = (a.M + 15) / 16;
  const int64_t n_full = a.M / 16;  // tiles with all 16 rows in range
  const int64_t tstride = static_cast<int64_t>(gridDim.x) * waves;
  int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave;
  auto store = [&](const Tile<W, NHD>& t, int64_t row) {
    if (row < a.M) {
      const int64_t drow = dense_row<ROWS>(a, row);
      if (g == 0) a.sigma[drow] = fmaxf(t.po[0], 0.0f);
      const int c0 = 4 * g;
      if (c0 + 3 < a.n_out && (a.color_stride & 3) == 0) {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(t.col[i], 0.0f);
        *reinterpret_cast<f4*>(a.color + drow * a.color_stride + c0) = v;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (c0 + i < a.n_out) a.color[drow * a.color_stride + c0 + i] = fmaxf(t.col[i], 0.0f);
      }
    }
  };
  auto body = [&](const Rows& cur, int64_t row) {
    Tile<W, NHD> t;
    const bool valid = row < a.M;
    tile_forward<W, NHD, 1, BF>(fw, &cur, &valid, g, &t, NoSink{});
    store(t, row);
  };
  if constexpr (UT) {
    const __amdgpu_buffer_rsrc_t rsig = out_rsrc(a.sigma, a.M * 4);
    const __amdgpu_buffer_rsrc_t rcol = out_rsrc(a.color, a.M * a.color_stride * 4);
    const uint32_t cs_bytes = static_cast<uint32_t>(a.color_stride) * 4u;
    auto enc_ptr = [&](int64_t t) {
      return reinterpret_cast<const h8*>(a.enc + (t * 16 + li) * a.enc_stride + g * a.enc_gstride);
    };
    h8 nxe;
    if (tile < n_full) {
      nxe = *enc_ptr(tile);
      // two dropped stores: the loop is entered with the vector-memory queue of its back
      // edge (an input load, then a tile's two stores)
      __builtin_amdgcn_raw_buffer_store_b32(0u, rsig, 0x80000000u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{0u, 0u, 0u, 0u}, rcol, 0x80000000u, 0, 0);
    }
    for (; tile < n_full; tile += tstride) {
      Rows cur;
      cur.xe = nxe;
      // wave-uniform ray and direction; readfirstlane (convergent) also keeps the loads from
      // being sunk into dir_input's g == 0 branch as vector loads
      const uint32_t ray =
          __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tile * 16) / a.n_per_ray);
      const const_f32* d = (const_f32*)(a.dirs + static_cast<int64_t>(ray) * 3);
      auto sdir = [&](int k) {
        return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, d[k])));
      };
      cur.dx = sdir(0) * 2.0f - 1.0f;
      cur.dy = sdir(1) * 2.0f - 1.0f;
      cur.dz = sdir(2) * 2.0f - 1.0f;
      cur.dc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      cur.ds = 0.0f;
      const int64_t tn = tile + tstride < n_full ? tile + tstride : tile;
      nxe = *enc_ptr(tn);
      Tile<W, NHD> t;
      const bool valid = true;
      tile_forward<W, NHD, 1, BF>(fw, &cur, &valid, g, &t, NoSink{});
      const uint32_t row = static_cast<uint32_t>(tile * 16 + li);
      const uint32_t so = g == 0 ? row * 4u : 0x80000000u;
      const uint32_t co = g == 0 ? row * cs_bytes : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaxf(t.po[0], 0.0f)), rsig, so, 0, 0);
      const u4v v = {__float_as_uint(fmaxf(t.col[0], 0.0f)), __float_as_uint(fmaxf(t.col[1], 0.0f)),
                     __float_as_uint(fmaxf(t.col[2], 0.0f)), __float_as_uint(fmaxf(t.col[3], 0.0f))};
      __builtin_amdgcn_raw_buffer_store_b128(v, rcol, co, 0, 0);
    }
  } else {
    // full tiles: the next tile's inputs are in flight while this one computes (the
    // prefetch index is clamped, so the loop body has no branch around the loads)
    FwdRaw nraw;
    if (tile < n_full) load_fwd_raw<ROWS>(a, tile * 16 + li, g, nraw);
    for (; tile < n_full; tile += tstride) {
      Rows cur;
      fwd_raw_to_rows(nraw, cur);
      const int64_t tn = tile + tstride < n_full ? tile + tstride : tile;
      load_fwd_raw<ROWS>(a, tn * 16 + li, g, nraw);
      body(cur, tile * 16 + li);
    }
  }
  for (; tile < n_tiles; tile += tstride) {  // the last, partial tile
    Rows cur;
    load_rows<ROWS>(a, tile * 16 + li, g, false, cur);
    body(cur, tile * 16 + li);
  }
}

// ---------------------------------------------------------------------------------
// Hash-grid forward + field forward in one kernel (r06). A wavefront
// takes 64 consecutive samples (one ray segment: n_per_ray is a multiple of 64) at a time:
//  1. hash phase, one lane per sample: the 16 levels as four level quads (plane_quad, the
//     arithmetic of anr_hashgrid_fwd_planes), each stored to its plane for the backward
//     and to the wavefront's LDS stage;
//  2. field phase, the four 16-sample tiles of the uniform-tile forward: lane group g reads
//     quad g of its sample from the stage -- exactly the B fragment of the first layer --
//     and tile_forward runs on weight fragments read from LDS.
// The planes are written once and never re-read by the forward (the separate field
// forward read all 64 B per sample back from HBM), and one wavefront's gathers overlap
// other wavefronts' MFMA tiles on the same CU. Bit-identical to anr_hashgrid_fwd_planes
// followed by anr_ingp_field_fwd (same per-level arithmetic, same MFMA sequence).
struct HashArgs {
  GridLevels G;
  const float* x;
  uint32_t x_bytes;
  const __half* table;
  uint32_t table_bytes;
  _Float16* planes;
  uint32_t plane_bytes;  // bytes from one level-quad plane to the next
  uint32_t out_bytes;    // bytes of the plane buffer (range check of the stores)
};

template <int W, int NHD, bool BF, int WAVES, int OCC, int DEDUP>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
hf_fwd_kernel(Args a, HashArgs h) {
  using N = Net<W, NHD>;
  typedef uint32_t u4q __attribute__((vector_size(16)));
  __shared__ __attribute__((aligned(16))) _Float16 wsm[N::n_fwd];
  // per wavefront: quad q of lane l's sample at stage[wave][q][l]
  __shared__ __attribute__((aligned(16))) u4q stage[WAVES][4][64];
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int e = threadIdx.x * 8; e < N::n_fwd; e += 64 * WAVES * 8)
    *reinterpret_cast<h8*>(wsm + e) = *reinterpret_cast<const h8*>(a.packed + e);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rx = wave_rsrc(h.x, h.x_bytes);
  const __amdgpu_buffer_rsrc_t rt = wave_rsrc(h.table, h.table_bytes);
  const __amdgpu_buffer_rsrc_t ro = wave_rsrc(h.planes, h.out_bytes);
  const __amdgpu_buffer_rsrc_t rsig = out_rsrc(a.sigma, a.M * 4);
  const __amdgpu_buffer_rsrc_t rcol = out_rsrc(a.color, a.M * a.color_stride * 4);
  const uint32_t cs_bytes = static_cast<uint32_t>(a.color_stride) * 4u;
  const int64_t n_super = (a.M + 63) / 64;
  const int64_t sstride = static_cast<int64_t>(gridDim.x) * WAVES;
  for (int64_t st = static_cast<int64_t>(blockIdx.x) * WAVES + wave; st < n_super; st += sstride) {
    const uint32_t m = static_cast<uint32_t>(st * 64) + lane;
    // ---- hash phase: lane = sample (coordinates past x's end read as 0, stores past M
    // dropped by the range check)
    const auto xr = __builtin_amdgcn_raw_buffer_load_b96(rx, m * 12u, 0, 0);
    const float xv[3] = {__uint_as_float(xr[0]), __uint_as_float(xr[1]), __uint_as_float(xr[2])};
    const uint32_t orow = m < a.M ? m * 16u : 0x80000000u;
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
      uint32_t p[4];
      plane_quad<3, __half, DEDUP>(h.G, 16, q, xv, rt, p);
      const u4q v = {p[0], p[1], p[2], p[3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, ro, static_cast<uint32_t>(q) * h.plane_bytes + orow,
                                             0, 0);
      stage[wave][q][lane] = v;
    }
    // one wavefront's LDS accesses complete in order: the stage is read back below without
    // a barrier (the fence keeps the compiler from hoisting the reads above the writes)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- field phase: the segment is one ray (n_per_ray % 64 == 0): scalar direction
    const uint32_t ray =
        __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(st * 64) / a.n_per_ray);
    const const_f32* d = (const_f32*)(a.dirs + static_cast<int64_t>(ray) * 3);
    auto sdir = [&](int k) {
      return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, d[k])));
    };
    Rows cur;
    cur.dx = sdir(0) * 2.0f - 1.0f;
    cur.dy = sdir(1) * 2.0f - 1.0f;
    cur.dz = sdir(2) * 2.0f - 1.0f;
    cur.dc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    cur.ds = 0.0f;
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      cur.xe = __builtin_bit_cast(h8, stage[wave][g][16 * t + li]);
      const uint32_t row = static_cast<uint32_t>(st * 64) + 16 * t + li;
      const bool valid = row < a.M;
      // per-tile opaque fragment base: the weight fragments are read from LDS at their
      // MFMAs instead of being hoisted out of the loops into 80 registers
      int zoff = 0;
      asm volatile("" : "+v"(zoff));
      const LdsWeights<W, NHD> fw{wsm + zoff, lane};
      Tile<W, NHD> tt;
      tile_forward<W, NHD, 1, BF>(fw, &cur, &valid, g, &tt, NoSink{});
      const uint32_t so = g == 0 && valid ? row * 4u : 0x80000000u;
      const uint32_t co = g == 0 && valid ? row * cs_bytes : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaxf(tt.po[0], 0.0f)), rsig, so, 0, 0);
      const u4v v = {__float_as_uint(fmaxf(tt.col[0], 0.0f)), __float_as_uint(fmaxf(tt.col[1], 0.0f)),
                     __float_as_uint(fmaxf(tt.col[2], 0.0f)), __float_as_uint(fmaxf(tt.col[3], 0.0f))};
      __builtin_amdgcn_raw_buffer_store_b128(v, rcol, co, 0, 0);
    }
    // the next segment's stage writes stay behind this segment's reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// C-layout (sample l&15, units 4g..4g+3) read back from row `mrow` of a row-major tile
__device__ __forceinline__ h4 ld4(const _Float16* base, int ld, int mrow, int col) {
  if constexpr ((FIELD_EXP & 8) != 0) return h4{1, 1, 1, 1};
  return *reinterpret_cast<const h4*>(base + mrow * ld + col);
}

// C-layout (sample l&15, units 4g..4g+3) store into row `mrow` of a row-major tile
__device__ __forceinline__ void st4(_Float16* base, int ld, int mrow, int col, h4 v) {
  *reinterpret_cast<h4*>(base + mrow * ld + col) = v;
}
// gradient-tile store (ablation bit 4)
__device__ __forceinline__ void st4g(_Float16* base, int ld, int mrow, int col, h4 v) {
  if constexpr ((FIELD_EXP & 4) != 0) return;
  *reinterpret_cast<h4*>(base + mrow * ld + col) = v;
}

// Density only: relu(pos_out[:, 0]) of tile_forward's pos MLP, the dir MLP (70 % of the
// field's MFMA work) skipped -- the extract loop (instant_ngp.py:208-247: only the
// extinction is read) and the occupancy grid's density. The same MFMA sequence as the
// full forward's pos half, so sigma is bit-identical to anr_ingp_field_fwd's. Weights in
// registers, one 16-row tile per wavefront step, the next tile's encodings in flight.
template <int W, int NHD, bool BF>
__global__ void __launch_bounds__(256) density_kernel(Args a) {
  using N = Net<W, NHD>;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int waves = blockDim.x >> 6, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  h8 p0[N::NT], p1[N::KB];
#pragma unroll
  for (int i = 0; i < N::NT; ++i)
    p0[i] = *reinterpret_cast<const h8*>(a.packed + N::oFP0 + i * N::F32 + lane * 8);
#pragma unroll
  for (int i = 0; i < N::KB; ++i)
    p1[i] = *reinterpret_cast<const h8*>(a.packed + N::oFP1 + i * N::F32 + lane * 8);
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t n_tiles = (a.M + 15) / 16;
  const int64_t tstride = static_cast<int64_t>(gridDim.x) * waves;
  int64_t tile = static_cast<int64_t>(blockIdx.x) * waves + wave;
  auto load = [&](int64_t t) -> h8 {
    const int64_t row = t * 16 + li;
    if (row < a.M) return *reinterpret_cast<const h8*>(a.enc + row * a.enc_stride + g * a.enc_gstride);
    return h8{};
  };
  h8 nxe = tile < n_tiles ? load(tile) : h8{};
  for (; tile < n_tiles; tile += tstride) {
    const h8 xe = enc_in<BF>(nxe);
    const int64_t tn = tile + tstride;
    if (tn < n_tiles) nxe = load(tn);
    h4 hp[N::NT];
#pragma unroll
    for (int nt = 0; nt < N::NT; ++nt) hp[nt] = relu_h4<BF>(mma32<BF>(p0[nt], xe, z4));
    f4 po = z4;
#pragma unroll
    for (int kb = 0; kb < N::KB; ++kb) po = mma32<BF>(p1[kb], cat(hp[2 * kb], hp[2 * kb + 1]), po);
    const int64_t row = tile * 16 + li;
    if (g == 0 && row < a.M) a.sigma[row] = fmaxf(po[0], 0.0f);
  }
}

// The f16 gradient scale's input for a wavefront with tiles [t_begin, t_end):
// absmax_kernel's value (0 for a wavefront without rows).
__device__ __forceinline__ float wave_grad_max(const Args& a, const float* wmax, int64_t w_id,
                                               int64_t t_begin, int64_t t_end) {
  (void)a;
  return t_begin >= t_end ? 0.0f : wmax[w_id];
}

// Rows of the backward's wavefront w: tiles [w*tpw, (w+1)*tpw) of 32 rows. The f16
// gradient scale of a wavefront is set from max(|dL/dcolor|, |dL/dsigma|) over its rows,
// which this kernel computes first (one block per wavefront range, full occupancy).
template <bool ROWS>
__global__ void __launch_bounds__(1024) absmax_kernel(Args a, int64_t rows_per_wave, float* wmax) {
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_wave;
  const int64_t r1 = r0 + rows_per_wave < a.M ? r0 + rows_per_wave : a.M;
  float m = 0.0f;
  if (a.n_out == 4 && (a.d_color_stride & 3) == 0) {
    // four rows per thread per iteration, loads issued before any max (one wait each)
    const int64_t step = blockDim.x;
    int64_t rr = r0 + threadIdx.x;
    for (; rr + 3 * step < r1; rr += 4 * step) {
      f4 d[4];
      float sg[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t r = dense_row<ROWS>(a, rr + k * step);
        d[k] = *reinterpret_cast<const f4*>(a.d_color + r * a.d_color_stride);
        sg[k] = a.d_sigma ? a.d_sigma[r] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(fabsf(d[k][0]), fabsf(d[k][1])),
                                 fmaxf(fabsf(d[k][2]), fabsf(d[k][3]))), fabsf(sg[k])));
    }
    for (; rr < r1; rr += step) {
      const int64_t r = dense_row<ROWS>(a, rr);
      const f4 d = *reinterpret_cast<const f4*>(a.d_color + r * a.d_color_stride);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(d[0]), fabsf(d[1])), fmaxf(fabsf(d[2]), fabsf(d[3]))));
      if (a.d_sigma) m = fmaxf(m, fabsf(a.d_sigma[r]));
    }
  } else {
    for (int64_t rr = r0 + threadIdx.x; rr < r1; rr += blockDim.x) {
      const int64_t r = dense_row<ROWS>(a, rr);
      for (int c = 0; c < a.n_out; ++c) m = fmaxf(m, fabsf(a.d_color[r * a.d_color_stride + c]));
      if (a.d_sigma) m = fmaxf(m, fabsf(a.d_sigma[r]));
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float part[16];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < static_cast<int>(blockDim.x >> 6); ++i) m = fmaxf(m, part[i]);
    wmax[blockIdx.x] = m;
  }
}

// Raw global inputs of one 16-sample half-tile of a FULL tile in the FAST case (n_out == 4,
// aligned d_color rows, d_sigma present), prefetched a tile ahead. Nothing is computed
// on the loaded values here — any use would make the compiler wait for the load right
// away; raw_to_rows() converts them one tile later. Every lane loads its row's direction,
// d_sigma and d_color (same addresses across the lane groups: no extra traffic).
struct RawRows {
  h8 xe;
  float d0, d1, d2, ds;
  f4 dc;
};

template <bool ROWS>
__device__ __forceinline__ void load_raw(const Args& a, int64_t row, int g, RawRows& r) {
  r.xe = *reinterpret_cast<const h8*>(a.enc + row * a.enc_stride + g * a.enc_gstride);
  const int64_t drow = dense_row<ROWS>(a, row);
  const uint32_t ray = static_cast<uint32_t>(drow) / a.n_per_ray;
  const float* d = a.dirs + static_cast<int64_t>(ray) * 3;
  r.d0 = d[0];
  r.d1 = d[1];
  r.d2 = d[2];
  r.ds = a.d_sigma[drow];
  r.dc = *reinterpret_cast<const f4*>(a.d_color + drow * a.d_color_stride);
}

__device__ __forceinline__ void raw_to_rows(const RawRows& r, int g, Rows& in) {
  in.xe = r.xe;
  in.dx = r.d0 * 2.0f - 1.0f;
  in.dy = r.d1 * 2.0f - 1.0f;
  in.dz = r.d2 * 2.0f - 1.0f;
  in.ds = r.ds;
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  in.dc = g == 0 ? r.dc : z4;
}

// ---------------------------------------------------------------------------------
// Backward, register-transposed: no layer input or gradient tile goes through LDS (LDS
// holds the packed weights and the block's dW sums). (The r01 generation that staged
// every tile in LDS and read it back with ds_read_b64_tr_b16, and r03's variant with only
// the dW operand transposes through LDS, were A/B generations; removed in r04.)
//
// dW += G^T · X contracts over the samples, so both operands need the samples along K
// (lane = unit, samples in the lane's registers) while the chain holds every tile with
// lane = sample. The transpose is one MFMA against a constant 0/1 matrix: a C-layout
// tile (lane = sample l&15, units 4g..4g+3) read as the A operand of a 16x16x16 MFMA is
// the tile with samples as rows, and times the identity it comes back in C layout with
// lane = unit l&15 and samples 4g..4g+3 — exact (one 1·x product per output, the other
// terms 0·x = 0 for finite x). Tiles held as 8-slot B operands (the encoding, the dir
// input) go through a 16x16x32 MFMA against [I|0] or [0|I]. The dW A operand of a
// 32-sample tile is then cat(transpose(half 0), transpose(half 1)), i.e. samples in the
// order (4g..4g+3, 16+4g..16+4g+3) along K, and the B operand the same: the contraction
// is order-blind.
// ReLU masks are the forward's activations, kept in registers.
// ---------------------------------------------------------------------------------
template <bool BF>
struct TrConst {
  h4 id;      // I16 as a 16x16x16 B operand: lane (column c = l&15) holds rows 4g..4g+3
  h8 sel[2];  // [I16; 0] and [0; I16] (32 x 16) as 16x16x32 B operands: slot 16kb + c
  __device__ void init(int lane) {
    const int c = lane & 15, g = lane >> 4;
    const _Float16 one = cvt1<BF>(1.0f), zero = cvt1<BF>(0.0f);
#pragma unroll
    for (int i = 0; i < 4; ++i) id[i] = 4 * g + i == c ? one : zero;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int j = 0; j < 8; ++j) sel[kb][j] = 8 * g + j == 16 * kb + c ? one : zero;
  }
};
// C-layout tile (lane = sample, 4 units) -> (lane = unit, 4 samples)
template <bool BF>
__device__ __forceinline__ h4 tr_c(h4 t, h4 id) {
  return to_h4<BF>(mma16<BF>(t, id, f4{0.0f, 0.0f, 0.0f, 0.0f}));
}
// B-operand tile (lane = sample, slots 8g..8g+7) -> (lane = slot 16kb + l&15, 4 samples)
template <bool BF>
__device__ __forceinline__ h4 tr_b(h8 x, h8 sel) {
  return to_h4<BF>(mma32<BF>(x, sel, f4{0.0f, 0.0f, 0.0f, 0.0f}));
}


// REF (reference numerics, f16 only): the gradient scale is tcnn's fixed loss scale
// (a.loss_scale = 128) instead of the per-wavefront power of two, the ReLU masks test the
// f16-rounded outputs, and the gradients that cross tinycudann module boundaries in the
// reference are rounded as they are there: dL/dpos_out[1:16] comes back from dir_mlp /
// dir_encoder as f16(f16(g_scaled) / 128) (a subnormal-flushing f16 division) and is
// rescaled for pos_mlp, and dL/denc is written as f16(f16(g_scaled) / 128)
// (tinycudann/modules.py: input_grad / loss_scale, cast to the f16 input's dtype).
// REF 2 (anr_ingp_field_bwd_ref16_rows): the same arithmetic, dL/denc written as f16 (its
// values are f16 numbers already, so the rows hold them exactly) plus one bit per row, set
// when any of the row's 32 values is nonzero (a.row_nz, one 32-bit word per 32-row tile)
// REF 4 (the pos pass of anr_ingp_field_bwd_ref16_rows with a workspace): REF 2 on the
// tiles whose dL/dcolor is zero in every row -- the pos network only, so the dir network's
// registers, dW accumulators and LDS sums are not part of the kernel and more waves fit a
// SIMD -- while a tile with a nonzero dL/dcolor is appended to a.tile_list (a.tile_count)
// and left alone. REF 3 (the list pass, launched after it): REF 2 on exactly the listed
// tiles (count read on the device), the whole network.
template <int W, int NHD, bool FAST, bool ROWS, bool BF, int REF = 0>
__global__ void __launch_bounds__(256) bwd_rt_kernel(Args a, float target, int64_t tpw,
                                                     const float* wmax) {
  static_assert(!(REF && BF), "reference numerics are f16");
  static_assert(REF < 3 || FAST, "the pos / list passes use the fast d_color layout");
  constexpr bool RMASK = REF >= 2;
  constexpr bool POS = REF == 4;  // no dir network in this kernel
  // MT 16-sample halves per tile, the dW contraction over NP pairs of them. (64-sample
  // tiles, MT = 4, measured 6 % slower at the same 1 wave/SIMD: profiles/r03_field_bwd_ab.log)
  constexpr int MT = 2, TR = 16 * MT, NP = MT / 2;
  using N = Net<W, NHD>;
  constexpr int NT = N::NT, KB = N::KB;
  if constexpr (REF == 3) {
    // the list pass: a block none of whose waves has a listed tile leaves before its
    // prologue (weights into LDS, sums zeroed): in the settled state the list is empty and
    // the whole launch was ~26 us of prologues (rocprof r06_c). Block-uniform exit.
    const uint32_t cnt = static_cast<uint32_t>(
        __builtin_amdgcn_readfirstlane(static_cast<int>(*a.tile_count)));
    if (static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) >= cnt) return;
  }
  __shared__ __attribute__((aligned(16))) _Float16 wsm[N::n_packed];
  // the block's dW partials (pos parameters, then dir), summed here before the one global
  // flush per block
  __shared__ float red[POS ? N::NPOS : N::NPOS + N::NDIR];
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int waves = blockDim.x >> 6, wave = threadIdx.x >> 6;
  for (int e = threadIdx.x * 8; e < N::n_packed; e += blockDim.x * 8)
    *reinterpret_cast<h8*>(wsm + e) = *reinterpret_cast<const h8*>(a.packed + e);
  constexpr int NRED = POS ? N::NPOS : N::NPOS + N::NDIR;
  for (int e = threadIdx.x; e < NRED; e += blockDim.x) red[e] = 0.0f;
  __syncthreads();
  // per-tile opaque copy of the fragment base: the weight fragments are re-read from LDS
  // each tile instead of being hoisted into registers
  const _Float16* wbt = wsm;
  auto bfrag32 = [&](int off) { return *reinterpret_cast<const h8*>(wbt + off + lane * 8); };
  auto bfrag16 = [&](int off) { return *reinterpret_cast<const h4*>(wbt + off + lane * 4); };
  TrConst<BF> tc;
  tc.init(lane);
  // dW operand transposes (MFMA against the constant 0/1 operands); the slot argument
  // names the r03 LDS image of the removed LT generation and is unused
  auto trc = [&](int, h4 x) -> h4 { return tr_c<BF>(x, tc.id); };
  auto trb = [&](int, h8 x, h4& o0, h4& o1) {
    o0 = tr_b<BF>(x, tc.sel[0]);
    o1 = tr_b<BF>(x, tc.sel[1]);
  };
  constexpr int R0 = 0, R1 = 16;

  const int64_t n_tiles = (a.M + TR - 1) / TR;
  const int64_t w_id = static_cast<int64_t>(blockIdx.x) * waves + wave;
  const int64_t t_begin = w_id * tpw;
  const int64_t t_end = t_begin + tpw < n_tiles ? t_begin + tpw : n_tiles;
  const int64_t n_full = a.M / TR;

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
  float s = 1.0f, inv_s = 1.0f;
  if constexpr (REF) {
    s = a.loss_scale;
    inv_s = 1.0f / a.loss_scale;
  } else if constexpr (!BF) {
    const float gm = wave_grad_max(a, wmax, w_id, t_begin, t_end);
    if (gm > 0.0f) {
      int e = static_cast<int>(floorf(log2f(target / gm)));
      e = e < -60 ? -60 : (e > 100 ? 100 : e);
      s = ldexpf(1.0f, e);
      inv_s = ldexpf(1.0f, -e);
    }
  }
  // f32 -> f16 -> f32 (the reference's f16 tensors between modules)
  auto r16 = [](float v) { return static_cast<float>(static_cast<_Float16>(v)); };
  // input-gradient products (REF: subnormal part of the gradient operand split off, see
  // split_sub); dx32 accumulates the K blocks of one product into (acc, accs), dx_join
  // adds the two partial sums
  constexpr bool SPLIT = REF && ANR_REF_SPLIT;
  auto dx16 = [&](h4 w, h4 gg) -> f4 {
    if constexpr (SPLIT) {
      h4 gn, gs;
      split_sub(gg, gn, gs);
      return mma16<BF>(w, gn, z4) + mma16<BF>(w, gs, z4) * 0x1p-10f;
    } else {
      return mma16<BF>(w, gg, z4);
    }
  };
  auto dx32 = [&](h8 w, h4 g0, h4 g1, f4& acc, f4& accs) {
    if constexpr (SPLIT) {
      h4 n0, s0, n1, s1;
      split_sub(g0, n0, s0);
      split_sub(g1, n1, s1);
      acc = mma32<BF>(w, cat(n0, n1), acc);
      accs = mma32<BF>(w, cat(s0, s1), accs);
    } else {
      acc = mma32<BF>(w, cat(g0, g1), acc);
    }
  };
  auto dx_join = [&](f4 (&acc)[MT], const f4 (&accs)[MT]) {
    if constexpr (SPLIT) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] += accs[mt] * 0x1p-10f;
    }
  };

  Rows cur[MT];
  // the next tile's raw inputs, loaded a tile ahead into alternating register sets (the
  // full-tile loop runs two tiles per trip): with one set, the loop-carried copy of the
  // prefetch registers lands wherever the register allocator puts it, and where that is
  // early in the tile it waits on the loads just issued (1 wave/SIMD: nothing hides it)
  RawRows nr0[MT], nr1[MT];
  const int64_t t_full_end = t_end < n_full ? t_end : n_full;
  if constexpr (FAST) {
    if (t_begin < t_full_end) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) load_raw<ROWS>(a, t_begin * TR + mt * 16 + li, g, nr0[mt]);
      // drained once, so the loop entry carries no pending loads: entered with the first
      // prefetch in flight, the waitcnt pass merges that state with the back edge's (the
      // prefetch, then the tile's d_enc stores) into a wait for everything, stores
      // included, at the head of every tile
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
  }
  // FAST full tiles hand their dL/denc rows to the NEXT tile's head, which stores them
  // between its input conversion and its prefetch. Stored at the tile's end, they were the
  // newest entries of the in-order vmcnt queue when the next head waited for its
  // prefetched inputs, so every tile head also waited for the previous tile's store acks
  // (vmcnt(0) a few instructions after the stores). The first head stores zeros to its own
  // rows (rewritten by that tile's real values later, same wave, same addresses).
  f4 pend[2][MT];
  int64_t pend_tile = t_begin;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pend[kt][mt] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  // one lane's 4 values of dL/denc row `row`, columns 16 kt + 4 g .. + 3
  auto put = [&](int64_t row, int kt, const f4& v) {
    if constexpr (RMASK) {
      const h4 hv = {static_cast<_Float16>(v[0]), static_cast<_Float16>(v[1]),
                     static_cast<_Float16>(v[2]), static_cast<_Float16>(v[3])};
      *reinterpret_cast<h4*>(a.d_enc_h + row * a.d_enc_stride + 16 * kt + 4 * g) = hv;
    } else {
      *reinterpret_cast<f4*>(a.d_enc + row * a.d_enc_stride + 16 * kt + 4 * g) = v;
    }
  };
  // RMASK: the tile's row bits from each lane's "my 8 values of row (mt, li) are not all
  // zero" (uniform control flow: the ballots need every lane); rows of a row's four lanes
  // g = 0..3 sit at ballot bits li + 16 g
  auto put_mask = [&](int64_t tile, const bool (&nz)[MT]) {
    if constexpr (RMASK) {
      uint32_t word = 0;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint64_t b = __ballot(nz[mt]);
        const uint32_t r = static_cast<uint32_t>((b | (b >> 16) | (b >> 32) | (b >> 48)) & 0xFFFFull);
        word |= r << (16 * mt);
      }
      if (lane == 0) a.row_nz[tile] = word;
    }
  };
  auto nz_of = [](const f4& v0, const f4& v1) {
    return v0[0] != 0.0f || v0[1] != 0.0f || v0[2] != 0.0f || v0[3] != 0.0f || v1[0] != 0.0f ||
           v1[1] != 0.0f || v1[2] != 0.0f || v1[3] != 0.0f;
  };
  auto store_pend = [&]() {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) put(pend_tile * TR + mt * 16 + li, kt, pend[kt][mt]);
    if constexpr (RMASK) {
      bool nz[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) nz[mt] = nz_of(pend[0][mt], pend[1][mt]);
      put_mask(pend_tile, nz);
    }
  };
  auto process = [&](auto full_c, int64_t tile, RawRows(&nraw)[MT], RawRows(&nnext)[MT]) {
    constexpr bool FULL = decltype(full_c)::value;
    {
      int zoff = 0;
      asm volatile("" : "+v"(zoff));
      wbt = wsm + zoff;
    }
    if constexpr (FAST && FULL) {
      // the tile's head: this tile's prefetched inputs are converted here (hoisted into the
      // previous tile, the conversion waits on loads just issued) and the next tile's loads
      // are issued here (the scheduler otherwise sinks them toward the tile's end)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // ordered (volatile) uses of the prefetched registers: without them the select /
        // remap of raw_to_rows floats up to the loads in the previous tile. The scalars
        // are copied by a real v_mov, not an empty tied asm: the remap's packed FMA wants
        // (d1, d2) in an aligned pair, and a tied operand would move that copy up to the
        // dwordx3 load (where it waits for it)
        RawRows rr = nraw[mt];
        asm volatile("v_mov_b32 %0, %1" : "=v"(rr.d0) : "v"(nraw[mt].d0));
        asm volatile("v_mov_b32 %0, %1" : "=v"(rr.d1) : "v"(nraw[mt].d1));
        asm volatile("v_mov_b32 %0, %1" : "=v"(rr.d2) : "v"(nraw[mt].d2));
        asm volatile("v_mov_b32 %0, %1" : "=v"(rr.ds) : "v"(nraw[mt].ds));
        asm volatile("" : "+v"(rr.dc));
        raw_to_rows(rr, g, cur[mt]);
      }
      store_pend();
      const int64_t tn = tile + 1 < t_full_end ? tile + 1 : tile;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) load_raw<ROWS>(a, tn * TR + mt * 16 + li, g, nnext[mt]);
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) load_rows<ROWS>(a, tile * TR + mt * 16 + li, g, true, cur[mt]);
    }
    const bool full = FULL;
    {
      // A tile whose incoming gradients (dL/dcolor, dL/dsigma) are zero in every row adds
      // exactly nothing to dW and has dL/denc = 0: store the zeros, skip the recompute and
      // the backward (wave-uniform). Under the reference numerics tcnn's x128 f16 backward
      // leaves most tiles so once training settles (profiles/r05_state160.log); the build
      // numerics' f32 gradients almost never are, and pay one test per tile.
      bool nz = false;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        nz = nz || cur[mt].ds != 0.0f || cur[mt].dc[0] != 0.0f || cur[mt].dc[1] != 0.0f ||
             cur[mt].dc[2] != 0.0f || cur[mt].dc[3] != 0.0f;
      const bool walk = __any(nz);
      if (a.tile_nz && lane == 0) a.tile_nz[tile] = walk ? 1 : 0;
      if (!walk) {
        const f4 zero4 = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (FAST && FULL) {
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) pend[kt][mt] = zero4;
          pend_tile = tile;
          return;
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int64_t row = tile * TR + mt * 16 + li;
          if (full || row < a.M) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) put(row, kt, zero4);
          }
        }
        if constexpr (RMASK) {
          bool nz[MT];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) nz[mt] = false;
          put_mask(tile, nz);
        }
        return;
      }
    }
    // A tile whose dL/dcolor is zero in every row (reference numerics: every tile once
    // training settles -- tcnn's f16 composite backward rounds the per-sample colour
    // gradients of the atmosphere's tiny weights to zero, profiles/r05_hash_bwd_state_tiles
    // .log): the dir network's backward adds exactly 0 to its dW and returns dX = 0, so
    // neither it nor the dir half of the forward recompute runs (wave-uniform); dL/dpos_out
    // is then dL/dsigma alone. Exact for finite weights and activations (0 * x = 0).
    // Reference numerics, fast d_color layout only: the build numerics' f32 colour
    // gradients are never all zero, and the branch costs their kernel registers (spills);
    // in the general-layout kernel the branch's register copies read dW accumulators right
    // behind their inline-asm MFMAs (tools/mfma_hazards.py)
    bool dir_walk = true;
    if constexpr (REF && FAST) {
      bool cnz = false;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        cnz = cnz || cur[mt].dc[0] != 0.0f || cur[mt].dc[1] != 0.0f || cur[mt].dc[2] != 0.0f ||
              cur[mt].dc[3] != 0.0f;
      dir_walk = __any(cnz);
    }
    if constexpr (POS) {
      if (dir_walk) {  // the list pass takes this tile (d_enc rows and bits included)
        if (lane == 0) a.tile_list[atomicAdd(a.tile_count, 1u)] = static_cast<int32_t>(tile);
        return;
      }
    }
    // ---- forward recompute of both 16-sample halves; every activation stays in registers
    Tile<W, NHD> t[MT];
    h4 gc[MT];
    bool dens[MT];
    {
      bool valid[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) valid[mt] = full || tile * TR + mt * 16 + li < a.M;
      FwdWeights<W, NHD> fwl;
      fwl.load(wbt, lane, !POS && dir_walk);
      tile_forward<W, NHD, MT, BF>(fwl, cur, valid, g, t, NoSink{}, !POS && dir_walk);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        dens[mt] = (REF ? r16(t[mt].po[0]) : t[mt].po[0]) > 0.0f;
        f4 gv;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          gv[i] = (REF ? r16(t[mt].col[i]) : t[mt].col[i]) > 0.0f ? cur[mt].dc[i] * s : 0.0f;
        gc[mt] = to_h4<BF>(gv);
      }
    }
    h4 dpo[MT];
    if (!POS && dir_walk) {
      auto last = [&](int mt, int kt) -> h4 { return NHD == 2 ? t[mt].hd1[kt] : t[mt].hd0[kt]; };
      // ---- dir output layer: dW_D2 (16 x W) += gc^T · X_last ; dX_last = D2^T gc
      // Each layer's W^T fragments are read from LDS at the start of the layer and pinned
      // there (sched_barrier): the dW half of the layer, which needs no weights, then covers
      // the LDS latency that a read placed at its use exposes (1 wave/SIMD).
      h4 dl[MT][NT];
      {
        h4 wd2[NT];
  #pragma unroll
        for (int kt = 0; kt < NT; ++kt) wd2[kt] = bfrag16(N::oBD2 + kt * N::F16);
        __builtin_amdgcn_sched_barrier(0);
        h8 ga[NP];
  #pragma unroll
        for (int pr = 0; pr < NP; ++pr)
          ga[pr] = cat(trc(R0 + 0, gc[2 * pr]), trc(R0 + 1, gc[2 * pr + 1]));
  #pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
  #pragma unroll
          for (int pr = 0; pr < NP; ++pr) {
            const h8 xl = cat(trc(R0 + 2 + 2 * kt, last(2 * pr, kt)), trc(R0 + 3 + 2 * kt, last(2 * pr + 1, kt)));
            mma32_acc_v<BF>(dD2[kt], ga[pr], xl);
          }
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) dl[mt][kt] = mask_h4<BF>(dx16(wd2[kt], gc[mt]), last(mt, kt));
        }
      }
      // ---- dir hidden layer 1 (NHD == 2): dW_D1 (W x W) += dl^T · X_d0 ; dh0 = D1^T dl
      h4 dh0[MT][NT];
      if constexpr (NHD == 2) {
        h8 wd1[NT * KB];
  #pragma unroll
        for (int i = 0; i < NT * KB; ++i) wd1[i] = bfrag32(N::oBD1 + i * N::F32);
        __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          h8 gb[NT];
  #pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            gb[nt] = cat(trc(R1 + 2 * nt, dl[2 * pr][nt]), trc(R1 + 1 + 2 * nt, dl[2 * pr + 1][nt]));
  #pragma unroll
          for (int kt = 0; kt < NT; ++kt) {
            const h8 xb = cat(trc(R1 + 8 + 2 * kt, t[2 * pr].hd0[kt]), trc(R1 + 9 + 2 * kt, t[2 * pr + 1].hd0[kt]));
  #pragma unroll
            for (int nt = 0; nt < NT; ++nt) mma32_acc_v<BF>(dD1[nt * NT + kt], gb[nt], xb);
          }
        }
  #pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
          f4 acc[MT], accs[MT];
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] = accs[mt] = z4;
  #pragma unroll
          for (int kb = 0; kb < KB; ++kb) {
  #pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              dx32(wd1[kt * KB + kb], dl[mt][2 * kb], dl[mt][2 * kb + 1], acc[mt], accs[mt]);
          }
          dx_join(acc, accs);
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) dh0[mt][kt] = mask_h4<BF>(acc[mt], t[mt].hd0[kt]);
        }
      } else {
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int kt = 0; kt < NT; ++kt) dh0[mt][kt] = dl[mt][kt];
      }
      // ---- dir input layer: dW_D0 (W x 32, k' order) += dh0^T · X_de ; dpos = D0^T dh0
      {
        h8 wd0[KB];
  #pragma unroll
        for (int kb = 0; kb < KB; ++kb) wd0[kb] = bfrag32(N::oBD0 + kb * N::F32);
        __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          h4 a0, a1, b0, b1;
          trb(R0 + 0, t[2 * pr].xd, a0, a1);
          trb(R0 + 2, t[2 * pr + 1].xd, b0, b1);
          const h8 x0 = cat(a0, b0), x1 = cat(a1, b1);
  #pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const h8 gd = cat(trc(R0 + 4 + 2 * nt, dh0[2 * pr][nt]), trc(R0 + 5 + 2 * nt, dh0[2 * pr + 1][nt]));
            mma32_acc_v<BF>(dD0[nt * 2], gd, x0);
            mma32_acc_v<BF>(dD0[nt * 2 + 1], gd, x1);
          }
        }
        f4 acc[MT], accs[MT];
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = accs[mt] = z4;
  #pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) dx32(wd0[kb], dh0[mt][2 * kb], dh0[mt][2 * kb + 1], acc[mt], accs[mt]);
        }
        dx_join(acc, accs);
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if constexpr (REF) {
  #pragma unroll
            for (int i = 0; i < 4; ++i) acc[mt][i] = r16(r16(r16(acc[mt][i]) * inv_s) * s);
          }
          // pos_out[:, 0] is the density: its gradient is dL/dsigma through the ReLU
          const float dsv = dens[mt] ? cur[mt].ds * s : 0.0f;
          acc[mt][0] = g == 0 ? dsv : acc[mt][0];
          dpo[mt] = to_h4<BF>(acc[mt]);
        }
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f4 acc = z4;
        acc[0] = g == 0 && dens[mt] ? cur[mt].ds * s : 0.0f;
        dpo[mt] = to_h4<BF>(acc);
      }
    }
    // ---- pos output layer: dW_P1 (16 x W) += dpo^T · X_ph ; dhp = P1^T dpo
    h4 dhp[MT][NT];
    {
      h4 wp1[NT];
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) wp1[kt] = bfrag16(N::oBP1 + kt * N::F16);
      __builtin_amdgcn_sched_barrier(0);
      h8 ga[NP];
#pragma unroll
      for (int pr = 0; pr < NP; ++pr)
        ga[pr] = cat(trc(R1 + 0, dpo[2 * pr]), trc(R1 + 1, dpo[2 * pr + 1]));
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          const h8 xp = cat(trc(R1 + 2 + 2 * kt, t[2 * pr].hp[kt]), trc(R1 + 3 + 2 * kt, t[2 * pr + 1].hp[kt]));
          mma32_acc_v<BF>(dP1[kt], ga[pr], xp);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) dhp[mt][kt] = mask_h4<BF>(dx16(wp1[kt], dpo[mt]), t[mt].hp[kt]);
      }
    }
    // ---- pos input layer: dW_P0 (W x 32) += dhp^T · X_pe ; d_enc = P0^T dhp
    {
      h8 wp0[2 * KB];
#pragma unroll
      for (int i = 0; i < 2 * KB; ++i) wp0[i] = bfrag32(N::oBP0 + i * N::F32);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pr = 0; pr < NP; ++pr) {
        h4 a0, a1, b0, b1;
        trb(R0 + 0, t[2 * pr].xe, a0, a1);
        trb(R0 + 2, t[2 * pr + 1].xe, b0, b1);
        const h8 x0 = cat(a0, b0), x1 = cat(a1, b1);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const h8 gp = cat(trc(R0 + 4 + 2 * nt, dhp[2 * pr][nt]), trc(R0 + 5 + 2 * nt, dhp[2 * pr + 1][nt]));
          mma32_acc_v<BF>(dP0[nt * 2], gp, x0);
          mma32_acc_v<BF>(dP0[nt * 2 + 1], gp, x1);
        }
      }
      // RMASK outside the pend path: the tile's rows, kept until both column halves are out
      f4 keep[RMASK && !(FAST && FULL) ? 2 : 1][MT];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f4 acc[MT], accs[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = accs[mt] = z4;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            dx32(wp0[kt * KB + kb], dhp[mt][2 * kb], dhp[mt][2 * kb + 1], acc[mt], accs[mt]);
        }
        dx_join(acc, accs);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int64_t row = tile * TR + mt * 16 + li;
          f4 v = acc[mt] * inv_s;
          if constexpr (REF) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = r16(r16(acc[mt][i]) * inv_s);
          }
          if constexpr (RMASK && !(FAST && FULL)) keep[kt][mt] = (full || row < a.M) ? v : z4;
          if (full || row < a.M) {
            if constexpr (FAST && FULL)
              pend[kt][mt] = v;
            else
              put(row, kt, v);
          }
        }
      }
      if constexpr (FAST && FULL) pend_tile = tile;
      if constexpr (RMASK && !(FAST && FULL)) {
        bool nz[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) nz[mt] = nz_of(keep[0][mt], keep[1][mt]);
        put_mask(tile, nz);
      }
    }
    // the last dW MFMAs of the tile have written their accumulators before anything
    // (a loop-exit copy) reads them
    agpr_fence();
    if constexpr (!POS) {
      agpr_pin(dD2);
      agpr_pin(dD1);
      agpr_pin(dD0);
    }
    agpr_pin(dP1);
    agpr_pin(dP0);
  };
  if constexpr (REF == 3) {
    // the listed tiles, strided over the grid's wavefronts (the general per-tile path: a
    // listed tile's neighbours are not this wave's)
    const int64_t nw = static_cast<int64_t>(gridDim.x) * waves;
    const int64_t cnt = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(
        static_cast<int>(*a.tile_count)));
    for (int64_t i = w_id; i < cnt; i += nw)
      process(std::integral_constant<bool, false>{},
              static_cast<int64_t>(__builtin_amdgcn_readfirstlane(a.tile_list[i])), nr0, nr1);
  } else {
    {
      const std::integral_constant<bool, true> full_tile;
      int64_t tile = t_begin;
      for (; tile + 1 < t_full_end; tile += 2) {
        process(full_tile, tile, nr0, nr1);
        process(full_tile, tile + 1, nr1, nr0);
      }
      if (tile < t_full_end) process(full_tile, tile, nr0, nr1);
      if constexpr (FAST) {
        if (t_begin < t_full_end) store_pend();
      }
    }
    for (int64_t tile = t_full_end > t_begin ? t_full_end : t_begin; tile < t_end; ++tile)
      process(std::integral_constant<bool, false>{}, tile, nr0, nr1);
  }

  agpr_fence();
  if constexpr (!POS) {
    agpr_pin(dD2);
    agpr_pin(dD1);
    agpr_pin(dD0);
  }
  agpr_pin(dP1);
  agpr_pin(dP0);
  // dW flush: each wavefront's partials (unscaled by its own gradient scale) go into the
  // block's LDS sums, then the block adds them to the f32 gradients with one coalesced
  // atomic per parameter: a quarter of the r03 memory-side requests (one set per
  // wavefront; ~33 us per launch at 1,024 wavefronts, fixed in M)
  float* const rpos = red;
  float* const rdir = red + N::NPOS;
  auto flush = [&](float* dst, int ld, const f4& d, int n0, int k) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (d[i] != 0.0f) atomicAdd(dst + (n0 + 4 * g + i) * ld + k, d[i] * inv_s);
  };
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    if constexpr (!POS) flush(rdir + N::D2, W, dD2[kt], 0, 16 * kt + li);
    flush(rpos + N::P1, W, dP1[kt], 0, 16 * kt + li);
  }
  if constexpr (NHD == 2 && !POS) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) flush(rdir + N::D1, W, dD1[nt * NT + kt], 16 * nt, 16 * kt + li);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      if constexpr (!POS) flush(rdir + N::D0, 32, dD0[nt * 2 + kt], 16 * nt, dir_col(16 * kt + li));
      flush(rpos + N::P0, 32, dP0[nt * 2 + kt], 16 * nt, 16 * kt + li);
    }
  __syncthreads();
  for (int e = threadIdx.x; e < NRED; e += blockDim.x) {
    const float v = red[e];
    if (v != 0.0f) atomicAdd(e < N::NPOS ? a.g_pos + e : a.g_dir + (e - N::NPOS), v);
  }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
static int g_target_log2 = 6;  // f16 gradient scale: max |dL/dout| of a wavefront -> 2^6
// forward form: 1 = the uniform-tile kernel where the shapes allow (default), 0 = always
// the general kernel; test / A-B hook anr_ingp_field_force_fwd
static int g_fwd_ut = 1;

// Backward launch geometry: one resident wavefront per slot (4 per block), each owning a
// contiguous range of 32-sample tiles. The f16 backward needs one float per wavefront of
// caller-owned workspace for the gradient maxima; bf16 needs none.
struct BwdGeom {
  int64_t blocks, nw, tpw;
};
template <int W, int NHD, bool BF>
static const void* bwd_fn(bool fast) {
  return fast ? reinterpret_cast<const void*>(&bwd_rt_kernel<W, NHD, true, false, BF>)
              : reinterpret_cast<const void*>(&bwd_rt_kernel<W, NHD, false, false, BF>);
}
template <int W, int NHD, bool BF>
static BwdGeom bwd_geom(int64_t M, bool fast) {
  const int waves = 4;
  static int pc[2] = {0, 0};
  int& p = pc[fast ? 1 : 0];
  if (p == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, bwd_fn<W, NHD, BF>(fast), 64 * waves, 0) != hipSuccess || nb < 1) nb = 1;
    p = nb;
  }
  const int64_t tiles = (M + 31) / 32;
  int64_t blocks = (tiles + waves - 1) / waves;
  if (blocks > 256LL * p) blocks = 256LL * p;
  if (blocks < 1) blocks = 1;
  const int64_t nw = blocks * waves;
  return {blocks, nw, (tiles + nw - 1) / nw};
}

// the reference-numerics pos pass (REF 4): its own occupancy (no dir network's registers
// or LDS sums); the list pass (REF 3): one block per CU slot of its occupancy
template <int W, int NHD>
static BwdGeom pos_geom(int64_t M) {
  const int waves = 4;
  static int p = 0;
  if (p == 0) {
    int nb = 0;
    const void* fn = reinterpret_cast<const void*>(&bwd_rt_kernel<W, NHD, true, false, false, 4>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * waves, 0) != hipSuccess || nb < 1) nb = 1;
    p = nb;
  }
  const int64_t tiles = (M + 31) / 32;
  int64_t blocks = (tiles + waves - 1) / waves;
  if (blocks > 256LL * p) blocks = 256LL * p;
  if (blocks < 1) blocks = 1;
  const int64_t nw = blocks * waves;
  return {blocks, nw, (tiles + nw - 1) / nw};
}
template <int W, int NHD>
static int64_t list_blocks() {
  static int p = 0;
  if (p == 0) {
    int nb = 0;
    const void* fn = reinterpret_cast<const void*>(&bwd_rt_kernel<W, NHD, true, false, false, 3>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, 0) != hipSuccess || nb < 1) nb = 1;
    p = nb;
  }
  return 256LL * p;
}

template <int W, int NHD, bool BF>
static int64_t bwd_workspace(int64_t M) {
  if (BF || M <= 0) return 0;
  // the larger wave count of the fast and general d_color layouts, so a workspace sized
  // once serves whichever runs
  int64_t n = 0;
  for (int f = 0; f < 2; ++f) {
    const int64_t w = bwd_geom<W, NHD, BF>(M, f == 1).nw;
    n = w > n ? w : n;
  }
  return static_cast<int64_t>(sizeof(float)) * n;
}

template <int W, int NHD, bool BF>
static int run(int op, const Args& a, float* ws, int64_t ws_bytes, hipStream_t st) {
  using N = Net<W, NHD>;
  const int waves = 4;
  if (op == 1) {
    const int64_t tiles = (a.M + 15) / 16;
    const void* fn = reinterpret_cast<const void*>(&fwd_kernel<W, NHD, false, BF, false>);
    static int pc = 0;
    if (pc == 0) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * waves, 0) != hipSuccess || nb < 1) nb = 1;
      pc = nb;
    }
    int64_t blocks = (tiles + waves - 1) / waves;
    if (blocks > 256LL * pc) blocks = 256LL * pc;
    if (blocks < 1) blocks = 1;
    // the uniform-tile form (see fwd_kernel): dense rows whose 16-row tiles are one ray each,
    // 4 colour outputs in 16-byte aligned rows, byte offsets of the outputs below 2^31
    const bool ut = g_fwd_ut && a.rows == nullptr && a.n_per_ray % 16 == 0 && a.n_out == 4 &&
                    (a.color_stride & 3) == 0 && a.M * a.color_stride * 4 < (int64_t{1} << 31);
#define ANR_FWD_LAUNCH(ROWSV, BSV) \
  hipLaunchKernelGGL((fwd_kernel<W, NHD, ROWSV, BF, BSV>), dim3(blocks), dim3(64 * waves), 0, st, a)
    if (a.rows)
      ANR_FWD_LAUNCH(true, false);
    else if (ut)
      ANR_FWD_LAUNCH(false, true);
    else
      ANR_FWD_LAUNCH(false, false);
#undef ANR_FWD_LAUNCH
    return 0;
  }
  if (op == 3) {
    const int64_t tiles = (a.M + 15) / 16;
    int64_t blocks = (tiles + waves - 1) / waves;
    if (blocks > 256LL * 8) blocks = 256LL * 8;  // 8 blocks (32 waves) per CU, grid-stride
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((density_kernel<W, NHD, BF>), dim3(blocks), dim3(64 * waves), 0, st, a);
    return 0;
  }
  const bool fast = a.n_out == 4 && (a.d_color_stride & 3) == 0 && a.d_sigma != nullptr;
  if (a.loss_scale > 0.0f) {  // reference numerics: the register-transposed kernel, REF
    if constexpr (BF) {
      return 1;
    } else {
      if (a.rows) return 1;
      const BwdGeom gm = bwd_geom<W, NHD, BF>(a.M, fast);
      const dim3 grid(static_cast<unsigned>(gm.blocks)), block(64 * waves);
#define ANR_REF_BWD(FASTV, REFV)                                                             \
  hipLaunchKernelGGL((bwd_rt_kernel<W, NHD, FASTV, false, false, REFV>), grid, block, 0, st, a, \
                     0.0f, gm.tpw, nullptr)
      if (a.d_enc_h && fast && a.tile_list) {
        // the pos pass over every tile (more waves per SIMD: no dir network in it), then the
        // list pass over the tiles it left (nonzero dL/dcolor), at most one per wavefront
        // of a grid of its occupancy
        const BwdGeom pg = pos_geom<W, NHD>(a.M);
        if (hipMemsetAsync(a.tile_count, 0, sizeof(uint32_t), st) != hipSuccess) return 1;
        hipLaunchKernelGGL((bwd_rt_kernel<W, NHD, true, false, false, 4>),
                           dim3(static_cast<unsigned>(pg.blocks)), block, 0, st, a, 0.0f, pg.tpw,
                           nullptr);
        hipLaunchKernelGGL((bwd_rt_kernel<W, NHD, true, false, false, 3>),
                           dim3(static_cast<unsigned>(list_blocks<W, NHD>())), block, 0, st, a,
                           0.0f, int64_t{0}, nullptr);
      } else if (a.d_enc_h) {
        if (fast) ANR_REF_BWD(true, 2);
        else ANR_REF_BWD(false, 2);
      } else {
        if (fast) ANR_REF_BWD(true, 1);
        else ANR_REF_BWD(false, 1);
      }
#undef ANR_REF_BWD
      return 0;
    }
  }
  const size_t lds = static_cast<size_t>(N::n_packed) * 2 + sizeof(float) * (N::NPOS + N::NDIR);
  if (lds > 160 * 1024) return 1;
  const BwdGeom gm = bwd_geom<W, NHD, BF>(a.M, fast);
  if (!BF && (ws == nullptr || ws_bytes < static_cast<int64_t>(sizeof(float)) * gm.nw))
    return 2;
  const float target = ldexpf(1.0f, g_target_log2);
  const dim3 grid(static_cast<unsigned>(gm.blocks)), block(64 * waves);
  if (!BF) {
    if (a.rows)
      hipLaunchKernelGGL(absmax_kernel<true>, dim3(gm.nw), dim3(1024), 0, st, a, gm.tpw * 32, ws);
    else
      hipLaunchKernelGGL(absmax_kernel<false>, dim3(gm.nw), dim3(1024), 0, st, a, gm.tpw * 32, ws);
  }
#define ANR_BWD_LAUNCH(FASTV, ROWSV) \
  hipLaunchKernelGGL((bwd_rt_kernel<W, NHD, FASTV, ROWSV, BF>), grid, block, 0, st, a, target, \
                     gm.tpw, ws)
  if (a.rows) {
    if (fast) ANR_BWD_LAUNCH(true, true); else ANR_BWD_LAUNCH(false, true);
  } else {
    if (fast) ANR_BWD_LAUNCH(true, false); else ANR_BWD_LAUNCH(false, false);
  }
#undef ANR_BWD_LAUNCH
  return 0;
}

template <int W, int NHD>
static void launch_pack(const float* pp, const float* pd, _Float16* out, bool bf, hipStream_t st) {
  using N = Net<W, NHD>;
  const dim3 grid((N::n_packed + 255) / 256);
  if (bf)
    hipLaunchKernelGGL((pack_kernel<W, NHD, true>), grid, dim3(256), 0, st, pp, pd, out);
  else
    hipLaunchKernelGGL((pack_kernel<W, NHD, false>), grid, dim3(256), 0, st, pp, pd, out);
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

// fused hash-grid + field forward: a persistent grid of HF_WAVES-wavefront blocks, as many
// as fit on the chip at once (the occupancy query), each wavefront walking 64-sample
// segments grid-stride
constexpr int HF_WAVES = 8;
// register cap (waves per SIMD) of the fused forward, ANR_HF_OCC = 4 / 5 / 6, and its
// run-leader gathers, ANR_HF_DEDUP = 0 / 1 (A/B hooks)
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static int hf_occ() {
  static const int v = env_int("ANR_HF_OCC", 6);
  return v;
}
static bool hf_dedup() {
  static const bool v = env_int("ANR_HF_DEDUP", 0) != 0;
  return v;
}
template <int W, int NHD, bool BF, int OCC, int DD>
static int launch_hf(const Args& a, const HashArgs& h, hipStream_t st) {
  const void* fn = reinterpret_cast<const void*>(&hf_fwd_kernel<W, NHD, BF, HF_WAVES, OCC, DD>);
  static int pc = 0;
  if (pc == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * HF_WAVES, 0) != hipSuccess || nb < 1) nb = 1;
    pc = nb;
  }
  const int64_t n_super = (a.M + 63) / 64;
  int64_t blocks = (n_super + HF_WAVES - 1) / HF_WAVES;
  if (blocks > 256LL * pc) blocks = 256LL * pc;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((hf_fwd_kernel<W, NHD, BF, HF_WAVES, OCC, DD>), dim3(blocks),
                     dim3(64 * HF_WAVES), 0, st, a, h);
  return 0;
}
template <int W, int NHD, bool BF, int DD>
static int run_hf_dd(const Args& a, const HashArgs& h, hipStream_t st) {
  switch (hf_occ()) {
    case 4: return launch_hf<W, NHD, BF, 4, DD>(a, h, st);
    case 5: return launch_hf<W, NHD, BF, 5, DD>(a, h, st);
    default: return launch_hf<W, NHD, BF, 6, DD>(a, h, st);
  }
}
template <int W, int NHD, bool BF>
static int run_hf(const Args& a, const HashArgs& h, hipStream_t st) {
  return hf_dedup() ? run_hf_dd<W, NHD, BF, HASH_DEDUP>(a, h, st) : run_hf_dd<W, NHD, BF, 0>(a, h, st);
}
template <bool BF>
static int dispatch_hf_t(int v, const Args& a, const HashArgs& h, hipStream_t st) {
  switch (v) {
    case 321: return run_hf<32, 1, BF>(a, h, st);
    case 322: return run_hf<32, 2, BF>(a, h, st);
    case 641: return run_hf<64, 1, BF>(a, h, st);
    case 642: return run_hf<64, 2, BF>(a, h, st);
  }
  return 1;
}

template <bool BF>
static int dispatch_t(int v, int op, const Args& a, float* ws, int64_t ws_bytes, hipStream_t st) {
  switch (v) {
    case 321: return run<32, 1, BF>(op, a, ws, ws_bytes, st);
    case 322: return run<32, 2, BF>(op, a, ws, ws_bytes, st);
    case 641: return run<64, 1, BF>(op, a, ws, ws_bytes, st);
    case 642: return run<64, 2, BF>(op, a, ws, ws_bytes, st);
  }
  return 1;
}
static int dispatch(int v, bool bf, int op, const Args& a, float* ws, int64_t ws_bytes,
                    hipStream_t st) {
  return bf ? dispatch_t<true>(v, op, a, ws, ws_bytes, st)
            : dispatch_t<false>(v, op, a, ws, ws_bytes, st);
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

extern "C" int64_t anr_ingp_field_bwd_workspace_bytes(const anr_mlp_desc* pos,
                                                      const anr_mlp_desc* dir,
                                                      int32_t mma_dtype, int64_t M) {
  if (mma_dtype == ANR_BF16) return 0;
  switch (variant(pos, dir)) {
    case 321: return bwd_workspace<32, 1, false>(M);
    case 322: return bwd_workspace<32, 2, false>(M);
    case 641: return bwd_workspace<64, 1, false>(M);
    case 642: return bwd_workspace<64, 2, false>(M);
  }
  return 0;
}

extern "C" int anr_ingp_field_force_fwd(int32_t mode) {
  const int prev = g_fwd_ut;
  if (mode == 0 || mode == 1) g_fwd_ut = mode;
  return prev;
}

extern "C" int anr_ingp_field_set_grad_scale(int32_t log2_target) {
  const int prev = g_target_log2;
  g_target_log2 = log2_target;
  return prev;
}

static bool mma_ok(int32_t t) { return t == ANR_F16 || t == ANR_BF16; }

// enc_stride >= 32 (multiple of 8): row layout; enc_stride = -P: level-quad planes of P
// f16 elements each (P >= 8 M, multiple of 8), as anr_hashgrid_fwd_planes writes them
static bool set_enc(Args& a, const void* enc, int64_t enc_stride, int64_t M) {
  a.enc = static_cast<const _Float16*>(enc);
  if (enc_stride >= 32 && enc_stride % 8 == 0) {
    a.enc_stride = enc_stride;
    a.enc_gstride = 8;
    return true;
  }
  if (enc_stride < 0 && -enc_stride >= 8 * M && (-enc_stride) % 8 == 0) {
    a.enc_stride = 8;
    a.enc_gstride = -enc_stride;
    return true;
  }
  return false;
}

extern "C" int anr_ingp_field_pack(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                   int32_t mma_dtype, const float* pos_params,
                                   const float* dir_params, void* packed, anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_pack: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(mma_ok(mma_dtype), "anr_ingp_field_pack: mma_dtype must be ANR_F16 or ANR_BF16");
  ANR_CHECK_ARG(pos_params && dir_params && packed, "anr_ingp_field_pack: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  _Float16* out = static_cast<_Float16*>(packed);
  const bool bf = mma_dtype == ANR_BF16;
  switch (v) {
    case 321: launch_pack<32, 1>(pos_params, dir_params, out, bf, st); break;
    case 322: launch_pack<32, 2>(pos_params, dir_params, out, bf, st); break;
    case 641: launch_pack<64, 1>(pos_params, dir_params, out, bf, st); break;
    case 642: launch_pack<64, 2>(pos_params, dir_params, out, bf, st); break;
  }
  ANR_CHECK_LAUNCH("anr_ingp_field_pack");
  return ANR_OK;
}

static int field_fwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                     const void* packed, const void* enc, int64_t enc_stride, const float* dirs,
                     int64_t n_per_ray, int64_t M, const int32_t* rows, float* sigma,
                     float* color, int64_t color_stride, anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_fwd: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(mma_ok(mma_dtype), "anr_ingp_field_fwd: mma_dtype must be ANR_F16 or ANR_BF16");
  ANR_CHECK_ARG(M >= 0 && M < (1LL << 31), "anr_ingp_field_fwd: bad M");
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(packed && enc && dirs && sigma && color, "anr_ingp_field_fwd: null pointer");
  ANR_CHECK_ARG(n_per_ray >= 1 && n_per_ray < (1LL << 31) && color_stride >= dir->n_output,
                "anr_ingp_field_fwd: bad shape/stride");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0,
                "anr_ingp_field_fwd: enc/packed must be 16-byte aligned");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  ANR_CHECK_ARG(set_enc(a, enc, enc_stride, M),
                "anr_ingp_field: bad enc_stride %lld (>= 32, multiple of 8: rows; -P: level-quad "
                "planes of P >= 8 M)", (long long)enc_stride);
  a.dirs = dirs;
  a.n_per_ray = static_cast<uint32_t>(n_per_ray);
  a.M = M;
  a.n_out = dir->n_output;
  a.sigma = sigma;
  a.color = color;
  a.color_stride = color_stride;
  a.rows = rows;
  ANR_CHECK_ARG(dispatch(v, mma_dtype == ANR_BF16, 1, a, nullptr, 0,
                         reinterpret_cast<hipStream_t>(stream)) == 0,
                "anr_ingp_field_fwd: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_field_fwd");
  return ANR_OK;
}

extern "C" int anr_ingp_hash_field_fwd(const anr_hashgrid_desc* grid, const float* x, int64_t M,
                                      const void* table, int32_t table_dtype, void* planes,
                                      int64_t plane_stride, const anr_mlp_desc* pos,
                                      const anr_mlp_desc* dir, int32_t mma_dtype,
                                      const void* packed, const float* dirs, int64_t n_per_ray,
                                      float* sigma, float* color, int64_t color_stride,
                                      anr_stream_t stream) {
  const int v = variant(pos, dir);
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(grid && x && table && planes && packed && dirs && sigma && color,
                "anr_ingp_hash_field_fwd: null pointer");
  if (v == 0 || !mma_ok(mma_dtype) || table_dtype != ANR_F16 || grid->n_dims != 3 ||
      grid->n_features != 2 || grid->n_levels != 16 || dir->n_output != 4 ||
      n_per_ray < 64 || n_per_ray % 64 != 0 || color_stride < 4 || color_stride % 4 != 0) {
    ::anr::set_error("anr_ingp_hash_field_fwd: unsupported configuration (3-D f16 grid of 16 "
                     "levels x 2 features, a supported field pair with 4 colour outputs, "
                     "samples per ray a multiple of 64, colour rows 16-byte aligned)");
    return ANR_E_UNSUPPORTED;
  }
  ANR_CHECK_ARG(M > 0 && plane_stride >= 8 * M && plane_stride % 8 == 0,
                "anr_ingp_hash_field_fwd: bad M / plane_stride (>= 8 M, multiple of 8)");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(planes) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(color) & 15) == 0,
                "anr_ingp_hash_field_fwd: planes / packed / color must be 16-byte aligned");
  ::anr::GridLevels G;
  ANR_CHECK_ARG(::anr::make_levels(grid, &G), "anr_ingp_hash_field_fwd: descriptor not initialised");
  const int64_t lim = int64_t(1) << 31;
  const int64_t t_bytes = static_cast<int64_t>(G.offset[15] + G.size[15]) * 4;
  const int64_t o_bytes = (3 * plane_stride + 8 * M) * 2;
  ANR_CHECK_ARG((M + 64) * 12 < lim && t_bytes < lim && o_bytes < lim && plane_stride * 2 < lim &&
                    M * color_stride * 4 < lim,
                "anr_ingp_hash_field_fwd: byte ranges must stay below 2^31");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  a.dirs = dirs;
  a.n_per_ray = static_cast<uint32_t>(n_per_ray);
  a.M = M;
  a.n_out = dir->n_output;
  a.sigma = sigma;
  a.color = color;
  a.color_stride = color_stride;
  HashArgs h{};
  h.G = G;
  h.x = x;
  h.x_bytes = static_cast<uint32_t>(M * 12);
  h.table = static_cast<const __half*>(table);
  h.table_bytes = static_cast<uint32_t>(t_bytes);
  h.planes = static_cast<_Float16*>(planes);
  h.plane_bytes = static_cast<uint32_t>(plane_stride * 2);
  h.out_bytes = static_cast<uint32_t>(o_bytes);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int rc = mma_dtype == ANR_BF16 ? dispatch_hf_t<true>(v, a, h, st)
                                       : dispatch_hf_t<false>(v, a, h, st);
  ANR_CHECK_ARG(rc == 0, "anr_ingp_hash_field_fwd: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_hash_field_fwd");
  return ANR_OK;
}

static int field_bwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                     const void* packed, const void* enc, int64_t enc_stride, const float* dirs,
                     int64_t n_per_ray, int64_t M, const int32_t* rows, const float* d_sigma,
                     const float* d_color, int64_t d_color_stride, float* d_enc,
                     int64_t d_enc_stride, float* g_pos, float* g_dir, void* workspace,
                     int64_t workspace_bytes, anr_stream_t stream, float loss_scale = 0.0f,
                     uint8_t* tile_nz = nullptr, void* d_enc_h = nullptr,
                     uint32_t* row_nz = nullptr, void* tiles_ws = nullptr) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_bwd: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(loss_scale == 0.0f || (loss_scale > 0.0f && mma_dtype == ANR_F16 && rows == nullptr),
                "anr_ingp_field_bwd: reference numerics need f16 MMA and dense rows");
  ANR_CHECK_ARG(mma_ok(mma_dtype), "anr_ingp_field_bwd: mma_dtype must be ANR_F16 or ANR_BF16");
  ANR_CHECK_ARG(M >= 0 && M < (1LL << 31), "anr_ingp_field_bwd: bad M");
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(packed && enc && dirs && d_color && (d_enc || (d_enc_h && row_nz)) && g_pos && g_dir,
                "anr_ingp_field_bwd: null pointer");
  ANR_CHECK_ARG(d_enc_h == nullptr || loss_scale > 0.0f,
                "anr_ingp_field_bwd: f16 rows and row bits are reference numerics only");
  ANR_CHECK_ARG(n_per_ray >= 1 && n_per_ray < (1LL << 31) && d_color_stride >= dir->n_output &&
                    d_enc_stride >= 32 && d_enc_stride % 4 == 0,
                "anr_ingp_field_bwd: bad shape/stride");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(d_enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(d_enc_h) & 7) == 0,
                "anr_ingp_field_bwd: enc/packed/d_enc must be 16-byte aligned (f16 rows: 8)");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  ANR_CHECK_ARG(set_enc(a, enc, enc_stride, M),
                "anr_ingp_field: bad enc_stride %lld (>= 32, multiple of 8: rows; -P: level-quad "
                "planes of P >= 8 M)", (long long)enc_stride);
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
  a.rows = rows;
  a.loss_scale = loss_scale;
  a.tile_nz = tile_nz;
  a.d_enc_h = static_cast<_Float16*>(d_enc_h);
  a.row_nz = row_nz;
  if (tiles_ws) {  // ref16_rows_workspace_bytes: the count, then one int32 per 32-row tile
    a.tile_count = static_cast<uint32_t*>(tiles_ws);
    a.tile_list = reinterpret_cast<int32_t*>(static_cast<char*>(tiles_ws) + 256);
  }
  const int rc = dispatch(v, mma_dtype == ANR_BF16, 2, a, static_cast<float*>(workspace),
                          workspace_bytes, reinterpret_cast<hipStream_t>(stream));
  ANR_CHECK_ARG(rc != 2,
                "anr_ingp_field_bwd: workspace missing or smaller than "
                "anr_ingp_field_bwd_workspace_bytes()");
  ANR_CHECK_ARG(rc == 0, "anr_ingp_field_bwd: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_field_bwd");
  return ANR_OK;
}

extern "C" int anr_ingp_field_fwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                  int32_t mma_dtype, const void* packed, const void* enc,
                                  int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                                  int64_t M, float* sigma, float* color, int64_t color_stride,
                                  anr_stream_t stream) {
  return field_fwd(pos, dir, mma_dtype, packed, enc, enc_stride, dirs, n_per_ray, M, nullptr,
                   sigma, color, color_stride, stream);
}

extern "C" int anr_ingp_field_density(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                      int32_t mma_dtype, const void* packed, const void* enc,
                                      int64_t enc_stride, int64_t M, float* sigma,
                                      anr_stream_t stream) {
  const int v = variant(pos, dir);
  ANR_CHECK_ARG(v != 0, "anr_ingp_field_density: unsupported pos/dir MLP pair");
  ANR_CHECK_ARG(mma_ok(mma_dtype), "anr_ingp_field_density: mma_dtype must be ANR_F16 or ANR_BF16");
  ANR_CHECK_ARG(M >= 0 && M < (1LL << 31), "anr_ingp_field_density: bad M");
  if (M == 0) return ANR_OK;
  ANR_CHECK_ARG(packed && enc && sigma, "anr_ingp_field_density: null pointer");

  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(enc) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(packed) & 15) == 0,
                "anr_ingp_field_density: enc/packed must be 16-byte aligned");
  Args a{};
  a.packed = static_cast<const _Float16*>(packed);
  ANR_CHECK_ARG(set_enc(a, enc, enc_stride, M), "anr_ingp_field_density: bad enc_stride");
  a.M = M;
  a.sigma = sigma;
  ANR_CHECK_ARG(dispatch(v, mma_dtype == ANR_BF16, 3, a, nullptr, 0,
                         reinterpret_cast<hipStream_t>(stream)) == 0,
                "anr_ingp_field_density: no kernel for this shape");
  ANR_CHECK_LAUNCH("anr_ingp_field_density");
  return ANR_OK;
}

extern "C" int anr_ingp_field_bwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                  int32_t mma_dtype, const void* packed, const void* enc,
                                  int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                                  int64_t M, const float* d_sigma, const float* d_color,
                                  int64_t d_color_stride, float* d_enc, int64_t d_enc_stride,
                                  float* g_pos, float* g_dir, void* workspace,
                                  int64_t workspace_bytes, anr_stream_t stream) {
  return field_bwd(pos, dir, mma_dtype, packed, enc, enc_stride, dirs, n_per_ray, M, nullptr,
                   d_sigma, d_color, d_color_stride, d_enc, d_enc_stride, g_pos, g_dir,
                   workspace, workspace_bytes, stream);
}

extern "C" int anr_ingp_field_bwd_ref16(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                        const void* packed, const void* enc, int64_t enc_stride,
                                        const float* dirs, int64_t n_per_ray, int64_t M,
                                        const float* d_sigma, const float* d_color,
                                        int64_t d_color_stride, float* d_enc,
                                        int64_t d_enc_stride, float* g_pos, float* g_dir,
                                        float loss_scale, anr_stream_t stream) {
  ANR_CHECK_ARG(loss_scale > 0.0f, "anr_ingp_field_bwd_ref16: loss_scale must be > 0");
  return field_bwd(pos, dir, ANR_F16, packed, enc, enc_stride, dirs, n_per_ray, M, nullptr,
                   d_sigma, d_color, d_color_stride, d_enc, d_enc_stride, g_pos, g_dir, nullptr,
                   0, stream, loss_scale);
}

extern "C" int anr_ingp_field_bwd_ref16_tiles(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                              const void* packed, const void* enc,
                                              int64_t enc_stride, const float* dirs,
                                              int64_t n_per_ray, int64_t M, const float* d_sigma,
                                              const float* d_color, int64_t d_color_stride,
                                              float* d_enc, int64_t d_enc_stride, float* g_pos,
                                              float* g_dir, float loss_scale, uint8_t* tile_nz,
                                              anr_stream_t stream) {
  ANR_CHECK_ARG(loss_scale > 0.0f, "anr_ingp_field_bwd_ref16_tiles: loss_scale must be > 0");
  ANR_CHECK_ARG(tile_nz != nullptr, "anr_ingp_field_bwd_ref16_tiles: null tile_nz");
  return field_bwd(pos, dir, ANR_F16, packed, enc, enc_stride, dirs, n_per_ray, M, nullptr,
                   d_sigma, d_color, d_color_stride, d_enc, d_enc_stride, g_pos, g_dir, nullptr,
                   0, stream, loss_scale, tile_nz);
}

extern "C" int64_t anr_ingp_field_bwd_ref16_rows_workspace_bytes(int64_t M) {
  return M <= 0 ? 0 : 256 + 4 * ((M + 31) / 32);
}

extern "C" int anr_ingp_field_bwd_ref16_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                             const void* packed, const void* enc,
                                             int64_t enc_stride, const float* dirs,
                                             int64_t n_per_ray, int64_t M, const float* d_sigma,
                                             const float* d_color, int64_t d_color_stride,
                                             void* d_enc_h, int64_t d_enc_stride, float* g_pos,
                                             float* g_dir, float loss_scale, uint32_t* row_nz,
                                             void* workspace, int64_t workspace_bytes,
                                             anr_stream_t stream) {
  ANR_CHECK_ARG(loss_scale > 0.0f, "anr_ingp_field_bwd_ref16_rows: loss_scale must be > 0");
  ANR_CHECK_ARG(d_enc_h != nullptr && row_nz != nullptr,
                "anr_ingp_field_bwd_ref16_rows: null d_enc / row_nz");
  ANR_CHECK_ARG(workspace == nullptr ||
                    workspace_bytes >= anr_ingp_field_bwd_ref16_rows_workspace_bytes(M),
                "anr_ingp_field_bwd_ref16_rows: workspace smaller than "
                "anr_ingp_field_bwd_ref16_rows_workspace_bytes()");
  ANR_CHECK_ARG((reinterpret_cast<uintptr_t>(workspace) & 255) == 0,
                "anr_ingp_field_bwd_ref16_rows: workspace must be 256-byte aligned");
  return field_bwd(pos, dir, ANR_F16, packed, enc, enc_stride, dirs, n_per_ray, M, nullptr,
                   d_sigma, d_color, d_color_stride, nullptr, d_enc_stride, g_pos, g_dir, nullptr,
                   0, stream, loss_scale, nullptr, d_enc_h, row_nz, workspace);
}

extern "C" int anr_ingp_field_fwd_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                       int32_t mma_dtype, const void* packed, const void* enc,
                                       int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                                       int64_t M, const int32_t* rows, float* sigma,
                                       float* color, int64_t color_stride,
                                       anr_stream_t stream) {
  ANR_CHECK_ARG(rows || M == 0, "anr_ingp_field_fwd_rows: null rows");
  return field_fwd(pos, dir, mma_dtype, packed, enc, enc_stride, dirs, n_per_ray, M, rows,
                   sigma, color, color_stride, stream);
}

extern "C" int anr_ingp_field_bwd_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                       int32_t mma_dtype, const void* packed, const void* enc,
                                       int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                                       int64_t M, const int32_t* rows, const float* d_sigma,
                                       const float* d_color, int64_t d_color_stride,
                                       float* d_enc, int64_t d_enc_stride, float* g_pos,
                                       float* g_dir, void* workspace, int64_t workspace_bytes,
                                       anr_stream_t stream) {
  ANR_CHECK_ARG(rows || M == 0, "anr_ingp_field_bwd_rows: null rows");
  return field_bwd(pos, dir, mma_dtype, packed, enc, enc_stride, dirs, n_per_ray, M, rows,
                   d_sigma, d_color, d_color_stride, d_enc, d_enc_stride, g_pos, g_dir,
                   workspace, workspace_bytes, stream);
}

#ifdef FIELD_STAMP
extern "C" int anr_debug_field_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(anr::field::g_stamp), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -1;
}
#endif
