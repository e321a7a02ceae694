// AtmoNeRF dense layers on the f32 matrix cores (configs/nerf.json, BASELINE configs[1];
// SURVEY §8 a15): the forward, input-gradient and weight-gradient GEMMs of
// /root/reference/src/atmonr/models/nerf.py:33-93 (eleven nn.Linear layers, ReLU, the
// fc6 skip concat, fc10's direction concat) with their element-wise work folded in:
//
//   anr_nerf_linear_fwd  Y = [A1 | A2] W^T + b, ReLU optional. The two column segments are
//                        the skip / direction concats (torch.cat + nn.Linear in the
//                        reference), read in place.
//   anr_nerf_linear_dx   dX = G W as [dX1 | dX2], dX1 zeroed where the saved layer input
//                        is <= 0. That is the ReLU backward of the layer that produced the
//                        input (torch's threshold_backward, exact), so G of the layer below
//                        comes out of the GEMM epilogue. dX2 may accumulate, for the fc6
//                        skip input that fc1 also reads.
//   anr_nerf_linear_dw   dW += G^T [A1 | A2], db += column sums of G. M is split over blocks
//                        into f32 partials, which a second pass sums in a fixed order, so the
//                        result is deterministic.
//
// v_mfma_f32_16x16x4_f32: lane l holds A[l&15][l>>4], B[l>>4][l&15] and
// C[4(l>>4)+r][l&15]. The contraction index of lane group g at sub-step t is 4g + t, so
// every lane reads four consecutive contraction elements with one 16-B load. That is the
// same order for both operands, and the contraction is blind to it. All operands are
// row-major f32 with 16-B-aligned rows (leading dimensions and segment widths multiples of
// 4; the host checks).
#include "anr_common.h"

namespace anr {
namespace nerfmlp {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// The GEMM loops accumulate in AGPRs (as tuned library kernels do) through inline asm: the
// builtin lets the compiler keep the accumulators in VGPRs. "s_nop 1" covers the VALU
// write -> MFMA read wait states of operands a zeroing select just wrote (the compiler
// pads nothing inside an asm statement); the accumulators are read back only after
// acc_fence() + acc_pin(), which cover the result latency (40 cycles for this shape).
#ifndef NERF_AGPR
#define NERF_AGPR 1
#endif
__device__ __forceinline__ void mfma4_acc(f4& acc, float a, float b) {
#if NERF_AGPR
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
#else
  acc = mfma4(a, b, acc);
#endif
}
__device__ __forceinline__ void acc_fence() {
#if NERF_AGPR
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
}
template <int N, int K>
__device__ __forceinline__ void acc_pin(f4 (&acc)[N][K]) {
#if NERF_AGPR
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < K; ++j) asm volatile("" : "+a"(acc[i][j]));
#endif
}

// ---------------------------------------------------------------------------------
// C (M x P) = A (M x Q, two column segments) . B^T (B: P x Q), fused epilogue
// ---------------------------------------------------------------------------------
struct NtArgs {
  const float* a1;
  const float* a2;
  int64_t lda1, lda2;
  int32_t q1, q2;          // A's segment widths; Q = q1 + q2 (q2 > 0: q1 % 16 == 0)
  const float* b;          // P x Q, row stride ldb
  int64_t ldb;
  int64_t M;               // rows of this launch (A below 2^31 bytes: 32-bit offsets)
  int32_t P, p1;           // output columns; [0, p1) -> c1, [p1, P) -> c2 (p1 % 4 == 0)
  float* c1;
  float* c2;
  int64_t ldc1, ldc2;
  const float* bias;       // P, or null
  uint64_t* bits;          // forward: ReLU bitmask out (M x ceil(P / 64) words), or null
  const uint64_t* mbits;   // input gradient: zero c1 where the bit is clear, or null
  int32_t wpr;             // bitmask words per row
  int32_t relu, acc2;
};

typedef uint32_t u4v __attribute__((vector_size(16)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes),
                                           0x00020000);
}
__device__ __forceinline__ f4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return f4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
            __uint_as_float(v[3])};
}
constexpr uint32_t kOob = 0x80000000u;  // past every num_records: the load returns zeros

// WR x WC waves per block, each owning (16 TI) x (16 TJ) output tiles (TI x TJ MFMA
// tiles), walking row tiles rt0, rt0 + stride, ... (persistent: the operand stream runs
// on across tiles, so a tile's epilogue overlaps the next tile's first loads and a wave
// pays its start-up latency once). The MFMA takes B as its A operand, so a lane's
// accumulator holds four consecutive COLUMNS of one row (lane c, group g: row 16i + c,
// columns 16j + 4g .. +3): the epilogue stores 16 B per lane. The main loop issues
// nothing but the TI + TJ buffer loads and the 4 TI TJ MFMAs of a k-step: lane offsets
// are fixed per tile (rows past M / columns past P are clamped onto real data, whose
// results are never stored), the k offset rides in the scalar offset, and only a
// segment's last, partial k-step zeroes lanes (B's, so the product vanishes whatever A
// holds there). Two operand stages alternate by unrolling the k loop by 2. The ReLU mask
// of the input-gradient epilogue is one bit per element, written by the forward (32x less
// than re-reading the f32 activations) and loaded a k-step before the tile ends.
template <int WR, int WC, int TI, int TJ, int WPE, int NSTG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
nt_kernel(NtArgs a) {
  constexpr int RT = 16 * TI, CT = 16 * TJ;
  constexpr int NW = (CT + 63) / 64;  // bitmask words a wave tile's row spans
  // the wave index through readfirstlane: the tile indices, the tile loop and its branches
  // are then scalar (a per-lane `more` made the loads after it waterfall loops)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int c = lane & 15, g = lane >> 4;
  // the bias, read by the epilogue, in LDS (zeros past P)
  __shared__ float sbias[16 * TJ * WC];
  const int cb0 = blockIdx.y * WC * CT;
  for (int e = threadIdx.x; e < 16 * TJ * WC; e += 256)
    sbias[e] = a.bias && cb0 + e < a.P ? a.bias[cb0 + e] : 0.0f;
  __syncthreads();
  const int cb = (blockIdx.y * WC + wave % WC) * CT;
  const int n_rt = static_cast<int>((a.M + RT - 1) / RT);
  const int rt0 = blockIdx.x * WR + wave / WC;
  const int rts = gridDim.x * WR;
  if (rt0 >= n_rt || cb >= a.P) return;  // wave-uniform: no barrier below
  const int s1steps = (a.q1 + 15) / 16;
  // an even k-step count (a padding step reads B as zeros): the two operand stages
  // alternate with no register copy at the tile seam
  const int nsteps = (s1steps + (a.q2 + 15) / 16 + 1) & ~1;
  const int Mi = static_cast<int>(a.M);

  // each descriptor ends where its operand's last row does: a segment that starts inside
  // a row (a view) must not reach past the allocation
  const auto ra1 = rsrc(a.a1, ((a.M - 1) * a.lda1 + a.q1) * 4);
  const auto ra2 = rsrc(a.a2, ((a.M - 1) * a.lda2 + (a.q2 ? a.q2 : a.q1)) * 4);
  const auto rbm = rsrc(a.b, (static_cast<int64_t>(a.P - 1) * a.ldb + a.q1 + a.q2) * 4);
  const uint32_t lda1b = static_cast<uint32_t>(a.lda1) * 4, lda2b = static_cast<uint32_t>(a.lda2) * 4;
  const uint32_t ldbb = static_cast<uint32_t>(a.ldb) * 4;
  uint32_t ob[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = min(cb + 16 * j + c, a.P - 1);
    ob[j] = static_cast<uint32_t>(col) * ldbb + 16 * g;
  }

  struct Offs {
    uint32_t a1[TI], a2[TI];
  };
  auto offsets = [&](int rt, Offs& o) {
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const uint32_t row = static_cast<uint32_t>(min(rt * RT + 16 * i + c, Mi - 1));
      o.a1[i] = row * lda1b + 16 * g;
      o.a2[i] = row * lda2b + 16 * g;
    }
  };
  struct Stage {
    f4 av[TI], bv[TJ];
  };
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  auto load = [&](const Offs& o, int s, Stage& st, bool zero_partial = true) {
    const bool seg1 = s < s1steps;
    const int kl = seg1 ? 16 * s : 16 * (s - s1steps);
    const uint32_t sa = static_cast<uint32_t>(kl) * 4;
    const uint32_t sb = static_cast<uint32_t>(seg1 ? kl : a.q1 + kl) * 4;
    const int qs = seg1 ? a.q1 : a.q2;
    if (seg1) {
#pragma unroll
      for (int i = 0; i < TI; ++i) st.av[i] = bload4(ra1, o.a1[i], sa);
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) st.av[i] = bload4(ra2, o.a2[i], sa);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) st.bv[j] = bload4(rbm, ob[j], sb);
    if (zero_partial && kl + 16 > qs) {  // the segment's partial last k-step (uniform)
      const bool ok = kl + 4 * g < qs;
#pragma unroll
      for (int j = 0; j < TJ; ++j) st.bv[j] = ok ? st.bv[j] : z4;
    }
  };

  f4 acc[TI][TJ];
  auto mma = [&](const Stage& st) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma4_acc(acc[i][j], st.bv[j][t], st.av[i][t]);
  };

  // epilogue of row tile rt: lane holds row RT rt + 16i + c, columns cb + 16j + 4g .. +3;
  // a column group that starts below P is stored whole (zeros past P: ldc >= round_up(P, 4))
  // bitmask layout (private to the forward / input-gradient pair): in the 64-bit word of
  // columns 64w .. 64w + 63, column 64w + 16j + 4g + r is bit 16g + 4j + r, so lane group
  // g's 16 bits of a word are one contiguous u16
  auto emit = [&](int row, int col, f4 v, uint32_t mnib) -> uint32_t {
    if (row >= Mi || col >= a.P) return 0u;
    const f4 bv = *reinterpret_cast<const f4*>(sbias + (col - cb0));
    v += bv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (a.relu) v[r] = v[r] > 0.0f ? v[r] : 0.0f;
      if (col + r >= a.P) v[r] = 0.0f;
    }
    if (col < a.p1) {
      if (a.mbits) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (mnib >> r) & 1u ? v[r] : 0.0f;
      }
      *reinterpret_cast<f4*>(a.c1 + static_cast<int64_t>(row) * a.ldc1 + col) = v;
    } else {
      f4* dst = reinterpret_cast<f4*>(a.c2 + static_cast<int64_t>(row) * a.ldc2 + (col - a.p1));
      if (a.acc2) v += *dst;
      *dst = v;
    }
    uint32_t nib = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) nib |= (v[r] > 0.0f ? 1u : 0u) << r;
    return nib;
  };
  // this lane's mask bits of the tile: row 16i + c, words cb/64 + w, the u16 of group g
  uint16_t mw[TI][NW];
  const uint16_t* mb16 = reinterpret_cast<const uint16_t*>(a.mbits);
  auto load_mask = [&](int rt) {
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = rt * RT + 16 * i + c;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const int wd = cb / 64 + w;
        mw[i][w] = a.mbits && row < Mi && wd < a.wpr
                       ? mb16[(static_cast<int64_t>(row) * a.wpr + wd) * 4 + g] : 0xFFFFu;
      }
    }
  };
  auto epilogue = [&](int rt) {
    const int rowb = rt * RT;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = rowb + 16 * i + c;
      uint64_t word[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) word[w] = 0;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = cb + 16 * j + 4 * g;
        const int w = (16 * j) / 64, jw = j & 3;
        const uint32_t nib = emit(row, col, acc[i][j], (mw[i][w] >> (4 * jw)) & 0xFu);
        word[w] |= static_cast<uint64_t>(nib) << (16 * g + 4 * jw);
      }
      if (a.bits) {  // the four lane groups' nibbles of the row -> 64-bit words
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          uint32_t lo = static_cast<uint32_t>(word[w]), hi = static_cast<uint32_t>(word[w] >> 32);
          lo |= __shfl_xor(lo, 16, 64);
          hi |= __shfl_xor(hi, 16, 64);
          lo |= __shfl_xor(lo, 32, 64);
          hi |= __shfl_xor(hi, 32, 64);
          const int wd = cb / 64 + w;
          if (g == 0 && row < Mi && wd < a.wpr)
            a.bits[static_cast<int64_t>(row) * a.wpr + wd] = (static_cast<uint64_t>(hi) << 32) | lo;
        }
      }
    }
  };

  Offs ocur;
  offsets(rt0, ocur);
  if constexpr (NSTG == 3) {
    // Three operand stages, loads two k-steps ahead (the SQ counters of the two-stage
    // loop still had its waves in s_waitcnt 27 % of their cycles: one k-step, 2 x 2,048
    // MFMA cycles per SIMD, did not cover the operand latency). The k loop runs in steps
    // of three; the padding steps (up to two) issue their loads but skip their MFMAs
    // (wave-uniform branches around MFMAs only, so the load counts stay path-independent).
    // Step indices past the tile's last are the next tile's (its row offsets, onext; the
    // last tile re-reads its own, unused).
    const int ns = s1steps + (a.q2 + 15) / 16;
    const int nst = (ns + 2) / 3 * 3;
    Offs onext;
    auto ldx = [&](int j, Stage& st) {
      const bool cur = j < nst;
      Offs o;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        o.a1[i] = cur ? ocur.a1[i] : onext.a1[i];
        o.a2[i] = cur ? ocur.a2[i] : onext.a2[i];
      }
      load(o, cur ? j : j - nst, st, false);
    };
    // k-step j of this tile: a padding step issues no MFMAs; a segment's partial last step
    // zeroes B's lanes past the segment here, at its use (at load time that select waited
    // for the loads just issued)
    auto mmz = [&](int j, Stage& st) {
      if (j >= ns) return;
      const bool seg1 = j < s1steps;
      const int kl = seg1 ? 16 * j : 16 * (j - s1steps);
      const int qs = seg1 ? a.q1 : a.q2;
      if (kl + 16 > qs) {
        const bool ok = kl + 4 * g < qs;
#pragma unroll
        for (int jj = 0; jj < TJ; ++jj) st.bv[jj] = ok ? st.bv[jj] : z4;
      }
      mma(st);
    };
    Stage A, B, C;
    load(ocur, 0, A, false);
    load(ocur, 1, B, false);
    for (int rt = rt0; rt < n_rt; rt += rts) {
      const bool more = rt + rts < n_rt;
      offsets(more ? rt + rts : rt, onext);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = z4;
      // invariant: A holds k-step s, B step s + 1
      for (int s = 0; s < nst; s += 3) {
        ldx(s + 2, C);
        if (s + 3 == nst) load_mask(rt);
        mmz(s, A);
        ldx(s + 3, A);
        mmz(s + 1, B);
        ldx(s + 4, B);
        mmz(s + 2, C);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        ocur.a1[i] = onext.a1[i];
        ocur.a2[i] = onext.a2[i];
      }
      acc_fence();
      acc_pin(acc);
      epilogue(rt);
    }
    return;
  }
  Stage A, B;
  load(ocur, 0, A);
  for (int rt = rt0; rt < n_rt; rt += rts) {
    const bool more = rt + rts < n_rt;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = z4;
    // invariant: A holds k-step s of this tile. Every path issues the A loads, the last
    // tile's final step included (it re-reads step 0 of its own tile, unused): the waitcnt
    // pass merges the paths into the smallest outstanding count, so one path without them
    // made mma(B) wait for the A loads just issued on every step (an exposed memory
    // latency per k-step pair)
    for (int s = 0; s < nsteps; s += 2) {
      load(ocur, s + 1, B);
      if (s + 2 == nsteps) load_mask(rt);
      mma(A);
      int sn = s + 2;
      if (sn == nsteps) {
        sn = 0;
        if (more) offsets(rt + rts, ocur);
      }
      load(ocur, sn, A);
      mma(B);
    }
    acc_fence();
    acc_pin(acc);
    epilogue(rt);
  }
}

// ---------------------------------------------------------------------------------
// dW partials: part[s] (Np x Kp) = G[rows of s]^T . X[rows of s], dbpart[s] (Np) = column
// sums of G over the same rows. Block = 4 waves over one 64 (n) x 64 (k) tile, each wave a
// quarter of the block's rows; the n and k of a tile are interleaved (tile element (rho,
// gamma) of MFMA tile (i, j) is n = nb + 4 rho + i, k = kb + 4 gamma + j) so that one 16-B
// load of a G row (X row) gives a lane its operand for all four n (k) tiles.
// ---------------------------------------------------------------------------------
struct DwArgs {
  const float* g;
  int64_t ldg;
  int32_t Nr;              // G's columns rounded up to 4 (the pad columns are zero)
  const float* a1;
  const float* a2;
  int64_t lda1, lda2;
  int32_t q1, q2;
  int64_t M, rows_per_block;  // rows_per_block: a multiple of 64
  float* part;
  float* dbpart;
  int32_t Np, Kp;          // padded partial tile extents (multiples of 64)
};

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
dw_kernel(DwArgs a) {
  __shared__ __attribute__((aligned(16))) float red[64 * 64];
  __shared__ float dbred[64];
  // a scalar wave index: the row range, and so every load's scalar offset, is then scalar
  // (per lane, each buffer load compiled to a waterfall loop)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int c = lane & 15, g = lane >> 4;
  const int nb = blockIdx.x * 64, kb = blockIdx.y * 64;
  const int s = blockIdx.z;
  const int K = a.q1 + a.q2;
  const int64_t wrows = a.rows_per_block / 4;
  const int64_t m_begin = s * a.rows_per_block + wave * wrows;
  int64_t m_end = m_begin + wrows;
  m_end = m_end < a.M ? m_end : a.M;

  // buffer loads: the lane's offsets within a row are fixed, the row advance rides in the
  // scalar offset, and the descriptors end at this wave's last row (rows past it read
  // zeros). Columns past the operand's width read real data of the same arrays, whose
  // results (partial rows n >= N, columns k >= K) are never summed.
  const int n4 = nb + 4 * c, k4 = kb + 4 * c;
  const bool seg1 = kb < a.q1;  // host: q1 % 64 == 0 when q2 > 0, so uniform per block
  const float* xb = seg1 ? a.a1 : a.a2;
  const uint32_t ldx4 = static_cast<uint32_t>(seg1 ? a.lda1 : a.lda2) * 4;
  const uint32_t ldg4 = static_cast<uint32_t>(a.ldg) * 4;
  const int xcol = seg1 ? k4 : k4 - a.q1;
  // the descriptors end at the wave's last row, at its last column of the operand
  const auto rg = rsrc(a.g, ((m_end - 1) * a.ldg + a.Nr) * 4);
  const auto rx = rsrc(xb, ((m_end - 1) * (seg1 ? a.lda1 : a.lda2) + (seg1 ? a.q1 : a.q2)) * 4);
  uint32_t vg[4], vx[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    vg[t] = static_cast<uint32_t>(4 * g + t) * ldg4 + static_cast<uint32_t>(n4) * 4;
    vx[t] = static_cast<uint32_t>(4 * g + t) * ldx4 + static_cast<uint32_t>(xcol) * 4;
  }
  const bool do_db = blockIdx.y == 0;
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = z4;
  f4 dbacc = z4;

  struct Stage {
    f4 gv[4], xv[4];
  };
  auto load = [&](int64_t m0, Stage& st) {
    const uint32_t sg = static_cast<uint32_t>(m0) * ldg4, sx = static_cast<uint32_t>(m0) * ldx4;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st.gv[t] = bload4(rg, vg[t], sg);
      st.xv[t] = bload4(rx, vx[t], sx);
    }
  };
  auto mma = [&](const Stage& st) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(st.gv[t][i], st.xv[t][j], acc[i][j]);
      if (do_db) dbacc += st.gv[t];
    }
  };
  if (m_begin < m_end) {
    // an even number of 16-row steps (a padding step past m_end reads zeros)
    const int nst = (static_cast<int>((m_end - m_begin + 15) / 16) + 1) & ~1;
    Stage A, B;
    load(m_begin, A);
    for (int st = 0; st < nst; st += 2) {
      const int64_t m0 = m_begin + 16LL * st;
      // stage order pinned (sched_barrier): with scalar offsets the scheduler otherwise
      // sinks each load to its first MFMA, where it waits for it
      load(m0 + 16, B);
      __builtin_amdgcn_sched_barrier(0);
      mma(A);
      __builtin_amdgcn_sched_barrier(0);
      // the last step's loads read past m_end (zeros, unused): with them every path issues
      // the same loads, and mma(B) waits for B only (see nt_kernel)
      load(m0 + 32, A);
      __builtin_amdgcn_sched_barrier(0);
      mma(B);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  acc_fence();
  acc_pin(acc);
  // the four waves' tiles summed in LDS in wave order (deterministic), then one partial
  // tile per block; acc[i][j][r] is (n = nb + 4(4g + r) + i, k = kb + 4c + j)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = 4 * (4 * g + r) + i;
          f4 v = {acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]};
          f4* dst = reinterpret_cast<f4*>(red + nl * 64 + 4 * c);
          *dst = w == 0 ? v : *dst + v;
        }
      if (do_db) {
        // lanes c of the four lane groups g hold partial sums of n = nb + 4c + i
        f4 v = dbacc;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] += __shfl_xor(v[i], 16, 64);
          v[i] += __shfl_xor(v[i], 32, 64);
        }
        if (g == 0) {
          f4* dst = reinterpret_cast<f4*>(dbred + 4 * c);
          *dst = w == 0 ? v : *dst + v;
        }
      }
    }
    __syncthreads();
  }
  float* out = a.part + static_cast<int64_t>(s) * a.Np * a.Kp;
  for (int e = threadIdx.x; e < 64 * 16; e += 256) {
    const int nl = e >> 4, kq = e & 15;
    *reinterpret_cast<f4*>(out + static_cast<int64_t>(nb + nl) * a.Kp + kb + 4 * kq) =
        *reinterpret_cast<const f4*>(red + nl * 64 + 4 * kq);
  }
  if (do_db && threadIdx.x < 64)
    a.dbpart[static_cast<int64_t>(s) * a.Np + nb + threadIdx.x] = dbred[threadIdx.x];
}

// dw[n][k] += sum_s part[s][n][k] (s in order), db[n] += sum_s dbpart[s][n]
__global__ void __launch_bounds__(256) dw_reduce_kernel(const float* __restrict__ part,
                                                        const float* __restrict__ dbpart,
                                                        int32_t S, int32_t N, int32_t K,
                                                        int32_t Np, int32_t Kp,
                                                        float* __restrict__ dw,
                                                        float* __restrict__ db) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nk = static_cast<int64_t>(N) * K;
  if (e < nk) {
    const int n = static_cast<int>(e / K), k = static_cast<int>(e % K);
    float v = 0.0f;
    for (int s = 0; s < S; ++s) v += part[(static_cast<int64_t>(s) * Np + n) * Kp + k];
    dw[e] += v;
  } else if (db && e < nk + N) {
    const int n = static_cast<int>(e - nk);
    float v = 0.0f;
    for (int s = 0; s < S; ++s) v += dbpart[static_cast<int64_t>(s) * Np + n];
    db[n] += v;
  }
}

// M in chunks whose A operands stay below 2^31 bytes (32-bit buffer offsets); a
// persistent grid walks each chunk's row tiles (64 x 64 wave tiles at two waves per SIMD,
// 1,024 blocks; ANR_NERF_BIG=1: 128 x 128 at one wave per SIMD, 256 blocks, for P = 256)
// Operand stages of the k loop: three (loads two k-steps ahead) unless ANR_NERF_STAGES=2
// (A/B hook). Against two stages on one box: the NeRF step 41.5 -> 40.6 ms, the narrow
// launches gaining most (256 x 260 forward 1.51 -> 1.40 ms: fc9's 4 density columns stream
// A with little MFMA work per load); the 256 x 256 layers, which pay two padding steps per
// tile, are unchanged (profiles/r05_nerf_stages_ab.log).
static int g_nt_stages = getenv("ANR_NERF_STAGES") ? atoi(getenv("ANR_NERF_STAGES")) : 3;
template <int WR, int WC, int TI, int TJ, int WPE>
static void launch_cfg(const NtArgs& a, int64_t blocks_cap, hipStream_t st) {
  const int64_t rows = 16LL * TI * WR;
  const unsigned gy = static_cast<unsigned>(ceil_div(a.P, 16LL * TJ * WC));
  int64_t gx = ceil_div(a.M, rows);
  const int64_t cap = ceil_div(blocks_cap, gy);
  gx = gx < cap ? gx : cap;
  const dim3 grid(static_cast<unsigned>(gx), gy);
  if (g_nt_stages != 2 && WPE == 2)
    nt_kernel<WR, WC, TI, TJ, WPE, 3><<<grid, 256, 0, st>>>(a);
  else
    nt_kernel<WR, WC, TI, TJ, WPE, 2><<<grid, 256, 0, st>>>(a);
}

// ANR_NERF_BIG=1: P = 256 layers on 128 x 128 wave tiles, 256 AGPR accumulators, one wave
// per SIMD (the compiler spills 24 VGPRs of the epilogue's temporaries to scratch). The
// kernels alone measured 3-6 % faster (profiles/r05_nerf_big_tiles.log), the NeRF step
// the same (43.22 vs 43.17 ms), so the spill-free 64 x 64 form stays the default.
static int g_nt_big = getenv("ANR_NERF_BIG") ? atoi(getenv("ANR_NERF_BIG")) : 0;
static void launch_nt(NtArgs a, hipStream_t st) {
  const int64_t ld = a.lda1 > a.lda2 ? a.lda1 : a.lda2;
  const int64_t chunk = ((0x7fffffffLL / (ld * 4)) / 256) * 256;
  const int64_t M = a.M;
  for (int64_t r0 = 0; r0 < M; r0 += chunk) {
    NtArgs b = a;
    b.M = M - r0 < chunk ? M - r0 : chunk;
    b.a1 = a.a1 + r0 * a.lda1;
    b.a2 = a.a2 + r0 * a.lda2;
    b.c1 = a.c1 + r0 * a.ldc1;
    b.c2 = a.c2 + r0 * a.ldc2;
    if (a.bits) b.bits = a.bits + r0 * a.wpr;
    if (a.mbits) b.mbits = a.mbits + r0 * a.wpr;
    if (g_nt_big && a.P == 256) {
      launch_cfg<2, 2, 8, 8, 1>(b, 256, st);
      continue;
    }
    if (a.P <= 128) {
      launch_cfg<2, 2, 4, 4, 2>(b, 1024, st);
      continue;
    }
    // the first 256 columns with four 64-wide column waves per block; columns past 256
    // (fc9's density outputs, fc6's skip input gradient) in a second launch of blocks
    // with two column waves, rather than a second block column that leaves 2-3 of its
    // four waves idle
    NtArgs m = b;
    m.P = a.P < 256 ? a.P : 256;
    m.p1 = a.p1 < m.P ? a.p1 : m.P;
    launch_cfg<1, 4, 4, 4, 2>(m, 1024, st);
    if (a.P > 256) {
      NtArgs t = b;
      t.P = a.P - 256;
      t.b = b.b + 256 * b.ldb;
      if (b.bias) t.bias = b.bias + 256;
      if (a.p1 > 256) {
        t.p1 = a.p1 - 256;
        t.c1 = b.c1 + 256;
        t.c2 = b.c2;
      } else {
        t.p1 = 0;
        t.c1 = b.c2 + (256 - a.p1);
        t.c2 = b.c2 + (256 - a.p1);
        t.ldc1 = b.ldc2;
        t.mbits = nullptr;
      }
      if (b.bits) t.bits = b.bits + 4;
      if (t.mbits) t.mbits = b.mbits + 4;
      launch_cfg<2, 2, 4, 4, 2>(t, 1024, st);
    }
  }
}

struct DwGeom {
  int32_t tn, tk, S;
  int64_t rows_per_block;
};

static DwGeom dw_geom(int64_t M, int32_t N, int32_t K) {
  DwGeom d;
  d.tn = static_cast<int32_t>(ceil_div(N, 64));
  d.tk = static_cast<int32_t>(ceil_div(K, 64));
  // about 2,048 blocks (8 per CU), at least 256 rows per block
  int64_t S = ceil_div(2048, static_cast<int64_t>(d.tn) * d.tk);
  const int64_t smax = ceil_div(M, 256);
  S = S < smax ? S : smax;
  S = S < 1 ? 1 : S;
  d.rows_per_block = ceil_div(ceil_div(M, S), 64) * 64;
  d.S = static_cast<int32_t>(ceil_div(M, d.rows_per_block));
  return d;
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace nerfmlp
}  // namespace anr

using namespace anr;
using namespace anr::nerfmlp;

extern "C" int anr_nerf_linear_fwd(const float* a1, int64_t lda1, int32_t q1, const float* a2,
                                   int64_t lda2, int32_t q2, int64_t M, const float* w,
                                   int32_t n, const float* bias, int32_t relu, float* y,
                                   int64_t ldy, uint64_t* relu_bits, anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && n > 0 && q1 > 0 && q2 >= 0, "anr_nerf_linear_fwd: bad sizes");
  if (M == 0) return ANR_OK;  // empty tensors carry null pointers
  ANR_CHECK_ARG(q1 % 4 == 0 && q2 % 4 == 0 && lda1 % 4 == 0 && (q2 == 0 || lda2 % 4 == 0),
                "anr_nerf_linear_fwd: segment widths and strides must be multiples of 4");
  ANR_CHECK_ARG(lda1 >= q1 && (q2 == 0 || lda2 >= q2) && ldy % 4 == 0 && ldy >= (n + 3) / 4 * 4,
                "anr_nerf_linear_fwd: strides below the widths (ldy: round_up(n, 4))");
  ANR_CHECK_ARG(q2 == 0 || q1 % 16 == 0,
                "anr_nerf_linear_fwd: with a second segment q1 must be a multiple of 16");
  ANR_CHECK_ARG(al16(a1) && (q2 == 0 || al16(a2)) && al16(w) && al16(y) && a1 && w && y,
                "anr_nerf_linear_fwd: operands must be 16-byte aligned");
  NtArgs a{};
  a.a1 = a1;
  a.a2 = q2 ? a2 : a1;
  a.lda1 = lda1;
  a.lda2 = q2 ? lda2 : lda1;
  a.q1 = q1;
  a.q2 = q2;
  a.b = w;
  a.ldb = q1 + q2;
  a.M = M;
  a.P = n;
  a.p1 = n;
  a.c1 = y;
  a.c2 = y;
  a.ldc1 = a.ldc2 = ldy;
  a.bias = bias;
  a.relu = relu;
  a.bits = relu_bits;
  a.wpr = static_cast<int32_t>((n + 63) / 64);
  launch_nt(a, as_stream(stream));
  ANR_CHECK_LAUNCH("anr_nerf_linear_fwd");
  return ANR_OK;
}

extern "C" int anr_nerf_linear_dx(const float* g, int64_t ldg, int64_t M, int32_t n,
                                  const float* wt, int64_t ldwt, int32_t p1, int32_t p2,
                                  const uint64_t* mask_bits, float* dx1, int64_t ldx1,
                                  float* dx2, int64_t ldx2, int32_t acc2,
                                  anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && n > 0 && p1 >= 0 && p2 >= 0 && p1 + p2 > 0,
                "anr_nerf_linear_dx: bad sizes");
  if (M == 0) return ANR_OK;  // empty tensors carry null pointers
  ANR_CHECK_ARG(ldg % 4 == 0 && ldwt % 4 == 0 && ldg >= n && ldwt >= n,
                "anr_nerf_linear_dx: G and W^T row strides must be multiples of 4 >= n");
  ANR_CHECK_ARG(al16(g) && al16(wt) && g && wt && (p1 == 0 || dx1) && (p2 == 0 || dx2),
                "anr_nerf_linear_dx: operands must be 16-byte aligned");
  ANR_CHECK_ARG((p1 == 0 || ldx1 >= p1) && (p2 == 0 || ldx2 >= p2),
                "anr_nerf_linear_dx: strides below the widths");
  ANR_CHECK_ARG(p1 % 4 == 0 && p2 % 4 == 0 && (p1 == 0 || (ldx1 % 4 == 0 && al16(dx1))) &&
                    (p2 == 0 || (ldx2 % 4 == 0 && al16(dx2))),
                "anr_nerf_linear_dx: p1 and p2 must be multiples of 4, the outputs 16-byte "
                "granular");
  // the contraction runs over n rounded up to 4: G's pad columns and W^T's are zero
  NtArgs a{};
  a.a1 = a.a2 = g;
  a.lda1 = a.lda2 = ldg;
  a.q1 = static_cast<int32_t>((n + 3) / 4 * 4);
  a.q2 = 0;
  a.b = wt;
  a.ldb = ldwt;
  a.M = M;
  a.P = p1 + p2;
  a.p1 = p1;
  a.c1 = p1 ? dx1 : dx2;
  a.c2 = p2 ? dx2 : dx1;
  a.ldc1 = p1 ? ldx1 : ldx2;
  a.ldc2 = p2 ? ldx2 : ldx1;
  a.mbits = p1 ? mask_bits : nullptr;
  a.wpr = static_cast<int32_t>((p1 + 63) / 64);
  a.acc2 = acc2;
  ANR_CHECK_ARG(a.q1 <= ldg && a.q1 <= ldwt, "anr_nerf_linear_dx: pad columns missing");
  launch_nt(a, as_stream(stream));
  ANR_CHECK_LAUNCH("anr_nerf_linear_dx");
  return ANR_OK;
}

extern "C" int64_t anr_nerf_linear_dw_workspace(int64_t M, int32_t n, int32_t k) {
  if (M <= 0 || n <= 0 || k <= 0) return 0;
  const DwGeom d = dw_geom(M, n, k);
  const int64_t np = 64LL * d.tn, kp = 64LL * d.tk;
  return static_cast<int64_t>(d.S) * np * (kp + 1) * 4;
}

extern "C" int anr_nerf_linear_dw(const float* g, int64_t ldg, int64_t M, int32_t n,
                                  const float* a1, int64_t lda1, int32_t q1, const float* a2,
                                  int64_t lda2, int32_t q2, float* dw, float* db, void* ws,
                                  int64_t ws_bytes, anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && n > 0 && q1 > 0 && q2 >= 0, "anr_nerf_linear_dw: bad sizes");
  if (M == 0) return ANR_OK;  // empty tensors carry null pointers
  ANR_CHECK_ARG(q2 == 0 || q1 % 64 == 0,
                "anr_nerf_linear_dw: with a second segment q1 must be a multiple of 64");
  ANR_CHECK_ARG(q1 % 4 == 0 && q2 % 4 == 0 && lda1 % 4 == 0 && (q2 == 0 || lda2 % 4 == 0) &&
                    ldg % 4 == 0 && ldg >= (n + 3) / 4 * 4,
                "anr_nerf_linear_dw: widths and strides must be multiples of 4 (G padded)");
  ANR_CHECK_ARG(al16(g) && al16(a1) && (q2 == 0 || al16(a2)) && al16(ws) && dw,
                "anr_nerf_linear_dw: operands must be 16-byte aligned");
  const int32_t K = q1 + q2;
  ANR_CHECK_ARG(ws_bytes >= anr_nerf_linear_dw_workspace(M, n, K),
                "anr_nerf_linear_dw: workspace of %lld bytes < %lld", (long long)ws_bytes,
                (long long)anr_nerf_linear_dw_workspace(M, n, K));
  // rows in chunks whose operands stay below 2^31 bytes (32-bit buffer offsets); every
  // chunk adds its own partial sums into dw / db
  int64_t ldmax = ldg > lda1 ? ldg : lda1;
  if (q2 && lda2 > ldmax) ldmax = lda2;
  const int64_t chunk = ((0x7fffffffLL / (ldmax * 4)) / 64) * 64;
  hipStream_t st = as_stream(stream);
  for (int64_t r0 = 0; r0 < M; r0 += chunk) {
    const int64_t Mc = M - r0 < chunk ? M - r0 : chunk;
    const DwGeom d = dw_geom(Mc, n, K);
    DwArgs a{};
    a.g = g + r0 * ldg;
    a.ldg = ldg;
    a.Nr = (n + 3) / 4 * 4;
    a.a1 = a1 + r0 * lda1;
    a.a2 = q2 ? a2 + r0 * lda2 : a.a1;
    a.lda1 = lda1;
    a.lda2 = q2 ? lda2 : lda1;
    a.q1 = q1;
    a.q2 = q2;
    a.M = Mc;
    a.rows_per_block = d.rows_per_block;
    a.Np = 64 * d.tn;
    a.Kp = 64 * d.tk;
    a.part = static_cast<float*>(ws);
    a.dbpart = a.part + static_cast<int64_t>(d.S) * a.Np * a.Kp;
    dim3 grid(static_cast<unsigned>(d.tn), static_cast<unsigned>(d.tk), static_cast<unsigned>(d.S));
    dw_kernel<<<grid, 256, 0, st>>>(a);
    ANR_CHECK_LAUNCH("anr_nerf_linear_dw");
    const int64_t total = static_cast<int64_t>(n) * K + (db ? n : 0);
    dw_reduce_kernel<<<static_cast<unsigned>(ceil_div(total, 256)), 256, 0, st>>>(
        a.part, a.dbpart, d.S, n, K, a.Np, a.Kp, dw, db);
    ANR_CHECK_LAUNCH("anr_nerf_linear_dw (reduce)");
  }
  return ANR_OK;
}
