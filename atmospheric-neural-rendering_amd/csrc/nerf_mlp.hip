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

// ---------------------------------------------------------------------------------
// C (M x P) = A (M x Q, two column segments) . B^T (B: P x Q), fused epilogue
// ---------------------------------------------------------------------------------
struct NtArgs {
  const float* a1;
  const float* a2;
  int64_t lda1, lda2;
  int32_t q1, q2;          // A's segment widths; Q = q1 + q2
  const float* b;          // P x Q, row stride ldb
  int64_t ldb;
  int64_t M;
  int32_t P, p1;           // output columns; [0, p1) -> c1, [p1, P) -> c2
  float* c1;
  float* c2;
  int64_t ldc1, ldc2;
  const float* bias;       // P, or null
  const float* mask;       // M x p1 (row stride ldm): zero the output where mask <= 0
  int64_t ldm;
  int32_t relu, acc2;
};

// WR x WC waves per block, each owning a 64 x 64 output tile (4 x 4 MFMA tiles).
template <int WR, int WC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
nt_kernel(NtArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t rb = (static_cast<int64_t>(blockIdx.x) * WR + wave / WC) * 64;
  const int cb = (blockIdx.y * WC + wave % WC) * 64;
  if (rb >= a.M || cb >= a.P) return;  // wave-uniform: no barrier below
  const int Q = a.q1 + a.q2;

  // the rows this lane loads (clamped; their results are not stored)
  const float* ar1[4];
  const float* ar2[4];
  const float* br[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t row = rb + 16 * i + c;
    row = row < a.M ? row : a.M - 1;
    ar1[i] = a.a1 + row * a.lda1;
    ar2[i] = a.a2 + row * a.lda2 - a.q1;
    int col = cb + 16 * i + c;
    col = col < a.P ? col : a.P - 1;
    br[i] = a.b + static_cast<int64_t>(col) * a.ldb;
  }
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  auto load = [&](int k0, f4 (&av)[4], f4 (&bv)[4]) {
    const int kk = k0 + 4 * g;
    const bool ok = kk < Q;
    const bool s1 = kk < a.q1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* pa = s1 ? ar1[i] + kk : ar2[i] + kk;
      av[i] = ok ? *reinterpret_cast<const f4*>(pa) : z4;
      bv[i] = ok ? *reinterpret_cast<const f4*>(br[i] + kk) : z4;
    }
  };

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = z4;

  f4 an[4], bn[4];
  load(0, an, bn);
  for (int k0 = 0; k0 < Q; k0 += 16) {
    f4 ac[4], bc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ac[i] = an[i];
      bc[i] = bn[i];
    }
    if (k0 + 16 < Q) load(k0 + 16, an, bn);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(ac[i][t], bc[j][t], acc[i][j]);
  }

  // epilogue: lane holds rows rb + 16i + 4g + r of column cb + 16j + c
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = cb + 16 * j + c;
    if (col >= a.P) continue;
    const float bias = a.bias ? a.bias[col] : 0.0f;
    const bool seg1 = col < a.p1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = rb + 16 * i + 4 * g + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] + bias;
        if (a.relu) v = v > 0.0f ? v : 0.0f;
        if (seg1) {
          if (a.mask && !(a.mask[row * a.ldm + col] > 0.0f)) v = 0.0f;
          a.c1[row * a.ldc1 + col] = v;
        } else {
          float* dst = a.c2 + row * a.ldc2 + (col - a.p1);
          *dst = a.acc2 ? *dst + v : v;
        }
      }
    }
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int nb = blockIdx.x * 64, kb = blockIdx.y * 64;
  const int s = blockIdx.z;
  const int K = a.q1 + a.q2;
  const int64_t wrows = a.rows_per_block / 4;
  const int64_t m_begin = s * a.rows_per_block + wave * wrows;
  int64_t m_end = m_begin + wrows;
  m_end = m_end < a.M ? m_end : a.M;

  const int n4 = nb + 4 * c, k4 = kb + 4 * c;
  const bool gok = n4 < a.Nr;
  const bool xok = k4 < K;
  const float* gcol = a.g + n4;
  const float* xcol = k4 < a.q1 ? a.a1 + k4 : a.a2 + (k4 - a.q1);
  const int64_t ldx = k4 < a.q1 ? a.lda1 : a.lda2;
  const bool do_db = blockIdx.y == 0;
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = z4;
  f4 dbacc = z4;

  auto load = [&](int64_t m0, f4 (&gv)[4], f4 (&xv)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t m = m0 + 4 * g + t;
      const bool ok = m < m_end;
      gv[t] = ok && gok ? *reinterpret_cast<const f4*>(gcol + m * a.ldg) : z4;
      xv[t] = ok && xok ? *reinterpret_cast<const f4*>(xcol + m * ldx) : z4;
    }
  };
  if (m_begin < m_end) {
    f4 gn[4], xn[4];
    load(m_begin, gn, xn);
    for (int64_t m0 = m_begin; m0 < m_end; m0 += 16) {
      f4 gc[4], xc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        gc[t] = gn[t];
        xc[t] = xn[t];
      }
      if (m0 + 16 < m_end) load(m0 + 16, gn, xn);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(gc[t][i], xc[t][j], acc[i][j]);
        if (do_db) dbacc += gc[t];
      }
    }
  }

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
                                   int64_t ldy, anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && n > 0 && q1 > 0 && q2 >= 0, "anr_nerf_linear_fwd: bad sizes");
  ANR_CHECK_ARG(q1 % 4 == 0 && q2 % 4 == 0 && lda1 % 4 == 0 && (q2 == 0 || lda2 % 4 == 0),
                "anr_nerf_linear_fwd: segment widths and strides must be multiples of 4");
  ANR_CHECK_ARG(lda1 >= q1 && (q2 == 0 || lda2 >= q2) && ldy >= n,
                "anr_nerf_linear_fwd: strides below the widths");
  ANR_CHECK_ARG(al16(a1) && (q2 == 0 || al16(a2)) && al16(w) && a1 && w && y,
                "anr_nerf_linear_fwd: operands must be 16-byte aligned");
  if (M == 0) return ANR_OK;
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
  hipStream_t st = as_stream(stream);
  if (n > 128) {
    dim3 grid(static_cast<unsigned>(ceil_div(M, 64)), static_cast<unsigned>(ceil_div(n, 256)));
    nt_kernel<1, 4><<<grid, 256, 0, st>>>(a);
  } else {
    dim3 grid(static_cast<unsigned>(ceil_div(M, 128)), static_cast<unsigned>(ceil_div(n, 128)));
    nt_kernel<2, 2><<<grid, 256, 0, st>>>(a);
  }
  ANR_CHECK_LAUNCH("anr_nerf_linear_fwd");
  return ANR_OK;
}

extern "C" int anr_nerf_linear_dx(const float* g, int64_t ldg, int64_t M, int32_t n,
                                  const float* wt, int64_t ldwt, int32_t p1, int32_t p2,
                                  const float* mask, int64_t ldm, float* dx1, int64_t ldx1,
                                  float* dx2, int64_t ldx2, int32_t acc2,
                                  anr_stream_t stream) {
  ANR_CHECK_ARG(M >= 0 && n > 0 && p1 >= 0 && p2 >= 0 && p1 + p2 > 0,
                "anr_nerf_linear_dx: bad sizes");
  ANR_CHECK_ARG(ldg % 4 == 0 && ldwt % 4 == 0 && ldg >= n && ldwt >= n,
                "anr_nerf_linear_dx: G and W^T row strides must be multiples of 4 >= n");
  ANR_CHECK_ARG(al16(g) && al16(wt) && g && wt && (p1 == 0 || dx1) && (p2 == 0 || dx2),
                "anr_nerf_linear_dx: operands must be 16-byte aligned");
  ANR_CHECK_ARG((p1 == 0 || ldx1 >= p1) && (p2 == 0 || ldx2 >= p2) && (!mask || ldm >= p1),
                "anr_nerf_linear_dx: strides below the widths");
  if (M == 0) return ANR_OK;
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
  a.mask = mask;
  a.ldm = ldm;
  a.acc2 = acc2;
  ANR_CHECK_ARG(a.q1 <= ldg && a.q1 <= ldwt, "anr_nerf_linear_dx: pad columns missing");
  hipStream_t st = as_stream(stream);
  const int P = p1 + p2;
  if (P > 128) {
    dim3 grid(static_cast<unsigned>(ceil_div(M, 64)), static_cast<unsigned>(ceil_div(P, 256)));
    nt_kernel<1, 4><<<grid, 256, 0, st>>>(a);
  } else {
    dim3 grid(static_cast<unsigned>(ceil_div(M, 128)), static_cast<unsigned>(ceil_div(P, 128)));
    nt_kernel<2, 2><<<grid, 256, 0, st>>>(a);
  }
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
  ANR_CHECK_ARG(q1 % 4 == 0 && q2 % 4 == 0 && lda1 % 4 == 0 && (q2 == 0 || lda2 % 4 == 0) &&
                    ldg % 4 == 0 && ldg >= (n + 3) / 4 * 4,
                "anr_nerf_linear_dw: widths and strides must be multiples of 4 (G padded)");
  ANR_CHECK_ARG(al16(g) && al16(a1) && (q2 == 0 || al16(a2)) && al16(ws) && dw,
                "anr_nerf_linear_dw: operands must be 16-byte aligned");
  if (M == 0) return ANR_OK;
  const int32_t K = q1 + q2;
  const DwGeom d = dw_geom(M, n, K);
  ANR_CHECK_ARG(ws_bytes >= anr_nerf_linear_dw_workspace(M, n, K),
                "anr_nerf_linear_dw: workspace of %lld bytes < %lld", (long long)ws_bytes,
                (long long)anr_nerf_linear_dw_workspace(M, n, K));
  DwArgs a{};
  a.g = g;
  a.ldg = ldg;
  a.Nr = (n + 3) / 4 * 4;
  a.a1 = a1;
  a.a2 = q2 ? a2 : a1;
  a.lda1 = lda1;
  a.lda2 = q2 ? lda2 : lda1;
  a.q1 = q1;
  a.q2 = q2;
  a.M = M;
  a.rows_per_block = d.rows_per_block;
  a.Np = 64 * d.tn;
  a.Kp = 64 * d.tk;
  a.part = static_cast<float*>(ws);
  a.dbpart = a.part + static_cast<int64_t>(d.S) * a.Np * a.Kp;
  hipStream_t st = as_stream(stream);
  dim3 grid(static_cast<unsigned>(d.tn), static_cast<unsigned>(d.tk), static_cast<unsigned>(d.S));
  dw_kernel<<<grid, 256, 0, st>>>(a);
  ANR_CHECK_LAUNCH("anr_nerf_linear_dw");
  const int64_t total = static_cast<int64_t>(n) * K + (db ? n : 0);
  dw_reduce_kernel<<<static_cast<unsigned>(ceil_div(total, 256)), 256, 0, st>>>(
      a.part, a.dbpart, d.S, n, K, a.Np, a.Kp, dw, db);
  ANR_CHECK_LAUNCH("anr_nerf_linear_dw (reduce)");
  return ANR_OK;
}
