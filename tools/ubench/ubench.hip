// Microbenchmarks that MEASURE the MI355X ceilings the hot-path rooflines are priced
// against: spec sheets are not peaks.
//
//   ub_copy     float4 stream copy            -> HBM GB/s (read + written bytes)
//   ub_read     float4 stream read (reduce)   -> HBM GB/s (read bytes)
//   ub_mfma     back-to-back 16x16x32 f16 / bf16 MFMAs on random operands, every SIMD
//               -> dense TFLOP/s
//   ub_atomic   no-return global_atomic_add_f32 wave-instructions cut into segments of
//               `seg_lanes` consecutive dwords, each segment at an independent random,
//               segment-aligned address of a `n_floats` table -> segment requests/s.
//               seg_lanes = 4 with 16 segments per instruction is the hash-grid
//               backward's shape (hashgrid.hip v2: lane = 4*level + 2*xbit + feature).
//   ub_gather   4-B loads (one f16x2 hash-grid corner, the forward's gather width) at
//               independent random addresses of an `n_words` table, `iters` per lane ->
//               a known count of requested bytes, to calibrate rocprofv3 FETCH_SIZE and
//               the TCC hit rate for this access shape.
//   ub_xcc_map  each workgroup records HW_REG_XCC_ID (spinning for (1 + b % 8) x `spin`
//               clocks first, an imbalanced grid like an XCD-partitioned kernel's) -> the
//               observed workgroup -> XCD placement.
//
// Test/measurement infrastructure, not product: built to tools/ubench/libanr_ubench.so
// by __graft_entry__.build(); bench.py loads it in its untimed phase. Plain C ABI
// (device pointers, sizes, a hipStream_t), int status.

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy_kernel(const float4* __restrict__ src,
                                                   float4* __restrict__ dst, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i + 3 * stride < n; i += 4 * stride) {  // 4 independent loads in flight
    float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

__global__ void __launch_bounds__(256) read_kernel(const float4* __restrict__ src, int64_t n,
                                                   float* __restrict__ sink) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (; i + 3 * stride < n; i += 4 * stride) {
    float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    acc += (a.x + b.y) + (c.z + d.w);
  }
  for (; i < n; i += stride) acc += src[i].x;
  if (acc == 1234.5f) sink[threadIdx.x] = acc;  // never true on the bench data; keeps loads
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // lowbias32 integer hash
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <bool BF16>
__global__ void __launch_bounds__(256) mfma_kernel(int iters, float* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // random operands (zeros would let the chip hold a higher clock: MICROARCH DVFS notes)
  h8 ah, bh;
  b8 ab, bb;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float va = (float)(mix32(t * 16 + j) & 0xffff) * (1.f / 65536.f) - 0.5f;
    float vb = (float)(mix32(t * 16 + 8 + j) & 0xffff) * (1.f / 65536.f) - 0.5f;
    ah[j] = (_Float16)va;
    bh[j] = (_Float16)vb;
    ab[j] = (__bf16)va;
    bb[j] = (__bf16)vb;
  }
  f4 c0 = {0, 0, 0, 0}, c1 = {1, 1, 1, 1}, c2 = {2, 2, 2, 2}, c3 = {3, 3, 3, 3};
  for (int i = 0; i < iters; ++i) {
    if constexpr (BF16) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c3, 0, 0, 0);
    }
  }
  f4 s = c0 + c1 + c2 + c3;
  out[t] = s[0] + s[1] + s[2] + s[3];
}

// f32-input MFMA (v_mfma_f32_16x16x4_f32: 2*16*16*4 FLOP), the NeRF MLP's GEMM precision
__global__ void __launch_bounds__(256) mfma_f32_kernel(int iters, float* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const float a = (float)(mix32(t) & 0xffff) * (1.f / 65536.f) - 0.5f;
  const float b = (float)(mix32(t + 7) & 0xffff) * (1.f / 65536.f) - 0.5f;
  f4 c0 = {0, 0, 0, 0}, c1 = {1, 1, 1, 1}, c2 = {2, 2, 2, 2}, c3 = {3, 3, 3, 3};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  f4 s = c0 + c1 + c2 + c3;
  out[t] = s[0] + s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(256) atomic_kernel(float* __restrict__ table, int64_t n_seg,
                                                     int seg_lanes, int iters, uint32_t seed) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int seg = lane / seg_lanes, j = lane - seg * seg_lanes;
  for (int i = 0; i < iters; ++i) {
    uint32_t h = mix32(seed ^ mix32(wave * 0x9E3779B9U + i * 131u + seg));
    int64_t s = (int64_t)(((uint64_t)h * (uint64_t)n_seg) >> 32);
    __hip_atomic_fetch_add(table + s * seg_lanes + j, 1.0f, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(256) gather_kernel(const uint32_t* __restrict__ table,
                                                     int64_t n_words, int iters, uint32_t seed,
                                                     uint32_t* __restrict__ sink) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < iters; ++i) {
    const uint32_t h = mix32(seed ^ mix32(gid * 0x9E3779B9U + (uint32_t)i * 0x85EBCA6BU));
    const int64_t w = (int64_t)(((uint64_t)h * (uint64_t)n_words) >> 32);
    acc ^= table[w];
  }
  if (acc == 0x12345678u) sink[gid & 255] = acc;  // keeps the loads; never true here
}

__global__ void __launch_bounds__(256) xcc_map_kernel(uint32_t* __restrict__ out, int spin) {
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const long long t0 = clock64();
  const long long until = static_cast<long long>(spin) * (1 + (blockIdx.x & 7));
  while (clock64() - t0 < until) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) out[blockIdx.x] = xcc & 0xFu;
}

// f16 subnormal handling (r04 reference-numerics drift probe): an MFMA operand, a
// conversion and a native f16 multiply of the subnormal 2^-20
typedef _Float16 ub_h8 __attribute__((ext_vector_type(8)));
typedef float ub_f4 __attribute__((ext_vector_type(4)));
__global__ void f16_denorm_kernel(float* out) {
  const int l = threadIdx.x;
  const float tiny = 9.5367431640625e-07f;  // 2^-20: an f16 subnormal
  ub_h8 a = {}, b = {};
  if (l == 0) {
    a[0] = static_cast<_Float16>(tiny);
    b[0] = static_cast<_Float16>(1.0f);
  }
  ub_f4 c = {0.0f, 0.0f, 0.0f, 0.0f};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  volatile float vt = tiny;
  const _Float16 h = static_cast<_Float16>(vt);
  volatile _Float16 one = static_cast<_Float16>(1.0f);
  const _Float16 m = h * one;
  if (l == 0) {
    out[0] = c[0];                        // MFMA: 2^-20 if f16 subnormal inputs are kept
    out[1] = static_cast<float>(h);       // f32 -> f16 -> f32 conversion
    out[2] = static_cast<float>(m);       // native f16 multiply
    out[3] = tiny;
  }
}

// MFMA accumulation precision (r05 PSNR-drift probe): n_mats independent products
// C = A0 B0 + A1 B1 (two chained v_mfma_f32_16x16x32_f16, the field backward's K = 64
// input-gradient shape). Operands in the instruction's register layout: lane l holds
// A[row l % 16][k = 8 (l / 16) .. + 7] and B[k = 8 (l / 16) .. + 7][col l % 16]; C lane l
// row 4 (l / 16) + i, col l % 16. a, b: n_mats * 2 * 64 * 8 halves (lane-linear); c:
// n_mats * 64 * 4 floats.
__global__ void mfma_dot_kernel(const _Float16* __restrict__ a, const _Float16* __restrict__ b,
                                float* __restrict__ c, int n_mats) {
  const int l = threadIdx.x & 63;
  const int mat = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (mat >= n_mats) return;
  ub_f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int kb = 0; kb < 2; ++kb) {
    const int64_t o = ((static_cast<int64_t>(mat) * 2 + kb) * 64 + l) * 8;
    ub_h8 av, bv;
    for (int e = 0; e < 8; ++e) {
      av[e] = a[o + e];
      bv[e] = b[o + e];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) c[(static_cast<int64_t>(mat) * 64 + l) * 4 + i] = acc[i];
}

extern "C" {

int ub_xcc_map(void* out, int blocks, int spin, void* stream) {
  if (blocks <= 0 || spin < 0) return 1;
  xcc_map_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>((uint32_t*)out, spin);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int ub_copy(const void* src, void* dst, int64_t n_float4, int blocks, void* stream) {
  if (n_float4 <= 0 || blocks <= 0) return 1;
  copy_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>((const float4*)src, (float4*)dst,
                                                      n_float4);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int ub_read(const void* src, int64_t n_float4, float* sink, int blocks, void* stream) {
  if (n_float4 <= 0 || blocks <= 0) return 1;
  read_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>((const float4*)src, n_float4, sink);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// kind 0 f16, 1 bf16, 2 f32. out: blocks*256 floats. FLOPs = blocks * 4 waves * iters * 4 *
// (2*16*16*32) for f16/bf16, (2*16*16*4) for f32.
int ub_mfma(int bf16, int iters, int blocks, float* out, void* stream) {
  if (iters <= 0 || blocks <= 0) return 1;
  if (bf16 == 2)
    mfma_f32_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(iters, out);
  else if (bf16)
    mfma_kernel<true><<<blocks, 256, 0, (hipStream_t)stream>>>(iters, out);
  else
    mfma_kernel<false><<<blocks, 256, 0, (hipStream_t)stream>>>(iters, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Segment requests = blocks * 4 waves * iters * (64 / seg_lanes).
int ub_atomic(float* table, int64_t n_floats, int seg_lanes, int iters, int blocks,
              uint32_t seed, void* stream) {
  if (seg_lanes <= 0 || 64 % seg_lanes || n_floats < seg_lanes || iters <= 0 || blocks <= 0)
    return 1;
  atomic_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(table, n_floats / seg_lanes, seg_lanes,
                                                         iters, seed);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Gathers = blocks * 256 * iters, 4 B each.
int ub_gather(const void* table, int64_t n_words, int iters, int blocks, uint32_t seed,
              void* sink, void* stream) {
  if (n_words <= 0 || iters <= 0 || blocks <= 0) return 1;
  gather_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>((const uint32_t*)table, n_words, iters,
                                                         seed, (uint32_t*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int ub_mfma_dot(const void* a, const void* b, float* c, int n_mats, void* stream) {
  if (n_mats <= 0) return 1;
  mfma_dot_kernel<<<(n_mats + 3) / 4, 256, 0, (hipStream_t)stream>>>(
      (const _Float16*)a, (const _Float16*)b, c, n_mats);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int ub_f16_denorm(float* out, void* stream) {
  f16_denorm_kernel<<<1, 64, 0, (hipStream_t)stream>>>(out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
