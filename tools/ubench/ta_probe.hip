// TA cost of a gather wave-instruction by active-lane pattern (r06 probe for the hash-grid
// forward): does the texture addresser spend its cycles per instruction, per active quad or
// per active lane? Each lane gathers ITER random dwords (or dword pairs) from an
// L2-resident table; inactive lanes are masked by EXEC (a divergent branch around the load).
// Build: hipcc -O3 --offload-arch=gfx950 ta_probe.hip -o ta_probe ; run: ./ta_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITER = 256;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// MODE: 0 all lanes, 1 one lane per quad (lane % 4 == 0), 2 lanes 0-15 (4 quads),
// 3 lanes 0-3 (1 quad), 4 all lanes b64 pairs, 5 one lane per quad, quads 0-3 only
template <int MODE>
__global__ void __launch_bounds__(256) probe(const uint32_t* __restrict__ t, uint32_t mask,
                                             uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  bool on;
  if (MODE == 0 || MODE == 4) on = true;
  else if (MODE == 1) on = (lane & 3) == 0;
  else if (MODE == 2) on = lane < 16;
  else if (MODE == 3) on = lane < 4;
  else on = (lane & 3) == 0 && lane < 16;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(t), 0, (mask + 2) * 4, 0x00020000);
  uint32_t s = blockIdx.x * 256 + threadIdx.x, acc = 0;
  for (int i = 0; i < ITER; ++i) {
    s = mix(s + i);
    const uint32_t o = (s & mask) * 4u;
    if (on) {
      if (MODE == 4) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, o & ~7u, 0, 0);
        acc += v[0] ^ v[1];
      } else {
        acc += __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint32_t n = 1u << 19;  // 2 MiB table: L2-resident
  uint32_t *t, *out;
  hipMalloc(&t, (n + 2) * 4);
  hipMalloc(&out, 4);
  hipMemset(t, 1, (n + 2) * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 32;
  const char* names[] = {"all 64 lanes b32", "1 lane per quad (16 quads)", "lanes 0-15 (4 quads)",
                         "lanes 0-3 (1 quad)", "all 64 lanes b64", "1 lane per quad, 4 quads"};
  for (int mode = 0; mode < 6; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      switch (mode) {
        case 0: hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
        case 1: hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
        case 2: hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
        case 3: hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
        case 4: hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
        case 5: hipLaunchKernelGGL(probe<5>, dim3(blocks), dim3(256), 0, 0, t, n - 1, out); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    const double insts = double(blocks) * 4 * ITER;  // wave-instructions
    printf("%-30s %8.3f ms  %6.2f ns/wave-instruction per CU  %5.2f CU-cycles @2.4GHz\n",
           names[mode], best, best * 1e6 / insts * 256, best * 1e6 / insts * 256 * 2.4);
  }
  return 0;
}
