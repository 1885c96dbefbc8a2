// Microbenchmark: v_mfma_f32_32x32x2_f32 throughput with N dependent VALU ops feeding the
// B operand of each MFMA (the NCF/W&D inner-loop shape), at 1 and 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NV, int CH>
__global__ __launch_bounds__(256) void probe(float* out, const float* in, int iters) {
  const int lane = threadIdx.x & 63;
  float a = in[lane], x = in[64 + lane], y = in[128 + lane];
  f32x16 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        float b = x + (float)(s + c);
#pragma unroll
        for (int v = 0; v < NV; ++v) b = (v & 1) ? fmaxf(b, y) : b + y;
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NV, int CH>
void run(int blocks_per_cu, const char* name) {
  float *out, *in;
  hipMalloc(&out, 256 * 256 * 8 * 4);
  hipMalloc(&in, 4096);
  hipMemset(in, 0, 4096);
  const int iters = 400;
  const int grid = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<NV, CH>), dim3(grid), dim3(256), 0, 0, out, in, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<NV, CH>), dim3(grid), dim3(256), 0, 0, out, in, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)grid * 4 * iters * 16 * CH;  // per wave: iters*16*CH
  const double tflops = mfmas * 4096 / (ms * 1e-3) / 1e12;
  printf("%-28s NV=%d CH=%d waves/SIMD=%d : %.3f ms  %.1f TF  (%.1f%% of 157.3)\n", name, NV, CH,
         blocks_per_cu, ms, tflops, 100 * tflops / 157.3);
  hipFree(out);
  hipFree(in);
}

int main() {
  run<0, 2>(1, "pure mfma");
  run<0, 2>(2, "pure mfma");
  run<2, 2>(1, "add+max");
  run<2, 2>(2, "add+max");
  run<2, 1>(2, "add+max 1chain");
  run<4, 2>(2, "4 valu");
  run<6, 2>(2, "6 valu");
  run<8, 2>(2, "8 valu");
  run<12, 2>(2, "12 valu");
  run<16, 2>(2, "16 valu");
  run<4, 2>(1, "4 valu");
  run<8, 2>(1, "8 valu");
  return 0;
}
