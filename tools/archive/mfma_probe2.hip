// Microbenchmark 2: the NCF pair-loop shape in isolation.  Variants:
//  V0: 1 A register, B = max(x + s, 0) (baseline shape of mfma_probe)
//  V1: 32 distinct A registers (W2 fragments), B = max(p + q[s], 0) with q[32] registers
//  V2: V1 + C-init of each chain from a bias register set (first MFMA src C != dst)
//  V3: V2 with an epilogue per pair (16 max + 16 fma on each acc, sum kept live)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0)

template <int V>
__global__ __launch_bounds__(256, 2) void probe(float* out, const float* in, int iters) {
  const int lane = threadIdx.x & 63;
  float a[32], q[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) { a[s] = in[(s * 64 + lane) & 1023]; q[s] = in[(s * 64 + lane + 7) & 1023]; }
  f32x16 bias;
#pragma unroll
  for (int r = 0; r < 16; ++r) bias[r] = in[r + 3];
  float p = in[lane + 5], keep = 0.f;
  f32x16 accA = bias, accB = bias;
  for (int it = 0; it < iters; ++it) {
    if (V >= 2) { accA = bias; accB = bias; }
    const float pa = p + (float)it, pb = p - (float)it;
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const float aa = V == 0 ? a[0] : a[s];
      const float qa = V == 0 ? (float)s : q[s];
      accA = MF(aa, fmaxf(pa + qa, 0.f), accA);
      accB = MF(aa, fmaxf(pb + qa, 0.f), accB);
    }
    if (V >= 3) {
      float m = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaf(fmaxf(accA[r], 0.f), q[r], m);
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaf(fmaxf(accB[r], 0.f), q[r], m);
      keep += m;
    }
  }
  float s = keep;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += accA[r] + accB[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int V>
void run(const char* name) {
  float *out, *in;
  (void)hipMalloc(&out, 256 * 256 * 8 * 4);
  (void)hipMalloc(&in, 8192);
  (void)hipMemset(in, 0, 8192);
  const int iters = 200, grid = 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<V>), dim3(grid), dim3(256), 0, 0, out, in, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((probe<V>), dim3(grid), dim3(256), 0, 0, out, in, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)grid * 4 * iters * 64;
  printf("%-34s %.3f ms  %.1f%% of fp32 MFMA peak\n", name, ms,
         100 * mfmas * 4096 / (ms * 1e-3) / 1e12 / 157.3);
}

int main() {
  run<0>("V0 single A reg");
  run<1>("V1 32 A regs + q regs");
  run<2>("V2 + bias C-init per pair");
  run<3>("V3 + per-pair epilogue");
  return 0;
}
