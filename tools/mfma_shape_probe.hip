// Probe: FLOP/s and sustained clock of the two f16 MFMA shapes on random operands, at the NCF
// scan's occupancy (3 workgroups of 4 waves per CU, every CU busy).  Per k step a wave forms
// its B operands with one packed add + clamp (like the scan's clamp(P~ + Q~)) and issues the
// same FLOP in either shape: 2 x v_mfma_f32_32x32x16_f16 (two chains) or 4 x
// v_mfma_f32_16x16x32_f16 (four chains).  Question: does the 16x16x32 shape buy clock under
// the power limit (MI355X_MICROARCH.md: ~1.15x FLOP/s in bare bf16 loops)?
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_shape_probe.hip -o tools/bin/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(256, 3) void probe(const h8* __restrict__ in, float* __restrict__ out,
                                                int iters, long long* cyc) {
  const int lane = threadIdx.x & 63;
  h8 a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    a[s] = in[(s * 64 + lane + blockIdx.x * 7) & 4095];
    b[s] = in[(s * 64 + lane + 2048 + blockIdx.x * 13) & 4095];
  }
  const long long t0 = __builtin_readcyclecounter();
  float keep = 0.f;
  if (SHAPE == 0) {
    f32x16 c0 = {}, c1 = {};
    for (int it = 0; it < iters; ++it) {
      const _Float16 d = (_Float16)((it & 7) * 0.0625f);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 x = b[s] + d;
        x = __builtin_elementwise_min(__builtin_elementwise_max(x, (h8){}), (h8)(_Float16)1.f);
        h8 y = b[s] - d;
        y = __builtin_elementwise_min(__builtin_elementwise_max(y, (h8){}), (h8)(_Float16)1.f);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], y, c1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) keep += c0[r] + c1[r];
  } else {
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
      const _Float16 d = (_Float16)((it & 7) * 0.0625f);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 x = b[s] + d;
        x = __builtin_elementwise_min(__builtin_elementwise_max(x, (h8){}), (h8)(_Float16)1.f);
        h8 y = b[s] - d;
        y = __builtin_elementwise_min(__builtin_elementwise_max(y, (h8){}), (h8)(_Float16)1.f);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[s], x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[s], y, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(s + 1) & 3], x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(s + 1) & 3], y, c3, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) keep += c0[r] + c1[r] + c2[r] + c3[r];
  }
  const long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 256 + threadIdx.x] = keep;
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
}

template <int SHAPE>
static void run(const h8* in, float* out, long long* cyc, int blocks, int iters, const char* name) {
  hipLaunchKernelGGL(probe<SHAPE>, dim3(blocks), dim3(256), 0, 0, in, out, iters, cyc);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  long long c = 0;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(probe<SHAPE>, dim3(blocks), dim3(256), 0, 0, in, out, iters, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    }
  }
  // FLOP per wave per iteration: 4 steps x 65536 (2 x 32x32x16 or 4 x 16x16x32)
  const double flop = (double)blocks * 4 * iters * 4 * 65536.0;
  printf("%-10s %8.3f ms  %7.1f TF/s  (block 0: %lld counter ticks)\n", name, best,
         flop / (best * 1e-3) / 1e12, c);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const bool zero = argc > 2 && atoi(argv[2]) == 0;  // all-zero operands: the clock without the power limit
  int cus = 256;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
  const int blocks = 3 * cus;
  _Float16 h[4096 * 8];
  unsigned x = 12345;
  for (int i = 0; i < 4096 * 8; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = zero ? (_Float16)0.f : (_Float16)(((x >> 8) * (1.0f / 16777216.0f)) - 0.5f);
  }
  h8* in;
  float* out;
  long long* cyc;
  (void)hipMalloc(&in, sizeof(h));
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(in, out, cyc, blocks, iters, "32x32x16");
    run<1>(in, out, cyc, blocks, iters, "16x16x32");
  }
  return 0;
}
