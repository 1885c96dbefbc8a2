// Probe: FLOP/s and sustained clock of the two f16 MFMA shapes on random operands, at the NCF
// scan's occupancy (3 workgroups of 4 waves per CU, every CU busy).  Per k step a wave forms
// its B operands with one packed add + clamp (the scan's clamp(P~ + Q~), one v_pk_add_f16 with
// the clamp modifier per 2 elements; round 6: pinned by inline asm) and issues the
// same FLOP in either shape: 2 x v_mfma_f32_32x32x16_f16 (two chains) or 4 x
// v_mfma_f32_16x16x32_f16 (four chains).  Question: does the 16x16x32 shape buy clock under
// the power limit (MI355X_MICROARCH.md: ~1.15x FLOP/s in bare bf16 loops)?
// Round 6: SHAPE 2 / 3, the block-scaled e4m3 32x32x64 (bare / with the scan's operand work).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_shape_probe.hip -o tools/bin/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// the scan's operand formation: clamp(P~ + Q~) as ONE v_pk_add_f16 with the clamp modifier per 2
// elements (clamp to [0, 1] = the ReLU on the scaled operands)
__device__ __forceinline__ h8 form(h8 v, int dd) {
  h8 r;
  const int* pv = reinterpret_cast<const int*>(&v);
  int* pr = reinterpret_cast<int*>(&r);
#pragma unroll
  for (int q = 0; q < 4; ++q) asm volatile("v_pk_add_f16 %0, %1, %2 clamp" : "=v"(pr[q]) : "v"(pv[q]), "v"(dd));
  return r;
}

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
      const int dx = (it & 7) * 0x2c002c00, dy = dx ^ 0x80008000;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const h8 x = form(b[s], dx), y = form(b[s], dy);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], y, c1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) keep += c0[r] + c1[r];
  } else if (SHAPE == 2 || SHAPE == 3) {
    // round 6: the block-scaled e4m3 MFMA, v_mfma_scale_f32_32x32x64_f8f6f4 (scale
    // 2^0), two chains, the same FLOP per iteration as the f16 shapes (2 x 32x32x64 = 8 x
    // 32x32x16).  SHAPE 2: fixed operands (the bare rate).  SHAPE 3: each chain's 32 B elements
    // a lane formed as the scan forms them -- packed f16 add + clamp -- then converted to e4m3
    // (v_cvt_scalef32_pk_fp8_f16, 2 elements an instruction): the operand work an e4m3 layer 2
    // of the NCF scan would issue per k = 64.
    i8v ai, bi;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int* pa = reinterpret_cast<const int*>(&a[s]);
      const int* pb = reinterpret_cast<const int*>(&b[s]);
      ai[2 * s] = pa[0] & 0x3f3f3f3f;  // finite e4m3 bytes
      ai[2 * s + 1] = pa[1] & 0x3f3f3f3f;
      bi[2 * s] = pb[0] & 0x3f3f3f3f;
      bi[2 * s + 1] = pb[1] & 0x3f3f3f3f;
    }
    f32x16 c0 = {}, c1 = {};
    for (int it = 0; it < iters; ++it) {
      if (SHAPE == 2) {
        c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ai, bi, c0, 0, 0, 0, 127, 0, 127);
        c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ai, bi, c1, 0, 0, 0, 127, 0, 127);
      } else {
        const int dx = (it & 7) * 0x2c002c00, dy = dx ^ 0x80008000;
        i8v x, y;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const h8 xs = form(b[s], dx), ys = form(b[s], dy);
          const h2* px = reinterpret_cast<const h2*>(&xs);
          const h2* py = reinterpret_cast<const h2*>(&ys);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            // the first convert's untouched half is overwritten by the second: any old value
            s2 rx = __builtin_bit_cast(s2, px[2 * q]), ry = __builtin_bit_cast(s2, py[2 * q]);
            rx = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(rx, px[2 * q], 1.0f, false);
            rx = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(rx, px[2 * q + 1], 1.0f, true);
            ry = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(ry, py[2 * q], 1.0f, false);
            ry = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(ry, py[2 * q + 1], 1.0f, true);
            x[2 * s + q] = *reinterpret_cast<int*>(&rx);
            y[2 * s + q] = *reinterpret_cast<int*>(&ry);
          }
        }
        c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ai, x, c0, 0, 0, 0, 127, 0, 127);
        c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ai, y, c1, 0, 0, 0, 127, 0, 127);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) keep += c0[r] + c1[r];
  } else {
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
      const int dx = (it & 7) * 0x2c002c00, dy = dx ^ 0x80008000;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const h8 x = form(b[s], dx), y = form(b[s], dy);
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
    run<2>(in, out, cyc, blocks, iters, "e4m3 bare");
    run<3>(in, out, cyc, blocks, iters, "e4m3 +ops");
  }
  return 0;
}
