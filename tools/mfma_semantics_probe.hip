// Probe of MFMA arithmetic semantics the NCF certified pre-filter relies on:
//  (a) v_mfma_f32_32x32x2_f32: is D = fma(a1, b1, fma(a0, b0, c)) bitwise (k = lane half)?
//  (b) v_mfma_f32_32x32x16_f16: are f16 denormal inputs kept (not flushed)?
//  (c) v_mfma_f32_32x32x16_f16: is the accumulation exact-product + fp32 rounding no worse
//      than a sequential fp32 sum (max |err| vs a double reference, in fp32 ulps)?
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_semantics_probe.hip -o build/mfma_sem
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// (a) one 32x32x2 step per launch slot: A[i][k], B[k][j], C[i][j] random
__global__ void f32_step(const float* A, const float* B, const float* C, float* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16 c;
  for (int q = 0; q < 16; ++q) c[q] = C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r];
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * 2 + h], B[h * 32 + r], c, 0, 0, 0);
  for (int q = 0; q < 16; ++q) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = c[q];
}

// (b)/(c) one 32x32x16 f16 MFMA: A[i][k] (32x16), B[k][j] (16x32), C = 0
__global__ void f16_step(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  h8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = A[r * 16 + 8 * h + e];
    b[e] = B[(8 * h + e) * 32 + r];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int q = 0; q < 16; ++q) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = c[q];
}

static float frand() { return (float)rand() / RAND_MAX * 2.f - 1.f; }

int main() {
  srand(1);
  float *A, *B, *C, *D;
  hipMallocManaged(&A, 4096 * 4);
  hipMallocManaged(&B, 4096 * 4);
  hipMallocManaged(&C, 4096 * 4);
  hipMallocManaged(&D, 4096 * 4);
  long m01 = 0, m10 = 0, msum = 0, n = 0;
  for (int trial = 0; trial < 200; ++trial) {
    for (int i = 0; i < 64; ++i) A[i] = frand() * powf(2.f, (float)(rand() % 20 - 10));
    for (int i = 0; i < 64; ++i) B[i] = frand() * powf(2.f, (float)(rand() % 20 - 10));
    for (int i = 0; i < 1024; ++i) C[i] = frand() * powf(2.f, (float)(rand() % 20 - 10));
    hipLaunchKernelGGL(f32_step, dim3(1), dim3(64), 0, 0, A, B, C, D);
    hipDeviceSynchronize();
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        const float a0 = A[i * 2], a1 = A[i * 2 + 1], b0 = B[j], b1 = B[32 + j], c = C[i * 32 + j];
        const float d = D[i * 32 + j];
        m01 += d != fmaf(a1, b1, fmaf(a0, b0, c));
        m10 += d != fmaf(a0, b0, fmaf(a1, b1, c));
        msum += d != (float)((double)a0 * b0 + (double)a1 * b1 + (double)c);
        ++n;
      }
  }
  printf("(a) f32 32x32x2: mismatches vs fma(a1,b1,fma(a0,b0,c)) %ld, vs fma(a0,b0,fma(a1,b1,c)) %ld, "
         "vs double-rounded-once %ld, of %ld\n", m01, m10, msum, n);

  _Float16 *Ah, *Bh;
  hipMallocManaged(&Ah, 512 * 2);
  hipMallocManaged(&Bh, 512 * 2);
  // (b) denormals: A = 2^-20 (f16 subnormal), B = 1 on the k=0 row only
  for (int i = 0; i < 512; ++i) { Ah[i] = (_Float16)0.f; Bh[i] = (_Float16)0.f; }
  for (int i = 0; i < 32; ++i) Ah[i * 16] = (_Float16)ldexpf(1.f, -20);
  for (int j = 0; j < 32; ++j) Bh[j] = (_Float16)1.f;
  hipLaunchKernelGGL(f16_step, dim3(1), dim3(64), 0, 0, Ah, Bh, D);
  hipDeviceSynchronize();
  printf("(b) f16 denormal input 2^-20 * 1 -> %g (expect %g)\n", D[0], ldexpf(1.f, -20));
  for (int i = 0; i < 32; ++i) Ah[i * 16] = (_Float16)ldexpf(1.f, -12);
  for (int j = 0; j < 32; ++j) Bh[j] = (_Float16)ldexpf(1.f, -12);
  hipLaunchKernelGGL(f16_step, dim3(1), dim3(64), 0, 0, Ah, Bh, D);
  hipDeviceSynchronize();
  printf("(b) f16 product 2^-12*2^-12 -> %g (expect %g)\n", D[0], ldexpf(1.f, -24));

  // (c) accumulation error vs double
  double worst = 0;
  for (int trial = 0; trial < 200; ++trial) {
    for (int i = 0; i < 512; ++i) {
      Ah[i] = (_Float16)(frand() * powf(2.f, (float)(rand() % 8)));
      Bh[i] = (_Float16)(frand() * powf(2.f, (float)(rand() % 8)));
    }
    hipLaunchKernelGGL(f16_step, dim3(1), dim3(64), 0, 0, Ah, Bh, D);
    hipDeviceSynchronize();
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double ref = 0, mag = 0;
        for (int k = 0; k < 16; ++k) {
          const double p = (double)(float)Ah[i * 16 + k] * (double)(float)Bh[k * 32 + j];
          ref += p;
          mag += fabs(p);
        }
        const double err = fabs(D[i * 32 + j] - ref) / (mag * ldexp(1.0, -24));
        if (err > worst) worst = err;
      }
  }
  printf("(c) f16 MFMA K=16: max |err| / (sum|a b| * 2^-24) = %.3f\n", worst);
  return 0;
}
