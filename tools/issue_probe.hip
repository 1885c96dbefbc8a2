// Issue-cost probe for the NCF scan's instruction mix on gfx950: cycles per wave-instruction
// of v_pk_add_f16 (clamp), v_cvt_pk_f16_f32 (clamp), v_dot2c_f32_f16, v_add_f32 and
// v_permlane32_swap, alone and interleaved with v_mfma_f32_32x32x16_f16, at 1, 2 and 3
// waves per SIMD.  Blocks of independent instructions (8 rotating destinations), timed
// per wave with s_memtime (shader cycles); "per SIMD" = waves x instructions / cycles.
// Build: hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o build/issue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define R8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)

// one block = 8 independent instructions of a kind
#define PKADD(i) asm volatile("v_pk_add_f16 %0, %0, %1 clamp" : "+v"(u[i]) : "v"(w[i]));
#define CVT(i) asm volatile("v_cvt_pk_f16_f32 %0, %1, %2 clamp" : "=v"(u[i]) : "v"(f[i]), "v"(g[i]));
#define DOT(i) asm volatile("v_dot2c_f32_f16 %0, %1, %2" : "+v"(f[i]) : "v"(u[i]), "v"(w[i]));
#define ADDF(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(g[i]));
#define SWAP(i) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(f[i]), "+v"(g[i]));
#define PKADDF(i) asm volatile("v_pk_add_f32 %0, %0, %1 clamp" : "+v"(d2[i]) : "v"(e2[i]));
#define PKFMAF(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(d2[i]) : "v"(e2[i]), "v"(e2[(i + 1) & 7]));
#define PKFMAH(i) asm volatile("v_pk_fma_f16 %0, %1, %2, %0" : "+v"(u[i]) : "v"(w[i]), "v"(w[(i + 1) & 7]));
#define DOT2(i) asm volatile("v_dot2_f32_f16 %0, %1, %2, %0" : "+v"(f[i]) : "v"(u[i]), "v"(w[i]));
#define FMAF(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[i]) : "v"(g[i]), "v"(g[(i + 1) & 7]));
#define FMAMIX(i) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(f[i]) : "v"(g[i]), "v"(w[i]));
#define CVTF(i) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(f[i]) : "v"(u[i]));
#define MAXF(i) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[i]) : "v"(g[i]));

template <int KIND, int NMF>
__global__ __launch_bounds__(256) void probe(const float* in, long long* cyc, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  uint32_t u[8], w[8];
  float f[8], g[8];
  double d2[8], e2[8];  // packed-f32 register pairs
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u[i] = __float_as_uint(in[(lane + i) & 255]);
    w[i] = __float_as_uint(in[(lane + 3 * i + 1) & 255]);
    f[i] = in[(lane + 5 * i + 2) & 255];
    g[i] = in[(lane + 7 * i + 3) & 255];
    d2[i] = (double)in[(lane + 11 * i + 4) & 255];
    e2[i] = (double)in[(lane + 13 * i + 5) & 255];
  }
  h8 a = {}, b = {};
#pragma unroll
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)in[e]; b[e] = (_Float16)in[8 + e]; }
  f32x16 acc[4] = {};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
      if (NMF > 0) acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[blk], 0, 0, 0);
      if (NMF > 1) acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[blk], 0, 0, 0);
      if (KIND == 1) { R8(PKADD) }
      if (KIND == 2) { R8(CVT) }
      if (KIND == 3) { R8(DOT) }
      if (KIND == 4) { R8(ADDF) }
      if (KIND == 5) { R8(SWAP) }
      if (KIND == 6) { R8(PKADDF) }
      if (KIND == 7) { R8(PKFMAF) }
      if (KIND == 8) { R8(PKFMAH) }
      if (KIND == 9) { R8(DOT2) }
      if (KIND == 10) { R8(FMAF) }
      if (KIND == 11) { R8(MAXF) }
      if (KIND == 12) { R8(FMAMIX) }
      if (KIND == 13) { R8(CVTF) }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += __uint_as_float(u[i]) + f[i] + g[i] + (float)d2[i];
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND, int NMF>
void run(const char* name, const float* in, long long* cyc, float* out, int W, int num_cus) {
  const int iters = 2000, grid = num_cus * W;  // W workgroups of 4 waves per CU -> W waves/SIMD
  hipLaunchKernelGGL((probe<KIND, NMF>), dim3(grid), dim3(256), 0, 0, in, cyc, out, iters);
  hipLaunchKernelGGL((probe<KIND, NMF>), dim3(grid), dim3(256), 0, 0, in, cyc, out, iters);
  (void)hipDeviceSynchronize();
  static long long h[256 * 4 * 4];
  (void)hipMemcpy(h, cyc, sizeof(long long) * grid * 4, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < grid * 4; ++i) mean += (double)h[i];
  mean /= grid * 4;
  const double nv = KIND ? 32.0 * iters : 0.0, nm = 4.0 * NMF * iters;
  // per SIMD: W waves share it for ~mean cycles
  printf("%-22s W=%d  cyc/wave-iter %7.1f  | per SIMD: %6.2f cyc per VALU-instr, %6.2f cyc per MFMA\n",
         name, W, mean / iters, nv ? mean / (nv * W) : 0.0, nm ? mean / (nm * W) : 0.0);
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  float* in;
  long long* cyc;
  float* out;
  (void)hipMalloc(&in, 256 * 4);
  (void)hipMalloc(&cyc, sizeof(long long) * cus * 4 * 4);
  (void)hipMalloc(&out, 4 * 256 * cus * 4);
  float hin[256];
  for (int i = 0; i < 256; ++i) hin[i] = 0.001f * (float)((i * 37) % 101) - 0.05f;
  (void)hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  for (int W = 1; W <= 3; W += 2) {
    run<0, 1>("mfma only (1/blk)", in, cyc, out, W, cus);
    run<1, 0>("pk_add_f16 clamp", in, cyc, out, W, cus);
    run<2, 0>("cvt_pk_f16_f32 clamp", in, cyc, out, W, cus);
    run<3, 0>("dot2c_f32_f16", in, cyc, out, W, cus);
    run<4, 0>("add_f32", in, cyc, out, W, cus);
    run<5, 0>("permlane32_swap", in, cyc, out, W, cus);
    run<6, 0>("pk_add_f32 clamp", in, cyc, out, W, cus);
    run<7, 0>("pk_fma_f32", in, cyc, out, W, cus);
    run<8, 0>("pk_fma_f16", in, cyc, out, W, cus);
    run<9, 0>("dot2_f32_f16 (vop3p)", in, cyc, out, W, cus);
    run<10, 0>("fma_f32", in, cyc, out, W, cus);
    run<11, 0>("max_f32", in, cyc, out, W, cus);
    run<12, 0>("fma_mix_f32", in, cyc, out, W, cus);
    run<13, 0>("cvt_f32_f16", in, cyc, out, W, cus);
    run<1, 1>("mfma + 8 pk_add", in, cyc, out, W, cus);
    run<2, 1>("mfma + 8 cvt_pk", in, cyc, out, W, cus);
    run<3, 1>("mfma + 8 dot2c", in, cyc, out, W, cus);
    run<5, 1>("mfma + 8 swap", in, cyc, out, W, cus);
    run<6, 1>("mfma + 8 pk_add_f32", in, cyc, out, W, cus);
    run<7, 1>("mfma + 8 pk_fma_f32", in, cyc, out, W, cus);
    run<8, 1>("mfma + 8 pk_fma_f16", in, cyc, out, W, cus);
    run<9, 1>("mfma + 8 dot2 vop3p", in, cyc, out, W, cus);
    run<10, 1>("mfma + 8 fma_f32", in, cyc, out, W, cus);
    run<11, 1>("mfma + 8 max_f32", in, cyc, out, W, cus);
    run<12, 1>("mfma + 8 fma_mix_f32", in, cyc, out, W, cus);
    run<13, 1>("mfma + 8 cvt_f32_f16", in, cyc, out, W, cus);
  }
  return 0;
}
