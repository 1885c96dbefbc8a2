// Timing harness of dot16_scan_kernel (THRESH, d = 64, no bias) at the MF / LightGCN bench
// shape (B = 4096 users x 105,542 items): synthetic f16 rows, one threshold for every row set
// at ~3.1 sigma of the approx scores (~100 appends per row, like the bench's 107-111), kernel
// time best of 7 after a clock warm-up.  Diagnostic build only:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDOT_SRC='"../hnm_recommendation_amd/csrc/dot_cert.hip"' \
//         -c tools/dot_scan_timing.hip -o build/dot_scan_timing.o && link with build/obj/*.o
#ifndef DOT_SRC
#define DOT_SRC "../hnm_recommendation_amd/csrc/dot_cert.hip"
#endif
#include DOT_SRC
#ifdef DOT_OLD
#define DOT_KERNEL dot16_scan_kernel<64, DSCAN_THRESH, false>
#else
#define DOT_KERNEL dot16_scan_kernel<64, DSCAN_THRESH, false, false>
#endif

#include <stdio.h>
#include <stdlib.h>
#include <vector>

static _Float16* dev_h16(size_t n, float a, unsigned seed) {
  std::vector<_Float16> h(n);
  unsigned x = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = (_Float16)(a * (2.f * ((x >> 8) * (1.0f / 16777216.0f)) - 1.f));
  }
  _Float16* d;
  (void)hipMalloc(&d, n * 2);
  (void)hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
  return d;
}

int main(int argc, char** argv) {
  // argv[1]: threshold in sigmas (default 3.1; 100 = no appends: the cost of the append path)
  const float fac = argc > 1 ? (float)atof(argv[1]) : 3.1f;
  const int64_t B = 4096, I = 105542;
  const int K = 12;
  int cus = 256;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
  const DotCertShape sh = dcert_shape(B, I, 64, K, cus);
  const float a = 0.125f, sigma = 8.f * a * a / 3.f;
  std::vector<float> ht(B, fac * sigma);
  DScanArgs s{};
  s.U16 = dev_h16(B * 64, a, 1);
  s.I16 = dev_h16(I * 64, a, 2);
  s.B = B;
  s.I = I;
  s.istride = 1;
  s.ipp = sh.part.ipp;
  s.NP = sh.part.np;
  s.capp = sh.capp;
  float* tau;
  (void)hipMalloc(&tau, B * 4);
  (void)hipMemcpy(tau, ht.data(), B * 4, hipMemcpyHostToDevice);
  s.tau = tau;
  (void)hipMalloc(&s.cnt, B * sh.part.np * 4);
  (void)hipMalloc(&s.buf, (size_t)B * sh.part.np * sh.capp * 4);
  dim3 grid((unsigned)sh.part.np, (unsigned)hnm_cdiv(B, 128));
  printf("grid %u x %u, ipp %ld, capp %d\n", grid.x, grid.y, (long)sh.part.ipp, sh.capp);
  for (int w = 0; w < 200; ++w)
    hipLaunchKernelGGL((DOT_KERNEL), grid, dim3(256), 0, 0, s);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 8; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((DOT_KERNEL), grid, dim3(256), 0, 0, s);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  std::vector<int> hc(B * sh.part.np);
  (void)hipMemcpy(hc.data(), s.cnt, hc.size() * 4, hipMemcpyDeviceToHost);
  double tot = 0;
  for (int v : hc) tot += v;
  const double flops = 2.0 * 64 * B * I;
  printf("tau %5.2f sigma  dot16_scan  %7.4f ms  %6.1f TF  appends/row %.1f\n", fac, best, flops / (best * 1e-3) / 1e12, tot / B);
  return 0;
}
