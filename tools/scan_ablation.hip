// Timing harness of ncf16_scan_kernel (THRESH mode, no appends) at the bench shape
// (B = 4096 users x 105,542 items, 24 partitions): kernel-only time, best of 7 after a
// clock warm-up, so scan variants can be compared without the rest of the step.
// Diagnostic build only:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/scan_ablation.hip -o build/scan_ablation.o
//   hipcc --offload-arch=gfx950 build/scan_ablation.o build/obj/{api,score,ncf,graph,widedeep}.o \
//         -o build/scan_ablation
#include "../hnm_recommendation_amd/csrc/ncf_cert.hip"

#include <vector>

template <typename T>
static T* dev_fill(size_t n, float lo, float hi, unsigned seed) {
  std::vector<T> h(n);
  unsigned x = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = (T)(lo + (hi - lo) * ((x >> 8) * (1.0f / 16777216.0f)));
  }
  T* d;
  (void)hipMalloc(&d, n * sizeof(T));
  (void)hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice);
  return d;
}

static float time_scan(dim3 grid, const ScanArgs& a) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 8; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((ncf16_scan_kernel<SCAN_THRESH>), grid, dim3(256), 0, 0, a);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    if (hipGetLastError() != hipSuccess) printf("launch error\n");
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int64_t B = 4096, I = 105542;
  const CertShape sh = cert_shape(B, I, 12, 256, CERT_WG_PER_CU);
  ScanArgs a{};
  a.P16 = dev_fill<_Float16>(B * 64, -0.25f, 0.25f, 1);
  a.WG16 = dev_fill<_Float16>(B * 64, -0.5f, 0.5f, 2);
  a.Q16 = dev_fill<_Float16>(I * 64, -0.25f, 0.25f, 3);
  a.G16 = dev_fill<_Float16>(I * 64, -0.5f, 0.5f, 4);
  a.W2h = dev_fill<_Float16>(32 * 64, -0.1f, 0.1f, 5);
  a.wmh = dev_fill<_Float16>(32, -0.5f, 0.5f, 6);
  a.b2s = dev_fill<float>(32, -0.01f, 0.01f, 7);
  a.Bi = dev_fill<float>(I, 0.f, 1.f, 8);
  a.Di = dev_fill<float>(I, 0.f, 1.f, 9);
  a.Cu = dev_fill<float>(B, 0.f, 1.f, 10);
  a.tau = dev_fill<float>(B, 1e30f, 1e30f, 11);  // no appends
  CertParams hp{};
  hp.unit = 1.f;
  hp.cg = 1.f;
  CertParams* prm;
  (void)hipMalloc(&prm, sizeof(CertParams));
  (void)hipMemcpy(prm, &hp, sizeof(hp), hipMemcpyHostToDevice);
  a.prm = prm;
  a.B = B;
  a.I = I;

  a.ipp = sh.part.ipp;
  a.NP = sh.part.np;
  a.capp = sh.capp;
  (void)hipMalloc(&a.cnt, B * sh.part.np * 4);
  (void)hipMalloc(&a.buf, (size_t)B * sh.part.np * sh.capp * 4);
  dim3 grid((unsigned)sh.part.np, (unsigned)hnm_cdiv(B, 128));
  const double pairs = (double)B * I, useful = 4352.0 * pairs;
  printf("grid %u x %u, ipp %ld\n", grid.x, grid.y, (long)sh.part.ipp);
  for (int w = 0; w < 100; ++w)  // clock warm-up (~0.2 s of scan work)
    hipLaunchKernelGGL((ncf16_scan_kernel<SCAN_THRESH>), grid, dim3(256), 0, 0, a);
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 3; ++rep) {
    const float ms = time_scan(grid, a);
    printf("ncf16_scan  %7.3f ms  %6.1f TF useful  %5.2f cyc/user-tile/SIMD @2.2GHz\n", ms,
           useful / (ms * 1e-3) / 1e12, ms * 1e-3 * 2.2e9 / (pairs / 32 / 1024));
  }
  return 0;
}
