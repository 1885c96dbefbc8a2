// Ablation timing of ncf32_kernel (diagnostic build only; see ABL bits in ncf.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ncf_ablation.hip -o build/ncf_ablation
#include "../hnm_recommendation_amd/csrc/ncf.hip"

#include <vector>

template <int ABL>
float time_variant(dim3 grid, size_t lds, float* P, float* WG, float* Q, float* G, float* W2,
                   float* b2, float* wm, float* bp, int64_t B, int64_t I, int64_t ipp, int K,
                   float* cv, int32_t* ci, int NP) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((ncf32_kernel<false, ABL>), grid, dim3(256), lds, 0, P, WG, Q, G, 64, 64, W2,
                       64, 32, b2, wm, bp, B, I, ipp, nullptr, nullptr, K, cv, ci, NP, nullptr, 0, nullptr, nullptr);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) printf("launch error: %s\n", hipGetErrorString(err));
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int64_t B = 4096, I = 105542;
  const int K = 12;
  std::vector<float> h(I * 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  float *P, *WG, *Q, *G, *W2, *b2, *wm, *bp, *cv;
  int32_t* ci;
  (void)hipMalloc(&P, B * 64 * 4);
  (void)hipMalloc(&WG, B * 64 * 4);
  (void)hipMalloc(&Q, I * 64 * 4);
  (void)hipMalloc(&G, I * 64 * 4);
  (void)hipMalloc(&W2, 32 * 64 * 4);
  (void)hipMalloc(&b2, 256);
  (void)hipMalloc(&wm, 256);
  (void)hipMalloc(&bp, 256);
  (void)hipMemcpy(P, h.data(), B * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(WG, h.data() + 7, B * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(Q, h.data(), I * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(G, h.data(), I * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(W2, h.data() + 3, 32 * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(b2, h.data() + 5, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(wm, h.data() + 9, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(bp, h.data() + 11, 256, hipMemcpyHostToDevice);
  Partition part = choose_partition(I, hnm_cdiv(B, 128), 256);
  (void)hipMalloc(&cv, B * part.np * K * 4 + (1 << 20));
  (void)hipMalloc(&ci, B * part.np * K * 4 + (1 << 20));
  dim3 grid((unsigned)hnm_cdiv(B, 128), part.np);
  const size_t lds = 4 * 32 * K * 8;
  const double flop = 4352.0 * B * I;
#define V(A)                                                                                   \
  {                                                                                            \
    float ms = time_variant<A>(grid, lds, P, WG, Q, G, W2, b2, wm, bp, B, I, part.ipp, K, cv, ci, \
                               part.np);                                                       \
    printf("ABL=%2d  %8.3f ms  %6.1f TF (useful)\n", A, ms, flop / (ms * 1e-3) / 1e12);        \
  }
  V(0) V(1) V(2) V(3) V(31)
  return 0;
}
