// Random row-gather rate vs row granule (32 / 64 / 128 / 256 B) and table size on MI355X
// (round 5): can the LightGCN SpMM's user half run as column slices of the
// item table (d = 64: 27 MB; a 64-column slice of G bytes per row is I * G bytes, stored
// slice-contiguous) fast enough that several passes beat the one-pass walk's 12.8 TB/s?
// Each probe gathers uniformly random rows of G bytes from a table of `rows` rows stored with
// stride G (what a slice-major layout gives), G / 16 lanes per row, 4 row loads in flight per
// lane group, and sums them (the SpMM's per-entry work without the scale).
// Build: hipcc --offload-arch=gfx950 -O3 tools/granule_probe.hip -o tools/bin/granule_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

template <int G>
__global__ __launch_bounds__(256) void gather_sum(const float4* __restrict__ X,
                                                  const int32_t* __restrict__ idx, int per,
                                                  int64_t nout, float4* __restrict__ out) {
  constexpr int LPR = G / 16, GPW = 64 / LPR, U = 4;
  const int lane = threadIdx.x & 63, grp = lane / LPR, sub = lane % LPR;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * GPW + grp;  // output row
  if (r >= nout) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int32_t* ir = idx + r * per;
  for (int p = 0; p < per; p += U) {  // per % U == 0
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = X[(int64_t)ir[p + u] * LPR + sub];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
    }
  }
  out[r * LPR + sub] = acc;
}

template <int G>
static double run(const float4* X, const int32_t* idx, int per, int64_t nout, float4* out,
                  hipEvent_t e0, hipEvent_t e1) {
  constexpr int GPW = 64 / (G / 16);
  float best = 1e30f;
  const unsigned blocks = (unsigned)((nout + 4 * GPW - 1) / (4 * GPW));
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(gather_sum<G>, dim3(blocks), dim3(256), 0, 0, X, idx, per, nout, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return (double)nout * per * G / (best * 1e-3) / 1e12;  // TB/s of gathered bytes
}

int main() {
  const int64_t table_bytes_max = 64ll << 20;
  float4* X;
  (void)hipMalloc(&X, table_bytes_max);
  (void)hipMemset(X, 0, table_bytes_max);
  const int per = 32;
  const int64_t gathers = 16ll << 20;  // 16.8M gathers per launch
  int32_t* idx;
  float4* out;
  (void)hipMalloc(&idx, gathers * 4);
  (void)hipMalloc(&out, (gathers / per) * 256);
  int32_t* h = (int32_t*)malloc(gathers * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("uniformly random row gathers, 4 in flight per lane group; TB/s of gathered bytes\n");
  for (double mb : {1.7, 3.4, 6.8, 13.5, 27.0, 54.0}) {
    printf("table %5.1f MB:", mb);
    for (int G : {32, 64, 128, 256}) {
      const int64_t rows = (int64_t)(mb * 1e6 / G);
      uint64_t s = 88172645463325252ull;
      for (int64_t k = 0; k < gathers; ++k) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[k] = (int32_t)(s % (uint64_t)rows);
      }
      (void)hipMemcpy(idx, h, gathers * 4, hipMemcpyHostToDevice);
      const int64_t nout = gathers / per;
      double r = 0;
      if (G == 32) r = run<32>(X, idx, per, nout, out, e0, e1);
      if (G == 64) r = run<64>(X, idx, per, nout, out, e0, e1);
      if (G == 128) r = run<128>(X, idx, per, nout, out, e0, e1);
      if (G == 256) r = run<256>(X, idx, per, nout, out, e0, e1);
      printf("  G=%3d %6.2f", G, r);
      fflush(stdout);
    }
    printf("\n");
  }
  return 0;
}
