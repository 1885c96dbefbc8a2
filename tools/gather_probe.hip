// Random 256-B row-gather bandwidth vs table size and loads in flight on MI355X: the
// ceiling the LightGCN SpMM's gathers run against (user half: 27 MB item table, item half:
// 351 MB user table at d = 64).  Round 1 measured U = 1 only (one load in flight per 16-lane
// group); round 4 adds U = 2 / 4 / 8 independent loads per group per step.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o build/gather_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// wave per output row, 16 lanes x float4 per gathered row, 4 groups x U rows in flight per wave
template <int U>
__global__ __launch_bounds__(256) void gather_sum(const float* __restrict__ X,
                                                  const int32_t* __restrict__ idx, int64_t nnz_per_out,
                                                  int64_t nout, float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nout) return;
  const int lane = threadIdx.x & 63, grp = lane >> 4, sub = lane & 15;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int32_t* ir = idx + r * nnz_per_out;
  for (int64_t p = grp * U; p < nnz_per_out; p += 4 * U) {  // nnz_per_out % (4 U) == 0
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = *reinterpret_cast<const float4*>(X + (int64_t)ir[p + u] * 64 + 4 * sub);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
    }
  }
  if (lane < 16) *reinterpret_cast<float4*>(out + r * 64 + 4 * sub) = acc;
}

template <int U>
static float run(const float* X, const int32_t* idx, int64_t per, int64_t nout, float* out,
                 hipEvent_t e0, hipEvent_t e1) {
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(gather_sum<U>, dim3((unsigned)(nout / 4)), dim3(256), 0, 0, X, idx, per,
                       nout, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int64_t maxrows = 1400000;  // 358 MB at 64 floats
  float* X;
  (void)hipMalloc(&X, maxrows * 64 * 4);
  (void)hipMemset(X, 0, maxrows * 64 * 4);
  const int64_t nout = 200000, per = 64;  // 12.8M gathers = 3.3 GB per launch
  int32_t* idx;
  float* out;
  (void)hipMalloc(&idx, nout * per * 4);
  (void)hipMalloc(&out, nout * 64 * 4);
  int32_t* h = (int32_t*)malloc(nout * per * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int64_t rows : {16384L, 65536L, 105542L, 262144L, 524288L, 1048576L, 1371980L}) {
    uint64_t s = 88172645463325252ull;
    for (int64_t k = 0; k < nout * per; ++k) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      h[k] = (int32_t)(s % (uint64_t)rows);
    }
    (void)hipMemcpy(idx, h, nout * per * 4, hipMemcpyHostToDevice);
    const double bytes = (double)nout * per * 256;
    const float t1 = run<1>(X, idx, per, nout, out, e0, e1);
    const float t2 = run<2>(X, idx, per, nout, out, e0, e1);
    const float t4 = run<4>(X, idx, per, nout, out, e0, e1);
    const float t8 = run<8>(X, idx, per, nout, out, e0, e1);
    printf("table %7.1f MB: gather TB/s  U=1 %.2f  U=2 %.2f  U=4 %.2f  U=8 %.2f\n",
           rows * 256.0 / 1e6, bytes / (t1 * 1e-3) / 1e12, bytes / (t2 * 1e-3) / 1e12,
           bytes / (t4 * 1e-3) / 1e12, bytes / (t8 * 1e-3) / 1e12);
  }
  return 0;
}
