// Premise check for a user-ordered ("slice walk") LightGCN item half: do item-row gathers from
// the 351 MB user table run faster when every wave of the chip walks its edges in ascending
// user id (so the chip's gathers at any moment fall in one narrow window of the table, which
// the XCD L2s and the Infinity Cache then hold) than in the CSR's random order?
//   A: the current item-half shape -- one wave per <= 2048-edge segment of an item row (random
//      user order), 4 groups of 16 lanes x float4, 4 gathers in flight per group;
//   B: persistent, one 1024-thread workgroup per CU owning ~412 items (LDS accumulators,
//      256 B each); each 16-lane group walks ONE user-sorted list of its items' edges (packed
//      user << 10 | LDS slot) with a read-modify-write of the slot per edge.
// Synthetic H&M shape: U = 1,371,980 users uniform, I = 105,542 items Zipf(0.9), E = 31.8M.
// Build: hipcc --offload-arch=gfx950 -O3 tools/slice_walk_probe.hip -o tools/bin/slice_walk_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <queue>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);          \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int D = 64;
constexpr int NG = 64;      // 16-lane groups per workgroup (1024 threads)
constexpr int MAXLOC = 560;  // LDS slots per workgroup (140 KB)

__global__ __launch_bounds__(256) void pull_segments(const int64_t* __restrict__ sst,
                                                     const int64_t* __restrict__ sen, int64_t nseg,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ val,
                                                     const float* __restrict__ X,
                                                     float* __restrict__ part) {
  const int64_t sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= nseg) return;
  const int lane = threadIdx.x & 63, grp = lane >> 4, sub = lane & 15;
  const int64_t s = sst[sg], e = sen[sg];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t p = s + grp;
  for (; p + 12 < e; p += 16) {
    int c[4];
    float w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { c[u] = col[p + 4 * u]; w[u] = val[p + 4 * u]; }
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const float4*>(X + (int64_t)c[u] * D + 4 * sub);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc.x = fmaf(w[u], x[u].x, acc.x); acc.y = fmaf(w[u], x[u].y, acc.y);
      acc.z = fmaf(w[u], x[u].z, acc.z); acc.w = fmaf(w[u], x[u].w, acc.w);
    }
  }
  for (; p < e; p += 4) {
    const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)col[p] * D + 4 * sub);
    const float w = val[p];
    acc.x = fmaf(w, x.x, acc.x); acc.y = fmaf(w, x.y, acc.y);
    acc.z = fmaf(w, x.z, acc.z); acc.w = fmaf(w, x.w, acc.w);
  }
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o); acc.y += __shfl_xor(acc.y, o);
    acc.z += __shfl_xor(acc.z, o); acc.w += __shfl_xor(acc.w, o);
  }
  if (lane < 16) *reinterpret_cast<float4*>(part + sg * D + 4 * sub) = acc;
}

template <int MODE>
__global__ __launch_bounds__(1024) void slice_walk(const int64_t* __restrict__ gptr,
                                                   const uint32_t* __restrict__ ent,
                                                   const float* __restrict__ wt,
                                                   const int32_t* __restrict__ slot_item,
                                                   const int32_t* __restrict__ nslot,
                                                   const float* __restrict__ X,
                                                   float* __restrict__ Y) {
  __shared__ float4 acc[MAXLOC * 16];
  const int tid = threadIdx.x, g = tid >> 4, sub = tid & 15;
  const int ns = nslot[blockIdx.x];
  for (int i = tid; i < ns * 16; i += 1024) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  int64_t p = gptr[blockIdx.x * NG + g];
  const int64_t e = gptr[blockIdx.x * NG + g + 1];
  float4 ra = make_float4(0.f, 0.f, 0.f, 0.f);
  for (; p + 3 < e; p += 4) {
    uint32_t c[4];
    float w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { c[u] = ent[p + u]; w[u] = wt[p + u]; }
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = *reinterpret_cast<const float4*>(X + (int64_t)(c[u] >> 10) * D + 4 * sub);
    if (MODE == 1) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ra.x = fmaf(w[u], x[u].x, ra.x); ra.y = fmaf(w[u], x[u].y, ra.y);
        ra.z = fmaf(w[u], x[u].z, ra.z); ra.w = fmaf(w[u], x[u].w, ra.w);
      }
      continue;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float4* a = &acc[(c[u] & 1023u) * 16 + sub];
      float4 v = *a;
      v.x = fmaf(w[u], x[u].x, v.x); v.y = fmaf(w[u], x[u].y, v.y);
      v.z = fmaf(w[u], x[u].z, v.z); v.w = fmaf(w[u], x[u].w, v.w);
      *a = v;
    }
  }
  if (MODE == 1) acc[(g & 31) * 16 + sub] = ra;
  for (; p < e; ++p) {
    const uint32_t c = ent[p];
    const float w = wt[p];
    const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)(c >> 10) * D + 4 * sub);
    float4* a = &acc[(c & 1023u) * 16 + sub];
    float4 v = *a;
    v.x = fmaf(w, x.x, v.x); v.y = fmaf(w, x.y, v.y);
    v.z = fmaf(w, x.z, v.z); v.w = fmaf(w, x.w, v.w);
    *a = v;
  }
  __syncthreads();
  for (int i = tid; i < ns * 16; i += 1024)
    *reinterpret_cast<float4*>(Y + (int64_t)slot_item[blockIdx.x * MAXLOC + (i >> 4)] * D + 4 * (i & 15)) = acc[i];
}

// v2: NB gathers in flight per group, the next batch's records prefetched one batch ahead
template <int NB>
__global__ __launch_bounds__(1024) void slice_walk2(const int64_t* __restrict__ gptr,
                                                    const uint32_t* __restrict__ ent,
                                                    const float* __restrict__ wt,
                                                    const int32_t* __restrict__ slot_item,
                                                    const int32_t* __restrict__ nslot,
                                                    const float* __restrict__ X,
                                                    float* __restrict__ Y) {
  __shared__ float4 acc[MAXLOC * 16];
  const int tid = threadIdx.x, g = tid >> 4, sub = tid & 15;
  const int ns = nslot[blockIdx.x];
  for (int i = tid; i < ns * 16; i += 1024) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  int64_t p = gptr[blockIdx.x * NG + g];
  const int64_t e = gptr[blockIdx.x * NG + g + 1];
  uint32_t c[NB];
  float w[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const bool ok = p + u < e;
    c[u] = ok ? ent[p + u] : 0u;
    w[u] = ok ? wt[p + u] : 0.f;
  }
  for (; p < e; p += NB) {
    float4 x[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      x[u] = *reinterpret_cast<const float4*>(X + (int64_t)(c[u] >> 10) * D + 4 * sub);
    uint32_t cn[NB];
    float wn[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const bool ok = p + NB + u < e;
      cn[u] = ok ? ent[p + NB + u] : 0u;
      wn[u] = ok ? wt[p + NB + u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (p + u < e) {
        float4* a = &acc[(c[u] & 1023u) * 16 + sub];
        float4 v = *a;
        v.x = fmaf(w[u], x[u].x, v.x); v.y = fmaf(w[u], x[u].y, v.y);
        v.z = fmaf(w[u], x[u].z, v.z); v.w = fmaf(w[u], x[u].w, v.w);
        *a = v;
      }
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) { c[u] = cn[u]; w[u] = wn[u]; }
  }
  __syncthreads();
  for (int i = tid; i < ns * 16; i += 1024)
    *reinterpret_cast<float4*>(Y + (int64_t)slot_item[blockIdx.x * MAXLOC + (i >> 4)] * D + 4 * (i & 15)) = acc[i];
}

static uint64_t rs = 88172645463325252ull;
static inline uint64_t xr() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }

int main(int argc, char** argv) {
  const int64_t U = 1371980, I = 105542, E = 31800000;
  const bool shuffle = argc > 1 && argv[1][0] == 's';
  int nwg = 256;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  nwg = prop.multiProcessorCount;
  // interactions: users uniform, items Zipf(0.9) through a random permutation
  std::vector<double> cdf(I);
  double s = 0;
  for (int64_t k = 0; k < I; ++k) { s += std::pow((double)(k + 1), -0.9); cdf[k] = s; }
  std::vector<int32_t> perm(I);
  std::iota(perm.begin(), perm.end(), 0);
  for (int64_t k = I - 1; k > 0; --k) std::swap(perm[k], perm[xr() % (k + 1)]);
  std::vector<int32_t> eu(E), ei(E);
  for (int64_t k = 0; k < E; ++k) {
    eu[k] = (int32_t)(xr() % U);
    const double r = (double)(xr() >> 11) * (1.0 / 9007199254740992.0) * s;
    ei[k] = perm[std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin() < I
                     ? std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin() : I - 1];
  }
  // item CSR, random user order (edge order), weight = pseudo-random
  std::vector<int64_t> rp(I + 1, 0);
  for (int64_t k = 0; k < E; ++k) rp[ei[k] + 1]++;
  for (int64_t i = 0; i < I; ++i) rp[i + 1] += rp[i];
  std::vector<int32_t> col(E);
  std::vector<float> val(E);
  {
    std::vector<int64_t> pos(rp.begin(), rp.end() - 1);
    for (int64_t k = 0; k < E; ++k) {
      const int64_t q = pos[ei[k]]++;
      col[q] = eu[k];
      val[q] = 1.f / (1.f + (float)(k % 97));
    }
  }
  int64_t maxdeg = 0;
  for (int64_t i = 0; i < I; ++i) maxdeg = std::max(maxdeg, rp[i + 1] - rp[i]);
  // A: segments of <= 2048
  std::vector<int64_t> sst, sen;
  for (int64_t i = 0; i < I; ++i)
    for (int64_t a = rp[i]; a < rp[i + 1]; a += 2048) { sst.push_back(a); sen.push_back(std::min(a + 2048, rp[i + 1])); }
  // B: pieces (items split interleaved when deg > cap), greedy to workgroups then groups
  const int64_t cap = E / ((int64_t)nwg * NG) / 2;
  struct Piece { int32_t item, k, n; int64_t len; };
  std::vector<Piece> pcs;
  for (int64_t i = 0; i < I; ++i) {
    const int64_t dg = rp[i + 1] - rp[i];
    if (!dg) continue;
    const int n = (int)((dg + cap - 1) / cap);
    for (int k = 0; k < n; ++k) pcs.push_back({(int32_t)i, k, n, (dg - k + n - 1) / n});
  }
  std::sort(pcs.begin(), pcs.end(), [](const Piece& a, const Piece& b) { return a.len > b.len; });
  std::vector<std::vector<int>> wgp(nwg);
  {
    std::priority_queue<std::pair<int64_t, int>, std::vector<std::pair<int64_t, int>>, std::greater<>> q;
    for (int w = 0; w < nwg; ++w) q.push({0, w});
    std::vector<std::pair<int64_t, int>> held;
    for (int pi = 0; pi < (int)pcs.size(); ++pi) {
      auto t = q.top(); q.pop();
      while ((int)wgp[t.second].size() >= MAXLOC) { t = q.top(); q.pop(); }
      wgp[t.second].push_back(pi);
      q.push({t.first + pcs[pi].len, t.second});
    }
  }
  std::vector<int64_t> gptr(nwg * NG + 1, 0);
  std::vector<uint32_t> ent;
  std::vector<float> wt;
  std::vector<int32_t> slot_item(nwg * MAXLOC, 0), nslot(nwg);
  ent.reserve(E); wt.reserve(E);
  int64_t split_pieces = 0;
  for (int w = 0; w < nwg; ++w) {
    nslot[w] = (int)wgp[w].size();
    std::vector<std::vector<int>> gp(NG);
    std::vector<int64_t> gl(NG, 0);
    for (int sl = 0; sl < (int)wgp[w].size(); ++sl) {  // pieces already in decreasing length
      int gb = (int)(std::min_element(gl.begin(), gl.end()) - gl.begin());
      gp[gb].push_back(sl);
      gl[gb] += pcs[wgp[w][sl]].len;
      slot_item[w * MAXLOC + sl] = pcs[wgp[w][sl]].item;
      split_pieces += pcs[wgp[w][sl]].n > 1;
    }
    for (int g = 0; g < NG; ++g) {
      std::vector<std::pair<uint32_t, float>> L;
      for (int sl : gp[g]) {
        const Piece& pc = pcs[wgp[w][sl]];
        for (int64_t q = rp[pc.item] + pc.k; q < rp[pc.item + 1]; q += pc.n)
          L.push_back({((uint32_t)col[q] << 10) | (uint32_t)sl, val[q]});
      }
      if (shuffle) {
        for (int64_t k = (int64_t)L.size() - 1; k > 0; --k) std::swap(L[k], L[xr() % (k + 1)]);
      } else {
        std::stable_sort(L.begin(), L.end(), [](auto& a, auto& b) { return (a.first >> 10) < (b.first >> 10); });
      }
      for (auto& x : L) { ent.push_back(x.first); wt.push_back(x.second); }
      gptr[w * NG + g + 1] = (int64_t)ent.size();
    }
  }
  int64_t mx = 0;
  for (int w = 0; w < nwg; ++w) mx = std::max(mx, gptr[(w + 1) * NG] - gptr[w * NG]);
  printf("E %ld maxdeg %ld segments %zu pieces %zu (split %ld) wg max/avg edges %.3f\n", (long)E,
         (long)maxdeg, sst.size(), pcs.size(), (long)split_pieces, (double)mx * nwg / E);

  float *X, *val_d, *part, *Y, *wt_d;
  int32_t *col_d, *si_d, *ns_d;
  int64_t *sst_d, *sen_d, *gp_d;
  uint32_t* ent_d;
  CK(hipMalloc(&X, U * D * 4));
  {
    std::vector<float> hx(U * D);
    for (auto& v : hx) v = (float)((xr() >> 40) & 1023) / 1024.f - 0.5f;
    CK(hipMemcpy(X, hx.data(), U * D * 4, hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&col_d, E * 4)); CK(hipMalloc(&val_d, E * 4));
  CK(hipMemcpy(col_d, col.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(val_d, val.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&sst_d, sst.size() * 8)); CK(hipMalloc(&sen_d, sst.size() * 8));
  CK(hipMemcpy(sst_d, sst.data(), sst.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(sen_d, sen.data(), sst.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&part, sst.size() * D * 4));
  CK(hipMalloc(&Y, I * D * 4));
  CK(hipMalloc(&gp_d, gptr.size() * 8)); CK(hipMalloc(&ent_d, E * 4)); CK(hipMalloc(&wt_d, E * 4));
  CK(hipMalloc(&si_d, slot_item.size() * 4)); CK(hipMalloc(&ns_d, nwg * 4));
  CK(hipMemcpy(gp_d, gptr.data(), gptr.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ent_d, ent.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wt_d, wt.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(si_d, slot_item.data(), slot_item.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ns_d, nslot.data(), nwg * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0) best = std::min(best, ms);
    }
    return best;
  };
  const double gb = (double)E * 256 / 1e9;
  const float ta = timeit([&] {
    hipLaunchKernelGGL(pull_segments, dim3((unsigned)((sst.size() + 3) / 4)), dim3(256), 0, 0, sst_d,
                       sen_d, (int64_t)sst.size(), col_d, val_d, X, part);
  });
  CK(hipGetLastError());
  printf("A pull segments (random order): %.3f ms  %.2f TB/s gathered\n", ta, gb / ta);
  const float tb = timeit([&] {
    hipLaunchKernelGGL(slice_walk<0>, dim3(nwg), dim3(1024), 0, 0, gp_d, ent_d, wt_d, si_d, ns_d, X, Y);
  });
  CK(hipGetLastError());
  printf("B slice walk (%s order):      %.3f ms  %.2f TB/s gathered\n", shuffle ? "random" : "user", tb, gb / tb);
  const float tc = timeit([&] {
    hipLaunchKernelGGL(slice_walk<1>, dim3(nwg), dim3(1024), 0, 0, gp_d, ent_d, wt_d, si_d, ns_d, X, Y);
  });
  printf("C walk, register acc only (no LDS per edge): %.3f ms  %.2f TB/s gathered\n", tc, gb / tc);
  const float t4 = timeit([&] {
    hipLaunchKernelGGL(slice_walk2<4>, dim3(nwg), dim3(1024), 0, 0, gp_d, ent_d, wt_d, si_d, ns_d, X, Y);
  });
  const float t8 = timeit([&] {
    hipLaunchKernelGGL(slice_walk2<8>, dim3(nwg), dim3(1024), 0, 0, gp_d, ent_d, wt_d, si_d, ns_d, X, Y);
  });
  printf("B2 prefetched records, 4 / 8 in flight: %.3f / %.3f ms  %.2f / %.2f TB/s\n", t4, t8, gb / t4, gb / t8);
  // check: B's unsplit items vs A's segment partial sums (same edges, different order)
  std::vector<float> hp(sst.size() * D), hy(I * D);
  CK(hipMemcpy(hp.data(), part, hp.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hy.data(), Y, hy.size() * 4, hipMemcpyDeviceToHost));
  double maxrel = 0;
  int64_t sg = 0, checked = 0;
  for (int64_t i = 0; i < I; ++i) {
    std::vector<double> a(D, 0.0);
    double mag = 1e-6;
    for (; sg < (int64_t)sst.size() && sst[sg] < rp[i + 1]; ++sg)
      for (int c = 0; c < D; ++c) { a[c] += hp[sg * D + c]; mag = std::max(mag, std::fabs(a[c])); }
    if (rp[i + 1] - rp[i] > cap || rp[i + 1] == rp[i]) continue;
    ++checked;
    for (int c = 0; c < D; ++c) maxrel = std::max(maxrel, std::fabs(a[c] - hy[i * D + c]) / mag);
  }
  printf("checked %ld items, max rel diff %.3g\n", (long)checked, maxrel);
  return 0;
}
