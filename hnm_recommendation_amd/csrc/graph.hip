// LightGCN graph path for gfx950: normalized-adjacency CSR build (a5) and SpMM with the
// fused layer combine (a6).
//
// CSR build (lightgcn.py:81-134): edges are radix-sorted by row (stable, so within a row
// the reference's edge order is kept) and each row gets its self-loop appended last, the
// same summation order as the reference's `cat([edges, loops])` (lightgcn.py:128-131).
// deg = row sum of the weights (exact integer counts for unweighted graphs), dinv =
// deg^-1/2 with inf -> 0, val = (dinv[row] * w) * dinv[col] (lightgcn.py:104-106).
//
// SpMM (lightgcn.py:152): a row's neighbours are gathered as whole embedding rows, d/4
// lanes x 16 B each, 64/(d/4) neighbours per wave instruction, 4-deep unrolled so ~16
// rows are in flight per wave.  Rows up to HEAVY neighbours take one wave; power-law item
// rows (up to ~1e6 neighbours on the H&M shape) are cut into SEG-long segments whose
// partial sums are added back in segment order, so results are deterministic and the
// longest wave is bounded.  Epilogue: Y = sum, acc_out = acc_in + alpha * Y
// (lightgcn.py:156-158).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "hnm_device.h"
#include "hnm_internal.h"

#define HEAVY 2048
#define SEG 2048

struct hnm_spmm_plan {
  int device;
  int64_t N;
  int64_t n_heavy;
  int64_t n_seg;
  int32_t* heavy_rows;  // [n_heavy]
  int64_t* seg_ptr;     // [n_heavy + 1]
  int32_t* seg_hrow;    // [n_seg]  index into heavy_rows
  int64_t* seg_start;   // [n_seg]
  int64_t* seg_end;     // [n_seg]
};

// ------------------------------------------------------------------ CSR build kernels
__global__ void csr_prep_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                                int32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                unsigned* err) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * 256) {
    int64_t r = ei[e], c = ei[E + e];
    if (r < 0 || r >= N || c < 0 || c >= N) {
      hnm_flag(err, HNM_ERR_OOB);
      r = 0;
    }
    keys[e] = (int32_t)r;
    vals[e] = (int32_t)e;
  }
}

// Row extents from the sorted keys (no atomics: power-law rows would serialize them):
// first[r] / last[r] = first and one-past-last sorted position of row r (0 / 0 if empty).
__global__ void csr_extent_kernel(const int32_t* __restrict__ skeys, int64_t E,
                                  int32_t* __restrict__ first, int32_t* __restrict__ last) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < E;
       p += (int64_t)gridDim.x * 256) {
    const int32_t r = skeys[p];
    if (p == 0 || skeys[p - 1] != r) first[r] = (int32_t)p;
    if (p == E - 1 || skeys[p + 1] != r) last[r] = (int32_t)(p + 1);
  }
}

__global__ void csr_counts_kernel(const int32_t* __restrict__ first,
                                  const int32_t* __restrict__ last, int64_t N,
                                  int64_t* __restrict__ counts) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r <= N;
       r += (int64_t)gridDim.x * 256)
    counts[r] = r < N ? (int64_t)(last[r] - first[r]) + 1 : 0;
}

__global__ void csr_place_kernel(const int64_t* __restrict__ ei, const float* __restrict__ w,
                                 int64_t E, int64_t N, const int32_t* __restrict__ skeys,
                                 const int32_t* __restrict__ svals,
                                 const int64_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                 float* __restrict__ wt) {
  const int64_t total = E + N;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * 256) {
    if (p < E) {
      const int64_t r = skeys[p];
      const int64_t e = svals[p];
      const int64_t dst = p + r;  // rows < r each hold one extra (self-loop) entry
      int64_t c = ei[E + e];
      if (c < 0 || c >= N) c = 0;
      col[dst] = (int32_t)c;
      wt[dst] = w ? w[e] : 1.f;
    } else {
      const int64_t r = p - E;
      const int64_t dst = rowptr[r + 1] - 1;
      col[dst] = (int32_t)r;
      wt[dst] = 1.f;
    }
  }
}

// dinv[r] = deg^-1/2 (inf -> 0); one wave per row, fixed-order reduction when weighted
__global__ __launch_bounds__(256) void csr_degree_kernel(const int64_t* __restrict__ rowptr,
                                                         const float* __restrict__ wt, int64_t N,
                                                         bool weighted,
                                                         float* __restrict__ dinv) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const int lane = threadIdx.x & 63;
  const int64_t s = rowptr[r], e = rowptr[r + 1];
  float deg;
  if (!weighted) {
    deg = (float)(e - s);
  } else {
    float acc = 0.f;
    for (int64_t p = s + lane; p < e; p += 64) acc += wt[p];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    deg = acc;
  }
  if (lane == 0) {
    float di = 1.0f / sqrtf(deg);
    if (isinf(di)) di = 0.f;
    dinv[r] = di;
  }
}

// val = (dinv[row] * w) * dinv[col]: one thread per entry (edges via the sorted keys,
// then the self-loops), so power-law rows cost nothing extra.
__global__ void csr_norm_kernel(const int32_t* __restrict__ skeys, int64_t E, int64_t N,
                                const int64_t* __restrict__ rowptr,
                                const int32_t* __restrict__ col, const float* __restrict__ dinv,
                                float* __restrict__ val) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < E + N;
       p += (int64_t)gridDim.x * 256) {
    int64_t r, dst;
    if (p < E) {
      r = skeys[p];
      dst = p + r;
    } else {
      r = p - E;
      dst = rowptr[r + 1] - 1;
    }
    val[dst] = (dinv[r] * val[dst]) * dinv[col[dst]];
  }
}

extern "C" hnm_status hnm_csr_build_norm(hnm_ctx* ctx, const int64_t* edge_index,
                                         const float* edge_weight, int64_t E, int64_t N,
                                         int64_t* rowptr, int32_t* col, float* val) {
  HNM_REQUIRE(ctx && rowptr && col && val && (edge_index || E == 0), HNM_EINVAL,
              "csr_build: NULL argument");
  HNM_REQUIRE(N > 0 && N < 0x7fffffff && E >= 0 && E < 0x7fffffff, HNM_EUNSUPPORTED,
              "csr_build: N and E must fit int32 (N=%lld, E=%lld)", (long long)N, (long long)E);
  hipStream_t st = ctx->stream;
  const int64_t En = std::max<int64_t>(E, 1);
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) < N) ++bits;
  size_t sort_tmp = 0, scan_tmp = 0;
  HNM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (int32_t*)nullptr,
                                                   (int32_t*)nullptr, (int32_t*)nullptr,
                                                   (int32_t*)nullptr, (int)En, 0, bits, st));
  HNM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (int64_t*)nullptr,
                                                 (int64_t*)nullptr, (int)(N + 1), st));
  const size_t s4 = hnm_align((size_t)En * 4);
  const size_t sc = hnm_align((size_t)(N + 1) * 4), sc8 = hnm_align((size_t)(N + 1) * 8);
  const size_t sd = hnm_align((size_t)N * 4);
  const size_t tmp = hnm_align(std::max(sort_tmp, scan_tmp));
  void* wsp;
  hnm_status s = hnm_workspace(ctx, 4 * s4 + 2 * sc + sc8 + sd + tmp, &wsp);
  if (s) return s;
  char* p = (char*)wsp;
  int32_t* kin = (int32_t*)p; p += s4;
  int32_t* kout = (int32_t*)p; p += s4;
  int32_t* vin = (int32_t*)p; p += s4;
  int32_t* vout = (int32_t*)p; p += s4;
  int32_t* first = (int32_t*)p; p += sc;
  int32_t* last = (int32_t*)p; p += sc;
  int64_t* counts = (int64_t*)p; p += sc8;
  float* dinv = (float*)p; p += sd;
  void* t = p;

  HNM_HIP_CHECK(hipMemsetAsync(first, 0, (size_t)(N + 1) * 4, st));
  HNM_HIP_CHECK(hipMemsetAsync(last, 0, (size_t)(N + 1) * 4, st));
  const unsigned g = 8 * 1024;
  if (E > 0) {
    hipLaunchKernelGGL(csr_prep_kernel, dim3(g), dim3(256), 0, st, edge_index, E, N, kin, vin,
                       ctx->err_dev);
    HNM_LAUNCH_CHECK();
    size_t tb = sort_tmp;
    HNM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(t, tb, kin, kout, vin, vout, (int)E, 0, bits, st));
    hipLaunchKernelGGL(csr_extent_kernel, dim3(g), dim3(256), 0, st, kout, E, first, last);
    HNM_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(csr_counts_kernel, dim3(g), dim3(256), 0, st, first, last, N, counts);
  HNM_LAUNCH_CHECK();
  size_t tb = scan_tmp;
  HNM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t, tb, counts, rowptr, (int)(N + 1), st));
  hipLaunchKernelGGL(csr_place_kernel, dim3(g), dim3(256), 0, st, edge_index, edge_weight, E, N,
                     kout, vout, rowptr, col, val);
  HNM_LAUNCH_CHECK();
  const dim3 rg((unsigned)hnm_cdiv(N, 4));
  hipLaunchKernelGGL(csr_degree_kernel, rg, dim3(256), 0, st, rowptr, val, N,
                     edge_weight != nullptr, dinv);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(csr_norm_kernel, dim3(g), dim3(256), 0, st, kout, E, N, rowptr, col, dinv,
                     val);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// ------------------------------------------------------------------ SpMM
// Sum of val[e] * X[col[e], :] over e in [s, e) with the lane layout of LPR lanes per row.
template <int LPR>
__device__ __forceinline__ float4 row_sum(const int32_t* __restrict__ col,
                                          const float* __restrict__ val,
                                          const float* __restrict__ X, int d, int64_t s,
                                          int64_t e, int lane) {
  constexpr int G = 64 / LPR;
  const int grp = lane / LPR, sub = lane % LPR;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t p = s + grp;
  for (; p + 3 * G < e; p += 4 * G) {
    int c[4];
    float w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = col[p + u * G];
      w[u] = val[p + u * G];
    }
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const float4*>(X + (int64_t)c[u] * d + 4 * sub);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc.x = fmaf(w[u], x[u].x, acc.x);
      acc.y = fmaf(w[u], x[u].y, acc.y);
      acc.z = fmaf(w[u], x[u].z, acc.z);
      acc.w = fmaf(w[u], x[u].w, acc.w);
    }
  }
  for (; p < e; p += G) {
    const int c = col[p];
    const float w = val[p];
    const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)c * d + 4 * sub);
    acc.x = fmaf(w, x.x, acc.x);
    acc.y = fmaf(w, x.y, acc.y);
    acc.z = fmaf(w, x.z, acc.z);
    acc.w = fmaf(w, x.w, acc.w);
  }
  // fixed-order tree across the G neighbour groups
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o);
    acc.y += __shfl_xor(acc.y, o);
    acc.z += __shfl_xor(acc.z, o);
    acc.w += __shfl_xor(acc.w, o);
  }
  return acc;
}

__device__ __forceinline__ void spmm_epilogue(int64_t r, int d, int sub, float4 y, float* Y,
                                              float alpha, const float* acc_in, float* acc_out) {
  const int64_t off = r * d + 4 * sub;
  if (Y) *reinterpret_cast<float4*>(Y + off) = y;
  if (acc_out) {
    float4 a = acc_in ? *reinterpret_cast<const float4*>(acc_in + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    a.x += alpha * y.x;
    a.y += alpha * y.y;
    a.z += alpha * y.z;
    a.w += alpha * y.w;
    *reinterpret_cast<float4*>(acc_out + off) = a;
  }
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm_light_kernel(int64_t N, const int64_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col,
                                                         const float* __restrict__ val,
                                                         const float* __restrict__ X, int d,
                                                         float* Y, float alpha,
                                                         const float* acc_in, float* acc_out,
                                                         int64_t heavy) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const int lane = threadIdx.x & 63;
  const int64_t s = rowptr[r], e = rowptr[r + 1];
  if (e - s > heavy) return;  // segmented path
  const float4 y = row_sum<LPR>(col, val, X, d, s, e, lane);
  if (lane < LPR) spmm_epilogue(r, d, lane, y, Y, alpha, acc_in, acc_out);
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm_segment_kernel(int64_t nseg,
                                                           const int64_t* __restrict__ seg_start,
                                                           const int64_t* __restrict__ seg_end,
                                                           const int32_t* __restrict__ col,
                                                           const float* __restrict__ val,
                                                           const float* __restrict__ X, int d,
                                                           float* __restrict__ partial) {
  const int64_t sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= nseg) return;
  const int lane = threadIdx.x & 63;
  const float4 y = row_sum<LPR>(col, val, X, d, seg_start[sg], seg_end[sg], lane);
  if (lane < LPR) *reinterpret_cast<float4*>(partial + sg * d + 4 * lane) = y;
}

__global__ __launch_bounds__(256) void spmm_finish_kernel(int64_t nheavy,
                                                          const int32_t* __restrict__ heavy_rows,
                                                          const int64_t* __restrict__ seg_ptr,
                                                          const float* __restrict__ partial,
                                                          int d, float* Y, float alpha,
                                                          const float* acc_in, float* acc_out) {
  const int64_t hr = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hr >= nheavy) return;
  const int lane = threadIdx.x & 63;
  const int64_t r = heavy_rows[hr];
  for (int sub = lane; sub < d / 4; sub += 64) {
    float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t sg = seg_ptr[hr]; sg < seg_ptr[hr + 1]; ++sg) {
      const float4 v = *reinterpret_cast<const float4*>(partial + sg * d + 4 * sub);
      y.x += v.x;
      y.y += v.y;
      y.z += v.z;
      y.w += v.w;
    }
    spmm_epilogue(r, d, sub, y, Y, alpha, acc_in, acc_out);
  }
}

extern "C" hnm_status hnm_spmm_plan_create(hnm_ctx* ctx, int64_t N, const int64_t* rowptr,
                                           hnm_spmm_plan** out) {
  HNM_REQUIRE(ctx && rowptr && out && N > 0, HNM_EINVAL, "spmm_plan: bad argument");
  std::vector<int64_t> rp((size_t)N + 1);
  HNM_HIP_CHECK(hipMemcpyAsync(rp.data(), rowptr, (N + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  std::vector<int32_t> hrows, shrow;
  std::vector<int64_t> sptr{0}, sstart, send;
  for (int64_t r = 0; r < N; ++r) {
    const int64_t s = rp[r], e = rp[r + 1];
    if (e - s <= HEAVY) continue;
    const int32_t hi = (int32_t)hrows.size();
    hrows.push_back((int32_t)r);
    for (int64_t q = s; q < e; q += SEG) {
      shrow.push_back(hi);
      sstart.push_back(q);
      send.push_back(std::min<int64_t>(q + SEG, e));
    }
    sptr.push_back((int64_t)sstart.size());
  }
  hnm_spmm_plan* pl = (hnm_spmm_plan*)calloc(1, sizeof(hnm_spmm_plan));
  HNM_REQUIRE(pl, HNM_ENOMEM, "spmm_plan: out of host memory");
  pl->device = ctx->device;
  pl->N = N;
  pl->n_heavy = (int64_t)hrows.size();
  pl->n_seg = (int64_t)sstart.size();
  if (pl->n_heavy > 0) {
    if (hipMalloc((void**)&pl->heavy_rows, pl->n_heavy * 4) != hipSuccess ||
        hipMalloc((void**)&pl->seg_ptr, (pl->n_heavy + 1) * 8) != hipSuccess ||
        hipMalloc((void**)&pl->seg_hrow, pl->n_seg * 4) != hipSuccess ||
        hipMalloc((void**)&pl->seg_start, pl->n_seg * 8) != hipSuccess ||
        hipMalloc((void**)&pl->seg_end, pl->n_seg * 8) != hipSuccess) {
      hnm_spmm_plan_destroy(pl);
      hnm_set_error("spmm_plan: hipMalloc failed");
      return HNM_ENOMEM;
    }
    HNM_HIP_CHECK(hipMemcpy(pl->heavy_rows, hrows.data(), pl->n_heavy * 4, hipMemcpyHostToDevice));
    HNM_HIP_CHECK(hipMemcpy(pl->seg_ptr, sptr.data(), (pl->n_heavy + 1) * 8, hipMemcpyHostToDevice));
    HNM_HIP_CHECK(hipMemcpy(pl->seg_hrow, shrow.data(), pl->n_seg * 4, hipMemcpyHostToDevice));
    HNM_HIP_CHECK(hipMemcpy(pl->seg_start, sstart.data(), pl->n_seg * 8, hipMemcpyHostToDevice));
    HNM_HIP_CHECK(hipMemcpy(pl->seg_end, send.data(), pl->n_seg * 8, hipMemcpyHostToDevice));
  }
  *out = pl;
  return HNM_OK;
}

extern "C" hnm_status hnm_spmm_plan_destroy(hnm_spmm_plan* pl) {
  if (!pl) return HNM_OK;
  if (pl->heavy_rows) (void)hipFree(pl->heavy_rows);
  if (pl->seg_ptr) (void)hipFree(pl->seg_ptr);
  if (pl->seg_hrow) (void)hipFree(pl->seg_hrow);
  if (pl->seg_start) (void)hipFree(pl->seg_start);
  if (pl->seg_end) (void)hipFree(pl->seg_end);
  free(pl);
  return HNM_OK;
}

template <int LPR>
static hnm_status spmm_launch(hnm_ctx* ctx, const hnm_spmm_plan* pl, int64_t N,
                              const int64_t* rowptr, const int32_t* col, const float* val,
                              const float* X, int d, float* Y, float alpha, const float* acc_in,
                              float* acc_out) {
  const int64_t heavy = (pl && pl->n_heavy > 0) ? HEAVY : INT64_MAX;
  hnm_timer_begin(ctx, HNM_TIME_SPMM);
  hipLaunchKernelGGL(spmm_light_kernel<LPR>, dim3((unsigned)hnm_cdiv(N, 4)), dim3(256), 0,
                     ctx->stream, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out, heavy);
  HNM_LAUNCH_CHECK();
  if (pl && pl->n_heavy > 0) {
    void* w;
    hnm_status s = hnm_workspace(ctx, (size_t)pl->n_seg * d * 4, &w);
    if (s) return s;
    float* partial = (float*)w;
    hipLaunchKernelGGL(spmm_segment_kernel<LPR>, dim3((unsigned)hnm_cdiv(pl->n_seg, 4)), dim3(256),
                       0, ctx->stream, pl->n_seg, pl->seg_start, pl->seg_end, col, val, X, d,
                       partial);
    HNM_LAUNCH_CHECK();
    hipLaunchKernelGGL(spmm_finish_kernel, dim3((unsigned)hnm_cdiv(pl->n_heavy, 4)), dim3(256), 0,
                       ctx->stream, pl->n_heavy, pl->heavy_rows, pl->seg_ptr, partial, d, Y,
                       alpha, acc_in, acc_out);
    HNM_LAUNCH_CHECK();
  }
  hnm_timer_end(ctx, HNM_TIME_SPMM);
  return HNM_OK;
}

extern "C" hnm_status hnm_spmm_csr_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                                       const int64_t* rowptr, const int32_t* col,
                                       const float* val, const float* X, int d, float* Y,
                                       float alpha, const float* acc_in, float* acc_out) {
  HNM_REQUIRE(ctx && rowptr && col && val && X, HNM_EINVAL, "spmm: NULL argument");
  HNM_REQUIRE(!plan || plan->N == N, HNM_EINVAL, "spmm: plan built for a different graph");
  HNM_REQUIRE((uintptr_t)X % 16 == 0 && (!Y || (uintptr_t)Y % 16 == 0) &&
                  (!acc_out || (uintptr_t)acc_out % 16 == 0) &&
                  (!acc_in || (uintptr_t)acc_in % 16 == 0),
              HNM_EUNSUPPORTED, "spmm: buffers must be 16-B aligned");
  if (N <= 0) return HNM_OK;
  switch (d) {
    case 4: return spmm_launch<1>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 8: return spmm_launch<2>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 16: return spmm_launch<4>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 32: return spmm_launch<8>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 64: return spmm_launch<16>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 128: return spmm_launch<32>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    case 256: return spmm_launch<64>(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out);
    default:
      hnm_set_error("spmm: d must be one of 4, 8, 16, 32, 64, 128, 256 (got %d)", d);
      return HNM_EUNSUPPORTED;
  }
}
