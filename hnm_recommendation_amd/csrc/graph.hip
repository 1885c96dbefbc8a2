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
#include <cstring>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

#include "hnm_device.h"
#include "hnm_internal.h"

// Fixed design constants (round 5: the measured-and-dropped A/B switches of rounds 2-4 --
// walk launch order / side stream, record prefetch in the long-row walk, column windows in the
// short walk, the CSR-order short rows, ... -- are gone; DESIGN.md §4 keeps their numbers).
//
// Row classes by entry count L (self-loop included), decided per row so that every kernel that
// sums a row (the layer kernels, rows_combine) uses the same order:
//   short  L <= SPMM_SHORT           one LPR-lane group per row, 64 / LPR rows per wave
//   long   SPMM_SHORT < L <= HEAVY   one wave per row (4 neighbour groups + a fixed tree)
//   heavy  L > HEAVY                 SEG-long segments + a finish kernel
// Graphs of up to 2^22 nodes (every BASELINE graph) run the two walks below instead: short rows
// by the column-ordered short walk, the others by the user-ordered walk; the classes above
// remain the plan-less path and the path of larger graphs (both tested).
#define HEAVY 2048
#define SEG 2048
#define SPMM_SHORT 128
// the long-row walk: 1024-thread workgroups (one per CU), 144 KiB of float4 row accumulators,
// lists cut at WALK_WIN column windows with a workgroup barrier after each (d=64 layer: no
// windows 1.635 ms, 4: 1.499, 8: 1.448, 16: 1.431-1.451, 32: 1.474), WALK_STEP entries a step
// (round 4, whole-graph layer d=64 / d=128: 4 entries 1.308 / 2.676 ms, 4 + records prefetched a
// step ahead 1.415 / 2.920, 8 entries 1.435 / 3.017), pieces cut for ~WALK_GROUPS_TARGET groups
#define WALK_THREADS 1024
#define WALK_WIN 12
// d >= 128 (512-B rows): more, narrower windows (round 6, A/B on one box, configs[4] d = 128
// step: 16 windows 7.09 ms, 24: 7.01, 32: 7.02, 64: 7.29; the d = 64 step: 8: 3.464, 12: 3.462,
// 16: 3.474, 32: 3.58 -- profiles/r11d_spmm_windows_ab.txt)
#define WALK_WIN_WIDE 24
static inline int walk_windows(int d) { return d >= 128 ? WALK_WIN_WIDE : WALK_WIN; }
#define WALK_STEP 4
#define WALK_LDS_F4 9216
#define WALK_GROUPS_TARGET 16384
// the short walk (round 4): 2 persistent 512-thread workgroups per CU, 72 KiB of float4 row
// accumulators each, 8 entries a step with the records loaded a step ahead.  Measured and
// dropped (A/B on one box, d = 64 layer, `git show a7c47dc`): the short rows one lane group
// each in CSR order 1.44 ms, two rows per group interleaved 1.72 ms, the ~600 most gathered item
// rows held in LDS 1.46-1.65 ms, column windows with barriers 1.537 / 1.602 ms (4 / 8 windows),
// vs 1.305 ms for this walk.
#define SWALK_WG_PER_CU 2
#define SWALK_THREADS 512
#define SWALK_LDS_F4 4608
#define SWALK_STEP 8
// d >= 128 (LPR >= 32): 4 entries a step (round 6, A/B on one box: configs[4] d = 128 step
// 7.02 -> 6.94 ms; 2 entries 7.33-7.37, 16 entries 8.21; d = 64 the same at 4 and 8; the long
// walk's WALK_STEP at d = 128: 2 entries 8.42, 8 entries 7.79 vs 6.94 ms at 4 --
// profiles/r11f_swalk_step_ab.txt)
#define SWALK_STEP_WIDE 4
__host__ __device__ constexpr int swalk_step(int lpr) { return lpr >= 32 ? SWALK_STEP_WIDE : SWALK_STEP; }
// Round 4, measured and dropped: aligning the workgroups of an XCD -- a bounded wait (per-XCD
// progress counters, atomics at agent scope) before each short-walk round until all but 1/8 of
// the XCD's workgroups finished the previous one, and the same before each of the long-row
// walk's column windows -- so their gathers share one window of the table in that L2: d=64
// layer 1.304 -> 1.586 ms (short walk aligned), 1.430 (walk windows), 1.699 (both); d=128
// 2.672 -> 3.235 / 2.680 / 3.237 ms.  The waits cost more than the L2 locality returns.
// (tools/gather_probe.hip: uniformly random 256-B rows gather at 8.4-8.6 TB/s from a 27 MB
// table and 7.0-7.3 TB/s from 351 MB whatever the loads in flight, 23 TB/s from an
// L2-resident 4 MB one; the two walks' 12.8 TB/s lies between: their column order already
// serves ~62 % of the gathered bytes from L2.  Round 5, tools/granule_probe.hip: gathers of
// column slices -- 32 / 64 / 128-B granules from slice tables of 3.4 / 6.8 / 13.5 MB -- run at
// 4.3 / 5.3 / 8.8 TB/s, below the walks' rate: slicing the item table per XCD cannot pay.)
// Also measured and dropped (round 4): the long-row walk split by XCD column ranges (668 ->
// 1,155 us a launch: ~4x the pieces for the same LDS slots), and the walk on the side stream
// beside the short rows (1.318 / 2.928 ms vs 1.308 / 2.676).

struct WalkSched;
struct ShortSched;

struct hnm_spmm_plan {
  int device;
  int num_cus;
  int64_t N, nnz;
  std::vector<int64_t>* h_rowptr;
  int64_t n_heavy;
  int64_t n_seg;
  int32_t* heavy_rows;  // [n_heavy]
  int64_t n_long;
  int32_t* long_rows;   // [n_long] rows of the long class, ascending (SPMM_SHORT > 0)
  std::vector<int32_t>* h_long;
  int64_t* seg_ptr;     // [n_heavy + 1]
  int32_t* seg_hrow;    // [n_seg]  index into heavy_rows
  int64_t* seg_start;   // [n_seg]
  int64_t* seg_end;     // [n_seg]
  std::vector<int32_t>* h_heavy;  // host copies (row-range launches)
  std::vector<int64_t>* h_seg_ptr;
  // user-ordered walk of the rows of more than SPMM_SHORT entries
  int walk;
  int swalk;            // short rows by the column-ordered short walk
  int64_t walk_cap;     // entries per piece: a row of L entries is cut into cdiv(L, cap) pieces
  int64_t n_walk, walk_nnz;
  std::vector<int32_t>* h_walk_rows;  // ascending
  std::vector<int32_t>* h_short_rows; // rows of <= SPMM_SHORT entries, ascending
  // The graph values the plan is bound to (first prepare / SpMM / rows_combine call): every
  // row's entries sorted by (col, CSR position) in CSR layout, on the device (rows_combine) and
  // on the host (schedule builds).  Later calls must pass the same col / val pointers.
  const int32_t* bound_col;
  const float* bound_val;
  int32_t* scol;
  float* sval;
  std::vector<int32_t>* h_scol;
  std::vector<float>* h_sval;
  std::mutex* mu;       // lazy preparation (first call with col/val, first call per d)
  WalkSched* sched[7];  // per d = 4 << i
  ShortSched* ssched[7];
  // hnm_spmm_plan_restrict: the row ranges [keep[2j], keep[2j+1]) this plan computes (NULL: all)
  std::vector<int64_t>* keep;
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
  HNM_CTX_DEVICE(ctx);
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
// (A variant issuing a whole batch of indices and then all row gathers before consuming
// any -- no serial remainder loop -- measured 3 % slower per layer: 2.145 vs 2.087 ms.)
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

// Epilogue of row r (layer combine, lightgcn.py:156-158): Y[r] = y and, for rows with an
// accumulator (r >= acc_row0), acc_out = fma(alpha, y, acc_in) where acc_in == NULL means
// beta * X[r] (the alpha_0 E_0 term folded into layer 1).  Accumulators are stored from
// row acc_row0 on (items only when acc_row0 = num_users).
struct SpmmEpi {
  float* Y;
  float alpha, beta;
  const float* acc_in;
  float* acc_out;
  int64_t acc_row0;
};

__device__ __forceinline__ void spmm_epilogue(int64_t r, int d, int sub, float4 y,
                                              const float* __restrict__ X, const SpmmEpi& ep) {
  const int64_t off = r * d + 4 * sub;
  if (ep.Y) *reinterpret_cast<float4*>(ep.Y + off) = y;
  if (ep.acc_out && r >= ep.acc_row0) {
    const int64_t ao = (r - ep.acc_row0) * d + 4 * sub;
    float4 a;
    if (ep.acc_in) {
      a = *reinterpret_cast<const float4*>(ep.acc_in + ao);
    } else if (ep.beta != 0.f) {
      const float4 x = *reinterpret_cast<const float4*>(X + off);
      a = make_float4(ep.beta * x.x, ep.beta * x.y, ep.beta * x.z, ep.beta * x.w);
    } else {
      a = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    a.x = fmaf(ep.alpha, y.x, a.x);
    a.y = fmaf(ep.alpha, y.y, a.y);
    a.z = fmaf(ep.alpha, y.z, a.z);
    a.w = fmaf(ep.alpha, y.w, a.w);
    *reinterpret_cast<float4*>(ep.acc_out + ao) = a;
  }
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm_light_kernel(int64_t r0, int64_t r1,
                                                         const int64_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col,
                                                         const float* __restrict__ val,
                                                         const float* __restrict__ X, int d,
                                                         SpmmEpi ep, int64_t heavy) {
  const int64_t r = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= r1) return;
  const int lane = threadIdx.x & 63;
  const int64_t s = rowptr[r], e = rowptr[r + 1];
  if (e - s > heavy) return;  // segmented path
  const float4 y = row_sum<LPR>(col, val, X, d, s, e, lane);
  if (lane < LPR) spmm_epilogue(r, d, lane, y, X, ep);
}

// Grouped light rows: lane group g = lane / LPR owns row r, lane sub = lane % LPR its float4
// column; the group walks the row's entries in order (4 loads in flight per group, 64 / LPR
// rows per wave) with one fma chain per column -- no cross-group tree.
template <int LPR>
__device__ __forceinline__ float4 row_sum_grouped(const int32_t* __restrict__ col,
                                                  const float* __restrict__ val,
                                                  const float* __restrict__ X, int d, int64_t s,
                                                  int64_t e, int sub) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t p = s;
  for (; p + 3 < e; p += 4) {
    int c[4];
    float w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = col[p + u];
      w[u] = val[p + u];
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
  for (; p < e; ++p) {
    const int c = col[p];
    const float w = val[p];
    const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)c * d + 4 * sub);
    acc.x = fmaf(w, x.x, acc.x);
    acc.y = fmaf(w, x.y, acc.y);
    acc.z = fmaf(w, x.z, acc.z);
    acc.w = fmaf(w, x.w, acc.w);
  }
  return acc;
}

// One launch for the light rows of [r0, r1): blocks [0, nlb) take the long rows listed in
// long_rows[l0, l1) (one wave per row, the light kernel's order; first, so the longest work
// starts first), the other blocks the short rows (one LPR-lane group per row), skipping rows
// of the other classes.
template <int LPR>
__global__ __launch_bounds__(256) void spmm_mixed_kernel(int64_t r0, int64_t r1,
                                                         const int32_t* __restrict__ long_rows,
                                                         int64_t l0, int64_t l1, int64_t nlb,
                                                         const int64_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col,
                                                         const float* __restrict__ val,
                                                         const float* __restrict__ X, int d,
                                                         SpmmEpi ep) {
  const int lane = threadIdx.x & 63;
  if ((int64_t)blockIdx.x < nlb) {
    const int64_t q = l0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= l1) return;
    const int64_t r = long_rows[q];
    const float4 y = row_sum<LPR>(col, val, X, d, rowptr[r], rowptr[r + 1], lane);
    if (lane < LPR) spmm_epilogue(r, d, lane, y, X, ep);
    return;
  }
  constexpr int RPW = 64 / LPR;
  const int sub = lane % LPR;
  const int64_t r = r0 + ((int64_t)(blockIdx.x - nlb) * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (r >= r1) return;
  const int64_t s = rowptr[r], e = rowptr[r + 1];
  if (e - s > SPMM_SHORT) return;  // long / heavy class
  spmm_epilogue(r, d, sub, row_sum_grouped<LPR>(col, val, X, d, s, e, sub), X, ep);
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm_segment_kernel(int64_t sg0, int64_t sg1,
                                                           const int64_t* __restrict__ seg_start,
                                                           const int64_t* __restrict__ seg_end,
                                                           const int32_t* __restrict__ col,
                                                           const float* __restrict__ val,
                                                           const float* __restrict__ X, int d,
                                                           float* __restrict__ partial) {
  const int64_t sg = sg0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= sg1) return;
  const int lane = threadIdx.x & 63;
  const float4 y = row_sum<LPR>(col, val, X, d, seg_start[sg], seg_end[sg], lane);
  if (lane < LPR) *reinterpret_cast<float4*>(partial + (sg - sg0) * d + 4 * lane) = y;
}

// One workgroup per heavy row: thread (slice, c) sums float4 column c of the row's segment
// partials sg = slice, slice + S, ... in order, then a fixed-order LDS tree over the S
// slices (deterministic; all 256 lanes busy instead of d/4 lanes walking every segment).
__global__ __launch_bounds__(256) void spmm_finish_kernel(int64_t h0,
                                                          const int32_t* __restrict__ heavy_rows,
                                                          const int64_t* __restrict__ seg_ptr,
                                                          int64_t sg0,
                                                          const float* __restrict__ partial,
                                                          const float* __restrict__ X, int d,
                                                          SpmmEpi ep) {
  __shared__ float4 red[256];
  const int64_t hr = h0 + blockIdx.x;
  const int t = threadIdx.x;
  const int d4 = d / 4;
  const int S = 256 / d4;  // d4 divides 256 (d in 4..256, powers of two)
  const int c = t % d4, sl = t / d4;
  const int64_t s0 = seg_ptr[hr] - sg0, s1 = seg_ptr[hr + 1] - sg0;
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t sg = s0 + sl; sg < s1; sg += S) {
    const float4 v = *reinterpret_cast<const float4*>(partial + sg * d + 4 * c);
    y.x += v.x;
    y.y += v.y;
    y.z += v.z;
    y.w += v.w;
  }
  red[t] = y;
  __syncthreads();
  for (int w = S / 2; w >= 1; w >>= 1) {
    if (sl < w) {
      const float4 o = red[t + w * d4];
      float4 m = red[t];
      m.x += o.x;
      m.y += o.y;
      m.z += o.z;
      m.w += o.w;
      red[t] = m;
    }
    __syncthreads();
  }
  if (sl == 0) spmm_epilogue((int64_t)heavy_rows[hr], d, c, red[t], X, ep);
}

// ---------------------------------------------------------------- user-ordered walk
// Rows of more than SPMM_SHORT entries (the item half: each item row gathers ~300 random rows
// of the 351 MB user table) as ONE persistent launch whose gathers move through the table in
// ascending column order.  Each walk row's entries are sorted by (col, CSR position) and cut
// into pieces: a row of L entries has n = cdiv(L, cap) pieces, piece j holding the sorted
// entries j, j + n, j + 2n, ... (so every piece spans the whole column range).  A workgroup
// (one per CU, 1024 threads) owns up to maxloc pieces with their fp32 accumulators in LDS;
// each LPR-lane group walks ONE list -- its pieces' entries merged by column, packed as
// col << 10 | slot -- and adds val * X[col] into the slot's accumulator.  All lists of the
// chip advance through the columns at the same pace, so the rows gathered at any moment lie
// in a narrow window of X that the XCD L2s hold: measured on the synthetic H&M item half
// (tools/slice_walk_probe.hip) 0.85 ms vs 1.16 ms for the segmented pull in CSR order.
// Order: piece j = fma chain from 0 over its entries in (col, position) order; y = p_0 for an
// unsplit row, else per-slice sums of the pieces and a fixed tree (spmm_walk_finish_kernel);
// rows_combine repeats it from wcol / wval (walk_row_sum), so listed rows stay bitwise equal
// to the layer kernels.
template <int LPR>
__global__ __launch_bounds__(WALK_THREADS) void spmm_walk_kernel(
    const int64_t* __restrict__ gptr, const uint32_t* __restrict__ ent,
    const float* __restrict__ wt, const int32_t* __restrict__ slot_out,
    const int32_t* __restrict__ nslot, int maxloc, int nwin, const float* __restrict__ X, int d,
    float* __restrict__ partial, SpmmEpi ep, int64_t r0, int64_t r1) {
  constexpr int NG = WALK_THREADS / LPR;
  __shared__ float4 acc[WALK_LDS_F4];
  const int tid = threadIdx.x, g = tid / LPR, sub = tid % LPR;
  const int ns = nslot[blockIdx.x];
  for (int i = tid; i < ns * LPR; i += WALK_THREADS) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  // WALK_STEP entries per step (round 3: 2: 1.741 ms per d=64 layer, 4: 1.694, 8: 1.848)
  const int K = nwin;  // column windows (walk_windows)
  constexpr int ST = WALK_STEP;
  auto consume = [&](const uint32_t* c, const float* w) {
    float4 x[ST];
#pragma unroll
    for (int u = 0; u < ST; ++u)
      x[u] = *reinterpret_cast<const float4*>(X + (int64_t)(c[u] >> 10) * d + 4 * sub);
#pragma unroll
    for (int u = 0; u < ST; ++u) {  // in list order: a slot's entries stay one fma chain
      float4* a = &acc[(c[u] & 1023u) * LPR + sub];
      float4 v = *a;
      v.x = fmaf(w[u], x[u].x, v.x);
      v.y = fmaf(w[u], x[u].y, v.y);
      v.z = fmaf(w[u], x[u].z, v.z);
      v.w = fmaf(w[u], x[u].w, v.w);
      *a = v;
    }
  };
  for (int k = 0; k < K; ++k) {
    int64_t p = gptr[((int64_t)blockIdx.x * NG + g) * K + k];
    const int64_t e = gptr[((int64_t)blockIdx.x * NG + g) * K + k + 1];
    for (; p + ST - 1 < e; p += ST) {
      uint32_t c[ST];
      float w[ST];
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        c[u] = ent[p + u];
        w[u] = wt[p + u];
      }
      consume(c, w);
    }
    for (; p < e; ++p) {
      const uint32_t c = ent[p];
      const float w = wt[p];
      const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)(c >> 10) * d + 4 * sub);
      float4* a = &acc[(c & 1023u) * LPR + sub];
      float4 v = *a;
      v.x = fmaf(w, x.x, v.x);
      v.y = fmaf(w, x.y, v.y);
      v.z = fmaf(w, x.z, v.z);
      v.w = fmaf(w, x.w, v.w);
      *a = v;
    }
    if (K > 1) __syncthreads();
  }
  __syncthreads();
  for (int i = tid; i < ns * LPR; i += WALK_THREADS) {
    const int o = slot_out[(int64_t)blockIdx.x * maxloc + i / LPR], c = i % LPR;
    if (o >= 0) {
      if (o >= r0 && o < r1) spmm_epilogue(o, d, c, acc[i], X, ep);
    } else {
      *reinterpret_cast<float4*>(partial + (int64_t)(-o - 1) * d + 4 * c) = acc[i];
    }
  }
}

// ------------------------------------------------------------- short walk (round 4)
// Rows of at most SPMM_SHORT entries (every user row of the bipartite graph: ~24 entries
// gathering the 27 MB item table at d=64) in blocks of up to S consecutive rows.  A persistent
// workgroup (one per CU) takes blocks b0 + blockIdx.x, + gridDim.x, ...; the block's rows hold
// their fp32 accumulators in LDS (slot = row - first row of the block, spare slot S for
// padding), each LPR-lane group owns a set of the block's rows and walks their entries merged by
// column (col << 10 | slot records, padded to 4 per list), adding val * X[col] into the slot.
// Every block's lists span the same column range at a similar pace, so the rows the 32 CUs of
// an XCD gather at any moment lie in a narrow window of the item table that their L2 holds.
// Order: row r's value is one fma chain from 0 over its entries sorted by (col, CSR position)
// -- rows_combine repeats it over the plan's sorted copy (row_sum_grouped on scol / sval).
template <int LPR>
__global__ __launch_bounds__(SWALK_THREADS) void spmm_swalk_kernel(
    const int64_t* __restrict__ gptr, const uint32_t* __restrict__ ent,
    const float* __restrict__ wt, const int32_t* __restrict__ srow,
    const int32_t* __restrict__ nslot, int S, const float* __restrict__ X, int d, SpmmEpi ep,
    int64_t r0, int64_t r1, int64_t b0, int64_t b1) {
  constexpr int NG = SWALK_THREADS / LPR;
  constexpr int ST = swalk_step(LPR);
  __shared__ float4 acc[SWALK_LDS_F4];
  const int tid = threadIdx.x, g = tid / LPR, sub = tid % LPR;
  for (int i = tid; i < SWALK_LDS_F4; i += SWALK_THREADS) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  auto consume = [&](const uint32_t* c, const float* w) {
    float4 x[ST];
#pragma unroll
    for (int u = 0; u < ST; ++u)
      x[u] = *reinterpret_cast<const float4*>(X + (int64_t)(c[u] >> 10) * d + 4 * sub);
#pragma unroll
    for (int u = 0; u < ST; ++u) {  // list order: a slot's entries stay one fma chain
      float4* a = &acc[(c[u] & 1023u) * LPR + sub];
      float4 v = *a;
      v.x = fmaf(w[u], x[u].x, v.x);
      v.y = fmaf(w[u], x[u].y, v.y);
      v.z = fmaf(w[u], x[u].z, v.z);
      v.w = fmaf(w[u], x[u].w, v.w);
      *a = v;
    }
  };
  for (int64_t b = b0 + blockIdx.x; b < b1; b += gridDim.x) {
    int64_t p = gptr[b * NG + g];
    const int64_t e = gptr[b * NG + g + 1];  // lists are padded to multiples of ST
    // the next step's records are loaded before this step's gathers
    uint32_t c[ST], cn[ST];
    float w[ST], wn[ST];
    if (p < e) {
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        cn[u] = ent[p + u];
        wn[u] = wt[p + u];
      }
    }
    for (; p < e; p += ST) {
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        c[u] = cn[u];
        w[u] = wn[u];
      }
      if (p + ST < e) {
#pragma unroll
        for (int u = 0; u < ST; ++u) {
          cn[u] = ent[p + ST + u];
          wn[u] = wt[p + ST + u];
        }
      }
      consume(c, w);
    }
    __syncthreads();
    const int ns = nslot[b];
    for (int i = tid; i < ns * LPR; i += SWALK_THREADS) {
      const int64_t r = srow[b * S + i / LPR];
      if (r >= r0 && r < r1) spmm_epilogue(r, d, i % LPR, acc[i], X, ep);
      acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
  }
}

// Split rows, one workgroup per row: thread (slice sl, column c) sums pieces sl, sl + S, ...
// (S = 256 / (d/4) slices) in order from 0, then the fixed pairwise tree over the slices, as
// spmm_finish_kernel does for segments (a per-row sequential sum over ~1,500 pieces of the most
// popular item took 70 us).
__global__ __launch_bounds__(256) void spmm_walk_finish_kernel(
    const int32_t* __restrict__ split_rows, const int64_t* __restrict__ split_ptr,
    const float* __restrict__ partial, const float* __restrict__ X, int d, SpmmEpi ep,
    int64_t r0, int64_t r1) {
  __shared__ float4 red[256];
  const int64_t r = split_rows[blockIdx.x];
  if (r < r0 || r >= r1) return;  // uniform
  const int t = threadIdx.x, d4 = d / 4, S = 256 / d4, c = t % d4, sl = t / d4;
  const int64_t a = split_ptr[blockIdx.x], n = split_ptr[blockIdx.x + 1] - a;
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t j = sl;
  for (; j + 3 * S < n; j += 4 * S) {  // 4 loads in flight, added in piece order
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(partial + (a + j + u * S) * d + 4 * c);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      y.x += v[u].x;
      y.y += v[u].y;
      y.z += v[u].z;
      y.w += v[u].w;
    }
  }
  for (; j < n; j += S) {
    const float4 v = *reinterpret_cast<const float4*>(partial + (a + j) * d + 4 * c);
    y.x += v.x;
    y.y += v.y;
    y.z += v.z;
    y.w += v.w;
  }
  red[t] = y;
  __syncthreads();
  for (int w = S / 2; w >= 1; w >>= 1) {
    if (sl < w) {
      const float4 o = red[t + w * d4];
      float4 m = red[t];
      m.x += o.x;
      m.y += o.y;
      m.z += o.z;
      m.w += o.w;
      red[t] = m;
    }
    __syncthreads();
  }
  if (sl == 0) spmm_epilogue(r, d, c, red[t], X, ep);
}

// Walk order of one row for a listed-row kernel (the whole wave calls it; valid in lanes <
// LPR): the pieces' fma chains over the sorted entries; one piece -> its chain; several ->
// the finish kernel's slices (S = 256 / LPR, pieces sl, sl + S, ... from 0) and pairwise tree.
template <int LPR>
__device__ float4 walk_row_sum(const int32_t* __restrict__ wcol, const float* __restrict__ wval,
                               int64_t ws, int64_t L, int64_t cap, const float* __restrict__ X,
                               int d, int lane, float4* red) {
  constexpr int S = 256 / LPR;
  const int sub = lane % LPR;
  const int64_t n = hnm_cdiv(L, cap);
  auto chain = [&](int64_t j) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t q = j; q < L; q += n) {
      const float w = wval[ws + q];
      const float4 x = *reinterpret_cast<const float4*>(X + (int64_t)wcol[ws + q] * d + 4 * sub);
      v.x = fmaf(w, x.x, v.x);
      v.y = fmaf(w, x.y, v.y);
      v.z = fmaf(w, x.z, v.z);
      v.w = fmaf(w, x.w, v.w);
    }
    return v;
  };
  if (n == 1) return chain(0);
  for (int sl = 0; sl < S; ++sl) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t j = sl; j < n; j += S) {
      const float4 v = chain(j);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (lane < LPR) red[sl * LPR + lane] = acc;
  }
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane < LPR) {
    for (int w = S / 2; w >= 1; w >>= 1)
      for (int sl = 0; sl < w; ++sl) {
        const float4 o = red[(sl + w) * LPR + lane];
        float4 m = red[sl * LPR + lane];
        m.x += o.x;
        m.y += o.y;
        m.z += o.z;
        m.w += o.w;
        red[sl * LPR + lane] = m;
      }
    y = red[lane];
  }
  return y;
}

// Final embeddings of listed rows (the batch's users) without their last layer over the
// whole graph: y = (A_hat E_{L-1})[r], out[b] = alpha_0 E_0[r] then
// fma(alpha_l, E_l[r], .) for l = 1..L-1 and fma(alpha_L, y, .) -- the same operations, in
// the same order, as the fused combine.  y is summed in the order the planned SpMM uses for
// that row: the light kernel's order for rows of <= HEAVY neighbours; for longer rows the
// SEG-long segments (row_sum each, as spmm_segment_kernel), S = 256 / LPR slices summing
// segments sl, sl + S, ... in order from 0, then the pairwise tree over the slices
// (w = S/2 .. 1), as spmm_finish_kernel does -- so listed heavy rows are bitwise equal to
// forward() too.  Each lane only touches its own float4 column of the slice sums (LDS, one
// S x LPR block per wave), so the wave needs no barrier.  Every row is summed in the order of
// its class as the layer kernels of the same plan sum it (CombineOrder below).
struct CombineLayers {
  const float* E[8];
  float a[9];
  int L;
};

// y = (A_hat X)[r] for a row of more than HEAVY entries, in the plan's segment + finish
// order (see above); the whole wave works on the row, the result is valid in lanes < LPR.
template <int LPR>
__device__ float4 heavy_row_sum(const int32_t* __restrict__ col, const float* __restrict__ val,
                                const float* __restrict__ X, int d, int64_t rs, int64_t re,
                                int lane, float4* red) {
  constexpr int S = 256 / LPR;
  const int64_t nseg = hnm_cdiv(re - rs, SEG);
  for (int sl = 0; sl < S; ++sl) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t sg = sl; sg < nseg; sg += S) {
      const int64_t a = rs + sg * SEG, z = a + SEG < re ? a + SEG : re;
      const float4 v = row_sum<LPR>(col, val, X, d, a, z, lane);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (lane < LPR) red[sl * LPR + lane] = acc;
  }
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane < LPR) {
    for (int w = S / 2; w >= 1; w >>= 1)
      for (int sl = 0; sl < w; ++sl) {
        const float4 o = red[(sl + w) * LPR + lane];
        float4 m = red[sl * LPR + lane];
        m.x += o.x;
        m.y += o.y;
        m.z += o.z;
        m.w += o.w;
        red[sl * LPR + lane] = m;
      }
    y = red[lane];
  }
  return y;
}

// out[b] = alpha_0 E_0[r] + sum_l alpha_l E_l[r] (fma chain in layer order) + alpha_L y
__device__ __forceinline__ void combine_store(const CombineLayers& cl, int64_t r, int d, int sub,
                                              float4 y, float* __restrict__ out, int64_t b) {
  const int64_t off = r * d + 4 * sub;
  const float4 x0 = *reinterpret_cast<const float4*>(cl.E[0] + off);
  float4 a = make_float4(cl.a[0] * x0.x, cl.a[0] * x0.y, cl.a[0] * x0.z, cl.a[0] * x0.w);
  for (int l = 1; l < cl.L; ++l) {
    const float4 x = *reinterpret_cast<const float4*>(cl.E[l] + off);
    a.x = fmaf(cl.a[l], x.x, a.x);
    a.y = fmaf(cl.a[l], x.y, a.y);
    a.z = fmaf(cl.a[l], x.z, a.z);
    a.w = fmaf(cl.a[l], x.w, a.w);
  }
  const float aL = cl.a[cl.L];
  a.x = fmaf(aL, y.x, a.x);
  a.y = fmaf(aL, y.y, a.y);
  a.z = fmaf(aL, y.z, a.z);
  a.w = fmaf(aL, y.w, a.w);
  *reinterpret_cast<float4*>(out + b * d + 4 * sub) = a;
}

// The summation order rows_combine must repeat (the plan's): mode 0 plan-less (one wave per
// row, row_sum, every row: spmm_light_kernel with no heavy class); mode 1 a plan without the
// walks (short rows grouped in CSR order, long rows one wave, heavy rows segments); mode 2 a
// walk plan (long rows in the walk's piece order over the sorted copy scol / sval; short rows
// grouped over the sorted copy when the short walk is on, else over col / val).
struct CombineOrder {
  int mode;
  int short_sorted;
  const int32_t* scol;
  const float* sval;
  int64_t cap;
};

template <int LPR>
__global__ __launch_bounds__(256) void spmm_rows_combine_kernel(
    const int64_t* __restrict__ rows, int64_t n, int64_t N, const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const float* __restrict__ val, int d, CombineLayers cl,
    CombineOrder co, float* __restrict__ out, unsigned* err) {
  __shared__ float4 slices[4][256];
  const int lane = threadIdx.x & 63;
  const float* Xl = cl.E[cl.L - 1];
  if (co.mode == 0) {
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= n) return;
    const int64_t r = rows[b];
    if (r < 0 || r >= N) {
      if (lane == 0) hnm_flag(err, HNM_ERR_OOB);
      for (int c = lane; c < d; c += 64) out[b * d + c] = __builtin_nanf("");
      return;
    }
    const int64_t rs = rowptr[r], re = rowptr[r + 1];
    const float4 y = co.mode == 0 || re - rs <= HEAVY
                         ? row_sum<LPR>(col, val, Xl, d, rs, re, lane)
                         : heavy_row_sum<LPR>(col, val, Xl, d, rs, re, lane, slices[threadIdx.x >> 6]);
    if (lane < LPR) combine_store(cl, r, d, lane, y, out, b);
    return;
  }
  // grouped: group g = lane / LPR owns listed row b; short rows in the grouped order, long and
  // heavy rows afterwards by the whole wave (uniform loop over the wave's groups)
  constexpr int RPW = 64 / LPR;
  const int g = lane / LPR, sub = lane % LPR;
  const int64_t b0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (b0 >= n) return;
  const int64_t b = b0 + g;
  int64_t r = -1, rs = 0, re = 0;
  bool ok = false;
  const int32_t* scl = co.short_sorted ? co.scol : col;
  const float* svl = co.short_sorted ? co.sval : val;
  if (b < n) {
    r = rows[b];
    ok = r >= 0 && r < N;
    if (!ok) {
      if (sub == 0) hnm_flag(err, HNM_ERR_OOB);
      const float nan = __builtin_nanf("");
      *reinterpret_cast<float4*>(out + b * d + 4 * sub) = make_float4(nan, nan, nan, nan);
    } else {
      rs = rowptr[r];
      re = rowptr[r + 1];
      if (re - rs <= SPMM_SHORT)
        combine_store(cl, r, d, sub, row_sum_grouped<LPR>(scl, svl, Xl, d, rs, re, sub), out, b);
    }
  }
  // long and heavy rows: the whole wave, one row at a time
  uint64_t hm = __ballot(ok && re - rs > SPMM_SHORT && sub == 0);
  while (hm) {
    const int src = __builtin_ctzll(hm);
    hm &= hm - 1;
    const int64_t hb = b0 + src / LPR;
    const int64_t hr = rows[hb];
    const int64_t hs = rowptr[hr], he = rowptr[hr + 1];
    float4 y;
    if (co.mode == 2) {  // the walk's order (every row of this class is a walk row)
      y = walk_row_sum<LPR>(co.scol, co.sval, hs, he - hs, co.cap, Xl, d, lane,
                            slices[threadIdx.x >> 6]);
    } else {
      y = he - hs <= HEAVY
              ? row_sum<LPR>(col, val, Xl, d, hs, he, lane)
              : heavy_row_sum<LPR>(col, val, Xl, d, hs, he, lane, slices[threadIdx.x >> 6]);
    }
    if (lane < LPR) combine_store(cl, hr, d, lane, y, out, hb);
  }
}


// ---------------------------------------------------------------- walk schedules (host)
struct WalkSched {
  int lpr, ng, nwg, maxloc, nwin;
  int64_t* gptr;       // [nwg * ng * nwin + 1] (nwin column windows per group list)
  uint32_t* ent;       // [walk_nnz] col << 10 | slot
  float* wt;
  int32_t* slot_out;   // [nwg * maxloc]: row (unsplit piece) or -(partial index) - 1
  int32_t* nslot;      // [nwg]
  int64_t n_split, n_part;
  int32_t* split_rows;  // [n_split]
  int64_t* split_ptr;   // [n_split + 1] partial indices, pieces in order
};

static void walk_sched_free(WalkSched* w) {
  if (!w) return;
  (void)hipFree(w->gptr);
  (void)hipFree(w->ent);
  (void)hipFree(w->wt);
  (void)hipFree(w->slot_out);
  (void)hipFree(w->nslot);
  (void)hipFree(w->split_rows);
  (void)hipFree(w->split_ptr);
  delete w;
}

// short walk: nb blocks of up to S consecutive short rows, ng lists per block (K windows each)
struct ShortSched {
  int lpr, ng, S, nwg;
  int64_t nb;
  int64_t* gptr;     // [nb * ng + 1]
  uint32_t* ent;     // col << 10 | slot (slot S: padding, weight 0)
  float* wt;
  int32_t* srow;     // [nb * S] row of each slot
  int32_t* nslot;    // [nb]
  std::vector<int32_t> first, last;  // first / last row of each block (row-range launches)
};

static void short_sched_free(ShortSched* w) {
  if (!w) return;
  (void)hipFree(w->gptr);
  (void)hipFree(w->ent);
  (void)hipFree(w->wt);
  (void)hipFree(w->srow);
  (void)hipFree(w->nslot);
  delete w;
}

template <typename F>
static void parallel_for(int64_t n, F fn) {
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(
      std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency())), n / 64 + 1));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int64_t i = t; i < n; i += nt) fn(i);
    });
  for (auto& x : th) x.join();
}

template <typename T>
static hnm_status upload(T** dst, const T* src, size_t n) {
  if (hipMalloc((void**)dst, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
    *dst = nullptr;
    hnm_set_error("spmm walk: hipMalloc of %zu bytes failed", n * sizeof(T));
    return HNM_ENOMEM;
  }
  if (n) HNM_HIP_CHECK(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
  return HNM_OK;
}

// A bipartite graph stored with contiguous sides -- rows [0, S) connected only to [S, N) and
// back, self-loops aside (the reference's user / item layout, lightgcn.py:81-112) -- has one
// side whose rows all gather the OTHER side's table.  The short walk suits the side that gathers
// the smaller table (users: the 27 MB item table at d = 64); the short rows of the side that
// gathers the larger table (the tail items, < 129 entries into the 351 MB user table) join the
// user-ordered walk instead, where their gathers ride the same column sweep as the long item
// rows.  A short row is one piece there, so its value is the same sorted-order fma chain
// either way (rows_combine is unchanged).  Called once at binding, before any schedule.
static void plan_bipartite_sides(hnm_spmm_plan* pl) {
  const std::vector<int64_t>& rp = *pl->h_rowptr;
  const std::vector<int32_t>& hc = *pl->h_scol;
  const int64_t N = pl->N;
  // per row the smallest / largest neighbour other than itself (entries are column-sorted);
  // a split S is valid when every row below it only reaches [S, N) and every row from it on
  // only reaches [0, S): prefix min of the minima >= S and suffix max of the maxima < S
  std::vector<int64_t> mn((size_t)N), mx((size_t)N);
  parallel_for(hnm_cdiv(N, 4096), [&](int64_t ch) {
    const int64_t r1 = std::min<int64_t>(N, (ch + 1) * 4096);
    for (int64_t r = ch * 4096; r < r1; ++r) {
      int64_t lo = N, hi = -1;
      for (int64_t q = rp[r]; q < rp[r + 1]; ++q)
        if (hc[q] != r) {
          lo = std::min<int64_t>(lo, hc[q]);
          hi = std::max<int64_t>(hi, hc[q]);
        }
      mn[r] = lo;
      mx[r] = hi;
    }
  });
  std::vector<int64_t> smax((size_t)N + 1, -1);
  for (int64_t r = N - 1; r >= 0; --r) smax[r] = std::max(smax[r + 1], mx[r]);
  int64_t S = -1, pmin = N;
  for (int64_t c = 1; c < N; ++c) {
    pmin = std::min(pmin, mn[c - 1]);
    if (pmin >= c && smax[c] < c && pmin < N && smax[c] >= 0) {
      S = c;
      break;
    }
  }
  if (S <= 0) return;
  // the side whose neighbours form the larger table moves its short rows into the walk
  const bool upper = S > N - S;  // rows [S, N) gather the S-row table
  const int64_t lo = upper ? S : 0, hi = upper ? N : S;
  std::vector<int32_t>& sr = *pl->h_short_rows;
  std::vector<int32_t>& wr = *pl->h_walk_rows;
  std::vector<int32_t> keep, moved;
  for (int32_t r : sr) (r >= lo && r < hi && rp[r + 1] > rp[r] ? moved : keep).push_back(r);
  if (moved.empty() || keep.empty()) return;
  std::vector<int32_t> merged((size_t)(wr.size() + moved.size()));
  std::merge(wr.begin(), wr.end(), moved.begin(), moved.end(), merged.begin());
  for (int32_t r : moved) pl->walk_nnz += rp[r + 1] - rp[r];
  wr.swap(merged);
  sr.swap(keep);
  pl->n_walk = (int64_t)wr.size();
  pl->walk_cap = std::max<int64_t>(512, hnm_cdiv(pl->walk_nnz, 2 * WALK_GROUPS_TARGET));
}

// Binds the plan to col / val on first use.  A walk plan then copies the CSR to the host,
// stable-sorts every row's entries by column (the walks' summation order: (col, CSR position))
// and uploads the sorted copy (rows_combine repeats the walks' order from it).  Later calls
// must pass the same col / val: a plan snapshots the graph's values.  Caller holds pl->mu.
static hnm_status plan_bind(hnm_ctx* ctx, hnm_spmm_plan* pl, const int32_t* col, const float* val) {
  if (pl->bound_col) {
    HNM_REQUIRE(col == pl->bound_col && val == pl->bound_val, HNM_EINVAL,
                "spmm: this plan is bound to the col / val of its first use (it snapshots the "
                "graph's values); create a new plan for other values");
    return HNM_OK;
  }
  if (pl->walk) {
    const int64_t T = pl->nnz;
    const std::vector<int64_t>& rp = *pl->h_rowptr;
    std::vector<int32_t> c0((size_t)T);
    std::vector<float> v0((size_t)T);
    HNM_HIP_CHECK(hipMemcpyAsync(c0.data(), col, T * 4, hipMemcpyDeviceToHost, ctx->stream));
    HNM_HIP_CHECK(hipMemcpyAsync(v0.data(), val, T * 4, hipMemcpyDeviceToHost, ctx->stream));
    HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    // all-or-nothing: the host copies and device uploads are installed in the plan only when
    // every step succeeded, so a failed bind leaves the plan unbound and a retry starts clean
    std::unique_ptr<std::vector<int32_t>> hcp(new std::vector<int32_t>((size_t)T));
    std::unique_ptr<std::vector<float>> hvp(new std::vector<float>((size_t)T));
    std::vector<int32_t>& hc = *hcp;
    std::vector<float>& hv = *hvp;
    const int64_t nchunk = hnm_cdiv(pl->N, 4096);
    parallel_for(nchunk, [&](int64_t ch) {
      std::vector<int32_t> ix;
      const int64_t r1 = std::min<int64_t>(pl->N, (ch + 1) * 4096);
      for (int64_t r = ch * 4096; r < r1; ++r) {
        const int64_t a = rp[r], L = rp[r + 1] - a;
        ix.resize((size_t)L);
        for (int64_t q = 0; q < L; ++q) ix[q] = (int32_t)q;
        std::stable_sort(ix.begin(), ix.end(),
                         [&](int32_t x, int32_t y) { return c0[a + x] < c0[a + y]; });
        for (int64_t q = 0; q < L; ++q) {
          hc[a + q] = c0[a + ix[q]];
          hv[a + q] = v0[a + ix[q]];
        }
      }
    });
    int32_t* dcol = nullptr;
    float* dval = nullptr;
    hnm_status st = upload(&dcol, hc.data(), (size_t)T);
    if (!st) st = upload(&dval, hv.data(), (size_t)T);
    if (st) {
      if (dcol) (void)hipFree(dcol);
      return st;
    }
    pl->scol = dcol;
    pl->sval = dval;
    pl->h_scol = hcp.release();
    pl->h_sval = hvp.release();
    if (pl->swalk) plan_bipartite_sides(pl);
  }
  pl->bound_col = col;
  pl->bound_val = val;
  return HNM_OK;
}

// Schedule for d (LPR = d / 4 lanes per row): pieces to workgroups (greedy, longest first,
// least-loaded workgroup with a free slot), then to the workgroup's groups (least-loaded), then
// each group's pieces merged by column.  The placement only moves work between lanes; the
// order inside each piece (and so every result) is fixed by the pieces themselves.
static hnm_status walk_build(hnm_spmm_plan* pl, int d, WalkSched** out) {
  const int lpr = d / 4, ng = WALK_THREADS / lpr;
  // slot maxloc absorbs the windows' padding entries (never stored)
  const int maxloc = std::min(1022, WALK_LDS_F4 / lpr - 1);
  const std::vector<int64_t>& rp = *pl->h_rowptr;
  const std::vector<int32_t>& wr = *pl->h_walk_rows;
  const int64_t cap = pl->walk_cap, T = pl->walk_nnz;
  struct Piece {
    int32_t k;     // walk row
    int32_t j, n;  // piece j of n
    int64_t len;
  };
  std::vector<Piece> pcs;
  for (int64_t k = 0; k < pl->n_walk; ++k) {
    const int64_t L = rp[wr[k] + 1] - rp[wr[k]];
    const int n = (int)hnm_cdiv(L, cap);
    for (int j = 0; j < n; ++j) pcs.push_back({(int32_t)k, j, n, (L - j + n - 1) / n});
  }
  std::stable_sort(pcs.begin(), pcs.end(), [](const Piece& a, const Piece& b) { return a.len > b.len; });
  int64_t nwg = std::max<int64_t>(1, std::min<int64_t>(hnm_cdiv(WALK_GROUPS_TARGET, ng),
                                                        hnm_cdiv(T, (int64_t)ng * 256)));
  while ((int64_t)pcs.size() > nwg * maxloc * 7 / 8) nwg *= 2;
  // a walk of a few entries a group (a restricted plan's item shard: ~260 entries a group at
  // d = 128 for 1/8 of the H&M items) is bound by the per-window latency, not by its gathers:
  // one round of workgroups (one per CU) instead of a second partial round, when the slots hold
  // every piece (placement only moves pieces between lanes; every result is unchanged)
  const int64_t cus = std::max(1, pl->num_cus);
  if (nwg > cus && (int64_t)pcs.size() <= cus * maxloc * 7 / 8 && T <= cus * ng * 1024) nwg = cus;
  std::vector<std::vector<int32_t>> wgp((size_t)nwg);
  {
    using E = std::pair<int64_t, int64_t>;
    std::priority_queue<E, std::vector<E>, std::greater<E>> q;
    for (int64_t w = 0; w < nwg; ++w) q.push({0, w});
    for (int32_t pi = 0; pi < (int32_t)pcs.size(); ++pi) {
      E t = q.top();
      q.pop();
      while ((int64_t)wgp[t.second].size() >= maxloc) {  // full: drop it from the heap
        t = q.top();
        q.pop();
      }
      wgp[t.second].push_back(pi);
      q.push({t.first + pcs[pi].len, t.second});
    }
  }
  // partial indices of split rows: row k's pieces j = 0..n-1 at split_ptr[si] + j
  std::vector<int32_t> srows;
  std::vector<int64_t> sptr{0}, kpart((size_t)pl->n_walk, -1);
  for (int64_t k = 0; k < pl->n_walk; ++k) {
    const int n = (int)hnm_cdiv(rp[wr[k] + 1] - rp[wr[k]], cap);
    if (n <= 1) continue;
    kpart[k] = sptr.back();
    srows.push_back(wr[k]);
    sptr.push_back(sptr.back() + n);
  }
  std::vector<int32_t> slot_out((size_t)(nwg * maxloc), 0), nslot((size_t)nwg);
  std::vector<std::vector<std::vector<int32_t>>> gslots((size_t)nwg);
  for (int64_t w = 0; w < nwg; ++w) {
    nslot[w] = (int32_t)wgp[w].size();
    gslots[w].resize(ng);
    std::vector<int64_t> gl((size_t)ng, 0);
    for (int sl = 0; sl < (int)wgp[w].size(); ++sl) {
      const Piece& pc = pcs[wgp[w][sl]];
      const int gb = (int)(std::min_element(gl.begin(), gl.end()) - gl.begin());
      gslots[w][gb].push_back(sl);
      gl[gb] += pc.len;
      slot_out[w * maxloc + sl] = pc.n == 1 ? wr[pc.k] : (int32_t)(-(kpart[pc.k] + pc.j) - 1);
    }
  }
  // each group's list is cut at K column bounds (k + 1) * cdiv(N, K), each window padded to a
  // multiple of 4 entries; the kernel syncs its groups after every window
  const int K = walk_windows(d);
  const int64_t wlen = hnm_cdiv(pl->N, K);
  const std::vector<int32_t>& hc = *pl->h_scol;
  const std::vector<float>& hv = *pl->h_sval;
  std::vector<int64_t> wcnt((size_t)(nwg * ng * K), 0);
  parallel_for(nwg, [&](int64_t w) {
    for (int g = 0; g < ng; ++g)
      for (int sl : gslots[w][g]) {
        const Piece& pc = pcs[wgp[w][sl]];
        const int64_t a = rp[wr[pc.k]], L = rp[wr[pc.k] + 1] - a;
        for (int64_t q = pc.j; q < L; q += pc.n) ++wcnt[(w * ng + g) * K + hc[a + q] / wlen];
      }
  });
  std::vector<int64_t> gptr((size_t)(nwg * ng * K + 1), 0);
  for (int64_t i = 0; i < nwg * ng * K; ++i)
    gptr[i + 1] = gptr[i] + (K > 1 ? hnm_cdiv(wcnt[i], WALK_STEP) * WALK_STEP : wcnt[i]);
  const int64_t Tp = gptr.back();
  std::vector<uint32_t> ent((size_t)Tp, (uint32_t)maxloc);  // padding: col 0, spare slot, 0.0
  std::vector<float> wt((size_t)Tp, 0.f);
  parallel_for(nwg, [&](int64_t w) {
    std::vector<std::pair<uint64_t, float>> Lst;
    for (int g = 0; g < ng; ++g) {
      Lst.clear();
      for (int sl : gslots[w][g]) {
        const Piece& pc = pcs[wgp[w][sl]];
        const int64_t a = rp[wr[pc.k]], L = rp[wr[pc.k] + 1] - a;
        for (int64_t q = pc.j; q < L; q += pc.n)
          Lst.push_back({((uint64_t)(uint32_t)hc[a + q] << 10) | (uint64_t)sl, hv[a + q]});
      }
      std::stable_sort(Lst.begin(), Lst.end(),
                       [](const auto& x, const auto& y) { return (x.first >> 10) < (y.first >> 10); });
      size_t i = 0;
      for (int k = 0; k < K; ++k) {
        int64_t o = gptr[(w * ng + g) * K + k];
        for (; i < Lst.size() && (int64_t)(Lst[i].first >> 10) / wlen == k; ++i) {
          ent[o] = (uint32_t)Lst[i].first;
          wt[o++] = Lst[i].second;
        }
      }
    }
  });
  WalkSched* ws = new WalkSched();
  memset(ws, 0, sizeof(WalkSched));
  ws->lpr = lpr;
  ws->ng = ng;
  ws->nwg = (int)nwg;
  ws->maxloc = maxloc;
  ws->nwin = K;
  ws->n_split = (int64_t)srows.size();
  ws->n_part = sptr.back();
  hnm_status st;
  if ((st = upload(&ws->gptr, gptr.data(), gptr.size())) || (st = upload(&ws->ent, ent.data(), ent.size())) ||
      (st = upload(&ws->wt, wt.data(), wt.size())) ||
      (st = upload(&ws->slot_out, slot_out.data(), slot_out.size())) ||
      (st = upload(&ws->nslot, nslot.data(), nslot.size())) ||
      (st = upload(&ws->split_rows, srows.data(), srows.size())) ||
      (st = upload(&ws->split_ptr, sptr.data(), sptr.size()))) {
    walk_sched_free(ws);
    return st;
  }
  *out = ws;
  return HNM_OK;
}

// Short-walk schedule for d: the short rows cut into nb blocks of consecutive rows at equal
// shares of their entries (at most S rows a block; nb a multiple of the persistent grid once the
// graph fills it), each block's rows dealt to its ng lane groups (longest first, least-loaded
// group), each group's rows' entries merged by column and padded to multiples of swalk_step with
// weight-0 entries into the spare slot S.  The placement only moves rows between lanes; each
// row's chain order is its sorted entries' order.
static hnm_status swalk_build(hnm_spmm_plan* pl, int d, ShortSched** out) {
  const int lpr = d / 4, ng = SWALK_THREADS / lpr;
  const int S = std::min(1022, SWALK_LDS_F4 / lpr - 1);
  const std::vector<int64_t>& rp = *pl->h_rowptr;
  const std::vector<int32_t>& sr = *pl->h_short_rows;
  const std::vector<int32_t>& hc = *pl->h_scol;
  const std::vector<float>& hv = *pl->h_sval;
  const int64_t ns = (int64_t)sr.size();
  const int64_t nwg_full = (int64_t)std::max(1, pl->num_cus) * SWALK_WG_PER_CU;
  std::vector<int64_t> cum((size_t)ns + 1, 0);
  for (int64_t i = 0; i < ns; ++i) cum[i + 1] = cum[i] + (rp[sr[i] + 1] - rp[sr[i]]);
  const int64_t total = cum[ns];
  int64_t nb0 = std::max<int64_t>(1, hnm_cdiv(ns, S));
  int64_t nb = nb0 >= nwg_full ? hnm_cdiv(nb0, nwg_full) * nwg_full : nb0;
  std::vector<int64_t> bstart;  // first short-row index of each block (+ end)
  for (;;) {
    bstart.assign(1, 0);
    int64_t i = 0;
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t target = total * (b + 1) / nb;
      int64_t j = i;
      while (j < ns && j - i < S && (b == nb - 1 || cum[j + 1] <= target || j == i)) ++j;
      i = j;
      bstart.push_back(i);
    }
    if (i >= ns) break;
    nb += nb >= nwg_full ? nwg_full : 1;  // the last block overflowed S rows
  }
  std::vector<int32_t> srow((size_t)(nb * S), -1), nslot((size_t)nb, 0);
  std::vector<int64_t> wcnt((size_t)(nb * ng), 0);
  std::vector<std::vector<std::vector<int32_t>>> gslot((size_t)nb);  // per block, per group: slots
  parallel_for(nb, [&](int64_t b) {
    const int64_t i0 = bstart[b], n = bstart[b + 1] - i0;
    nslot[b] = (int32_t)n;
    std::vector<int32_t> ord((size_t)n);
    for (int64_t s = 0; s < n; ++s) {
      srow[b * S + s] = sr[i0 + s];
      ord[s] = (int32_t)s;
    }
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) {
      return cum[i0 + x + 1] - cum[i0 + x] > cum[i0 + y + 1] - cum[i0 + y];
    });
    gslot[b].assign(ng, {});
    std::vector<int64_t> gl((size_t)ng, 0);
    for (int32_t s : ord) {
      const int g = (int)(std::min_element(gl.begin(), gl.end()) - gl.begin());
      gslot[b][g].push_back(s);
      gl[g] += cum[i0 + s + 1] - cum[i0 + s];
      const int32_t r = sr[i0 + s];
      wcnt[b * ng + g] += rp[r + 1] - rp[r];
    }
  });
  std::vector<int64_t> gptr((size_t)(nb * ng + 1), 0);
  for (int64_t i = 0; i < nb * ng; ++i)
    gptr[i + 1] = gptr[i] + hnm_cdiv(wcnt[i], swalk_step(lpr)) * swalk_step(lpr);
  const int64_t Tp = gptr.back();
  std::vector<uint32_t> ent((size_t)Tp, (uint32_t)S);
  std::vector<float> wt((size_t)Tp, 0.f);
  parallel_for(nb, [&](int64_t b) {
    const int64_t i0 = bstart[b];
    std::vector<std::pair<uint64_t, float>> Lst;
    for (int g = 0; g < ng; ++g) {
      Lst.clear();
      std::vector<int32_t> sl = gslot[b][g];
      std::sort(sl.begin(), sl.end());
      for (int32_t s : sl) {
        const int32_t r = sr[i0 + s];
        for (int64_t q = rp[r]; q < rp[r + 1]; ++q)
          Lst.push_back({((uint64_t)(uint32_t)hc[q] << 10) | (uint64_t)s, hv[q]});
      }
      std::stable_sort(Lst.begin(), Lst.end(),
                       [](const auto& x, const auto& y) { return (x.first >> 10) < (y.first >> 10); });
      int64_t o = gptr[b * ng + g];
      const int64_t e = gptr[b * ng + g + 1];
      uint32_t pad = (uint32_t)S;
      for (size_t i = 0; i < Lst.size(); ++i) {
        ent[o] = (uint32_t)Lst[i].first;
        wt[o++] = Lst[i].second;
        pad = (uint32_t)((Lst[i].first >> 10) << 10) | (uint32_t)S;  // re-gather a cached row
      }
      for (; o < e; ++o) ent[o] = pad;
    }
  });
  ShortSched* ws = new ShortSched();
  ws->lpr = lpr;
  ws->ng = ng;
  ws->S = S;
  ws->nb = nb;
  ws->nwg = (int)std::min<int64_t>(nb, nwg_full);
  ws->gptr = nullptr;
  ws->ent = nullptr;
  ws->wt = nullptr;
  ws->srow = nullptr;
  ws->nslot = nullptr;
  ws->first.resize((size_t)nb);
  ws->last.resize((size_t)nb);
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t n = bstart[b + 1] - bstart[b];
    ws->first[b] = n ? sr[bstart[b]] : (b ? ws->last[b - 1] : 0);
    ws->last[b] = n ? sr[bstart[b + 1] - 1] : ws->first[b];
  }
  hnm_status st;
  if ((st = upload(&ws->gptr, gptr.data(), gptr.size())) || (st = upload(&ws->ent, ent.data(), ent.size())) ||
      (st = upload(&ws->wt, wt.data(), wt.size())) || (st = upload(&ws->srow, srow.data(), srow.size())) ||
      (st = upload(&ws->nslot, nslot.data(), nslot.size()))) {
    short_sched_free(ws);
    return st;
  }
  *out = ws;
  return HNM_OK;
}

static int walk_index(int d) {
  int i = 0;
  while ((4 << i) < d) ++i;
  return i;
}

static bool spmm_d_ok(int d) {
  for (int i = 0; i < 7; ++i)
    if (d == (4 << i)) return true;
  return false;
}

// Binding + the walk schedules for d, built on first use (one-time, host work with stream syncs).
static hnm_status walk_get(hnm_ctx* ctx, const hnm_spmm_plan* cpl, const int32_t* col,
                           const float* val, int d, const WalkSched** out,
                           const ShortSched** sout) {
  hnm_spmm_plan* pl = const_cast<hnm_spmm_plan*>(cpl);
  std::lock_guard<std::mutex> lk(*pl->mu);
  hnm_status s = plan_bind(ctx, pl, col, val);
  if (s) return s;
  if (!pl->walk || d <= 0) return HNM_OK;
  const int i = walk_index(d);
  if (!pl->sched[i] && (s = walk_build(pl, d, &pl->sched[i]))) return s;
  if (pl->swalk && !pl->ssched[i] && (s = swalk_build(pl, d, &pl->ssched[i]))) return s;
  if (out) *out = pl->sched[i];
  if (sout) *sout = pl->ssched[i];
  return HNM_OK;
}

extern "C" hnm_status hnm_spmm_plan_create(hnm_ctx* ctx, int64_t N, const int64_t* rowptr,
                                           hnm_spmm_plan** out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && rowptr && out && N > 0, HNM_EINVAL, "spmm_plan: bad argument");
  std::vector<int64_t> rp((size_t)N + 1);
  HNM_HIP_CHECK(hipMemcpyAsync(rp.data(), rowptr, (N + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  std::vector<int32_t> hrows, shrow;
  std::vector<int64_t> sptr{0}, sstart, send;
  std::vector<int32_t> lrows;
  for (int64_t r = 0; r < N; ++r) {
    const int64_t s = rp[r], e = rp[r + 1];
    HNM_REQUIRE(e >= s, HNM_EINVAL, "spmm_plan: rowptr decreases at row %lld", (long long)r);
    if (e - s > SPMM_SHORT && e - s <= HEAVY) lrows.push_back((int32_t)r);
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
  pl->num_cus = ctx->num_cus;
  pl->N = N;
  pl->nnz = rp[N] - rp[0];
  pl->n_heavy = (int64_t)hrows.size();
  pl->n_seg = (int64_t)sstart.size();
  pl->h_heavy = new std::vector<int32_t>(hrows);
  pl->h_seg_ptr = new std::vector<int64_t>(sptr);
  pl->n_long = (int64_t)lrows.size();
  pl->h_long = new std::vector<int32_t>(lrows);
  pl->mu = new std::mutex();
  // walk rows: every row of more than SPMM_SHORT entries (col << 10 must fit 32 bits)
  pl->walk = N <= (int64_t)1 << 22 && rp[0] == 0 &&
             rp[N] < ((int64_t)1 << 32);
  if (pl->walk) {
    std::vector<int32_t> wr, sr;
    int64_t wn = 0;
    for (int64_t r = 0; r < N; ++r) {
      const int64_t L = rp[r + 1] - rp[r];
      if (L <= SPMM_SHORT) {
        sr.push_back((int32_t)r);
        continue;
      }
      wr.push_back((int32_t)r);
      wn += L;
    }
    pl->n_walk = (int64_t)wr.size();
    pl->walk_nnz = wn;
    // pieces of at most cap entries: half a group's share of a big graph's walk (so the
    // longest list is ~2x the mean), never below 512
    pl->walk_cap = std::max<int64_t>(512, hnm_cdiv(pl->walk_nnz, 2 * WALK_GROUPS_TARGET));
    pl->h_walk_rows = new std::vector<int32_t>(wr);
    pl->h_short_rows = new std::vector<int32_t>(sr);
    pl->h_rowptr = new std::vector<int64_t>(std::move(rp));
    pl->swalk = !sr.empty();
  }
  if (pl->n_long > 0) {
    if (hipMalloc((void**)&pl->long_rows, pl->n_long * 4) != hipSuccess) {
      hnm_spmm_plan_destroy(pl);
      hnm_set_error("spmm_plan: hipMalloc failed");
      return HNM_ENOMEM;
    }
    HNM_HIP_CHECK(hipMemcpy(pl->long_rows, lrows.data(), pl->n_long * 4, hipMemcpyHostToDevice));
  }
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

extern "C" hnm_status hnm_spmm_plan_prepare(hnm_ctx* ctx, hnm_spmm_plan* plan, const int32_t* col,
                                            const float* val, int d) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && plan && col && val, HNM_EINVAL, "spmm_plan_prepare: NULL argument");
  HNM_REQUIRE(d == 0 || spmm_d_ok(d), HNM_EUNSUPPORTED,
              "spmm_plan_prepare: d must be 0 or one of 4, 8, 16, 32, 64, 128, 256 (got %d)", d);
  return walk_get(ctx, plan, col, val, d, nullptr, nullptr);
}

extern "C" hnm_status hnm_spmm_plan_destroy(hnm_spmm_plan* pl) {
  if (!pl) return HNM_OK;
  const HnmDeviceGuard guard(pl->device);
  if (pl->heavy_rows) (void)hipFree(pl->heavy_rows);
  if (pl->seg_ptr) (void)hipFree(pl->seg_ptr);
  if (pl->seg_hrow) (void)hipFree(pl->seg_hrow);
  if (pl->seg_start) (void)hipFree(pl->seg_start);
  if (pl->seg_end) (void)hipFree(pl->seg_end);
  if (pl->long_rows) (void)hipFree(pl->long_rows);
  for (WalkSched* w : pl->sched) walk_sched_free(w);
  for (ShortSched* w : pl->ssched) short_sched_free(w);
  if (pl->scol) (void)hipFree(pl->scol);
  if (pl->sval) (void)hipFree(pl->sval);
  delete pl->h_walk_rows;
  delete pl->h_short_rows;
  delete pl->h_rowptr;
  delete pl->h_scol;
  delete pl->h_sval;
  delete pl->mu;
  delete pl->h_long;
  delete pl->h_heavy;
  delete pl->h_seg_ptr;
  delete pl->keep;
  free(pl);
  return HNM_OK;
}

template <typename T>
static hnm_status dup_device(T** dst, const T* src, int64_t n) {
  *dst = nullptr;
  if (!src || n <= 0) return HNM_OK;
  if (hipMalloc((void**)dst, (size_t)n * sizeof(T)) != hipSuccess) {
    *dst = nullptr;
    hnm_set_error("spmm_plan_restrict: hipMalloc of %lld bytes failed", (long long)(n * sizeof(T)));
    return HNM_ENOMEM;
  }
  HNM_HIP_CHECK(hipMemcpy(*dst, src, (size_t)n * sizeof(T), hipMemcpyDeviceToDevice));
  return HNM_OK;
}

// Item-sharded propagation: a copy of a bound plan that computes
// only the rows of `ranges` -- e.g. every user row plus this rank's item rows.  A walk plan keeps
// the base's piece length (cap), its bipartite routing and its sorted copy, and filters the walk
// and short-walk row lists, so every kept row is cut into the same pieces and summed in the same
// order as by the base (bitwise equal rows), while the walks' schedules -- built per d on first
// use -- hold only the kept rows' entries (work proportional to them).  A plan without the walks
// runs the kept sub-ranges of each call with its row-class kernels (per-row order independent of
// the range).
extern "C" hnm_status hnm_spmm_plan_restrict(hnm_ctx* ctx, const hnm_spmm_plan* base,
                                             const int64_t* ranges, int n_ranges,
                                             hnm_spmm_plan** out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && base && out && n_ranges >= 0 && (ranges || n_ranges == 0), HNM_EINVAL,
              "spmm_plan_restrict: bad argument");
  HNM_REQUIRE(!base->keep, HNM_EINVAL, "spmm_plan_restrict: the base plan is itself restricted");
  for (int j = 0; j < n_ranges; ++j)
    HNM_REQUIRE(ranges[2 * j] >= (j ? ranges[2 * j - 1] : 0) && ranges[2 * j] <= ranges[2 * j + 1] &&
                    ranges[2 * j + 1] <= base->N,
                HNM_EINVAL, "spmm_plan_restrict: ranges must be ascending, disjoint, inside [0, N)");
  hnm_spmm_plan* bp = const_cast<hnm_spmm_plan*>(base);
  std::lock_guard<std::mutex> lk(*bp->mu);
  HNM_REQUIRE(bp->bound_col, HNM_EINVAL,
              "spmm_plan_restrict: bind the base plan first (hnm_spmm_plan_prepare, d = 0)");
  std::vector<int64_t> kr(ranges, ranges + 2 * n_ranges);
  auto kept = [&](int64_t r) {
    // first range whose end is past r
    int lo = 0, hi = n_ranges;
    while (lo < hi) {
      const int m = (lo + hi) / 2;
      if (kr[2 * m + 1] <= r) lo = m + 1; else hi = m;
    }
    return lo < n_ranges && kr[2 * lo] <= r;
  };
  hnm_spmm_plan* pl = (hnm_spmm_plan*)calloc(1, sizeof(hnm_spmm_plan));
  HNM_REQUIRE(pl, HNM_ENOMEM, "spmm_plan_restrict: out of host memory");
  pl->device = bp->device;
  pl->num_cus = bp->num_cus;
  pl->N = bp->N;
  pl->nnz = bp->nnz;
  pl->walk = bp->walk;
  pl->swalk = bp->swalk;
  pl->walk_cap = bp->walk_cap;
  pl->bound_col = bp->bound_col;
  pl->bound_val = bp->bound_val;
  pl->mu = new std::mutex();
  pl->keep = new std::vector<int64_t>(kr);
  hnm_status st = HNM_OK;
  if (bp->walk) {
    const std::vector<int64_t>& rp = *bp->h_rowptr;
    pl->h_rowptr = new std::vector<int64_t>(rp);
    pl->h_scol = new std::vector<int32_t>(*bp->h_scol);
    pl->h_sval = new std::vector<float>(*bp->h_sval);
    pl->h_walk_rows = new std::vector<int32_t>();
    pl->h_short_rows = new std::vector<int32_t>();
    for (int32_t r : *bp->h_walk_rows)
      if (kept(r)) {
        pl->h_walk_rows->push_back(r);
        pl->walk_nnz += rp[r + 1] - rp[r];
      }
    for (int32_t r : *bp->h_short_rows)
      if (kept(r)) pl->h_short_rows->push_back(r);
    pl->n_walk = (int64_t)pl->h_walk_rows->size();
    pl->h_long = new std::vector<int32_t>();
    pl->h_heavy = new std::vector<int32_t>();
    pl->h_seg_ptr = new std::vector<int64_t>(1, 0);
    if (!(st = dup_device(&pl->scol, bp->scol, bp->nnz))) st = dup_device(&pl->sval, bp->sval, bp->nnz);
  } else {
    pl->n_heavy = bp->n_heavy;
    pl->n_seg = bp->n_seg;
    pl->n_long = bp->n_long;
    pl->h_long = new std::vector<int32_t>(*bp->h_long);
    pl->h_heavy = new std::vector<int32_t>(*bp->h_heavy);
    pl->h_seg_ptr = new std::vector<int64_t>(*bp->h_seg_ptr);
    if (!(st = dup_device(&pl->long_rows, bp->long_rows, bp->n_long)) &&
        !(st = dup_device(&pl->heavy_rows, bp->heavy_rows, bp->n_heavy)) &&
        !(st = dup_device(&pl->seg_ptr, bp->seg_ptr, bp->n_heavy + 1)) &&
        !(st = dup_device(&pl->seg_hrow, bp->seg_hrow, bp->n_seg)) &&
        !(st = dup_device(&pl->seg_start, bp->seg_start, bp->n_seg)))
      st = dup_device(&pl->seg_end, bp->seg_end, bp->n_seg);
  }
  if (st) {
    hnm_spmm_plan_destroy(pl);
    return st;
  }
  *out = pl;
  return HNM_OK;
}

template <int LPR>
static hnm_status spmm_launch(hnm_ctx* ctx, const hnm_spmm_plan* pl, int64_t N,
                              const int64_t* rowptr, const int32_t* col, const float* val,
                              const float* X, int d, const SpmmEpi& ep, int64_t r0, int64_t r1,
                              bool timer = true) {
  const bool has_heavy = pl && pl->n_heavy > 0;
  const int64_t heavy = has_heavy ? HEAVY : INT64_MAX;
  // the live roofline times whole-plan layers only (row-range calls do less work; a restricted
  // plan's whole layer is timed as such -- bench.py prices its kept rows)
  const bool timed = timer && r0 == 0 && r1 == N;
  if (pl) {
    hnm_status s = walk_get(ctx, pl, col, val, 0, nullptr, nullptr);  // binding check
    if (s) return s;
  }
  if (pl && pl->keep && !pl->walk) {
    // a restricted plan without the walks: its kept sub-ranges of [r0, r1), one at a time
    if (timed) hnm_timer_begin(ctx, HNM_TIME_SPMM);
    const std::vector<int64_t>& kr = *pl->keep;
    for (size_t j = 0; j + 1 < kr.size(); j += 2) {
      const int64_t a = std::max(r0, kr[j]), b = std::min(r1, kr[j + 1]);
      if (a >= b) continue;
      hnm_spmm_plan unrestricted = *pl;
      unrestricted.keep = nullptr;
      hnm_status s = spmm_launch<LPR>(ctx, &unrestricted, N, rowptr, col, val, X, d, ep, a, b, false);
      if (s) return s;
    }
    if (timed) hnm_timer_end(ctx, HNM_TIME_SPMM);
    return HNM_OK;
  }
  if (pl && pl->walk) {
    // short rows (<= SPMM_SHORT entries) by the short walk, then the rows of more entries by the
    // user-ordered walk (+ the split rows' finish), one stream, disjoint output rows
    const WalkSched* ws = nullptr;
    const ShortSched* ss = nullptr;
    hnm_status s = walk_get(ctx, pl, col, val, d, &ws, &ss);
    if (s) return s;
    const std::vector<int32_t>& wr = *pl->h_walk_rows;
    const bool any = std::lower_bound(wr.begin(), wr.end(), (int32_t)std::min<int64_t>(r0, INT32_MAX)) !=
                     std::lower_bound(wr.begin(), wr.end(), (int32_t)std::min<int64_t>(r1, INT32_MAX));
    float* partial = nullptr;
    if (any && ws->n_part > 0) {
      void* w;
      s = hnm_workspace(ctx, (size_t)ws->n_part * d * 4, &w);
      if (s) return s;
      partial = (float*)w;
    }
    if (timed) hnm_timer_begin(ctx, HNM_TIME_SPMM);
    auto short_rows = [&]() -> hnm_status {
      if (r1 <= r0) return HNM_OK;
      if (ss) {
        // blocks whose rows meet [r0, r1) (blocks are in ascending row order)
        const int64_t b0 = std::lower_bound(ss->last.begin(), ss->last.end(),
                                            (int32_t)std::min<int64_t>(r0, INT32_MAX)) - ss->last.begin();
        const int64_t b1 = std::lower_bound(ss->first.begin(), ss->first.end(),
                                            (int32_t)std::min<int64_t>(r1, INT32_MAX)) - ss->first.begin();
        if (b1 > b0) {
          const unsigned grid = (unsigned)std::min<int64_t>(b1 - b0, ss->nwg);
          hipLaunchKernelGGL(spmm_swalk_kernel<LPR>, dim3(grid), dim3(SWALK_THREADS), 0, ctx->stream,
                             ss->gptr, ss->ent, ss->wt, ss->srow, ss->nslot, ss->S, X, d, ep, r0, r1,
                             b0, b1);
          HNM_LAUNCH_CHECK();
        }
        return HNM_OK;
      }
      hipLaunchKernelGGL(spmm_mixed_kernel<LPR>,
                         dim3((unsigned)hnm_cdiv(r1 - r0, 4 * (64 / LPR))), dim3(256), 0,
                         ctx->stream, r0, r1, pl->long_rows, (int64_t)0, (int64_t)0, (int64_t)0,
                         rowptr, col, val, X, d, ep);
      HNM_LAUNCH_CHECK();
      return HNM_OK;
    };
    if ((s = short_rows())) return s;
    if (any) {
      hipLaunchKernelGGL(spmm_walk_kernel<LPR>, dim3((unsigned)ws->nwg), dim3(WALK_THREADS), 0,
                         ctx->stream, ws->gptr, ws->ent, ws->wt, ws->slot_out, ws->nslot, ws->maxloc,
                         ws->nwin, X, d, partial, ep, r0, r1);
      HNM_LAUNCH_CHECK();
      if (ws->n_split > 0) {
        hipLaunchKernelGGL(spmm_walk_finish_kernel, dim3((unsigned)ws->n_split), dim3(256), 0,
                           ctx->stream, ws->split_rows, ws->split_ptr, partial, X, d, ep, r0, r1);
        HNM_LAUNCH_CHECK();
      }
    }
    if (timed) hnm_timer_end(ctx, HNM_TIME_SPMM);
    return HNM_OK;
  }
  if (timed) hnm_timer_begin(ctx, HNM_TIME_SPMM);
  // the heavy rows' segments + finish run on the ctx's side stream, concurrent with the light
  // kernel (disjoint output rows, X read-only): they fill the CUs the light kernel's long item
  // rows leave idle at its tail; the ctx stream joins before anything reads Y
  bool forked = false;
  if (has_heavy) {
    // heavy rows inside [r0, r1): heavy rows are ascending
    const std::vector<int32_t>& hv = *pl->h_heavy;
    const int64_t h0 = std::lower_bound(hv.begin(), hv.end(), (int32_t)std::min<int64_t>(r0, INT32_MAX)) - hv.begin();
    const int64_t h1 = std::lower_bound(hv.begin(), hv.end(), (int32_t)std::min<int64_t>(r1, INT32_MAX)) - hv.begin();
    if (h1 > h0) {
      const int64_t sg0 = (*pl->h_seg_ptr)[h0], sg1 = (*pl->h_seg_ptr)[h1];
      void* w;
      hnm_status s = hnm_workspace(ctx, (size_t)(sg1 - sg0) * d * 4, &w);
      if (s) return s;
      float* partial = (float*)w;
      HNM_HIP_CHECK(hipEventRecord(ctx->side_in, ctx->stream));
      HNM_HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->side_in, 0));
      const hipStream_t hs = ctx->side;
      hipLaunchKernelGGL(spmm_segment_kernel<LPR>, dim3((unsigned)hnm_cdiv(sg1 - sg0, 4)),
                         dim3(256), 0, hs, sg0, sg1, pl->seg_start, pl->seg_end, col, val,
                         X, d, partial);
      HNM_LAUNCH_CHECK();
      hipLaunchKernelGGL(spmm_finish_kernel, dim3((unsigned)(h1 - h0)), dim3(256), 0, hs,
                         h0, pl->heavy_rows, pl->seg_ptr, sg0, partial, X, d, ep);
      HNM_LAUNCH_CHECK();
      HNM_HIP_CHECK(hipEventRecord(ctx->side_out, ctx->side));
      forked = true;
    }
  }
  if (r1 > r0) {
    if (pl) {
      // long rows inside [r0, r1) (ascending list) + every short row of the range
      const std::vector<int32_t>& lv = *pl->h_long;
      const int64_t l0 = std::lower_bound(lv.begin(), lv.end(), (int32_t)std::min<int64_t>(r0, INT32_MAX)) - lv.begin();
      const int64_t l1 = std::lower_bound(lv.begin(), lv.end(), (int32_t)std::min<int64_t>(r1, INT32_MAX)) - lv.begin();
      const int64_t nlb = hnm_cdiv(l1 - l0, 4), nsb = hnm_cdiv(r1 - r0, 4 * (64 / LPR));
      hipLaunchKernelGGL(spmm_mixed_kernel<LPR>, dim3((unsigned)(nlb + nsb)), dim3(256), 0,
                         ctx->stream, r0, r1, pl->long_rows, l0, l1, nlb, rowptr, col, val, X, d,
                         ep);
    } else {
      hipLaunchKernelGGL(spmm_light_kernel<LPR>, dim3((unsigned)hnm_cdiv(r1 - r0, 4)), dim3(256), 0,
                         ctx->stream, r0, r1, rowptr, col, val, X, d, ep, heavy);
    }
    HNM_LAUNCH_CHECK();
  }
  if (forked) HNM_HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->side_out, 0));
  if (timed) hnm_timer_end(ctx, HNM_TIME_SPMM);
  return HNM_OK;
}

#define HNM_SPMM_DISPATCH(FN, ...)                                                        \
  switch (d) {                                                                            \
    case 4: return FN<1>(__VA_ARGS__);                                                    \
    case 8: return FN<2>(__VA_ARGS__);                                                    \
    case 16: return FN<4>(__VA_ARGS__);                                                   \
    case 32: return FN<8>(__VA_ARGS__);                                                   \
    case 64: return FN<16>(__VA_ARGS__);                                                  \
    case 128: return FN<32>(__VA_ARGS__);                                                 \
    case 256: return FN<64>(__VA_ARGS__);                                                 \
    default:                                                                              \
      hnm_set_error("spmm: d must be one of 4, 8, 16, 32, 64, 128, 256 (got %d)", d);     \
      return HNM_EUNSUPPORTED;                                                            \
  }

extern "C" hnm_status hnm_spmm_csr_range_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                                             const int64_t* rowptr, const int32_t* col,
                                             const float* val, const float* X, int d, float* Y,
                                             float alpha, const float* acc_in, float* acc_out,
                                             float beta, int64_t row_begin, int64_t row_end,
                                             int64_t acc_row0) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && rowptr && col && val && X, HNM_EINVAL, "spmm: NULL argument");
  HNM_REQUIRE(!plan || plan->N == N, HNM_EINVAL, "spmm: plan built for a different graph");
  HNM_REQUIRE((uintptr_t)X % 16 == 0 && (!Y || (uintptr_t)Y % 16 == 0) &&
                  (!acc_out || (uintptr_t)acc_out % 16 == 0) &&
                  (!acc_in || (uintptr_t)acc_in % 16 == 0),
              HNM_EUNSUPPORTED, "spmm: buffers must be 16-B aligned");
  HNM_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= N && 0 <= acc_row0 &&
                  acc_row0 <= N,
              HNM_EINVAL, "spmm: bad row range");
  if (N <= 0) return HNM_OK;
  const SpmmEpi ep{Y, alpha, beta, acc_in, acc_out, acc_row0};
  HNM_SPMM_DISPATCH(spmm_launch, ctx, plan, N, rowptr, col, val, X, d, ep, row_begin, row_end)
}

extern "C" hnm_status hnm_spmm_csr_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                                       const int64_t* rowptr, const int32_t* col,
                                       const float* val, const float* X, int d, float* Y,
                                       float alpha, const float* acc_in, float* acc_out) {
  HNM_CTX_DEVICE(ctx);
  return hnm_spmm_csr_range_f32(ctx, plan, N, rowptr, col, val, X, d, Y, alpha, acc_in, acc_out,
                                0.f, 0, N, 0);
}

template <int LPR>
static hnm_status combine_launch(hnm_ctx* ctx, const int64_t* rows, int64_t n, int64_t N,
                                 const int64_t* rowptr, const int32_t* col, const float* val,
                                 int d, const CombineLayers& cl, const CombineOrder& co, float* out) {
  const int64_t rows_per_block = co.mode != 0 ? 4 * (64 / LPR) : 4;
  hipLaunchKernelGGL(spmm_rows_combine_kernel<LPR>, dim3((unsigned)hnm_cdiv(n, rows_per_block)),
                     dim3(256), 0,
                     ctx->stream, rows, n, N, rowptr, col, val, d, cl, co, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_spmm_rows_combine_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan,
                                                int64_t N, const int64_t* rowptr,
                                                const int32_t* col, const float* val,
                                                const int64_t* rows, int64_t n, int d,
                                                const float* const* layers, const float* alphas,
                                                int L, float* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && rowptr && col && val && layers && alphas && ((rows && out) || n == 0),
              HNM_EINVAL, "spmm_rows_combine: NULL argument");
  HNM_REQUIRE(!plan || plan->N == N, HNM_EINVAL, "spmm_rows_combine: plan built for a different graph");
  HNM_REQUIRE(L >= 1 && L <= 8, HNM_EUNSUPPORTED, "spmm_rows_combine: 1 <= L <= 8");
  CombineOrder co{};
  co.mode = plan ? 1 : 0;
  if (plan) {
    hnm_status s = walk_get(ctx, plan, col, val, 0, nullptr, nullptr);
    if (s) return s;
    if (plan->walk) {
      co.mode = 2;
      co.short_sorted = plan->swalk;
      co.scol = plan->scol;
      co.sval = plan->sval;
      co.cap = plan->walk_cap;
    }
  }
  CombineLayers cl;
  cl.L = L;
  for (int l = 0; l < L; ++l) {
    HNM_REQUIRE(layers[l] && (uintptr_t)layers[l] % 16 == 0, HNM_EINVAL,
                "spmm_rows_combine: layer %d NULL or not 16-B aligned", l);
    cl.E[l] = layers[l];
  }
  for (int l = 0; l <= L; ++l) cl.a[l] = alphas[l];
  if (n <= 0) return HNM_OK;
  HNM_REQUIRE((uintptr_t)out % 16 == 0, HNM_EINVAL, "spmm_rows_combine: out not 16-B aligned");
  HNM_SPMM_DISPATCH(combine_launch, ctx, rows, n, N, rowptr, col, val, d, cl, co, out)
}
