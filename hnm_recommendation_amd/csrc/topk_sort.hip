// Row top-k for k > 128 (a12 beyond the fused/row-select kernels' range).
//
// The reference ends every recommend() in torch.topk(scores, top_k, dim=1)
// (neural_cf.py:324, lightgcn.py:356, wide_deep.py:433, matrix_factorization.py:244) and the
// server in torch.topk(scores[0], num_items) (serve.py:355): any k <= num_items is legal.
// k <= 128 is served by rows_topk_kernel (score.hip); larger k -- never the hot path -- by a
// stable segmented radix sort of whole rows in chunks of rows:
//   keys  = scores with the CSR mask applied (-inf) and -0 folded into +0 (torch compares
//           them equal; the radix order would not), values = item ids 0..I-1;
//   rocPRIM's segmented radix sort (descending, stable) -> (score desc, item asc), the same
//   total order as every other top-k kernel of the library;
//   the first k of each sorted row are copied out, their values re-read from `scores` so the
//   returned bits are the input's.
#include <hipcub/hipcub.hpp>

#include "hnm_device.h"
#include "hnm_internal.h"

namespace {

__global__ void __launch_bounds__(256) sort_keys_kernel(const float* __restrict__ scores,
                                                        int64_t ld, int64_t r0, int64_t R,
                                                        int64_t I, float* __restrict__ keys,
                                                        int32_t* __restrict__ vals,
                                                        int32_t* __restrict__ offsets) {
  const int64_t n = R * I;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / I, j = e - r * I;
    keys[e] = scores[(r0 + r) * ld + j] + 0.0f;  // -0 -> +0
    vals[e] = (int32_t)j;
  }
  const int64_t t = blockIdx.x * 256ll + threadIdx.x;
  if (t <= R) offsets[t] = (int32_t)(t * I);
}

// one wave per row of the chunk: mask entries -> -inf
__global__ void __launch_bounds__(256) sort_mask_kernel(const int64_t* __restrict__ mask_ptr,
                                                        const int32_t* __restrict__ mask_idx,
                                                        int64_t r0, int64_t R, int64_t I,
                                                        float* __restrict__ keys) {
  const int64_t r = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  for (int64_t p = mask_ptr[r0 + r] + lane; p < mask_ptr[r0 + r + 1]; p += 64) {
    const int32_t j = mask_idx[p];
    if (j >= 0 && j < I) keys[r * I + j] = -INFINITY;
  }
}

__global__ void __launch_bounds__(256) sort_out_kernel(const float* __restrict__ scores,
                                                       int64_t ld, const int64_t* mask_ptr,
                                                       const int32_t* __restrict__ mask_idx,
                                                       int64_t r0, int64_t R, int64_t I, int k,
                                                       const int32_t* __restrict__ sorted_vals,
                                                       float* __restrict__ out_val,
                                                       int64_t* __restrict__ out_idx) {
  const int64_t n = R * k;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / k, t = e - r * k;
    const int32_t j = sorted_vals[r * I + t];
    float v = scores[(r0 + r) * ld + j];
    if (mask_ptr) {  // masked entries report -inf (binary search of the sorted row)
      int64_t lo = mask_ptr[r0 + r], hi = mask_ptr[r0 + r + 1];
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (mask_idx[mid] < j) lo = mid + 1; else hi = mid;
      }
      if (lo < mask_ptr[r0 + r + 1] && mask_idx[lo] == j) v = -INFINITY;
    }
    if (out_val) out_val[(r0 + r) * (int64_t)k + t] = v;
    out_idx[(r0 + r) * (int64_t)k + t] = j;
  }
}

}  // namespace

hnm_status hnm_topk_rows_sort(hnm_ctx* ctx, const float* scores, int64_t ld, int64_t B,
                              int64_t I, const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                              float* out_val, int64_t* out_idx) {
  // rows per chunk: keys/values in and out (16 B per entry) within ~512 MB
  const int64_t R = std::max<int64_t>(1, std::min<int64_t>(B, (int64_t(512) << 20) / (16 * I)));
  HNM_REQUIRE(R * I < INT_BIG, HNM_EUNSUPPORTED, "topk_rows: row too long for the sort path");
  size_t temp = 0;
  hipError_t he = hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
      nullptr, temp, (const float*)nullptr, (float*)nullptr, (const int32_t*)nullptr,
      (int32_t*)nullptr, (int)(R * I), (int)R, (const int32_t*)nullptr, (const int32_t*)nullptr,
      0, 32, ctx->stream);
  HNM_REQUIRE(he == hipSuccess, HNM_EHIP, "topk_rows: sort size query failed");
  const size_t ent = (size_t)R * I, align = 256;
  const size_t off_b = ((size_t)(R + 1) * 4 + align - 1) / align * align;
  const size_t ent_b = (ent * 4 + align - 1) / align * align;
  void* w;
  hnm_status st = hnm_workspace(ctx, off_b + 4 * ent_b + temp, &w);
  if (st) return st;
  char* base = (char*)w;
  int32_t* offsets = (int32_t*)base;
  float* keys_in = (float*)(base + off_b);
  float* keys_out = (float*)(base + off_b + ent_b);
  int32_t* vals_in = (int32_t*)(base + off_b + 2 * ent_b);
  int32_t* vals_out = (int32_t*)(base + off_b + 3 * ent_b);
  void* tmp = base + off_b + 4 * ent_b;
  for (int64_t r0 = 0; r0 < B; r0 += R) {
    const int64_t rr = std::min<int64_t>(R, B - r0);
    const unsigned g = (unsigned)std::min<int64_t>(hnm_cdiv(std::max<int64_t>(rr * I, rr + 1), 256),
                                                   (int64_t)ctx->num_cus * 16);
    hipLaunchKernelGGL(sort_keys_kernel, dim3(std::max<unsigned>(g, (unsigned)hnm_cdiv(rr + 1, 256))),
                       dim3(256), 0, ctx->stream, scores, ld, r0, rr, I, keys_in, vals_in, offsets);
    HNM_LAUNCH_CHECK();
    if (mask_ptr) {
      hipLaunchKernelGGL(sort_mask_kernel, dim3((unsigned)hnm_cdiv(rr, 4)), dim3(256), 0,
                         ctx->stream, mask_ptr, mask_idx, r0, rr, I, keys_in);
      HNM_LAUNCH_CHECK();
    }
    size_t t = temp;
    he = hipcub::DeviceSegmentedRadixSort::SortPairsDescending(
        tmp, t, keys_in, keys_out, vals_in, vals_out, (int)(rr * I), (int)rr, offsets,
        offsets + 1, 0, 32, ctx->stream);
    HNM_REQUIRE(he == hipSuccess, HNM_EHIP, "topk_rows: segmented sort failed");
    const unsigned go = (unsigned)std::min<int64_t>(hnm_cdiv(rr * k, 256), (int64_t)ctx->num_cus * 16);
    hipLaunchKernelGGL(sort_out_kernel, dim3(go), dim3(256), 0, ctx->stream, scores, ld, mask_ptr,
                       mask_idx, r0, rr, I, k, vals_out, out_val, out_idx);
    HNM_LAUNCH_CHECK();
  }
  return HNM_OK;
}
