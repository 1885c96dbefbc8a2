// (f)4: ranking metrics over top-K lists -- MAP@K, Recall@K, Precision@K, NDCG@K.
//
// Reference: `src/evaluation/metrics.py` -- the per-user loops of evaluate_recommendations
// (`:193-255`) and of the torchmetrics classes MeanAveragePrecision (`:49-62`), RecallAtK
// (`:95-100`), PrecisionAtK (`:133-137`), NDCGAtK (`:176-186`).  Each user's four values
// are computed with the reference's own float64 formulas and summation order, so they are
// bitwise the values the Python loops produce:
//   ap   = (sum over hit positions i, in order, of nh / (i + 1.0)) / min(n_true, k)
//   rec  = hits / n_true            prec = hits / n_pred
//   ndcg = (sum over hit positions of inv_log2[i]) / (sum_{i < min(n_true, k)} inv_log2[i])
// with inv_log2[i] = 1.0 / np.log2(i + 2) supplied by the caller (computed by numpy, so the
// terms are the reference's to the bit).  Zero denominators give 0.0 (the reference's
// guards; evaluate_recommendations' ZeroDivisionError for a present user with an empty
// truth set is raised by the host wrapper, which sees the dict).
//
// Work per user: k predicted ids (<= 128), n_true truth ids, one 4 x f64 result -- a few
// hundred bytes; the kernels are latency/HBM-bound gathers, one wave per user.
#include "hnm_device.h"
#include "hnm_internal.h"

namespace {

constexpr int EV_WAVES = 4;  // users per 256-thread block
constexpr int EV_RED_BLOCKS = 256;

// One wave per user: lanes hold predicted positions p and p + 64; the truth row streams
// through the wave 64 entries at a time (coalesced) and each entry is broadcast with a
// uniform readlane; hit flags become two 64-bit ballots that lane 0 walks in position
// order (the reference's loop order, so the float64 sums round identically).
__global__ __launch_bounds__(256) void rank_metrics_kernel(
    const int64_t* __restrict__ pred, int64_t B, int64_t ldp, const int64_t* __restrict__ pred_len,
    int k, const int64_t* __restrict__ tptr, const int64_t* __restrict__ tidx, int64_t ldt,
    const uint8_t* __restrict__ tmask, const double* __restrict__ inv_log2,
    double* __restrict__ per_user, int64_t* __restrict__ n_true_out) {
  const int64_t r = (int64_t)blockIdx.x * EV_WAVES + (threadIdx.x >> 6);
  if (r >= B) return;
  const int lane = threadIdx.x & 63;
  int64_t np_ = pred_len ? pred_len[r] : ldp;
  if (np_ > ldp) np_ = ldp;
  if (np_ > k) np_ = k;
  if (np_ < 0) np_ = 0;
  const int npred = (int)np_;
  const int64_t* prow = pred + r * ldp;
  const int64_t p0 = lane < npred ? prow[lane] : 0;
  const int64_t p1 = lane + 64 < npred ? prow[lane + 64] : 0;
  bool h0 = false, h1 = false;

  int64_t t0, t1;
  if (tptr) {
    t0 = tptr[r];
    t1 = tptr[r + 1];
  } else {
    t0 = r * ldt;
    t1 = t0 + ldt;
  }
  int64_t nt = 0;
  for (int64_t c = t0; c < t1; c += 64) {
    const int64_t e = c + lane;
    const bool in = e < t1 && (tmask == nullptr || tmask[e] != 0);
    const int64_t g = in ? tidx[e] : 0;
    uint64_t live = __ballot(in);
    nt += __popcll(live);
    while (live) {  // uniform loop over the chunk's kept entries
      const int s = __builtin_ctzll(live);
      live &= live - 1;
      const int lo = __builtin_amdgcn_readlane((int)(uint32_t)g, s);
      const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)g >> 32), s);
      const int64_t gv = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
      h0 |= (p0 == gv);
      h1 |= (p1 == gv);
    }
  }
  const uint64_t m0 = __ballot(h0 && lane < npred);
  const uint64_t m1 = __ballot(h1 && lane + 64 < npred);
  if (lane != 0) return;

  double nh = 0.0, ap = 0.0, dcg = 0.0;
  for (int half = 0; half < 2; ++half) {
    uint64_t m = half ? m1 : m0;
    while (m) {
      const int i = __builtin_ctzll(m) + 64 * half;
      m &= m - 1;
      nh += 1.0;
      ap += nh / ((double)i + 1.0);
      dcg += inv_log2[i];
    }
  }
  const int64_t lim = nt < k ? nt : k;
  double idcg = 0.0;
  for (int64_t i = 0; i < lim; ++i) idcg += inv_log2[i];
  double* o = per_user + r * 4;
  o[0] = lim > 0 ? ap / (double)lim : 0.0;
  o[1] = nt > 0 ? nh / (double)nt : 0.0;
  o[2] = npred > 0 ? nh / (double)npred : 0.0;
  o[3] = idcg > 0.0 ? dcg / idcg : 0.0;
  if (n_true_out) n_true_out[r] = nt;
}

// Deterministic two-level reduction: block j sums a fixed contiguous user range (strided
// lanes, then a fixed tree), the final block sums the partials in block order.
// partial[j*8 + m]: m < 4 sums of metric m over all users; m = 4..7 the same restricted to
// users with n_true > 0 (the torchmetrics classes count Recall/NDCG only for those).
__global__ __launch_bounds__(256) void rank_metrics_partial_kernel(
    const double* __restrict__ per_user, const int64_t* __restrict__ n_true, int64_t B,
    double* __restrict__ partial, int64_t* __restrict__ pcount) {
  __shared__ double sh[8][256];
  __shared__ int64_t shc[256];
  const int64_t per = hnm_cdiv(B, gridDim.x);
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < B ? lo + per : B;
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t cnt = 0;
  for (int64_t r = lo + threadIdx.x; r < hi; r += blockDim.x) {
    const bool has = n_true[r] > 0;
    cnt += has;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const double v = per_user[r * 4 + m];
      a[m] += v;
      a[4 + m] += has ? v : 0.0;
    }
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) sh[m][threadIdx.x] = a[m];
  shc[threadIdx.x] = cnt;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
#pragma unroll
      for (int m = 0; m < 8; ++m) sh[m][threadIdx.x] += sh[m][threadIdx.x + s];
      shc[threadIdx.x] += shc[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x < 8) partial[blockIdx.x * 8 + threadIdx.x] = sh[threadIdx.x][0];
  if (threadIdx.x == 0) pcount[blockIdx.x] = shc[0];
}

__global__ __launch_bounds__(64) void rank_metrics_final_kernel(const double* __restrict__ partial,
                                                                const int64_t* __restrict__ pcount,
                                                                int nb, double* __restrict__ sums) {
  const int m = threadIdx.x;
  if (m < 8) {
    double s = 0.0;
    for (int j = 0; j < nb; ++j) s += partial[j * 8 + m];
    sums[m] = s;
  } else if (m == 8) {
    int64_t c = 0;
    for (int j = 0; j < nb; ++j) c += pcount[j];
    sums[8] = (double)c;
  }
}

}  // namespace

extern "C" hnm_status hnm_rank_metrics_f64(hnm_ctx* ctx, const int64_t* pred, int64_t B,
                                           int64_t ldp, const int64_t* pred_len, int k,
                                           const int64_t* truth_ptr, const int64_t* truth_idx,
                                           int64_t ldt, const uint8_t* truth_mask,
                                           const double* inv_log2, double* per_user,
                                           int64_t* n_true, double* sums) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && inv_log2, HNM_EINVAL, "rank_metrics: NULL argument");
  HNM_REQUIRE(k >= 1 && k <= 128, HNM_EINVAL, "rank_metrics: 1 <= k <= 128");
  HNM_REQUIRE(B >= 0 && ldp >= 0 && (ldp == 0 || pred || B == 0), HNM_EINVAL,
              "rank_metrics: bad prediction shape");
  HNM_REQUIRE(truth_ptr || ldt >= 0, HNM_EINVAL, "rank_metrics: bad truth shape");
  HNM_REQUIRE(!(truth_ptr && truth_mask), HNM_EINVAL,
              "rank_metrics: truth_mask applies to the dense truth layout only");
  HNM_REQUIRE(per_user || sums, HNM_EINVAL, "rank_metrics: no output");
  if (B == 0) {
    if (sums) HNM_HIP_CHECK(hipMemsetAsync(sums, 0, 9 * sizeof(double), ctx->stream));
    return HNM_OK;
  }
  const int nb = (int)std::min<int64_t>(EV_RED_BLOCKS, hnm_cdiv(B, 256));
  double* pu = per_user;
  int64_t* nt = n_true;
  if (!pu || !nt || sums) {
    const size_t need = (pu ? 0 : hnm_align((size_t)B * 4 * sizeof(double))) +
                        (nt ? 0 : hnm_align((size_t)B * sizeof(int64_t))) +
                        hnm_align((size_t)nb * 8 * sizeof(double)) +
                        hnm_align((size_t)nb * sizeof(int64_t));
    char* ws = nullptr;
    hnm_status st = hnm_workspace(ctx, need, (void**)&ws);
    if (st != HNM_OK) return st;
    if (!pu) {
      pu = (double*)ws;
      ws += hnm_align((size_t)B * 4 * sizeof(double));
    }
    if (!nt) {
      nt = (int64_t*)ws;
      ws += hnm_align((size_t)B * sizeof(int64_t));
    }
    double* partial = (double*)ws;
    ws += hnm_align((size_t)nb * 8 * sizeof(double));
    int64_t* pcount = (int64_t*)ws;
    hipLaunchKernelGGL(rank_metrics_kernel, dim3((unsigned)hnm_cdiv(B, EV_WAVES)), dim3(256), 0,
                       ctx->stream, pred, B, ldp, pred_len, k, truth_ptr, truth_idx, ldt,
                       truth_mask, inv_log2, pu, nt);
    HNM_LAUNCH_CHECK();
    if (sums) {
      hipLaunchKernelGGL(rank_metrics_partial_kernel, dim3(nb), dim3(256), 0, ctx->stream, pu,
                         nt, B, partial, pcount);
      HNM_LAUNCH_CHECK();
      hipLaunchKernelGGL(rank_metrics_final_kernel, dim3(1), dim3(64), 0, ctx->stream, partial,
                         pcount, nb, sums);
      HNM_LAUNCH_CHECK();
    }
    return HNM_OK;
  }
  hipLaunchKernelGGL(rank_metrics_kernel, dim3((unsigned)hnm_cdiv(B, EV_WAVES)), dim3(256), 0,
                     ctx->stream, pred, B, ldp, pred_len, k, truth_ptr, truth_idx, ldt,
                     truth_mask, inv_log2, pu, nt);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
