// Sample K-th kernel of the certified pre-filters (score.hip launches the plain form through
// hnm_sample_kth; ncf_cert.hip / dot_cert.hip instantiate it with an epilogue that turns each
// row's K-th into its bound and scan threshold in the same launch -- one kernel boundary less on
// the per-call latency chain, round 6).
#pragma once
#include "hnm_device.h"
#include "hnm_internal.h"

struct KthNoEpi {
  __device__ void operator()(int64_t, float) const {}
};

// ------------------------------------------------------------------ sample K-th (lower bound)
// For the certified pre-filters: a LOWER BOUND of the K-th best value of each row of a
// dense [B, Ns] sample (masked columns excluded; column c is item sidx[c], or
// (c / grp) * period + c % grp -- increasing in c either way).  Each lane keeps its own top-4;
// the K-th best of the survivors is <= the row's K-th best (dropping values can only lower it).
// ~3 VALU per element, no serial inserts.  A NaN in the row makes the result NaN (the caller then
// takes the exact fallback).  R rows per wave, G = 64 / R lanes per row: R > 1 only when every
// lane holds <= 4 columns (Ns <= 4 G) and no mask -- then no value is dropped, as with R = 1 at
// that Ns, so the output is the same; the K pops of a row (the cost at the 8 x 4,096 rows of an
// item-sharded rank's few-column sample) run for R rows at once.
template <int R, class Epi = KthNoEpi>
__global__ __launch_bounds__(256) void sample_kth_kernel(const float* __restrict__ s, int64_t ld,
                                                         int64_t B, int64_t Ns,
                                                         const int64_t* __restrict__ mptr,
                                                         const int32_t* __restrict__ midx, int K,
                                                         int64_t grp, int64_t period,
                                                         const int32_t* __restrict__ sidx,
                                                         float* __restrict__ out,
                                                         const int* __restrict__ gate,
                                                         Epi epi = Epi{}) {
  constexpr int G = 64 / R;
  const int lane = threadIdx.x & 63, gl = lane % G, gi = lane / G;
  const int64_t b = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * R + gi;
  if (((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * R >= B) return;  // wave-uniform
  if (gate && *gate == 0) return;  // a gated sample (ncf_cert.hip) that did not run
  const bool live = b < B;
  const uint64_t gmask = G == 64 ? ~0ull : (((1ull << G) - 1) << (gi * G));
  float t0 = -__builtin_inff(), t1 = t0, t2 = t0, t3 = t0;
  bool nan = false;
  int64_t mpos = 0, mend = 0;
  int nm = INT_BIG;
  if (R == 1 && mptr) {
    mpos = mptr[b];
    mend = mptr[b + 1];
    nm = mpos < mend ? midx[mpos] : INT_BIG;
  }
  // column -> item (increasing in the column), matched against the row's sorted mask
  auto item_of = [&](int64_t c) { return sidx ? (int64_t)sidx[c] : (c / grp) * period + c % grp; };
  auto insert = [&](float x) {  // into the lane's sorted top-4
    nan |= x != x;
    if (x > t3) {
      const float a = fminf(x, t2), c2 = fmaxf(x, t2);
      t3 = a;
      t2 = fminf(c2, t1);
      const float c1 = fmaxf(c2, t1);
      t1 = fminf(c1, t0);
      t0 = fmaxf(c1, t0);
    }
  };
  const float* row = s + (live ? b : 0) * ld;
  for (int64_t base = 0; base < Ns; base += 4 * G) {  // 4 loads per lane in flight
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t c = base + G * q + gl;
      v[q] = (live && c < Ns) ? row[c] : -__builtin_inff();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t cb = base + 64 * q;
      if (R == 1 && mptr && cb < Ns) {
        const int64_t c = std::min<int64_t>(cb + lane, Ns - 1);
        const int64_t cl = std::min<int64_t>(cb + 64, Ns) - 1;
        const int64_t it = item_of(c), end = item_of(cl) + 1;  // real ids < end
        while (nm < end) {
          if (cb + lane < Ns && it == nm) v[q] = -__builtin_inff();
          ++mpos;
          nm = mpos < mend ? midx[mpos] : INT_BIG;
        }
      }
      insert(v[q]);
    }
  }
  // K-th largest of the row's G x 4 survivors (a multiset: the value is unique whatever the tie
  // order): K rounds of popping the group maximum off its lane's sorted list (NaN never
  // enters a list; -inf once the survivors run out)
  // The r-th popped value (r < K) lands in out[b * K + r]: the row's K largest survivors,
  // descending -- each a lower bound of the sample's r-th best, on distinct columns (items).
  const bool anynan = (__ballot(nan) & gmask) != 0;
  float kv = -__builtin_inff();
  for (int r = 0; r < K; ++r) {
    const float m = hnm_group_max<G>(t0);  // DPP / permlane steps (a shfl chain: ~6 LDS trips)
    kv = m;
    if (live && gl == 0 && r < K - 1) out[b * K + r] = anynan ? __builtin_nanf("") : m;
    const uint64_t hit = __ballot(t0 == m && m != -__builtin_inff());
    if (hit == 0) {  // every row of the wave ran out of survivors: -inf from here on
      for (++r; r < K - 1; ++r)
        if (live && gl == 0) out[b * K + r] = anynan ? __builtin_nanf("") : -__builtin_inff();
      break;
    }
    const uint64_t gh = hit & gmask;
    if (gh && lane == __builtin_ctzll(gh)) {
      t0 = t1;
      t1 = t2;
      t2 = t3;
      t3 = -__builtin_inff();
    }
  }
  if (live && gl == 0) {
    const float kk = anynan ? __builtin_nanf("") : kv;
    out[b * K + (K - 1)] = kk;
    epi(b, kk);  // per-row consumer of the K-th (a caller's bound / threshold), same lane
  }
}


// launch with the row-grouping hnm_sample_kth uses (R rows a wave when lossless)
template <class Epi>
hnm_status sample_kth_launch(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t Ns,
                             const int64_t* mptr, const int32_t* midx, int K, int64_t grp,
                             int64_t period, const int32_t* sidx, float* out, const int* gate,
                             Epi epi) {
  HNM_REQUIRE(K >= 1 && K <= 64, HNM_EINVAL, "sample_kth: 1 <= K <= 64");
  HNM_REQUIRE(grp >= 1 && period >= grp, HNM_EINVAL, "sample_kth: 1 <= grp <= period");
  const int R = mptr ? 1 : Ns <= 64 ? 4 : Ns <= 128 ? 2 : 1;
  const unsigned grid = (unsigned)hnm_cdiv(B, 4 * R);
  if (R == 4)
    hipLaunchKernelGGL((sample_kth_kernel<4, Epi>), dim3(grid), dim3(256), 0, ctx->stream, s, ld,
                       B, Ns, mptr, midx, K, grp, period, sidx, out, gate, epi);
  else if (R == 2)
    hipLaunchKernelGGL((sample_kth_kernel<2, Epi>), dim3(grid), dim3(256), 0, ctx->stream, s, ld,
                       B, Ns, mptr, midx, K, grp, period, sidx, out, gate, epi);
  else
    hipLaunchKernelGGL((sample_kth_kernel<1, Epi>), dim3(grid), dim3(256), 0, ctx->stream, s, ld,
                       B, Ns, mptr, midx, K, grp, period, sidx, out, gate, epi);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
