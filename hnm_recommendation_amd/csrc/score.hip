// Fused all-items scoring + filter + top-K for gfx950.
//
// dot_score_kernel  (LightGCN / MatrixFactorization, lightgcn.py:188-204 + 332-358,
//                    matrix_factorization.py:108-131 + 220-246)
//   one workgroup = 4 waves x 32 users; the 32-user tile of each wave is the MFMA A
//   operand, held in registers for the whole item stream (user rows gathered by id: the
//   a1 gather is fused).  32-item tiles are staged in LDS (shared by the 4 waves),
//   permuted into lane-half order so each lane reads its B operand with ds_read_b128.
//   v_mfma_f32_32x32x2_f32 = exact fp32 fma chain (no bf16 shortcut).  C[user][item]
//   rows stay in registers; a 32-list wave top-K (one list per user) with per-lane
//   threshold registers pre-filters every score with one compare.
//
// The kernel covers one item PARTITION per blockIdx.y; partial top-K lists go to a
// [B, NP, K] candidate buffer merged by topk_merge_kernel (total order: score desc,
// item asc, so the merged result is unique).  The NeuralCF kernels live in ncf.hip.
#include <algorithm>

#include "hnm_device.h"
#include "hnm_internal.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);


// ------------------------------------------------------------------ dot kernel
template <int DP, bool DENSE, bool BIAS>
__global__ __launch_bounds__(256, 2) void dot_score_kernel(
    const float* __restrict__ ut, int64_t num_users, int64_t ldu,
    const int64_t* __restrict__ uids, int64_t B, const float* __restrict__ it, int64_t I,
    int64_t ldi, int d, const float* __restrict__ ubias, const float* __restrict__ ibias,
    const float* __restrict__ cbias, int64_t ipp, const int64_t* __restrict__ mptr,
    const int32_t* __restrict__ midx, int K, float* __restrict__ cand_v,
    int32_t* __restrict__ cand_i, int NP, float* __restrict__ dense, int64_t ldo,
    unsigned* err) {
  constexpr int KS = DP / 2;        // MFMA k-steps (K = 2 each)
  constexpr int RS = DP + 4;        // LDS row stride (floats): conflict-free b128 reads
  constexpr int F4_PER_ROW = DP / 4;
  constexpr int F4_PER_THREAD = TILE * F4_PER_ROW / 256;
  __shared__ __attribute__((aligned(16))) float vs[2][TILE * RS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;
  const int j = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * 128 + wave * 32;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + ipp);

  // ---- A operand: this lane's user (b0 + j), k = 2s + h
  float a[KS];
  bool uvalid;
  {
    const int64_t b = b0 + j;
    int64_t uid = -1;
    if (b < B) uid = uids[b];
    uvalid = (b < B) && uid >= 0 && uid < num_users;
    if (b < B && !uvalid && h == 0) hnm_flag(err, HNM_ERR_OOB);
    const float* row = ut + (uvalid ? uid : 0) * ldu;
#pragma unroll
    for (int m = 0; m < KS / 2; ++m) {
      const int k0 = 4 * m;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (uvalid && k0 < d) v = *reinterpret_cast<const float4*>(row + k0);
      a[2 * m] = h ? v.y : v.x;
      a[2 * m + 1] = h ? v.w : v.z;
    }
  }
  // per-row user bias for the 16 C rows of this lane
  float ub[16];
  if (BIAS) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t b = b0 + mfma32_row(r, h);
      float v = 0.f;
      if (ubias && b < B) {
        const int64_t uid = uids[b];
        if (uid >= 0 && uid < num_users) v = ubias[uid];
      }
      ub[r] = v + (cbias ? cbias[0] : 0.f);
    }
  }

  // ---- top-K state: list for user row i lives in (lv[i], li[i]); threshold per C reg
  float lv[DENSE ? 1 : 32];
  int li[DENSE ? 1 : 32];
  float tv[16];
  if (!DENSE) {
#pragma unroll
    for (int i = 0; i < 32; ++i) { lv[i] = -__builtin_inff(); li[i] = HNM_SENTINEL_IDX; }
#pragma unroll
    for (int r = 0; r < 16; ++r) tv[r] = -__builtin_inff();
  }
  // mask cursor of user (b0 + lane), lanes < 32
  int nm = INT_BIG;
  int64_t mpos = 0, mend = 0;
  if (!DENSE && mptr && lane < 32 && b0 + lane < B) {
    const int64_t lo = mptr[b0 + lane], hi = mptr[b0 + lane + 1];
    mpos = mask_lower_bound(midx, lo, hi, (int)part_start);
    mend = hi;
    nm = mpos < mend ? midx[mpos] : INT_BIG;
  }

  // ---- item tile staging (pair-permuted: vs[row][h*KS + s] = V[row][2s+h])
  float4 stage[F4_PER_THREAD];
  auto load_tile = [&](int64_t base) {
#pragma unroll
    for (int q = 0; q < F4_PER_THREAD; ++q) {
      const int f = tid + 256 * q;
      const int row = f / F4_PER_ROW, c4 = f % F4_PER_ROW;
      const int64_t item = base + row;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (item < part_end && 4 * c4 < d) v = *reinterpret_cast<const float4*>(it + item * ldi + 4 * c4);
      stage[q] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int q = 0; q < F4_PER_THREAD; ++q) {
      const int f = tid + 256 * q;
      const int row = f / F4_PER_ROW, c4 = f % F4_PER_ROW;
      float* dst = &vs[buf][row * RS];
      *reinterpret_cast<float2*>(dst + 2 * c4) = make_float2(stage[q].x, stage[q].z);
      *reinterpret_cast<float2*>(dst + KS + 2 * c4) = make_float2(stage[q].y, stage[q].w);
    }
  };

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, TILE) : 0;
  if (ntiles > 0) {
    load_tile(part_start);
    store_tile(0);
  }
  __syncthreads();

  for (int64_t t = 0; t < ntiles; ++t) {
    const int buf = (int)(t & 1);
    const int64_t base = part_start + t * TILE;
    if (t + 1 < ntiles) load_tile(base + TILE);

    f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* brow = &vs[buf][j * RS + h * KS];
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
      const float4 bv = *reinterpret_cast<const float4*>(brow + 4 * s4);
      acc = mfma32x32x2(a[4 * s4 + 0], bv.x, acc);
      acc = mfma32x32x2(a[4 * s4 + 1], bv.y, acc);
      acc = mfma32x32x2(a[4 * s4 + 2], bv.z, acc);
      acc = mfma32x32x2(a[4 * s4 + 3], bv.w, acc);
    }

    const int64_t item = base + j;
    const bool ivalid = item < part_end;
    float sc[16];
    {
      float ib = 0.f;
      if (BIAS && ibias && ivalid) ib = ibias[item];
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = BIAS ? (acc[r] + ub[r]) + ib : acc[r];
    }

    if (DENSE) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t b = b0 + mfma32_row(r, h);
        if (ivalid && b < B) dense[b * ldo + item] = sc[r];
      }
    } else {
      const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);
      // -inf for masked (user, item) pairs inside this tile (rare path)
      uint64_t mm = __ballot(lane < 32 && nm < tile_end) & 0xffffffffull;
      while (mm) {
        const int u = __builtin_ctzll(mm);
        mm &= mm - 1;
        while (true) {
          const int tgt = hnm_readlane_i(nm, u);
          if (tgt >= tile_end) break;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (mfma32_row(r, h) == u && item == tgt) sc[r] = -__builtin_inff();
          if (lane == u) {
            ++mpos;
            nm = mpos < mend ? midx[mpos] : INT_BIG;
          }
        }
      }
      // threshold pre-filter, then exact serial insertion per user list
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint64_t m = __ballot(ivalid && sc[r] >= tv[r]);
        if (m) {
          uint64_t lo = m & 0xffffffffull, hi = m >> 32;
          const int i0 = mfma32_row(r, 0), i1 = mfma32_row(r, 1);
          while (lo) {
            const int l = __builtin_ctzll(lo);
            lo &= lo - 1;
            list1_insert(lv[i0], li[i0], hnm_readlane_f(sc[r], l), (int)(base + l), K);
          }
          while (hi) {
            const int l = __builtin_ctzll(hi);
            hi &= hi - 1;
            list1_insert(lv[i1], li[i1], hnm_readlane_f(sc[r], 32 + l), (int)(base + l), K);
          }
          const float t0 = hnm_readlane_f(lv[i0], K - 1);
          const float t1 = hnm_readlane_f(lv[i1], K - 1);
          tv[r] = h ? t1 : t0;
        }
      }
    }

    if (t + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  if (!DENSE) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int64_t b = b0 + i;
      if (b < B && lane < K) {
        const int64_t o = (b * NP + p) * K + lane;
        cand_v[o] = lv[i];
        cand_i[o] = li[i] == HNM_SENTINEL_IDX ? -1 : li[i];
      }
    }
  }
}

// ------------------------------------------------------------------ row top-K (dense in)
// torch.topk(scores, k) replacement over a dense [B, I] matrix with an optional CSR mask
// (serve.py:350-355).  One wave per row; K <= 128.
template <int NS>
__global__ __launch_bounds__(256) void rows_topk_kernel(const float* __restrict__ s,
                                                        int64_t ld, int64_t B, int64_t I,
                                                        const int64_t* __restrict__ mptr,
                                                        const int32_t* __restrict__ midx,
                                                        int K, float* __restrict__ ov,
                                                        int64_t* __restrict__ oi) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  WaveTopK<NS> L;
  L.init();
  int64_t mpos = 0, mend = 0;
  int nm = INT_BIG;
  if (mptr) {
    mpos = mptr[b];
    mend = mptr[b + 1];
    nm = mpos < mend ? midx[mpos] : INT_BIG;
  }
  const float* row = s + b * ld;
  for (int64_t base = 0; base < I; base += 64) {
    const int64_t item = base + lane;
    const bool valid = item < I;
    float v = valid ? row[item] : -__builtin_inff();
    const int64_t end = std::min<int64_t>(base + 64, I);
    while (nm < end) {
      if (item == nm) v = -__builtin_inff();
      ++mpos;
      nm = mpos < mend ? midx[mpos] : INT_BIG;
    }
    L.offer(v, (int)item, valid, K);
  }
  L.store(ov ? ov + b * K : nullptr, oi + b * K, K);
}

// ------------------------------------------------------------------ host side
template <int DP, bool DENSE, bool BIAS>
static void launch_dot(hnm_ctx* ctx, dim3 grid, const float* ut, int64_t U, int64_t ldu,
                       const int64_t* ids, int64_t B, const float* it, int64_t I, int64_t ldi,
                       int d, const float* ub, const float* ib, const float* cb, int64_t ipp,
                       const int64_t* mptr, const int32_t* midx, int K, float* cv, int32_t* ci,
                       int NP, float* dense, int64_t ldo) {
  hipLaunchKernelGGL((dot_score_kernel<DP, DENSE, BIAS>), grid, dim3(256), 0, ctx->stream, ut,
                     U, ldu, ids, B, it, I, ldi, d, ub, ib, cb, ipp, mptr, midx, K, cv, ci, NP,
                     dense, ldo, ctx->err_dev);
}

template <bool DENSE>
static hnm_status dot_common(hnm_ctx* ctx, const float* ut, int64_t U, int64_t ldu,
                             const int64_t* ids, int64_t B, const float* it, int64_t I,
                             int64_t ldi, int d, const float* ub, const float* ib,
                             const float* cb, const int64_t* mptr, const int32_t* midx, int K,
                             float* ov, int64_t* oi, float* dense, int64_t ldo) {
  HNM_REQUIRE(ctx && ut && ids && it, HNM_EINVAL, "dot: NULL argument");
  HNM_REQUIRE(d >= 1 && d <= 128 && ldu >= d && ldi >= d && U > 0 && I > 0, HNM_EINVAL,
              "dot: bad shape (d=%d)", d);
  HNM_REQUIRE(d % 4 == 0 && ldu % 4 == 0 && ldi % 4 == 0 && (uintptr_t)ut % 16 == 0 &&
                  (uintptr_t)it % 16 == 0,
              HNM_EUNSUPPORTED, "dot: tables must be 16-B aligned with d %% 4 == 0");
  HNM_REQUIRE(I < INT_BIG, HNM_EUNSUPPORTED, "dot: too many items");
  if (B <= 0) return HNM_OK;
  const int64_t ublocks = hnm_cdiv(B, 128);
  Partition part = choose_partition(I, ublocks, ctx->num_cus);
  dim3 grid((unsigned)ublocks, (unsigned)part.np);
  const bool bias = ub || ib || cb;
  float* cv = nullptr;
  int32_t* ci = nullptr;
  if (!DENSE) {
    HNM_REQUIRE(K >= 1 && K <= 64, HNM_EINVAL, "dot_topk: fused path needs 1 <= k <= 64");
    HNM_REQUIRE(oi, HNM_EINVAL, "dot_topk: out_idx is NULL");
    const size_t n = (size_t)B * part.np * K;
    void* w;
    hnm_status st = hnm_workspace(ctx, hnm_align(n * 4) * 2, &w);
    if (st) return st;
    cv = (float*)w;
    ci = (int32_t*)((char*)w + hnm_align(n * 4));
  }
#define HNM_DOT(DPV)                                                                       \
  if (bias)                                                                                \
    launch_dot<DPV, DENSE, true>(ctx, grid, ut, U, ldu, ids, B, it, I, ldi, d, ub, ib, cb, \
                                 part.ipp, mptr, midx, K, cv, ci, part.np, dense, ldo);    \
  else                                                                                     \
    launch_dot<DPV, DENSE, false>(ctx, grid, ut, U, ldu, ids, B, it, I, ldi, d, ub, ib,    \
                                  cb, part.ipp, mptr, midx, K, cv, ci, part.np, dense, ldo);
  hnm_timer_begin(ctx);
  if (d <= 64) {
    HNM_DOT(64)
  } else {
    HNM_DOT(128)
  }
#undef HNM_DOT
  hnm_timer_end(ctx);
  HNM_LAUNCH_CHECK();
  if (!DENSE) return hnm_topk_merge_i32(ctx, cv, ci, B, 1, 0, (int64_t)part.np * K,
                                        part.np * K, K, ov, oi);
  return HNM_OK;
}

extern "C" hnm_status hnm_dot_topk_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                       int64_t ldu, const int64_t* user_ids, int64_t B,
                                       const float* item_tab, int64_t num_items, int64_t ldi,
                                       int d, const float* user_bias, const float* item_bias,
                                       const float* const_bias, const int64_t* mask_ptr,
                                       const int32_t* mask_idx, int k, float* out_val,
                                       int64_t* out_idx) {
  return dot_common<false>(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi,
                           d, user_bias, item_bias, const_bias, mask_ptr, mask_idx, k, out_val,
                           out_idx, nullptr, 0);
}

extern "C" hnm_status hnm_dot_scores_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                         int64_t ldu, const int64_t* user_ids, int64_t B,
                                         const float* item_tab, int64_t num_items, int64_t ldi,
                                         int d, const float* user_bias, const float* item_bias,
                                         const float* const_bias, float* out, int64_t ldo) {
  HNM_REQUIRE(out && ldo >= num_items, HNM_EINVAL, "dot_scores: bad output");
  return dot_common<true>(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi,
                          d, user_bias, item_bias, const_bias, nullptr, nullptr, 1, nullptr,
                          nullptr, out, ldo);
}

extern "C" hnm_status hnm_topk_rows_f32(hnm_ctx* ctx, const float* scores, int64_t ld, int64_t B,
                                        int64_t I, const int64_t* mask_ptr,
                                        const int32_t* mask_idx, int k, float* out_val,
                                        int64_t* out_idx) {
  HNM_REQUIRE(ctx && scores && out_idx, HNM_EINVAL, "topk_rows: NULL argument");
  HNM_REQUIRE(k >= 1 && k <= 128 && k <= I && ld >= I, HNM_EINVAL, "topk_rows: bad k/shape");
  HNM_REQUIRE(I < INT_BIG, HNM_EUNSUPPORTED, "topk_rows: too many items");
  if (B <= 0) return HNM_OK;
  dim3 grid((unsigned)hnm_cdiv(B, 4));
  if (k <= 64)
    hipLaunchKernelGGL(rows_topk_kernel<1>, grid, dim3(256), 0, ctx->stream, scores, ld, B, I,
                       mask_ptr, mask_idx, k, out_val, out_idx);
  else
    hipLaunchKernelGGL(rows_topk_kernel<2>, grid, dim3(256), 0, ctx->stream, scores, ld, B, I,
                       mask_ptr, mask_idx, k, out_val, out_idx);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

