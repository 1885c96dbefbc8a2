// Fused all-items scoring + filter + top-K for gfx950.
//
// dot_score_kernel  (LightGCN / MatrixFactorization, lightgcn.py:188-204 + 332-358,
//                    matrix_factorization.py:108-131 + 220-246)
//   one workgroup = 4 waves x 32 users; the 32-user tile of each wave is the MFMA A
//   operand, held in registers for the whole item stream (user rows gathered by id: the
//   a1 gather is fused).  32-item tiles are staged in LDS (shared by the 4 waves),
//   permuted into lane-half order so each lane reads its B operand with ds_read_b128.
//   v_mfma_f32_32x32x2_f32 = exact fp32 fma chain (no bf16 shortcut).  C[user][item]
//   rows stay in registers.
//
// Top-K (total order: score desc, item asc -- unique, so partitions/shards merge exactly):
//   THRESH (large item sets): a LIST pass over a strided ~4k-item sample gives every user
//     tau_u = its K-th best sample score, a lower bound of its true K-th best (same fp32
//     arithmetic in both passes).  The main pass appends only scores >= tau_u to a per-user
//     buffer (one compare per score; ~K*I/S appends per user); thresh_select takes the
//     exact top-K of the buffer.  Users whose buffer overflows (degenerate / adversarial
//     scores) are re-run on device through the LIST path -- results are always exact.
//   LIST: per item partition, a 32-list wave top-K (one list per user) with per-lane
//     threshold registers; partial lists are merged by topk_merge_kernel.
// The NeuralCF kernels live in ncf.hip.
#include <algorithm>

#include "hnm_device.h"
#include "dot_internal.h"
#include "sample_kth.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);


// ------------------------------------------------------------------ dot kernel
// LIST keeps 32 user lists in registers (2 workgroups/CU); the list-free d<=64 modes run 4 (measured faster than 3 despite a small spill).
template <int DP, int MODE, bool BIAS>
__global__ __launch_bounds__(256, (MODE == DOT_LIST || DP > 64) ? 2 : 4) void dot_score_kernel(DotArgs A) {
  constexpr bool LIST = MODE == DOT_LIST, DENSE = MODE == DOT_DENSE, THRESH = MODE == DOT_THRESH;
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
  const int64_t Bl = A.nrows ? (int64_t)*A.nrows : A.B;  // rows of this launch
  int64_t ublk = (int64_t)blockIdx.x * 128;
  int64_t ipp = A.ipp;
  int NP = A.NP;
  int p = blockIdx.y;
  if (A.rows && A.dyn_cus > 0) {  // flat grid: (user block, partition) from *nrows
    const int64_t nb = hnm_cdiv(Bl, 128);
    const Partition dp = choose_partition(A.I, nb, A.dyn_cus);
    ipp = dp.ipp;
    NP = dp.np;
    const int64_t w = blockIdx.x;
    if (w >= nb * NP) return;  // whole workgroup
    ublk = w / NP * 128;
    p = (int)(w % NP);
  }
  if (ublk >= Bl || p >= NP) return;  // whole workgroup idle (fallback launches)
  const int64_t b0 = ublk + wave * 32;
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(A.I, part_start + ipp);
  const int64_t K = A.K;
  auto req = [&](int64_t b) -> int64_t { return A.rows ? (int64_t)A.rows[b] : b; };

  // ---- A operand: this lane's user (b0 + j), k = 2s + h
  float a[KS];
  {
    const int64_t b = b0 + j;
    int64_t uid = -1;
    if (b < Bl) uid = A.uids[req(b)];
    const bool uvalid = (b < Bl) && uid >= 0 && uid < A.num_users;
    if (b < Bl && !uvalid && h == 0) hnm_flag(A.err, HNM_ERR_OOB);
    const float* row = A.ut + (uvalid ? uid : 0) * A.ldu;
#pragma unroll
    for (int m = 0; m < KS / 2; ++m) {
      const int k0 = 4 * m;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (uvalid && k0 < A.d) v = *reinterpret_cast<const float4*>(row + k0);
      a[2 * m] = h ? v.y : v.x;
      a[2 * m + 1] = h ? v.w : v.z;
    }
  }
  // per C-row constants of this lane: user bias, threshold
  float ub[BIAS ? 16 : 1];
  float tv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t b = b0 + mfma32_row(r, h);
    tv[r] = -__builtin_inff();
    if (THRESH) tv[r] = b < Bl ? A.tau[req(b) * A.tau_ld] : __builtin_inff();
    if (BIAS) {
      float v = 0.f;
      if (A.ubias && b < Bl) {
        const int64_t uid = A.uids[req(b)];
        if (uid >= 0 && uid < A.num_users) v = A.ubias[uid];
      }
      ub[r] = v + (A.cbias ? A.cbias[0] : 0.f);
    }
  }
  // LIST state: list for user row i lives in (lv[i], li[i])
  float lv[LIST ? 32 : 1];
  int li[LIST ? 32 : 1];
  if (LIST) {
#pragma unroll
    for (int i = 0; i < 32; ++i) { lv[i] = -__builtin_inff(); li[i] = HNM_SENTINEL_IDX; }
  }
  // mask cursor of user (b0 + lane), lanes < 32 (real item ids; item i is i * istride)
  const int64_t S = A.istride;
  int nm = INT_BIG;
  int64_t mpos = 0, mend = 0;
  if (!DENSE && A.mptr && lane < 32 && b0 + lane < Bl) {
    const int64_t r = req(b0 + lane);
    const int64_t lo = A.mptr[r], hi = A.mptr[r + 1];
    mpos = mask_lower_bound(A.midx, lo, hi, (int)(part_start * S));
    mend = hi;
    nm = mpos < mend ? A.midx[mpos] : INT_BIG;
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
      if (item < part_end && 4 * c4 < A.d)
        v = *reinterpret_cast<const float4*>(A.it + item * S * A.ldi + 4 * c4);
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
      if (BIAS && A.ibias && ivalid) ib = A.ibias[item * S];
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = BIAS ? (acc[r] + ub[r]) + ib : acc[r];
    }

    if (DENSE) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t b = b0 + mfma32_row(r, h);
        if (ivalid && b < Bl) A.dense[req(b) * A.ldo + item] = sc[r];
      }
    } else {
      const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);
      const int64_t real_end = (tile_end - 1) * S + 1;  // real ids of this tile are < real_end
      // -inf for masked (user, item) pairs inside this tile (rare path)
      uint64_t mm = __ballot(lane < 32 && nm < real_end) & 0xffffffffull;
      while (mm) {
        const int u = __builtin_ctzll(mm);
        mm &= mm - 1;
        while (true) {
          const int tgt = hnm_readlane_i(nm, u);
          if (tgt >= real_end) break;
          if (tgt % S == 0) {
            const int64_t ti = tgt / S;
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (mfma32_row(r, h) == u && item == ti) sc[r] = -__builtin_inff();
          }
          if (lane == u) {
            ++mpos;
            nm = mpos < mend ? A.midx[mpos] : INT_BIG;
          }
        }
      }
      if (THRESH) {
        // append every score >= tau_u (rare after the sample pass): one ballot per tile
        bool any = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) any |= sc[r] >= tv[r];
        if (__ballot(ivalid && any))
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (ivalid && sc[r] >= tv[r]) {
            const int64_t rq = req(b0 + mfma32_row(r, h));
            const int slot = atomicAdd(&A.cnt[rq], 1);
            if (slot < A.cap) {
              A.buf_v[rq * A.cap + slot] = sc[r];
              A.buf_i[rq * A.cap + slot] = (int)item;
            }
          }
        }
      } else {
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
              list1_insert(lv[i0], li[i0], hnm_readlane_f(sc[r], l), (int)(base + l), (int)K);
            }
            while (hi) {
              const int l = __builtin_ctzll(hi);
              hi &= hi - 1;
              list1_insert(lv[i1], li[i1], hnm_readlane_f(sc[r], 32 + l), (int)(base + l), (int)K);
            }
            const float t0 = hnm_readlane_f(lv[i0], K - 1);
            const float t1 = hnm_readlane_f(lv[i1], K - 1);
            tv[r] = h ? t1 : t0;
          }
        }
      }
    }

    if (t + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  if (LIST) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int64_t b = b0 + i;
      if (b < Bl && lane < K) {
        const int64_t o = (b * NP + p) * K + lane;
        A.cand_v[o] = lv[i];
        A.cand_i[o] = li[i] == HNM_SENTINEL_IDX ? -1 : li[i];
      }
    }
  }
}

// ------------------------------------------------------------------ threshold select
// Row b: exact top-K of its appended candidates.  A row with more than `cap` appends, or
// fewer than K (NaN thresholds), is queued for the LIST fallback instead.
__global__ __launch_bounds__(256) void thresh_select_kernel(const int* __restrict__ cnt,
                                                            const float* __restrict__ bv,
                                                            const int32_t* __restrict__ bi,
                                                            int cap, int64_t B, int K,
                                                            float* __restrict__ ov,
                                                            int64_t* __restrict__ oi,
                                                            int32_t* __restrict__ ovf_rows,
                                                            int32_t* __restrict__ ovf_cnt) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const int n = cnt[b];
  if (n > cap || n < K) {
    if (lane == 0) ovf_rows[atomicAdd(ovf_cnt, 1)] = (int32_t)b;
    return;
  }
  WaveTopK<1> L;
  L.init();
  for (int base = 0; base < n; base += 64) {
    const int q = base + lane;
    const bool ok = q < n;
    L.offer(ok ? bv[b * cap + q] : -__builtin_inff(), ok ? bi[b * cap + q] : HNM_SENTINEL_IDX,
            ok, K);
  }
  L.store(ov ? ov + b * K : nullptr, oi + b * K, K);
}

// ------------------------------------------------------------------ row top-K (dense in)
// torch.topk(scores, k) replacement over a dense [B, I] matrix with an optional CSR mask
// (serve.py:350-355).  One wave per row; K <= 128.
// `istride`: column c holds real item c * istride (mask ids are real item ids).
template <int NS>
__global__ __launch_bounds__(256) void rows_topk_kernel(const float* __restrict__ s,
                                                        int64_t ld, int64_t B, int64_t I,
                                                        const int64_t* __restrict__ mptr,
                                                        const int32_t* __restrict__ midx,
                                                        int K, float* __restrict__ ov,
                                                        int64_t* __restrict__ oi,
                                                        int64_t istride = 1) {
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
    const int64_t end = (std::min<int64_t>(base + 64, I) - 1) * istride + 1;  // real ids < end
    while (nm < end) {
      if (nm % istride == 0 && item == nm / istride) v = -__builtin_inff();
      ++mpos;
      nm = mpos < mend ? midx[mpos] : INT_BIG;
    }
    L.offer(v, (int)item, valid, K);
  }
  L.store(ov ? ov + b * K : nullptr, oi + b * K, K);
}

// Small batches (serve path: one user per request, k up to 100): each row is cut into P
// column chunks, one wave per (row, chunk) keeps the chunk's top-K (int32 ids), and the
// P partial lists are merged by topk_merge (same total order => same result as one wave).
template <int NS>
__global__ __launch_bounds__(256) void rows_topk_split_kernel(const float* __restrict__ s,
                                                              int64_t ld, int64_t B, int64_t I,
                                                              int64_t chunk,
                                                              const int64_t* __restrict__ mptr,
                                                              const int32_t* __restrict__ midx,
                                                              int K, float* __restrict__ pv,
                                                              int32_t* __restrict__ pi) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const int64_t lo = (int64_t)blockIdx.y * chunk, hi = std::min<int64_t>(I, lo + chunk);
  WaveTopK<NS> L;
  L.init();
  int64_t mpos = 0, mend = 0;
  int nm = INT_BIG;
  if (mptr) {
    mend = mptr[b + 1];
    mpos = mask_lower_bound(midx, mptr[b], mend, (int)lo);
    nm = mpos < mend ? midx[mpos] : INT_BIG;
  }
  const float* row = s + b * ld;
  for (int64_t base = lo; base < hi; base += 64) {
    const int64_t item = base + lane;
    const bool valid = item < hi;
    float v = valid ? row[item] : -__builtin_inff();
    const int64_t end = std::min<int64_t>(base + 64, hi);
    while (nm < end) {
      if (item == nm) v = -__builtin_inff();
      ++mpos;
      nm = mpos < mend ? midx[mpos] : INT_BIG;
    }
    L.offer(v, (int)item, valid, K);
  }
  const int64_t o = ((int64_t)blockIdx.y * B + b) * K;
  L.store(pv + o, pi + o, K);
}

// ------------------------------------------------------------------ host side
hnm_status hnm_sample_kth(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t Ns,
                          const int64_t* mptr, const int32_t* midx, int K, int64_t grp,
                          int64_t period, const int32_t* sidx, float* out, const int* gate) {
  return sample_kth_launch(ctx, s, ld, B, Ns, mptr, midx, K, grp, period, sidx, out, gate,
                           KthNoEpi{});
}

hnm_status hnm_topk_rows_strided(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t I,
                                 const int64_t* mptr, const int32_t* midx, int K, float* ov,
                                 int64_t* oi, int64_t istride) {
  HNM_REQUIRE(K >= 1 && K <= 64, HNM_EINVAL, "topk_rows_strided: 1 <= K <= 64");
  hipLaunchKernelGGL(rows_topk_kernel<1>, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0,
                     ctx->stream, s, ld, B, I, mptr, midx, K, ov, oi, istride);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}


template <int MODE>
static void launch_dot(hnm_ctx* ctx, dim3 grid, const DotArgs& a, bool bias) {
#define HNM_DOT(DPV)                                                                     \
  if (bias)                                                                              \
    hipLaunchKernelGGL((dot_score_kernel<DPV, MODE, true>), grid, dim3(256), 0, ctx->stream, a); \
  else                                                                                   \
    hipLaunchKernelGGL((dot_score_kernel<DPV, MODE, false>), grid, dim3(256), 0, ctx->stream, a);
  if (a.d <= 64) {
    HNM_DOT(64)
  } else {
    HNM_DOT(128)
  }
#undef HNM_DOT
}

// Sample-threshold design parameters (see the header comment).
#define THRESH_MIN_ITEMS 8192
#define THRESH_SAMPLE 4096

static hnm_status dot_validate(hnm_ctx* ctx, const float* ut, int64_t U, int64_t ldu,
                               const int64_t* ids, int64_t B, const float* it, int64_t I,
                               int64_t ldi, int d) {
  HNM_REQUIRE(ctx && ut && (ids || B == 0) && it, HNM_EINVAL, "dot: NULL argument");
  HNM_REQUIRE(d >= 1 && d <= 128 && ldu >= d && ldi >= d && U > 0 && I > 0, HNM_EINVAL,
              "dot: bad shape (d=%d)", d);
  HNM_REQUIRE(d % 4 == 0 && ldu % 4 == 0 && ldi % 4 == 0 && (uintptr_t)ut % 16 == 0 &&
                  (uintptr_t)it % 16 == 0,
              HNM_EUNSUPPORTED, "dot: tables must be 16-B aligned with d %% 4 == 0");
  HNM_REQUIRE(I < INT_BIG, HNM_EUNSUPPORTED, "dot: too many items");
  return HNM_OK;
}

DotArgs dot_args(hnm_ctx* ctx, const float* ut, int64_t U, int64_t ldu, const int64_t* ids,
                        int64_t B, const float* it, int64_t I, int64_t ldi, int d, const float* ub,
                        const float* ib, const float* cb, const int64_t* mptr,
                        const int32_t* midx, int K) {
  DotArgs a = {};
  a.ut = ut; a.num_users = U; a.ldu = ldu; a.uids = ids; a.B = B;
  a.it = it; a.I = I; a.ldi = ldi; a.istride = 1; a.d = d;
  a.ubias = ub; a.ibias = ib; a.cbias = cb;
  a.mptr = mptr; a.midx = midx; a.K = K;
  a.err = ctx->err_dev;
  return a;
}

// LIST pass over `a` (items a.I with stride a.istride) -> merged top-K into ov/oi rows
// (rows remapped through a.rows when set).
hnm_status dot_list_pass(hnm_ctx* ctx, DotArgs a, bool bias, float* cv, int32_t* ci,
                                float* ov, int64_t* oi) {
  const int64_t ublocks = hnm_cdiv(a.B, 128);
  a.cand_v = cv;
  a.cand_i = ci;
  if (a.rows) {
    // the queued rows are known only on the device: the widest grid, the partitions used
    // derived from *nrows in the kernel and the merge (hnm_internal.h list_rows_np)
    a.ipp = 0;
    a.NP = 1;
    a.dyn_cus = ctx->num_cus;
    launch_dot<DOT_LIST>(ctx, dim3((unsigned)list_rows_grid(a.B, a.I, ctx->num_cus), 1), a, bias);
    HNM_LAUNCH_CHECK();
    return hnm_topk_merge_rows(ctx, cv, ci, a.B, 1, 0, a.K, a.K, a.K, ov, oi, a.rows, a.nrows,
                               a.I, ctx->num_cus);
  }
  Partition part = choose_partition(a.I, ublocks, ctx->num_cus);
  a.ipp = part.ipp;
  a.NP = part.np;
  launch_dot<DOT_LIST>(ctx, dim3((unsigned)ublocks, (unsigned)part.np), a, bias);
  HNM_LAUNCH_CHECK();
  return hnm_topk_merge_rows(ctx, cv, ci, a.B, 1, 0, (int64_t)part.np * a.K, part.np * a.K, a.K,
                             ov, oi, a.rows, a.nrows);
}

size_t list_cand_bytes(int64_t B, int64_t I, int K, int num_cus) {
  Partition part = choose_partition(I, hnm_cdiv(B, 128), num_cus);
  const int64_t slots = std::max<int64_t>(B * part.np, list_rows_slots(B, I, num_cus));
  return hnm_align((size_t)slots * K * 4);
}

extern "C" hnm_status hnm_dot_topk_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                       int64_t ldu, const int64_t* user_ids, int64_t B,
                                       const float* item_tab, int64_t num_items, int64_t ldi,
                                       int d, const float* user_bias, const float* item_bias,
                                       const float* const_bias, const int64_t* mask_ptr,
                                       const int32_t* mask_idx, int k, float* out_val,
                                       int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = dot_validate(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d);
  if (st) return st;
  HNM_REQUIRE(k >= 1 && k <= 64 && (out_idx || B == 0), HNM_EINVAL, "dot_topk: fused path needs 1 <= k <= 64");
  if (B <= 0) return HNM_OK;
  const int64_t I = num_items;
  const bool bias = user_bias || item_bias || const_bias;
  DotArgs a = dot_args(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, I, ldi, d, user_bias,
                       item_bias, const_bias, mask_ptr, mask_idx, k);
  if (ctx->prefilter && dot_cert_eligible(d, I, k)) {  // certified f16 scan (dot_cert.hip)
    void* w;
    st = hnm_workspace(ctx, dot_cert_bytes(B, I, d, k, ctx->num_cus), &w);
    if (st) return st;
    return dot_cert_topk(ctx, a, bias, w, out_val, out_idx);
  }
  if (I < THRESH_MIN_ITEMS || I < 4 * (int64_t)k) {
    const size_t sc = list_cand_bytes(B, I, k, ctx->num_cus);
    void* w;
    st = hnm_workspace(ctx, 2 * sc, &w);
    if (st) return st;
    hnm_timer_begin(ctx, HNM_TIME_SCORE);
    st = dot_list_pass(ctx, a, bias, (float*)w, (int32_t*)((char*)w + sc), out_val, out_idx);
    hnm_timer_end(ctx, HNM_TIME_SCORE);
    return st;
  }
  // ---- threshold path
  const int64_t stride = std::max<int64_t>(1, I / THRESH_SAMPLE);
  const int64_t Ns = hnm_cdiv(I, stride);
  const int cap = (int)std::min<int64_t>(8192, std::max<int64_t>(256, 8 * (int64_t)k * stride));
  const size_t s_samp = list_cand_bytes(B, Ns, k, ctx->num_cus);
  const size_t s_full = list_cand_bytes(B, I, k, ctx->num_cus);
  const size_t s_tau = hnm_align((size_t)B * k * 4), s_taui = hnm_align((size_t)B * k * 8);
  const size_t s_cnt = hnm_align((size_t)B * 4), s_buf = hnm_align((size_t)B * cap * 4);
  const size_t s_rows = hnm_align((size_t)B * 4 + 256);
  const size_t s_cand = std::max(s_samp, s_full);
  const size_t s_sd = hnm_align((size_t)B * Ns * 4);
  void* w;
  st = hnm_workspace(ctx, 2 * s_cand + s_tau + s_taui + s_cnt + 2 * s_buf + s_rows + s_sd, &w);
  if (st) return st;
  char* q = (char*)w;
  float* cv = (float*)q; q += s_cand;
  int32_t* ci = (int32_t*)q; q += s_cand;
  float* tau = (float*)q; q += s_tau;
  int64_t* taui = (int64_t*)q; q += s_taui;
  int* cnt = (int*)q; q += s_cnt;
  float* bv = (float*)q; q += s_buf;
  int32_t* bi = (int32_t*)q; q += s_buf;
  int32_t* ovf_cnt = (int32_t*)q; q += s_rows;
  int32_t* ovf_rows = ovf_cnt + 64;
  float* sdense = (float*)q;
  HNM_HIP_CHECK(hipMemsetAsync(cnt, 0, (size_t)B * 4, ctx->stream));
  HNM_HIP_CHECK(hipMemsetAsync(ovf_cnt, 0, 4, ctx->stream));
  // 1. sample pass: dense scores of items 0, stride, 2*stride, ... (masks applied by the
  //    row top-K), tau_u = K-th best of them
  {
    DotArgs as = a;
    as.istride = stride;
    as.I = Ns;
    as.mptr = nullptr;
    as.midx = nullptr;
    Partition ps = choose_partition(Ns, hnm_cdiv(B, 128), 2 * ctx->num_cus);
    as.ipp = ps.ipp;
    as.NP = ps.np;
    as.dense = sdense;
    as.ldo = Ns;
    launch_dot<DOT_DENSE>(ctx, dim3((unsigned)hnm_cdiv(B, 128), (unsigned)ps.np), as, bias);
    HNM_LAUNCH_CHECK();
    hipLaunchKernelGGL(rows_topk_kernel<1>, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0,
                       ctx->stream, sdense, Ns, B, Ns, mask_ptr, mask_idx, k, tau, taui, stride);
    HNM_LAUNCH_CHECK();
  }
  // 2. main pass: append scores >= tau_u
  DotArgs am = a;
  const int64_t ublocks = hnm_cdiv(B, 128);
  Partition part = choose_partition(I, ublocks, 2 * ctx->num_cus);
  am.ipp = part.ipp;
  am.NP = part.np;
  am.tau = tau + (k - 1);
  am.tau_ld = k;
  am.cnt = cnt;
  am.buf_v = bv;
  am.buf_i = bi;
  am.cap = cap;
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
  launch_dot<DOT_THRESH>(ctx, dim3((unsigned)ublocks, (unsigned)part.np), am, bias);
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  // 3. exact top-K of the appended candidates; overflowing rows -> fallback list
  hipLaunchKernelGGL(thresh_select_kernel, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0,
                     ctx->stream, cnt, bv, bi, cap, B, k, out_val, out_idx, ovf_rows, ovf_cnt);
  HNM_LAUNCH_CHECK();
  // 4. fallback: exact LIST pass restricted (on device) to the queued rows
  DotArgs af = a;
  af.rows = ovf_rows;
  af.nrows = ovf_cnt;
  return dot_list_pass(ctx, af, bias, cv, ci, out_val, out_idx);
}

// Two-phase hnm_dot_topk_f32 for item-sharded serving (see hnm_ncf_topk_begin_f32): one
// lower bound per row (lower_bound) or the row's k best sample lower bounds (lists, [B, k]).
static hnm_status dot_topk_begin(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                 int64_t ldu, const int64_t* user_ids, int64_t B,
                                 const float* item_tab, int64_t num_items, int64_t ldi, int d,
                                 const float* user_bias, const float* item_bias,
                                 const float* const_bias, const int64_t* mask_ptr,
                                 const int32_t* mask_idx, int k, float* lower_bound,
                                 float* lists) {
  hnm_status st = dot_validate(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d);
  if (st) return st;
  HNM_REQUIRE(k >= 1 && k <= 64 && (lower_bound || lists || B == 0), HNM_EINVAL,
              "dot_topk_begin: bad argument");
  HNM_REQUIRE(!ctx->pend.kind, HNM_EINVAL, "dot_topk_begin: a two-phase call is already open");
  if (B <= 0) return HNM_OK;
  const bool cert = ctx->prefilter && dot_cert_eligible(d, num_items, k);
  if (cert) {
    const bool bias = user_bias || item_bias || const_bias;
    DotArgs a = dot_args(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                         user_bias, item_bias, const_bias, mask_ptr, mask_idx, k);
    void* w;
    st = hnm_workspace(ctx, dot_cert_bytes(B, num_items, d, k, ctx->num_cus), &w);
    if (st) return st;
    st = dot_cert_begin(ctx, a, bias, w, lower_bound, lists);
    if (st) return st;
  } else {
    if (lower_bound && (st = hnm_fill_f32(ctx, lower_bound, B, -__builtin_inff()))) return st;
    if (lists && (st = hnm_fill_f32(ctx, lists, B * k, -__builtin_inff()))) return st;
  }
  ctx->pend = {cert ? HNM_PEND_DOT_CERT : HNM_PEND_DOT_EXACT, B, num_items, k, user_ids, item_tab};
  return HNM_OK;
}

extern "C" hnm_status hnm_dot_topk_begin_f32(hnm_ctx* ctx, const float* user_tab,
                                             int64_t num_users, int64_t ldu,
                                             const int64_t* user_ids, int64_t B,
                                             const float* item_tab, int64_t num_items,
                                             int64_t ldi, int d, const float* user_bias,
                                             const float* item_bias, const float* const_bias,
                                             const int64_t* mask_ptr, const int32_t* mask_idx,
                                             int k, float* lower_bound) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(lower_bound || B == 0, HNM_EINVAL, "dot_topk_begin: lower_bound is NULL");
  return dot_topk_begin(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                        user_bias, item_bias, const_bias, mask_ptr, mask_idx, k, lower_bound,
                        nullptr);
}

extern "C" hnm_status hnm_dot_topk_begin_lists_f32(hnm_ctx* ctx, const float* user_tab,
                                                   int64_t num_users, int64_t ldu,
                                                   const int64_t* user_ids, int64_t B,
                                                   const float* item_tab, int64_t num_items,
                                                   int64_t ldi, int d, const float* user_bias,
                                                   const float* item_bias,
                                                   const float* const_bias,
                                                   const int64_t* mask_ptr,
                                                   const int32_t* mask_idx, int k,
                                                   float* lower_lists) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(lower_lists || B == 0, HNM_EINVAL, "dot_topk_begin_lists: lower_lists is NULL");
  return dot_topk_begin(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                        user_bias, item_bias, const_bias, mask_ptr, mask_idx, k, nullptr,
                        lower_lists);
}

extern "C" hnm_status hnm_dot_topk_finish_f32(hnm_ctx* ctx, const float* user_tab,
                                              int64_t num_users, int64_t ldu,
                                              const int64_t* user_ids, int64_t B,
                                              const float* item_tab, int64_t num_items,
                                              int64_t ldi, int d, const float* user_bias,
                                              const float* item_bias, const float* const_bias,
                                              const int64_t* mask_ptr, const int32_t* mask_idx,
                                              int k, const float* lower_bound, int short_ok,
                                              float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && (out_idx || B == 0), HNM_EINVAL, "dot_topk_finish: bad argument");
  if (B <= 0) return HNM_OK;
  const int kind = ctx->pend.kind;
  HNM_REQUIRE((kind == HNM_PEND_DOT_CERT || kind == HNM_PEND_DOT_EXACT) && ctx->pend.B == B &&
                  ctx->pend.K == k && ctx->pend.I == num_items && ctx->pend.ids == user_ids &&
                  ctx->pend.items == item_tab,
              HNM_EINVAL, "dot_topk_finish: no matching hnm_dot_topk_begin_f32 on this ctx");
  ctx->pend.kind = 0;
  if (kind == HNM_PEND_DOT_EXACT)
    return hnm_dot_topk_f32(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi,
                            d, user_bias, item_bias, const_bias, mask_ptr, mask_idx, k, out_val,
                            out_idx);
  HNM_REQUIRE(lower_bound, HNM_EINVAL, "dot_topk_finish: lower_bound is NULL");
  hnm_status st = dot_validate(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d);
  if (st) return st;
  HNM_REQUIRE(ctx->ws && ctx->ws_size >= dot_cert_bytes(B, num_items, d, k, ctx->num_cus),
              HNM_EINVAL, "dot_topk_finish: the begin phase's workspace is gone");
  const bool bias = user_bias || item_bias || const_bias;
  DotArgs a = dot_args(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                       user_bias, item_bias, const_bias, mask_ptr, mask_idx, k);
  return dot_cert_finish(ctx, a, bias, ctx->ws, lower_bound, short_ok, out_val, out_idx);
}

extern "C" hnm_status hnm_dot_scores_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                         int64_t ldu, const int64_t* user_ids, int64_t B,
                                         const float* item_tab, int64_t num_items, int64_t ldi,
                                         int d, const float* user_bias, const float* item_bias,
                                         const float* const_bias, float* out, int64_t ldo) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = dot_validate(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d);
  if (st) return st;
  HNM_REQUIRE((out || B == 0) && ldo >= num_items, HNM_EINVAL, "dot_scores: bad output");
  if (B <= 0) return HNM_OK;
  DotArgs a = dot_args(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                       user_bias, item_bias, const_bias, nullptr, nullptr, 1);
  const int64_t ublocks = hnm_cdiv(B, 128);
  Partition part = choose_partition(num_items, ublocks, 2 * ctx->num_cus);
  a.ipp = part.ipp;
  a.NP = part.np;
  a.dense = out;
  a.ldo = ldo;
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
  launch_dot<DOT_DENSE>(ctx, dim3((unsigned)ublocks, (unsigned)part.np), a,
                        user_bias || item_bias || const_bias);
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_topk_rows_f32(hnm_ctx* ctx, const float* scores, int64_t ld, int64_t B,
                                        int64_t I, const int64_t* mask_ptr,
                                        const int32_t* mask_idx, int k, float* out_val,
                                        int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((scores && out_idx) || B == 0), HNM_EINVAL, "topk_rows: NULL argument");
  HNM_REQUIRE(k >= 1 && k <= I && ld >= I, HNM_EINVAL, "topk_rows: bad k/shape");
  HNM_REQUIRE(I < INT_BIG, HNM_EUNSUPPORTED, "topk_rows: too many items");
  if (B <= 0) return HNM_OK;
  if (k > 128)  // whole-row stable sort (topk_sort.hip)
    return hnm_topk_rows_sort(ctx, scores, ld, B, I, mask_ptr, mask_idx, k, out_val, out_idx);
  // fewer rows than ~1024 waves: split the rows into column chunks of >= 2048 items
  const int64_t P = std::min<int64_t>(hnm_cdiv(1024, B), hnm_cdiv(I, 2048));
  if (P > 1) {
    const int64_t chunk = hnm_cdiv(I, P);
    void* w;
    hnm_status st = hnm_workspace(ctx, (size_t)P * B * k * 8, &w);
    if (st) return st;
    float* pv = (float*)w;
    int32_t* pi = (int32_t*)(pv + P * B * k);
    dim3 g2((unsigned)hnm_cdiv(B, 4), (unsigned)P);
    if (k <= 64)
      hipLaunchKernelGGL(rows_topk_split_kernel<1>, g2, dim3(256), 0, ctx->stream, scores, ld, B,
                         I, chunk, mask_ptr, mask_idx, k, pv, pi);
    else
      hipLaunchKernelGGL(rows_topk_split_kernel<2>, g2, dim3(256), 0, ctx->stream, scores, ld, B,
                         I, chunk, mask_ptr, mask_idx, k, pv, pi);
    HNM_LAUNCH_CHECK();
    return hnm_topk_merge_rows(ctx, pv, pi, B, P, B * k, k, k, k, out_val, out_idx, nullptr,
                               nullptr);
  }
  dim3 grid((unsigned)hnm_cdiv(B, 4));
  if (k <= 64)
    hipLaunchKernelGGL(rows_topk_kernel<1>, grid, dim3(256), 0, ctx->stream, scores, ld, B, I,
                       mask_ptr, mask_idx, k, out_val, out_idx, (int64_t)1);
  else
    hipLaunchKernelGGL(rows_topk_kernel<2>, grid, dim3(256), 0, ctx->stream, scores, ld, B, I,
                       mask_ptr, mask_idx, k, out_val, out_idx, (int64_t)1);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}


extern "C" hnm_status hnm_dot_prefilter_debug_f32(hnm_ctx* ctx, const float* user_tab,
                                                  int64_t num_users, int64_t ldu,
                                                  const int64_t* user_ids, int64_t B,
                                                  const float* item_tab, int64_t num_items,
                                                  int64_t ldi, int d, const float* user_bias,
                                                  const float* item_bias, const float* const_bias,
                                                  float* approx, int64_t lda, float* bound) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = dot_validate(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d);
  if (st) return st;
  HNM_REQUIRE(approx && bound && lda >= num_items, HNM_EINVAL, "dot_prefilter_debug: bad output");
  HNM_REQUIRE(num_items * (d <= 64 ? 64 : 128) * 2 < ((int64_t)1 << 31), HNM_EUNSUPPORTED,
              "dot_prefilter_debug: the scan's f16 item copy must stay below 2 GiB");
  if (B <= 0) return HNM_OK;
  const bool bias = user_bias || item_bias || const_bias;
  DotArgs a = dot_args(ctx, user_tab, num_users, ldu, user_ids, B, item_tab, num_items, ldi, d,
                       user_bias, item_bias, const_bias, nullptr, nullptr, 1);
  void* w;
  st = hnm_workspace(ctx, dot_cert_bytes(B, num_items, d, 1, ctx->num_cus), &w);
  if (st) return st;
  return dot_cert_debug(ctx, a, bias, w, approx, lda, bound);
}
