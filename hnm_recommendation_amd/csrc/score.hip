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
// ncf_score_kernel  (NeuralCF, neural_cf.py:143-208 + 300-326)
//   layer 1 is decomposed: W1 [m_u; m_i] + b1 = P_u + Q_i (per-user / per-item
//   projections computed once per call by hnm_linear_rows_f32).  Per (user, 32 items):
//   B = relu(P_u + Q_i) is built in registers, layer 2 runs on MFMA with W2 as the A
//   operand held in registers (D = W2 . H1^T: rows = hidden units, cols = items), the
//   ReLU + prediction dot is a 16-register epilogue + one cross-half shuffle, and the
//   GMF term (wp_gmf * g_u) . g_i is a 32-FMA lane-half dot.  Only the per-user score
//   stream touches the wave top-K list.
//
// Both kernels cover one item PARTITION per blockIdx.y; partial top-K lists go to a
// [B, NP, K] candidate buffer merged by topk_merge_kernel (total order: score desc,
// item asc, so the merged result is unique).
#include <algorithm>

#include "hnm_device.h"
#include "hnm_internal.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);

#define TILE 32
#define INT_BIG 0x7fffffff

// ------------------------------------------------------------------ list helpers
// Insert (cv, ci) into a single-register wave list (slot s in lane s, K <= 64).
__device__ __forceinline__ void list1_insert(float& lv, int& li, float cv, int ci, int K) {
  const float tv = hnm_readlane_f(lv, K - 1);
  const int ti = hnm_readlane_i(li, K - 1);
  if (!hnm_better(cv, ci, tv, ti)) return;
  const int lane = hnm_lane();
  const bool b = (lane < K) && hnm_better(lv, li, cv, ci);
  const int pos = __popcll(__ballot(b));
  const float up = __shfl_up(lv, 1);
  const int upi = __shfl_up(li, 1);
  lv = lane > pos ? up : (lane == pos ? cv : lv);
  li = lane > pos ? upi : (lane == pos ? ci : li);
}

// First masked item >= start in the sorted row [lo, hi) of midx.
__device__ __forceinline__ int64_t mask_lower_bound(const int32_t* midx, int64_t lo, int64_t hi,
                                                    int start) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (midx[mid] < start) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

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

// ------------------------------------------------------------------ NCF kernel
template <int WU, int H1P, int MFH, bool DENSE>
__global__ __launch_bounds__(256, 2) void ncf_score_kernel(
    const float* __restrict__ Pu,   // [B, H1P]  pair-permuted  W1u m_u + b1
    const float* __restrict__ WGu,  // [B, 2*MFH] wp_gmf * g_u
    const float* __restrict__ Qi,   // [I, H1P]  pair-permuted  W1i m_i
    const float* __restrict__ Gi, int64_t ldg,  // [I, >= 2*MFH] gmf item table (zero pad)
    const float* __restrict__ W2, int h1, int h2, const float* __restrict__ b2,
    const float* __restrict__ wm, const float* __restrict__ bp, int64_t B, int64_t I,
    int64_t ipp, const int64_t* __restrict__ mptr, const int32_t* __restrict__ midx, int K,
    float* __restrict__ cand_v, int32_t* __restrict__ cand_i, int NP,
    float* __restrict__ dense, int64_t ldo) {
  constexpr int KS = H1P / 2;
  constexpr int GW = 2 * MFH;
  constexpr int QRS = H1P + 4;
  constexpr int GRS = GW + 4;
  constexpr int NU = 4 * WU;
  constexpr int QF4 = TILE * H1P / 4 / 256;  // float4 per thread per tile
  constexpr int GF4 = TILE * GW / 4 / 256;
  static_assert(QF4 >= 1 && GF4 >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) float qs[2][TILE * QRS];
  __shared__ __attribute__((aligned(16))) float gs[2][TILE * GRS];
  __shared__ __attribute__((aligned(16))) float ps[NU * H1P];
  __shared__ __attribute__((aligned(16))) float ws[NU * GW];
  __shared__ __attribute__((aligned(16))) float2 bw[32];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;
  const int j = lane & 31;
  const int64_t ublk = (int64_t)blockIdx.x * NU;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + ipp);

  // user rows of the block -> LDS
  for (int e = tid; e < NU * H1P / 4; e += 256) {
    const int r = e / (H1P / 4), c = e % (H1P / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ublk + r < B) v = *reinterpret_cast<const float4*>(Pu + (ublk + r) * H1P + 4 * c);
    *reinterpret_cast<float4*>(&ps[r * H1P + 4 * c]) = v;
  }
  for (int e = tid; e < NU * GW / 4; e += 256) {
    const int r = e / (GW / 4), c = e % (GW / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ublk + r < B) v = *reinterpret_cast<const float4*>(WGu + (ublk + r) * GW + 4 * c);
    *reinterpret_cast<float4*>(&ws[r * GW + 4 * c]) = v;
  }

  // A operand = W2 rows (hidden unit i = lane&31), k = 2s + h; epilogue constants per C reg
  float a[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    a[s] = (j < h2 && k < h1) ? W2[j * h1 + k] : 0.f;
  }
  // (b2, wm) per hidden unit, read by the epilogue from LDS (keeps 32 VGPRs free)
  if (tid < 32) bw[tid] = tid < h2 ? make_float2(b2[tid], wm[tid]) : make_float2(0.f, 0.f);
  const float bpv = bp[0];

  WaveTopK<1> L[WU];
  int nm[WU], mpos[WU], mend[WU];  // wave-uniform mask cursors (mask nnz < 2^31)
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    L[u].init();
    nm[u] = INT_BIG;
    mpos[u] = 0;
    mend[u] = 0;
    const int64_t b = ublk + wave * WU + u;
    if (!DENSE && mptr && b < B) {
      const int64_t lo = mptr[b], hi = mptr[b + 1];
      mpos[u] = (int)mask_lower_bound(midx, lo, hi, (int)part_start);
      mend[u] = (int)hi;
      nm[u] = mpos[u] < mend[u] ? midx[mpos[u]] : INT_BIG;
    }
  }

  float4 qst[QF4], gst[GF4];
  auto load_tile = [&](int64_t base) {
#pragma unroll
    for (int q = 0; q < QF4; ++q) {
      const int f = tid + 256 * q;
      const int row = f / (H1P / 4), c = f % (H1P / 4);
      const int64_t item = base + row;
      qst[q] = item < part_end ? *reinterpret_cast<const float4*>(Qi + item * H1P + 4 * c)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < GF4; ++q) {
      const int f = tid + 256 * q;
      const int row = f / (GW / 4), c = f % (GW / 4);
      const int64_t item = base + row;
      gst[q] = item < part_end ? *reinterpret_cast<const float4*>(Gi + item * ldg + 4 * c)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int q = 0; q < QF4; ++q) {
      const int f = tid + 256 * q;
      const int row = f / (H1P / 4), c = f % (H1P / 4);
      *reinterpret_cast<float4*>(&qs[buf][row * QRS + 4 * c]) = qst[q];
    }
#pragma unroll
    for (int q = 0; q < GF4; ++q) {
      const int f = tid + 256 * q;
      const int row = f / (GW / 4), c = f % (GW / 4);
      *reinterpret_cast<float4*>(&gs[buf][row * GRS + 4 * c]) = gst[q];
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

    // 64-wide hidden layer: this lane's Q values stay in registers across the WU users;
    // the 128-wide variant re-reads them from LDS per user (register budget).
    constexpr bool QREG = false;  // q re-read per user pair (shared by both chains)
    float q[QREG ? KS : 1];
    const float* qrow = &qs[buf][j * QRS + h * KS];
    const float* grow = &gs[buf][j * GRS + h * MFH];
    if (QREG) {
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 v = *reinterpret_cast<const float4*>(qrow + 4 * s4);
        q[4 * s4] = v.x; q[4 * s4 + 1] = v.y; q[4 * s4 + 2] = v.z; q[4 * s4 + 3] = v.w;
      }
    }
    const int64_t item = base + j;
    const bool ivalid = (lane < 32) && item < part_end;
    const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);

    // Users are processed in pairs: two independent accumulator chains interleaved so
    // each MFMA's accumulator dependency is two issues back, with the LDS reads of the
    // next 4-step group issued before the current group's MFMAs.
#pragma unroll
    for (int up = 0; up < WU; up += 2) {
      constexpr int dummy = 0;
      (void)dummy;
      const bool pair = (up + 1 < WU);  // compile-time after unrolling
      const int urA = wave * WU + up;
      const int urB = pair ? urA + 1 : urA;
      const int64_t bA = ublk + urA, bB = ublk + urB;
      if (bA >= B) break;
      f32x16 accA = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      f32x16 accB = accA;
      const float* prA = &ps[urA * H1P + h * KS];
      const float* prB = &ps[urB * H1P + h * KS];
      float4 pa = *reinterpret_cast<const float4*>(prA);
      float4 pb = *reinterpret_cast<const float4*>(prB);
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        float4 na = pa, nb = pb;
        if (s4 + 1 < KS / 4) {
          na = *reinterpret_cast<const float4*>(prA + 4 * (s4 + 1));
          if (pair) nb = *reinterpret_cast<const float4*>(prB + 4 * (s4 + 1));
        }
        float4 qv;
        if (QREG) qv = make_float4(q[4 * s4], q[4 * s4 + 1], q[4 * s4 + 2], q[4 * s4 + 3]);
        else qv = *reinterpret_cast<const float4*>(qrow + 4 * s4);
        accA = mfma32x32x2(a[4 * s4 + 0], fmaxf(pa.x + qv.x, 0.f), accA);
        if (pair) accB = mfma32x32x2(a[4 * s4 + 0], fmaxf(pb.x + qv.x, 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 1], fmaxf(pa.y + qv.y, 0.f), accA);
        if (pair) accB = mfma32x32x2(a[4 * s4 + 1], fmaxf(pb.y + qv.y, 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 2], fmaxf(pa.z + qv.z, 0.f), accA);
        if (pair) accB = mfma32x32x2(a[4 * s4 + 2], fmaxf(pb.z + qv.z, 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 3], fmaxf(pa.w + qv.w, 0.f), accA);
        if (pair) accB = mfma32x32x2(a[4 * s4 + 3], fmaxf(pb.w + qv.w, 0.f), accB);
        pa = na;
        pb = nb;
      }
      // GMF term for both users with one pass over this lane's g_i half
      float gmfA = 0.f, gmfB = 0.f;
      const float* wA = &ws[urA * GW + h * MFH];
      const float* wB = &ws[urB * GW + h * MFH];
#pragma unroll
      for (int t4 = 0; t4 < MFH / 4; ++t4) {
        const float4 gv = *reinterpret_cast<const float4*>(grow + 4 * t4);
        const float4 xa = *reinterpret_cast<const float4*>(wA + 4 * t4);
        gmfA = fmaf(xa.x, gv.x, gmfA);
        gmfA = fmaf(xa.y, gv.y, gmfA);
        gmfA = fmaf(xa.z, gv.z, gmfA);
        gmfA = fmaf(xa.w, gv.w, gmfA);
        if (pair) {
          const float4 xb = *reinterpret_cast<const float4*>(wB + 4 * t4);
          gmfB = fmaf(xb.x, gv.x, gmfB);
          gmfB = fmaf(xb.y, gv.y, gmfB);
          gmfB = fmaf(xb.z, gv.z, gmfB);
          gmfB = fmaf(xb.w, gv.w, gmfB);
        }
      }
#pragma unroll
      for (int side = 0; side < (pair ? 2 : 1); ++side) {
        const int u = up + side;
        const int64_t b = side ? bB : bA;
        if (b >= B) break;
        const f32x16& acc = side ? accB : accA;
        float mlp = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float2 c = bw[mfma32_row(r, h)];
          mlp = fmaf(fmaxf(acc[r] + c.x, 0.f), c.y, mlp);
        }
        float tot = (side ? gmfB : gmfA) + mlp;
        tot += __shfl_xor(tot, 32);
        float score = tot + bpv;
        if (DENSE) {
          if (ivalid) dense[b * ldo + item] = score;
        } else {
          while (nm[u] < tile_end) {  // wave-uniform mask cursor
            if (item == nm[u]) score = -__builtin_inff();
            ++mpos[u];
            nm[u] = mpos[u] < mend[u] ? midx[mpos[u]] : INT_BIG;
          }
          L[u].offer(score, (int)item, ivalid, K);
        }
      }
    }

    if (t + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  if (!DENSE) {
#pragma unroll
    for (int u = 0; u < WU; ++u) {
      const int64_t b = ublk + wave * WU + u;
      if (b < B) L[u].store(cand_v + (b * NP + p) * K, cand_i + (b * NP + p) * K, K);
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
struct Partition {
  int np;
  int64_t ipp;
};

// Choose item partitions so the grid has ~2 workgroups per CU, each partition >= 4 tiles.
static Partition choose_partition(int64_t I, int64_t ublocks, int num_cus) {
  const int64_t want = std::max<int64_t>(1, hnm_cdiv(2 * (int64_t)num_cus, std::max<int64_t>(ublocks, 1)));
  const int64_t maxp = std::max<int64_t>(1, hnm_cdiv(I, 4 * TILE));
  int64_t np = std::min(want, maxp);
  int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), TILE) * TILE;
  np = hnm_cdiv(I, ipp);
  return {(int)np, ipp};
}

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

// ------------------------------------------------------------------ NCF host side
__global__ __launch_bounds__(256) void gather_scale_kernel(const float* __restrict__ tab,
                                                           int64_t rows, int ld, int d,
                                                           const int64_t* __restrict__ ids,
                                                           int64_t n, const float* __restrict__ s,
                                                           float* __restrict__ out, int ldo,
                                                           unsigned* err) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = ids[r];
  const bool ok = id >= 0 && id < rows;
  if (!ok && lane == 0) hnm_flag(err, HNM_ERR_OOB);
  for (int c = lane; c < ldo; c += 64)
    out[r * ldo + c] = (ok && c < d) ? tab[id * ld + c] * s[c] : 0.f;
}

// pairwise NeuralCF.forward: one thread per (user, item) pair
__global__ __launch_bounds__(256) void ncf_pair_kernel(hnm_ncf_weights w,
                                                       const int64_t* __restrict__ uids,
                                                       const int64_t* __restrict__ iids,
                                                       int64_t n, float* __restrict__ out,
                                                       unsigned* err) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int64_t u = uids[e], i = iids[e];
  if (u < 0 || u >= w.num_users || i < 0 || i >= w.num_items) {
    hnm_flag(err, HNM_ERR_OOB);
    out[e] = __builtin_nanf("");
    return;
  }
  float gm = 0.f;
  for (int k = 0; k < w.mf; ++k) gm = fmaf(w.wp[k], w.gmf_user[u * w.mf + k] * w.gmf_item[i * w.mf + k], gm);
  float x1[128];
  for (int o = 0; o < w.h1; ++o) {
    float acc = 0.f;
    for (int k = 0; k < w.h0; ++k) acc = fmaf(w.w1[o * 2 * w.h0 + k], w.mlp_user[u * w.h0 + k], acc);
    for (int k = 0; k < w.h0; ++k)
      acc = fmaf(w.w1[o * 2 * w.h0 + w.h0 + k], w.mlp_item[i * w.h0 + k], acc);
    x1[o] = fmaxf(acc + w.b1[o], 0.f);
  }
  float ml = 0.f;
  for (int o = 0; o < w.h2; ++o) {
    float acc = 0.f;
    for (int k = 0; k < w.h1; ++k) acc = fmaf(w.w2[o * w.h1 + k], x1[k], acc);
    ml = fmaf(w.wp[w.mf + o], fmaxf(acc + w.b2[o], 0.f), ml);
  }
  out[e] = gm + ml + w.bp[0];
}

static hnm_status ncf_check(const hnm_ncf_weights* w) {
  HNM_REQUIRE(w && w->gmf_user && w->gmf_item && w->mlp_user && w->mlp_item && w->w1 && w->b1 &&
                  w->w2 && w->b2 && w->wp && w->bp,
              HNM_EINVAL, "ncf: NULL weight pointer");
  HNM_REQUIRE(w->num_users > 0 && w->num_items > 0 && w->num_items < INT_BIG, HNM_EINVAL,
              "ncf: bad table sizes");
  HNM_REQUIRE(w->mf >= 1 && w->mf <= 128 && w->h0 >= 1 && w->h1 >= 1 && w->h1 <= 128 &&
                  w->h2 >= 1 && w->h2 <= 32,
              HNM_EUNSUPPORTED, "ncf: needs mf <= 128, h1 <= 128, h2 <= 32 (got %d, %d, %d)",
              w->mf, w->h1, w->h2);
  return HNM_OK;
}

template <int WU, int H1P, int MFH, bool DENSE>
static void launch_ncf(hnm_ctx* ctx, dim3 grid, const float* Pu, const float* WGu,
                       const float* Qi, const float* Gi, int64_t ldg, const hnm_ncf_weights* w,
                       int64_t B, int64_t ipp, const int64_t* mptr, const int32_t* midx, int K,
                       float* cv, int32_t* ci, int NP, float* dense, int64_t ldo) {
  hipLaunchKernelGGL((ncf_score_kernel<WU, H1P, MFH, DENSE>), grid, dim3(256), 0, ctx->stream,
                     Pu, WGu, Qi, Gi, ldg, w->w2, w->h1, w->h2, w->b2, w->wp + w->mf, w->bp, B,
                     w->num_items, ipp, mptr, midx, K, cv, ci, NP, dense, ldo);
}

template <bool DENSE>
static hnm_status ncf_common(hnm_ctx* ctx, const hnm_ncf_weights* w, const int64_t* ids,
                             int64_t B, const int64_t* mptr, const int32_t* midx, int K,
                             float* ov, int64_t* oi, float* dense, int64_t ldo) {
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ids, HNM_EINVAL, "ncf: NULL argument");
  if (B <= 0) return HNM_OK;
  const bool big = w->h1 > 64 || w->mf > 64;
  const int H1P = big ? 128 : 64, MFH = big ? 64 : 32, GW = 2 * MFH;
  const int64_t I = w->num_items;
  const int WU = B >= 256 ? 4 : 1;
  const int64_t ublocks = hnm_cdiv(B, 4 * WU);
  Partition part = choose_partition(I, ublocks, ctx->num_cus);
  // workspace: Pu [B,H1P], WGu [B,GW], Qi [I,H1P], G copy [I,GW] (if needed), candidates
  const bool gcopy = (w->mf != GW) || ((uintptr_t)w->gmf_item % 16 != 0);
  const size_t szP = hnm_align((size_t)B * H1P * 4), szW = hnm_align((size_t)B * GW * 4);
  const size_t szQ = hnm_align((size_t)I * H1P * 4), szG = gcopy ? hnm_align((size_t)I * GW * 4) : 0;
  const size_t ncand = DENSE ? 0 : (size_t)B * part.np * K;
  const size_t szC = hnm_align(ncand * 4);
  void* wsp;
  st = hnm_workspace(ctx, szP + szW + szQ + szG + 2 * szC, &wsp);
  if (st) return st;
  char* base = (char*)wsp;
  float* Pu = (float*)base; base += szP;
  float* WGu = (float*)base; base += szW;
  float* Qi = (float*)base; base += szQ;
  float* Gc = (float*)base; base += szG;
  float* cv = (float*)base; base += szC;
  int32_t* ci = (int32_t*)base;

  if (w->h1 < H1P) {
    HNM_HIP_CHECK(hipMemsetAsync(Pu, 0, szP, ctx->stream));
    HNM_HIP_CHECK(hipMemsetAsync(Qi, 0, szQ, ctx->stream));
  }
  // P_u = W1[:, :h0] m_u + b1 ; Q_i = W1[:, h0:] m_i  (pair-permuted, lane-half order)
  st = hnm_linear_rows_f32(ctx, w->mlp_user, w->h0, ids, w->num_users, B, w->h0, w->w1,
                           2 * w->h0, w->b1, w->h1, Pu, H1P, 1);
  if (st) return st;
  st = hnm_linear_rows_f32(ctx, w->mlp_item, w->h0, nullptr, I, I, w->h0, w->w1 + w->h0,
                           2 * w->h0, nullptr, w->h1, Qi, H1P, 1);
  if (st) return st;
  hipLaunchKernelGGL(gather_scale_kernel, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0,
                     ctx->stream, w->gmf_user, w->num_users, w->mf, w->mf, ids, B, w->wp, WGu,
                     GW, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  const float* G = w->gmf_item;
  int64_t ldg = w->mf;
  if (gcopy) {
    HNM_HIP_CHECK(hipMemsetAsync(Gc, 0, szG, ctx->stream));
    HNM_HIP_CHECK(hipMemcpy2DAsync(Gc, GW * 4, w->gmf_item, w->mf * 4, w->mf * 4, I,
                                   hipMemcpyDeviceToDevice, ctx->stream));
    G = Gc;
    ldg = GW;
  }

  dim3 grid((unsigned)ublocks, (unsigned)part.np);
#define HNM_NCF(WUV)                                                                          \
  if (big)                                                                                    \
    launch_ncf<WUV, 128, 64, DENSE>(ctx, grid, Pu, WGu, Qi, G, ldg, w, B, part.ipp, mptr,     \
                                    midx, K, cv, ci, part.np, dense, ldo);                    \
  else                                                                                        \
    launch_ncf<WUV, 64, 32, DENSE>(ctx, grid, Pu, WGu, Qi, G, ldg, w, B, part.ipp, mptr, midx, \
                                   K, cv, ci, part.np, dense, ldo);
  hnm_timer_begin(ctx);
  if (WU == 4) {
    HNM_NCF(4)
  } else {
    HNM_NCF(1)
  }
#undef HNM_NCF
  hnm_timer_end(ctx);
  HNM_LAUNCH_CHECK();
  if (!DENSE)
    return hnm_topk_merge_i32(ctx, cv, ci, B, 1, 0, (int64_t)part.np * K, part.np * K, K, ov, oi);
  return HNM_OK;
}

extern "C" hnm_status hnm_ncf_topk_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                       const int64_t* user_ids, int64_t B,
                                       const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                                       float* out_val, int64_t* out_idx) {
  HNM_REQUIRE(k >= 1 && k <= 64 && out_idx, HNM_EINVAL, "ncf_topk: fused path needs 1 <= k <= 64");
  return ncf_common<false>(ctx, w, user_ids, B, mask_ptr, mask_idx, k, out_val, out_idx,
                           nullptr, 0);
}

extern "C" hnm_status hnm_ncf_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                         const int64_t* user_ids, int64_t B, float* out,
                                         int64_t ldo) {
  HNM_REQUIRE(out && w && ldo >= w->num_items, HNM_EINVAL, "ncf_scores: bad output");
  return ncf_common<true>(ctx, w, user_ids, B, nullptr, nullptr, 1, nullptr, nullptr, out, ldo);
}

extern "C" hnm_status hnm_ncf_pair_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                              const int64_t* user_ids, const int64_t* item_ids,
                                              int64_t n, float* out) {
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && user_ids && item_ids && out, HNM_EINVAL, "ncf_pair: NULL argument");
  if (n <= 0) return HNM_OK;
  hipLaunchKernelGGL(ncf_pair_kernel, dim3((unsigned)hnm_cdiv(n, 256)), dim3(256), 0, ctx->stream,
                     *w, user_ids, item_ids, n, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
