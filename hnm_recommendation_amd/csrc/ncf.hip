// NeuralCF all-items scoring fused with filter + top-K on gfx950
// (neural_cf.py:143-208 predict_all_items, :300-326 recommend, :112-141 forward).
//
//   s(u, i) = wp_gmf . (g_u * g_i) + wp_mlp . relu(W2 relu(W1 [m_u; m_i] + b1) + b2) + bp
//
// Layer 1 is decomposed, W1 [m_u; m_i] + b1 = P_u + Q_i (per-user / per-item projections
// computed once per call by hnm_linear_rows_f32, stored in lane-half order).
//
// ncf32_kernel (h1 <= 64, mf <= 64: the reference config): a wave owns 32 users, a
// workgroup 128; the item partition streams through LDS in 32-item tiles.  Per tile:
//   * the GMF term of all 32 users is ONE 32-step MFMA chain  D_g = (wp_gmf*G_u) . G_i^T
//     (users x items), parked in LDS for the per-user epilogues;
//   * per user, layer 2 runs as a 32-step v_mfma_f32_32x32x2_f32 chain with W2 as the A
//     operand (registers, whole kernel), B = relu(P_u + Q_i) built in registers from the
//     tile's Q (registers) and P_u (LDS broadcast), and b2 as the chain's C input; two
//     users' chains are interleaved;
//   * epilogue: relu . wp_mlp over the 16 accumulator rows + one cross-half shuffle,
//     + GMF + bp; the (score desc, item asc) top-K of each user lives in LDS and is only
//     touched when a score beats the user's threshold (a per-lane register vector).
// Exact fp32 throughout (the f32 MFMA is an fp32 fma chain).
#include <algorithm>

#include "hnm_device.h"
#include "ncf_internal.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);

// ------------------------------------------------------------------ 32-user kernel
template <bool DENSE>
__global__ __launch_bounds__(256, 2) void ncf32_kernel(
    const float* __restrict__ Pu,   // [B, 64]  pair-permuted  W1u m_u + b1
    const float* __restrict__ WGu,  // [B, 64]  pair-permuted  wp_gmf * g_u
    const float* __restrict__ Qi,   // [I, 64]  pair-permuted  W1i m_i
    const float* __restrict__ Gi, int64_t ldg, int mf,  // [I, ldg] gmf item table
    const float* __restrict__ W2, int h1, int h2, const float* __restrict__ b2,
    const float* __restrict__ wm, const float* __restrict__ bp, int64_t B, int64_t I,
    int64_t ipp, const int64_t* __restrict__ mptr, const int32_t* __restrict__ midx, int K,
    float* __restrict__ cand_v, int32_t* __restrict__ cand_i, int NP,
    float* __restrict__ dense, int64_t ldo, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ nrows, int dyn_cus) {
  // rows != nullptr: batch row b is request row rows[b], b < *nrows (device-side list of
  // the rows the certified path queued); candidates stay at the compact index b.  dyn_cus > 0:
  // the item partitions follow *nrows (hnm_internal.h list_rows_np; grid.y is the maximum).
  constexpr int KS = 32;          // MFMA k-steps of layer 2 (h1 <= 64) and of GMF (mf <= 64)
  constexpr int RS = 68;          // LDS row stride (floats): conflict-free b128 reads
  constexpr int NU = 128;         // users per workgroup
  __shared__ __attribute__((aligned(16))) float qs[TILE * RS];
  __shared__ __attribute__((aligned(16))) float gs[TILE * RS];
  __shared__ __attribute__((aligned(16))) float ps[NU * 64];
  __shared__ __attribute__((aligned(16))) float gsm[4 * 32 * 32];
  extern __shared__ __attribute__((aligned(16))) float lists[];  // [4][32][K] v, then i

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  int64_t ublk = (int64_t)blockIdx.x * NU;
  int p = blockIdx.y;
  if (rows) B = *nrows;
  if (rows && dyn_cus > 0) {  // flat grid: (user block, partition) from *nrows (list_rows_grid)
    const int64_t nb = hnm_cdiv(B, NU);
    const Partition dp = choose_partition(I, nb, dyn_cus);
    NP = dp.np;
    ipp = dp.ipp;
    const int64_t w = blockIdx.x;
    if (w >= nb * NP) return;  // whole workgroup: before any barrier
    ublk = w / NP * NU;
    p = (int)(w % NP);
  }
  if (ublk >= B || p >= NP) return;  // whole workgroup: before any barrier
  auto R = [&](int64_t b) -> int64_t { return rows ? (int64_t)rows[b] : b; };
  const int64_t u0 = ublk + wave * 32;  // first user of this wave
  const int nu = (int)std::max<int64_t>(0, std::min<int64_t>(32, B - u0));
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + ipp);
  float* lv_s = lists + wave * 32 * K;
  int* li_s = reinterpret_cast<int*>(lists + 4 * 32 * K) + wave * 32 * K;

  for (int e = tid; e < NU * 16; e += 256) {
    const int r = e >> 4, c = e & 15;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ublk + r < B) v = *reinterpret_cast<const float4*>(Pu + R(ublk + r) * 64 + 4 * c);
    *reinterpret_cast<float4*>(&ps[r * 64 + 4 * c]) = v;
  }
  // A operands: W2 rows (hidden unit j), and this wave's users' wp_gmf*g_u rows
  float a[KS], ag[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + h;
    a[s] = (j < h2 && k < h1) ? W2[j * h1 + k] : 0.f;
  }
  {
    const bool ok = j < nu;
    const float* row = WGu + (ok ? R(u0 + j) : 0) * 64 + h * KS;
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
      float4 v = ok ? *reinterpret_cast<const float4*>(row + 4 * s4) : make_float4(0.f, 0.f, 0.f, 0.f);
      ag[4 * s4] = v.x; ag[4 * s4 + 1] = v.y; ag[4 * s4 + 2] = v.z; ag[4 * s4 + 3] = v.w;
    }
  }
  f32x16 b2acc;
  float wmr[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = mfma32_row(r, h);
    b2acc[r] = i < h2 ? b2[i] : 0.f;
    wmr[r] = i < h2 ? wm[i] : 0.f;
  }
  const float bpv = bp[0];
  // top-K state: lists in LDS, thresholds in lane u of (tvv, tvi)
  float tvv = -__builtin_inff();
  int tvi = HNM_SENTINEL_IDX;
  if (!DENSE)
    for (int e = lane; e < 32 * K; e += 64) { lv_s[e] = -__builtin_inff(); li_s[e] = HNM_SENTINEL_IDX; }
  // mask cursors: lane u < 32 follows user u0 + u
  int nm = INT_BIG, mpos = 0, mend = 0;
  const bool masked = !DENSE && mptr != nullptr;
  if (masked && lane < nu) {
    const int64_t ur = R(u0 + lane);
    const int64_t lo = mptr[ur], hi = mptr[ur + 1];
    mpos = (int)mask_lower_bound(midx, lo, hi, (int)part_start);
    mend = (int)hi;
    nm = mpos < mend ? midx[mpos] : INT_BIG;
  }

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, TILE) : 0;
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t base = part_start + t * TILE;
    __syncthreads();  // every wave is done with the previous tile
    // stage Q (already pair-permuted) and G (pair-permuted here) for items base..base+31
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f = tid + 256 * q;
      const int row = f >> 4, c = f & 15;
      const int64_t item = base + row;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (item < part_end) v = *reinterpret_cast<const float4*>(Qi + item * 64 + 4 * c);
      *reinterpret_cast<float4*>(&qs[row * RS + 4 * c]) = v;
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      if (item < part_end && 4 * c < mf) g = *reinterpret_cast<const float4*>(Gi + item * ldg + 4 * c);
      *reinterpret_cast<float2*>(&gs[row * RS + 2 * c]) = make_float2(g.x, g.z);
      *reinterpret_cast<float2*>(&gs[row * RS + KS + 2 * c]) = make_float2(g.y, g.w);
    }
    __syncthreads();
    if (nu == 0) continue;

    // GMF of the wave's 32 users x 32 items: one MFMA chain, parked in LDS
    {
      f32x16 gacc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const float* grow = &gs[j * RS + h * KS];
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 gv = *reinterpret_cast<const float4*>(grow + 4 * s4);
        gacc = mfma32x32x2(ag[4 * s4 + 0], gv.x, gacc);
        gacc = mfma32x32x2(ag[4 * s4 + 1], gv.y, gacc);
        gacc = mfma32x32x2(ag[4 * s4 + 2], gv.z, gacc);
        gacc = mfma32x32x2(ag[4 * s4 + 3], gv.w, gacc);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) gsm[(wave * 32 + mfma32_row(r, h)) * 32 + j] = gacc[r];
    }
    float q[KS];
    {
      const float* qrow = &qs[j * RS + h * KS];
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 v = *reinterpret_cast<const float4*>(qrow + 4 * s4);
        q[4 * s4] = v.x; q[4 * s4 + 1] = v.y; q[4 * s4 + 2] = v.z; q[4 * s4 + 3] = v.w;
      }
    }
    const int64_t item = base + j;
    const bool ivalid = lane < 32 && item < part_end;
    const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);
    // per-user 32-bit masks of filtered items in this tile (rare path)
    unsigned mbits = 0;
    if (masked) {
      uint64_t pend = __ballot(lane < 32 && nm < tile_end) & 0xffffffffull;
      while (pend) {
        const int u = __builtin_ctzll(pend);
        pend &= pend - 1;
        while (true) {
          const int tgt = hnm_readlane_i(nm, u);
          if (tgt >= tile_end) break;
          if (lane == u) {
            mbits |= 1u << (tgt - (int)base);
            ++mpos;
            nm = mpos < mend ? midx[mpos] : INT_BIG;
          }
        }
      }
    }

    for (int up = 0; up < nu; up += 2) {
      const int uA = up, uB = up + 1 < nu ? up + 1 : up;
      // GMF values of both users, read before the MFMA block so the LDS latency hides
      const float gmA = gsm[(wave * 32 + uA) * 32 + j];
      const float gmB = gsm[(wave * 32 + uB) * 32 + j];
      const float* prA = &ps[(wave * 32 + uA) * 64 + h * KS];
      const float* prB = &ps[(wave * 32 + uB) * 64 + h * KS];
      f32x16 accA = b2acc, accB = b2acc;
      float4 pa = *reinterpret_cast<const float4*>(prA);
      float4 pb = *reinterpret_cast<const float4*>(prB);
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        float4 na = pa, nb = pb;
        if (s4 + 1 < KS / 4) {
          na = *reinterpret_cast<const float4*>(prA + 4 * (s4 + 1));
          nb = *reinterpret_cast<const float4*>(prB + 4 * (s4 + 1));
        }
        accA = mfma32x32x2(a[4 * s4 + 0], fmaxf(pa.x + q[4 * s4 + 0], 0.f), accA);
        accB = mfma32x32x2(a[4 * s4 + 0], fmaxf(pb.x + q[4 * s4 + 0], 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 1], fmaxf(pa.y + q[4 * s4 + 1], 0.f), accA);
        accB = mfma32x32x2(a[4 * s4 + 1], fmaxf(pb.y + q[4 * s4 + 1], 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 2], fmaxf(pa.z + q[4 * s4 + 2], 0.f), accA);
        accB = mfma32x32x2(a[4 * s4 + 2], fmaxf(pb.z + q[4 * s4 + 2], 0.f), accB);
        accA = mfma32x32x2(a[4 * s4 + 3], fmaxf(pa.w + q[4 * s4 + 3], 0.f), accA);
        accB = mfma32x32x2(a[4 * s4 + 3], fmaxf(pb.w + q[4 * s4 + 3], 0.f), accB);
        pa = na;
        pb = nb;
      }
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int u = side ? uB : uA;
        if (side && uB == uA) break;
        const f32x16& acc = side ? accB : accA;
        float m4[4] = {0.f, 0.f, 0.f, 0.f};  // 4 short chains instead of one 16-deep
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaf(fmaxf(acc[r], 0.f), wmr[r], m4[r & 3]);
        const float mlp = (m4[0] + m4[1]) + (m4[2] + m4[3]);
        const float gm = side ? gmB : gmA;
        const float tot = hnm_sum_halves(mlp + (h == 0 ? gm : 0.f));
        float score = tot + bpv;
        if (masked) {
          const unsigned bits = (unsigned)hnm_readlane_i((int)mbits, u);
          if ((bits >> j) & 1u) score = -__builtin_inff();
        }
        if (DENSE) {
          if (ivalid) dense[(u0 + u) * ldo + item] = score;
        } else {
          const float thv = hnm_readlane_f(tvv, u);
          const int thi = hnm_readlane_i(tvi, u);
          uint64_t m = __ballot(ivalid && (score > thv || (score == thv && (int)item < thi)));
          if (m) {
            float lv = lane < K ? lv_s[u * K + lane] : -__builtin_inff();
            int li = lane < K ? li_s[u * K + lane] : HNM_SENTINEL_IDX;
            while (m) {
              const int l = __builtin_ctzll(m);
              m &= m - 1;
              list1_insert(lv, li, hnm_readlane_f(score, l), (int)base + l, K);
            }
            if (lane < K) { lv_s[u * K + lane] = lv; li_s[u * K + lane] = li; }
            const float nv = hnm_readlane_f(lv, K - 1);
            const int ni = hnm_readlane_i(li, K - 1);
            if (lane == u) { tvv = nv; tvi = ni; }
          }
        }
      }
    }
  }
  if (!DENSE) {
    for (int e = lane; e < nu * K; e += 64) {
      const int u = e / K, s = e % K;
      const int64_t o = ((u0 + u) * NP + p) * K + s;
      cand_v[o] = lv_s[e];
      cand_i[o] = li_s[e] == HNM_SENTINEL_IDX ? -1 : li_s[e];
    }
  }
}

// ------------------------------------------------------------------ generic NCF kernel
// Any hidden/GMF width up to 128 (WU users per wave, two interleaved MFMA chains).
template <int WU, int H1P, int MFH, bool DENSE>
__global__ __launch_bounds__(256, 2) void ncf_generic_kernel(
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

// ------------------------------------------------------------------ host side
__global__ __launch_bounds__(256) void gather_scale_kernel(const float* __restrict__ tab,
                                                           int64_t rows, int ld, int d,
                                                           const int64_t* __restrict__ ids,
                                                           int64_t n, const float* __restrict__ s,
                                                           float* __restrict__ out, int ldo,
                                                           unsigned* err, int permute) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = ids[r];
  const bool ok = id >= 0 && id < rows;
  if (!ok && lane == 0) hnm_flag(err, HNM_ERR_OOB);
  for (int c = lane; c < ldo; c += 64) {
    const int o = permute ? (c & 1) * (ldo / 2) + (c >> 1) : c;
    out[r * ldo + o] = (ok && c < d) ? tab[id * ld + c] * s[c] : 0.f;
  }
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
  // item_proj is read with 16-B loads as the Qi table (a caller that filled the
  // struct field by field without zeroing it passes garbage here -- refused when misaligned)
  HNM_REQUIRE((uintptr_t)w->item_proj % 16 == 0, HNM_EINVAL,
              "ncf: item_proj must be NULL or 16-B aligned (zero the hnm_ncf_weights struct)");
  return HNM_OK;
}

template <bool DENSE>
static void launch_ncf32(hnm_ctx* ctx, dim3 grid, const NcfTabs& t, const hnm_ncf_weights* w,
                         int64_t B, int64_t ipp, const int64_t* mptr, const int32_t* midx, int K,
                         float* cv, int32_t* ci, int NP, float* dense, int64_t ldo,
                         const int32_t* rows = nullptr, const int32_t* nrows = nullptr,
                         int dyn_cus = 0) {
  const size_t lds = DENSE ? 0 : (size_t)4 * 32 * K * 8;
  hipLaunchKernelGGL((ncf32_kernel<DENSE>), grid, dim3(256), lds, ctx->stream, t.Pu, t.WGu, t.Qi,
                     t.G, t.ldg, w->mf, w->w2, w->h1, w->h2, w->b2, w->wp + w->mf, w->bp, B,
                     w->num_items, ipp, mptr, midx, K, cv, ci, NP, dense, ldo, rows, nrows,
                     dyn_cus);
}

template <int WU, int H1P, int MFH, bool DENSE>
static void launch_ncf(hnm_ctx* ctx, dim3 grid, const NcfTabs& t, const hnm_ncf_weights* w,
                       int64_t B, int64_t ipp, const int64_t* mptr, const int32_t* midx, int K,
                       float* cv, int32_t* ci, int NP, float* dense, int64_t ldo) {
  hipLaunchKernelGGL((ncf_generic_kernel<WU, H1P, MFH, DENSE>), grid, dim3(256), 0, ctx->stream,
                     t.Pu, t.WGu, t.Qi, t.G, t.ldg, w->w2, w->h1, w->h2, w->b2, w->wp + w->mf,
                     w->bp, B, w->num_items, ipp, mptr, midx, K, cv, ci, NP, dense, ldo);
}

size_t ncf_list_bytes(int64_t B, int64_t I, int K, int num_cus) {
  const Partition part = choose_partition(I, hnm_cdiv(B, 128), num_cus);
  const int64_t slots = std::max<int64_t>(B * part.np, list_rows_slots(B, I, num_cus));
  return hnm_align((size_t)slots * K * 4);
}

hnm_status ncf_list_rows(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                         const int64_t* mptr, const int32_t* midx, int K, const int32_t* rows,
                         const int32_t* nrows, float* cv, int32_t* ci, float* ov, int64_t* oi) {
  // the queued rows are known only on the device: the widest grid, the partitions used
  // derived from *nrows in the kernel and the merge (hnm_internal.h list_rows_np)
  const int64_t grid = list_rows_grid(B, w->num_items, ctx->num_cus);
  launch_ncf32<false>(ctx, dim3((unsigned)grid, 1), t, w, B, 0, mptr, midx, K, cv, ci, 1, nullptr,
                      0, rows, nrows, ctx->num_cus);
  HNM_LAUNCH_CHECK();
  return hnm_topk_merge_rows(ctx, cv, ci, B, 1, 0, K, K, K, ov, oi, rows, nrows, w->num_items,
                             ctx->num_cus);
}

// Per-call tables: P_u, wp*g_u (users), Q_i (items), the GMF item table (padded copy when
// needed), then `extra` bytes of scratch for the caller.
struct NcfCall {
  NcfTabs t;
  bool big;
  void* extra;
};

// fill = false: only re-derive the pointers into the workspace the begin phase of a
// two-phase call filled (hnm_ncf_topk_finish_f32).
static hnm_status ncf_tables(hnm_ctx* ctx, const hnm_ncf_weights* w, const int64_t* ids,
                             int64_t B, size_t extra, NcfCall* out, bool fill = true) {
  const bool big = w->h1 > 64 || w->mf > 64;  // generic kernel; else the 32-user kernels
  const int H1P = big ? 128 : 64, GW = big ? 128 : 64;
  const int64_t I = w->num_items;
  const bool gcopy = (big ? w->mf != GW : w->mf % 4 != 0) || ((uintptr_t)w->gmf_item % 16 != 0);
  const bool qcache = w->item_proj != nullptr;  // the caller's item projection (fixed tables)
  const size_t szP = hnm_align((size_t)B * H1P * 4), szW = hnm_align((size_t)B * GW * 4);
  const size_t szQ = qcache ? 0 : hnm_align((size_t)I * H1P * 4);
  const size_t szG = gcopy ? hnm_align((size_t)I * GW * 4) : 0;
  void* wsp = ctx->ws;
  hnm_status st = HNM_OK;
  if (fill) {
    st = hnm_workspace(ctx, szP + szW + szQ + szG + extra, &wsp);
    if (st) return st;
  } else {
    HNM_REQUIRE(ctx->ws && ctx->ws_size >= szP + szW + szQ + szG + extra, HNM_EINVAL,
                "ncf: the begin phase's workspace is gone");
  }
  char* base = (char*)wsp;
  float* Pu = (float*)base; base += szP;
  float* WGu = (float*)base; base += szW;
  float* Qi = (float*)base; base += szQ;
  float* Gc = (float*)base; base += szG;
  out->extra = base;
  out->big = big;
  const float* G = w->gmf_item;
  int64_t ldg = w->mf;
  if (gcopy) {
    G = Gc;
    ldg = GW;
  }
  out->t = {Pu, WGu, qcache ? w->item_proj : Qi, G, ldg};
  if (!fill) return HNM_OK;
  if (w->h1 < H1P) {
    HNM_HIP_CHECK(hipMemsetAsync(Pu, 0, szP, ctx->stream));
    if (!qcache) HNM_HIP_CHECK(hipMemsetAsync(Qi, 0, szQ, ctx->stream));
  }
  // P_u = W1[:, :h0] m_u + b1 ; Q_i = W1[:, h0:] m_i  (pair-permuted, lane-half order)
  st = hnm_linear_rows_f32(ctx, w->mlp_user, w->h0, ids, w->num_users, B, w->h0, w->w1,
                           2 * w->h0, w->b1, w->h1, Pu, H1P, 1);
  if (st) return st;
  if (!qcache) {
    st = hnm_linear_rows_f32(ctx, w->mlp_item, w->h0, nullptr, I, I, w->h0, w->w1 + w->h0,
                             2 * w->h0, nullptr, w->h1, Qi, H1P, 1);
    if (st) return st;
  }
  hipLaunchKernelGGL(gather_scale_kernel, dim3((unsigned)hnm_cdiv(B, 4)), dim3(256), 0,
                     ctx->stream, w->gmf_user, w->num_users, w->mf, w->mf, ids, B, w->wp, WGu,
                     GW, ctx->err_dev, big ? 0 : 1);
  HNM_LAUNCH_CHECK();
  if (gcopy) {
    HNM_HIP_CHECK(hipMemsetAsync(Gc, 0, szG, ctx->stream));
    HNM_HIP_CHECK(hipMemcpy2DAsync(Gc, GW * 4, w->gmf_item, w->mf * 4, w->mf * 4, I,
                                   hipMemcpyDeviceToDevice, ctx->stream));
  }
  return HNM_OK;
}

template <bool DENSE>
static hnm_status ncf_common(hnm_ctx* ctx, const hnm_ncf_weights* w, const int64_t* ids,
                             int64_t B, const int64_t* mptr, const int32_t* midx, int K,
                             float* ov, int64_t* oi, float* dense, int64_t ldo) {
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && (ids || B == 0), HNM_EINVAL, "ncf: NULL argument");
  if (B <= 0) return HNM_OK;
  const int64_t I = w->num_items;
  const bool big = w->h1 > 64 || w->mf > 64;
  // below ~16 rows the certified path's fixed launches cost more than the exact scan saves
  // (serve path, B = 1: exact 0.38 ms vs certified 0.44 ms per request, profiles/r2b_*)
  const bool cert = !DENSE && !big && ctx->prefilter && B >= 16 && ncf_cert_eligible(w, K);
  const int WU = B >= 256 ? 4 : 1;
  const int64_t ublocks = big ? hnm_cdiv(B, 4 * WU) : hnm_cdiv(B, 128);
  const Partition part = choose_partition(I, ublocks, ctx->num_cus);
  const size_t szC = DENSE ? 0 : hnm_align((size_t)B * part.np * K * 4);
  const bool strided = ctx->strided != 0;
  const size_t extra =
      cert ? ncf_cert_bytes(B, I, K, ctx->num_cus, ncf_cert_wg(ctx), strided) : 2 * szC;
  NcfCall c;
  st = ncf_tables(ctx, w, ids, B, extra, &c);
  if (st) return st;
  if (cert) return ncf_cert_topk(ctx, w, c.t, B, mptr, midx, K, c.extra, strided, ov, oi);
  float* cv = (float*)c.extra;
  int32_t* ci = (int32_t*)((char*)c.extra + szC);

  dim3 grid((unsigned)ublocks, (unsigned)part.np);
#define HNM_NCF(WUV)                                                                          \
  if (big)                                                                                    \
    launch_ncf<WUV, 128, 64, DENSE>(ctx, grid, c.t, w, B, part.ipp, mptr, midx, K, cv, ci,    \
                                    part.np, dense, ldo);                                     \
  else                                                                                        \
    launch_ncf<WUV, 64, 32, DENSE>(ctx, grid, c.t, w, B, part.ipp, mptr, midx, K, cv, ci,     \
                                   part.np, dense, ldo);
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
  if (!big) {
    launch_ncf32<DENSE>(ctx, grid, c.t, w, B, part.ipp, mptr, midx, K, cv, ci, part.np, dense,
                        ldo);
  } else if (WU == 4) {
    HNM_NCF(4)
  } else {
    HNM_NCF(1)
  }
#undef HNM_NCF
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  if (!DENSE)
    return hnm_topk_merge_i32(ctx, cv, ci, B, 1, 0, (int64_t)part.np * K, part.np * K, K, ov, oi);
  return HNM_OK;
}

extern "C" hnm_status hnm_ncf_topk_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                       const int64_t* user_ids, int64_t B,
                                       const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                                       float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(k >= 1 && k <= 64 && (out_idx || B == 0), HNM_EINVAL, "ncf_topk: fused path needs 1 <= k <= 64");
  // very large batches in chunks of rows: the certified path's per-row scratch (samples,
  // candidate segments) stays bounded; the mask CSR holds absolute offsets, so a chunk reads
  // its rows' slice of mask_ptr as is
  constexpr int64_t CHUNK = 32768;
  for (int64_t b0 = 0; b0 < B || b0 == 0; b0 += CHUNK) {
    const int64_t nb = std::min<int64_t>(CHUNK, B - b0);
    hnm_status st = ncf_common<false>(ctx, w, user_ids ? user_ids + b0 : nullptr, nb,
                                      mask_ptr ? mask_ptr + b0 : nullptr, mask_idx, k,
                                      out_val ? out_val + b0 * k : nullptr,
                                      out_idx ? out_idx + b0 * k : nullptr, nullptr, 0);
    if (st || B <= 0) return st;
  }
  return HNM_OK;
}

// Two-phase fused top-K for item-sharded serving (sharding.py): begin computes the per-call
// tables and each row's certified lower bound of its exact K-th best score over this
// call's items (real units, -inf when unknown); the caller may replace the bounds by any
// valid lower bounds -- the max over the item shards of a node (one all-reduce) -- and
// finish scans with them.  Rows may then keep fewer than K entries (short_ok), padded with
// (-inf, -1); the merge across shards completes them.  Exact mode (pre-filter off or not
// eligible): begin writes -inf, finish runs the exact fused scan.
static hnm_status ncf_topk_begin(hnm_ctx* ctx, const hnm_ncf_weights* w, const int64_t* user_ids,
                                 int64_t B, const int64_t* mask_ptr, const int32_t* mask_idx,
                                 int k, float* lower_bound, float* lists) {
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ((user_ids && (lower_bound || lists)) || B == 0) && k >= 1 && k <= 64,
              HNM_EINVAL, "ncf_topk_begin: bad argument");
  HNM_REQUIRE(!ctx->pend.kind, HNM_EINVAL, "ncf_topk_begin: a two-phase call is already open");
  if (B <= 0) return HNM_OK;
  const bool big = w->h1 > 64 || w->mf > 64;
  const bool cert = !big && ctx->prefilter && ncf_cert_eligible(w, k);
  // the scratch layout (with / without the strided sample's) is the begin's, kept for finish
  const bool strided = ctx->strided != 0;
  if (cert) {
    NcfCall c;
    st = ncf_tables(ctx, w, user_ids, B,
                    ncf_cert_bytes(B, w->num_items, k, ctx->num_cus, ncf_cert_wg(ctx), strided),
                    &c);
    if (st) return st;
    st = ncf_cert_begin(ctx, w, c.t, B, mask_ptr, mask_idx, k, c.extra, strided, lower_bound,
                        lists);
    if (st) return st;
  } else {
    if (lower_bound && (st = hnm_fill_f32(ctx, lower_bound, B, -__builtin_inff()))) return st;
    if (lists && (st = hnm_fill_f32(ctx, lists, B * k, -__builtin_inff()))) return st;
  }
  ctx->pend = {cert ? HNM_PEND_NCF_CERT : HNM_PEND_NCF_EXACT, B, w->num_items, k, user_ids,
               w->mlp_item, strided ? HNM_PEND_STRIDED : 0};
  return HNM_OK;
}

extern "C" hnm_status hnm_ncf_topk_begin_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                             const int64_t* user_ids, int64_t B,
                                             const int64_t* mask_ptr, const int32_t* mask_idx,
                                             int k, float* lower_bound) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(lower_bound || B == 0, HNM_EINVAL, "ncf_topk_begin: lower_bound is NULL");
  return ncf_topk_begin(ctx, w, user_ids, B, mask_ptr, mask_idx, k, lower_bound, nullptr);
}

extern "C" hnm_status hnm_ncf_topk_begin_lists_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                                   const int64_t* user_ids, int64_t B,
                                                   const int64_t* mask_ptr,
                                                   const int32_t* mask_idx, int k,
                                                   float* lower_lists) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(lower_lists || B == 0, HNM_EINVAL, "ncf_topk_begin_lists: lower_lists is NULL");
  return ncf_topk_begin(ctx, w, user_ids, B, mask_ptr, mask_idx, k, nullptr, lower_lists);
}

extern "C" hnm_status hnm_ncf_topk_finish_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                              const int64_t* user_ids, int64_t B,
                                              const int64_t* mask_ptr, const int32_t* mask_idx,
                                              int k, const float* lower_bound, int short_ok,
                                              float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && w && (out_idx || B == 0), HNM_EINVAL, "ncf_topk_finish: bad argument");
  if (B <= 0) return HNM_OK;
  const int kind = ctx->pend.kind;
  HNM_REQUIRE((kind == HNM_PEND_NCF_CERT || kind == HNM_PEND_NCF_EXACT) && ctx->pend.B == B &&
                  ctx->pend.K == k && ctx->pend.I == w->num_items && ctx->pend.ids == user_ids &&
                  ctx->pend.items == w->mlp_item,
              HNM_EINVAL, "ncf_topk_finish: no matching hnm_ncf_topk_begin_f32 on this ctx");
  ctx->pend.kind = 0;
  if (kind == HNM_PEND_NCF_EXACT)
    return ncf_common<false>(ctx, w, user_ids, B, mask_ptr, mask_idx, k, out_val, out_idx,
                             nullptr, 0);
  HNM_REQUIRE(lower_bound, HNM_EINVAL, "ncf_topk_finish: lower_bound is NULL");
  const bool strided = (ctx->pend.flags & HNM_PEND_STRIDED) != 0;  // the begin's layout
  NcfCall c;
  hnm_status st = ncf_tables(
      ctx, w, user_ids, B,
      ncf_cert_bytes(B, w->num_items, k, ctx->num_cus, ncf_cert_wg(ctx), strided), &c, false);
  if (st) return st;
  return ncf_cert_finish(ctx, w, c.t, B, mask_ptr, mask_idx, k, c.extra, strided, lower_bound,
                         short_ok, out_val, out_idx);
}

extern "C" hnm_status hnm_ncf_item_proj_f32(hnm_ctx* ctx, const hnm_ncf_weights* w, float* out) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && out, HNM_EINVAL, "ncf_item_proj: NULL argument");
  const int H1P = (w->h1 > 64 || w->mf > 64) ? 128 : 64;  // ncf_tables' layout
  const int64_t I = w->num_items;
  if (w->h1 < H1P) HNM_HIP_CHECK(hipMemsetAsync(out, 0, (size_t)I * H1P * 4, ctx->stream));
  return hnm_linear_rows_f32(ctx, w->mlp_item, w->h0, nullptr, I, I, w->h0, w->w1 + w->h0,
                             2 * w->h0, nullptr, w->h1, out, H1P, 1);
}

extern "C" hnm_status hnm_ncf_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                         const int64_t* user_ids, int64_t B, float* out,
                                         int64_t ldo) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE((out || B == 0) && w && ldo >= w->num_items, HNM_EINVAL, "ncf_scores: bad output");
  return ncf_common<true>(ctx, w, user_ids, B, nullptr, nullptr, 1, nullptr, nullptr, out, ldo);
}

extern "C" hnm_status hnm_ncf_prefilter_debug_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                                  const int64_t* user_ids, int64_t B,
                                                  float* approx, int64_t lda, float* bound) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && user_ids && approx && bound && lda >= w->num_items, HNM_EINVAL,
              "ncf_prefilter_debug: bad argument");
  HNM_REQUIRE(w->h1 <= 64 && w->mf <= 64 && w->num_items * 64 < ((int64_t)1 << 31),
              HNM_EUNSUPPORTED,
              "ncf_prefilter_debug: the f16 pre-filter covers h1 <= 64, mf <= 64, < 2^25 items");
  if (B <= 0) return HNM_OK;
  NcfCall c;
  st = ncf_tables(ctx, w, user_ids, B,
                  ncf_cert_bytes(B, w->num_items, 1, ctx->num_cus, ncf_cert_wg(ctx), false), &c);
  if (st) return st;
  return ncf_cert_debug(ctx, w, c.t, B, c.extra, approx, lda, bound);
}

// ------------------------------------------------------------------ deep towers, certified
// A deep tower [2 h0, h1, h2, h3] seen as the two-layer tower's tables (layers 1 and 2) plus its
// third layer (CertDeep): the certified f16 scan with the layer-3 epilogue and the exact deep
// re-scoring (ncf_cert.hip).
static void deep_view(const hnm_ncf_deep_weights* dw, const int64_t* ids, hnm_ncf_weights* w,
                      CertDeep* dp) {
  *w = hnm_ncf_weights{};
  w->gmf_user = dw->gmf_user;
  w->gmf_item = dw->gmf_item;
  w->mlp_user = dw->mlp_user;
  w->mlp_item = dw->mlp_item;
  w->w1 = dw->w[0];
  w->b1 = dw->b[0];
  w->w2 = dw->w[1];
  w->b2 = dw->b[1];
  w->wp = dw->wp;  // [mf + h3]: only its GMF part is read through this view
  w->bp = dw->bp;
  w->num_users = dw->num_users;
  w->num_items = dw->num_items;
  w->mf = dw->mf;
  w->h0 = dw->dims[0] / 2;
  w->h1 = dw->dims[1];
  w->h2 = dw->dims[2];
  *dp = CertDeep{dw->w[2], dw->b[2], dw->wp + dw->mf, dw->dims[3], dw->gmf_user, dw->gmf_item,
                 dw->wp, ids};
}

bool ncf_deep_cert_eligible(const hnm_ncf_deep_weights* dw, int K) {
  if (dw->nl != 3 || dw->dims[1] > 64 || dw->dims[2] > 32 || dw->dims[3] > 16 || dw->mf > 64 ||
      dw->mf % 4 != 0 || (uintptr_t)dw->gmf_item % 16 != 0)
    return false;
  hnm_ncf_weights w;
  CertDeep dp;
  deep_view(dw, nullptr, &w, &dp);
  return ncf_cert_eligible(&w, K);
}

hnm_status ncf_deep_cert(hnm_ctx* ctx, const hnm_ncf_deep_weights* dw, const int64_t* ids,
                         int64_t B, const int64_t* mptr, const int32_t* midx, int K, float* ov,
                         int64_t* oi, int32_t** ovf_rows, int32_t** ovf_cnt, bool* pruned) {
  hnm_ncf_weights w;
  CertDeep dp;
  deep_view(dw, ids, &w, &dp);
  NcfCall c;
  hnm_status st = ncf_tables(
      ctx, &w, ids, B, ncf_cert_bytes(B, w.num_items, K, ctx->num_cus, ncf_cert_wg(ctx), false), &c);
  if (st) return st;
  return ncf_deep_cert_topk(ctx, &w, dp, c.t, B, mptr, midx, K, c.extra, ov, oi, ovf_rows, ovf_cnt,
                            pruned);
}

hnm_status ncf_deep_cert_debug(hnm_ctx* ctx, const hnm_ncf_deep_weights* dw, const int64_t* ids,
                               int64_t B, float* approx, int64_t lda, float* bound) {
  hnm_ncf_weights w;
  CertDeep dp;
  deep_view(dw, ids, &w, &dp);
  NcfCall c;
  hnm_status st = ncf_tables(
      ctx, &w, ids, B, ncf_cert_bytes(B, w.num_items, 1, ctx->num_cus, ncf_cert_wg(ctx), false), &c);
  if (st) return st;
  return ncf_cert_debug(ctx, &w, c.t, B, c.extra, approx, lda, bound, &dp);
}

extern "C" hnm_status hnm_ncf_pair_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                              const int64_t* user_ids, const int64_t* item_ids,
                                              int64_t n, float* out) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = ncf_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ((user_ids && item_ids && out) || n == 0), HNM_EINVAL, "ncf_pair: NULL argument");
  if (n <= 0) return HNM_OK;
  hipLaunchKernelGGL(ncf_pair_kernel, dim3((unsigned)hnm_cdiv(n, 256)), dim3(256), 0, ctx->stream,
                     *w, user_ids, item_ids, n, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
