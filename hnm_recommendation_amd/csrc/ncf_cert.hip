// NeuralCF top-K with a CERTIFIED f16 pre-filter and exact fp32 re-scoring
// (neural_cf.py:300-326 recommend over :143-208 predict_all_items).
//
// The fp32 MFMA rate is 1/16 of the f16 rate on gfx950, and the NCF pair MLP is MFMA-bound.
// So the all-items scan runs in f16 (v_mfma_f32_32x32x16_f16, fp32 accumulate) and only
// PRUNES; every returned score is recomputed in exact fp32 by the same arithmetic as the
// fp32 kernel (ncf32_kernel), so outputs are bit-identical to the fp32 path.  Pruning is
// safe because of a rigorous per-user error bound E_u:
//
//   |approx(u, i) - (exact(u, i) - bp)| <= E_u   for every item i            (*)
//
// Let T = the K-th best exact score of user u (bp excluded) and e(u, i) the bound of (*) for
// pair (u, i).  A strided item sample scored by the f16 kernel gives L_u = K-th best of
// (approx - e) over the sample <= T.  Every item of the exact top-K has approx + e >= exact
// >= T >= L_u, so the main f16 pass appends every item with approx + e(u, i) >= L_u, and
// the exact top-K of the appended candidates IS the exact top-K.  Rows whose candidate
// segments overflow (or whose bound is not usable) are recomputed by the exact fp32 kernel
// over all items (on-device fallback).  No atomics in the scan: a wave owns its 32 users
// within its item partition, so per-(user, partition) counters live in registers.
//
// Bound (*).  Let z_k = |P_k| + |Q_k| (the fp32 layer-1 values both paths read), v_k =
// sum_j |wm_j||W2_jk|, A_u = sum_k v_k |P_uk|, B_i = sum_k v_k |Q_ik|, c0 = sum_j |wm_j b2_j|,
// C_u = ||wp_gmf * g_u||_2, D_i = ||g_i||_2.  With f16 unit roundoff u = 2^-11, RNE
// conversions (denormals kept: tools/mfma_semantics_probe.hip) and products exact in the
// fp32 accumulator: the layer-1 sum and its operands contribute <= 2.01u z_k, W2 rounding
// u|W2|, so |dH_j| <= 3.02u sum_k |W2_jk| z_k; relu is 1-Lipschitz; rounding relu(H) and wm
// adds 2u |wm_j| R_j with R_j = |b2_j| + sum_k |W2_jk| z_k; the GMF dot adds 2.01u C_u D_i;
// fp32 accumulation of both paths (<= 110 * 2^-24 relative) and the final adds are far
// below u.  Hence |err| <= 5.1u (c0 + A_u + B_i) + 2.1u C_u D_i + (subnormal terms) and
// we use e(u, i) = 6u (c0 + A_u + B_i + C_u D_i) + abs_slack.
// tests/test_gpu_prefilter.py checks (*) pair by pair on the full catalogue.
//
// Scaling: every f16 operand is scaled by a power of two so its magnitude is <= 1 (layer-1
// inputs <= 0.5, which also makes the packed add's [0,1] CLAMP an exact ReLU:
// v_pk_add_f16 ... clamp).  Scores are compared in the scaled unit s1*sw*sm.
#include <algorithm>

#include "hnm_device.h"
#include "ncf_internal.h"
#include "sample_kth.h"

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));


namespace {

constexpr int64_t CERT_MIN_ITEMS = 8192;  // below this the exact LIST kernel is cheaper
constexpr float CERT_RHO = 0.0029296875f; // 6 u16 = 3 * 2^-10
// Deep towers [2 h0, h1, h2, h3] (round 6): the same scan with a third layer; the bound keeps
// its separable form with v = |wp3|^T |W3| |W2| and a factor 7.03 u < 8 u = 2^-8 (derivation at
// cert_deep_scales below)
constexpr float CERT_RHO_DEEP = 0.00390625f;
constexpr int CERT_MAX_NP = 64;           // item partitions (candidate segments per row)
constexpr int CERT_PROXY_USERS = 8;       // batch rows that pick the champion sample
#ifndef CERT_CHAMPIONS_AB  // A/B builds only (tools/build_variant.sh)
#define CERT_CHAMPIONS_AB 2048
#endif
constexpr int64_t CERT_CHAMPIONS = CERT_CHAMPIONS_AB;  // champion sample size (item groups), at most
constexpr int64_t CERT_GROUP_MIN = 48;    // items per champion group, at least
// Gated per-user strided sample (round 5).  The champion sample is tight when the rows' best
// items are shared (init weights at the H&M shape: ~70 candidates a row) and degrades to a
// ~1/52 random sample when they are user-specific (trained-like weights: 600+ candidates and
// overflowing segments).  A sample pass over one 32-item tile in CERT_STRIDE for every row gives
// a second lower bound (the larger of the two is used) at ~1/CERT_STRIDE of the scan's cost.
// Whether it pays is predicted on the proxy rows, whose every item the proxy pass scored:
// cert_gate_kernel takes each proxy's K-th over its LEAVE-ONE-OUT champions (picked by the
// other proxies: what a non-proxy row sees) and over the strided tiles, and counts, per proxy,
// the items the main scan would append under each bound (approx + e_i >= tau, tau = kv - 2 Eu:
// cert_tau_kernel); the pass runs when it saves more than CERT_GATE_GAIN
// candidates a row on average -- re-scoring ~250 candidates costs about what the 1/8 pass does
// (bench step: 65 us for 4,096 x 70 candidates against 1/8 of a 1.85 ms scan).  Gated off, the
// pass and its K-th exit at launch.
// Opt-in (HNM_OPT_STRIDED = 1; round 5, A/B on one box: init weights 2.002 -> 2.046 ms a step,
// the gate and the gated-off launches; "norms" weights 3.683 -> 3.092 ms).
constexpr int CERT_STRIDE = 8;
constexpr int64_t CERT_GATE_GAIN = 150;  // (the proxies under-predict the saving: 235 predicted
                                         // for 468 measured on "norms" batch 1)
// scan workgroups per CU (LDS 51.7 KB each; the scan's 168 VGPRs fit three waves per SIMD)
#define HNM_SCAN_OCC 3
constexpr int CERT_WG_PER_CU = HNM_SCAN_OCC;

enum { CM_P, CM_Q, CM_WG, CM_G, CM_B, CM_D, CM_N };

struct CertParams {
  unsigned mx[CM_N];  // float bits of non-negative maxima (reduced from per-block partials)
  float s1, sw, sm, sgu, sgi;
  float s3;           // deep towers: the layer-3 weight scale (1 otherwise)
  float unit, cg;     // scaled score unit; GMF accumulator -> score unit
  float rho;          // the bound's relative factor (CERT_RHO; deep towers CERT_RHO_DEEP)
  float c0, absb, Bmax, Dmax;
  int bad;            // bound not usable: every row takes the exact fallback
};

__device__ __forceinline__ float nmax(float a, float b) { return (b > a || b != b) ? b : a; }

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = nmax(x, __shfl_xor(x, o));
  return x;
}

// layer-1 unit stored at pair-permuted position t (x[h*32+s] = x[2s+h])
__device__ __forceinline__ int korig(int t) { return 2 * (t & 31) + (t >> 5); }

// ------------------------------------------------------------------ bound statistics
__global__ __launch_bounds__(256) void cert_stats_kernel(NcfTabs t, int64_t B, int64_t I, int mf,
                                                         const float* __restrict__ W2, int h1,
                                                         int h2, const float* __restrict__ wm,
                                                         CertParams* prm, float* __restrict__ Au,
                                                         float* __restrict__ Cu,
                                                         float* __restrict__ Bi,
                                                         float* __restrict__ Di,
                                                         float* __restrict__ part, int item_blocks,
                                                         int user_blocks) {
  __shared__ float vs[64];
  __shared__ float red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 64) {
    float v = 0.f;
    const int k = korig(tid);
    if (k < h1)
      for (int j = 0; j < h2; ++j) v += fabsf(wm[j]) * fabsf(W2[j * h1 + k]);
    vs[tid] = v;
  }
  __syncthreads();
  const float vt = vs[lane];
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;  // items: Q, G, B, D / users: P, WG
  const bool items = (int)blockIdx.x < item_blocks;
  if (items) {
    // four items per step, their loads issued together (one item a step waited on each)
    const int64_t stride = (int64_t)item_blocks * 4;
    for (int64_t i0 = (int64_t)blockIdx.x * 4 + wave; i0 < I; i0 += 4 * stride) {
      float aq[4], g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = std::min<int64_t>(i0 + u * stride, I - 1);
        aq[u] = fabsf(t.Qi[i * 64 + lane]);
        g[u] = lane < mf ? t.G[i * t.ldg + lane] : 0.f;
      }
      // the 8 wave sums (vt . |q|, |g|^2 of the 4 items) as one reduce-scatter butterfly: each
      // xor step halves the values a lane carries (10 shuffles instead of 48); every sum is
      // formed along the same xor 32, 16, ..., 1 pairing as wave_sum, so bitwise the same
      float v8[8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v8[u] = vt * aq[u];
        v8[4 + u] = g[u] * g[u];
        if (i0 + u * stride < I) {  // uniform
          m0 = nmax(m0, aq[u]);
          m1 = nmax(m1, fabsf(g[u]));
        }
      }
      const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
      float w4[4], w2[2];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w4[q] = (b5 ? v8[2 * q + 1] : v8[2 * q]) + __shfl_xor(b5 ? v8[2 * q] : v8[2 * q + 1], 32);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        w2[q] = (b4 ? w4[2 * q + 1] : w4[2 * q]) + __shfl_xor(b4 ? w4[2 * q] : w4[2 * q + 1], 16);
      float w1 = (b3 ? w2[1] : w2[0]) + __shfl_xor(b3 ? w2[0] : w2[1], 8);
      w1 += __shfl_xor(w1, 4);
      w1 += __shfl_xor(w1, 2);
      w1 += __shfl_xor(w1, 1);
      const int idx = (b5 ? 1 : 0) + (b4 ? 2 : 0) + (b3 ? 4 : 0);  // the sum this lane holds
      const int64_t i = i0 + (idx & 3) * stride;
      if (i < I) {
        if (idx < 4) {
          m2 = nmax(m2, w1);
          if ((lane & 7) == 0) Bi[i] = w1;
        } else {
          const float dq = sqrtf(w1);
          m3 = nmax(m3, dq);
          if ((lane & 7) == 0) Di[i] = dq;
        }
      }
    }
  } else {
    const int ub = (int)blockIdx.x - item_blocks;
    for (int64_t b = (int64_t)ub * 4 + wave; b < B; b += (int64_t)user_blocks * 4) {
      const float ap = fabsf(t.Pu[b * 64 + lane]);
      const float wg = t.WGu[b * 64 + lane];
      m0 = nmax(m0, ap);
      m1 = nmax(m1, fabsf(wg));
      const float a = wave_sum(vt * ap), c2 = wave_sum(wg * wg);
      if (lane == 0) {
        Au[b] = a;
        Cu[b] = sqrtf(c2);
      }
    }
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  m3 = wave_max(m3);
  if (lane == 0) {
    red[wave][0] = m0;
    red[wave][1] = m1;
    red[wave][2] = m2;
    red[wave][3] = m3;
  }
  __syncthreads();
  if (tid < 4) {
    float m = red[0][tid];
    for (int w = 1; w < 4; ++w) m = nmax(m, red[w][tid]);
    // per-block partials (no same-address atomics); reduced by cert_scales_kernel
    part[blockIdx.x * 4 + tid] = m;
  }
}

__device__ __forceinline__ float pow2_below_inv(float m) {  // 2^-e with m < 2^e (m > 0)
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, -e);
}

// One block: weight statistics, scales, slack.
__global__ __launch_bounds__(256) void cert_scales_kernel(const float* __restrict__ W2, int h1,
                                                          int h2, const float* __restrict__ b2,
                                                          const float* __restrict__ wm,
                                                          const float* __restrict__ bp,
                                                          CertParams* prm,
                                                          const float* __restrict__ part,
                                                          int item_blocks, int user_blocks,
                                                          int* __restrict__ ovf_cnt, CertDeep dp) {
  __shared__ float red[7][4];
  __shared__ float pm[4][6];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {  // per-block partial maxima of cert_stats_kernel: items Q G B D, users P WG
    float q = 0.f, g = 0.f, bb = 0.f, dd = 0.f, pp = 0.f, wg = 0.f;
    // partials in batches of 8 per thread: every load of a batch issued before the first use
    // (one L2 round trip per batch instead of one per partial: this single block is latency)
    const int nblk = item_blocks + user_blocks;
    for (int b0 = 0; b0 < nblk; b0 += 8 * 256) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[k] = *reinterpret_cast<const float4*>(part + 4 * std::min(b0 + 256 * k + tid, nblk - 1));
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int blk = b0 + 256 * k + tid;
        if (blk < item_blocks) {
          q = nmax(q, v[k].x); g = nmax(g, v[k].y); bb = nmax(bb, v[k].z); dd = nmax(dd, v[k].w);
        } else if (blk < nblk) {
          pp = nmax(pp, v[k].x); wg = nmax(wg, v[k].y);
        }
      }
    }
    q = wave_max(q); g = wave_max(g); bb = wave_max(bb); dd = wave_max(dd);
    pp = wave_max(pp); wg = wave_max(wg);
    if (lane == 0) {
      pm[wave][0] = q; pm[wave][1] = g; pm[wave][2] = bb; pm[wave][3] = dd;
      pm[wave][4] = pp; pm[wave][5] = wg;
    }
    __syncthreads();
    if (tid < 6) {
      float m = pm[0][tid];
      for (int w = 1; w < 4; ++w) m = nmax(m, pm[w][tid]);
      const int slot = tid == 0 ? CM_Q : tid == 1 ? CM_G : tid == 2 ? CM_B : tid == 3 ? CM_D
                     : tid == 4 ? CM_P : CM_WG;
      prm->mx[slot] = __float_as_uint(m);
    }
    if (tid == 0 && ovf_cnt) *ovf_cnt = 0;
    __syncthreads();
  }
  float mW = 0.f, vsum = 0.f, mwm = 0.f, mb2 = 0.f, c0 = 0.f, swm = 0.f;
  for (int e = tid; e < h2 * h1; e += 256) {
    const float w = fabsf(W2[e]);
    mW = nmax(mW, w);
    vsum += fabsf(wm[e / h1]) * w;
  }
  float mrow = 0.f;  // max_j sum_k |W2_jk|: 8 threads a row, strided partials + 3 xor steps
  for (int j0 = 0; j0 < h2; j0 += 32) {
    const int j = j0 + (tid >> 3);
    float rs = 0.f;
    if (j < h2)
      for (int k = tid & 7; k < h1; k += 8) rs += fabsf(W2[j * h1 + k]);
    rs += __shfl_xor(rs, 1);
    rs += __shfl_xor(rs, 2);
    rs += __shfl_xor(rs, 4);
    mrow = nmax(mrow, rs);
  }
  for (int j = tid; j < h2; j += 256) {
    mwm = nmax(mwm, fabsf(wm[j]));
    mb2 = nmax(mb2, fabsf(b2[j]));
    c0 += fabsf(wm[j]) * fabsf(b2[j]);
    swm += fabsf(wm[j]);
  }
  mW = wave_max(mW);
  mrow = wave_max(mrow);
  mwm = wave_max(mwm);
  mb2 = wave_max(mb2);
  vsum = wave_sum(vsum);
  c0 = wave_sum(c0);
  swm = wave_sum(swm);
  if (lane == 0) {
    red[0][wave] = mW;
    red[1][wave] = mwm;
    red[2][wave] = mb2;
    red[3][wave] = vsum;
    red[4][wave] = c0;
    red[5][wave] = swm;
    red[6][wave] = mrow;
  }
  __syncthreads();
  if (tid != 0) return;
  for (int w = 1; w < 4; ++w) {
    red[0][0] = nmax(red[0][0], red[0][w]);
    red[1][0] = nmax(red[1][0], red[1][w]);
    red[2][0] = nmax(red[2][0], red[2][w]);
    red[3][0] += red[3][w];
    red[4][0] += red[4][w];
    red[5][0] += red[5][w];
    red[6][0] = nmax(red[6][0], red[6][w]);
  }
  mW = red[0][0];
  mwm = red[1][0];
  mb2 = red[2][0];
  vsum = red[3][0];
  c0 = red[4][0];
  swm = red[5][0];
  mrow = red[6][0];
  const float mP = __uint_as_float(prm->mx[CM_P]), mQ = __uint_as_float(prm->mx[CM_Q]);
  const float mWG = __uint_as_float(prm->mx[CM_WG]), mG = __uint_as_float(prm->mx[CM_G]);
  const float Bmax = __uint_as_float(prm->mx[CM_B]), Dmax = __uint_as_float(prm->mx[CM_D]);
  const float lim = 1099511627776.f;  // 2^40
  bool bad = false;
  for (float m : {mP, mQ, mWG, mG, Bmax, Dmax, mW, mrow, mwm, mb2, vsum, c0, fabsf(bp[0])})
    bad |= !(m <= lim);  // also catches NaN / inf
  const float zmax = mP + mQ;
  const float s1 = zmax > 0.f ? 0.5f * pow2_below_inv(zmax) : 1.f;  // s1 * z <= 0.5
  // W2 / b2 scale: |H~| <= s1 sw |b2| + sw sum_k |W2_jk| x~_k (x~ <= 0.5 (1 + u)^2) stays
  // below 1, so the [0, 1] clamp of the f32 -> f16 convert is an exact ReLU
  const float hmax = (s1 * mb2 + 0.51f * mrow) * 1.01f;
  const float sw = hmax > 0.f ? pow2_below_inv(hmax) : 1.f;
  float sm = mwm > 0.f ? pow2_below_inv(mwm) : 1.f;
  const float sgu = mWG > 0.f ? pow2_below_inv(mWG) : 1.f;
  const float sgi = mG > 0.f ? pow2_below_inv(mG) : 1.f;
  const float phi = 2.98023224e-08f;  // 2^-25: half the f16 subnormal spacing
  const float rmax = mb2 + 64.f * mW * zmax;
  float s3 = 1.f, rho = CERT_RHO;
  // the per-rounding absolute slack terms (real units, x 16 phi below): layer-1 operands and
  // sum, W2 rounding, relu(H) rounding, GMF operands -- and the last weights' rounding
  float abst = 3.f * vsum / s1 + 64.f * swm * zmax / sw + swm / (s1 * sw) + 64.f * mG / sgu +
               64.f * mWG / sgi;
  if (dp.W3) {
    // Deep tower (round 6).  `wm` is u = |wp3|^T |W3| here, so vsum = sum_k v_k, swm = sum_l u_l
    // and c0 = u . |b2| with v = |wp3|^T |W3| |W2| (the stats kernel's A_u / B_i).  Error of the
    // scan against the exact chain, u = 2^-11: layer-2 output dH_l <= 3.02u sum_k |W2_lk| z_k as
    // before; y~ = f16(relu(H~)) adds u R_l (R_l = |b2_l| + sum_k |W2_lk| z_k >= |H_l|); the f16
    // W3 and layer-3 accumulation give dH3_m <= sum_l |W3_ml| ((1 + u) dH_l + 2u R_l); z~ =
    // f16(relu(H3~)) adds u R3_m (R3_m = |b3_m| + sum_l |W3_ml| R_l) and the f16 wp3 another u
    // R3_m: |err| <= u (7.03 (A_u + B_i) + 4 c0 + 2 cb3) + 2.01u C_u D_i + O(u^2) <= 8u (c0 + cb3
    // + A_u + B_i + C_u D_i) (fp32 accumulation ~2^-22 relative, inside the margin); absolute
    // slack for f16 subnormals per rounding site, each through the weights after it.
    float mW3 = 0.f, mrow3 = 0.f, mb3 = 0.f, mwp = 0.f, swp = 0.f, cb3 = 0.f;
    for (int m = 0; m < dp.h3; ++m) {
      float rs = 0.f;
      for (int l = 0; l < h2; ++l) {
        const float a = fabsf(dp.W3[m * h2 + l]);
        mW3 = nmax(mW3, a);
        rs += a;
      }
      mrow3 = nmax(mrow3, rs);
      mb3 = nmax(mb3, fabsf(dp.b3[m]));
      mwp = nmax(mwp, fabsf(dp.wp3[m]));
      swp += fabsf(dp.wp3[m]);
      cb3 += fabsf(dp.wp3[m]) * fabsf(dp.b3[m]);
    }
    for (float m : {mW3, mrow3, mb3, mwp, swp, cb3}) bad |= !(m <= lim);
    // relu(H~) <= 1 after the clamp, so |H3~| <= s3 (s1 sw |b3| + sum_l |W3_ml|) <= 1
    const float hmax3 = (s1 * sw * mb3 + mrow3) * 1.01f;
    s3 = hmax3 > 0.f ? pow2_below_inv(hmax3) : 1.f;
    sm = mwp > 0.f ? pow2_below_inv(mwp) : 1.f;
    const float r3max = mb3 + (float)h2 * mW3 * rmax;
    c0 += cb3;
    abst += 32.f * swp * rmax / s3 + swp / (s1 * sw * s3) + 16.f * r3max / sm;
    rho = CERT_RHO_DEEP;
  } else {
    abst += 32.f * rmax / sm;  // wm rounding
  }
  const float unit = s1 * sw * s3 * sm;
  const float cg = unit / (sgu * sgi);
  bad |= !(unit >= 1e-30f && unit <= 1e30f && cg >= 1e-30f && cg <= 1e30f);
  const float absb = 16.f * phi * abst + 2.4e-7f * fabsf(bp[0]);
  prm->s1 = s1;
  prm->sw = sw;
  prm->sm = sm;
  prm->s3 = s3;
  prm->sgu = sgu;
  prm->sgi = sgi;
  prm->unit = unit;
  prm->cg = cg;
  prm->rho = rho;
  prm->c0 = c0;
  prm->absb = absb;
  prm->Bmax = Bmax;
  prm->Dmax = Dmax;
  prm->bad = bad || !(absb <= lim);
}

// f16 operand tables.  Q16/P16 keep the pair-permuted order (the layer-1 unit order is
// free as long as W2h's columns follow it); G16/WG16 use the natural GMF order.
__global__ __launch_bounds__(256) void cert_convert_kernel(
    NcfTabs t, int64_t B, int64_t I, int mf, const CertParams* __restrict__ prm,
    _Float16* __restrict__ P16, _Float16* __restrict__ WG16, _Float16* __restrict__ Q16,
    _Float16* __restrict__ G16, const float* __restrict__ W2, int h1, int h2,
    const float* __restrict__ b2, const float* __restrict__ wm, _Float16* __restrict__ W2h,
    _Float16* __restrict__ wmh, float* __restrict__ b2s, const float* __restrict__ Bi,
    const float* __restrict__ Cu, float* __restrict__ Bs, float* __restrict__ Cs, CertDeep dp,
    _Float16* __restrict__ W3h, _Float16* __restrict__ wph, float* __restrict__ b3s) {
  const float s1 = prm->s1, sgu = prm->sgu, sgi = prm->sgi;
  // the scan's bound terms in test units (rho * unit * B_i, ... * C_u): the same fp32
  // products the scan formed itself before, computed once here so the scan keeps no scale
  // factor live across its tile loop
  const int64_t nthreads = (int64_t)gridDim.x * 256;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const float ru = prm->rho * prm->unit;
  for (int64_t e = g; e < I; e += nthreads) Bs[e] = ru * Bi[e];
  for (int64_t e = g; e < B; e += nthreads) Cs[e] = ru * Cu[e];
  // items: 16 chunks of 4 per row
  for (int64_t e = g; e < I * 16; e += nthreads) {
    const int64_t i = e >> 4;
    const int c = (int)(e & 15);
    const float4 q = *reinterpret_cast<const float4*>(t.Qi + i * 64 + 4 * c);
    _Float16* qo = Q16 + i * 64 + 4 * c;
    qo[0] = (_Float16)(q.x * s1);
    qo[1] = (_Float16)(q.y * s1);
    qo[2] = (_Float16)(q.z * s1);
    qo[3] = (_Float16)(q.w * s1);
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (4 * c < mf) gv = *reinterpret_cast<const float4*>(t.G + i * t.ldg + 4 * c);
    _Float16* go = G16 + i * 64 + 4 * c;
    go[0] = (_Float16)(4 * c + 0 < mf ? gv.x * sgi : 0.f);
    go[1] = (_Float16)(4 * c + 1 < mf ? gv.y * sgi : 0.f);
    go[2] = (_Float16)(4 * c + 2 < mf ? gv.z * sgi : 0.f);
    go[3] = (_Float16)(4 * c + 3 < mf ? gv.w * sgi : 0.f);
  }
  for (int64_t e = g; e < B * 64; e += nthreads) {
    const int64_t b = e >> 6;
    const int k = (int)(e & 63);
    P16[e] = (_Float16)(t.Pu[e] * s1);
    WG16[e] = (_Float16)(t.WGu[b * 64 + (k & 1) * 32 + (k >> 1)] * sgu);
  }
  if (blockIdx.x == 0) {
    const float sw = prm->sw, sm = prm->sm;
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int j = e >> 6, k = korig(e & 63);
      W2h[e] = (_Float16)((j < h2 && k < h1) ? W2[j * h1 + k] * sw : 0.f);
    }
    if (threadIdx.x < 32) {
      const int j = threadIdx.x;
      wmh[j] = (_Float16)(j < h2 && !dp.W3 ? wm[j] * sm : 0.f);
      b2s[j] = j < h2 ? b2[j] * s1 * sw : 0.f;
    }
    if (dp.W3) {  // layer 3 (unit m, hidden l) x s3, its bias x s1 sw s3, wp3 x sm
      const float s3 = prm->s3;
      for (int e = threadIdx.x; e < 16 * 32; e += 256) {
        const int m = e >> 5, l = e & 31;
        W3h[e] = (_Float16)((m < dp.h3 && l < h2) ? dp.W3[m * h2 + l] * s3 : 0.f);
      }
      if (threadIdx.x < 16) {
        const int m = threadIdx.x;
        wph[m] = (_Float16)(m < dp.h3 ? dp.wp3[m] * sm : 0.f);
        b3s[m] = m < dp.h3 ? dp.b3[m] * s1 * sw * s3 : 0.f;
      }
    }
  }
}

// Deep towers: u_l = sum_m |wp3_m| |W3_ml| (l < h2), the weights the bound statistics take in
// place of the two-layer tower's |wm| (v = |wp3|^T |W3| |W2|)
__global__ __launch_bounds__(64) void cert_deep_u_kernel(CertDeep dp, int h2, float* __restrict__ u) {
  const int l = threadIdx.x;
  if (l >= 32) return;
  float v = 0.f;
  if (l < h2)
    for (int m = 0; m < dp.h3; ++m) v += fabsf(dp.wp3[m]) * fabsf(dp.W3[m * h2 + l]);
  u[l] = v;
}

// ------------------------------------------------------------------ f16 scan kernel
// SAMPLE: dense[b][n] = approx - e_i (scanned item n = sidx[n] if set), e_i = the per-item part
//         of the bound, 6u unit (B_i + C_u D_i);
// THRESH: append item n to segment (b, partition) when approx + e_i >= tau_b;
// DEBUG:  dense[b][n] = approx, dense2[b][n] = Eu_b + e_i (the whole bound), scaled units.
enum { SCAN_SAMPLE = 0, SCAN_THRESH = 1, SCAN_DEBUG = 2 };

struct ScanArgs {
  const _Float16* P16;   // [B, 64]
  const _Float16* WG16;  // [B, 64]
  const _Float16* Q16;   // [Itot, 64]
  const _Float16* G16;   // [Itot, 64]
  const _Float16* W2h;   // [32, 64]
  const _Float16* wmh;   // [32]
  const float* b2s;      // [32]
  const _Float16* W3h;   // DEEP: [16, 32] layer-3 weights x s3 (unit, hidden)
  const _Float16* wph;   // DEEP: [16] prediction weights of the layer-3 units x sm
  const float* b3s;      // DEEP: [16] layer-3 bias x s1 sw s3
  const float* Bi;       // [Itot] per-item bound terms (x rho * unit: test units)
  const float* Di;
  const float* Cu;       // [B] per-user bound terms (x rho * unit)
  const float* Eu;       // [B] user-constant part of the bound, scaled (DEBUG)
  const CertParams* prm;
  int64_t B;
  int64_t I;        // scanned items (sample count for the sample pass)
  const int32_t* sidx;  // SAMPLE: scanned item n is item sidx[n] (gather map), if set
  int64_t ipp;
  int NP;
  int upw;  // users per wave (32; fewer for the 8-row proxy pass: every wave gets a pair)
  const int64_t* mptr;
  const int32_t* midx;
  const float* tau;  // [B] scaled thresholds (THRESH)
  int* cnt;          // [B, NP] appended counts (THRESH)
  int32_t* buf;      // [B, NP, capp] appended item ids (THRESH)
  float* segd;       // [B, NP, capp] their test values approx + e_i - tau (THRESH)
  int capp;
  float* dense;      // [B, ldo]
  float* dense2;     // [B, ldo] (DEBUG)
  int64_t ldo;
  const int* gate;   // SAMPLE: *gate == 0 -> the launch does nothing (gated strided sample)
};

__device__ __forceinline__ f32x16 mfma16(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// A wave owns 32 users, a workgroup 128; 32-item tiles of Q16/G16 go through LDS.
// Per (user pair, tile): layer 2 as 4 + 4 v_mfma_f32_32x32x16_f16 (two independent chains;
// A = W2~, B = clamp(P~ + Q~) built with 16 packed adds per user; v_mfma_f32_32x32x16_f16 B
// operand: lane (j, h) holds B[k = 8h + e][col j], e = 0..7), GMF once per tile for all 32
// users (4 MFMAs).  THRESH / SAMPLE: the epilogue wm . relu(H~) of BOTH users runs on the matrix
// pipe as 4 v_mfma_f32_16x16x32_f16 -- relu(H~) by the [0, 1] clamp of the f32 -> f16
// converts, the 16x16x32 B operand taking each lane's 8 converted accumulator rows as they lie
// (k-group g = lanes 16g..16g+15 = half g >> 1, items 16 (g & 1) + c), A rows 0/1 = wm on user
// a's k-groups of items 0-15 / 16-31, rows 2/3 the same for user b -- so one MFMA sums both
// halves of a column (no cross-lane swap), and the accumulator is seeded with the tile's folded
// per-pair term (GMF + bound - threshold, pair-interleaved in LDS so lanes 0-15 read their 4
// seeds as one b128).  Lanes 0-15 end with the 64 test values; 4 ballots assemble the pair's
// 64-bit pass mask with bit u*32 + item (the lane layout of the append).  Measured against the
// earlier packed-dot epilogue (16 v_dot2c + a permlane32 swap per pair, 1.94 ms) and a
// software-pipelined two-waves-per-SIMD variant (2.1-2.2 ms): 1.87 ms (tools/scan_ablation.hip,
// profiles/r2_ncf_scan_variants.txt); splitting it (user a on the matrix pipe, user b by packed
// dots) measured 2.03 vs 1.88 ms (round 3, profiles/r3c_ncf_epilogue_ab.txt): the VALU side is
// the binding one.  DEBUG keeps a VALU epilogue (packed dots + swap).
// DEEP (round 6, towers [2 h0, h1 <= 64, h2 <= 32, h3 <= 16]): layer 2 as above, then layer 3 on
// the matrix pipe in place of the wm epilogue -- per user and item half g (items c / c + 16) two
// v_mfma_f32_16x16x32_f16 whose A rows are W3's 16 units with the k-groups of the other item half
// zeroed (the 16x16x32 B operand mixes items c and c + 16 across k-groups), accumulator seeded
// with b3 -- relu by the clamp of the f32 -> f16 converts, and the prediction wp3 . relu(h3) as a
// v_mfma_f32_16x16x16_f16 whose B operand is that accumulator as it lies (rows 4 (lane >> 4) + r =
// units, columns = items) and whose A row idx = 2 user + g holds wp3: four of them chained on the
// folded seeds leave the test values where the two-layer epilogue leaves them.  DEBUG uses the
// same matrix epilogue (seeds = GMF only).  Two waves per SIMD (28 more live registers).
template <int MODE, bool DEEP = false>
__global__ __launch_bounds__(256, DEEP ? 2 : HNM_SCAN_OCC) void ncf16_scan_kernel(ScanArgs A) {
  constexpr int RS = 72;   // LDS row stride in halfs (144 B): conflict-free b128 reads
  constexpr int NU = 128;  // users per workgroup
  // the matrix-pipe epilogue and its folded seed table (FOLD: GMF + bound - threshold; the deep
  // DEBUG pass: GMF alone)
  constexpr bool FOLD = MODE == SCAN_THRESH || MODE == SCAN_SAMPLE || (DEEP && MODE == SCAN_DEBUG);
  if (MODE == SCAN_SAMPLE && A.gate && *A.gate == 0) return;  // whole grid: gated off
  __shared__ __attribute__((aligned(16))) _Float16 qs[2][TILE * RS];  // double-buffered tiles
  __shared__ __attribute__((aligned(16))) _Float16 gs[2][TILE * RS];
  __shared__ __attribute__((aligned(16))) _Float16 ps[NU * 64];
  // per wave: the GMF table of its 32 users x the tile's 32 items (FOLD: folded test terms,
  // pair-interleaved: g7 index below; DEBUG: gsm[row][item])
  __shared__ __attribute__((aligned(16))) float gsm[4][32][33];
  __shared__ float2 ut[4][32];  // FOLD: (tau or 0, cu) per user

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar loop state
  // grid: x = item partition (NP a multiple of 8), y = user block -> the round-robin
  // workgroup -> XCD placement keeps partition p on XCD p % 8 (its tiles stay in that L2)
  const int upw = A.upw;  // <= 32 (NU / 4)
  const int64_t ublk = (int64_t)blockIdx.y * 4 * upw;
  const int64_t u0 = ublk + wave * upw;
  const int nu = (int)std::max<int64_t>(0, std::min<int64_t>(upw, A.B - u0));
  const int p = blockIdx.x;
  const int64_t part_start = (int64_t)p * A.ipp;
  const int64_t part_end = std::min<int64_t>(A.I, part_start + A.ipp);

  for (int e = tid; e < NU * 8; e += 256) {
    const int r = e >> 3, c = e & 7;
    h8 v = {};
    if (ublk + r < A.B) v = *reinterpret_cast<const h8*>(A.P16 + (ublk + r) * 64 + 8 * c);
    *reinterpret_cast<h8*>(&ps[r * 64 + 8 * c]) = v;
  }
  h8 aw[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) aw[s] = *reinterpret_cast<const h8*>(A.W2h + j * 64 + 16 * s + 8 * h);
  h8 ag[4];  // GMF A operand: this wave's users' wp*g_u rows
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    h8 z = {};
    ag[s] = j < nu ? *reinterpret_cast<const h8*>(A.WG16 + (u0 + j) * 64 + 16 * s + 8 * h) : z;
  }
  f32x16 b2c;
#pragma unroll
  for (int r = 0; r < 16; ++r) b2c[r] = A.b2s[mfma32_row(r, h)];
  // epilogue A operands (16x16x32: lane holds A[row lane & 15][k = 8 (lane >> 4) + e])
  h8 ewa[2], ewb[2];
  h2 wm2[8];  // DEBUG: wm of this lane's accumulator rows, in pairs
  h8 e3[2][2];  // DEEP: layer-3 A operands [item half g][accumulator half f]
  h4 ep[4];     // DEEP: prediction A operands, wp3 in row idx = 2 user + g
  f32x4 b3c;    // DEEP: layer-3 accumulator seeds (rows 4 (lane >> 4) + r)
  if constexpr (DEEP) {
    const int m = lane & 15, kg = lane >> 4;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          e3[g][f][e] = (kg & 1) == g ? A.W3h[m * 32 + mfma32_row(8 * f + e, kg >> 1)] : (_Float16)0.f;
#pragma unroll
    for (int idx = 0; idx < 4; ++idx)
#pragma unroll
      for (int e = 0; e < 4; ++e) ep[idx][e] = m == idx ? A.wph[4 * kg + e] : (_Float16)0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) b3c[r] = A.b3s[4 * kg + r];
  } else {
    const int erow = lane & 15, eg = lane >> 4;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const _Float16 wv = A.wmh[mfma32_row(8 * f + e, eg >> 1)];
        ewa[f][e] = erow == (eg & 1) ? wv : (_Float16)0.f;
        ewb[f][e] = erow == 2 + (eg & 1) ? wv : (_Float16)0.f;
      }
#pragma unroll
    for (int r = 0; r < 16; r += 2)
      wm2[r >> 1] = (h2){A.wmh[mfma32_row(r, h)], A.wmh[mfma32_row(r + 1, h)]};
  }
  float* const g7 = &gsm[wave][0][0];
  // uniform scalars in SGPRs (the compiler cannot prove prm read-only, so it would keep them
  // in VGPRs -- which are the scarce resource at three waves per SIMD)
  const float cg = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(A.prm->cg)));
  // per-user registers: lane u < nu follows user u0 + u
  const float cu = lane < nu ? A.Cu[u0 + lane] : 0.f;
  float tv = __builtin_inff(), eu = 0.f;
  if (MODE == SCAN_THRESH && lane < nu) tv = A.tau[u0 + lane];
  if (MODE == SCAN_DEBUG && lane < nu) eu = A.Eu[u0 + lane];
  if (FOLD && lane < 32)
    ut[wave][lane] = make_float2(MODE == SCAN_THRESH ? tv : 0.f, cu);  // lanes >= nu: (inf | 0, 0)
  int ccount = 0;  // THRESH: appended items of user u0 + lane in this partition
  int nm = INT_BIG, mpos = 0, mend = 0;
  const bool masked = MODE == SCAN_THRESH && A.mptr != nullptr;
  if (masked && lane < nu) {
    const int64_t lo = A.mptr[u0 + lane], hi = A.mptr[u0 + lane + 1];
    mpos = (int)mask_lower_bound(A.midx, lo, hi, (int)part_start);
    mend = (int)hi;
    nm = mpos < mend ? A.midx[mpos] : INT_BIG;
  }
  int32_t* seg = MODE == SCAN_THRESH ? A.buf + ((u0 * A.NP) + p) * (int64_t)A.capp : nullptr;
  // the wave's 32 rows of candidate ids / test values (THRESH): buffer resources over the rows'
  // segments, partition p's slots at row * segstride + slot (NP * capp * 128 < 2^31: cert_shape)
  const __amdgpu_buffer_rsrc_t segrs = __builtin_amdgcn_make_buffer_rsrc(
      MODE == SCAN_THRESH ? (void*)seg : (void*)A.buf, 0,
      MODE == SCAN_THRESH ? (int)(32 * (int64_t)A.NP * A.capp * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t segdrs = __builtin_amdgcn_make_buffer_rsrc(
      MODE == SCAN_THRESH ? (void*)(A.segd + ((u0 * A.NP) + p) * (int64_t)A.capp) : (void*)A.buf,
      0, MODE == SCAN_THRESH ? (int)(32 * (int64_t)A.NP * A.capp * 4) : 0, 0x00020000);
  const int64_t segstride = (int64_t)A.NP * A.capp;  // next user's segment

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, TILE) : 0;
  // tile staging: thread (row, c) moves 16 B of Q~ and of G~; tile t + 1 is fetched into
  // registers while tile t is scored, then stored to the other LDS buffer (one barrier
  // per tile)
  // (row, 16-B chunk) of the thread's staging slot, recomputed where used: held across the
  // tile loop they were spilled, and a spill reload's vmcnt wait also waits for the prefetch
  auto srow_of = [&]() {
    int v;
    asm volatile("v_lshrrev_b32 %0, 3, %1" : "=v"(v) : "v"(tid));
    return v;
  };
  auto sc_of = [&]() {
    int v;
    asm volatile("v_and_b32 %0, 7, %1" : "=v"(v) : "v"(tid));
    return v;
  };
  h8 nq = {}, ng = {};
  float nb = 0.f, nd = 0.f;  // per-item bound terms of lane j's next item
  // the champion gather map is a SAMPLE-pass input only (compile-time null elsewhere: no
  // dependent index loads, hence no mid-tile vmcnt waits, in the THRESH scan)
  const int32_t* const sidx = MODE == SCAN_SAMPLE ? A.sidx : nullptr;
  // 32-bit element offsets from the (uniform) table bases: the loads take an SGPR base and a
  // VGPR offset, so no 64-bit per-lane addresses stay live across the tile loop (I * 64 <
  // 2^31: ncf_cert_eligible)
  auto fetch = [&](int64_t base) {
    const int srow = srow_of(), sc = sc_of();
    const int n = (int)(base + srow);
    nq = (h8){};
    ng = (h8){};
    if (n < part_end) {
      const int it = sidx ? sidx[n] : n;
      nq = *reinterpret_cast<const h8*>(A.Q16 + (uint32_t)(it * 64 + 8 * sc));
      ng = *reinterpret_cast<const h8*>(A.G16 + (uint32_t)(it * 64 + 8 * sc));
    }
    const int cj = (int)std::min<int64_t>(base + j, part_end - 1);
    const int nj = sidx ? sidx[cj] : cj;
    nb = A.Bi[(uint32_t)nj];
    nd = A.Di[(uint32_t)nj];
  };
  auto stash = [&](int buf) {
    const int srow = srow_of(), sc = sc_of();
    *reinterpret_cast<h8*>(&qs[buf][srow * RS + 8 * sc]) = nq;
    *reinterpret_cast<h8*>(&gs[buf][srow * RS + 8 * sc]) = ng;
  };
  int64_t t = 0;
  if (t < ntiles) {
    fetch(part_start + t * TILE);
    stash(0);
  }
  __syncthreads();
  // drain every prologue load on every path into the loop (incl. ntiles == 0): otherwise the
  // waitcnt pass merges a pending prologue load into the loop and waits vmcnt(0) -- i.e. for
  // the tile prefetch too -- at the first use of a prologue register in every iteration
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15)
  for (int cur = 0; t < ntiles; cur ^= 1) {
    const int64_t base = part_start + t * TILE;
    const int64_t tn = t + 1;
    const float bj = nb, dj = nd;  // bound terms of this tile's item j (test units)
    // the prefetch is the only global load in the tile body (vmcnt waits are in order: any
    // later load's wait would also wait for it)
    if (tn < ntiles) fetch(part_start + tn * TILE);
    int lrow;  // lane (j, h)'s operand row offset in the tile buffers (recomputed: see srow_of)
    asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(lrow) : "v"(j), "v"(RS), "v"(8 * h));

    if (nu > 0) {
    {  // GMF of the wave's 32 users x 32 items, in score units
      f32x16 gacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        gacc = mfma16(ag[s], *reinterpret_cast<const h8*>(&gs[cur][lrow + 16 * s]), gacc);
      if constexpr (FOLD) {
        // folded test term gmf + sgn * e_i - tau (sgn = +1 for the threshold test, -1 for the
        // sample's lower bound; the deep DEBUG pass: gmf alone)
        constexpr float sgn = MODE == SCAN_THRESH ? 1.f : -1.f;
        // (measured, round 5: the same stores from one lane base + immediate offsets -- 6 fewer
        // VGPRs -- scheduled the pair loop's LDS reads differently, +1-2 % scan time)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = mfma32_row(r, h);
          const float2 tc = ut[wave][row];
          g7[(((row >> 1) * 16 + (j & 15)) << 2) + ((row & 1) << 1) + (j >> 4)] =
              MODE == SCAN_DEBUG ? gacc[r] * cg : (gacc[r] * cg + sgn * fmaf(tc.y, dj, bj)) - tc.x;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) gsm[wave][mfma32_row(r, h)][j] = gacc[r] * cg;
      }
    }
    h8 q[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) q[s] = *reinterpret_cast<const h8*>(&qs[cur][lrow + 16 * s]);
    const int64_t n = base + j;
    const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);
    const int nv = (int)(tile_end - base);  // valid items of the tile
    const uint64_t vm32 = nv >= 32 ? 0xffffffffull : ((1ull << nv) - 1ull);
    unsigned mbits = 0;
    if (masked) {  // scanned items are real items here (identity map in the THRESH pass)
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
            nm = mpos < mend ? A.midx[mpos] : INT_BIG;
          }
        }
      }
    }

    const _Float16* pw = &ps[(wave * upw) * 64 + 8 * h];  // user r, k-step s: pw[r * 64 + 16 s]
    for (int u = 0; u < nu; u += 2) {
      // user b = u + 1 even past nu (zero P~ rows; FOLD: folded term -inf / not stored)
      const int ua = u, ub = u + 1;
      const bool hasb = ub < nu;
      const int uh = h ? ub : ua;
      f32x16 acc0 = b2c, acc1 = b2c;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        // each fragment is read right before its MFMA (fewer live registers than a prefetch)
        const h8 pa = *reinterpret_cast<const h8*>(&pw[ua * 64 + 16 * s]);
        const h8 pb = *reinterpret_cast<const h8*>(&pw[ub * 64 + 16 * s]);
        h8 x = pa + q[s];
        x = __builtin_elementwise_min(__builtin_elementwise_max(x, (h8){}), (h8)(_Float16)1.f);
        h8 y = pb + q[s];
        y = __builtin_elementwise_min(__builtin_elementwise_max(y, (h8){}), (h8)(_Float16)1.f);
        acc0 = mfma16(aw[s], x, acc0);
        acc1 = mfma16(aw[s], y, acc1);
      }
      if constexpr (FOLD) {
        h8 ya[2], yb[2];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ya[0][e] = (_Float16)acc0[e];
          ya[1][e] = (_Float16)acc0[8 + e];
          yb[0][e] = (_Float16)acc1[e];
          yb[1][e] = (_Float16)acc1[8 + e];
        }
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          ya[f] = __builtin_elementwise_min(__builtin_elementwise_max(ya[f], (h8){}), (h8)(_Float16)1.f);
          yb[f] = __builtin_elementwise_min(__builtin_elementwise_max(yb[f], (h8){}), (h8)(_Float16)1.f);
        }
        // lanes 0-15: (a, c), (a, c + 16), (b, c), (b, c + 16); other lanes' rows are unused
        f32x4 d = *reinterpret_cast<const f32x4*>(&g7[((u >> 1) * 16 + (lane & 15)) << 2]);
        if constexpr (DEEP) {
#pragma unroll
          for (int uu = 0; uu < 2; ++uu)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
              f32x4 t3 = b3c;
              t3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(e3[g][0], uu ? yb[0] : ya[0], t3, 0, 0, 0);
              t3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(e3[g][1], uu ? yb[1] : ya[1], t3, 0, 0, 0);
              h4 z = {(_Float16)t3[0], (_Float16)t3[1], (_Float16)t3[2], (_Float16)t3[3]};
              z = __builtin_elementwise_min(__builtin_elementwise_max(z, (h4){}), (h4)(_Float16)1.f);
              d = __builtin_amdgcn_mfma_f32_16x16x16f16(ep[2 * uu + g], z, d, 0, 0, 0);
            }
        } else {
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ewa[0], ya[0], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ewa[1], ya[1], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ewb[0], yb[0], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ewb[1], yb[1], d, 0, 0, 0);
        }
        const uint64_t vmask = vm32 | (hasb ? vm32 << 32 : 0ull);
        if (MODE == SCAN_DEBUG) {  // DEEP: approx and the whole bound, per pair, scaled units
          float bjr[2], djr[2];  // the bound terms of items c and c + 16 (lanes c, c + 16)
#pragma unroll
          for (int q2 = 0; q2 < 2; ++q2) {
            bjr[q2] = __shfl(bj, (lane & 15) + 16 * q2);
            djr[q2] = __shfl(dj, (lane & 15) + 16 * q2);
          }
          const float cua = hnm_readlane_f(cu, ua), cub = hnm_readlane_f(cu, ub);
          const float eua = hnm_readlane_f(eu, ua), eub = hnm_readlane_f(eu, ub);
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int it = lane + 16 * (r & 1);
              if ((vmask >> (32 * (r >> 1) + it)) & 1) {
                const int64_t o = (u0 + ua + (r >> 1)) * A.ldo + base + it;
                A.dense[o] = d[r];
                A.dense2[o] = (r >> 1 ? eub : eua) + fmaf(r >> 1 ? cub : cua, djr[r & 1], bjr[r & 1]);
              }
            }
          }
        } else if (MODE == SCAN_SAMPLE) {
          if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int it = lane + 16 * (r & 1);
              if ((vmask >> (32 * (r >> 1) + it)) & 1)
                A.dense[(u0 + ua + (r >> 1)) * A.ldo + base + it] = d[r];  // score - e_i
            }
          }
        } else {
          const uint64_t m0 = __ballot(!(d[0] < 0.f)) & 0xffffull;
          const uint64_t m1 = __ballot(!(d[1] < 0.f)) & 0xffffull;
          const uint64_t m2 = __ballot(!(d[2] < 0.f)) & 0xffffull;
          const uint64_t m3 = __ballot(!(d[3] < 0.f)) & 0xffffull;
          uint64_t m = (m0 | (m1 << 16) | (m2 << 32) | (m3 << 48)) & vmask;  // !(score + e_i < tau)
          // filtered items of the two users, looked up only for a pair with a pass (a few % of
          // pairs): two readlanes per pair in the issue-bound loop cost ~7 % of the scan
          if (masked && m) {  // uniform
            const unsigned mba = (unsigned)hnm_readlane_i((int)mbits, ua);
            const unsigned mbb = (unsigned)hnm_readlane_i((int)mbits, ub);
            m &= ~((uint64_t)mba | ((uint64_t)mbb << 32));
          }
          if (m) {
            // lane c < 16 holds d[0..3] = the test values of (a, c), (a, c + 16), (b, c),
            // (b, c + 16): it appends its passing pairs itself -- the id and, for the
            // re-scoring's best-first order, the test value -- at the slot the pair's rank in the
            // pass mask gives (no cross-lane moves; the store addresses are uniform bases)
            const int ca = hnm_readlane_i(ccount, ua), cb = hnm_readlane_i(ccount, ub);
            if (lane < 16) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int uu = r >> 1, it = lane + 16 * (r & 1);
                const unsigned mu = (unsigned)(m >> (32 * uu));
                const int ps = (uu ? cb : ca) + __builtin_popcount(mu & ((1u << it) - 1u));
                if (((mu >> it) & 1u) && ps < A.capp) {
                  // buffer stores: uniform row offset in an SGPR, the slot in one VGPR (the
                  // tile loop runs at the 168-VGPR limit; 64-bit addresses here spilled)
                  const int so = (uu ? ub : ua) * (int)segstride * 4;
                  __builtin_amdgcn_raw_buffer_store_b32((int)(base + it), segrs, ps * 4, so, 0);
                  __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(d[r]), segdrs, ps * 4, so, 0);
                }
              }
            }
            if (lane == ua) ccount += __builtin_popcount((unsigned)m);
            if (lane == ub && hasb) ccount += __builtin_popcount((unsigned)(m >> 32));
          }
        }
      } else {  // DEBUG: approx score and the whole bound, per pair, in scaled units
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          h2 ya = {(_Float16)acc0[r], (_Float16)acc0[r + 1]};
          ya = __builtin_elementwise_min(__builtin_elementwise_max(ya, (h2){}), (h2)(_Float16)1.f);
          h2 yb = {(_Float16)acc1[r], (_Float16)acc1[r + 1]};
          yb = __builtin_elementwise_min(__builtin_elementwise_max(yb, (h2){}), (h2)(_Float16)1.f);
          ma = __builtin_amdgcn_fdot2(ya, wm2[r >> 1], ma, false);
          mb = __builtin_amdgcn_fdot2(yb, wm2[r >> 1], mb, false);
        }
        // after the swap lanes 0-31 hold user a's total, lanes 32-63 user b's
        const auto sw2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(ma), __float_as_uint(mb),
                                                          false, false);
        const float score = (__uint_as_float(sw2[0]) + __uint_as_float(sw2[1])) + gsm[wave][uh][j];
        const float cuh = h ? hnm_readlane_f(cu, ub) : hnm_readlane_f(cu, ua);
        const float euh = h ? hnm_readlane_f(eu, ub) : hnm_readlane_f(eu, ua);
        if (n < part_end && (h == 0 || hasb)) {
          A.dense[(u0 + uh) * A.ldo + n] = score;
          A.dense2[(u0 + uh) * A.ldo + n] = euh + fmaf(cuh, dj, bj);
        }
      }
    }
    }  // nu > 0
    if (tn < ntiles) stash(cur ^ 1);
    __syncthreads();
    t = tn;
  }
  if (MODE == SCAN_THRESH && lane < nu) A.cnt[(u0 + lane) * A.NP + p] = ccount;
}

// Per row: Eu = user-constant part of the bound (scaled): 6u unit (c0 + A_u) + unit abs.
// Exact scores and the scan's values satisfy |approx - (exact - bp) unit| <= Eu + e_i, so
// the sample's K-th best of (approx - e_i), kv, certifies a lower bound of the row's exact
// K-th best score in real units: L = (kv - Eu) / unit + bp (unit is a power of two; the
// relative 2^-21 covers the fp32 rounding of the subtraction and of + bp).  Rows with an
// unusable bound get L = -inf.  Any lower bound works downstream -- e.g. the max of the
// item shards' L over the ranks of a node (hnm_ncf_topk_begin_f32 / _finish_f32).
// The larger of two samples' lower bounds (kth2 used when *gate: the strided sample ran); a NaN
// in either (a row with a NaN score) stays NaN.
__device__ __forceinline__ float kth_pick(const float* kth, const float* kth2, const int* gate,
                                          int64_t x) {
  const float a = kth[x];
  if (!gate || *gate == 0) return a;
  const float c = kth2[x];
  return (a != a || c != c) ? __builtin_nanf("") : fmaxf(a, c);
}

__global__ __launch_bounds__(256) void cert_bound_kernel(const float* __restrict__ kth,
                                                         const float* __restrict__ kth2,
                                                         const int* __restrict__ gate, int K,
                                                         const float* __restrict__ Au,
                                                         const CertParams* __restrict__ prm,
                                                         const float* __restrict__ bp, int64_t B,
                                                         float* __restrict__ lb,
                                                         float* __restrict__ Eu) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float unit = prm->unit;
  const float e = unit * (prm->rho * (prm->c0 + Au[b]) + prm->absb);
  if (Eu) Eu[b] = e;
  if (!kth) return;
  float l = (kth_pick(kth, kth2, gate, b * K + (K - 1)) - e) / unit + bp[0];
  l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
  lb[b] = (!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(e)) ? l : -__builtin_inff();
}

// Per (row, r < K): the certified lower bound of the exact score of the sample's r-th best
// item (real units, as cert_bound_kernel for the K-th), for an exchange of whole lists across
// item shards: the K-th best of the union of every shard's lists bounds the global K-th.
__global__ __launch_bounds__(256) void cert_bound_lists_kernel(const float* __restrict__ kth,
                                                               const float* __restrict__ kth2,
                                                               const int* __restrict__ gate,
                                                               int K,
                                                               const float* __restrict__ Eu,
                                                               const CertParams* __restrict__ prm,
                                                               const float* __restrict__ bp,
                                                               int64_t B, float* __restrict__ lists) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= B * K) return;
  const float unit = prm->unit, e = Eu[x / K];
  // slot r of either sample's list lower-bounds the row's (r+1)-th best item of this shard,
  // so the larger of the two does too (the lists exchange needs exactly that per slot)
  float l = (kth_pick(kth, kth2, gate, x) - e) / unit + bp[0];
  l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
  lists[x] = (!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(e)) ? l : -__builtin_inff();
}

// Per row: the scan threshold in this call's scaled units from a lower bound L of the exact
// K-th (real units): an item can be in the top-K only if exact >= L, i.e. approx + e_i >=
// (L - bp) unit - Eu; minus a guard for the fp32 rounding of the test quantities (2^-18 of
// the row's absolute score scale, 2^-20 relative).  Unusable rows: tau = +inf, flag = 1
// (the exact fallback scan).
__global__ __launch_bounds__(256) void cert_tau_kernel(const float* __restrict__ lb,
                                                       const float* __restrict__ Au,
                                                       const float* __restrict__ Cu,
                                                       const float* __restrict__ Eu,
                                                       const CertParams* __restrict__ prm,
                                                       const float* __restrict__ bp, int64_t B,
                                                       float* __restrict__ tau,
                                                       int* __restrict__ flag) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float unit = prm->unit;
  const float scale = unit * (prm->c0 + Au[b] + prm->Bmax + Cu[b] * prm->Dmax);
  float tv = (lb[b] - bp[0]) * unit - Eu[b] - 3.814697265625e-06f * scale;  // 2^-18
  tv -= fabsf(tv) * 9.5367431640625e-07f;                                     // 2^-20
  const bool ok = !prm->bad && __builtin_isfinite(tv) && __builtin_isfinite(scale);
  tau[b] = ok ? tv : __builtin_inff();
  flag[b] = ok ? 0 : 1;
}

// One-shot calls (ncf_cert_topk, the deep towers' certified call): cert_bound_kernel's lower
// bound and cert_tau_kernel's threshold per row in the epilogue of the champion sample's K-th
// launch (round 6) -- the same arithmetic (L stored and reused as a register: bit for bit),
// two launches and kernel boundaries less on the per-call latency chain.  Not with the gated
// strided sample (its K-th comes from a second launch).
struct NcfBoundTauEpi {
  const CertParams* prm;
  const float* Au;
  const float* Cu;
  const float* bp;
  float* Eu;
  float* lb;
  float* tau;
  int* flag;
  __device__ void operator()(int64_t b, float kv) const {
    const float unit = prm->unit;
    const float e = unit * (prm->rho * (prm->c0 + Au[b]) + prm->absb);
    Eu[b] = e;
    float l = (kv - e) / unit + bp[0];
    l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
    l = (!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(e)) ? l : -__builtin_inff();
    lb[b] = l;
    const float scale = unit * (prm->c0 + Au[b] + prm->Bmax + Cu[b] * prm->Dmax);
    float tv = (l - bp[0]) * unit - e - 3.814697265625e-06f * scale;  // 2^-18
    tv -= fabsf(tv) * 9.5367431640625e-07f;                           // 2^-20
    const bool ok = !prm->bad && __builtin_isfinite(tv) && __builtin_isfinite(scale);
    tau[b] = ok ? tv : __builtin_inff();
    flag[b] = ok ? 0 : 1;
  }
};

// Champion sample: items split into nch contiguous groups of gsz; each group's item with the
// best mean (approx - e_i) over the proxy rows (the first users of the batch) -- a
// popularity-like sample in increasing item order.  Any item subset gives a valid lower
// bound of a row's K-th; this one tends to hold the rows' best items.  One wave per group.
// sloo (optional): also each proxy row r's leave-one-out champions, by the mean over the OTHER
// rows, at sloo[r * nch + g] (cert_gate_kernel's quality check).
__global__ __launch_bounds__(256) void cert_champion_kernel(const float* __restrict__ pd,
                                                            int64_t ld, int np_rows, int64_t I,
                                                            int64_t gsz, int64_t nch,
                                                            int32_t* __restrict__ sidx,
                                                            int32_t* __restrict__ sloo,
                                                            int64_t ns, int32_t* __restrict__ sidx2,
                                                            unsigned long long* __restrict__ gcnt) {
  // the gate's inputs: its counters zeroed, the strided sample's item map (tiles 0, S, 2S, ...
  // of 32 items: sidx2[0, ns)) -- both read only by later launches
  if (gcnt && blockIdx.x == 0 && threadIdx.x < 4) gcnt[threadIdx.x] = 0;
  if (sidx2)
    for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < ns; n += (int64_t)gridDim.x * 256)
      sidx2[n] = (int32_t)((n >> 5) * (32 * CERT_STRIDE) + (n & 31));
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nch) return;
  const int lane = threadIdx.x & 63;
  const int64_t i0 = g * gsz, i1 = std::min<int64_t>(I, i0 + gsz);
  float best = -__builtin_inff();
  int64_t bi = i0;
  float lbest[CERT_PROXY_USERS];
  int64_t lbi[CERT_PROXY_USERS];
#pragma unroll
  for (int r = 0; r < CERT_PROXY_USERS; ++r) {
    lbest[r] = -__builtin_inff();
    lbi[r] = i0;
  }
  for (int64_t i = i0 + lane; i < i1; i += 64) {
    float v[CERT_PROXY_USERS];
    float m = 0.f;
#pragma unroll
    for (int r = 0; r < CERT_PROXY_USERS; ++r) {
      v[r] = r < np_rows ? pd[r * ld + i] : 0.f;
      if (r < np_rows) m += v[r];
    }
    if (m > best) {  // NaN never wins; the lane's items are visited in increasing order
      best = m;
      bi = i;
    }
    if (sloo) {
#pragma unroll
      for (int r = 0; r < CERT_PROXY_USERS; ++r) {
        const float mr = m - v[r];
        if (mr > lbest[r]) {
          lbest[r] = mr;
          lbi[r] = i;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {  // wave argmax, ties -> smaller item
    const float ob = __shfl_xor(best, o);
    const int64_t oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) sidx[g] = (int32_t)bi;
  if (!sloo) return;
#pragma unroll
  for (int r = 0; r < CERT_PROXY_USERS; ++r) {
    float b = lbest[r];
    int64_t x = lbi[r];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ob = __shfl_xor(b, o);
      const int64_t oi = __shfl_xor(x, o);
      if (ob > b || (ob == b && oi < x)) {
        b = ob;
        x = oi;
      }
    }
    if (lane == 0 && r < np_rows) sloo[r * nch + g] = (int32_t)x;
  }
}

// Lane top-4 insert and the K-th of a wave's lists by K pops (sample_kth_kernel's scheme: a
// lower bound of the K-th best of the values offered; -inf when fewer).
struct Top4 {
  float t0 = -__builtin_inff(), t1 = -__builtin_inff(), t2 = -__builtin_inff(),
        t3 = -__builtin_inff();
  __device__ void offer(float x) {
    if (x > t3) {
      const float a = fminf(x, t2), c2 = fmaxf(x, t2);
      t3 = a;
      t2 = fminf(c2, t1);
      const float c1 = fmaxf(c2, t1);
      t1 = fminf(c1, t0);
      t0 = fmaxf(c1, t0);
    }
  }
  __device__ float kth(int K, int lane) {
    float kv = -__builtin_inff();
    for (int r = 0; r < K; ++r) {
      const float m = hnm_wave_max(t0);
      kv = m;
      if (m == -__builtin_inff()) break;  // wave-uniform
      const int wl = __builtin_ctzll(__ballot(t0 == m));
      if (lane == wl) {
        t0 = t1;
        t1 = t2;
        t2 = t3;
        t3 = -__builtin_inff();
      }
    }
    return kv;
  }
};

// The gate (one 1,024-thread workgroup per proxy row r).  Two lower bounds of the row's K-th best
// (approx - e_i): kc over its leave-one-out champions, ks over the strided sample's items (lane
// top-4 lists, each wave's K pops, the K-th of the 16 waves' lists); then, over the strided items
// -- a uniform 1/CERT_STRIDE sample of the catalogue, already in registers -- the count of those
// the main scan would append with the champion bound alone (approx + e_i >= kc - 2 Eu) and with
// the strided sample's bound too, times CERT_STRIDE.  The last workgroup writes *gate = 1 when
// the pass is predicted to save more than CERT_GATE_GAIN candidates a row.  Every load is issued
// in one of three batches (the proxy rows were just written: each dependent round trip costs
// microseconds).  Round 5, earlier forms: a kth kernel + a full-catalogue count kernel 25 + 24
// us, one fused kernel counting the whole catalogue 32 us a call.
constexpr int GATE_SPT = 16;  // strided items per thread (16,384 per row: I <= 524,288 fully)
__global__ __launch_bounds__(1024) void cert_gate_kernel(
    const float* __restrict__ pd, int64_t ld, int np_rows, const int32_t* __restrict__ sloo,
    int64_t nch, int K, int64_t ns, const float* __restrict__ Bs, const float* __restrict__ Di,
    const float* __restrict__ Cs, const float* __restrict__ Au, const CertParams* __restrict__ prm,
    unsigned long long* __restrict__ cnt, int* __restrict__ gate, int64_t B,
    unsigned long long* __restrict__ stats) {
  constexpr int NW = 16;
  __shared__ float wl[2][NW][64];
  __shared__ float kvs[2];
  __shared__ int part[2][NW];
  const int r = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const float* row = pd + r * ld;
  const int32_t* sl = sloo + r * nch;
  // the strided sample: thread tid takes its items n = tid + 1024 u (u < GATE_SPT); with more
  // than 16,384 sampled items the rest are left out (a lower bound / a sample of the count)
  const int64_t nsg = std::min<int64_t>(ns, 1024 * GATE_SPT);
  int32_t ix[4];
  float v[GATE_SPT], bsv[GATE_SPT], dv[GATE_SPT];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t q = u * 1024 + tid;
    ix[u] = q < nch ? sl[q] : -1;  // nch <= CERT_CHAMPIONS (<= 4,096 loaded)
  }
#pragma unroll
  for (int u = 0; u < GATE_SPT; ++u) {
    const int64_t n = u * 1024 + tid;
    const int64_t it = (n >> 5) * (32 * CERT_STRIDE) + (n & 31);
    const bool ok = n < nsg;
    v[u] = ok ? row[it] : -__builtin_inff();
    bsv[u] = ok ? Bs[it] : 0.f;
    dv[u] = ok ? Di[it] : 0.f;
  }
  Top4 c, t;
#pragma unroll
  for (int u = 0; u < 4; ++u) c.offer(ix[u] >= 0 ? row[ix[u]] : -__builtin_inff());
#pragma unroll
  for (int u = 0; u < GATE_SPT; ++u) t.offer(v[u]);
  for (int i = 0; i < 2; ++i) {  // each wave's K best survivors, descending
    Top4& L = i ? t : c;
    for (int q = 0; q < K; ++q) {
      const float m = hnm_wave_max(L.t0);
      if (lane == 0) wl[i][w][q] = m;
      if (m == -__builtin_inff()) {
        for (int z = q + 1 + lane; z < K; z += 64) wl[i][w][z] = -__builtin_inff();
        break;  // wave-uniform
      }
      const int wk = __builtin_ctzll(__ballot(L.t0 == m));
      if (lane == wk) {
        L.t0 = L.t1;
        L.t1 = L.t2;
        L.t2 = L.t3;
        L.t3 = -__builtin_inff();
      }
    }
  }
  __syncthreads();
  if (w < 2) {  // wave i: the K-th of the 16 waves' lists (exact for K <= 16: at most 4 values a
                // lane; a lower bound of it beyond, as good for a prediction)
    Top4 M;
    for (int z = lane; z < NW * K; z += 64) M.offer(wl[w][z / K][z % K]);
    const float kv = M.kth(K, lane);
    if (lane == 0) kvs[w] = kv;
  }
  __syncthreads();
  const float eu2 = 2.f * prm->unit * (prm->rho * (prm->c0 + Au[r]) + prm->absb);
  const float tc = kvs[0] - eu2, ts = fmaxf(kvs[0], kvs[1]) - eu2, cr = Cs[r];
  int nc = 0, nsv = 0;
#pragma unroll
  for (int u = 0; u < GATE_SPT; ++u) {
    const float ub = v[u] + 2.f * fmaf(cr, dv[u], bsv[u]);  // approx + e_i
    nc += ub >= tc;
    nsv += ub >= ts;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    nc += __shfl_xor(nc, o);
    nsv += __shfl_xor(nsv, o);
  }
  if (lane == 0) {
    part[0][w] = nc;
    part[1][w] = nsv;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long s0 = 0, s1 = 0;
    for (int q = 0; q < NW; ++q) {
      s0 += (unsigned)part[0][q];
      s1 += (unsigned)part[1][q];
    }
    // scaled to the catalogue: the sampled share of the items
    const double scale = (double)ns / (double)std::max<int64_t>(nsg, 1) * CERT_STRIDE;
    atomicAdd(&cnt[0], (unsigned long long)(s0 * scale));
    atomicAdd(&cnt[1], (unsigned long long)(s1 * scale));
    __threadfence();
    const unsigned long long ticket = atomicAdd(&cnt[2], 1ull);
    if (ticket == (unsigned long long)gridDim.x - 1) {  // every count is in
      __threadfence();
      const unsigned long long c0 = atomicAdd(&cnt[0], 0ull), c1 = atomicAdd(&cnt[1], 0ull);
      const int on = (np_rows >= 4 && !prm->bad &&
                      c0 > c1 + (unsigned long long)(CERT_GATE_GAIN * np_rows)) ? 1 : 0;
      *gate = on;
      if (stats) {
        if (on) atomicAdd(&stats[3], (unsigned long long)B);
        // diagnostics (last call): the proxies' predicted candidates under each bound
        stats[4] = c0;
        stats[5] = c1;
      }
    }
  }
}

// ------------------------------------------------------------------ exact re-scoring
// One wave per user: the exact fp32 score of each appended candidate, computed with the
// arithmetic of ncf32_kernel (same MFMA chain for layer 2, the GMF dot as the fma chain
// the f32 MFMA is bitwise equal to: tools/mfma_semantics_probe.hip (a)), then the exact
// (score desc, item asc) top-K.  Candidates sit in NP per-partition segments; a row with a
// flagged bound, an overflowing segment or fewer than K candidates is queued for the
// fallback.
// Four k steps' LDS operands per round trip in the layer-2 chain (round 4, under rocprofv3:
// 1 step 67.3 us, 2 steps 65.8-66.3, 4 steps 64.8 -- the operand waits are not what bounds it;
// the candidates' G / Q row gathers are).  RESCORE_PERSIST persistent workgroups per CU loop
// over rows (round 4, per-rank step of the sharded NCF, tools/rank_shape_probe.py: W = 1 2.172
// -> 2.147 ms, W = 8 (32,768 rows of ~1/8 the candidates) 2.381 -> 2.284 ms at 3 per CU, 6 per
// CU 2.151 / 2.315, against one workgroup per 4 rows): the W2 fragments are staged into LDS once
// per workgroup instead of once per 4 rows.
// DEEP (round 6): the candidates' exact scores by the deep tower's chain in ncf_deep_kernel's
// order (bitwise the exact deep kernels): layer 2 as an f32-MFMA chain FROM ZERO over k = 0..63
// (the staged A rows permuted so that accumulator register r of lane half h holds unit 2r + h),
// relu(acc + b2); layer 3 the same way over l = 2s + h with W3 row m on A row mfma32_row(m, 0)
// (so lane half 0 holds every unit of a candidate), relu(acc + b3); then in lane half 0 ONE fmaf
// chain over the GMF terms wp_j (g_u,j g_i,j) and the units' wp3_m z_m, + bp.
#ifndef RESCORE_PERSIST  // A/B builds only (tools/build_variant.sh)
#define RESCORE_PERSIST 3
#endif
#ifndef RESCORE_BEST_FIRST_AB
#define RESCORE_BEST_FIRST_AB 96
#endif
constexpr int RESCORE_BEST_FIRST = RESCORE_BEST_FIRST_AB;  // rows with more candidates score the best 64 first
template <bool DEEP>
__global__ __launch_bounds__(256, DEEP ? 2 : 3) void ncf_rescore_kernel(
    NcfTabs t, int mf, const float* __restrict__ W2, int h1, int h2, const float* __restrict__ b2,
    const float* __restrict__ wm, const float* __restrict__ bp, int64_t B,
    const int* __restrict__ flag, const int* __restrict__ cnt, const int32_t* __restrict__ buf,
    const float* __restrict__ bufd, const float* __restrict__ tau, const float* __restrict__ Eu,
    const float* __restrict__ Au, const float* __restrict__ Cu, const CertParams* __restrict__ prm,
    int NP, int capp, int K, int short_ok, float* __restrict__ ov, int64_t* __restrict__ oi,
    int32_t* __restrict__ ovf_rows, int32_t* __restrict__ ovf_cnt,
    unsigned long long* __restrict__ stats, CertDeep dp, int64_t num_users) {
  constexpr int KS = 32;
  __shared__ int stg[4][96];  // best-first: staged candidate ordinals
  // DEEP: layer-3 A fragments (16 k steps), b3, the prediction weights, each wave's user GMF row
  __shared__ float w3l[DEEP ? 16 * 64 : 1];
  __shared__ float b3l[16], wpl[DEEP ? 128 + 16 : 1];
  __shared__ float g0l[DEEP ? 4 : 1][64];
  __shared__ __attribute__((aligned(16))) float wgs[4][64];
  __shared__ __attribute__((aligned(16))) float b2l[32], wml[32];  // 0 beyond h2
  __shared__ int pref[4][CERT_MAX_NP + 1];
  // the layer-2 MFMA operands that do not change along a row -- W2 fragments (k step s, lane)
  // and the user's P row -- come from LDS (a broadcast read per MFMA) instead of 64 VGPRs, so
  // three waves per SIMD fit without spills
  __shared__ float w2l[KS * 64];
  __shared__ __attribute__((aligned(16))) float pl[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  if (tid < 32) {
    b2l[tid] = tid < h2 ? b2[tid] : 0.f;
    wml[tid] = !DEEP && tid < h2 ? wm[tid] : 0.f;  // (deep towers: wp holds mf + h3 only)
  }
  for (int e = tid; e < KS * 64; e += 256) {
    const int s = e >> 6, jj = e & 31, k = 2 * s + ((e >> 5) & 1);
    // DEEP: A row jj = mfma32_row(r, h) carries unit 2r + h
    const int row = DEEP ? 2 * ((jj & 3) + 4 * (jj >> 3)) + ((jj >> 2) & 1) : jj;
    w2l[e] = (row < h2 && k < h1) ? W2[row * h1 + k] : 0.f;
  }
  if constexpr (DEEP) {
    for (int e = tid; e < 16 * 64; e += 256) {
      const int s = e >> 6, jj = e & 31, k = 2 * s + ((e >> 5) & 1);
      const int m = (jj & 3) + 4 * (jj >> 3);  // rows mfma32_row(m, 0): lane half 0
      w3l[e] = (((jj >> 2) & 1) == 0 && m < dp.h3 && k < h2) ? dp.W3[m * h2 + k] : 0.f;
    }
    if (tid < 16) b3l[tid] = tid < dp.h3 ? dp.b3[tid] : 0.f;
    for (int e = tid; e < mf + dp.h3; e += 256) wpl[e] = dp.wp[e];
  }
  // persistent: the workgroup's shared operands loaded once, then each wave takes rows
  // b, b + 4 * gridDim.x, ... (its per-row LDS arrays are its own: no workgroup barrier inside)
  __syncthreads();
  for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < B; b += (int64_t)gridDim.x * 4) {
  const bool live = true;
  int c = 0;
  if (live) {
    wgs[wave][lane] = t.WGu[b * 64 + lane];  // pair-permuted wp*g_u
    pl[wave][lane] = t.Pu[b * 64 + lane];
    c = lane < NP ? cnt[b * NP + lane] : 0;
    if constexpr (DEEP) {
      const int64_t uid = dp.ids[b];  // out of range: flagged by the tables' gather
      g0l[wave][lane] = (lane < mf && uid >= 0 && uid < num_users) ? dp.gmf_user[uid * mf + lane] : 0.f;
    }
  }
  // inclusive scan of the segment counts over the lanes
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (live) {
    if (lane == 0) pref[wave][0] = 0;
    if (lane < NP) pref[wave][lane + 1] = incl;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this wave's LDS writes, then its reads
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int n = hnm_readlane_i(incl, 63);
  const bool over = __ballot(c > capp) != 0;
  // fewer than K candidates: the row's bound came from another item shard (short_ok: the
  // merge across shards completes the list) or the threshold is unusable -> fallback
  if (flag[b] || over || (n < K && !short_ok)) {
    if (lane == 0) {
      ovf_rows[atomicAdd(ovf_cnt, 1)] = (int32_t)b;
      if (stats) {
        atomicAdd(&stats[2], 1ull);
        if (b == 0) atomicAdd(&stats[0], (unsigned long long)B);
      }
    }
    continue;
  }
  const float bpv = bp[0];
  WaveTopK<1> L;
  L.init();
  const int32_t* rowbuf = buf + b * (int64_t)NP * capp;
  const float* rowd = bufd + b * (int64_t)NP * capp;
  // candidate g's slot in the row's segments (g < n): segment = last p with pref[p] <= g
  auto slot = [&](int g) {
    int lo = 0, hi = NP;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pref[wave][mid] <= g) lo = mid;
      else hi = mid;
    }
    return (int64_t)lo * capp + (g - pref[wave][lo]);
  };
  auto cand = [&](int g) { return g < n ? rowbuf[slot(g)] : 0; };
  // exact fp32 score of lane j's candidate (both halves of the wave), offered to the top-K
  auto score_deep = [&](int item, bool ok) {
    float q[KS];
    const float* qrow = t.Qi + (int64_t)item * 64 + h * KS;
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
      const float4 v = *reinterpret_cast<const float4*>(qrow + 4 * s4);
      q[4 * s4] = v.x; q[4 * s4 + 1] = v.y; q[4 * s4 + 2] = v.z; q[4 * s4 + 3] = v.w;
    }
    f32x16 acc = {};
    typedef __attribute__((address_space(3))) const float* lds_ptr;
#pragma unroll
    for (int s = 0; s < KS; s += 4) {
      float w[4], pv[4];
      asm volatile("ds_read_b32 %0, %8\n\tds_read_b32 %1, %9\n\tds_read_b32 %2, %10\n\t"
                   "ds_read_b32 %3, %11\n\tds_read_b32 %4, %12\n\tds_read_b32 %5, %13\n\t"
                   "ds_read_b32 %6, %14\n\tds_read_b32 %7, %15\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]),
                     "=&v"(pv[0]), "=&v"(pv[1]), "=&v"(pv[2]), "=&v"(pv[3])
                   : "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[s * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 1) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 2) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 3) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 1]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 2]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 3]));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = mfma32x32x2(w[e], fmaxf(pv[e] + q[s + e], 0.f), acc);
    }
    // layer 3: register s of half h is unit 2s + h, its relu(acc + b2) the k = 2s + h operand
    f32x16 a3 = {};
#pragma unroll
    for (int s = 0; s < 16; ++s)
      a3 = mfma32x32x2(w3l[s * 64 + lane], fmaxf(acc[s] + b2l[2 * s + h], 0.f), a3);
    float sc = 0.f;
    if (h == 0 && ok) {
      const float* grow = dp.gmf_item + (int64_t)item * mf;
      for (int j4 = 0; j4 < mf; j4 += 4) {
        const float4 gv = *reinterpret_cast<const float4*>(grow + j4);
        sc = fmaf(wpl[j4], g0l[wave][j4] * gv.x, sc);
        sc = fmaf(wpl[j4 + 1], g0l[wave][j4 + 1] * gv.y, sc);
        sc = fmaf(wpl[j4 + 2], g0l[wave][j4 + 2] * gv.z, sc);
        sc = fmaf(wpl[j4 + 3], g0l[wave][j4 + 3] * gv.w, sc);
      }
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m < dp.h3) sc = fmaf(wpl[mf + m], fmaxf(a3[m] + b3l[m], 0.f), sc);
    }
    L.offer(sc + bp[0], item, ok && h == 0, K);
  };
  auto score_item = [&](int item, bool ok) {
    if constexpr (DEEP) {
      score_deep(item, ok);
      return;
    }
    // GMF: fma chain in the f32 MFMA's order (k = 2s, then 2s + 1) over all 64 k (zero
    // beyond mf, as the fp32 kernel's padded operands); loads in two batches of 8 float4
    // issued together (a runtime-bounded loop would wait on each load)
    float gm = 0.f;
    const float* grow = t.G + (int64_t)item * t.ldg;
    const int glast = (int)t.ldg - 4;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float4 gv[8];
#pragma unroll
      for (int q4 = 0; q4 < 8; ++q4)
        gv[q4] = *reinterpret_cast<const float4*>(grow + std::min(4 * (8 * half + q4), glast));
#pragma unroll
      for (int q4 = 0; q4 < 8; ++q4) {
        const int c4 = 8 * half + q4;
        const bool in = 4 * c4 < mf;
        // pair-permuted: wgs[2c4], wgs[2c4+1] = k 4c4, 4c4+2; wgs[32+2c4], [32+2c4+1] = 4c4+1, 4c4+3
        const float2 wv = *reinterpret_cast<const float2*>(&wgs[wave][2 * c4]);
        const float2 wv1 = *reinterpret_cast<const float2*>(&wgs[wave][KS + 2 * c4]);
        gm = fmaf(wv1.x, in ? gv[q4].y : 0.f, fmaf(wv.x, in ? gv[q4].x : 0.f, gm));
        gm = fmaf(wv1.y, in ? gv[q4].w : 0.f, fmaf(wv.y, in ? gv[q4].z : 0.f, gm));
      }
    }
    float q[KS];
    const float* qrow = t.Qi + (int64_t)item * 64 + h * KS;
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
      const float4 v = *reinterpret_cast<const float4*>(qrow + 4 * s4);
      q[4 * s4] = v.x; q[4 * s4 + 1] = v.y; q[4 * s4 + 2] = v.z; q[4 * s4 + 3] = v.w;
    }
    f32x16 acc;
    float wmr[16];
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {  // rows mfma32_row(4 r4 + e, h) = 8 r4 + 4 h + e
      const float4 bb = *reinterpret_cast<const float4*>(&b2l[8 * r4 + 4 * h]);
      const float4 ww = *reinterpret_cast<const float4*>(&wml[8 * r4 + 4 * h]);
      acc[4 * r4] = bb.x; acc[4 * r4 + 1] = bb.y; acc[4 * r4 + 2] = bb.z; acc[4 * r4 + 3] = bb.w;
      wmr[4 * r4] = ww.x; wmr[4 * r4 + 1] = ww.y; wmr[4 * r4 + 2] = ww.z; wmr[4 * r4 + 3] = ww.w;
    }
    typedef __attribute__((address_space(3))) const float* lds_ptr;
    // four k steps' operands per LDS round trip
#pragma unroll
    for (int s = 0; s < KS; s += 4) {
      float w[4], pv[4];
      asm volatile("ds_read_b32 %0, %8\n\tds_read_b32 %1, %9\n\tds_read_b32 %2, %10\n\t"
                   "ds_read_b32 %3, %11\n\tds_read_b32 %4, %12\n\tds_read_b32 %5, %13\n\t"
                   "ds_read_b32 %6, %14\n\tds_read_b32 %7, %15\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]),
                     "=&v"(pv[0]), "=&v"(pv[1]), "=&v"(pv[2]), "=&v"(pv[3])
                   : "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[s * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 1) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 2) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&w2l[(s + 3) * 64 + lane]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 1]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 2]),
                     "v"((unsigned)(uintptr_t)(lds_ptr)&pl[wave][h * KS + s + 3]));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = mfma32x32x2(w[e], fmaxf(pv[e] + q[s + e], 0.f), acc);
    }
    float m4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 16; ++r) m4[r & 3] = fmaf(fmaxf(acc[r], 0.f), wmr[r], m4[r & 3]);
    const float mlp = (m4[0] + m4[1]) + (m4[2] + m4[3]);
    const float tot = hnm_sum_halves(mlp + (h == 0 ? gm : 0.f));
    const float score = tot + bpv;
    L.offer(score, item, ok && h == 0, K);
  };
  // Best first (round 5), rows of more than RESCORE_BEST_FIRST candidates: the 64 with the best
  // scan test values are scored first; their K-th exact score thr lower-bounds the row's K-th,
  // so a remaining candidate is scored only if it would have passed the scan against thr -- its
  // test value against the threshold tau2 that cert_tau_kernel derives from thr, with twice that
  // kernel's guard (the extra rounding of d + tau).  Rows whose scan bound came from a poor
  // sample (user-specific best items: ~300 candidates a row) drop to about what a perfect
  // sample would leave (tools/ncf_bound_limit_probe.py).  Shorter rows: every candidate, in
  // order.  Candidates are staged 32 at a time (one scoring site: the kernel stays at 168 VGPRs).
  int* st = stg[wave];
  int ns = 0, nscored = 0;
  float v63 = 0.f, t2 = 0.f;
  int i63 = 0;
  bool usable = false;
  const float tb = tau[b];
  const bool bf = n > RESCORE_BEST_FIRST;
  int ti = HNM_SENTINEL_IDX;
  if (bf) {
    float tv = -__builtin_inff();
    for (int c0 = 0; c0 < n; c0 += 64) {  // the 64 best (test value desc, ordinal asc)
      const int g = c0 + lane;
      const float d = g < n ? rowd[slot(g)] : -__builtin_inff();
      float v1 = d != d ? __builtin_inff() : d;  // a NaN test value is scored first
      int i1 = g < n ? g : HNM_SENTINEL_IDX;
      // only a chunk holding an entry above the current 64th can change the 64 best
      const float c63 = hnm_readlane_f(tv, 63);
      const int c63i = hnm_readlane_i(ti, 63);
      if (__ballot(hnm_better(v1, i1, c63, c63i))) hnm_sort128(tv, ti, v1, i1);
    }
    v63 = hnm_readlane_f(tv, 63);
    i63 = hnm_readlane_i(ti, 63);
  }
  for (int phase = bf ? 0 : 2; phase < (bf ? 2 : 3); ++phase) {  // bf: 0, 1; else 2
    if (phase == 0) {  // the 64 best, already in ti (lane = rank)
      st[lane] = ti;
      ns = 64;
    }
    if (phase == 1) {
      const float thr = L.thr_v;  // 64 >= K items scored: a valid K-th
      const float unit = prm->unit;
      const float scale = unit * (prm->c0 + Au[b] + prm->Bmax + Cu[b] * prm->Dmax);
      t2 = (thr - bpv) * unit - Eu[b] - 2.f * 3.814697265625e-06f * scale;  // 2 x 2^-18
      t2 -= fabsf(t2) * 1.9073486328125e-06f;                                 // 2 x 2^-20
      usable = __builtin_isfinite(t2);
    }
    for (int c0 = 0; c0 < (phase == 0 ? 1 : n); c0 += 64) {
      if (phase != 0) {
        const int g = c0 + lane;
        bool keep = g < n;
        if (keep && phase == 1) {
          const float d = rowd[slot(g)];
          const bool top = !hnm_better(v63, i63, d != d ? __builtin_inff() : d, g);
          keep = !top && (!usable || !(d + tb < t2));
        }
        const uint64_t m = __ballot(keep);
        if (keep) st[ns + __popcll(m & ((1ull << lane) - 1))] = g;
        ns += __popcll(m);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const bool last = phase == 0 || c0 + 64 >= n;
      while (ns >= 32 || (last && ns > 0)) {
        const int nv = ns < 32 ? ns : 32;
        score_item(cand(st[j < nv ? j : 0]), j < nv);
        nscored += nv;
        const int rest = ns - nv;
        const int mv = lane < rest ? st[32 + lane] : 0;
        __builtin_amdgcn_wave_barrier();
        if (lane < rest) st[lane] = mv;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ns = rest;
      }
    }
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[1], (unsigned long long)nscored);
    if (b == 0) atomicAdd(&stats[0], (unsigned long long)B);
  }
  L.store(ov ? ov + b * K : nullptr, oi + b * K, K);
  }
}

// Deep towers: the candidates the main scan would append for the proxy rows (whose every item the
// proxy pass scored: pd = approx - e_i), approx + e_i >= tau with tau ~ kv - 2 Eu (cert_tau_kernel)
// -- where the worst-case bound through two absolute-value layers is wider than the rows' score
// spread (init-like weights) the certified scan cannot prune and the call takes the exact kernels
// instead.  An unusable bound counts every item.
__global__ __launch_bounds__(256) void cert_predict_kernel(const float* __restrict__ pd, int64_t I,
                                                           int K, const float* __restrict__ kthv,
                                                           const float* __restrict__ Eu,
                                                           const float* __restrict__ Bs,
                                                           const float* __restrict__ Cs,
                                                           const float* __restrict__ Di,
                                                           const CertParams* __restrict__ prm,
                                                           unsigned long long* __restrict__ cnt) {
  const int r = blockIdx.y;
  const float thr = kthv[(int64_t)r * K + K - 1] - 2.f * Eu[r], cs = Cs[r];
  const bool bad = prm->bad || !__builtin_isfinite(thr);
  unsigned n = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < I; i += (int64_t)gridDim.x * 256)
    n += bad || !(pd[(int64_t)r * I + i] + 2.f * fmaf(cs, Di[i], Bs[i]) < thr);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(cnt, (unsigned long long)n);
}

// scaled -> real units, for the diagnostics entry point
__global__ void cert_unscale_kernel(float* __restrict__ a, float* __restrict__ e, int64_t lda,
                                    int64_t B, int64_t I, const CertParams* __restrict__ prm) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= B * I) return;
  const int64_t o = (x / I) * lda + x % I;
  a[o] /= prm->unit;
  e[o] /= prm->unit;
}

struct CertWs {
  CertParams* prm;
  float *Au, *Cu, *Bi, *Di, *tau, *Eu, *b2s, *kthv, *lb, *pdense, *cdense, *part;
  float *Bs, *Cs;  // Bi, Cu in the scan's test units (cert_convert_kernel)
  int32_t* sidx;  // champion items
  int32_t* sloo;  // [CERT_PROXY_USERS, nch] leave-one-out champions (gate)
  int32_t* sidx2; // [ns] strided sample items
  float* sdense;  // [B, ns] strided sample values (gated)
  float* kth2;    // [B, K] its K best
  int* gate;
  unsigned long long* gcnt;  // [4] gate counters
  int64_t* kthi;
  int *cnt, *flag;
  int32_t *buf, *ovf_cnt, *ovf_rows;
  float* bufd;  // the appended candidates' test values
  _Float16 *P16, *WG16, *Q16, *G16, *W2h, *wmh;
  _Float16 *W3h, *wph;  // deep towers: layer 3 and the prediction weights (f16, scaled)
  float *b3s, *u;       // deep towers: layer-3 bias (scaled); |wp3|^T |W3| (bound statistics)
  float* cv;
  int32_t* ci;
};

// ~wg workgroups per CU (the scan variant's occupancy), NP a multiple of 8 (XCD-aware),
// <= CERT_MAX_NP
Partition scan_partition(int64_t I, int64_t ublocks, int num_cus, int wg) {
  int64_t np = std::max<int64_t>(1, (int64_t)wg * num_cus / std::max<int64_t>(ublocks, 1));
  np = std::min<int64_t>(np, std::max<int64_t>(1, hnm_cdiv(I, 4 * TILE)));
  np = std::min<int64_t>(np, CERT_MAX_NP);
  if (np >= 8) np = np / 8 * 8;
  const int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), TILE) * TILE;
  return {(int)hnm_cdiv(I, ipp), ipp};
}

struct CertShape {
  int64_t nch, gsz;  // champion sample: nch groups of gsz items
  int64_t ns;        // strided sample: items of tiles 0, S, 2S, ... (CERT_STRIDE)
  Partition part;    // of the main scan
  int capp;          // candidate slots per (row, partition)
};

CertShape cert_shape(int64_t B, int64_t I, int K, int num_cus, int wg) {
  CertShape sh;
  sh.gsz = std::max<int64_t>(CERT_GROUP_MIN, hnm_cdiv(I, CERT_CHAMPIONS));
  sh.nch = hnm_cdiv(I, sh.gsz);
  const int64_t nst = hnm_cdiv(hnm_cdiv(I, TILE), CERT_STRIDE);  // sampled tiles
  sh.ns = (nst - 1) * TILE + std::min<int64_t>(TILE, I - (nst - 1) * CERT_STRIDE * TILE);
  sh.part = scan_partition(I, hnm_cdiv(B, 128), num_cus, wg);
  // a row's candidates: items within the bound's margin of the champion sample's K-th --
  // at worst (no shared best items) the K-th of a 1/gsz sample, ~K * gsz items; each
  // partition gets 4x its even share of 8x that, >= 64 slots (overflow: fallback row).
  // Round 5: 8x (was 2x) -- with the best-first re-scoring a long candidate list costs the
  // scan's appends and one sort, while an overflowing row costs an exact scan of the whole
  // catalogue ("norms" trained-like weights: 44 fallback rows -> 0, 3.50 -> 3.24 ms a step;
  // init weights unchanged: profiles/r6k_ncf_capp_ab.txt)
  const int64_t total = std::min<int64_t>(8192, std::max<int64_t>(512, 8 * (int64_t)K * sh.gsz));
  sh.capp = (int)std::max<int64_t>(64, std::min<int64_t>(total, hnm_cdiv(4 * total, sh.part.np)));
  return sh;
}

// carve (or size, when base == nullptr) the scratch region
// strided: carve the gated strided sample's scratch (sloo, sidx2, sdense [B, ns], kth2) -- only
// for calls that may run it (HNM_OPT_STRIDED; ADVICE r5: ~0.2 GB a B = 4,096 call otherwise)
size_t cert_carve(char* base, int64_t B, int64_t I, int K, int num_cus, int wg, bool strided,
                  CertWs* w) {
  const CertShape sh = cert_shape(B, I, K, num_cus, wg);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += hnm_align(bytes);
    return p;
  };
  CertWs x;
  x.prm = (CertParams*)take(sizeof(CertParams));
  x.Au = (float*)take(B * 4);
  x.Cu = (float*)take(B * 4);
  x.Cs = (float*)take(B * 4);
  x.Bs = (float*)take(I * 4);
  x.part = (float*)take(4 * 4 * (1024 + 256));
  x.Bi = (float*)take(I * 4);
  x.Di = (float*)take(I * 4);
  x.tau = (float*)take(B * 4);
  x.Eu = (float*)take(B * 4);
  x.b2s = (float*)take(32 * 4);
  x.kthv = (float*)take((size_t)B * K * 4);
  x.lb = (float*)take((size_t)B * 4);
  x.pdense = (float*)take((size_t)CERT_PROXY_USERS * I * 4);
  x.cdense = (float*)take((size_t)B * sh.nch * 4);
  x.sidx = (int32_t*)take((size_t)sh.nch * 4);
  x.sloo = strided ? (int32_t*)take((size_t)CERT_PROXY_USERS * sh.nch * 4) : nullptr;
  x.sidx2 = strided ? (int32_t*)take((size_t)sh.ns * 4) : nullptr;
  x.sdense = strided ? (float*)take((size_t)B * sh.ns * 4) : nullptr;
  x.kth2 = strided ? (float*)take((size_t)B * K * 4) : nullptr;
  x.gate = (int*)take(4);
  x.gcnt = (unsigned long long*)take(4 * 8);
  x.kthi = (int64_t*)take((size_t)B * K * 8);
  x.cnt = (int*)take((size_t)B * sh.part.np * 4);
  x.flag = (int*)take(B * 4);
  x.ovf_cnt = (int32_t*)take(256);
  x.ovf_rows = (int32_t*)take(B * 4);
  x.buf = (int32_t*)take((size_t)B * sh.part.np * sh.capp * 4);
  x.bufd = (float*)take((size_t)B * sh.part.np * sh.capp * 4);
  x.P16 = (_Float16*)take((size_t)B * 64 * 2);
  x.WG16 = (_Float16*)take((size_t)B * 64 * 2);
  x.Q16 = (_Float16*)take((size_t)I * 64 * 2);
  x.G16 = (_Float16*)take((size_t)I * 64 * 2);
  x.W2h = (_Float16*)take(32 * 64 * 2);
  x.wmh = (_Float16*)take(32 * 2);
  x.W3h = (_Float16*)take(16 * 32 * 2);
  x.wph = (_Float16*)take(16 * 2);
  x.b3s = (float*)take(16 * 4);
  x.u = (float*)take(32 * 4);
  const size_t lb = ncf_list_bytes(B, I, K, num_cus);
  x.cv = (float*)take(lb);
  x.ci = (int32_t*)take(lb);
  if (w) *w = x;
  return off;
}

hnm_status cert_prepare(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                        const CertWs& x, const CertDeep* dp) {
  const int64_t I = w->num_items;
  const int ib = (int)std::min<int64_t>(1024, hnm_cdiv(I, 4));
  const int ub = (int)std::min<int64_t>(256, hnm_cdiv(B, 4));
  // the weights behind layer 2's outputs: wm (two-layer tower) or u = |wp3|^T |W3| (deep)
  const float* wm = w->wp + w->mf;
  const CertDeep dv = dp ? *dp : CertDeep{};
  if (dp) {
    hipLaunchKernelGGL(cert_deep_u_kernel, dim3(1), dim3(64), 0, ctx->stream, dv, w->h2, x.u);
    HNM_LAUNCH_CHECK();
    wm = x.u;
  }
  hipLaunchKernelGGL(cert_stats_kernel, dim3(ib + ub), dim3(256), 0, ctx->stream, t, B, I, w->mf,
                     w->w2, w->h1, w->h2, wm, x.prm, x.Au, x.Cu, x.Bi, x.Di, x.part, ib, ub);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(cert_scales_kernel, dim3(1), dim3(256), 0, ctx->stream, w->w2, w->h1, w->h2,
                     w->b2, wm, w->bp, x.prm, x.part, ib, ub, x.ovf_cnt, dv);
  HNM_LAUNCH_CHECK();
  const int cb = (int)std::min<int64_t>(2048, std::max<int64_t>(1, hnm_cdiv(I * 16, 256)));
  hipLaunchKernelGGL(cert_convert_kernel, dim3(cb), dim3(256), 0, ctx->stream, t, B, I, w->mf,
                     x.prm, x.P16, x.WG16, x.Q16, x.G16, w->w2, w->h1, w->h2, w->b2, wm, x.W2h,
                     x.wmh, x.b2s, x.Bi, x.Cu, x.Bs, x.Cs, dv, x.W3h, x.wph, x.b3s);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

template <int MODE>
void launch_scan(hnm_ctx* ctx, dim3 grid, const ScanArgs& a) {
  if (a.W3h)
    hipLaunchKernelGGL((ncf16_scan_kernel<MODE, true>), grid, dim3(256), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL((ncf16_scan_kernel<MODE, false>), grid, dim3(256), 0, ctx->stream, a);
}

ScanArgs scan_args(const CertWs& x, int64_t B, bool deep) {
  ScanArgs a{};
  a.W3h = deep ? x.W3h : nullptr;  // selects the deep scan (launch_scan)
  a.wph = x.wph;
  a.b3s = x.b3s;
  a.P16 = x.P16;
  a.WG16 = x.WG16;
  a.Q16 = x.Q16;
  a.G16 = x.G16;
  a.W2h = x.W2h;
  a.wmh = x.wmh;
  a.b2s = x.b2s;
  a.Bi = x.Bs;
  a.Di = x.Di;
  a.Cu = x.Cs;
  a.Eu = x.Eu;
  a.prm = x.prm;
  a.B = B;
  a.sidx = nullptr;
  a.upw = 32;
  return a;
}

}  // namespace

bool ncf_cert_eligible(const hnm_ncf_weights* w, int K) {
  // the scan addresses Q16 / G16 by 32-bit element offsets (item * 64 < 2^31: 33.5M items)
  return w->h1 <= 64 && w->mf <= 64 && w->h2 <= 32 && K <= 64 &&
         w->num_items >= CERT_MIN_ITEMS && w->num_items >= 64 * (int64_t)K &&
         w->num_items * 64 < ((int64_t)1 << 31);
}

int ncf_cert_wg(const hnm_ctx* ctx) {
  (void)ctx;
  return CERT_WG_PER_CU;
}

size_t ncf_cert_bytes(int64_t B, int64_t I, int K, int num_cus, int wg, bool strided) {
  return cert_carve(nullptr, B, I, K, num_cus, wg, strided, nullptr);
}

// Phase 1: per-call bound statistics and f16 copies, the champion sample, and every row's
// certified lower bound of the exact K-th best score (real units) into lb[B].
hnm_status ncf_cert_begin(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                          const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                          bool strided, float* lb, float* lists, const CertDeep* dp) {
  const int64_t I = w->num_items;
  const int wg = ncf_cert_wg(ctx);
  const CertShape sh = cert_shape(B, I, K, ctx->num_cus, wg);
  CertWs x;
  cert_carve((char*)scratch, B, I, K, ctx->num_cus, wg, strided, &x);
  hnm_status st = cert_prepare(ctx, w, t, B, x, dp);
  if (st) return st;
  const int64_t ublocks = hnm_cdiv(B, 128);
  const bool deep = dp != nullptr;
  // champion sample: the first rows' approx - e over all items -> the best item of each of
  // nch groups -> every row's K-th best approx - e over those items -> L (a lower bound of
  // the exact K-th for any item subset; this one tends to hold the rows' best items)
  const int64_t bp = std::min<int64_t>(CERT_PROXY_USERS, B);
  ScanArgs a = scan_args(x, bp, deep);
  a.I = I;
  a.dense = x.pdense;
  a.ldo = I;
  const int64_t np = std::min<int64_t>(3 * (int64_t)ctx->num_cus, hnm_cdiv(I, 4 * TILE));
  a.ipp = hnm_cdiv(hnm_cdiv(I, np), TILE) * TILE;
  a.NP = (int)hnm_cdiv(I, a.ipp);
  a.upw = 2;  // the <= 8 proxy rows as one user pair per wave (4x shorter per tile than one wave)
  launch_scan<SCAN_SAMPLE>(ctx, dim3((unsigned)a.NP, 1), a);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(cert_champion_kernel, dim3((unsigned)hnm_cdiv(sh.nch, 4)), dim3(256), 0,
                     ctx->stream, x.pdense, I, (int)bp, I, sh.gsz, sh.nch, x.sidx,
                     strided ? x.sloo : nullptr, sh.ns, strided ? x.sidx2 : nullptr,
                     strided ? x.gcnt : nullptr);
  HNM_LAUNCH_CHECK();
  // the gate (8 workgroups, latency-bound: ~22 us) runs on the ctx's side stream beside the
  // champion pass of every row below (independent: both read the proxy rows and the champions);
  // the ctx stream joins before the strided pass reads the gate
  const bool gated = strided && bp >= 4;
  if (gated) {
    HNM_HIP_CHECK(hipEventRecord(ctx->side_in, ctx->stream));
    HNM_HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->side_in, 0));
    hipLaunchKernelGGL(cert_gate_kernel, dim3((unsigned)bp), dim3(1024), 0, ctx->side,
                       x.pdense, I, (int)bp, x.sloo, sh.nch, K, sh.ns, x.Bs, x.Di, x.Cs, x.Au,
                       x.prm, x.gcnt, x.gate, B, ctx->stats_on ? ctx->stats_dev : nullptr);
    HNM_LAUNCH_CHECK();
    HNM_HIP_CHECK(hipEventRecord(ctx->side_out, ctx->side));
  } else if (strided) {
    HNM_HIP_CHECK(hipMemsetAsync(x.gate, 0, 4, ctx->stream));
  }
  ScanArgs c = scan_args(x, B, deep);
  c.I = sh.nch;
  c.sidx = x.sidx;
  c.dense = x.cdense;
  c.ldo = sh.nch;
  // as many partitions as one round of workgroups holds (the main scan's >= 4-tile,
  // multiple-of-8 partitions would leave a third of the slots idle on 2,048 champions)
  const int64_t npc = std::max<int64_t>(1, (int64_t)wg * ctx->num_cus / ublocks);
  c.ipp = hnm_cdiv(hnm_cdiv(sh.nch, npc), TILE) * TILE;
  c.NP = (int)hnm_cdiv(sh.nch, c.ipp);
  launch_scan<SCAN_SAMPLE>(ctx, dim3((unsigned)c.NP, (unsigned)ublocks), c);
  if (gated) HNM_HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->side_out, 0));  // join
  HNM_LAUNCH_CHECK();
  // one-shot call (no bound out, no lists, no strided sample): bound + threshold fused into the
  // K-th launch; ncf_cert_finish then skips cert_tau_kernel (same condition there)
  const bool fuse = lb == nullptr && lists == nullptr && !strided;
  if (fuse)
    return sample_kth_launch(ctx, x.cdense, sh.nch, B, sh.nch, mptr, midx, K, 1, 1, x.sidx, x.kthv,
                             nullptr, NcfBoundTauEpi{x.prm, x.Au, x.Cu, w->bp, x.Eu, x.lb, x.tau,
                                                     x.flag});
  st = hnm_sample_kth(ctx, x.cdense, sh.nch, B, sh.nch, mptr, midx, K, 1, 1, x.sidx, x.kthv);
  if (st) return st;
  // gated strided sample: every row against one tile in CERT_STRIDE (exits when gated off)
  ScanArgs g2 = scan_args(x, B, deep);
  g2.I = sh.ns;
  g2.sidx = x.sidx2;
  g2.dense = x.sdense;
  g2.ldo = sh.ns;
  g2.gate = x.gate;
  const Partition p2 = scan_partition(sh.ns, ublocks, ctx->num_cus, wg);
  g2.ipp = p2.ipp;
  g2.NP = p2.np;
  if (strided) {
    launch_scan<SCAN_SAMPLE>(ctx, dim3((unsigned)p2.np, (unsigned)ublocks), g2);
    HNM_LAUNCH_CHECK();
    st = hnm_sample_kth(ctx, x.sdense, sh.ns, B, sh.ns, mptr, midx, K, 1, 1, x.sidx2, x.kth2, x.gate);
    if (st) return st;
  }
  const int* gp = strided ? x.gate : nullptr;
  hipLaunchKernelGGL(cert_bound_kernel, dim3((unsigned)hnm_cdiv(B, 256)), dim3(256), 0,
                     ctx->stream, x.kthv, x.kth2, gp, K, x.Au, x.prm, w->bp, B, lb ? lb : x.lb,
                     x.Eu);
  HNM_LAUNCH_CHECK();
  if (lists) {
    hipLaunchKernelGGL(cert_bound_lists_kernel, dim3((unsigned)hnm_cdiv(B * K, 256)), dim3(256), 0,
                       ctx->stream, x.kthv, x.kth2, gp, K, x.Eu, x.prm, w->bp, B, lists);
    HNM_LAUNCH_CHECK();
  }
  return HNM_OK;
}

// Phase 2: thresholds from the lower bounds lb (this call's, or the max over item shards),
// the main f16 scan, exact fp32 re-scoring + top-K, the exact fallback for unusable rows.
// short_ok: a row may keep fewer than K candidates (its bound came from another shard).
hnm_status ncf_cert_finish(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                           const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                           bool strided, const float* lb, int short_ok, float* ov, int64_t* oi,
                           const CertDeep* dp, int32_t** ovf_rows, int32_t** ovf_cnt) {
  const int64_t I = w->num_items;
  const int wg = ncf_cert_wg(ctx);
  const CertShape sh = cert_shape(B, I, K, ctx->num_cus, wg);
  CertWs x;
  cert_carve((char*)scratch, B, I, K, ctx->num_cus, wg, strided, &x);
  const int64_t ublocks = hnm_cdiv(B, 128);
  if (lb != nullptr || strided) {  // else tau / flag came with the begin phase's K-th
    hipLaunchKernelGGL(cert_tau_kernel, dim3((unsigned)hnm_cdiv(B, 256)), dim3(256), 0,
                       ctx->stream, lb ? lb : x.lb, x.Au, x.Cu, x.Eu, x.prm, w->bp, B, x.tau,
                       x.flag);
    HNM_LAUNCH_CHECK();
  }
  // main f16 scan: append items with approx + e >= tau_u to per-partition segments
  ScanArgs a = scan_args(x, B, dp != nullptr);
  a.I = I;
  a.mptr = mptr;
  a.midx = midx;
  a.tau = x.tau;
  a.cnt = x.cnt;
  a.buf = x.buf;
  a.segd = x.bufd;
  a.capp = sh.capp;
  a.ipp = sh.part.ipp;
  a.NP = sh.part.np;
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
  launch_scan<SCAN_THRESH>(ctx, dim3((unsigned)sh.part.np, (unsigned)ublocks), a);
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  // exact fp32 re-scoring + top-K of the candidates; unusable rows -> queue
  const int64_t rgrid = std::min<int64_t>(hnm_cdiv(B, 4), (int64_t)RESCORE_PERSIST * ctx->num_cus);
  const CertDeep dv = dp ? *dp : CertDeep{};
#define HNM_RESCORE(DEEPV)                                                                       \
  hipLaunchKernelGGL(ncf_rescore_kernel<DEEPV>, dim3((unsigned)rgrid), dim3(256), 0, ctx->stream, \
                     t, w->mf, w->w2, w->h1, w->h2, w->b2, w->wp + w->mf, w->bp, B, x.flag,       \
                     x.cnt, x.buf, x.bufd, x.tau, x.Eu, x.Au, x.Cu, x.prm, sh.part.np, sh.capp,  \
                     K, short_ok, ov, oi, x.ovf_rows, x.ovf_cnt,                                 \
                     ctx->stats_on ? ctx->stats_dev : nullptr, dv, w->num_users);
  if (dp) {
    HNM_RESCORE(true)
  } else {
    HNM_RESCORE(false)
  }
#undef HNM_RESCORE
  HNM_LAUNCH_CHECK();
  if (dp) {  // the deep tower's exact scan of the queued rows is the caller's (ncf_deep.hip)
    *ovf_rows = x.ovf_rows;
    *ovf_cnt = x.ovf_cnt;
    return HNM_OK;
  }
  // exact fp32 scan over all items for the queued rows (device-side row list)
  return ncf_list_rows(ctx, w, t, B, mptr, midx, K, x.ovf_rows, x.ovf_cnt, x.cv, x.ci, ov, oi);
}

hnm_status ncf_cert_topk(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                         const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                         bool strided, float* ov, int64_t* oi) {
  hnm_status st = ncf_cert_begin(ctx, w, t, B, mptr, midx, K, scratch, strided, nullptr);
  if (st) return st;
  return ncf_cert_finish(ctx, w, t, B, mptr, midx, K, scratch, strided, nullptr, 0, ov, oi);
}

hnm_status ncf_deep_cert_topk(hnm_ctx* ctx, const hnm_ncf_weights* w, const CertDeep& dp,
                              const NcfTabs& t, int64_t B, const int64_t* mptr,
                              const int32_t* midx, int K, void* scratch, float* ov, int64_t* oi,
                              int32_t** ovf_rows, int32_t** ovf_cnt, bool* pruned) {
  hnm_status st = ncf_cert_begin(ctx, w, t, B, mptr, midx, K, scratch, false, nullptr, nullptr, &dp);
  if (st) return st;
  // can the bound prune?  the proxy rows' predicted candidates (one read-back)
  const int64_t I = w->num_items;
  const CertShape sh = cert_shape(B, I, K, ctx->num_cus, ncf_cert_wg(ctx));
  CertWs x;
  cert_carve((char*)scratch, B, I, K, ctx->num_cus, ncf_cert_wg(ctx), false, &x);
  const int np_rows = (int)std::min<int64_t>(CERT_PROXY_USERS, B);
  HNM_HIP_CHECK(hipMemsetAsync(x.gcnt, 0, 8, ctx->stream));
  hipLaunchKernelGGL(cert_predict_kernel,
                     dim3((unsigned)std::min<int64_t>(64, hnm_cdiv(I, 256)), (unsigned)np_rows),
                     dim3(256), 0, ctx->stream, x.pdense, I, K, x.kthv, x.Eu, x.Bs, x.Cs, x.Di,
                     x.prm, x.gcnt);
  HNM_LAUNCH_CHECK();
  unsigned long long pc = 0;
  HNM_HIP_CHECK(hipMemcpyAsync(&pc, x.gcnt, 8, hipMemcpyDeviceToHost, ctx->stream));
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  // prune when a row would re-score at most 1/16 of the catalogue (re-scoring a candidate costs
  // several pairs of the exact tiled scan) and half its segments' capacity
  const int64_t limit = std::min<int64_t>(I / 16, (int64_t)sh.part.np * sh.capp / 2);
  *pruned = (int64_t)(pc / (unsigned long long)np_rows) <= limit;
  if (!*pruned) return HNM_OK;
  return ncf_cert_finish(ctx, w, t, B, mptr, midx, K, scratch, false, nullptr, 0, ov, oi, &dp,
                         ovf_rows, ovf_cnt);
}

hnm_status ncf_cert_debug(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                          void* scratch, float* approx, int64_t lda, float* bound,
                          const CertDeep* dp) {
  const int64_t I = w->num_items;
  CertWs x;
  cert_carve((char*)scratch, B, I, 1, ctx->num_cus, ncf_cert_wg(ctx), false, &x);
  hnm_status st = cert_prepare(ctx, w, t, B, x, dp);
  if (st) return st;
  hipLaunchKernelGGL(cert_bound_kernel, dim3((unsigned)hnm_cdiv(B, 256)), dim3(256), 0, ctx->stream,
                     nullptr, nullptr, nullptr, 1, x.Au, x.prm, w->bp, B, nullptr, x.Eu);
  HNM_LAUNCH_CHECK();
  ScanArgs a = scan_args(x, B, dp != nullptr);
  a.I = I;
  a.dense = approx;
  a.dense2 = bound;
  a.ldo = lda;
  const int64_t ublocks = hnm_cdiv(B, 128);
  Partition part = choose_partition(I, ublocks, ctx->num_cus);
  a.ipp = part.ipp;
  a.NP = part.np;
  launch_scan<SCAN_DEBUG>(ctx, dim3((unsigned)part.np, (unsigned)ublocks), a);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(cert_unscale_kernel, dim3((unsigned)hnm_cdiv(B * I, 256)), dim3(256), 0,
                     ctx->stream, approx, bound, lda, B, I, x.prm);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
