// Dot-product top-K (LightGCN lightgcn.py:332-358 over :188-204, MatrixFactorization
// matrix_factorization.py:220-246 over :108-131) with a CERTIFIED f16 pre-filter and
// exact fp32 re-scoring -- the dot-model counterpart of ncf_cert.hip.
//
//   exact score (dot_score_kernel):  s(u, i) = (fma-chain_k u_k i_k + ub_u) + ib_i
//
// The all-items scan multiplies f16 copies of the user rows and item table on
// v_mfma_f32_32x32x16_f16 (16x the fp32 MFMA rate) and only prunes; every returned score
// is recomputed by the fp32 fma chain the fp32 MFMA is bitwise equal to
// (tools/mfma_semantics_probe.hip (a)), so results are bit-identical to the fp32 scan.
//
// Bound: with u~ = rn16(u su), i~ = rn16(i si) (powers of two, |u su|, |i si| <= 1, f16
// denormals kept), |u~ i~ - s u i| <= 2.01 u16 s |u_k||i_k| + subnormal terms, the f16
// MFMA's fp32 accumulation and the exact path's fp32 chain add <= (DP + 18) 2^-24 of
// sum |u_k i_k| <= ||u|| ||i|| (Cauchy-Schwarz), the bias adds 2^-23 of |ub| + |ib| + |dot|.
// Per user:  E_u = 3 u16 ||u|| max_i ||i|| + 2^-22 (|ub_u| + max|ib|) + abs_slack,
// |approx - exact| <= E_u for every item (tests/test_gpu_prefilter.py checks it).
// Pruning as in ncf_cert.hip: tau_u = (K-th best approx over a strided sample) - 2 E_u;
// the scan appends items with approx >= tau_u; exact re-scoring + top-K of the
// candidates; rows that overflow / have < K candidates / an unusable bound take the
// exact LIST scan (device-side row list).
//
// Grid: blockIdx.x = item partition (NP a multiple of 8), blockIdx.y = 128-user block,
// so the hardware's round-robin workgroup -> XCD placement pins partition p to XCD p % 8:
// each XCD's L2 holds only its partitions' item tiles (XCD-aware mapping).
#include <algorithm>

#include "dot_internal.h"
#include "hnm_device.h"
#include "sample_kth.h"

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int64_t DCERT_MIN_ITEMS = 8192;
// Sample density (round 3, profiles/r3g_dot_sample_ab.txt; MF d=64, B=4096): stride 8 -> 111
// candidates a row, scan 0.105 ms; stride 4 -> 55, 0.096 ms; stride 2 -> 28, 0.087 ms -- the
// step is the same for 4 and 2 (the sample pass grows by what the scan saves), 10 % shorter
// than stride 8 once the sample pass's max runs as one v_max3 per row and sub-tile pair.
// Round 6, with the two-block main scan (profiles/r10p_dot_sample_stride_ab.txt, MF step, three
// interleaved rounds): stride 2 0.1767-0.1825 ms (27.6 candidates a row), 3 0.1755-0.1780 (40.7),
// 4 0.1776-0.1801 (55.3): stride 3.
constexpr int64_t DCERT_SAMPLE = 35181;  // sampled items: stride max(DCERT_MIN_STRIDE, I / this)
#ifndef DCERT_MIN_STRIDE_AB  // A/B builds only (tools/build_variant.sh)
#define DCERT_MIN_STRIDE_AB 3
#endif
constexpr int64_t DCERT_MIN_STRIDE = DCERT_MIN_STRIDE_AB;
constexpr float DCERT_RHO = 0.00146484375f;  // 3 u16 = 3 * 2^-11
constexpr int DCERT_MAX_NP = 64;
constexpr int DCERT_USER_BLOCKS = 2048;  // dcert_stats_kernel user blocks (4 waves x 4 rows), at most

// user blocks of 32 per scan wave (each item fragment feeds NB MFMAs).  Round 4 A/B (MF d=64
// step / THRESH scan, one box): NB = 1 0.1827 / 0.0835 ms, NB = 2 at 2 workgroups per CU
// 0.1845 / 0.0866, the sample pass at NB = 2 0.2011 (its running max then costs 3 instructions
// a value); round 3's 64-bit tile addressing 0.1872 / 0.0886.  Round 6: the THRESH scan at
// NB = 2 now fits three workgroups per CU in 168 VGPRs without spills where DP = 64 and no
// filter is applied: half the LDS fragment reads and half the L2 tile traffic per MFMA, MF scan
// 0.0853-0.0877 -> 0.0773-0.0805 ms, step 0.181-0.186 -> 0.172-0.178 ms
// (profiles/r10k_dot_nb2_ab.txt); the masked and DP = 128 variants spill at NB = 2 (filtered
// LightGCN -3 %) and the sample pass at NB = 2 is slower (44 vs 39.5 us): both stay at NB = 1.
enum { DSCAN_DENSE = 0, DSCAN_THRESH = 1, DSCAN_SAMPLE = 2 };  // scan modes (below)
// scan occupancy (workgroups per CU): three at NB = 1 and NB = 2 (168 VGPRs).  Round 4 A/B (MF
// step / THRESH scan): 3 workgroups per CU 0.1805 / 0.0832 ms, 2 per CU 0.1911 / 0.0953; 64-item
// tiles 0.1804 / 0.0859; 256-item tiles at 2 per CU 0.1899 / 0.0923
__host__ __device__ constexpr int dcert_wg_per_cu(int NB) { return 3; }
// the main scan's NB for a call (host): unfiltered calls at DP = 64
static inline int dscan_thresh_nb(int d, bool masked) { return d <= 64 && !masked ? 2 : 1; }

enum { DM_U, DM_I, DM_NI, DM_IB, DM_N };

struct DParams {
  unsigned mx[DM_N];  // float bits of non-negative maxima (reduced from per-block partials)
  float su, si, s;    // f16 scales; s = su * si is the scan's score unit
  float absb;         // subnormal slack, scaled units
  int bad;
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
__device__ __forceinline__ float pow2_below_inv(float m) {  // 2^-e with m < 2^e (m > 0)
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, -e);
}

struct DotCertWs {
  DParams* prm;
  float *Nu, *Ni, *ubr, *ibs, *tau, *E, *kthv, *lb, *sdense, *part;
  int64_t* kthi;
  int *cnt, *flag;
  int32_t *buf, *ovf_cnt, *ovf_rows;
  _Float16 *U16, *I16;
  float* cv;
  int32_t* ci;
};

struct DotCertShape {
  int DP;
  int64_t stride, Ns;
  Partition spart;  // of the sample pass (NB = 1)
  Partition part;   // of the main scan (NB = nb)
  int capp;
  int nb;
};

Partition xcd_partition(int64_t I, int64_t ublocks, int num_cus, int NB) {
  // ~dcert_wg_per_cu workgroups per CU, NP a multiple of 8 (XCD-aware), <= DCERT_MAX_NP
  int64_t np = std::max<int64_t>(
      1, (int64_t)dcert_wg_per_cu(NB) * num_cus / std::max<int64_t>(ublocks, 1));
  np = std::min<int64_t>(np, std::max<int64_t>(1, hnm_cdiv(I, 4 * TILE)));
  np = std::min<int64_t>(np, DCERT_MAX_NP);
  if (np >= 8) np = np / 8 * 8;
  int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), TILE) * TILE;
  return {(int)hnm_cdiv(I, ipp), ipp};
}

DotCertShape dcert_shape(int64_t B, int64_t I, int d, int K, int num_cus, int nb = 1) {
  DotCertShape sh;
  sh.DP = d <= 64 ? 64 : 128;
  sh.nb = nb;
  sh.stride = std::max<int64_t>(DCERT_MIN_STRIDE, I / DCERT_SAMPLE);  // sample <= 1/stride of the items
  sh.Ns = hnm_cdiv(I, sh.stride);
  sh.part = xcd_partition(I, hnm_cdiv(B, 128 * nb), num_cus, nb);
  sh.spart = xcd_partition(sh.Ns, hnm_cdiv(B, 128), num_cus, 1);
  const int64_t total = std::min<int64_t>(8192, std::max<int64_t>(256, 8 * (int64_t)K * sh.stride));
  sh.capp = (int)std::max<int64_t>(32, std::min<int64_t>(total, hnm_cdiv(4 * total, sh.part.np)));
  return sh;
}

// the main scan's segments (cnt, buf: sized by its NB) come last, so the begin phase's tables
// sit at the same offsets whichever NB the finish phase takes (its own filter decides)
size_t dcert_carve(char* base, int64_t B, int64_t I, int d, int K, int num_cus, DotCertWs* w,
                   int nb = 1) {
  const DotCertShape sh = dcert_shape(B, I, d, K, num_cus, nb);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += hnm_align(bytes);
    return p;
  };
  DotCertWs x;
  x.prm = (DParams*)take(sizeof(DParams));
  x.Nu = (float*)take(B * 4);
  x.part = (float*)take(4 * 4 * (2048 + DCERT_USER_BLOCKS));
  x.Ni = (float*)take(I * 4);
  x.ubr = (float*)take(B * 4);
  x.ibs = (float*)take(I * 4);
  x.tau = (float*)take(B * 4);
  x.E = (float*)take(B * 4);
  x.kthv = (float*)take((size_t)B * K * 4);
  x.lb = (float*)take((size_t)B * 4);
  x.kthi = (int64_t*)take((size_t)B * K * 8);
  x.flag = (int*)take(B * 4);
  x.ovf_cnt = (int32_t*)take(256);
  x.ovf_rows = (int32_t*)take(B * 4);
  x.sdense = (float*)take((size_t)B * sh.spart.np * 32 * 4);
  x.U16 = (_Float16*)take((size_t)B * sh.DP * 2);
  x.I16 = (_Float16*)take((size_t)I * sh.DP * 2);
  const size_t lb = list_cand_bytes(B, I, K, num_cus);
  x.cv = (float*)take(lb);
  x.ci = (int32_t*)take(lb);
  x.cnt = (int*)take((size_t)B * sh.part.np * 4);
  x.buf = (int32_t*)take((size_t)B * sh.part.np * sh.capp * 4);
  if (w) *w = x;
  return off;
}

// ------------------------------------------------------------------ statistics + f16 copies
// Users: wave per request row (the a1 gather fused), ||u||, user bias (+ global bias).
// Items: ||i|| with LPI lanes per row.  Per-block partial maxima -> part[block][4].
__global__ __launch_bounds__(256) void dcert_stats_kernel(DotArgs a, float* __restrict__ part,
                                                          float* __restrict__ Nu,
                                                          float* __restrict__ Ni,
                                                          float* __restrict__ ubr, int item_blocks,
                                                          int user_blocks) {
  __shared__ float red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m0 = 0.f, m1 = 0.f, m2 = 0.f;
  const bool items = (int)blockIdx.x < item_blocks;
  if (items) {  // m0 = max|i_k|, m1 = max ||i||, m2 = max |ib|
    // LPI lanes x float4 per item row (d <= 4 LPI), 64 / LPI items per wave step
    const int LPI = a.d <= 64 ? 16 : 32, ipw = 64 / LPI;
    const int sub = lane / LPI, l = lane % LPI;
    for (int64_t i0 = ((int64_t)blockIdx.x * 4 + wave) * ipw; i0 < a.I;
         i0 += (int64_t)item_blocks * 4 * ipw) {
      const int64_t i = i0 + sub;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < a.I && 4 * l < a.d) v = *reinterpret_cast<const float4*>(a.it + i * a.ldi + 4 * l);
      m0 = nmax(m0, nmax(nmax(fabsf(v.x), fabsf(v.y)), nmax(fabsf(v.z), fabsf(v.w))));
      float q = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      for (int o = LPI / 2; o >= 1; o >>= 1) q += __shfl_xor(q, o);
      const float n = sqrtf(q);
      if (i < a.I) {
        m1 = nmax(m1, n);
        if (l == 0) {
          Ni[i] = n;
          if (a.ibias) m2 = nmax(m2, fabsf(a.ibias[i]));
        }
      }
    }
  } else {  // m0 = max|u_k|; LPU lanes x float4 per request row (the a1 gather fused), 64 / LPU
            // rows per wave step (a wave per row was a serial latency chain per wave at the
            // 8 x 4,096 rows of an 8-rank item-sharded step)
    const int LPU = a.d <= 64 ? 16 : 32, upw = 64 / LPU;
    const int sub = lane / LPU, l = lane % LPU;
    const int ub = (int)blockIdx.x - item_blocks;
    for (int64_t b0 = ((int64_t)ub * 4 + wave) * upw; b0 < a.B;
         b0 += (int64_t)user_blocks * 4 * upw) {
      const int64_t b = b0 + sub;
      const bool live = b < a.B;
      const int64_t uid = live ? a.uids[b] : 0;
      const bool ok = uid >= 0 && uid < a.num_users;
      if (live && !ok && l == 0) hnm_flag(a.err, HNM_ERR_OOB);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (live && ok && 4 * l < a.d) v = *reinterpret_cast<const float4*>(a.ut + uid * a.ldu + 4 * l);
      m0 = nmax(m0, nmax(nmax(fabsf(v.x), fabsf(v.y)), nmax(fabsf(v.z), fabsf(v.w))));
      float q = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      for (int o = LPU / 2; o >= 1; o >>= 1) q += __shfl_xor(q, o);
      if (live && l == 0) {
        Nu[b] = sqrtf(q);
        const float bv = (a.ubias && ok) ? a.ubias[uid] : 0.f;
        ubr[b] = bv + (a.cbias ? a.cbias[0] : 0.f);  // the exact kernel's ub[r]
      }
    }
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  if (lane == 0) {
    red[wave][0] = m0;
    red[wave][1] = m1;
    red[wave][2] = m2;
  }
  __syncthreads();
  if (tid < 3) {
    float m = red[0][tid];
    for (int w = 1; w < 4; ++w) m = nmax(m, red[w][tid]);
    part[blockIdx.x * 4 + tid] = m;  // per-block partials, reduced by dcert_scales_kernel
  }
}

__global__ __launch_bounds__(256) void dcert_scales_kernel(DParams* prm, int DP,
                                                           const float* __restrict__ part,
                                                           int item_blocks, int user_blocks,
                                                           int* __restrict__ ovf_cnt) {
  __shared__ float pm[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float mi = 0.f, mn = 0.f, mb = 0.f, mu = 0.f;  // items: max|i|, max||i||, max|ib|; users: max|u|
  // partials in batches of 8 per thread, every load of a batch issued before the first use
  // (this single block is latency: one L2 round trip per batch instead of one per partial)
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
        mi = nmax(mi, v[k].x); mn = nmax(mn, v[k].y); mb = nmax(mb, v[k].z);
      } else if (blk < nblk) {
        mu = nmax(mu, v[k].x);
      }
    }
  }
  mi = wave_max(mi); mn = wave_max(mn); mb = wave_max(mb); mu = wave_max(mu);
  if (lane == 0) { pm[wave][0] = mi; pm[wave][1] = mn; pm[wave][2] = mb; pm[wave][3] = mu; }
  __syncthreads();
  if (tid != 0) return;
  for (int w = 1; w < 4; ++w)
    for (int q = 0; q < 4; ++q) pm[0][q] = nmax(pm[0][q], pm[w][q]);
  prm->mx[DM_I] = __float_as_uint(pm[0][0]);
  prm->mx[DM_NI] = __float_as_uint(pm[0][1]);
  prm->mx[DM_IB] = __float_as_uint(pm[0][2]);
  prm->mx[DM_U] = __float_as_uint(pm[0][3]);
  if (ovf_cnt) *ovf_cnt = 0;
  const float mU = __uint_as_float(prm->mx[DM_U]), mI = __uint_as_float(prm->mx[DM_I]);
  const float mN = __uint_as_float(prm->mx[DM_NI]), mB = __uint_as_float(prm->mx[DM_IB]);
  const float lim = 1099511627776.f;  // 2^40
  bool bad = false;
  for (float m : {mU, mI, mN, mB}) bad |= !(m <= lim);
  const float su = mU > 0.f ? pow2_below_inv(mU) : 1.f;
  const float si = mI > 0.f ? pow2_below_inv(mI) : 1.f;
  const float s = su * si;
  bad |= !(s >= 1e-30f && s <= 1e30f);
  prm->su = su;
  prm->si = si;
  prm->s = s;
  // subnormal terms: sum_k phi (|u~_k| + |i~_k|) <= 2 DP phi, phi = 2^-25; x4 slack
  prm->absb = 8.f * DP * 2.98023224e-08f;
  prm->bad = bad;
}

__global__ __launch_bounds__(256) void dcert_convert_kernel(DotArgs a, int DP,
                                                            const DParams* __restrict__ prm,
                                                            _Float16* __restrict__ U16,
                                                            _Float16* __restrict__ I16,
                                                            float* __restrict__ ibs) {
  const float su = prm->su, si = prm->si, s = prm->s;
  const int64_t nthreads = (int64_t)gridDim.x * 256;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c4n = DP / 4;
  for (int64_t e = g; e < a.I * c4n; e += nthreads) {
    const int64_t i = e / c4n;
    const int c = (int)(e % c4n);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (4 * c < a.d) v = *reinterpret_cast<const float4*>(a.it + i * a.ldi + 4 * c);
    _Float16* o = I16 + i * DP + 4 * c;
    o[0] = (_Float16)(v.x * si);
    o[1] = (_Float16)(v.y * si);
    o[2] = (_Float16)(v.z * si);
    o[3] = (_Float16)(v.w * si);
    if (c == 0 && a.ibias) ibs[i] = a.ibias[i] * s;
  }
  for (int64_t e = g; e < a.B * c4n; e += nthreads) {
    const int64_t b = e / c4n;
    const int c = (int)(e % c4n);
    const int64_t uid = a.uids[b];
    const bool ok = uid >= 0 && uid < a.num_users;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok && 4 * c < a.d) v = *reinterpret_cast<const float4*>(a.ut + uid * a.ldu + 4 * c);
    _Float16* o = U16 + b * DP + 4 * c;
    o[0] = (_Float16)(v.x * su);
    o[1] = (_Float16)(v.y * su);
    o[2] = (_Float16)(v.z * su);
    o[3] = (_Float16)(v.w * su);
  }
}

// ------------------------------------------------------------------ f16 scan
// DENSE: dense[b][n] = scaled approx (diagnostics).  SAMPLE: per (user, partition, item
// lane) running max of the scaled approx over the strided sample (masked items excluded)
// -> dense[b][p * 32 + j]; the K-th best of those maxima is a lower bound of the sample's
// K-th best.  THRESH: append approx >= tau_b to the (user, partition) segment.

struct DScanArgs {
  const _Float16* U16;  // [B, DP]
  const _Float16* I16;  // [Itot, DP]
  const float* ibs;     // [Itot] item bias, scaled (BIAS)
  int64_t B, I, istride, ipp;
  int64_t itab;         // rows of the I16 / ibs tables (buffer-load extents)
  int NP;
  const int64_t* mptr;
  const int32_t* midx;
  const float* tau;     // [B] scaled thresholds (THRESH)
  int* cnt;             // [B, NP]
  int32_t* buf;         // [B, NP, capp]
  int capp;
  float* dense;         // [B, ldo] scaled approx (SAMPLE)
  int64_t ldo;
};

__device__ __forceinline__ f32x16 mfma16(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// A wave holds NB blocks of 32 users' f16 rows as MFMA A operands; TI-item tiles of I16 (128
// items at DP = 64, 64 at DP = 128) stream through LDS, double-buffered with one barrier per
// tile (LD 16-B chunks per thread: a whole tile of work for the prefetch to land).  Every step
// runs two independent MFMA chains: NB = 1 two sub-tiles of one user block, NB = 2 one sub-tile
// of two user blocks -- each item fragment read from LDS then feeds two MFMAs, which halves the
// LDS traffic per MFMA (round 4: at NB = 1 the 12 waves of a CU read 192 KB of fragments per
// tile, as many LDS cycles as the tile's matrix-pipe cycles, and the scan ran at ~0.5 of the
// random-data MFMA rate).  acc[r] = approx dot of user row 32 nb + mfma32_row(r, h) with item
// lane j of the sub-tile.  THRESH: a lane's 16 rows reduced by one max tree and one ballot per
// chain; only a chain with a pass forms its row bits and appends.
// MASK (compile-time): a filter CSR is present.  Its per-row cursor loads are the only global
// loads inside the tile loop; in a kernel without them the waitcnt pass never has to assume a
// pending load there (which otherwise costs vmcnt(0) -- the tile prefetch too -- per step).
// Item tiles are fetched by buffer loads (SGPR tile offsets, one per-thread VGPR offset; the
// 64-bit per-chunk addresses of round 3 cost ~38 VALU a tile): rows past the partition end
// hold the next partition's items (finite; every consumer tests n < part_end), past the table
// end the buffer reads zeros (the host keeps itab * DP * 2 < 2^31: dot_cert_eligible).
template <int DP, int MODE, bool BIAS, bool MASK, int NB>
__global__ __launch_bounds__(256, dcert_wg_per_cu(NB)) void dot16_scan_kernel(DScanArgs A) {
  constexpr int KS = DP / 16;     // f16 MFMA k-steps
  constexpr int RS = DP + 8;      // LDS row stride (halfs): conflict-free b128 reads
  constexpr int CH = DP / 8;      // 16-B chunks per item row
  constexpr int TI = DP <= 64 ? 128 : 64;  // items per LDS tile
  constexpr int SUB = TI / TILE;
  constexpr int LD = TI * CH / 256;  // chunks per thread per tile (4)
  constexpr int UW = 32 * NB;        // users per wave
  constexpr int NTS = NB == 1 ? 2 : 1;  // sub-tiles per step: two MFMA chains
  constexpr int NC = NTS * NB;  // MFMA chains per step
  __shared__ __attribute__((aligned(16))) _Float16 vs[2][TI * RS];
  __shared__ float ibl[2][BIAS ? TI : 1];  // the tile's scaled item biases
  __shared__ int lcnt[4][MODE == DSCAN_THRESH ? UW : 1];  // THRESH: appends per (wave, user row)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  const int p = blockIdx.x;
  const int64_t b0 = (int64_t)blockIdx.y * 4 * UW + wave * UW;
  const int nu = (int)std::max<int64_t>(0, std::min<int64_t>(UW, A.B - b0));
  const int64_t part_start = (int64_t)p * A.ipp;
  const int64_t part_end = std::min<int64_t>(A.I, part_start + A.ipp);
  const int64_t S = MODE == DSCAN_SAMPLE ? A.istride : 1;  // the strided sample is the only S > 1 pass

  h8 a[NB][KS];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      h8 z = {};
      a[nb][s] = 32 * nb + j < nu
                     ? *reinterpret_cast<const h8*>(A.U16 + (b0 + 32 * nb + j) * DP + 16 * s + 8 * h)
                     : z;
    }
  // THRESH: minus the threshold of accumulator row r's user -- the MFMA chain's initial value,
  // so the accumulator ends as approx - tau (-inf for rows past the batch: never passes).  The
  // extra fp32 rounding of the chain by |tau| (a few 2^-24 of the score scale) is inside the
  // 2^-18 guard dcert_tau_kernel leaves.
  // (loads unconditional at a clamped row, then a select: a load inside the branch would be
  // waited for right there, 16 serial round trips)
  f32x16 ntv[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t b = b0 + 32 * nb + mfma32_row(r, h);
      if (MODE == DSCAN_THRESH) {
        const float tb = A.tau[std::min<int64_t>(b, A.B - 1)];
        ntv[nb][r] = b < A.B ? -tb : -__builtin_inff();
      } else {
        ntv[nb][r] = -__builtin_inff();
      }
    }
  if (MODE == DSCAN_THRESH && lane < UW) lcnt[wave][lane] = 0;
  constexpr int NR = MODE == DSCAN_SAMPLE ? 16 * NB : 1;
  float rmax[NR];  // SAMPLE: running max per C row (block nb: rmax[16 nb + r])
#pragma unroll
  for (int r = 0; r < NR; ++r) rmax[r] = -__builtin_inff();
  int nm = INT_BIG;
  int64_t mpos = 0, mend = 0;
  constexpr bool masked = MODE != DSCAN_DENSE && MASK;
  if (masked && lane < nu) {  // lane u follows user b0 + u (UW <= 64)
    const int64_t lo = A.mptr[b0 + lane], hi = A.mptr[b0 + lane + 1];
    mpos = mask_lower_bound(A.midx, lo, hi, (int)(part_start * S));
    mend = hi;
    nm = mpos < mend ? A.midx[mpos] : INT_BIG;
  }
  int32_t* seg = MODE == DSCAN_THRESH ? A.buf + (b0 * A.NP + p) * (int64_t)A.capp : nullptr;
  const int segstride = A.NP * A.capp;  // row r's segment at r * segstride (< 2^31 / 64)
  // Appends are queued in two registers per lane and stored once per tile, after the tile's
  // prefetch has landed: vmcnt waits are in order, so a store inside the tile would make the
  // next wait (at the first MFMA after it) also wait for the prefetch issued before it
  // (round 4 A/B: direct stores with one ballot per row, 0.105 vs 0.089 ms)
  int qo0 = -1, qo1 = -1, qi0 = 0, qi1 = 0;

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, TI) : 0;
  h8 st[LD];
  float nib = 0.f;  // thread tid < TI: the bias of tile item tid
  const __amdgpu_buffer_rsrc_t irs =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.I16, 0, (int)(A.itab * DP * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      BIAS ? (void*)A.ibs : (void*)A.I16, 0, BIAS ? (int)(A.itab * 4) : 0, 0x00020000);
  const int vrow = (int)((tid / CH) * S * DP * 2 + (tid % CH) * 16);  // this thread's chunk
  const int qstride = (int)((256 / CH) * S * DP * 2);                 // next q: 256 / CH rows on
  auto fetch = [&](int64_t base) {
    const int soff = (int)(base * S * DP * 2);
#pragma unroll
    for (int q = 0; q < LD; ++q)
      st[q] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(irs, vrow, soff + q * qstride, 0));
    if (BIAS && tid < TI)
      nib = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brs, (int)(tid * S * 4), (int)(base * S * 4), 0));
  };
  auto stash = [&](int bf) {
#pragma unroll
    for (int q = 0; q < LD; ++q) {
      const int f = tid + 256 * q, row = f / CH, c = f % CH;
      *reinterpret_cast<h8*>(&vs[bf][row * RS + 8 * c]) = st[q];
    }
    if (BIAS && tid < TI) ibl[bf][tid] = nib;
  };
  if (ntiles > 0) {
    fetch(part_start);
    stash(0);
  }
  __syncthreads();
  // drain every prologue load on every path into the loop (incl. ntiles == 0): otherwise the
  // waitcnt pass merges a pending prologue load into the loop and waits vmcnt(0) -- i.e. for
  // the tile prefetch too -- at the first use of a prologue register in every iteration
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15)
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t tbase = part_start + t * TI;
    const int cur = (int)(t & 1);
    // fetch / stash run on every iteration (the last one re-reads its own tile into the idle
    // buffer): made conditional, the waitcnt pass assumes the tile loads may still be pending
    // at the loop head and waits vmcnt(0) there -- which waits for the append stores flushed
    // just before the barrier (a store round trip per tile)
    fetch(t + 1 < ntiles ? tbase + TI : tbase);
    if (nu > 0) {
      // filtered (user, item) pairs of block nb's sub-tile at base -> -inf (rare path)
      auto apply_mask = [&](f32x16& sc, int nb, int64_t base, int64_t n) {
        const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);
        const int64_t real_end = (tile_end - 1) * S + 1;  // real ids of this tile are < real_end
        uint64_t mm = __ballot(lane >= 32 * nb && lane < 32 * nb + 32 && nm < real_end);
        while (mm) {
          const int uu = __builtin_ctzll(mm);
          mm &= mm - 1;
          while (true) {
            const int tgt = hnm_readlane_i(nm, uu);
            if (tgt >= real_end) break;
            if (tgt % S == 0) {
#pragma unroll
              for (int r = 0; r < 16; ++r)
                if (mfma32_row(r, h) == (uu & 31) && n == tgt / S) sc[r] = -__builtin_inff();
            }
            if (lane == uu) {
              ++mpos;
              nm = mpos < mend ? A.midx[mpos] : INT_BIG;
            }
          }
        }
      };
      // THRESH: acc[r] = approx - tau of row r's user (the MFMA chain starts from -tau), so a
      // lane's test is one max3 tree over its 16 rows, + the item bias, and one ballot (about
      // one pass per 32 x 32 sub-tile at ~100 candidates per row).  On a pass, every passing
      // lane appends its own (row, item) passes: slot = the wave's LDS counter of that user
      // row (ds_add_rtn), the store queued.  Measured against a scalar-unit walk of the
      // passing lanes by the rows' owner lanes: 0.094 vs 0.107 ms (the walk alone 0.027 ms of
      // it), and a per-quarter test (4 maxima, 4 ballots): 4-6 % slower
      // (tools/dot_scan_timing.hip, profiles/r2_dot_scan_timing.txt).  Round 4 on the MF step:
      // row bits formed only for the 4-row groups with a pass (group maxima as the max tree)
      // 0.092 vs 0.083 ms; one ballot per row with direct stores 0.105 vs 0.089 ms.
      auto thresh = [&](const f32x16& acc, int nb, float ib, int64_t base, bool ivalid) {
        float lm = acc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) lm = fmaxf(lm, acc[r]);
        if (!__ballot(ivalid && !(lm + ib < 0.f))) return;
        unsigned rb = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) rb |= !(acc[r] + ib < 0.f) ? 1u << r : 0u;
        if (!ivalid) rb = 0;
        const int nl = (int)(base + j);
        while (rb) {  // divergent: usually one pass in one lane
          const int r = __builtin_ctz(rb);
          rb &= rb - 1;
          const int row = 32 * nb + (r & 3) + 8 * (r >> 2) + 4 * h;  // 32 nb + mfma32_row(r, h)
          const int slot = atomicAdd(&lcnt[wave][row], 1);
          if (slot < A.capp) {
            const int off = row * segstride + slot;
            if (qo0 < 0) {
              qo0 = off;
              qi0 = nl;
            } else if (qo1 < 0) {
              qo1 = off;
              qi1 = nl;
            } else {
              seg[off] = nl;  // queue full (rare)
            }
          }
        }
      };
#pragma unroll 1
      for (int u = 0; u < SUB; u += NTS) {
        const int64_t baseA = tbase + TILE * u;
        if (baseA >= part_end) break;  // uniform: partial last tile
        const bool hasB = NTS == 1 || baseA + TILE < part_end;
        // chain c: user block c % NB, sub-tile u + c / NB
        f32x16 acc[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] = MODE == DSCAN_THRESH ? ntv[c % NB] : f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int t = 0; t < NTS; ++t) {
            const h8 bf = *reinterpret_cast<const h8*>(&vs[cur][(TILE * (u + t) + j) * RS + 16 * s + 8 * h]);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) acc[t * NB + nb] = mfma16(a[nb][s], bf, acc[t * NB + nb]);
          }
        if (MODE == DSCAN_SAMPLE && hasB && baseA + NTS * TILE <= part_end) {
          // the step's sub-tiles fully inside the partition (uniform).  No NaN handling needed:
          // a non-finite table entry marks the whole call bad (dcert_scales_kernel,
          // NaN-propagating maxima) and every row takes the exact path.  NB = 1: one v_max3 per
          // row and sub-tile pair; NB = 2: one v_med3(x, m, +inf) = max per row and block (an
          // fmaxf would first canonicalize the MFMA result: 3 instructions)
          const float ibA = BIAS ? ibl[cur][TILE * u + j] : 0.f;
          const float ibB = BIAS && NTS == 2 ? ibl[cur][TILE * (u + 1) + j] : 0.f;
#pragma unroll
          for (int c = 0; c < NC; ++c)
            if (masked) apply_mask(acc[c], c % NB, baseA + TILE * (c / NB), baseA + TILE * (c / NB) + j);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if constexpr (NB == 1) {
              rmax[r] = fmaxf(rmax[r], fmaxf(BIAS ? acc[0][r] + ibA : acc[0][r], BIAS ? acc[1][r] + ibB : acc[1][r]));
            } else {
#pragma unroll
              for (int nb = 0; nb < NB; ++nb)
                rmax[16 * nb + r] = __builtin_amdgcn_fmed3f(BIAS ? acc[nb][r] + ibA : acc[nb][r],
                                                            rmax[16 * nb + r], __builtin_inff());
            }
          }
          continue;
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int t = c / NB, nb = c % NB;
          if (t == 1 && !hasB) break;
          const int sub = u + t;
          const int64_t base = tbase + TILE * sub;
          const int64_t n = base + j;
          const bool ivalid = n < part_end;
          f32x16 sc = acc[c];
          const float ib = BIAS ? ibl[cur][TILE * sub + j] : 0.f;
          if (masked) apply_mask(sc, nb, base, n);
          if (MODE == DSCAN_THRESH) {
            thresh(sc, nb, ib, base, ivalid);
            continue;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[r] = BIAS ? sc[r] + ib : sc[r];
          if (MODE == DSCAN_DENSE) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int64_t b = b0 + 32 * nb + mfma32_row(r, h);
              if (ivalid && b < A.B) A.dense[b * A.ldo + n] = sc[r];
            }
          } else {  // SAMPLE
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float& m = rmax[16 * nb + r];
              if (ivalid) m = (sc[r] > m || sc[r] != sc[r]) ? sc[r] : m;  // NaN sticks
            }
          }
        }
      }
    }
    stash(cur ^ 1);
    if (MODE == DSCAN_THRESH) {  // flush the queued appends (the prefetch has landed)
      if (qo0 >= 0) seg[qo0] = qi0;
      if (qo1 >= 0) seg[qo1] = qi1;
      qo0 = qo1 = -1;
    }
    __syncthreads();
  }
  if (MODE == DSCAN_THRESH && lane < nu) A.cnt[(b0 + lane) * A.NP + p] = lcnt[wave][lane];
  if (MODE == DSCAN_SAMPLE) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t b = b0 + 32 * nb + mfma32_row(r, h);
        if (b < A.B) A.dense[b * A.ldo + p * 32 + j] = rmax[16 * nb + r];
      }
  }
}

// Per row: E = the bound (scaled units; exact = approx / s + ubr up to E / s for every item).
// The sample's K-th best approx kv certifies a lower bound of the row's exact K-th best
// score in real units, L = (kv - E) / s + ubr (s a power of two; 2^-21 relative covers the
// fp32 rounding); unusable rows get L = -inf.  Any lower bound works downstream -- e.g. the
// max of the item shards' L over the ranks of a node (hnm_dot_topk_begin_f32 / _finish_f32).
__global__ __launch_bounds__(256) void dcert_bound_kernel(const float* __restrict__ kth, int K,
                                                          const float* __restrict__ Nu,
                                                          const float* __restrict__ ubr,
                                                          const DParams* __restrict__ prm,
                                                          int64_t B, float* __restrict__ lb,
                                                          float* __restrict__ Eout) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float s = prm->s;
  const float nimax = __uint_as_float(prm->mx[DM_NI]), ibmax = __uint_as_float(prm->mx[DM_IB]);
  const float E = s * (DCERT_RHO * Nu[b] * nimax + 2.4e-7f * (fabsf(ubr[b]) + ibmax)) + prm->absb;
  if (Eout) Eout[b] = E / s;
  if (!kth) return;
  float l = (kth[b * K + (K - 1)] - E) / s + ubr[b];
  l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
  lb[b] = (!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(E)) ? l : -__builtin_inff();
}

// Per (row, r < K): the certified lower bound of the exact score of the sample's r-th best
// item (real units, as dcert_bound_kernel for the K-th; the sample's columns are distinct
// items), for an exchange of whole lists across item shards: the K-th best of the union of
// every shard's lists bounds the global K-th.  Runs after dcert_bound_kernel (reads its E).
__global__ __launch_bounds__(256) void dcert_bound_lists_kernel(const float* __restrict__ kth,
                                                                int K,
                                                                const float* __restrict__ Eds,
                                                                const float* __restrict__ ubr,
                                                                const DParams* __restrict__ prm,
                                                                int64_t B,
                                                                float* __restrict__ lists) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= B * K) return;
  const int64_t b = x / K;
  const float E = Eds[b];  // E / s
  float l = kth[x] / prm->s - E + ubr[b];
  l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
  lists[x] = (!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(E)) ? l : -__builtin_inff();
}

// Per row: the scan threshold (scaled units) from a lower bound L of the exact K-th: an item
// can be in the top-K only if exact >= L, i.e. approx >= (L - ubr) s - E; minus the guard for
// the fp32 rounding of the test quantities (2^-18 of the row's score scale, 2^-20 relative).
__global__ __launch_bounds__(256) void dcert_tau_kernel(const float* __restrict__ lb,
                                                        const float* __restrict__ Nu,
                                                        const float* __restrict__ ubr,
                                                        const DParams* __restrict__ prm,
                                                        int64_t B, float* __restrict__ tau,
                                                        int* __restrict__ flag) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float s = prm->s;
  const float nimax = __uint_as_float(prm->mx[DM_NI]), ibmax = __uint_as_float(prm->mx[DM_IB]);
  const float scale = s * (Nu[b] * nimax + fabsf(ubr[b]) + ibmax);
  const float E = s * (DCERT_RHO * Nu[b] * nimax + 2.4e-7f * (fabsf(ubr[b]) + ibmax)) + prm->absb;
  float tv = (lb[b] - ubr[b]) * s - E - 3.814697265625e-06f * scale;  // 2^-18
  tv -= fabsf(tv) * 9.5367431640625e-07f;                               // 2^-20
  const bool ok = !prm->bad && __builtin_isfinite(tv) && __builtin_isfinite(scale);
  tau[b] = ok ? tv : __builtin_inff();
  flag[b] = ok ? 0 : 1;
}

// One-shot calls (dot_cert_topk): dcert_bound_kernel's lower bound and dcert_tau_kernel's
// threshold per row in the epilogue of the sample K-th launch -- the same arithmetic, L kept in
// a register (round 5 fused the two into one kernel after the K-th; round 6 folds that kernel
// into the K-th launch: one launch and one kernel boundary less on the per-call latency chain).
struct DotTauEpi {
  const DParams* prm;
  const float* Nu;
  const float* ubr;
  float* tau;
  int* flag;
  __device__ void operator()(int64_t b, float kv) const {
    const float s = prm->s;
    const float nimax = __uint_as_float(prm->mx[DM_NI]), ibmax = __uint_as_float(prm->mx[DM_IB]);
    const float E = s * (DCERT_RHO * Nu[b] * nimax + 2.4e-7f * (fabsf(ubr[b]) + ibmax)) + prm->absb;
    float l = (kv - E) / s + ubr[b];
    l -= fabsf(l) * 4.76837158203125e-07f;  // 2^-21
    if (!(!prm->bad && __builtin_isfinite(l) && __builtin_isfinite(E))) l = -__builtin_inff();
    const float scale = s * (Nu[b] * nimax + fabsf(ubr[b]) + ibmax);
    float tv = (l - ubr[b]) * s - E - 3.814697265625e-06f * scale;  // 2^-18
    tv -= fabsf(tv) * 9.5367431640625e-07f;                          // 2^-20
    const bool ok = !prm->bad && __builtin_isfinite(tv) && __builtin_isfinite(scale);
    tau[b] = ok ? tv : __builtin_inff();
    flag[b] = ok ? 0 : 1;
  }
};

// ------------------------------------------------------------------ exact re-scoring
// One wave per user; each lane re-scores one candidate with the sequential fp32 fma chain
// (k = 0 .. DP-1, zero padding included) the f32 MFMA computes, then (acc + ub) + ib as
// dot_score_kernel does; exact (score desc, item asc) top-K.
template <int DP, bool BIAS>
__global__ __launch_bounds__(256, 4) void dcert_rescore_kernel(
    DotArgs a, const float* __restrict__ ubr, const int* __restrict__ flag,
    const int* __restrict__ cnt, const int32_t* __restrict__ buf, int NP, int capp, int K,
    int short_ok, float* __restrict__ ov, int64_t* __restrict__ oi, int32_t* __restrict__ ovf_rows,
    int32_t* __restrict__ ovf_cnt, unsigned long long* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float urow[4][DP];
  __shared__ int pref[4][DCERT_MAX_NP + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  const bool live = b < a.B;
  int c = 0;
  if (live) {
    const int64_t uid = a.uids[b];
    const bool ok = uid >= 0 && uid < a.num_users;
    for (int k = lane; k < DP; k += 64) urow[wave][k] = (ok && k < a.d) ? a.ut[uid * a.ldu + k] : 0.f;
    c = lane < NP ? cnt[b * NP + lane] : 0;
  }
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
  __syncthreads();
  if (!live) return;
  const int n = hnm_readlane_i(incl, 63);
  // fewer than K candidates: the bound came from another item shard (short_ok: the merge
  // across shards completes the row) or the threshold is unusable -> fallback
  if (flag[b] || __ballot(c > capp) != 0 || (n < K && !short_ok)) {
    if (lane == 0) {
      ovf_rows[atomicAdd(ovf_cnt, 1)] = (int32_t)b;
      if (stats) {
        atomicAdd(&stats[2], 1ull);
        if (b == 0) atomicAdd(&stats[0], (unsigned long long)a.B);
      }
    }
    return;
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[1], (unsigned long long)n);
    if (b == 0) atomicAdd(&stats[0], (unsigned long long)a.B);
  }
  const float ub = ubr[b];
  const int32_t* rowbuf = buf + b * (int64_t)NP * capp;
  auto cand = [&](int g) -> int {  // segment of candidate g: last p with pref[p] <= g
    int lo = 0, hi = NP;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pref[wave][mid] <= g) lo = mid;
      else hi = mid;
    }
    return rowbuf[(int64_t)lo * capp + (g - pref[wave][lo])];
  };
  // Rounds of 128 slots: slots 0..K-1 carry the running top-K, slots K..127 take the next
  // candidates; one bitonic sort per round (no serial list inserts).
  auto score = [&](int it) -> float {
    // 32 dims = 8 float4 loads issued together (addresses clamped in range, zero padding by
    // select); groups of 32 run one after another (32 VGPRs of row data: four waves per SIMD)
    const float* r0 = a.it + (int64_t)it * a.ldi;
    float acc = 0.f;
#pragma unroll 1
    for (int g = 0; g < DP / 32; ++g) {
      float4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = 32 * g + 4 * q;
        v[q] = *reinterpret_cast<const float4*>(r0 + std::min(k, a.d - 4));
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = 32 * g + 4 * q;
        const bool in = k < a.d;
        const float4 uv = *reinterpret_cast<const float4*>(&urow[wave][k]);
        acc = fmaf(uv.x, in ? v[q].x : 0.f, acc);
        acc = fmaf(uv.y, in ? v[q].y : 0.f, acc);
        acc = fmaf(uv.z, in ? v[q].z : 0.f, acc);
        acc = fmaf(uv.w, in ? v[q].w : 0.f, acc);
      }
    }
    return BIAS ? (acc + ub) + (a.ibias ? a.ibias[it] : 0.f) : acc;
  };
  float v0 = -__builtin_inff(), v1 = -__builtin_inff();
  int i0 = HNM_SENTINEL_IDX, i1 = HNM_SENTINEL_IDX;
  bool nan = false;
  if (n <= 64) {
    // one round: lane l re-scores candidate l, one sort of the first 16 / 32 / 64 lanes (the
    // same total order as the 128-slot rounds, so the same output; the item-sharded step's
    // ranks see a few candidates a row over 8x the rows, where the 128-slot sort dominated)
    if (lane < n) {
      i0 = cand(lane);
      v0 = score(i0);
    }
    nan = v0 != v0;
    if (__ballot(nan) == 0) {
      if (n <= 16) hnm_sort_lanes<16>(v0, i0);
      else if (n <= 32) hnm_sort_lanes<32>(v0, i0);
      else hnm_sort_lanes<64>(v0, i0);
    }
  }
  for (int c0 = 0; n > 64 && c0 < n; c0 += 128 - K) {
    const int g0 = c0 + lane - K, g1 = c0 + 64 + lane - K;  // candidate of slot lane / lane+64
    if (lane >= K) {
      const bool ok = g0 < n;
      i0 = ok ? cand(g0) : HNM_SENTINEL_IDX;
      v0 = ok ? score(i0) : -__builtin_inff();
    }
    {
      const bool ok = g1 < n;
      i1 = ok ? cand(g1) : HNM_SENTINEL_IDX;
      v1 = ok ? score(i1) : -__builtin_inff();
    }
    nan |= (v0 != v0) || (v1 != v1);
    hnm_sort128(v0, i0, v1, i1);
  }
  if (__ballot(nan)) {  // NaN scores: exact LIST semantics via the fallback
    if (lane == 0) ovf_rows[atomicAdd(ovf_cnt, 1)] = (int32_t)b;
    return;
  }
  if (lane < K) {
    if (ov) ov[b * K + lane] = v0;
    oi[b * K + lane] = i0 == HNM_SENTINEL_IDX ? -1 : i0;
  }
}

__global__ void dcert_debug_out_kernel(float* __restrict__ ap, int64_t lda, int64_t B, int64_t I,
                                       const float* __restrict__ ubr,
                                       const DParams* __restrict__ prm) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= B * I) return;
  const int64_t b = x / I, o = b * lda + x % I;
  ap[o] = ap[o] / prm->s + ubr[b];  // scaled approx (item bias included) -> score units
}

hnm_status dcert_prepare(hnm_ctx* ctx, const DotArgs& a, const DotCertShape& sh,
                         const DotCertWs& x) {
  const int ib = (int)std::min<int64_t>(2048, hnm_cdiv(a.I, 16));
  const int ub = (int)std::min<int64_t>(DCERT_USER_BLOCKS, hnm_cdiv(a.B, 4 * (a.d <= 64 ? 4 : 2)));
  hipLaunchKernelGGL(dcert_stats_kernel, dim3(ib + ub), dim3(256), 0, ctx->stream, a, x.part,
                     x.Nu, x.Ni, x.ubr, ib, ub);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(dcert_scales_kernel, dim3(1), dim3(256), 0, ctx->stream, x.prm, sh.DP, x.part,
                     ib, ub, x.ovf_cnt);
  HNM_LAUNCH_CHECK();
  const int cb = (int)std::min<int64_t>(2048, std::max<int64_t>(1, hnm_cdiv(a.I * sh.DP / 4, 256)));
  hipLaunchKernelGGL(dcert_convert_kernel, dim3(cb), dim3(256), 0, ctx->stream, a, sh.DP, x.prm,
                     x.U16, x.I16, x.ibs);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

template <int MODE>
void launch_dscan(hnm_ctx* ctx, dim3 grid, const DScanArgs& s, int DP, bool bias, int nb = 1) {
  // NB = 2: the unfiltered DP = 64 main scan only (dscan_thresh_nb)
#define HNM_DS2(DPV, BV)                                                                      \
  if (s.mptr && MODE != DSCAN_DENSE)                                                          \
    hipLaunchKernelGGL((dot16_scan_kernel<DPV, MODE, BV, MODE != DSCAN_DENSE, 1>), grid,       \
                       dim3(256), 0, ctx->stream, s);                                         \
  else if (MODE == DSCAN_THRESH && DPV == 64 && nb == 2)                                      \
    hipLaunchKernelGGL((dot16_scan_kernel<DPV, MODE, BV, false, (MODE == DSCAN_THRESH && DPV == 64) ? 2 : 1>), \
                       grid, dim3(256), 0, ctx->stream, s);                                   \
  else                                                                                        \
    hipLaunchKernelGGL((dot16_scan_kernel<DPV, MODE, BV, false, 1>), grid, dim3(256), 0,       \
                       ctx->stream, s);
#define HNM_DS(DPV)    \
  if (bias) {          \
    HNM_DS2(DPV, true) \
  } else {             \
    HNM_DS2(DPV, false) \
  }
  if (DP == 64) {
    HNM_DS(64)
  } else {
    HNM_DS(128)
  }
#undef HNM_DS
#undef HNM_DS2
}

DScanArgs dscan_args(const DotCertWs& x, const DotArgs& a) {
  DScanArgs s{};
  s.U16 = x.U16;
  s.I16 = x.I16;
  s.ibs = x.ibs;
  s.B = a.B;
  s.istride = 1;
  s.itab = a.I;
  return s;
}

}  // namespace

bool dot_cert_eligible(int d, int64_t I, int K) {
  // buffer-load extents: the f16 table's bytes < 2^31 (16.7M items at d <= 64, 8.3M at 128)
  return d <= 128 && K <= 64 && I >= DCERT_MIN_ITEMS && I >= 64 * (int64_t)K &&
         I * (d <= 64 ? 64 : 128) * 2 < ((int64_t)1 << 31);
}

size_t dot_cert_bytes(int64_t B, int64_t I, int d, int K, int num_cus) {
  return std::max(dcert_carve(nullptr, B, I, d, K, num_cus, nullptr, 1),
                  dcert_carve(nullptr, B, I, d, K, num_cus, nullptr, 2));
}

// Phase 1: bound statistics, f16 copies, the sample pass and every row's certified lower
// bound of its exact K-th best score (real units) into lb (nullptr: kept in the scratch).
static hnm_status dot_cert_begin_impl(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                                      float* lb, float* lists, bool fused) {
  const DotCertShape sh = dcert_shape(a.B, a.I, a.d, a.K, ctx->num_cus);
  DotCertWs x;
  dcert_carve((char*)scratch, a.B, a.I, a.d, a.K, ctx->num_cus, &x);
  hnm_status st = dcert_prepare(ctx, a, sh, x);
  if (st) return st;
  const int64_t ublocks = hnm_cdiv(a.B, (int64_t)128);  // the sample pass: NB = 1
  DScanArgs s = dscan_args(x, a);
  s.I = sh.Ns;
  s.istride = sh.stride;
  s.mptr = a.mptr;
  s.midx = a.midx;
  s.dense = x.sdense;
  s.ldo = sh.spart.np * 32;
  s.ipp = sh.spart.ipp;
  s.NP = sh.spart.np;
  launch_dscan<DSCAN_SAMPLE>(ctx, dim3((unsigned)sh.spart.np, (unsigned)ublocks), s, sh.DP, bias);
  HNM_LAUNCH_CHECK();
  const int64_t nmax_cols = (int64_t)sh.spart.np * 32;
  if (fused)  // the one-shot call: bound + threshold in the K-th launch's epilogue
    return sample_kth_launch(ctx, x.sdense, nmax_cols, a.B, nmax_cols, nullptr, nullptr, a.K, 1, 1,
                             nullptr, x.kthv, nullptr, DotTauEpi{x.prm, x.Nu, x.ubr, x.tau, x.flag});
  st = hnm_sample_kth(ctx, x.sdense, nmax_cols, a.B, nmax_cols, nullptr, nullptr, a.K, 1, 1,
                      nullptr, x.kthv);
  if (st) return st;
  hipLaunchKernelGGL(dcert_bound_kernel, dim3((unsigned)hnm_cdiv(a.B, 256)), dim3(256), 0,
                     ctx->stream, x.kthv, a.K, x.Nu, x.ubr, x.prm, a.B, lb ? lb : x.lb, x.E);
  HNM_LAUNCH_CHECK();
  if (lists) {
    hipLaunchKernelGGL(dcert_bound_lists_kernel, dim3((unsigned)hnm_cdiv(a.B * a.K, 256)), dim3(256),
                       0, ctx->stream, x.kthv, a.K, x.E, x.ubr, x.prm, a.B, lists);
    HNM_LAUNCH_CHECK();
  }
  return HNM_OK;
}

hnm_status dot_cert_begin(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch, float* lb,
                          float* lists) {
  return dot_cert_begin_impl(ctx, a, bias, scratch, lb, lists, false);
}

// Phase 2: thresholds from lower bounds lb (this call's, or the max over item shards), the
// main f16 scan, exact re-scoring + top-K, the exact LIST scan for unusable rows.  fused: the
// one-shot call, thresholds already written by the sample K-th launch (DotTauEpi).
static hnm_status dot_cert_finish_impl(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                                       const float* lb, int short_ok, float* ov, int64_t* oi,
                                       bool fused) {
  const int nb = dscan_thresh_nb(a.d, a.mptr != nullptr);
  const DotCertShape sh = dcert_shape(a.B, a.I, a.d, a.K, ctx->num_cus, nb);
  DotCertWs x;
  dcert_carve((char*)scratch, a.B, a.I, a.d, a.K, ctx->num_cus, &x, nb);
  const int64_t ublocks = hnm_cdiv(a.B, (int64_t)128 * nb);
  if (!fused) {  // fused: tau / flag came with the sample K-th (DotTauEpi)
    hipLaunchKernelGGL(dcert_tau_kernel, dim3((unsigned)hnm_cdiv(a.B, 256)), dim3(256), 0,
                       ctx->stream, lb ? lb : x.lb, x.Nu, x.ubr, x.prm, a.B, x.tau, x.flag);
    HNM_LAUNCH_CHECK();
  }
  {  // main f16 scan: append approx >= tau_u
    DScanArgs s = dscan_args(x, a);
    s.I = a.I;
    s.mptr = a.mptr;
    s.midx = a.midx;
    s.tau = x.tau;
    s.cnt = x.cnt;
    s.buf = x.buf;
    s.capp = sh.capp;
    s.ipp = sh.part.ipp;
    s.NP = sh.part.np;
    hnm_timer_begin(ctx, HNM_TIME_SCORE);
    launch_dscan<DSCAN_THRESH>(ctx, dim3((unsigned)sh.part.np, (unsigned)ublocks), s, sh.DP, bias,
                               nb);
    hnm_timer_end(ctx, HNM_TIME_SCORE);
    HNM_LAUNCH_CHECK();
  }
  // exact re-scoring + top-K; unusable rows queued
  unsigned long long* stp = ctx->stats_on ? ctx->stats_dev : nullptr;
#define HNM_RS(DPV, BV)                                                                         \
  hipLaunchKernelGGL((dcert_rescore_kernel<DPV, BV>), dim3((unsigned)hnm_cdiv(a.B, 4)), dim3(256), \
                     0, ctx->stream, a, x.ubr, x.flag, x.cnt, x.buf, sh.part.np, sh.capp, a.K,   \
                     short_ok, ov, oi, x.ovf_rows, x.ovf_cnt, stp);
  if (sh.DP == 64) {
    if (bias) { HNM_RS(64, true) } else { HNM_RS(64, false) }
  } else {
    if (bias) { HNM_RS(128, true) } else { HNM_RS(128, false) }
  }
#undef HNM_RS
  HNM_LAUNCH_CHECK();
  // exact LIST scan for the queued rows
  DotArgs af = a;
  af.rows = x.ovf_rows;
  af.nrows = x.ovf_cnt;
  return dot_list_pass(ctx, af, bias, x.cv, x.ci, ov, oi);
}

hnm_status dot_cert_finish(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                           const float* lb, int short_ok, float* ov, int64_t* oi) {
  return dot_cert_finish_impl(ctx, a, bias, scratch, lb, short_ok, ov, oi, false);
}

hnm_status dot_cert_topk(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch, float* ov,
                         int64_t* oi) {
  hnm_status st = dot_cert_begin_impl(ctx, a, bias, scratch, nullptr, nullptr, true);
  if (st) return st;
  return dot_cert_finish_impl(ctx, a, bias, scratch, nullptr, 0, ov, oi, true);
}

hnm_status dot_cert_debug(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                          float* approx, int64_t lda, float* bound) {
  const DotCertShape sh = dcert_shape(a.B, a.I, a.d, 1, ctx->num_cus);
  DotCertWs x;
  dcert_carve((char*)scratch, a.B, a.I, a.d, 1, ctx->num_cus, &x);
  hnm_status st = dcert_prepare(ctx, a, sh, x);
  if (st) return st;
  DScanArgs s = dscan_args(x, a);
  s.I = a.I;
  s.dense = approx;
  s.ldo = lda;
  const int64_t ublocks = hnm_cdiv(a.B, (int64_t)128);
  const Partition ps = xcd_partition(a.I, ublocks, ctx->num_cus, 1);
  s.ipp = ps.ipp;
  s.NP = ps.np;
  launch_dscan<DSCAN_DENSE>(ctx, dim3((unsigned)ps.np, (unsigned)ublocks), s, sh.DP,
                            bias);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(dcert_debug_out_kernel, dim3((unsigned)hnm_cdiv(a.B * a.I, 256)), dim3(256),
                     0, ctx->stream, approx, lda, a.B, a.I, x.ubr, x.prm);
  HNM_LAUNCH_CHECK();
  hipLaunchKernelGGL(dcert_bound_kernel, dim3((unsigned)hnm_cdiv(a.B, 256)), dim3(256), 0,
                     ctx->stream, nullptr, 1, x.Nu, x.ubr, x.prm, a.B, nullptr, bound);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
