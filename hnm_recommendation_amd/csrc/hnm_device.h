// Device-side building blocks shared by the gfx950 kernels of libhnm_mi355x.
//
// * Top-K order is (score desc, item asc): a TOTAL order, so a top-K computed over item
//   partitions, shards or GPUs and then merged is unique and reproducible.  torch.topk
//   (`neural_cf.py:324`, `lightgcn.py:356`, `serve.py:355`) leaves ties unspecified.
// * A wave-resident top-K list keeps slot s in lane (s % 64) of register (s / 64): sorted
//   insertion is one ballot + popcount + shfl_up, no LDS.  Candidates reach it through a
//   wave-uniform threshold pre-filter, so after warm-up almost every tile costs one
//   compare + ballot per score.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HNM_WAVE 64

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define HNM_SENTINEL_IDX 0x7fffffff

__device__ __forceinline__ bool hnm_better(float va, int ia, float vb, int ib) {
  return va > vb || (va == vb && ia < ib);
}

__device__ __forceinline__ int hnm_lane() { return __lane_id(); }

__device__ __forceinline__ float hnm_readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int hnm_readlane_i(int v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}

// Wave-wide sorted list of NS*64 slots (K <= NS*64).
template <int NS>
struct WaveTopK {
  float v[NS];
  int i[NS];
  float thr_v;  // wave-uniform copy of slot K-1
  int thr_i;

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      v[r] = -__builtin_inff();
      i[r] = HNM_SENTINEL_IDX;
    }
    thr_v = -__builtin_inff();
    thr_i = HNM_SENTINEL_IDX;
  }

  __device__ __forceinline__ void refresh(int K) {
    const int r = (K - 1) >> 6, l = (K - 1) & 63;
#pragma unroll
    for (int q = 0; q < NS; ++q)
      if (q == r) {
        thr_v = hnm_readlane_f(v[q], l);
        thr_i = hnm_readlane_i(i[q], l);
      }
  }

  // Insert one wave-uniform candidate (no-op if it does not beat slot K-1).
  __device__ __forceinline__ void insert(float cv, int ci, int K) {
    if (!hnm_better(cv, ci, thr_v, thr_i)) return;
    const int lane = hnm_lane();
    int pos = 0;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      const bool b = (lane + 64 * r < K) && hnm_better(v[r], i[r], cv, ci);
      pos += __popcll(__ballot(b));
    }
    float nv[NS];
    int ni[NS];
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      float up = __shfl_up(v[r], 1);
      int upi = __shfl_up(i[r], 1);
      if (r > 0) {
        const float cv2 = hnm_readlane_f(v[r - 1], 63);
        const int ci2 = hnm_readlane_i(i[r - 1], 63);
        if (lane == 0) { up = cv2; upi = ci2; }
      }
      const int slot = lane + 64 * r;
      nv[r] = slot > pos ? up : (slot == pos ? cv : v[r]);
      ni[r] = slot > pos ? upi : (slot == pos ? ci : i[r]);
    }
#pragma unroll
    for (int r = 0; r < NS; ++r) { v[r] = nv[r]; i[r] = ni[r]; }
    refresh(K);
  }

  // Offer one candidate per lane (only lanes with `valid`).  Serial over the lanes whose
  // candidate passes the current threshold; the threshold only rises, so every later
  // candidate is re-checked against the updated value inside insert().
  __device__ __forceinline__ void offer(float sv, int si, bool valid, int K) {
    uint64_t m = __ballot(valid && (sv > thr_v || (sv == thr_v && si < thr_i)));
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      insert(hnm_readlane_f(sv, l), hnm_readlane_i(si, l), K);
    }
  }

  // Write slots [0, K) to out_v/out_i (int32 or int64 indices).
  template <typename IdxT>
  __device__ __forceinline__ void store(float* out_v, IdxT* out_i, int K) const {
    const int lane = hnm_lane();
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      const int s = lane + 64 * r;
      if (s < K) {
        if (out_v) out_v[s] = v[r];
        out_i[s] = (IdxT)(i[r] == HNM_SENTINEL_IDX ? -1 : i[r]);
      }
    }
  }
};

// x of lane (lane ^ J), J a power of two < 64, without LDS: DPP quad permutes (J = 1, 2), row
// rotates (J = 4, 8: row_ror:n reads lane (i - n) mod 16 of the row) and the gfx950 row / half
// swaps (J = 16, 32) -- 1-3 VALU instead of a ds_bpermute round trip (~100+ cycles of latency
// on a dependent chain such as a sort network or a reduction).
template <int J>
__device__ __forceinline__ int hnm_xor_lane(int x) {
  static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "J");
  if constexpr (J == 1) {
    return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const int a = __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);  // row_ror:4
    const int b = __builtin_amdgcn_update_dpp(0, x, 0x12C, 0xF, 0xF, false);  // row_ror:12
    return (__lane_id() & 4) ? a : b;
  } else if constexpr (J == 8) {
    return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (J == 16) {
    // (vdst, src) = (x, x): vdst's odd rows <-> src's even rows: r[0] = rows (0,0,2,2),
    // r[1] = rows (1,1,3,3)
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (__lane_id() & 16) ? (int)r[0] : (int)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // r[0] = lo, r[1] = hi
    return (__lane_id() & 32) ? (int)r[0] : (int)r[1];
  }
}
template <int J>
__device__ __forceinline__ float hnm_xor_lane(float x) {
  return __int_as_float(hnm_xor_lane<J>(__float_as_int(x)));
}

// Maximum over each aligned group of G lanes (G = 16, 32, 64) in every lane of the group
// (fmaxf: a NaN lane is ignored unless all are NaN), by DPP / permlane steps (no LDS).
template <int G>
__device__ __forceinline__ float hnm_group_max(float x) {
  static_assert(G == 16 || G == 32 || G == 64, "G");
  x = fmaxf(x, hnm_xor_lane<1>(x));
  x = fmaxf(x, hnm_xor_lane<2>(x));
  x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF,
                                                          false)));  // quads q, q - 1
  x = fmaxf(x, hnm_xor_lane<8>(x));  // row max in every lane of the row
  if constexpr (G >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                    false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));  // rows 2k, 2k + 1
  }
  if constexpr (G == 64) {
    const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                    false);
    x = fmaxf(__uint_as_float(h[0]), __uint_as_float(h[1]));
  }
  return x;
}
__device__ __forceinline__ float hnm_wave_max(float x) { return hnm_group_max<64>(x); }

// One compare-exchange step of a bitonic network across lanes: partner lane ^ J; `up`: this
// lane's block is ordered best-first ((value desc, index asc), hnm_better).
template <int J>
__device__ __forceinline__ void hnm_cx(float& v, int& ix, bool up) {
  const float pv = hnm_xor_lane<J>(v);
  const int pi = hnm_xor_lane<J>(ix);
  const bool lower = (hnm_lane() & J) == 0;
  const bool pb = hnm_better(pv, pi, v, ix);   // partner ranks before mine
  const bool take = (lower == up) ? pb : !pb;  // lower slot of an up block keeps the better
  v = take ? pv : v;
  ix = take ? pi : ix;
}
__device__ __forceinline__ void hnm_cx_rt(int j, float& v, int& ix, bool up) {
  switch (j) {  // a compile-time constant after unrolling
    case 1: hnm_cx<1>(v, ix, up); break;
    case 2: hnm_cx<2>(v, ix, up); break;
    case 4: hnm_cx<4>(v, ix, up); break;
    case 8: hnm_cx<8>(v, ix, up); break;
    case 16: hnm_cx<16>(v, ix, up); break;
    default: hnm_cx<32>(v, ix, up); break;
  }
}

// Bitonic sort of one (value, index) pair per lane over each aligned group of W lanes (W = 16,
// 32, 64) into (value desc, index asc) order -- lane 0 of the group = best.  Total order on the
// inputs as hnm_sort128.
template <int W>
__device__ __forceinline__ void hnm_sort_lanes(float& v, int& ix) {
  const int lane = hnm_lane();
#pragma unroll
  for (int k = 2; k <= W; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) hnm_cx_rt(j, v, ix, k == W || (lane & k) == 0);
}

// Wave-wide bitonic sort of 128 (value, index) pairs, two per lane (slot e = lane + 64 r:
// (v0, i0) is slot lane, (v1, i1) slot lane + 64), into (value desc, index asc) order --
// slot 0 = best.  28 compare-exchange steps of one lane exchange each (hnm_xor_lane: DPP /
// permlane, no LDS); no serial inserts.  The order must be total on the inputs: distinct
// indices, no NaN (callers check).
__device__ __forceinline__ void hnm_sort128(float& v0, int& i0, float& v1, int& i1) {
  const int lane = hnm_lane();
#pragma unroll
  for (int k = 2; k <= 128; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j == 64) {  // k == 128: partner is the other register of this lane; slot lane first
        if (hnm_better(v1, i1, v0, i0)) {
          const float tv = v0; v0 = v1; v1 = tv;
          const int ti = i0; i0 = i1; i1 = ti;
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = lane + 64 * r;
        hnm_cx_rt(j, r ? v1 : v0, r ? i1 : i0, (e & k) == 0);  // up: block ordered best-first
      }
    }
  }
}

// v_mfma_f32_32x32x2_f32: A[i=l&31][k=l>>5], B[k=l>>5][j=l&31], exact fp32 fma chain.
// C/D: col j = lane&31, row i = (r&3) + 8*(r>>2) + 4*(lane>>5) for register r.
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int mfma32_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// x(lane) + x(lane ^ 32) without LDS: one v_permlane32_swap (VALU) instead of a
// ds_bpermute round trip.
__device__ __forceinline__ float hnm_sum_halves(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// c + a.lo * b.lo and c + a.hi * b.hi in fp32 from packed f16 operands (v_fma_mix_f32:
// f16 x f16 products are exact in fp32).  Unlike v_dot2_f32_f16 it co-issues with MFMA.
typedef _Float16 hnm_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float hnm_fma_mix_lo(hnm_h2 a, hnm_h2 b, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ float hnm_fma_mix_hi(hnm_h2 a, hnm_h2 b, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

#define TILE 32
#define INT_BIG 0x7fffffff

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

// Error word in device memory (ctx-owned): bit 0 = an id out of range was seen.
#define HNM_ERR_OOB 1u
#define HNM_ERR_MASK_CAP 4u  // hnm_mask_gather_csr: the batch mask exceeded its capacity
__device__ __forceinline__ void hnm_flag(unsigned* err, unsigned bit) {
  if (err) atomicOr(err, bit);
}
