// Wide&Deep all-items scoring for gfx950 (wide_deep.py:157-285, recommend :405-435).
//
// Reference per pair: deep = BN3(relu(L3(BN2(relu(L2(BN1(relu(L1([e_u; e_i]))))))))),
// score = final_layer([onehot(u); onehot(i); deep]) = w[u] + w[U + i] + w_d . deep + b.
// The one-hot wide part (a 2.7 GB scatter per user per chunk in the reference) is two
// weight lookups; eval-mode BatchNorm is an affine map folded into the next layer:
//   L2(BN1(x)) = (W2 diag a1) x + (W2 c1 + b2),  a = g / sqrt(var + eps), c = beta - mean a
// and BN3 into w_d.  Layer 1 is decomposed (P_u + Q_i, computed once per call).
//
// Per (user, 32-item tile) a wave runs, with v_mfma_f32_32x32x2_f32 (exact fp32):
//   layer 2: D2 = W2' . relu(P_u + Q_i)^T   (rows = layer-2 units, cols = items); the A
//            fragments are pre-permuted in HBM so each lane streams them with 16-B loads
//            (weights are L2-resident: 640 KB)
//   layer 3: D3 = W3' . relu(D2 + b2')^T   -- D2's accumulator registers ARE the B
//            operand: k-step (rb, r) pairs row (r&3)+8(r>>2) of half 0 with +4 of half 1,
//            and W3' is pre-permuted to the same k order, so no LDS round trip.
//   final:   relu(D3 + b3') . w_d' (16-register epilogue + one cross-half shuffle)
// Layer-2 row blocks are processed 4 at a time (64 accumulator registers) and fed into
// the layer-3 accumulators (64 registers) as they complete.
#include <algorithm>
#include <type_traits>

#include "hnm_device.h"
#include "hnm_internal.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);

#define WD_TILE 32
#define WD_INT_BIG 0x7fffffff

// ------------------------------------------------------------------ weight preparation
struct WdPrep {
  int K1P;     // layer-1 width padded to a multiple of 8
  int RB2;     // layer-2 row blocks of 32
  int OB;      // layer-3 row blocks of 32 (0: two-layer tower)
  float4* W2f; // [RB2][K1P/8][64] float4
  float4* W3f; // [OB][RB2][4][64] float4
  float* b2p;  // [RB2*32] folded layer-2 bias
  float* b3p;  // [OB*32]  folded layer-3 bias
  float* wdp;  // [32*max(OB,RB2)] folded final weights on the last hidden layer
  float* bias; // [1] folded final bias
};

__device__ __forceinline__ float bn_a(const float* g, const float* v, int i, float eps) {
  return g[i] / sqrtf(v[i] + eps);
}
__device__ __forceinline__ float bn_c(const float* g, const float* b, const float* m,
                                      const float* v, int i, float eps) {
  return b[i] - m[i] * bn_a(g, v, i, eps);
}

// W2f[rb][s4][lane].e = W2[o][k] * a1[k], o = rb*32 + (lane&31), k = 2(4 s4 + e) + (lane>>5)
__global__ void wd_prep_w2(hnm_widedeep_weights w, WdPrep p) {
  const int64_t n = (int64_t)p.RB2 * (p.K1P / 8) * 64 * 4;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int e = t & 3, lane = (t >> 2) & 63;
    const int64_t rest = t >> 8;
    const int s4 = (int)(rest % (p.K1P / 8)), rb = (int)(rest / (p.K1P / 8));
    const int o = rb * 32 + (lane & 31), k = 2 * (4 * s4 + e) + (lane >> 5);
    float v = 0.f;
    if (o < w.l2 && k < w.l1) v = w.w2[(int64_t)o * w.l1 + k] * bn_a(w.bn1_w, w.bn1_var, k, w.eps);
    reinterpret_cast<float*>(p.W2f)[t] = v;
  }
}

// W3f[ob][rb][r4][lane].e = W3[o][i] * a2[i], o = ob*32 + (lane&31),
// i = rb*32 + row(4 r4 + e, lane>>5)
__global__ void wd_prep_w3(hnm_widedeep_weights w, WdPrep p) {
  const int64_t n = (int64_t)p.OB * p.RB2 * 4 * 64 * 4;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int e = t & 3, lane = (t >> 2) & 63;
    int64_t rest = t >> 8;
    const int r4 = (int)(rest & 3);
    rest >>= 2;
    const int rb = (int)(rest % p.RB2), ob = (int)(rest / p.RB2);
    const int o = ob * 32 + (lane & 31);
    const int i = rb * 32 + mfma32_row(4 * r4 + e, lane >> 5);
    float v = 0.f;
    if (o < w.l3 && i < w.l2) v = w.w3[(int64_t)o * w.l2 + i] * bn_a(w.bn2_w, w.bn2_var, i, w.eps);
    reinterpret_cast<float*>(p.W3f)[t] = v;
  }
}

// b2' = b2 + W2 c1 [RB2*32], b3' = b3 + W3 c2 [OB*32], w_d' = w_d * a_last and the folded
// bias (zero padded); one thread per output.
__global__ void wd_prep_bias(hnm_widedeep_weights w, WdPrep p) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int last = p.OB > 0 ? w.l3 : w.l2;  // width of the last hidden layer
  const float* lg = p.OB > 0 ? w.bn3_w : w.bn2_w;
  const float* lb = p.OB > 0 ? w.bn3_b : w.bn2_b;
  const float* lm = p.OB > 0 ? w.bn3_mean : w.bn2_mean;
  const float* lv = p.OB > 0 ? w.bn3_var : w.bn2_var;
  const float* wd = w.final_deep;
  for (int o = t; o < p.RB2 * 32; o += gridDim.x * 256) {
    float v = 0.f;
    if (o < w.l2) {
      float s = 0.f;
      for (int i = 0; i < w.l1; ++i)
        s = fmaf(w.w2[(int64_t)o * w.l1 + i],
                 bn_c(w.bn1_w, w.bn1_b, w.bn1_mean, w.bn1_var, i, w.eps), s);
      v = w.b2[o] + s;
    }
    p.b2p[o] = v;
  }
  for (int o = t; o < p.OB * 32; o += gridDim.x * 256) {
    float v = 0.f;
    if (o < w.l3) {
      float s = 0.f;
      for (int i = 0; i < w.l2; ++i)
        s = fmaf(w.w3[(int64_t)o * w.l2 + i],
                 bn_c(w.bn2_w, w.bn2_b, w.bn2_mean, w.bn2_var, i, w.eps), s);
      v = w.b3[o] + s;
    }
    p.b3p[o] = v;
  }
  const int nlast = (p.OB > 0 ? p.OB : p.RB2) * 32;
  for (int o = t; o < nlast; o += gridDim.x * 256)
    p.wdp[o] = o < last ? wd[o] * bn_a(lg, lv, o, w.eps) : 0.f;
  if (t == 0) {
    float s = w.final_b[0];
    for (int o = 0; o < last; ++o) s = fmaf(wd[o], bn_c(lg, lb, lm, lv, o, w.eps), s);
    p.bias[0] = s;
  }
}

// per-user constant: folded bias + wide user weight (+ wide user-feature term)
__global__ void wd_user_const(hnm_widedeep_weights w, const int64_t* __restrict__ ids, int64_t B,
                              const float* __restrict__ wuf, const float* __restrict__ bias,
                              float* __restrict__ cu) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const int64_t u = ids[b];
  float v = bias[0];
  if (u >= 0 && u < w.num_users) v += w.wide_user[u];
  if (wuf) {
    const float* wf = w.wide_feat;
    for (int f = 0; f < w.num_user_features; ++f) v = fmaf(wuf[b * w.num_user_features + f], wf[f], v);
  }
  cu[b] = v;
}

// One wave's exact fp32 deep score for its user against a 32-item tile (the per-pair
// arithmetic of widedeep_score_kernel, shared with the certified path's re-scoring kernel
// so both produce bitwise the same values).  prow / qrow: the user's / lane item's
// pair-permuted layer-1 rows offset by h * K1P / 2 (LDS or global); returns the lane's
// half of w_d' . relu(layer 3) (the caller adds the other half with one shfl_xor 32).
template <int RB2, int OB>
__device__ __forceinline__ float wd_tile_fp32(const float* __restrict__ prow,
                                              const float* __restrict__ qrow, int S4,
                                              const float4* __restrict__ W2f,
                                              const float4* __restrict__ W3f,
                                              const float* __restrict__ cb2,
                                              const float* __restrict__ cb3,
                                              const float* __restrict__ cwd, int lane, int h) {
  constexpr int G2 = RB2 < 4 ? RB2 : 4;  // layer-2 row blocks per pass
  f32x16 acc3[OB > 0 ? OB : 1];
  float fin = 0.f;
#pragma unroll
  for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob)
    acc3[ob] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int g = 0; g < RB2 / G2; ++g) {
    f32x16 acc2[G2];
#pragma unroll
    for (int gi = 0; gi < G2; ++gi)
      acc2[gi] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // ---- layer 2 for row blocks g*G2 .. g*G2+G2-1
    float4 af[G2];
#pragma unroll
    for (int gi = 0; gi < G2; ++gi) af[gi] = W2f[((int64_t)(g * G2 + gi) * S4 + 0) * 64 + lane];
    for (int s4 = 0; s4 < S4; ++s4) {
      float4 an[G2];
      const int sn = s4 + 1 < S4 ? s4 + 1 : s4;
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) an[gi] = W2f[((int64_t)(g * G2 + gi) * S4 + sn) * 64 + lane];
      const float4 pv = *reinterpret_cast<const float4*>(prow + 4 * s4);
      const float4 qv = *reinterpret_cast<const float4*>(qrow + 4 * s4);
      const float x0 = fmaxf(pv.x + qv.x, 0.f), x1 = fmaxf(pv.y + qv.y, 0.f);
      const float x2 = fmaxf(pv.z + qv.z, 0.f), x3 = fmaxf(pv.w + qv.w, 0.f);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) acc2[gi] = mfma32x32x2(af[gi].x, x0, acc2[gi]);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) acc2[gi] = mfma32x32x2(af[gi].y, x1, acc2[gi]);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) acc2[gi] = mfma32x32x2(af[gi].z, x2, acc2[gi]);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) acc2[gi] = mfma32x32x2(af[gi].w, x3, acc2[gi]);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) af[gi] = an[gi];
    }
    // ---- relu(D2 + b2') feeds layer 3 (or the final dot for a two-layer tower).
    // Layer-3 A fragments are streamed one (gi, r4) step ahead; the scheduling barrier
    // keeps hipcc from hoisting all of them (which spills).
    float4 a3c[OB > 0 ? OB : 1], a3n[OB > 0 ? OB : 1];
    if (OB > 0) {
#pragma unroll
      for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob)
        a3c[ob] = W3f[((int64_t)(ob * RB2 + g * G2) * 4 + 0) * 64 + lane];
    }
#pragma unroll
    for (int gi = 0; gi < G2; ++gi) {
      const int rb = g * G2 + gi;
      float hv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) hv[r] = fmaxf(acc2[gi][r] + cb2[rb * 32 + mfma32_row(r, h)], 0.f);
      if (OB > 0) {
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int st = gi * 4 + r4;
          if (st + 1 < G2 * 4) {
            const int gn = (st + 1) >> 2, rn = (st + 1) & 3;
#pragma unroll
            for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob)
              a3n[ob] = W3f[((int64_t)(ob * RB2 + g * G2 + gn) * 4 + rn) * 64 + lane];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob) {
            acc3[ob] = mfma32x32x2(a3c[ob].x, hv[4 * r4 + 0], acc3[ob]);
            acc3[ob] = mfma32x32x2(a3c[ob].y, hv[4 * r4 + 1], acc3[ob]);
            acc3[ob] = mfma32x32x2(a3c[ob].z, hv[4 * r4 + 2], acc3[ob]);
            acc3[ob] = mfma32x32x2(a3c[ob].w, hv[4 * r4 + 3], acc3[ob]);
          }
#pragma unroll
          for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob) a3c[ob] = a3n[ob];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) fin = fmaf(hv[r], cwd[rb * 32 + mfma32_row(r, h)], fin);
      }
    }
  }
  if (OB > 0) {
#pragma unroll
    for (int ob = 0; ob < (OB > 0 ? OB : 1); ++ob) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = ob * 32 + mfma32_row(r, h);
        fin = fmaf(fmaxf(acc3[ob][r] + cb3[o], 0.f), cwd[o], fin);
      }
    }
  }
  return fin;
}

// ------------------------------------------------------------------ main kernel
template <int RB2, int OB, bool DENSE>
__global__ __launch_bounds__(256, (RB2 >= 8 || OB >= 4) ? 1 : 2) void widedeep_score_kernel(
    const float* __restrict__ Pu, const float* __restrict__ Qi, int K1P,
    const float4* __restrict__ W2f, const float4* __restrict__ W3f,
    const float* __restrict__ b2p, const float* __restrict__ b3p,
    const float* __restrict__ wdp, const float* __restrict__ cu, const float* __restrict__ wI,
    int64_t B, int64_t I, int64_t ipp, const int64_t* __restrict__ mptr,
    const int32_t* __restrict__ midx, int K, float* __restrict__ cand_v,
    int32_t* __restrict__ cand_i, int NP, float* __restrict__ dense, int64_t ldo,
    const int32_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KS1 = K1P / 2, S4 = K1P / 8, QRS = K1P + 4;
  float* qs = smem;                    // [32][QRS]
  float* ps = smem + WD_TILE * QRS;    // [4][K1P]
  float* cb2 = ps + 4 * K1P;           // [RB2*32] b2'
  float* cb3 = cb2 + RB2 * 32;         // [OB*32]  b3'
  float* cwd = cb3 + OB * 32;          // [32*max(OB,RB2)] w_d'

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  // rows (the certified path's fallback): slot -> batch row; outputs stay at the slot
  const int64_t slot = (int64_t)blockIdx.x * 4 + wave;
  const int64_t b = rows ? (slot < B ? (int64_t)rows[slot] : 0) : slot;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + ipp);

  for (int e = tid; e < 4 * K1P / 4; e += 256) {
    const int r = e / (K1P / 4), c = e % (K1P / 4);
    const int64_t bb = (int64_t)blockIdx.x * 4 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bb < B) v = *reinterpret_cast<const float4*>(Pu + (rows ? (int64_t)rows[bb] : bb) * K1P + 4 * c);
    *reinterpret_cast<float4*>(&ps[r * K1P + 4 * c]) = v;
  }
  for (int e = tid; e < RB2 * 32; e += 256) cb2[e] = b2p[e];
  for (int e = tid; e < OB * 32; e += 256) cb3[e] = b3p[e];
  for (int e = tid; e < (OB > 0 ? OB : RB2) * 32; e += 256) cwd[e] = wdp[e];
  const bool active = slot < B;
  const float cub = active ? cu[b] : 0.f;
  WaveTopK<1> L;
  L.init();
  int nm = WD_INT_BIG, mpos = 0, mend = 0;
  if (!DENSE && mptr && active) {
    int64_t lo = mptr[b], hi = mptr[b + 1];
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (midx[mid] < part_start) lo = mid + 1;
      else hi = mid;
    }
    mpos = (int)lo;
    mend = (int)mptr[b + 1];
    nm = mpos < mend ? midx[mpos] : WD_INT_BIG;
  }

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, WD_TILE) : 0;
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t base = part_start + t * WD_TILE;
    __syncthreads();  // previous tile's reads of qs are done
    for (int e = tid; e < WD_TILE * K1P / 4; e += 256) {
      const int r = e / (K1P / 4), c = e % (K1P / 4);
      const int64_t item = base + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (item < part_end) v = *reinterpret_cast<const float4*>(Qi + item * K1P + 4 * c);
      *reinterpret_cast<float4*>(&qs[r * QRS + 4 * c]) = v;
    }
    __syncthreads();
    if (!active) continue;

    const float* prow = &ps[wave * K1P + h * KS1];
    const float* qrow = &qs[j * QRS + h * KS1];
    float fin = wd_tile_fp32<RB2, OB>(prow, qrow, S4, W2f, W3f, cb2, cb3, cwd, lane, h);
    fin += __shfl_xor(fin, 32);
    const int64_t item = base + j;
    const bool ivalid = lane < 32 && item < part_end;
    float score = fin + cub + (ivalid ? wI[item] : 0.f);
    if (DENSE) {
      if (ivalid) dense[b * ldo + item] = score;
    } else {
      const int64_t tile_end = std::min<int64_t>(base + WD_TILE, part_end);
      while (nm < tile_end) {
        if (item == nm) score = -__builtin_inff();
        ++mpos;
        nm = mpos < mend ? midx[mpos] : WD_INT_BIG;
      }
      L.offer(score, (int)item, ivalid, K);
    }
  }
  if (!DENSE && active) L.store(cand_v + (slot * NP + p) * K, cand_i + (slot * NP + p) * K, K);
}

// ------------------------------------------------------------------ pairwise forward
// WideDeep.forward(user_ids, item_ids[, features]) (wide_deep.py:157-230): one workgroup per
// pair, the unfolded reference op order (Linear -> ReLU -> BatchNorm per layer).
__global__ __launch_bounds__(256) void widedeep_pair_kernel(
    hnm_widedeep_weights w, const int64_t* __restrict__ uids, const int64_t* __restrict__ iids,
    int64_t n, const float* __restrict__ xu, int ldxu, const float* __restrict__ wide_extra,
    const float* __restrict__ wide_extra2, float* __restrict__ out, unsigned* err) {
  __shared__ float x0[512], x1[512];
  __shared__ float red[256];
  const int64_t e = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t u = uids[e], i = iids[e];
  if (u < 0 || u >= w.num_users || i < 0 || i >= w.num_items) {
    if (t == 0) {
      hnm_flag(err, HNM_ERR_OOB);
      out[e] = __builtin_nanf("");
    }
    return;
  }
  const int din = w.l1_in;
  for (int c = t; c < din; c += 256) {
    float v;
    if (c < w.d) v = w.deep_user[u * w.d + c];
    else if (c < 2 * w.d) v = w.deep_item[i * w.d + c - w.d];
    else v = xu[e * ldxu + c - 2 * w.d];  // [deep user-feature | deep item-feature] chunks
    x0[c] = v;
  }
  __syncthreads();
  const int widths[3] = {w.l1, w.l2, w.l3};
  const float* W[3] = {w.w1, w.w2, w.w3};
  const float* Bs[3] = {w.b1, w.b2, w.b3};
  const float* G[3] = {w.bn1_w, w.bn2_w, w.bn3_w};
  const float* Be[3] = {w.bn1_b, w.bn2_b, w.bn3_b};
  const float* M[3] = {w.bn1_mean, w.bn2_mean, w.bn3_mean};
  const float* V[3] = {w.bn1_var, w.bn2_var, w.bn3_var};
  const int depth = w.l3 > 0 ? 3 : 2;
  float* cur = x0;
  float* nxt = x1;
  int in = din;
  for (int l = 0; l < depth; ++l) {
    for (int o = t; o < widths[l]; o += 256) {
      float s = 0.f;
      for (int k = 0; k < in; ++k) s = fmaf(W[l][(int64_t)o * in + k], cur[k], s);
      s = fmaxf(s + Bs[l][o], 0.f);
      s = (s - M[l][o]) / sqrtf(V[l][o] + w.eps) * G[l][o] + Be[l][o];
      nxt[o] = s;
    }
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
    in = widths[l];
    __syncthreads();
  }
  const float* wd = w.final_deep;
  float s = 0.f;
  for (int o = t; o < in; o += 256) s = fmaf(wd[o], cur[o], s);
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    // wide part in the reference's concat order: user one-hot, item one-hot (both absent
    // when use_wide_user_item=False), user-feature cross, item-feature cross
    float v = red[0];
    if (w.wide_user) v += w.wide_user[u];
    if (w.wide_item) v += w.wide_item[i];
    v += w.final_b[0];
    if (wide_extra) v += wide_extra[e];
    if (wide_extra2) v += wide_extra2[e];
    out[e] = v;
  }
}

// ------------------------------------------------------------------ certified f16x3 scan
// Wide&Deep top-K with a CERTIFIED split-f16 pre-filter and exact fp32 re-scoring.
//
// The fp32 MFMA rate is 1/16 of the f16 rate.  A plain f16 scan cannot prune W&D: its
// rigorous error bound (f16 rounding of every operand, propagated through |W3||W2|) spans
// a third of the score spread.  Split operands can: every f16 operand is x = x_hi + x_lo
// (x_hi = f16(x), x_lo = f16(x - x_hi)); layer 2 runs the f16 MFMA passes W_hi x_hi + W_hi x_lo,
// layer 3 W_hi x_hi only (WD_SPLIT_PASSES / WD_SPLIT_PASSES3), with fp32 accumulation: the
// activation's split error is 2^-22 (x_lo kept) or 2^-11 |x| (dropped), and the weights'
// residual R = W - W_hi (known, fixed per call) enters the bound exactly: (|R|^T v) . x.
// Nothing the scan computes is returned: it only prunes; every returned score is recomputed
// by wd_tile_fp32 (the fp32 kernel's own arithmetic), so outputs are bitwise those of the
// exact fp32 path (tests/test_gpu_prefilter.py).
//
// Bound (per pair, real units).  Let x1 = relu(P_u + Q_i) (the fp32 layer-1 values both
// paths read), x2 = relu(D2 + b2'), x3 = relu(D3 + b3') (this scan's values), and
// v3 = |w_d'|, v2 = |W3'|^T v3, v1 = |W2'|^T v2 (for a two-layer tower v2 = |w_d'|).
// The fp32 path's K-term fma chain errs by <= K u sum|terms| (u = 2^-24); the split path's
// MFMA chain by <= 6u (sum|terms| + |acc|) per MFMA (measured <= 3.4u:
// profiles/r1_mfma_semantics_probe.txt (c)) plus 3 * 2^-22 for the split operands; ReLU is
// 1-Lipschitz and errors propagate through |W|, so
//   |approx - exact| <= rho (g1 v1.x1 + g2 v2.x2 + g3 v3.x3 + g4 (|fin| + |c_u| + |w_I|)
//                            + cb) + absb
// and for the dropped passes v1 += (|R2|^T v2) / g1, v2 += (|R3|^T v3) / g2 (W_lo x_hi), and
// v2 *= 1 + 2^-11 / g2 for layer 3's dropped W_hi x_lo (wdc_params_kernel).
// with g1 = (2.125 K1 + 22)u, g2 = (2.125 n2 + 22)u (layer 3) or (32 RB2 + 12)u (final dot
// of a two-layer tower), g3 = (32 NOB + 10)u, g4 = 10u, cb the bias-add roundings, absb the
// f16 subnormal slack (2^-25 per rounding, scaled back), rho = 1 + 2^-6.  The v.x terms are
// three dot products per pair computed next to the MFMAs.
//
// Selection.  Each (user, item partition) keeps a wave-resident top-K of lower bounds
// lb = approx - e: its K-th is a lower bound of the exact K-th score at every moment, so an
// item is appended to the (user, partition) segment when ub = approx + e reaches it (every
// exact top-K item does).  The K-th of the merged lower-bound lists, L_u, filters the
// segments; the survivors (a few hundred per user) are re-scored in fp32.  Rows with an
// unusable bound, fewer than K finite items or an overflowing segment take the exact kernel.
typedef _Float16 wh8 __attribute__((ext_vector_type(8)));

// f16 MFMA passes per split layer: 3 = W_hi x_hi + W_hi x_lo + W_lo x_hi; 2 drops W_lo x_hi
// and bounds it explicitly: the dropped term of layer 2 is R2 x1 with R2 = W2' - W2'_hi the
// known residual of the f16 weights, so the bound adds (|R2|^T v2) . x1 (and (|R3|^T v3) . x2
// for layer 3), folded into v1 / v2 by wdc_params_kernel -- a per-element residual, about
// 2^-12.5 |W| on average instead of the 2^-11 worst case.
// Measured (random-init bench weights, 4,096 users x 105,542 items): 3/3 passes 392 ms (51
// candidates a row), 2/2 295 ms (360), **2/1 272-275 ms (393)**, 3/2 375 ms (56), 2/3 314 ms
// (349); one pass on layer 2 with x_lo bounded by 2^-11 |x| overflows every row's segments,
// with the per-pair exact x_lo term (v1o . |x - x_hi|, WD_SPLIT_PASSES = 1) it holds (788
// candidates a row) but runs 283 ms: at half the MFMAs the k loop's operand VALU bounds it.
// Round 3: one pass on layer 2 with the bound's layer-2 terms on the matrix pipe
// (WD_BOUND_MFMA below) and packed operand formation: 232 ms (1,145 candidates a row; their
// exact fp32 re-scoring ~14 ms) vs 2 passes 262-267 ms (393) -- W&D 15.1 k -> 16.5 k users/s
// (profiles/r3g_widedeep_ab.txt).
// The product (round 5: the alternatives above and below are gone from the source; git
// history and DESIGN.md §4 keep them): layer 2 and layer 3 one W_hi x_hi pass each, the
// layer-2 bound terms on the matrix pipe, the k loop in register-set pairs with the weight
// fragments two steps ahead, the accumulators pinned by asm.
// One-pass layer 2 (WD_SPLIT_PASSES = 1) with the bound's layer-2 terms on the matrix pipe: per k
// step and user two v_mfma_f32_16x16x32_f16 whose A rows 0 / 1 carry sb v1 (B = x_hi) and
// sb (v1 + 1.001 v1o / g1) (B = |x_lo|) for the items c / c + 16 of the 32x32 operand layout,
// rounded UP to f16 (wdc_boundfrag_kernel), accumulated over the first row-block pass only:
//   g1 v1.x + 1.001 v1o.|x - x_hi|  <=  g1 (v1.x_hi + (v1 + 1.001 v1o / g1).|x_lo|)
// (x = x_hi + x_lo exactly, |x_lo| rounded to f16 costs 2^-10 relative, in the A rows).  This
// replaces the 16 VALU fmas per user and k step that bound the VALU-bound one-pass kernel.
// (Measured and dropped, round 3: |x_lo| := 0 where z < 0 -- 789 instead of 1,145 candidates
// a row but a 5.7 ms slower scan, the same step; weight fragments three steps ahead.)

// one 16-B fragment per lane from a buffer: a uniform byte offset (SGPR) + lane * 16, so a
// fragment costs one scalar add instead of a 64-bit per-lane address (8 of those held across
// the k loop were spilled and reloaded every step, each reload's vmcnt wait also waiting for
// the prefetched fragments)
// Fragments are held as 4 x 32-bit registers and viewed as 8 f16 only at the MFMA: arrays of
// wh8 were merged into one <64 x half> value whose lane moves the backend emitted as
// v_bfi_b32 "copies" of freshly loaded fragments, each waiting for its load (the prefetch
// distance dropped to zero)
typedef unsigned wfr __attribute__((ext_vector_type(4)));
__device__ __forceinline__ wh8 wd_h(wfr f) { return __builtin_bit_cast(wh8, f); }
__device__ __forceinline__ wfr wd_frag(__amdgpu_buffer_rsrc_t rs, int lane, int byte_off) {
  return __builtin_bit_cast(wfr, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, byte_off, 0));
}

__device__ __forceinline__ f32x16 wd_mfma16(wh8 a, wh8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// One pass over k with every layer-2 row block (G2 = RB2 = 8, two users: 256 accumulator
// registers = the whole AGPR file).  Every other accumulator is pinned by inline asm so the
// compiler keeps layer 2's in place (left to it, it moved ~140 accumulator registers per k step
// between the files): the bound MFMAs' in VGPRs ("+v"), layer 3's in the AGPRs layer 2 has
// released ("=a" / "+a").  Layer 2's own MFMAs stay builtins: as asm they were issued in one
// block, with no vector work between them (a step then costs MFMA + VALU time, not the max).
// Wait states (nothing is padded inside an asm string): NOP = 2 states before an MFMA whose
// B operand a VALU instruction may just have written; an accumulate chain (C = the previous
// MFMA's D, same shape) needs none; the results -> any other reader: the s_nop fences after
// each loop.
// (As builtins the bound MFMAs cost 128 accumulator moves a step, measured.)
template <bool NOP>
__device__ __forceinline__ void wd_mfma16x_accv(f32x4& c, const wh8& a, const wh8& b) {
  if (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
// D = a b (C = 0), D in accumulator registers
template <bool NOP>
__device__ __forceinline__ void wd_mfma_acc0(f32x16& d, const wh8& a, const wh8& b) {
  if (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=a"(d) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=a"(d) : "v"(a), "v"(b));
}
// c += a b in place, c in accumulator registers
template <bool NOP>
__device__ __forceinline__ void wd_mfma_acc(f32x16& c, const wh8& a, const wh8& b) {
  if (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// c - (float)h for the low (SEL = 0) or high (SEL = 1) f16 half of a packed register: one
// v_fma_mix_f32 instead of a convert and a subtract (the split operand's remainder, exact)
template <int SEL>
__device__ __forceinline__ float wd_sub_half(unsigned packed, float c) {
  float d;
  if (SEL == 0)
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(packed), "v"(c));
  else
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(packed), "v"(c));
  return d;
}

// One-pass layer 2 operands from the unclamped layer-1 sums z (WD_BOUND_MFMA): per pair of
// elements one packed fma (z = q s1 + p), one RNE convert, one packed max: x_hi = relu(z)_hi
// (= max(f16(z), 0): rounding is monotonic), and |x_lo| = |f16(z - f16(z))| by v_fma_mix{lo,hi}
// (exact difference, one RNE rounding) + one and.  For z < 0 the true x_lo is 0, so |x_lo| here
// only over-estimates the bound term it feeds.  6 VALU per 2 elements instead of 9.
typedef _Float16 wh2 __attribute__((ext_vector_type(2)));
typedef float wf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wd_split_relu2(wf2 z, wh2& hi, unsigned& alo) {
  const wh2 hu = __builtin_convertvector(z, wh2);
  hi = __builtin_elementwise_max(hu, (wh2){(_Float16)0.f, (_Float16)0.f});
  const unsigned hub = __builtin_bit_cast(unsigned, hu);
  unsigned d;  // both halves written by the pair (no initialising move)
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(d) : "v"(hub), "v"(z.x), "v"(z.y));
  alo = d & 0x7fff7fffu;
}

// Split 8 fp32 values into f16 hi / lo halves: hi = f16(x), lo = f16(x - hi) (RNE; the
// remainder is exact in fp32).
__device__ __forceinline__ void wd_split8(const float* x, wh8& hi, wh8& lo) {
  typedef _Float16 wh2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    wh2 hp;
    hp[0] = (_Float16)x[e];
    hp[1] = (_Float16)x[e + 1];
    hi[e] = hp[0];
    hi[e + 1] = hp[1];
    lo[e] = (_Float16)__builtin_fmaf((float)hp[0], -1.f, x[e]);
    lo[e + 1] = (_Float16)__builtin_fmaf((float)hp[1], -1.f, x[e + 1]);
  }
}

struct WdCertParams {
  unsigned mx[2];       // max|P| over the batch rows, max|Q| over the items (float bits)
  float s1, sw2, s2, sw3;  // f16 operand scales (powers of two)
  float c2, c3;            // layer-2 accumulator -> x2 scale, layer-3 accumulator -> real
  float inv_s2;
  float g1, g2, g3, g4, cb, absb, rho;
  float sb, inv_sb;        // scale of the bound A rows (one-pass layer 2, WD_BOUND_MFMA)
  int bad;                 // bound unusable: every row takes the exact path
};

// pair-permuted position t of a layer-1 row -> layer-1 unit (hnm_linear_rows_f32 layout)
__device__ __forceinline__ int wd_korig(int t, int K1P) {
  const int half = K1P >> 1;
  return t < half ? 2 * t : 2 * (t - half) + 1;
}

__device__ __forceinline__ float wd_pow2_below_inv(float m) {  // largest 2^e with m 2^e <= 1
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, -e);
}

__device__ __forceinline__ float wd_nmax(float a, float b) { return (b > a || b != b) ? b : a; }

// per-block maxima of |P| (rows [0, B)) and |Q| (items) -> part[blk * 2 + {0, 1}]
__global__ __launch_bounds__(256) void wdc_stats_kernel(const float* __restrict__ Pu,
                                                        int64_t nP, const float* __restrict__ Qi,
                                                        int64_t nQ, float* __restrict__ part) {
  __shared__ float red[2][4];
  float mp = 0.f, mq = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; e < nP; e += stride) {
    const float4 v = *reinterpret_cast<const float4*>(Pu + e);
    mp = wd_nmax(mp, wd_nmax(wd_nmax(fabsf(v.x), fabsf(v.y)), wd_nmax(fabsf(v.z), fabsf(v.w))));
  }
  for (int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; e < nQ; e += stride) {
    const float4 v = *reinterpret_cast<const float4*>(Qi + e);
    mq = wd_nmax(mq, wd_nmax(wd_nmax(fabsf(v.x), fabsf(v.y)), wd_nmax(fabsf(v.z), fabsf(v.w))));
  }
  for (int o = 32; o >= 1; o >>= 1) {
    mp = wd_nmax(mp, __shfl_xor(mp, o));
    mq = wd_nmax(mq, __shfl_xor(mq, o));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = mp;
    red[1][wave] = mq;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    float m = red[threadIdx.x][0];
    for (int w = 1; w < 4; ++w) m = wd_nmax(m, red[threadIdx.x][w]);
    part[blockIdx.x * 2 + threadIdx.x] = m;
  }
}

// One block: bound vectors v1 (pair-permuted positions), v2, scales, coefficients.
__global__ __launch_bounds__(256) void wdc_params_kernel(hnm_widedeep_weights w, WdPrep p,
                                                         const float* __restrict__ part, int nblk,
                                                         float* __restrict__ v1,
                                                         float* __restrict__ v2,
                                                         float* __restrict__ b2s,
                                                         WdCertParams* prm,
                                                         float* __restrict__ v1o,
                                                         float* __restrict__ v2o) {
  __shared__ float sv2[256];
  __shared__ float red[8][4];
  __shared__ float bc[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K1P = p.K1P, n2 = p.RB2 * 32, NOB = p.OB > 0 ? p.OB : 1;
  const int l1 = w.l1, l2 = w.l2, l3 = w.l3;
  float mp = 0.f, mq = 0.f;
  for (int b = tid; b < nblk; b += 256) {
    mp = wd_nmax(mp, part[2 * b]);
    mq = wd_nmax(mq, part[2 * b + 1]);
  }
  // v2 (layer-2 rows): OB > 0: sum_m |W3'_mj| |wd'_m|; two-layer tower: |wd'_j|
  float mW3 = 0.f, sv2b = 0.f, swdb3 = 0.f, sumwd = 0.f;
  for (int jx = tid; jx < n2; jx += 256) {
    float v = 0.f;
    if (jx < l2) {
      if (p.OB > 0) {
        const float a2 = bn_a(w.bn2_w, w.bn2_var, jx, w.eps);
        for (int m = 0; m < l3; ++m) {
          const float wv = fabsf(w.w3[(int64_t)m * l2 + jx] * a2);
          mW3 = wd_nmax(mW3, wv);
          v = fmaf(wv, fabsf(p.wdp[m]), v);
        }
      } else {
        v = fabsf(p.wdp[jx]);
      }
    }
    sv2[jx] = v;
    v2[jx] = v;
    v2o[jx] = v;  // before the dropped-pass terms (the re-scoring cascade's three-pass tile)
    sv2b = fmaf(v, fabsf(p.b2p[jx]), sv2b);
  }
  for (int m = tid; m < NOB * 32; m += 256) {
    if (p.OB > 0) swdb3 = fmaf(fabsf(p.wdp[m]), fabsf(p.b3p[m]), swdb3);
    sumwd += fabsf(p.wdp[m]);
  }
  __syncthreads();
  // v1 (pair-permuted positions) and layer-2 row statistics
  float mW2 = 0.f, sv1 = 0.f;
  for (int t = tid; t < K1P; t += 256) {
    const int k = wd_korig(t, K1P);
    float v = 0.f;
    if (k < l1) {
      const float a1 = bn_a(w.bn1_w, w.bn1_var, k, w.eps);
      for (int jx = 0; jx < l2; ++jx) {
        const float wv = fabsf(w.w2[(int64_t)jx * l1 + k] * a1);
        mW2 = wd_nmax(mW2, wv);
        v = fmaf(wv, sv2[jx], v);
      }
    }
    v1[t] = v;
    v1o[t] = v;  // before the dropped-pass terms: the per-pair x_lo term of a one-pass layer 2
    sv1 += v;
  }
  const float zmax = mp + mq;
  float m2 = 0.f, sumv2 = 0.f;  // max_j (zmax sum_k |W2'_jk| + |b2'_j|)
  for (int jx = tid; jx < l2; jx += 256) {
    float rs = 0.f;
    for (int k = 0; k < l1; ++k)
      rs += fabsf(w.w2[(int64_t)jx * l1 + k] * bn_a(w.bn1_w, w.bn1_var, k, w.eps));
    m2 = wd_nmax(m2, fmaf(zmax, rs, fabsf(p.b2p[jx])));
    sumv2 += sv2[jx];
  }
  float vals[8] = {mp, mq, mW2, mW3, m2, sv1, sv2b, swdb3};
  for (int q = 0; q < 8; ++q) {
    float x = vals[q];
    for (int o = 32; o >= 1; o >>= 1) {
      const float y = __shfl_xor(x, o);
      x = q < 5 ? wd_nmax(x, y) : x + y;
    }
    if (lane == 0) red[q][wave] = x;
  }
  float sums2[2] = {sumv2, sumwd};
  for (int q = 0; q < 2; ++q)
    for (int o = 32; o >= 1; o >>= 1) sums2[q] += __shfl_xor(sums2[q], o);
  __shared__ float red2[2][4];
  if (lane == 0) {
    red2[0][wave] = sums2[0];
    red2[1][wave] = sums2[1];
  }
  __syncthreads();
  if (tid < 8) {
    float x = red[tid][0];
    for (int wv = 1; wv < 4; ++wv) x = tid < 5 ? wd_nmax(x, red[tid][wv]) : x + red[tid][wv];
    bc[tid] = x;
  }
  __syncthreads();
  const float M2 = bc[4];
  const float lim = 1.0e30f;
  bool bad = (K1P & 15) != 0;
  for (int q = 0; q < 8; ++q) bad |= !(bc[q] <= lim);
  const float F16R = 16384.f;  // scaled operand magnitudes <= 2^14
  const float s1 = bc[0] + bc[1] > 0.f ? F16R * wd_pow2_below_inv(bc[0] + bc[1]) : 1.f;
  const float sw2 = bc[2] > 0.f ? F16R * wd_pow2_below_inv(bc[2]) : 1.f;
  const float s2 = M2 > 0.f ? F16R * wd_pow2_below_inv(M2) : 1.f;
  const float sw3 = bc[3] > 0.f ? F16R * wd_pow2_below_inv(bc[3]) : 1.f;
  for (float sc : {s1, sw2, s2, sw3}) bad |= !(sc >= 1e-25f && sc <= 1e25f);
  // b2' in x2 units
  for (int jx = tid; jx < n2; jx += 256) b2s[jx] = p.b2p[jx] * s2;
  if (!bad) {
    // the dropped W_lo x_hi passes: v1 += (|R2|^T v2) / g1 and, with a
    // third layer, v2 += (|R3|^T v3) / g2, R = W' - f16(W' sw) / sw exactly as wdc_convert_kernel
    // rounds it; 1 + 2^-10 covers |x_hi| <= (1 + 2^-11)|x| and the fp32 sums.  Each thread
    // updates the entries it wrote above (same t / jx mapping).
    const float uu = 5.9604645e-08f;
    const float g1c = (2.125f * K1P + 22.f) * uu;
    const float g2c = (2.125f * n2 + 22.f) * uu;
    const float fr = 1.0009765625f;
    // one pass on layer 3 also drops W_hi x_lo: |x_lo| <= 2^-11 |x| (RNE), i.e. v2 += 2^-11 v2 /
    // g2; a one-pass layer 2 bounds its x_lo term per pair instead (scan: v1o . |x - x_hi|)
    const float xl1 = 0.f;
    const float xl3 = 4.8828125e-4f;
    for (int t = tid; t < K1P; t += 256) {
      const int k = wd_korig(t, K1P);
      if (k >= l1) continue;
      float r = 0.f;
      for (int jx = 0; jx < l2; ++jx) {
        float v = w.w2[(int64_t)jx * l1 + k] * bn_a(w.bn1_w, w.bn1_var, k, w.eps);
        v *= sw2;
        r = fmaf(fabsf(v - (float)(_Float16)v), sv2[jx], r);
      }
      v1[t] = v1[t] * (1.f + fr * xl1 / g1c) + fr * (r / sw2) / g1c;
    }
    if (p.OB > 0) {
      for (int jx = tid; jx < l2; jx += 256) {
        float r = 0.f;
        for (int m = 0; m < l3; ++m) {
          float v = w.w3[(int64_t)m * l2 + jx] * bn_a(w.bn2_w, w.bn2_var, jx, w.eps);
          v *= sw3;
          r = fmaf(fabsf(v - (float)(_Float16)v), fabsf(p.wdp[m]), r);
        }
        v2[jx] = v2[jx] * (1.f + fr * xl3 / g2c) + fr * (r / sw3) / g2c;
      }
    }
  }
  // scale of the bound A rows: max over k of v1 + (1.001 / g1) v1o, the larger row
  __shared__ float ared[4];
  __syncthreads();  // every thread's v1 / v1o entries are written
  float amax = 0.f;
  {
    const float g1c = (2.125f * K1P + 22.f) * 5.9604645e-08f;
    for (int t = tid; t < K1P; t += 256) amax = wd_nmax(amax, v1[t] + (1.0009765625f / g1c) * v1o[t]);
  }
  for (int o = 32; o >= 1; o >>= 1) amax = wd_nmax(amax, __shfl_xor(amax, o));
  if (lane == 0) ared[wave] = amax;
  __syncthreads();
  if (tid != 0) return;
  amax = wd_nmax(wd_nmax(ared[0], ared[1]), wd_nmax(ared[2], ared[3]));
  const float u = 5.9604645e-08f;  // 2^-24
  const float phi = 2.98023224e-08f;  // 2^-25: half the f16 subnormal spacing
  const float sumv2t = red2[0][0] + red2[0][1] + red2[0][2] + red2[0][3];
  const float sumwdt = red2[1][0] + red2[1][1] + red2[1][2] + red2[1][3];
  WdCertParams c;
  c.mx[0] = __float_as_uint(bc[0]);
  c.mx[1] = __float_as_uint(bc[1]);
  c.s1 = s1;
  c.sw2 = sw2;
  c.s2 = s2;
  c.sw3 = sw3;
  c.c2 = s2 / (s1 * sw2);
  c.c3 = 1.f / (s2 * sw3);
  c.inv_s2 = 1.f / s2;
  c.g1 = (2.125f * K1P + 22.f) * u;
  c.g2 = (p.OB > 0 ? 2.125f * n2 + 22.f : 32.f * p.RB2 + 12.f) * u;
  c.g3 = p.OB > 0 ? (32.f * NOB + 10.f) * u : 0.f;
  c.g4 = 10.f * u;
  c.cb = 4.f * u * (bc[6] + bc[7]);
  // subnormal slack: x1 / W2 / x2 / W3 roundings, 2 per operand (hi and lo), doubled
  c.absb = 4.f * phi *
           (bc[5] / s1 + sumv2t * K1P * (bc[0] + bc[1]) / sw2 + sumv2t / s2 +
            (p.OB > 0 ? sumwdt * n2 * M2 / sw3 : 0.f));
  c.rho = 1.015625f;
  c.sb = amax > 0.f ? 16384.f * wd_pow2_below_inv(amax * 1.01f) : 1.f;
  c.inv_sb = 1.f / c.sb;
  bad |= !(amax <= lim) || !(c.sb >= 1e-30f && c.sb <= 1e30f);
  bad |= !(c.absb <= lim) || !(c.c2 > 0.f && c.c2 <= lim) || !(c.c3 > 0.f && c.c3 <= lim);
  c.bad = bad;
  *prm = c;
}

// Split-f16 A operands.  W2hl[((rb * KB + kb) * 2 + hl) * 64 + lane][t]: row rb*32 +
// (lane & 31), pair-permuted position 16 kb + 8 (lane >> 5) + t; W3hl[((ob * 2 RB2 + kb3) *
// 2 + hl) * 64 + lane][t]: row ob*32 + (lane & 31), layer-2 row (kb3 >> 1) * 32 +
// mfma32_row(8 (kb3 & 1) + t, lane >> 5) -- the order in which layer 2's accumulator
// registers become layer 3's B operand.
__global__ __launch_bounds__(256) void wdc_convert_kernel(hnm_widedeep_weights w, WdPrep p,
                                                          const WdCertParams* __restrict__ prm,
                                                          wh8* __restrict__ W2hl,
                                                          wh8* __restrict__ W3hl) {
  const int K1P = p.K1P, KB = K1P / 16;
  const float sw2 = prm->sw2, sw3 = prm->sw3;
  const int64_t n2 = (int64_t)p.RB2 * KB * 64, n3 = (int64_t)p.OB * 2 * p.RB2 * 64;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n2 + n3;
       e += (int64_t)gridDim.x * 256) {
    const int lane = (int)(e & 63), h = lane >> 5, r = lane & 31;
    wh8 hi, lo;
    if (e < n2) {
      const int64_t q = e >> 6;
      const int kb = (int)(q % KB), rb = (int)(q / KB);
      const int o = rb * 32 + r;
      for (int t = 0; t < 8; ++t) {
        const int k = wd_korig(16 * kb + 8 * h + t, K1P);
        float v = 0.f;
        if (o < w.l2 && k < w.l1) v = w.w2[(int64_t)o * w.l1 + k] * bn_a(w.bn1_w, w.bn1_var, k, w.eps);
        v *= sw2;
        const _Float16 vh = (_Float16)v;
        hi[t] = vh;
        lo[t] = (_Float16)(v - (float)vh);
      }
      W2hl[(q * 2 + 0) * 64 + lane] = hi;
      W2hl[(q * 2 + 1) * 64 + lane] = lo;
    } else {
      const int64_t q = (e - n2) >> 6;
      const int kb3 = (int)(q % (2 * p.RB2)), ob = (int)(q / (2 * p.RB2));
      const int o = ob * 32 + r;
      for (int t = 0; t < 8; ++t) {
        const int jx = (kb3 >> 1) * 32 + mfma32_row(8 * (kb3 & 1) + t, h);
        float v = 0.f;
        if (o < w.l3 && jx < w.l2) v = w.w3[(int64_t)o * w.l2 + jx] * bn_a(w.bn2_w, w.bn2_var, jx, w.eps);
        v *= sw3;
        const _Float16 vh = (_Float16)v;
        hi[t] = vh;
        lo[t] = (_Float16)(v - (float)vh);
      }
      W3hl[(q * 2 + 0) * 64 + lane] = hi;
      W3hl[(q * 2 + 1) * 64 + lane] = lo;
    }
  }
}

// f16 rounded toward +inf (for v >= 0: every bound operand is nonnegative)
__device__ __forceinline__ _Float16 wd_f16_up(float v) {
  _Float16 h = (_Float16)v;
  if ((float)h < v) h = __builtin_bit_cast(_Float16, (unsigned short)(__builtin_bit_cast(unsigned short, h) + 1));
  return h;
}

// Bound A fragments of the one-pass layer 2 (WD_BOUND_MFMA): WBf[(typ * KB + kb) * 64 + lane], the
// 16x16x32 A operand (lane l holds A[l & 15][8 (l >> 4) + t]).  Row 0 takes the k-groups of items
// c (lane groups 0 / 2 of the 32x32 B layout: k = 16 kb + 8 (g >> 1) + t), row 1 those of items
// c + 16 (groups 1 / 3); every other entry is 0.  typ 0 multiplies x_hi: sb v1; typ 1 multiplies
// |x_lo|: sb (v1 + 1.001 v1o / g1) (1 + 2^-10) -- the 2^-10 covers |x_lo|'s f16 rounding, the
// 2^-20 the fp32 evaluation; rounded up.
__global__ __launch_bounds__(256) void wdc_boundfrag_kernel(const WdCertParams* __restrict__ prm,
                                                            const float* __restrict__ v1,
                                                            const float* __restrict__ v1o, int K1P,
                                                            wh8* __restrict__ WBf) {
  const int KB = K1P / 16;
  const float sb = prm->sb;
  const float c1 = 1.0009765625f / ((2.125f * K1P + 22.f) * 5.9604645e-08f);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < KB * 2 * 64; e += gridDim.x * 256) {
    const int lane = e & 63, q = e >> 6, kb = q % KB, typ = q / KB;
    const int row = lane & 15, g = lane >> 4;
    wh8 out = {};
    if (row == (g & 1)) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int k = 16 * kb + 8 * (g >> 1) + t;
        const float v = typ == 0 ? v1[k] : (v1[k] + c1 * v1o[k]) * (1.0009765625f * 1.00000095367f);
        out[t] = wd_f16_up(v * sb);
      }
    }
    WBf[e] = out;
  }
}

struct WdScanArgs {
  const float* Pu;  // [B, K1P]  pair-permuted layer-1 user part (+ b1)
  const float* Qi;  // [I, K1P]  pair-permuted layer-1 item part
  int K1P;
  const wh8* W2hl;
  const wh8* W3hl;
  const wh8* WBf;    // [KB * 2 * 64] bound A fragments (WD_BOUND_MFMA)
  const float* v1;   // [K1P]
  const float* v1o;  // [K1P] v1 without the dropped-pass terms (one-pass layer 2)
  const float* v2;   // [RB2*32]
  const float* b2s;  // [RB2*32] b2' s2
  const float* b3p;  // [OB*32]
  const float* wdp;  // [NL*32]
  const float* cu;   // [B] per-user constant
  const float* wI;   // [I] wide item weight
  const WdCertParams* prm;
  int64_t B, I, ipp;
  int NP;
  const int64_t* mptr;
  const int32_t* midx;
  int K;
  float* lbv;    // [B, NP, K] lower-bound lists
  int32_t* lbi;
  int32_t* segi;  // [B, NP, cap] appended items
  float* segu;    // [B, NP, cap] their upper bounds
  int* cnt;       // [B, NP]
  int cap;
  float* dbg_a;   // DEBUG: [B, lda] approx score, bound
  float* dbg_e;
  int64_t lda;
};

#define WDC_THRESH 0
#define WDC_DEBUG 1
#define WDC_VPM 4  // VALU instructions scheduled per MFMA in the k loop's interleave
#define WDC_G2 8   // layer-2 row blocks per pass over k (the x operands are formed once per pass)
#ifndef WD_STAMPS  // diagnostic builds only: per-phase s_memtime cycle sums (tools/wd_stamps.py)
#define WD_STAMPS 0
#endif
#if WD_STAMPS
__device__ unsigned long long wd_stamp_acc[4];  // k loop, layer-2 epilogue + layer 3, final, tiles
extern "C" int hnm_debug_wd_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(wd_stamp_acc), sizeof(wd_stamp_acc));
}
extern "C" int hnm_debug_wd_stamps_reset() {
  const unsigned long long z[4] = {0, 0, 0, 0};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(wd_stamp_acc), z, sizeof(z));
}
#endif

// Block = 4 waves x UPW users each (rows blockIdx.x * 4 UPW + wave * UPW + v) x item
// partition blockIdx.y; the Q tile (32 items, fp32) is shared through LDS.  Per tile a wave
// runs layer 2 as RB2 x K1P/16 f16 MFMAs per user (one W_hi x_hi pass; G2 row blocks per pass
// over k, the next layer fed from the accumulators as each pass completes), layer 3 as
// OB x 2 RB2, then the bound.  UPW = 2: every weight fragment loaded from
// L2 feeds two users' MFMAs -- the fragment stream is what bounds the one-user variant
// (tools/wd_ablation.sh: no weight loads = -19% time).  Round 3 product: G2 = RB2 = 8, one
// pass over k (the x operands, most of the k loop's vector work, formed once per tile instead
// of once per pass: 217 -> 160-164 ms), layer 2's 256 accumulators in the AGPR file, layer 3
// after all of layer 2 (ASMACC below).
template <int RB2, int OB, int G2, int MODE, int UPW>
__global__ __launch_bounds__(256, UPW == 1 ? 2 : 1) void wdc_scan_kernel(WdScanArgs A) {
  constexpr int NOB = OB > 0 ? OB : 1;
  constexpr int NL = OB > 0 ? OB : RB2;
  constexpr int NU = 4 * UPW;  // users per block
  constexpr bool ASMACC = G2 == RB2;  // accumulators pinned by asm (the 8 x 4 product shape)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K1P = A.K1P, KB = K1P / 16, QRS = K1P + 4;
  float* qs = smem;               // [32][QRS]
  float* ps = qs + 32 * QRS;      // [NU][K1P]
  float* b2l = ps + NU * K1P;     // [RB2*32]
  float* v2l = b2l + RB2 * 32;    // [RB2*32]
  float* b3l = v2l + RB2 * 32;    // [NOB*32]
  float* wdl = b3l + NOB * 32;    // [NL*32]
  // qs / qn (offset qn_off): the Q tile being scored and the next one, filled during its k loop
  const int qn_off = (int)(wdl + NL * 32 - smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  const __amdgpu_buffer_rsrc_t w2rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.W2hl, 0, RB2 * KB * 2 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t wbrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.WBf, 0, KB * 2 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t w3rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.W3hl, 0, NOB * 2 * RB2 * 2 * 1024, 0x00020000);
  const int64_t ublk = (int64_t)blockIdx.x * NU;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * A.ipp;
  const int64_t part_end = std::min<int64_t>(A.I, part_start + A.ipp);
  // P and Q are staged pre-scaled by s1 (a power of two: relu(s1 p + s1 q) = s1 relu(p + q)
  // exactly), so the k loop forms the f16 operands without a multiply
  const float s1 = A.prm->s1, inv_s1 = 1.f / s1;
  for (int e = tid; e < NU * K1P / 4; e += 256) {
    const int r = e / (K1P / 4), c = e % (K1P / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ublk + r < A.B) v = *reinterpret_cast<const float4*>(A.Pu + (ublk + r) * K1P + 4 * c);
    v.x *= s1; v.y *= s1; v.z *= s1; v.w *= s1;
    *reinterpret_cast<float4*>(ps + r * K1P + 4 * c) = v;
  }
  for (int e = tid; e < RB2 * 32; e += 256) {
    b2l[e] = A.b2s[e];
    v2l[e] = A.v2[e];
  }
  for (int e = tid; e < NOB * 32; e += 256) b3l[e] = OB > 0 ? A.b3p[e] : 0.f;
  for (int e = tid; e < NL * 32; e += 256) wdl[e] = A.wdp[e];
  const float c2 = A.prm->c2, c3 = A.prm->c3, inv_s2 = A.prm->inv_s2;
  const float g1 = A.prm->g1, g2 = A.prm->g2, g3 = A.prm->g3, g4 = A.prm->g4;
  const float cbd = A.prm->cb, absb = A.prm->absb, rho = A.prm->rho;

  int64_t bu[UPW];
  bool act[UPW];
  float cub[UPW];
  WaveTopK<1> L[UPW];
  int nm[UPW], mpos[UPW], mend[UPW], count[UPW];
#pragma unroll
  for (int v = 0; v < UPW; ++v) {
    bu[v] = ublk + wave * UPW + v;
    act[v] = bu[v] < A.B;
    cub[v] = act[v] ? A.cu[bu[v]] : 0.f;
    L[v].init();
    nm[v] = WD_INT_BIG;
    mpos[v] = mend[v] = count[v] = 0;
    if (A.mptr && act[v]) {
      int64_t lo = A.mptr[bu[v]], hi = A.mptr[bu[v] + 1];
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (A.midx[mid] < part_start) lo = mid + 1;
        else hi = mid;
      }
      mpos[v] = (int)lo;
      mend[v] = (int)A.mptr[bu[v] + 1];
      nm[v] = mpos[v] < mend[v] ? A.midx[mpos[v]] : WD_INT_BIG;
    }
  }

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, WD_TILE) : 0;
  // Q tiles are double-buffered: tile t + 1 is copied into the other buffer while tile t is
  // scored, one 8-column slice of its 32 rows per k step (K1P / 8 = NG KB / QPS steps; a
  // thread moves one dword of row tid / 8): step s writes the slice loaded during step s - 1
  // and loads slice s + 1 -- no exposed load latency, one barrier a tile, no branches in the
  // k loop (kernel 270 -> 261 ms; the tile load + barrier it replaces cost 6 %).  The loads are
  // buffer loads over the next tile's valid rows (a scalar column offset; rows past the
  // partition, and the slice after the last, read as 0 by the bounds check).  Q is staged
  // unscaled: the k loop forms s1 x1 = fma(q, s1, p s1), which rounds exactly like s1 (p + q)
  // (s1 is a power of two; scaling in the copy instead, one more VALU a step: 275 ms).
  constexpr int NG = RB2 / G2, QPS = 2 / NG;
  static_assert(NG * QPS == 2, "one tile's copy spans the tile's k steps");
  const int qrow_t = tid >> 3, qcol_t = tid & 7;
  const int qvoff = (qrow_t * K1P + qcol_t) * 4;
  auto qrsrc = [&](int64_t nb) {  // the tile at nb: its rows inside the partition
    const int64_t rows = std::max<int64_t>(0, std::min<int64_t>(WD_TILE, part_end - nb));
    const float* src = A.Qi + std::min<int64_t>(nb, part_end - 1) * K1P;
    return __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)(rows * K1P * 4), 0x00020000);
  };
  auto qload = [&](__amdgpu_buffer_rsrc_t rs, int c) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, qvoff, c * 4, 0));
  };
  if (ntiles > 0) {
    const __amdgpu_buffer_rsrc_t rs = qrsrc(part_start);
    for (int c = 0; c < K1P; c += 8) smem[qrow_t * QRS + qcol_t + c] = qload(rs, c);
  }
  unsigned long long st_acc[4] = {0, 0, 0, 0}, st_t0 = 0, st_t1 = 0;
  for (int64_t t = 0; t < ntiles; ++t) {
    if (WD_STAMPS) st_t0 = __builtin_amdgcn_s_memtime();
    const int64_t base = part_start + t * WD_TILE;
    const int cur_off = (t & 1) ? qn_off : 0, nxt_off = (t & 1) ? 0 : qn_off;
    const __amdgpu_buffer_rsrc_t qrs = qrsrc(base + WD_TILE);
    float* const qdst = smem + nxt_off + qrow_t * QRS + qcol_t;
    __syncthreads();
    if (!act[0]) {  // users are assigned in order: the wave has none, it only copies
      for (int c = 0; c < K1P; c += 8) qdst[c] = qload(qrs, c);
      continue;
    }
    float qv[QPS];
#pragma unroll
    for (int e = 0; e < QPS; ++e) qv[e] = qload(qrs, 8 * e);

    const float* qrow = smem + cur_off + j * QRS + 8 * h;
    f32x16 acc3[UPW][NOB];
    float fin[UPW], bx2[UPW], bx3[UPW];
#pragma unroll
    for (int v = 0; v < UPW; ++v) fin[v] = bx2[v] = bx3[v] = 0.f;
    // the bound's layer-2 terms on the matrix pipe: 16x16 accumulators, rows 0 / 1
    // of lanes 0-15 = items c / c + 16
    f32x4 accb[UPW];
#pragma unroll
    for (int v = 0; v < UPW; ++v) accb[v] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one pass over k per G2 row blocks (NG passes); the bound MFMAs: with NG = 2 pass 0 takes
    // the x_hi rows, pass 1 the |x_lo| rows (one 16x16x32 MFMA per user and k step each); NG = 1
    // both.  One loop body for every pass: duplicating it for the passes spilled 300+ registers
    constexpr int NG2 = RB2 / G2;
    static_assert(NG2 <= 2, "bound MFMA split assumes at most two row-block passes");
#pragma unroll 1
    for (int g = 0; g < NG2; ++g) {
      f32x16 acc2[UPW][G2];
#pragma unroll
      for (int v = 0; v < UPW; ++v)
#pragma unroll
        for (int gi = 0; gi < G2; ++gi)
          acc2[v][gi] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      // k loop, software-pipelined: the f16 operands of step kb + 1 (LDS reads, relu, split:
      // ~45 VALU per user) are formed while step kb's 3 G2 UPW MFMAs run -- one wave per
      // SIMD issues ~5 VALU per 32-cycle MFMA gap nearly for free (MI355X_MICROARCH.md,
      // cycle constants), so a step costs its MFMAs instead of VALU + MFMA.  hi weight
      // fragments are prefetched one step ahead, lo fragments at the top of their step (first
      // used 2 G2 UPW MFMAs later).
      auto frag = [&](int gi, int kk, int hl) {
        const int q = ((g * G2 + gi) * KB + kk) * 2;
        return wd_frag(w2rs, lane, (q + hl) * 1024);
      };
      // x_hi and |x_lo| of step kk (the layer-2 MFMAs' and the bound MFMAs' B operands), packed
      auto form = [&](int kk, wh8* oh, wh8* ol) {
        const float4 q0 = *reinterpret_cast<const float4*>(qrow + 16 * kk);
        const float4 q1 = *reinterpret_cast<const float4*>(qrow + 16 * kk + 4);
#pragma unroll
        for (int v = 0; v < UPW; ++v) {
          const float* prow = ps + (wave * UPW + v) * K1P + 8 * h + 16 * kk;
          const float4 p0 = *reinterpret_cast<const float4*>(prow);
          const float4 p1 = *reinterpret_cast<const float4*>(prow + 4);
          {
            const wf2 s2v = {s1, s1};
            const wf2 zq[4] = {{q0.x, q0.y}, {q0.z, q0.w}, {q1.x, q1.y}, {q1.z, q1.w}};
            const wf2 zp[4] = {{p0.x, p0.y}, {p0.z, p0.w}, {p1.x, p1.y}, {p1.z, p1.w}};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              wh2 hi;
              unsigned alo;
              wd_split_relu2(__builtin_elementwise_fma(zq[e], s2v, zp[e]), hi, alo);
              const wh2 lo2 = __builtin_bit_cast(wh2, alo);
              oh[v][2 * e] = hi[0];
              oh[v][2 * e + 1] = hi[1];
              ol[v][2 * e] = lo2[0];
              ol[v][2 * e + 1] = lo2[1];
            }
          }
        }
      };
      // the weight and bound fragments of step kb + 2 are loaded into the registers step kb's
      // MFMAs have just read -- a two-step prefetch distance with two register sets (the
      // one-pass step is half as long as a two-pass one, so one step ahead left its MFMAs
      // waiting on L2)
      auto stepd = [&](int kb, wfr (&a)[G2], const wh8 (&xh)[UPW], const wh8 (&xl)[UPW],
                       wh8 (&nxh)[UPW], wh8 (&nxl)[UPW], wfr (&bq)[2]) {
        const bool more = kb + 1 < KB;
        const int kn = more ? kb + 1 : kb;
        const int kf = kb + 2 < KB ? kb + 2 : KB - 1;
#pragma unroll
        for (int gi = 0; gi < G2; ++gi)
#pragma unroll
          for (int v = 0; v < UPW; ++v) {
            acc2[v][gi] = wd_mfma16(wd_h(a[gi]), xh[v], acc2[v][gi]);
          }
#pragma unroll
        for (int v = 0; v < UPW; ++v) {
          if constexpr (ASMACC && NG2 == 1) {
            wd_mfma16x_accv<true>(accb[v], wd_h(bq[0]), xh[v]);
            wd_mfma16x_accv<true>(accb[v], wd_h(bq[1]), xl[v]);
          } else if (NG2 == 1) {
            accb[v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wd_h(bq[0]), xh[v], accb[v], 0, 0, 0);
            accb[v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wd_h(bq[1]), xl[v], accb[v], 0, 0, 0);
          } else {
            const wh8 bop = g == 0 ? xh[v] : xl[v];
            accb[v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wd_h(bq[0]), bop, accb[v], 0, 0, 0);
          }
        }
#pragma unroll
        for (int gi = 0; gi < G2; ++gi) a[gi] = frag(gi, kf, 0);
        bq[0] = wd_frag(wbrs, lane, (int)(((NG2 == 1 ? 0 : g) * KB + kf)) * 1024);
        if (NG2 == 1) bq[1] = wd_frag(wbrs, lane, (int)((KB + kf)) * 1024);
        form(kn, nxh, nxl);
#pragma unroll
        for (int e = 0; e < QPS; ++e) {
          const int c = 8 * ((g * KB + kb) * QPS + e);
          qdst[c] = qv[e];
          qv[e] = qload(qrs, c + 8 * QPS);
        }
        // the next step's LDS reads first, then one MFMA + WDC_VPM VALU at a time (2+1 passes:
        // 268-272 ms; 2, 3, 5, 6, 8 VALU per MFMA 305-315 ms, compiler order 331 ms)
        __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * UPW, 0);
#pragma unroll
        for (int i = 0; i < G2 * UPW + (3 - NG2) * UPW; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, WDC_VPM, 0);
        }
      };
      wfr fa[G2], fb[G2], ba[2], bb[2];
      wh8 xha[UPW], xla[UPW], xhb[UPW], xlb[UPW];
      form(0, xha, xla);
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) fa[gi] = frag(gi, 0, 0);
      {
        const int k1 = KB > 1 ? 1 : 0;
#pragma unroll
        for (int gi = 0; gi < G2; ++gi) fb[gi] = frag(gi, k1, 0);
        const int bo = (NG2 == 1 ? 0 : g) * KB;
        ba[0] = wd_frag(wbrs, lane, (int)(bo) * 1024);
        bb[0] = wd_frag(wbrs, lane, (int)((bo + k1)) * 1024);
        if (NG2 == 1) {
          ba[1] = wd_frag(wbrs, lane, (int)(KB) * 1024);
          bb[1] = wd_frag(wbrs, lane, (int)((KB + k1)) * 1024);
        }
      }
      {
        // steps in pairs with the two register sets swapped (the one-pass kernel is issue-bound:
        // copying one set into the other was 28 v_mov per step)
        int kb = 0;
        for (; kb + 1 < KB; kb += 2) {
          stepd(kb, fa, xha, xla, xhb, xlb, ba);
          stepd(kb + 1, fb, xhb, xlb, xha, xla, bb);
        }
        if (kb < KB) stepd(kb, fa, xha, xla, xhb, xlb, ba);
      }
      if constexpr (ASMACC) {
        // the last MFMAs' results -> any reader: 8-pass XDL, 12+ wait states; the fence names
        // every accumulator so no read is scheduled above it
        asm volatile("s_nop 7\n\ts_nop 7");
#pragma unroll
        for (int v = 0; v < UPW; ++v)
#pragma unroll
          for (int gi = 0; gi < G2; ++gi) asm volatile("" : "+a"(acc2[v][gi]));
#pragma unroll
        for (int v = 0; v < UPW; ++v) asm volatile("" : "+v"(accb[v]));
        if (WD_STAMPS) {
          st_t1 = __builtin_amdgcn_s_memtime();
          st_acc[0] += st_t1 - st_t0;
        }
      }
      if (G2 < RB2 && g == 0) {  // zeroed after the k loop (G2 = RB2: by the first MFMA's C = 0)
#pragma unroll
        for (int v = 0; v < UPW; ++v)
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob)
            acc3[v][ob] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      }
      // One pass over k (G2 = RB2) with a layer 3: every row block's x2 first (its f16 B operand
      // kept in 8 registers per row block and user, its bound term summed), then layer 3 -- so
      // layer 3's accumulators take the registers of layer 2's, which are all dead by then
      // (one phase per row block kept both sets live and spilled).
      if constexpr (G2 == RB2 && OB > 0) {
        // in halves of RH row blocks: x2 of the half's blocks (their f16 B operands, their
        // bound terms), then their layer-3 MFMAs -- layer 3's accumulators take the registers of
        // the first half's layer-2 ones (all 256 accumulator registers hold layer 2 until then)
        constexpr int RH = RB2 >= 2 ? RB2 / 2 : 1;
        // the bias / bound rows are loop-invariant LDS reads: an opaque offset per tile keeps
        // them from being hoisted out of the tile loop (256 registers held across it: spilled)
        int lz = 0;
        asm volatile("" : "+v"(lz));
        const float* b2t = b2l + lz;
        const float* v2t = v2l + lz;
        const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // layer 3's weight fragments, W3D row-block halves (kb3 steps) ahead of their MFMAs: the
        // first ones are in flight while layer 2's accumulators are converted
        constexpr int W3D = 2, NK3 = 2 * RB2;
        wfr w3b[W3D + 1][NOB];
        auto w3load = [&](int kb3) {
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob) {
            const int q = (ob * 2 * RB2 + kb3) * 2;
            w3b[kb3 % (W3D + 1)][ob] = wd_frag(w3rs, lane, q * 1024);
          }
        };
#pragma unroll
        for (int k3 = 0; k3 < W3D && k3 < NK3; ++k3) w3load(k3);
#pragma unroll
        for (int r0 = 0; r0 < RB2; r0 += RH) {
          wh8 yh_h[UPW][RH][2];
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) {
            // one row block at a time: hoisting every block's accumulator reads needs 256 VGPRs
            __builtin_amdgcn_sched_barrier(0);
            const int rb = r0 + rr;
            float bias16[16], vv16[16];
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
              const float4 bb = *reinterpret_cast<const float4*>(b2t + rb * 32 + 8 * r4 + 4 * h);
              const float4 vq = *reinterpret_cast<const float4*>(v2t + rb * 32 + 8 * r4 + 4 * h);
              bias16[4 * r4] = bb.x; bias16[4 * r4 + 1] = bb.y; bias16[4 * r4 + 2] = bb.z; bias16[4 * r4 + 3] = bb.w;
              vv16[4 * r4] = vq.x; vv16[4 * r4 + 1] = vq.y; vv16[4 * r4 + 2] = vq.z; vv16[4 * r4 + 3] = vq.w;
            }
#pragma unroll
            for (int v = 0; v < UPW; ++v) {
              // four independent chains (a nonnegative sum: its rounding is inside rho in any
              // order) instead of one 16-deep dependent chain per row block
              float part[4] = {bx2[v], 0.f, 0.f, 0.f};
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                const float y = fmaxf(fmaf(acc2[v][rb][r], c2, bias16[r]), 0.f);
                part[r & 3] = fmaf(vv16[r], y, part[r & 3]);
                yh_h[v][rr][r >> 3][r & 7] = (_Float16)y;
              }
              bx2[v] = (part[0] + part[1]) + (part[2] + part[3]);
              // the bound sum is due here: otherwise it is sunk to its use after layer 3,
              // holding every fp32 x2 value live (spilled)
              asm volatile("" : "+v"(bx2[v]));
            }
          }
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) {
#pragma unroll
            for (int half2 = 0; half2 < 2; ++half2) {
              __builtin_amdgcn_sched_barrier(0);
              const int kb3 = 2 * (r0 + rr) + half2;
              if (kb3 + W3D < NK3) w3load(kb3 + W3D);
              const wfr* bh = w3b[kb3 % (W3D + 1)];
              const bool first = r0 == 0 && rr == 0 && half2 == 0;
#pragma unroll
              for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
                for (int v = 0; v < UPW; ++v) {
                  if constexpr (ASMACC) {
                    if (first) {
                      if (ob == 0) wd_mfma_acc0<true>(acc3[v][ob], wd_h(bh[ob]), yh_h[v][rr][half2]);
                      else wd_mfma_acc0<false>(acc3[v][ob], wd_h(bh[ob]), yh_h[v][rr][half2]);
                    } else {
                      if (ob == 0) wd_mfma_acc<true>(acc3[v][ob], wd_h(bh[ob]), yh_h[v][rr][half2]);
                      else wd_mfma_acc<false>(acc3[v][ob], wd_h(bh[ob]), yh_h[v][rr][half2]);
                    }
                  } else {
                    acc3[v][ob] = wd_mfma16(wd_h(bh[ob]), yh_h[v][rr][half2], first ? zero16 : acc3[v][ob]);
                  }
                }
            }
          }
        }
        if constexpr (ASMACC) {  // layer 3's results -> the VALU readers below
          asm volatile("s_nop 7\n\ts_nop 7");
#pragma unroll
          for (int v = 0; v < UPW; ++v)
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) asm volatile("" : "+a"(acc3[v][ob]));
        }
        if (WD_STAMPS) {
          const unsigned long long t2 = __builtin_amdgcn_s_memtime();
          st_acc[1] += t2 - st_t1;
          st_t1 = t2;
        }
        continue;
      }
      // x2 = relu(D2 + b2') in s2 units feeds layer 3 (or the final dot)
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) {
        // fence: keeps the scheduler from hoisting every row block's layer-3 fragment loads
        // (G2 = 8: 64 x 16 B a lane) above the first block's MFMAs
        if (G2 == RB2) __builtin_amdgcn_sched_barrier(0);
        const int rb = g * G2 + gi;
        float y[UPW][16];
        float bias16[16], vv16[16];
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {  // rows 8 r4 + 4 h + 0..3: one 16-B read each
          const float4 bb = *reinterpret_cast<const float4*>(b2l + rb * 32 + 8 * r4 + 4 * h);
          const float4 vq = *reinterpret_cast<const float4*>(v2l + rb * 32 + 8 * r4 + 4 * h);
          bias16[4 * r4] = bb.x; bias16[4 * r4 + 1] = bb.y; bias16[4 * r4 + 2] = bb.z; bias16[4 * r4 + 3] = bb.w;
          vv16[4 * r4] = vq.x; vv16[4 * r4 + 1] = vq.y; vv16[4 * r4 + 2] = vq.z; vv16[4 * r4 + 3] = vq.w;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rb * 32 + mfma32_row(r, h);
          const float bias = bias16[r], vv = vv16[r], wv = wdl[OB == 0 ? row : 0];
#pragma unroll
          for (int v = 0; v < UPW; ++v) {
            y[v][r] = fmaxf(fmaf(acc2[v][gi][r], c2, bias), 0.f);
            bx2[v] = fmaf(vv, y[v][r], bx2[v]);
            if (OB == 0) fin[v] = fmaf(y[v][r], wv, fin[v]);
          }
        }
        if (OB > 0) {
#pragma unroll
          for (int half2 = 0; half2 < 2; ++half2) {
            wh8 yh[UPW], yl[UPW];
#pragma unroll
            for (int v = 0; v < UPW; ++v) wd_split8(&y[v][8 * half2], yh[v], yl[v]);
            const int kb3 = 2 * rb + half2;
            wh8 bh[NOB];
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) {
              const int q = (ob * 2 * RB2 + kb3) * 2;
              bh[ob] = wd_h(wd_frag(w3rs, lane, q * 1024));
            }
            // G2 = RB2: the chain starts at the first row block with C = 0 (an inline constant),
            // so acc3 becomes live only as acc2's registers are consumed
            const bool first = G2 == RB2 && gi == 0 && half2 == 0;
            const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
              for (int v = 0; v < UPW; ++v)
                acc3[v][ob] = wd_mfma16(bh[ob], yh[v], first ? zero16 : acc3[v][ob]);

          }
        }
      }
    }
    const int64_t item = base + j;
    const bool ivalid = lane < 32 && item < part_end;
    const float wi = ivalid ? A.wI[item] : 0.f;
    const int64_t tile_end = std::min<int64_t>(base + WD_TILE, part_end);
#pragma unroll
    for (int v = 0; v < UPW; ++v) {
      if (OB > 0) {
        // four independent chains each (at most 16 NOB + 3 roundings on any path, within the
        // 32 NOB of g3) instead of two 16 NOB-deep dependent chains
        float fp[4] = {fin[v], 0.f, 0.f, 0.f}, bp[4] = {bx3[v], 0.f, 0.f, 0.f};
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) {
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const float4 b3 = *reinterpret_cast<const float4*>(b3l + ob * 32 + 8 * r4 + 4 * h);
            const float4 w4 = *reinterpret_cast<const float4*>(wdl + ob * 32 + 8 * r4 + 4 * h);
            const float bq[4] = {b3.x, b3.y, b3.z, b3.w}, wq[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float z = fmaxf(fmaf(acc3[v][ob][4 * r4 + e], c3, bq[e]), 0.f);
              fp[e] = fmaf(z, wq[e], fp[e]);
              bp[e] = fmaf(fabsf(wq[e]), z, bp[e]);
            }
          }
        }
        fin[v] = (fp[0] + fp[1]) + (fp[2] + fp[3]);
        bx3[v] = (bp[0] + bp[1]) + (bp[2] + bp[3]);
      } else {
        fin[v] *= inv_s2;
      }
      const float fv = hnm_sum_halves(fin[v]);
      // item j's row of the bound accumulators: lane j (< 16) row 0, lane j - 16 row 1; the
      // layer-2 x_lo term is inside (the A rows of the |x_lo| operand)
      const float d0 = __shfl(accb[v][0], lane & 15), d1 = __shfl(accb[v][1], lane & 15);
      const float b1 = ((lane & 31) < 16 ? d0 : d1) * (A.prm->inv_sb * inv_s1);
      const float bl1 = 0.f;
      const float b2 = hnm_sum_halves(bx2[v]);
      const float b3 = hnm_sum_halves(bx3[v]);
      const float score = fv + cub[v] + wi;
      const float e = rho * (g1 * b1 + bl1 + g2 * (b2 * inv_s2) + g3 * b3 +
                             g4 * (fabsf(fv) + fabsf(cub[v]) + fabsf(wi)) + cbd) + absb;
      bool masked = false;
      while (nm[v] < tile_end) {
        if (item == nm[v]) masked = true;
        ++mpos[v];
        nm[v] = mpos[v] < mend[v] ? A.midx[mpos[v]] : WD_INT_BIG;
      }
      if (!act[v]) continue;
      if (MODE == WDC_DEBUG) {
        if (ivalid) {
          A.dbg_a[bu[v] * A.lda + item] = score;
          A.dbg_e[bu[v] * A.lda + item] = e;
        }
        continue;
      }
      const bool ok = ivalid && !masked;
      const float lb = score - e, ub = score + e;
      L[v].offer(lb, (int)item, ok, A.K);
      const bool app = ok && ub >= L[v].thr_v;
      const uint64_t m = __ballot(app);
      const int pos = count[v] + __popcll(m & ((1ull << lane) - 1));
      const int64_t seg = (bu[v] * A.NP + p) * (int64_t)A.cap;
      if (app && pos < A.cap) {
        A.segi[seg + pos] = (int32_t)item;
        A.segu[seg + pos] = ub;
      }
      count[v] += __popcll(m);
    }
    if (WD_STAMPS) {
      const unsigned long long t3 = __builtin_amdgcn_s_memtime();
      st_acc[2] += t3 - st_t1;
      st_acc[3] += t3 - st_t0;
    }
  }
  if (WD_STAMPS && lane == 0) {
#if WD_STAMPS
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&wd_stamp_acc[i], st_acc[i]);
#endif
  }
  if (MODE == WDC_THRESH) {
#pragma unroll
    for (int v = 0; v < UPW; ++v) {
      if (!act[v]) continue;
      L[v].store(A.lbv + (bu[v] * A.NP + p) * A.K, A.lbi + (bu[v] * A.NP + p) * A.K, A.K);
      if (lane == 0) A.cnt[bu[v] * A.NP + p] = count[v];
    }
  }
}

struct WdRescoreArgs {
  const float* Pu;
  const float* Qi;
  int K1P;
  const float4* W2f;
  const float4* W3f;
  const float* b2p;
  const float* b3p;
  const float* wdp;
  const float* cu;
  const float* wI;
  const WdCertParams* prm;
  int64_t B;
  int NP, K, cap;
  const float* Lk;   // [B, K] merged lower-bound lists (slot K-1 = L_u)
  int32_t* segi;     // [B, NP * cap] the scan's segments; wdc_collect compacts each row's
  float* segu;       //   survivors to its front (items, then the refined upper bounds)
  float* segl;       // [B, NP * cap] the survivors' refined lower bounds
  const int* cnt;
  int* ns;           // [B] survivors of each row; -1: the row takes the exact kernel
  int* toff;         // [B + 1] exclusive prefix of the rows' refining tiles (toff[B] = total)
  int32_t* fbrows;   // rows that take the exact kernel
  int* nfb;
  float* ov;
  int64_t* oi;
  unsigned long long* stats;  // HNM_OPT_STATS: rows, candidates re-scored in fp32, fallback rows
  // the refining stage (three-pass split-f16 tile, wd_tile_f16x3)
  const wh8* W2hl;
  const wh8* W3hl;
  const float* v1p;  // [K1P] plain v1 (no dropped-pass terms)
  const float* v2p;  // [RB2*32] plain v2
  const float* b2s;  // [RB2*32] b2' s2
  int64_t rstride;   // row stride of segi / segu / segl (NP * cap)
  float* segs;       // [B, NP * cap] the survivors' SCAN upper bounds, compacted by wdc_collect
  const int* rstart; // refining stage: row b's tiles start at position rstart[b] (nullptr: 0)
  float* dbg_a;      // hnm_widedeep_refine_debug_f32: refined score / bound per item, [B, lda]
  float* dbg_e;
  int64_t lda;
};

// Refined certified score of the re-scoring cascade (round 5): one user against the 32 gathered
// items of a tile (lane (j, h): item j), both layers as three split-f16 MFMA passes
// (W_hi x_hi + W_hi x_lo + W_lo x_hi; the dropped W_lo x_lo is 2^-22 relative), fp32
// accumulation -- the configuration the header's g1 / g2 constants were derived for, so the
// bound there holds with the PLAIN v1 / v2 (the scan's one-pass vectors carry dropped-pass
// terms): |approx - exact| <= e.  About 3/16 of the fp32 tile's matrix-pipe time.  Layer 2 in
// RB2 / G2 passes over k of G2 row blocks each (the x operands re-formed per pass), each pass's
// x2 feeding layer 3 at once: G2 = 4 keeps the tile within 256 registers (two waves a SIMD).
//   psr: the user's layer-1 row scaled by s1, offset 8 h (LDS); qrow: item j's row + 8 h
//   (global); v1s / b2l / v2l / b3l / wdl: LDS copies.  Returns (score - cu - wI) in every lane
//   and the bound's three dot products (real units, summed over the halves).
template <int RB2, int OB, int G2>
__device__ __forceinline__ void wd_tile_f16x3(const float* __restrict__ psr,
                                              const float* __restrict__ qrow, int KB,
                                              __amdgpu_buffer_rsrc_t w2rs,
                                              __amdgpu_buffer_rsrc_t w3rs,
                                              const float* __restrict__ v1s,
                                              const float* __restrict__ b2l,
                                              const float* __restrict__ v2l,
                                              const float* __restrict__ b3l,
                                              const float* __restrict__ wdl, float s1, float c2,
                                              float c3, float inv_s2, int lane, int h,
                                              float& fv, float& b1, float& b2, float& b3) {
  constexpr int NOB = OB > 0 ? OB : 1;
  f32x16 acc3[NOB];
#pragma unroll
  for (int ob = 0; ob < NOB; ++ob)
    acc3[ob] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float bx1 = 0.f, bx2 = 0.f, fin = 0.f, bx3 = 0.f;
  auto qload = [&](int kb, float4 (&q)[2]) {
    q[0] = *reinterpret_cast<const float4*>(qrow + 16 * kb);
    q[1] = *reinterpret_cast<const float4*>(qrow + 16 * kb + 4);
  };
#pragma unroll 1
  for (int g = 0; g < RB2 / G2; ++g) {
    f32x16 acc2[G2];
#pragma unroll
    for (int gi = 0; gi < G2; ++gi)
      acc2[gi] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // item rows two k steps ahead (gathered rows); each weight fragment is reloaded for step
    // kb + 1 right after step kb's MFMAs read it (one register set, a whole step of lead)
    wfr w[G2][2];
#pragma unroll
    for (int gi = 0; gi < G2; ++gi)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) w[gi][hl] = wd_frag(w2rs, lane, ((g * G2 + gi) * KB * 2 + hl) * 1024);
    auto step = [&](int kb, const float4 (&q)[2]) {
      const float4 p0 = *reinterpret_cast<const float4*>(psr + 16 * kb);
      const float4 p1 = *reinterpret_cast<const float4*>(psr + 16 * kb + 4);
      const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
      const float qv[8] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w};
      float x[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) x[t] = fmaxf(fmaf(qv[t], s1, pv[t]), 0.f);  // s1 x1 exactly
      if (g == 0) {  // the layer-2 bound term, once
        const float4 w0 = *reinterpret_cast<const float4*>(v1s + 16 * kb + 8 * h);
        const float4 w1 = *reinterpret_cast<const float4*>(v1s + 16 * kb + 8 * h + 4);
        const float vv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int t = 0; t < 8; ++t) bx1 = fmaf(vv[t], x[t], bx1);
      }
      wh8 xh, xl;
      wd_split8(x, xh, xl);
      const int kn = kb + 1 < KB ? kb + 1 : kb;
#pragma unroll
      for (int gi = 0; gi < G2; ++gi) {
        acc2[gi] = wd_mfma16(wd_h(w[gi][0]), xh, acc2[gi]);
        acc2[gi] = wd_mfma16(wd_h(w[gi][0]), xl, acc2[gi]);
        acc2[gi] = wd_mfma16(wd_h(w[gi][1]), xh, acc2[gi]);
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          w[gi][hl] = wd_frag(w2rs, lane, (((g * G2 + gi) * KB + kn) * 2 + hl) * 1024);
      }
    };
    {
      // item rows QD k steps ahead: four register sets in rotation (the gathered rows come from
      // MALL / HBM; two steps of lead left the MFMAs waiting on them)
      constexpr int QD = 4;
      float4 qr[QD][2];
      auto kc = [&](int k) { return k < KB ? k : KB - 1; };
#pragma unroll
      for (int d = 0; d < QD; ++d) qload(kc(d), qr[d]);
      int kb = 0;
      for (; kb + QD <= KB; kb += QD) {
#pragma unroll
        for (int d = 0; d < QD; ++d) {
          step(kb + d, qr[d]);
          qload(kc(kb + d + QD), qr[d]);
        }
      }
#pragma unroll
      for (int d = 0; d < QD; ++d)
        if (kb + d < KB) step(kb + d, qr[d]);
    }
    // x2 = relu(D2 + b2') in s2 units, its bound term, then its layer-3 passes (or the final
    // dot of a two-layer tower).  Layer-3 fragments run W3D kb3 steps ahead in a ring of
    // W3D + 1 register sets (the steps are unrolled: compile-time slots); bias / bound rows are
    // read as float4 (rows 8 r4 + 4 h + 0..3 of a row block hold registers 4 r4 .. 4 r4 + 3).
    constexpr int W3D = 2, NK3 = 2 * G2;
    wfr w3b[W3D + 1][NOB][2];
    auto w3load = [&](int k3) {  // k3: this pass's kb3 step (2 gi + half2)
      const int kb3 = 2 * g * G2 + k3;
#pragma unroll
      for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          w3b[k3 % (W3D + 1)][ob][hl] = wd_frag(w3rs, lane, ((ob * 2 * RB2 + kb3) * 2 + hl) * 1024);
    };
    if constexpr (OB > 0) {
#pragma unroll
      for (int k3 = 0; k3 < W3D && k3 < NK3; ++k3) w3load(k3);
    }
#pragma unroll
    for (int gi = 0; gi < G2; ++gi) {
      const int rb = g * G2 + gi;
      float y[16];
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 bb = *reinterpret_cast<const float4*>(b2l + rb * 32 + 8 * r4 + 4 * h);
        const float4 vq = *reinterpret_cast<const float4*>(v2l + rb * 32 + 8 * r4 + 4 * h);
        const float bq[4] = {bb.x, bb.y, bb.z, bb.w}, vv[4] = {vq.x, vq.y, vq.z, vq.w};
        float wq[4] = {0.f, 0.f, 0.f, 0.f};
        if (OB == 0) {
          const float4 w4 = *reinterpret_cast<const float4*>(wdl + rb * 32 + 8 * r4 + 4 * h);
          wq[0] = w4.x; wq[1] = w4.y; wq[2] = w4.z; wq[3] = w4.w;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * r4 + e;
          y[r] = fmaxf(fmaf(acc2[gi][r], c2, bq[e]), 0.f);
          bx2 = fmaf(vv[e], y[r], bx2);
          if (OB == 0) fin = fmaf(y[r], wq[e], fin);
        }
      }
      if constexpr (OB > 0) {
#pragma unroll
        for (int half2 = 0; half2 < 2; ++half2) {
          const int k3 = 2 * gi + half2;
          if (k3 + W3D < NK3) w3load(k3 + W3D);
          wh8 yh, yl;
          wd_split8(&y[8 * half2], yh, yl);
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob) {
            const wh8 bh = wd_h(w3b[k3 % (W3D + 1)][ob][0]);
            const wh8 bl = wd_h(w3b[k3 % (W3D + 1)][ob][1]);
            acc3[ob] = wd_mfma16(bh, yh, acc3[ob]);
            acc3[ob] = wd_mfma16(bh, yl, acc3[ob]);
            acc3[ob] = wd_mfma16(bl, yh, acc3[ob]);
          }
        }
      }
    }
  }
  if constexpr (OB > 0) {
    float fp[4] = {0.f, 0.f, 0.f, 0.f}, bp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 b3 = *reinterpret_cast<const float4*>(b3l + ob * 32 + 8 * r4 + 4 * h);
        const float4 w4 = *reinterpret_cast<const float4*>(wdl + ob * 32 + 8 * r4 + 4 * h);
        const float bq[4] = {b3.x, b3.y, b3.z, b3.w}, wq[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float z = fmaxf(fmaf(acc3[ob][4 * r4 + e], c3, bq[e]), 0.f);
          fp[e] = fmaf(z, wq[e], fp[e]);
          bp[e] = fmaf(fabsf(wq[e]), z, bp[e]);
        }
      }
    fin = (fp[0] + fp[1]) + (fp[2] + fp[3]);
    bx3 = (bp[0] + bp[1]) + (bp[2] + bp[3]);
  } else {
    fin *= inv_s2;
  }
  fv = hnm_sum_halves(fin);
  b1 = hnm_sum_halves(bx1) / s1;
  b2 = hnm_sum_halves(bx2) * inv_s2;
  b3 = hnm_sum_halves(bx3);
}

// The re-scoring cascade (round 5; round 4 sent all ~1,145 scan survivors a row through the
// fp32 tile: 15.7 ms a batch):
//   wdc_collect_kernel  one wave per row: fallback rows queued; the row's scan survivors
//                       (ub >= L_u) compacted to the front of its segment area, their count;
//   wdc_best_kernel     (round 6) one wave per row: the refining list's first phase -- the
//                       WDC_BF survivors of best scan upper bound (rows of <= WDC_BF_MIN: all);
//   wdc_tiles_kernel    exclusive prefix of the rows' 32-item refining tiles (one block);
//   wdc_refine_kernel   a fixed grid, each wave a contiguous run of tiles (balanced whatever
//                       the rows' survivor counts): wd_tile_f16x3 -> refined bounds
//                       lb2 <= exact <= ub2 per listed survivor;
//   wdc_filter_kernel   (round 6) one wave per row: the remaining survivors whose scan upper
//                       bound reaches the first phase's K-th refined lower bound appended to
//                       the list, then tiles + refine again over them (~1,145 -> ~570 refined
//                       a row at configs[3]: profiles/r10c_wd_best_first_probe.txt);
//   wdc_rescore_kernel  one wave per row: L2 = the K-th best lb2 (a lower bound of the row's
//                       exact K-th best), then the survivors with ub2 >= max(L2, L_u) -- every
//                       item that can be in the top-K -- through wd_tile_fp32, the exact
//                       kernel's arithmetic, into a wave top-K: bitwise the exact path's output.
__global__ __launch_bounds__(256) void wdc_collect_kernel(WdRescoreArgs R) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= R.B) return;
  const float Lu = R.Lk[b * R.K + R.K - 1];
  bool fb = R.prm->bad || !(Lu > -__builtin_inff());
  for (int p = 0; p < R.NP; ++p) fb |= R.cnt[b * R.NP + p] > R.cap;
  if (fb) {
    if (lane == 0) {
      R.ns[b] = -1;
      R.fbrows[atomicAdd(R.nfb, 1)] = (int32_t)b;
      if (R.stats) {
        atomicAdd(R.stats + 0, 1ull);
        atomicAdd(R.stats + 2, 1ull);
      }
    }
    return;
  }
  // in place: the write position never passes the read position, and a chunk's loads are
  // issued before its stores
  const int64_t rowbase = b * R.rstride;
  int no = 0;
  for (int p = 0; p < R.NP; ++p) {
    const int n = R.cnt[b * R.NP + p];
    const int64_t base = rowbase + (int64_t)p * R.cap;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int e = c0 + lane;
      const bool in = e < n;
      const int32_t it = in ? R.segi[base + e] : 0;
      const float u = in ? R.segu[base + e] : 0.f;
      const bool ok = in && u >= Lu;
      const uint64_t m = __ballot(ok);
      if (ok) {
        const int64_t o = rowbase + no + __popcll(m & ((1ull << lane) - 1));
        R.segi[o] = it;
        R.segs[o] = u;  // a separate array: the scan's upper bounds are read in place above
      }
      no += __popcll(m);
    }
  }
  if (lane == 0) R.ns[b] = no;
}

__global__ __launch_bounds__(1024) void wdc_tiles_kernel(const int* __restrict__ ns,
                                                         const int* __restrict__ start, int64_t B,
                                                         int* __restrict__ toff) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < B; b0 += 1024) {
    const int64_t b = b0 + tid;
    const int t = b < B ? (int)hnm_cdiv(std::max(ns[b] - (start ? start[b] : 0), 0), WD_TILE) : 0;
    int incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    if (b < B) toff[b] = before + incl - t;
    __syncthreads();
    if (tid == 1023) carry = before + incl;
    __syncthreads();
  }
  if (tid == 0) toff[B] = carry;
}

template <int RB2, int OB>
__global__ __launch_bounds__(256, 1) void wdc_refine_kernel(WdRescoreArgs R) {
  constexpr int NOB = OB > 0 ? OB : 1, NL = OB > 0 ? OB : RB2;
  constexpr int G2 = RB2;
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const int K1P = R.K1P, KB = K1P / 16;
  float* const v1s = wsm;                  // [K1P]
  float* const b2l = v1s + K1P;            // [RB2 * 32]
  float* const v2l = b2l + RB2 * 32;       // [RB2 * 32]
  float* const b3l = v2l + RB2 * 32;       // [NOB * 32]
  float* const wdl = b3l + NOB * 32;       // [NL * 32]
  float* const psm = wdl + NL * 32;        // [4][K1P] the wave's current user row, scaled by s1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  for (int e = tid; e < K1P; e += 256) v1s[e] = R.v1p[e];
  for (int e = tid; e < RB2 * 32; e += 256) {
    b2l[e] = R.b2s[e];
    v2l[e] = R.v2p[e];
  }
  for (int e = tid; e < NOB * 32; e += 256) b3l[e] = OB > 0 ? R.b3p[e] : 0.f;
  for (int e = tid; e < NL * 32; e += 256) wdl[e] = R.wdp[e];
  __syncthreads();  // the only block-level barrier
  const WdCertParams& P = *R.prm;
  const float s1 = P.s1, c2 = P.c2, c3 = P.c3, inv_s2 = P.inv_s2;
  const float g1 = P.g1, g2 = P.g2, g3 = P.g3, g4 = P.g4, cbd = P.cb, absb = P.absb, rho = P.rho;
  const __amdgpu_buffer_rsrc_t w2rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)R.W2hl, 0, RB2 * KB * 2 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t w3rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)R.W3hl, 0, NOB * 2 * RB2 * 2 * 1024, 0x00020000);
  // this wave's tiles: a contiguous run of the T tiles (rows in order)
  const int64_t T = R.toff[R.B];
  const int64_t nw = (int64_t)gridDim.x * 4, w = (int64_t)blockIdx.x * 4 + wave;
  const int64_t t0 = T * w / nw, t1 = T * (w + 1) / nw;
  if (t0 >= t1) return;
  int64_t lo = 0, hi = R.B;  // the row holding tile t0: last b with toff[b] <= t0
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (R.toff[mid] <= t0) lo = mid;
    else hi = mid;
  }
  int64_t b = lo, cb = -1;
  float* const ps = psm + wave * K1P;
  float cub = 0.f;
  for (int64_t t = t0; t < t1; ++t) {
    while (R.toff[b + 1] <= t) ++b;  // rows without tiles are skipped
    if (b != cb) {
      __builtin_amdgcn_wave_barrier();
      for (int e = lane; e < K1P; e += 64) ps[e] = R.Pu[b * K1P + e] * s1;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      cub = R.cu[b];
      cb = b;
    }
    const int k = (int)(t - R.toff[b]);
    const int st = R.rstart ? R.rstart[b] : 0;
    const int nv = std::min(WD_TILE, R.ns[b] - st - WD_TILE * k);
    const int64_t at = b * R.rstride + st + (int64_t)WD_TILE * k;
    const bool ivalid = lane < 32 && j < nv;
    const int it = R.segi[at + (j < nv ? j : 0)];
    float fv, b1, b2, b3;
    wd_tile_f16x3<RB2, OB, G2>(ps + 8 * h, R.Qi + (int64_t)it * K1P + 8 * h, KB, w2rs, w3rs, v1s,
                               b2l, v2l, b3l, wdl, s1, c2, c3, inv_s2, lane, h, fv, b1, b2, b3);
    const float wi = R.wI[it];
    const float score = fv + cub + wi;
    const float e = rho * (g1 * b1 + g2 * b2 + g3 * b3 +
                           g4 * (fabsf(fv) + fabsf(cub) + fabsf(wi)) + cbd) + absb;
    if (ivalid) {
      if (R.dbg_a) {
        R.dbg_a[b * R.lda + it] = score;
        R.dbg_e[b * R.lda + it] = e;
      } else {
        R.segl[at + j] = score - e;
        R.segu[at + j] = score + e;
      }
    }
  }
}

// Best-first refining (round 6).  A row of more than WDC_BF_MIN survivors
// refines its WDC_BF survivors of best scan upper bound first (wdc_best_kernel); their K-th best
// refined lower bound L2' is a certified lower bound of the row's exact K-th, so a remaining
// survivor is refined only if its scan upper bound reaches max(L2', L_u) (wdc_filter_kernel):
// otherwise exact <= scan ub < L2' <= the exact K-th, and it cannot be in the top-K.  The rows'
// refining lists (cli: the first phase, then the filtered rest) replace the survivor lists in
// the refining stage and in wdc_rescore_kernel, whose output is unchanged (bitwise the exact
// path).  Rows of at most WDC_BF_MIN survivors refine them all in the first phase.
constexpr int WDC_BF = 64;
constexpr int WDC_BF_MIN = 96;

// one wave per row: cli[0, nA) = the first phase's items (the WDC_BF best by (scan ub desc,
// survivor position asc), or every survivor), tv / tg = the WDC_BF-th (ub, position)
__global__ __launch_bounds__(256) void wdc_best_kernel(WdRescoreArgs R, int32_t* __restrict__ cli,
                                                       int* __restrict__ nA,
                                                       float* __restrict__ tv,
                                                       int* __restrict__ tg) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= R.B) return;
  const int ns = R.ns[b];
  const int64_t rowbase = b * R.rstride;
  if (ns <= WDC_BF_MIN) {  // incl. the exact kernel's rows (-1)
    for (int e = lane; e < ns; e += 64) cli[rowbase + e] = R.segi[rowbase + e];
    if (lane == 0) nA[b] = ns;
    return;
  }
  float v0 = -__builtin_inff();
  int i0 = HNM_SENTINEL_IDX;
  for (int c0 = 0; c0 < ns; c0 += 64) {  // running WDC_BF best; survivors' ubs are finite
    const int g = c0 + lane;
    float v1 = g < ns ? R.segs[rowbase + g] : -__builtin_inff();
    int i1 = g < ns ? g : HNM_SENTINEL_IDX;
    const float c63 = hnm_readlane_f(v0, 63);
    const int c63i = hnm_readlane_i(i0, 63);
    if (__ballot(hnm_better(v1, i1, c63, c63i))) hnm_sort128(v0, i0, v1, i1);
  }
  cli[rowbase + lane] = R.segi[rowbase + i0];
  if (lane == 63) {
    tv[b] = v0;
    tg[b] = i0;
  }
  if (lane == 0) nA[b] = WDC_BF;
}

// one wave per row (after the first phase's refining): L2' from the first phase's refined lower
// bounds; the remaining survivors with scan ub >= max(L2', L_u) appended to cli; ns = the list's
// final length
__global__ __launch_bounds__(256) void wdc_filter_kernel(WdRescoreArgs R, int32_t* __restrict__ cli,
                                                         const float* __restrict__ tv,
                                                         const int* __restrict__ tg) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= R.B) return;
  const int ns = R.ns[b];
  if (ns <= WDC_BF_MIN) return;  // single phase (or the exact kernel's row): the list is complete
  const int K = R.K;
  const int64_t rowbase = b * R.rstride;
  WaveTopK<1> T2;  // K <= 64 = WDC_BF distinct items
  T2.init();
  T2.offer(R.segl[rowbase + lane], cli[rowbase + lane], true, K);
  const float thr = fmaxf(T2.thr_v, R.Lk[b * K + K - 1]);
  const float v64 = tv[b];
  const int g64 = tg[b];
  int no = WDC_BF;
  for (int c0 = 0; c0 < ns; c0 += 64) {
    const int g = c0 + lane;
    const bool in = g < ns;
    const float u = in ? R.segs[rowbase + g] : -__builtin_inff();
    const bool first = u > v64 || (u == v64 && g <= g64);  // refined in the first phase
    const bool keep = in && !first && u >= thr;
    const uint64_t m = __ballot(keep);
    if (keep) cli[rowbase + no + __popcll(m & ((1ull << lane) - 1))] = R.segi[rowbase + g];
    no += __popcll(m);
  }
  if (lane == 0) R.ns[b] = no;
}

template <int RB2, int OB>
__global__ __launch_bounds__(256, 1) void wdc_rescore_kernel(WdRescoreArgs R) {
  __shared__ int stage[4][96];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  if (b >= R.B) return;  // no block-level barriers below
  const int ns = R.ns[b];
  if (ns < 0) return;  // queued for the exact kernel by wdc_collect
  const int K = R.K;
  const float Lu = R.Lk[b * K + K - 1];
  const int64_t rowbase = b * R.rstride;
  // L2: the K-th best refined lower bound (K distinct items)
  WaveTopK<1> T2;
  T2.init();
  for (int c0 = 0; c0 < ns; c0 += 64) {
    const int e = c0 + lane;
    const bool in = e < ns;
    T2.offer(in ? R.segl[rowbase + e] : -__builtin_inff(), in ? R.segi[rowbase + e] : 0, in, K);
  }
  const float thr = fmaxf(T2.thr_v, Lu);
  const int KS1 = R.K1P / 2, S4 = R.K1P / 8;
  const float cub = R.cu[b];
  const float* prow = R.Pu + b * R.K1P + h * KS1;
  int* st = stage[wave];
  WaveTopK<1> T;
  T.init();
  int nsurv = 0, nst = 0;
  auto run_tile = [&](int nv) {
    const int it = st[j < nv ? j : 0];
    const float* qrow = R.Qi + (int64_t)it * R.K1P + h * KS1;
    float fin = wd_tile_fp32<RB2, OB>(prow, qrow, S4, R.W2f, R.W3f, R.b2p, R.b3p, R.wdp, lane, h);
    fin += __shfl_xor(fin, 32);
    const bool ivalid = lane < 32 && j < nv;
    const float score = fin + cub + (ivalid ? R.wI[it] : 0.f);
    T.offer(score, it, ivalid, K);
  };
  for (int c0 = 0; c0 < ns; c0 += 64) {
    const int e = c0 + lane;
    const bool ok = e < ns && R.segu[rowbase + e] >= thr;
    const uint64_t m = __ballot(ok);
    if (ok) st[nst + __popcll(m & ((1ull << lane) - 1))] = R.segi[rowbase + e];
    nst += __popcll(m);
    nsurv += __popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    while (nst >= 32) {
      run_tile(32);
      const int rest = nst - 32;
      const int mv = lane < rest ? st[32 + lane] : 0;
      __builtin_amdgcn_wave_barrier();
      if (lane < rest) st[lane] = mv;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      nst = rest;
    }
  }
  if (nst > 0) run_tile(nst);
  T.store(R.ov + b * K, R.oi + b * K, K);
  if (R.stats && lane == 0) {
    atomicAdd(R.stats + 0, 1ull);
    atomicAdd(R.stats + 1, (unsigned long long)nsurv);
  }
}

// out rows <- the fallback's compact rows
__global__ void wdc_scatter_kernel(const float* __restrict__ cv, const int64_t* __restrict__ ci,
                                   const int32_t* __restrict__ rows, int n, int K,
                                   float* __restrict__ ov, int64_t* __restrict__ oi) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n * K) return;
  const int r = e / K, s = e % K;
  const int64_t b = rows[r];
  if (ov) ov[b * K + s] = cv[e];
  oi[b * K + s] = ci[e];
}

// ------------------------------------------------------------------ host side
static hnm_status wd_check(const hnm_widedeep_weights* w) {
  HNM_REQUIRE(w && w->deep_user && w->deep_item && w->w1 && w->b1 && w->w2 && w->b2 &&
                  w->wide_user && w->wide_item && w->final_deep && w->final_b && w->bn1_w &&
                  w->bn2_w,
              HNM_EINVAL, "widedeep: NULL weight pointer");
  HNM_REQUIRE(w->num_users > 0 && w->num_items > 0 && w->num_items < WD_INT_BIG, HNM_EINVAL,
              "widedeep: bad table sizes");
  HNM_REQUIRE(w->d >= 1 && w->l1 >= 1 && w->l1 <= 512 && w->l2 >= 1 && w->l2 <= 256 &&
                  w->l3 >= 0 && w->l3 <= 128 && (w->l3 == 0 || w->w3),
              HNM_EUNSUPPORTED,
              "widedeep: the fused kernel covers 2- or 3-layer towers with widths <= "
              "512/256/128 (got %d/%d/%d)", w->l1, w->l2, w->l3);
  HNM_REQUIRE(w->l1_in == 2 * w->d + (w->num_user_features > 0 ? w->d : 0), HNM_EUNSUPPORTED,
              "widedeep: deep input must be [e_u; e_i(; user features)] (item features are "
              "not available to predict_all_items, wide_deep.py:275)");
  return HNM_OK;
}

static int pow2_blocks(int width) {
  const int nb = (width + 31) / 32;
  int p = 1;
  while (p < nb) p <<= 1;
  return p;
}

template <int RB2, int OB, bool DENSE>
static void launch_wd(hnm_ctx* ctx, dim3 grid, size_t lds, const float* Pu, const float* Qi,
                      int K1P, const WdPrep& pr, const float* cu, const float* wI, int64_t B,
                      int64_t I, int64_t ipp, const int64_t* mptr, const int32_t* midx, int K,
                      float* cv, int32_t* ci, int NP, float* dense, int64_t ldo,
                      const int32_t* rows = nullptr) {
  hipLaunchKernelGGL((widedeep_score_kernel<RB2, OB, DENSE>), grid, dim3(256), lds, ctx->stream,
                     Pu, Qi, K1P, pr.W2f, pr.W3f, pr.b2p, pr.b3p, pr.wdp, cu, wI, B, I, ipp, mptr,
                     midx, K, cv, ci, NP, dense, ldo, rows);
}

// Per-call preparation shared by the exact and the certified paths: folded weights,
// layer-1 projections P (batch rows) / Q (all items), per-user constants.  `extra` bytes of
// caller scratch follow in the same workspace carve.
struct WdSetup {
  WdPrep pr;
  int K1P;
  float* Pu;
  float* Qi;
  float* cu;
  char* extra;
};

static hnm_status wd_shape(const hnm_widedeep_weights* w, WdPrep* pr) {
  hnm_status st = wd_check(w);
  if (st) return st;
  pr->K1P = (w->l1 + 7) / 8 * 8;
  pr->RB2 = pow2_blocks(w->l2);
  pr->OB = w->l3 > 0 ? pow2_blocks(w->l3) : 0;
  const bool ok = (pr->RB2 == 8 && pr->OB == 4) || (pr->RB2 == 4 && pr->OB == 2) ||
                  (pr->RB2 == 2 && pr->OB == 1) || (pr->RB2 == 1 && pr->OB == 0) ||
                  (pr->RB2 == 2 && pr->OB == 0) || (pr->RB2 == 4 && pr->OB == 0) ||
                  (pr->RB2 == 8 && pr->OB == 0) || (pr->RB2 == 1 && pr->OB == 1) ||
                  (pr->RB2 == 4 && pr->OB == 4) || (pr->RB2 == 8 && pr->OB == 2);
  if (!ok) {
    hnm_set_error("widedeep: layer widths %d/%d not instantiated", w->l2, w->l3);
    return HNM_EUNSUPPORTED;
  }
  return HNM_OK;
}

static void wd_partition(const hnm_ctx* ctx, int64_t B, int64_t I, int64_t* np, int64_t* ipp,
                         int upb = 4) {
  const int64_t ublocks = hnm_cdiv(B, upb);
  const int64_t want = std::max<int64_t>(1, hnm_cdiv(2 * (int64_t)ctx->num_cus, ublocks));
  int64_t n = std::min<int64_t>(want, std::max<int64_t>(1, hnm_cdiv(I, 4 * WD_TILE)));
  *ipp = hnm_cdiv(hnm_cdiv(I, n), WD_TILE) * WD_TILE;
  *np = hnm_cdiv(I, *ipp);
}

// candidate-list scratch (values + int32 items) of the exact list pass over n rows
static size_t wd_list_bytes(const hnm_ctx* ctx, int64_t n, int64_t I, int K) {
  int64_t np, ipp;
  wd_partition(ctx, n, I, &np, &ipp);
  return 2 * hnm_align((size_t)n * np * K * 4);
}

static hnm_status wd_setup(hnm_ctx* ctx, const hnm_widedeep_weights* w, const int64_t* ids,
                           int64_t B, const float* ufeat, size_t extra, WdSetup* S) {
  const int64_t I = w->num_items;
  WdPrep& pr = S->pr;
  const int K1P = pr.K1P;
  S->K1P = K1P;
  const int nlast = pr.OB > 0 ? pr.OB : pr.RB2;
  const size_t szW2 = hnm_align((size_t)pr.RB2 * (K1P / 8) * 64 * 16);
  const size_t szW3 = hnm_align((size_t)std::max(pr.OB, 1) * pr.RB2 * 4 * 64 * 16);
  const size_t szb2 = hnm_align((size_t)pr.RB2 * 32 * 4);
  const size_t szb3 = hnm_align((size_t)std::max(pr.OB, 1) * 32 * 4);
  const size_t szwd = hnm_align((size_t)nlast * 32 * 4);
  const size_t szP = hnm_align((size_t)B * K1P * 4), szQ = hnm_align((size_t)I * K1P * 4);
  const size_t szX = w->num_user_features > 0 ? hnm_align((size_t)B * w->d * 4) : 0;
  const size_t szF = ufeat ? hnm_align((size_t)B * w->num_user_features * 4) : 0;
  const size_t szU = hnm_align((size_t)B * 4);
  const size_t szT = w->num_user_features > 0 ? hnm_align((size_t)B * K1P * 4) : 0;
  void* wsp;
  hnm_status st = hnm_workspace(ctx, szW2 + szW3 + szb2 + szb3 + szwd + 256 + szP + szQ + szX +
                                         szF + szU + szT + hnm_align(extra), &wsp);
  if (st) return st;
  char* q = (char*)wsp;
  pr.W2f = (float4*)q; q += szW2;
  pr.W3f = (float4*)q; q += szW3;
  pr.b2p = (float*)q; q += szb2;
  pr.b3p = (float*)q; q += szb3;
  pr.wdp = (float*)q; q += szwd;
  pr.bias = (float*)q; q += 256;
  float* Pu = (float*)q; q += szP;
  float* Qi = (float*)q; q += szQ;
  float* Xf = (float*)q; q += szX;
  float* WFu = (float*)q; q += szF;
  float* cu = (float*)q; q += szU;
  float* Tf = (float*)q; q += szT;
  S->Pu = Pu;
  S->Qi = Qi;
  S->cu = cu;
  S->extra = q;

  hipStream_t s = ctx->stream;
  hipLaunchKernelGGL(wd_prep_w2, dim3(256), dim3(256), 0, s, *w, pr);
  if (pr.OB > 0) hipLaunchKernelGGL(wd_prep_w3, dim3(128), dim3(256), 0, s, *w, pr);
  hipLaunchKernelGGL(wd_prep_bias, dim3(64), dim3(256), 0, s, *w, pr);
  HNM_LAUNCH_CHECK();
  // layer-1 decomposition: P_u = W1[:, :d] e_u + b1 (+ W1[:, 2d:3d] (Wf f_u + bf)),
  // Q_i = W1[:, d:2d] e_i, both pair-permuted with row stride K1P
  if (K1P != w->l1) {
    HNM_HIP_CHECK(hipMemsetAsync(Pu, 0, szP, s));
    HNM_HIP_CHECK(hipMemsetAsync(Qi, 0, szQ, s));
  }
  st = hnm_linear_rows_f32(ctx, w->deep_user, w->d, ids, w->num_users, B, w->d, w->w1, w->l1_in,
                           w->b1, w->l1, Pu, K1P, 1);
  if (st) return st;
  st = hnm_linear_rows_f32(ctx, w->deep_item, w->d, nullptr, I, I, w->d, w->w1 + w->d, w->l1_in,
                           nullptr, w->l1, Qi, K1P, 1);
  if (st) return st;
  const float* wuf = nullptr;
  if (w->num_user_features > 0) {
    HNM_REQUIRE(ufeat && w->duf_w && w->duf_b, HNM_EINVAL,
                "widedeep: user_features required (num_user_features > 0)");
    // deep user features -> Xf [B, d] (deep_user_features Linear(F, d), wide_deep.py:113)
    st = hnm_linear_rows_f32(ctx, ufeat, w->num_user_features, nullptr, B, B,
                             w->num_user_features, w->duf_w, w->num_user_features, w->duf_b,
                             w->d, Xf, w->d, 0);
    if (st) return st;
    // wide user features Linear(F, F)
    if (w->wuf_w && w->wide_feat) {
      st = hnm_linear_rows_f32(ctx, ufeat, w->num_user_features, nullptr, B, B,
                               w->num_user_features, w->wuf_w, w->num_user_features, w->wuf_b,
                               w->num_user_features, WFu, w->num_user_features, 0);
      if (st) return st;
      wuf = WFu;
    }
  }
  hipLaunchKernelGGL(wd_user_const, dim3((unsigned)hnm_cdiv(B, 256)), dim3(256), 0, s, *w, ids, B,
                     wuf, pr.bias, cu);
  HNM_LAUNCH_CHECK();
  if (w->num_user_features > 0) {
    // P_u += W1[:, 2d:3d] (deep user-feature projection), pair-permuted like P_u
    HNM_HIP_CHECK(hipMemsetAsync(Tf, 0, szT, s));
    st = hnm_linear_rows_f32(ctx, Xf, w->d, nullptr, B, B, w->d, w->w1 + 2 * w->d, w->l1_in,
                             nullptr, w->l1, Tf, K1P, 1);
    if (st) return st;
    st = hnm_axpby_f32(ctx, (int64_t)B * K1P, 1.f, Pu, 1.f, Tf, Pu);
    if (st) return st;
  }
  return HNM_OK;
}

// Exact fp32 pass: dense scores (dense != nullptr) or the per-partition top-K lists +
// merge for the rows rows[0, n) (rows == nullptr: batch rows 0 .. n).  cv/ci: list scratch
// of wd_list_bytes(n) bytes; outputs at the compact row index.
static hnm_status wd_exact(hnm_ctx* ctx, const hnm_widedeep_weights* w, const WdSetup& S,
                           int64_t n, const int64_t* mptr, const int32_t* midx, int K,
                           const int32_t* rows, float* cv, int32_t* ci, float* ov, int64_t* oi,
                           float* dense, int64_t ldo, bool timed) {
  const WdPrep& pr = S.pr;
  const int64_t I = w->num_items;
  int64_t np, ipp;
  wd_partition(ctx, n, I, &np, &ipp);
  const int K1P = S.K1P;
  const int nlast = pr.OB > 0 ? pr.OB : pr.RB2;
  const size_t lds = (size_t)(WD_TILE * (K1P + 4) + 4 * K1P + (pr.RB2 + pr.OB + nlast) * 32) * 4;
  dim3 grid((unsigned)hnm_cdiv(n, 4), (unsigned)np);
  const float* wI = w->wide_item;
  if (timed) hnm_timer_begin(ctx, HNM_TIME_SCORE);
#define WD_CASE(R, O)                                                                         \
  if (pr.RB2 == R && pr.OB == O) {                                                            \
    if (dense)                                                                                \
      launch_wd<R, O, true>(ctx, grid, lds, S.Pu, S.Qi, K1P, pr, S.cu, wI, n, I, ipp, mptr,   \
                            midx, K, cv, ci, (int)np, dense, ldo, rows);                      \
    else                                                                                      \
      launch_wd<R, O, false>(ctx, grid, lds, S.Pu, S.Qi, K1P, pr, S.cu, wI, n, I, ipp, mptr,  \
                             midx, K, cv, ci, (int)np, dense, ldo, rows);                     \
  }
  WD_CASE(8, 4)
  WD_CASE(4, 2)
  WD_CASE(2, 1)
  WD_CASE(1, 0)
  WD_CASE(2, 0)
  WD_CASE(4, 0)
  WD_CASE(8, 0)
  WD_CASE(1, 1)
  WD_CASE(4, 4)
  WD_CASE(8, 2)
#undef WD_CASE
  if (timed) hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  if (dense) return HNM_OK;
  return hnm_topk_merge_i32(ctx, cv, ci, n, 1, 0, np * K, (int)(np * K), K, ov, oi);
}

// ------------------------------------------------------------------ certified path host
#define WDC_CAP 4096  // appended candidates per (user, partition) segment

static bool wdc_instantiated(int RB2, int OB) {
  return (RB2 == 8 && OB == 4) || (RB2 == 4 && OB == 2) || (RB2 == 2 && OB == 1) ||
         (RB2 == 1 && OB == 1) || (RB2 == 1 && OB == 0) || (RB2 == 2 && OB == 0);
}

static bool wdc_eligible(const hnm_ctx* ctx, const WdPrep& pr, int64_t I, int K, bool debug) {
  return (debug || (ctx->prefilter && I >= 4096)) && K <= 64 && pr.K1P % 16 == 0 &&
         wdc_instantiated(pr.RB2, pr.OB);
}

struct WdcWs {
  WdCertParams* prm;
  wh8* W2hl;
  wh8* W3hl;
  wh8* WBf;
  float* v1;
  float* v1o;
  float* v2o;
  float* v2;
  float* b2s;
  float* part;
  float* lbv;
  int32_t* lbi;
  float* Lv;
  int64_t* Li;
  int32_t* segi;
  float* segu;
  int* cnt;
  float* segl;
  float* segs;
  int32_t* cli;
  int* nA;
  float* tv;
  int* tg;
  int* ns;
  int* toff;
  int32_t* fbrows;
  int* nfb;
  float* fcv;
  int32_t* fci;
  float* fov;
  int64_t* foi;
  int64_t np, ipp;
  int cap;
};
constexpr int WDC_STAT_BLOCKS = 1024;

// users per wave of the certified scan: 2 for the wide default tower (weight-fragment reuse)
static int wdc_upw(const WdPrep& pr) { return pr.RB2 == 8 && pr.OB == 4 ? 2 : 1; }

static size_t wdc_carve(const hnm_ctx* ctx, const WdPrep& pr, int64_t B, int64_t I, int K,
                        char* base, WdcWs* c) {
  int64_t np, ipp;
  wd_partition(ctx, B, I, &np, &ipp, 4 * wdc_upw(pr));
  const int cap = (int)std::min<int64_t>(WDC_CAP, ipp);
  const int K1P = pr.K1P, KB = K1P / 16;
  const int64_t fbn = 8 * (int64_t)ctx->num_cus + 4 + B;  // bound on n * np(n) over n <= B
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += hnm_align(bytes);
    return p;
  };
  WdcWs t;
  t.prm = (WdCertParams*)take(sizeof(WdCertParams));
  t.W2hl = (wh8*)take((size_t)pr.RB2 * KB * 2 * 64 * 16);
  t.W3hl = (wh8*)take((size_t)std::max(pr.OB, 1) * 2 * pr.RB2 * 2 * 64 * 16);
  t.WBf = (wh8*)take((size_t)KB * 2 * 64 * 16);
  t.v1 = (float*)take((size_t)K1P * 4);
  t.v1o = (float*)take((size_t)K1P * 4);
  t.v2 = (float*)take((size_t)pr.RB2 * 32 * 4);
  t.v2o = (float*)take((size_t)pr.RB2 * 32 * 4);
  t.b2s = (float*)take((size_t)pr.RB2 * 32 * 4);
  t.part = (float*)take((size_t)WDC_STAT_BLOCKS * 2 * 4);
  t.lbv = (float*)take((size_t)B * np * K * 4);
  t.lbi = (int32_t*)take((size_t)B * np * K * 4);
  t.Lv = (float*)take((size_t)B * K * 4);
  t.Li = (int64_t*)take((size_t)B * K * 8);
  t.segi = (int32_t*)take((size_t)B * np * cap * 4);
  t.segu = (float*)take((size_t)B * np * cap * 4);
  t.cnt = (int*)take((size_t)B * np * 4);
  t.segl = (float*)take((size_t)B * np * cap * 4);
  t.segs = (float*)take((size_t)B * np * cap * 4);
  t.cli = (int32_t*)take((size_t)B * np * cap * 4);
  t.nA = (int*)take((size_t)B * 4);
  t.tv = (float*)take((size_t)B * 4);
  t.tg = (int*)take((size_t)B * 4);
  t.ns = (int*)take((size_t)B * 4);
  t.toff = (int*)take((size_t)(B + 1) * 4);
  t.fbrows = (int32_t*)take((size_t)B * 4);
  t.nfb = (int*)take(4);
  t.fcv = (float*)take((size_t)fbn * K * 4);
  t.fci = (int32_t*)take((size_t)fbn * K * 4);
  t.fov = (float*)take((size_t)B * K * 4);
  t.foi = (int64_t*)take((size_t)B * K * 8);
  t.np = np;
  t.ipp = ipp;
  t.cap = cap;
  if (c) *c = t;
  return off;
}

static hnm_status wdc_prepare(hnm_ctx* ctx, const hnm_widedeep_weights* w, const WdSetup& S,
                              int64_t B, const WdcWs& c) {
  hipStream_t s = ctx->stream;
  const int64_t I = w->num_items;
  hipLaunchKernelGGL(wdc_stats_kernel, dim3(WDC_STAT_BLOCKS), dim3(256), 0, s, S.Pu,
                     B * S.K1P, S.Qi, I * S.K1P, c.part);
  hipLaunchKernelGGL(wdc_params_kernel, dim3(1), dim3(256), 0, s, *w, S.pr, c.part,
                     WDC_STAT_BLOCKS, c.v1, c.v2, c.b2s, c.prm, c.v1o, c.v2o);
  hipLaunchKernelGGL(wdc_convert_kernel, dim3(256), dim3(256), 0, s, *w, S.pr, c.prm, c.W2hl,
                     c.W3hl);
  hipLaunchKernelGGL(wdc_boundfrag_kernel, dim3((unsigned)hnm_cdiv(S.K1P / 16 * 2 * 64, 256)),
                       dim3(256), 0, s, c.prm, c.v1, c.v1o, S.K1P, c.WBf);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

template <int RB2, int OB, int MODE>
static void wdc_launch_scan(hnm_ctx* ctx, dim3 grid, size_t lds, const WdScanArgs& a) {
  constexpr int G2 = RB2 < WDC_G2 ? RB2 : WDC_G2;
  constexpr int UPW = RB2 == 8 && OB == 4 ? 2 : 1;  // = wdc_upw
  auto kern = wdc_scan_kernel<RB2, OB, G2, MODE, UPW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, ctx->stream, a);
}

template <int RB2, int OB>
static void wdc_launch_refine(hnm_ctx* ctx, const WdRescoreArgs& r) {
  constexpr int NOB = OB > 0 ? OB : 1, NL = OB > 0 ? OB : RB2;
  hipLaunchKernelGGL(wdc_tiles_kernel, dim3(1), dim3(1024), 0, ctx->stream, r.ns, r.rstart, r.B,
                     r.toff);
  const size_t lds = (size_t)(5 * r.K1P + 2 * RB2 * 32 + NOB * 32 + NL * 32) * 4;
  auto kern = wdc_refine_kernel<RB2, OB>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(ctx->num_cus), dim3(256), lds, ctx->stream, r);
}

struct WdcBestFirst {
  int32_t* cli;  // [B, rstride] the rows' refining lists
  int* nA;       // [B] first-phase length
  float* tv;     // [B] the first phase's last (scan ub, position)
  int* tg;
};

template <int RB2, int OB>
static void wdc_launch_rescore(hnm_ctx* ctx, dim3 grid, const WdRescoreArgs& r,
                               const WdcBestFirst& bf) {
  hipStream_t s = ctx->stream;
  hipLaunchKernelGGL(wdc_collect_kernel, grid, dim3(256), 0, s, r);
  hipLaunchKernelGGL(wdc_best_kernel, grid, dim3(256), 0, s, r, bf.cli, bf.nA, bf.tv, bf.tg);
  WdRescoreArgs q = r;  // the refining lists replace the survivor lists from here on
  q.segi = bf.cli;
  WdRescoreArgs qa = q;  // first phase: cli[0, nA)
  qa.ns = bf.nA;
  qa.rstart = nullptr;
  wdc_launch_refine<RB2, OB>(ctx, qa);
  hipLaunchKernelGGL(wdc_filter_kernel, grid, dim3(256), 0, s, r, bf.cli, bf.tv, bf.tg);
  WdRescoreArgs qb = q;  // second phase: cli[nA, ns)
  qb.rstart = bf.nA;
  wdc_launch_refine<RB2, OB>(ctx, qb);
  hipLaunchKernelGGL((wdc_rescore_kernel<RB2, OB>), grid, dim3(256), 0, s, q);
}

static hnm_status wdc_scan(hnm_ctx* ctx, const hnm_widedeep_weights* w, const WdSetup& S,
                           int64_t B, const int64_t* mptr, const int32_t* midx, int K,
                           const WdcWs& c, int mode, float* dbg_a, float* dbg_e, int64_t lda) {
  const WdPrep& pr = S.pr;
  const int NOB = pr.OB > 0 ? pr.OB : 1, NL = pr.OB > 0 ? pr.OB : pr.RB2;
  WdScanArgs a;
  a.Pu = S.Pu;
  a.Qi = S.Qi;
  a.K1P = S.K1P;
  a.W2hl = c.W2hl;
  a.W3hl = c.W3hl;
  a.WBf = c.WBf;
  a.v1 = c.v1;
  a.v1o = c.v1o;
  a.v2 = c.v2;
  a.b2s = c.b2s;
  a.b3p = pr.b3p;
  a.wdp = pr.wdp;
  a.cu = S.cu;
  a.wI = w->wide_item;
  a.prm = c.prm;
  a.B = B;
  a.I = w->num_items;
  a.ipp = c.ipp;
  a.NP = (int)c.np;
  a.mptr = mptr;
  a.midx = midx;
  a.K = K;
  a.lbv = c.lbv;
  a.lbi = c.lbi;
  a.segi = c.segi;
  a.segu = c.segu;
  a.cnt = c.cnt;
  a.cap = c.cap;
  a.dbg_a = dbg_a;
  a.dbg_e = dbg_e;
  a.lda = lda;
  const int upb = 4 * wdc_upw(pr);
  const size_t lds =
      (size_t)(2 * 32 * (S.K1P + 4) + upb * S.K1P + 2 * pr.RB2 * 32 + NOB * 32 + NL * 32) * 4;
  dim3 grid((unsigned)hnm_cdiv(B, upb), (unsigned)c.np);
  if (mode == WDC_THRESH) hnm_timer_begin(ctx, HNM_TIME_SCORE);
#define WDC_CASE(R, O)                                                        \
  if (pr.RB2 == R && pr.OB == O) {                                            \
    if (mode == WDC_THRESH) wdc_launch_scan<R, O, WDC_THRESH>(ctx, grid, lds, a); \
    else wdc_launch_scan<R, O, WDC_DEBUG>(ctx, grid, lds, a);                 \
  }
  WDC_CASE(8, 4)
  WDC_CASE(4, 2)
  WDC_CASE(2, 1)
  WDC_CASE(1, 1)
  WDC_CASE(1, 0)
  WDC_CASE(2, 0)
#undef WDC_CASE
  if (mode == WDC_THRESH) hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

static hnm_status wdc_topk(hnm_ctx* ctx, const hnm_widedeep_weights* w, const WdSetup& S,
                           int64_t B, const int64_t* mptr, const int32_t* midx, int K,
                           const WdcWs& c, float* ov, int64_t* oi) {
  hnm_status st = wdc_prepare(ctx, w, S, B, c);
  if (st) return st;
  st = wdc_scan(ctx, w, S, B, mptr, midx, K, c, WDC_THRESH, nullptr, nullptr, 0);
  if (st) return st;
  st = hnm_topk_merge_i32(ctx, c.lbv, c.lbi, B, 1, 0, c.np * K, (int)(c.np * K), K, c.Lv, c.Li);
  if (st) return st;
  hipStream_t s = ctx->stream;
  HNM_HIP_CHECK(hipMemsetAsync(c.nfb, 0, sizeof(int), s));
  const WdPrep& pr = S.pr;
  WdRescoreArgs r;
  r.Pu = S.Pu;
  r.Qi = S.Qi;
  r.K1P = S.K1P;
  r.W2f = pr.W2f;
  r.W3f = pr.W3f;
  r.b2p = pr.b2p;
  r.b3p = pr.b3p;
  r.wdp = pr.wdp;
  r.cu = S.cu;
  r.wI = w->wide_item;
  r.prm = c.prm;
  r.B = B;
  r.NP = (int)c.np;
  r.K = K;
  r.cap = c.cap;
  r.Lk = c.Lv;
  r.segi = c.segi;
  r.segu = c.segu;
  r.cnt = c.cnt;
  r.fbrows = c.fbrows;
  r.nfb = c.nfb;
  r.ov = ov;
  r.oi = oi;
  r.stats = ctx->stats_on ? ctx->stats_dev : nullptr;
  r.segl = c.segl;
  r.rstride = c.np * (int64_t)c.cap;
  r.dbg_a = r.dbg_e = nullptr;
  r.lda = 0;
  r.ns = c.ns;
  r.toff = c.toff;
  r.W2hl = c.W2hl;
  r.W3hl = c.W3hl;
  r.v1p = c.v1o;
  r.v2p = c.v2o;
  r.b2s = c.b2s;
  r.segs = c.segs;
  r.rstart = nullptr;
  const WdcBestFirst bf = {c.cli, c.nA, c.tv, c.tg};
  dim3 grid((unsigned)hnm_cdiv(B, 4));
#define WDC_CASE(R, O) \
  if (pr.RB2 == R && pr.OB == O) wdc_launch_rescore<R, O>(ctx, grid, r, bf);
  WDC_CASE(8, 4)
  WDC_CASE(4, 2)
  WDC_CASE(2, 1)
  WDC_CASE(1, 1)
  WDC_CASE(1, 0)
  WDC_CASE(2, 0)
#undef WDC_CASE
  HNM_LAUNCH_CHECK();
  // fallback rows: the count comes back to the host (a W&D call is long; one sync is noise)
  int nfb = 0;
  HNM_HIP_CHECK(hipMemcpyAsync(&nfb, c.nfb, sizeof(int), hipMemcpyDeviceToHost, s));
  HNM_HIP_CHECK(hipStreamSynchronize(s));
  if (nfb > 0) {
    st = wd_exact(ctx, w, S, nfb, mptr, midx, K, c.fbrows, c.fcv, c.fci, c.fov, c.foi, nullptr,
                  0, false);
    if (st) return st;
    hipLaunchKernelGGL(wdc_scatter_kernel, dim3((unsigned)hnm_cdiv((int64_t)nfb * K, 256)),
                       dim3(256), 0, s, c.fov, c.foi, c.fbrows, nfb, K, ov, oi);
    HNM_LAUNCH_CHECK();
  }
  return HNM_OK;
}

extern "C" hnm_status hnm_widedeep_topk_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                            const int64_t* user_ids, int64_t B,
                                            const float* user_features, const int64_t* mask_ptr,
                                            const int32_t* mask_idx, int k, float* out_val,
                                            int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(k >= 1 && k <= 64 && (out_idx || B == 0), HNM_EINVAL, "widedeep_topk: fused path needs 1 <= k <= 64");
  HNM_REQUIRE(ctx && (user_ids || B == 0), HNM_EINVAL, "widedeep: NULL argument");
  WdSetup S;
  hnm_status st = wd_shape(w, &S.pr);
  if (st) return st;
  if (B <= 0) return HNM_OK;
  const int64_t I = w->num_items;
  if (wdc_eligible(ctx, S.pr, I, k, false)) {
    const size_t extra = wdc_carve(ctx, S.pr, B, I, k, nullptr, nullptr);
    st = wd_setup(ctx, w, user_ids, B, user_features, extra, &S);
    if (st) return st;
    WdcWs c;
    wdc_carve(ctx, S.pr, B, I, k, S.extra, &c);
    return wdc_topk(ctx, w, S, B, mask_ptr, mask_idx, k, c, out_val, out_idx);
  }
  const size_t lb = wd_list_bytes(ctx, B, I, k);
  st = wd_setup(ctx, w, user_ids, B, user_features, lb, &S);
  if (st) return st;
  int64_t np, ipp;
  wd_partition(ctx, B, I, &np, &ipp);
  float* cv = (float*)S.extra;
  int32_t* ci = (int32_t*)(S.extra + hnm_align((size_t)B * np * k * 4));
  return wd_exact(ctx, w, S, B, mask_ptr, mask_idx, k, nullptr, cv, ci, out_val, out_idx,
                  nullptr, 0, true);
}

extern "C" hnm_status hnm_widedeep_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                              const int64_t* user_ids, int64_t B,
                                              const float* user_features, float* out,
                                              int64_t ldo) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE((out || B == 0) && w && ldo >= w->num_items, HNM_EINVAL, "widedeep_scores: bad output");
  HNM_REQUIRE(ctx && (user_ids || B == 0), HNM_EINVAL, "widedeep: NULL argument");
  WdSetup S;
  hnm_status st = wd_shape(w, &S.pr);
  if (st) return st;
  if (B <= 0) return HNM_OK;
  st = wd_setup(ctx, w, user_ids, B, user_features, 0, &S);
  if (st) return st;
  return wd_exact(ctx, w, S, B, nullptr, nullptr, 1, nullptr, nullptr, nullptr, nullptr,
                  nullptr, out, ldo, true);
}

extern "C" hnm_status hnm_widedeep_prefilter_debug_f32(hnm_ctx* ctx,
                                                       const hnm_widedeep_weights* w,
                                                       const int64_t* user_ids, int64_t B,
                                                       const float* user_features,
                                                       float* approx, int64_t lda,
                                                       float* bound) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && user_ids && approx && bound && w && lda >= w->num_items, HNM_EINVAL,
              "widedeep_prefilter_debug: bad argument");
  WdSetup S;
  hnm_status st = wd_shape(w, &S.pr);
  if (st) return st;
  HNM_REQUIRE(wdc_eligible(ctx, S.pr, w->num_items, 1, true), HNM_EUNSUPPORTED,
              "widedeep_prefilter_debug: tower shape not covered by the certified scan");
  if (B <= 0) return HNM_OK;
  const int64_t I = w->num_items;
  const size_t extra = wdc_carve(ctx, S.pr, B, I, 1, nullptr, nullptr);
  st = wd_setup(ctx, w, user_ids, B, user_features, extra, &S);
  if (st) return st;
  WdcWs c;
  wdc_carve(ctx, S.pr, B, I, 1, S.extra, &c);
  st = wdc_prepare(ctx, w, S, B, c);
  if (st) return st;
  return wdc_scan(ctx, w, S, B, nullptr, nullptr, 1, c, WDC_DEBUG, approx, bound, lda);
}

// every row's item list = the whole catalogue (the refine stage's debug input)
__global__ void wdc_debug_rows_kernel(int32_t* __restrict__ segi, int* __restrict__ ns, int64_t B,
                                      int64_t I) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < B * I) segi[e] = (int32_t)(e % I);
  if (e < B) ns[e] = (int)I;
}

extern "C" hnm_status hnm_widedeep_refine_debug_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                                    const int64_t* user_ids, int64_t B,
                                                    const float* user_features, float* approx,
                                                    int64_t lda, float* bound) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && user_ids && approx && bound && w && lda >= w->num_items, HNM_EINVAL,
              "widedeep_refine_debug: bad argument");
  WdSetup S;
  hnm_status st = wd_shape(w, &S.pr);
  if (st) return st;
  HNM_REQUIRE(wdc_eligible(ctx, S.pr, w->num_items, 1, true), HNM_EUNSUPPORTED,
              "widedeep_refine_debug: tower shape not covered by the certified scan");
  if (B <= 0) return HNM_OK;
  const int64_t I = w->num_items;
  HNM_REQUIRE(B * I < ((int64_t)1 << 31), HNM_EINVAL, "widedeep_refine_debug: B * I >= 2^31");
  const size_t cb = wdc_carve(ctx, S.pr, B, I, 1, nullptr, nullptr);
  const size_t lb = hnm_align((size_t)B * I * 4) + hnm_align((size_t)B * 4) + hnm_align((size_t)(B + 1) * 4);
  st = wd_setup(ctx, w, user_ids, B, user_features, cb + lb, &S);
  if (st) return st;
  WdcWs c;
  wdc_carve(ctx, S.pr, B, I, 1, S.extra, &c);
  st = wdc_prepare(ctx, w, S, B, c);
  if (st) return st;
  char* x = (char*)S.extra + cb;
  int32_t* segi = (int32_t*)x;
  int* ns = (int*)(x + hnm_align((size_t)B * I * 4));
  int* toff = (int*)(x + hnm_align((size_t)B * I * 4) + hnm_align((size_t)B * 4));
  hipLaunchKernelGGL(wdc_debug_rows_kernel, dim3((unsigned)hnm_cdiv(B * I, 256)), dim3(256), 0,
                     ctx->stream, segi, ns, B, I);
  const WdPrep& pr = S.pr;
  WdRescoreArgs r{};
  r.Pu = S.Pu;
  r.Qi = S.Qi;
  r.K1P = S.K1P;
  r.b3p = pr.b3p;
  r.wdp = pr.wdp;
  r.cu = S.cu;
  r.wI = w->wide_item;
  r.prm = c.prm;
  r.B = B;
  r.segi = segi;
  r.ns = ns;
  r.toff = toff;
  r.W2hl = c.W2hl;
  r.W3hl = c.W3hl;
  r.v1p = c.v1o;
  r.v2p = c.v2o;
  r.b2s = c.b2s;
  r.rstride = I;
  r.dbg_a = approx;
  r.dbg_e = bound;
  r.lda = lda;
#define WDC_CASE(R, O) \
  if (pr.RB2 == R && pr.OB == O) wdc_launch_refine<R, O>(ctx, r);
  WDC_CASE(8, 4)
  WDC_CASE(4, 2)
  WDC_CASE(2, 1)
  WDC_CASE(1, 1)
  WDC_CASE(1, 0)
  WDC_CASE(2, 0)
#undef WDC_CASE
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_widedeep_pair_scores_ex_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                                      const hnm_widedeep_item_features* itf,
                                                      const int64_t* user_ids,
                                                      const int64_t* item_ids,
                                                      const float* user_features,
                                                      const float* item_features, int64_t n,
                                                      float* out) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && w && ((user_ids && item_ids && out) || n == 0), HNM_EINVAL, "widedeep_pair: NULL argument");
  HNM_REQUIRE(w->l1 <= 512 && w->l2 <= 512 && w->l3 <= 512 && w->l1_in <= 512, HNM_EUNSUPPORTED,
              "widedeep_pair: widths must be <= 512");
  const int Fu = w->num_user_features, Fi = itf ? itf->num_item_features : 0;
  const int nch = (Fu > 0) + (Fi > 0);  // deep feature chunks after [e_u; e_i]
  HNM_REQUIRE(w->l1_in == (2 + nch) * w->d, HNM_EINVAL,
              "widedeep_pair: layer-1 input %d != %d x embedding_dim (features given)", w->l1_in,
              2 + nch);
  if (n <= 0) return HNM_OK;
  float* xf = nullptr;
  float* wide = nullptr;
  float* wide2 = nullptr;
  const int ldx = nch * w->d;
  if (nch > 0) {
    HNM_REQUIRE(Fu == 0 || (user_features && w->duf_w), HNM_EINVAL,
                "widedeep_pair: user_features required");
    HNM_REQUIRE(Fi == 0 || (item_features && itf->dif_w), HNM_EINVAL,
                "widedeep_pair: item_features required");
    const int Fm = std::max(Fu, Fi);
    const size_t szx = hnm_align((size_t)n * ldx * 4), szf = hnm_align((size_t)n * Fm * 4);
    const size_t szw = hnm_align((size_t)n * 4);
    void* wsp;
    hnm_status st = hnm_workspace(ctx, szx + szf + 2 * szw, &wsp);
    if (st) return st;
    xf = (float*)wsp;
    float* wf = (float*)((char*)wsp + szx);
    float* w1 = (float*)((char*)wsp + szx + szf);
    float* w2 = (float*)((char*)wsp + szx + szf + szw);
    if (Fu > 0) {  // deep_user_features (wide_deep.py:214-215) + its wide cross (:190-192)
      st = hnm_linear_rows_f32(ctx, user_features, Fu, nullptr, n, n, Fu, w->duf_w, Fu, w->duf_b,
                               w->d, xf, ldx, 0);
      if (st) return st;
      if (w->wuf_w && w->wide_feat) {
        st = hnm_linear_rows_f32(ctx, user_features, Fu, nullptr, n, n, Fu, w->wuf_w, Fu,
                                 w->wuf_b, Fu, wf, Fu, 0);
        if (st) return st;
        // wide feature term = wf . final_w[U + I : U + I + Fu]
        st = hnm_linear_rows_f32(ctx, wf, Fu, nullptr, n, n, Fu, w->wide_feat, Fu, nullptr, 1, w1,
                                 1, 0);
        if (st) return st;
        wide = w1;
      }
    }
    if (Fi > 0) {  // deep_item_features (:216-217) + its wide cross (:193-195)
      st = hnm_linear_rows_f32(ctx, item_features, Fi, nullptr, n, n, Fi, itf->dif_w, Fi,
                               itf->dif_b, w->d, xf + (Fu > 0 ? w->d : 0), ldx, 0);
      if (st) return st;
      if (itf->wif_w && itf->wide_feat) {
        st = hnm_linear_rows_f32(ctx, item_features, Fi, nullptr, n, n, Fi, itf->wif_w, Fi,
                                 itf->wif_b, Fi, wf, Fi, 0);
        if (st) return st;
        st = hnm_linear_rows_f32(ctx, wf, Fi, nullptr, n, n, Fi, itf->wide_feat, Fi, nullptr, 1,
                                 w2, 1, 0);
        if (st) return st;
        wide2 = w2;
      }
    }
  }
  hipLaunchKernelGGL(widedeep_pair_kernel, dim3((unsigned)n), dim3(256), 0, ctx->stream, *w,
                     user_ids, item_ids, n, xf, ldx, wide, wide2, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

extern "C" hnm_status hnm_widedeep_pair_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                                   const int64_t* user_ids,
                                                   const int64_t* item_ids,
                                                   const float* user_features, int64_t n,
                                                   float* out) {
  HNM_CTX_DEVICE(ctx);
  return hnm_widedeep_pair_scores_ex_f32(ctx, w, nullptr, user_ids, item_ids, user_features,
                                         nullptr, n, out);
}
