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

// ------------------------------------------------------------------ main kernel
template <int RB2, int OB, bool DENSE>
__global__ __launch_bounds__(256, (RB2 >= 8 || OB >= 4) ? 1 : 2) void widedeep_score_kernel(
    const float* __restrict__ Pu, const float* __restrict__ Qi, int K1P,
    const float4* __restrict__ W2f, const float4* __restrict__ W3f,
    const float* __restrict__ b2p, const float* __restrict__ b3p,
    const float* __restrict__ wdp, const float* __restrict__ cu, const float* __restrict__ wI,
    int64_t B, int64_t I, int64_t ipp, const int64_t* __restrict__ mptr,
    const int32_t* __restrict__ midx, int K, float* __restrict__ cand_v,
    int32_t* __restrict__ cand_i, int NP, float* __restrict__ dense, int64_t ldo) {
  constexpr int G2 = RB2 < 4 ? RB2 : 4;  // layer-2 row blocks per pass
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KS1 = K1P / 2, S4 = K1P / 8, QRS = K1P + 4;
  float* qs = smem;                    // [32][QRS]
  float* ps = smem + WD_TILE * QRS;    // [4][K1P]
  float* cb2 = ps + 4 * K1P;           // [RB2*32] b2'
  float* cb3 = cb2 + RB2 * 32;         // [OB*32]  b3'
  float* cwd = cb3 + OB * 32;          // [32*max(OB,RB2)] w_d'

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, j = lane & 31;
  const int64_t b = (int64_t)blockIdx.x * 4 + wave;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + ipp);

  for (int e = tid; e < 4 * K1P / 4; e += 256) {
    const int r = e / (K1P / 4), c = e % (K1P / 4);
    const int64_t bb = (int64_t)blockIdx.x * 4 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bb < B) v = *reinterpret_cast<const float4*>(Pu + bb * K1P + 4 * c);
    *reinterpret_cast<float4*>(&ps[r * K1P + 4 * c]) = v;
  }
  for (int e = tid; e < RB2 * 32; e += 256) cb2[e] = b2p[e];
  for (int e = tid; e < OB * 32; e += 256) cb3[e] = b3p[e];
  for (int e = tid; e < (OB > 0 ? OB : RB2) * 32; e += 256) cwd[e] = wdp[e];
  const bool active = b < B;
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
  if (!DENSE && active) L.store(cand_v + (b * NP + p) * K, cand_i + (b * NP + p) * K, K);
}

// ------------------------------------------------------------------ pairwise forward
// WideDeep.forward(user_ids, item_ids[, features]) (wide_deep.py:157-230): one workgroup per
// pair, the unfolded reference op order (Linear -> ReLU -> BatchNorm per layer).
__global__ __launch_bounds__(256) void widedeep_pair_kernel(
    hnm_widedeep_weights w, const int64_t* __restrict__ uids, const int64_t* __restrict__ iids,
    int64_t n, const float* __restrict__ xu, const float* __restrict__ wide_extra,
    float* __restrict__ out, unsigned* err) {
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
    else v = xu[e * w.d + c - 2 * w.d];
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
    float v = red[0] + w.wide_user[u] + w.wide_item[i] + w.final_b[0];
    if (wide_extra) v += wide_extra[e];
    out[e] = v;
  }
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
                      float* cv, int32_t* ci, int NP, float* dense, int64_t ldo) {
  hipLaunchKernelGGL((widedeep_score_kernel<RB2, OB, DENSE>), grid, dim3(256), lds, ctx->stream,
                     Pu, Qi, K1P, pr.W2f, pr.W3f, pr.b2p, pr.b3p, pr.wdp, cu, wI, B, I, ipp, mptr,
                     midx, K, cv, ci, NP, dense, ldo);
}

template <bool DENSE>
static hnm_status wd_common(hnm_ctx* ctx, const hnm_widedeep_weights* w, const int64_t* ids,
                            int64_t B, const float* ufeat, const int64_t* mptr,
                            const int32_t* midx, int K, float* ov, int64_t* oi, float* dense,
                            int64_t ldo) {
  hnm_status st = wd_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ids, HNM_EINVAL, "widedeep: NULL argument");
  if (B <= 0) return HNM_OK;
  const int64_t I = w->num_items;
  WdPrep pr;
  pr.K1P = (w->l1 + 7) / 8 * 8;
  pr.RB2 = pow2_blocks(w->l2);
  pr.OB = w->l3 > 0 ? pow2_blocks(w->l3) : 0;
  if (pr.RB2 > 8 || pr.OB > 4) {
    hnm_set_error("widedeep: unsupported widths");
    return HNM_EUNSUPPORTED;
  }
  // instantiated (RB2, OB) pairs
  const bool ok = (pr.RB2 == 8 && pr.OB == 4) || (pr.RB2 == 4 && pr.OB == 2) ||
                  (pr.RB2 == 2 && pr.OB == 1) || (pr.RB2 == 1 && pr.OB == 0) ||
                  (pr.RB2 == 2 && pr.OB == 0) || (pr.RB2 == 4 && pr.OB == 0) ||
                  (pr.RB2 == 8 && pr.OB == 0) || (pr.RB2 == 1 && pr.OB == 1) ||
                  (pr.RB2 == 4 && pr.OB == 4) || (pr.RB2 == 8 && pr.OB == 2);
  if (!ok) {
    hnm_set_error("widedeep: layer widths %d/%d not instantiated", w->l2, w->l3);
    return HNM_EUNSUPPORTED;
  }
  const int K1P = pr.K1P;
  const int64_t ublocks = hnm_cdiv(B, 4);
  const int64_t want = std::max<int64_t>(1, hnm_cdiv(2 * (int64_t)ctx->num_cus, ublocks));
  int64_t np = std::min<int64_t>(want, std::max<int64_t>(1, hnm_cdiv(I, 4 * WD_TILE)));
  int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), WD_TILE) * WD_TILE;
  np = hnm_cdiv(I, ipp);

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
  const size_t ncand = DENSE ? 0 : (size_t)B * np * K;
  const size_t szC = hnm_align(ncand * 4);
  void* wsp;
  st = hnm_workspace(ctx, szW2 + szW3 + szb2 + szb3 + szwd + 256 + szP + szQ + szX + szF + szU +
                              szT + 2 * szC, &wsp);
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
  float* cv = (float*)q; q += szC;
  int32_t* ci = (int32_t*)q;

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

  const size_t lds = (size_t)(WD_TILE * (K1P + 4) + 4 * K1P + (pr.RB2 + pr.OB + nlast) * 32) * 4;
  dim3 grid((unsigned)ublocks, (unsigned)np);
  const float* wI = w->wide_item;
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
#define WD_CASE(R, O)                                                                     \
  if (pr.RB2 == R && pr.OB == O)                                                          \
    launch_wd<R, O, DENSE>(ctx, grid, lds, Pu, Qi, K1P, pr, cu, wI, B, I, ipp, mptr, midx, K, \
                           cv, ci, (int)np, dense, ldo);
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
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  if (!DENSE) return hnm_topk_merge_i32(ctx, cv, ci, B, 1, 0, np * K, (int)(np * K), K, ov, oi);
  return HNM_OK;
}

extern "C" hnm_status hnm_widedeep_topk_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                            const int64_t* user_ids, int64_t B,
                                            const float* user_features, const int64_t* mask_ptr,
                                            const int32_t* mask_idx, int k, float* out_val,
                                            int64_t* out_idx) {
  HNM_REQUIRE(k >= 1 && k <= 64 && out_idx, HNM_EINVAL, "widedeep_topk: fused path needs 1 <= k <= 64");
  return wd_common<false>(ctx, w, user_ids, B, user_features, mask_ptr, mask_idx, k, out_val,
                          out_idx, nullptr, 0);
}

extern "C" hnm_status hnm_widedeep_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                              const int64_t* user_ids, int64_t B,
                                              const float* user_features, float* out,
                                              int64_t ldo) {
  HNM_REQUIRE(out && w && ldo >= w->num_items, HNM_EINVAL, "widedeep_scores: bad output");
  return wd_common<true>(ctx, w, user_ids, B, user_features, nullptr, nullptr, 1, nullptr,
                         nullptr, out, ldo);
}

extern "C" hnm_status hnm_widedeep_pair_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                                   const int64_t* user_ids,
                                                   const int64_t* item_ids,
                                                   const float* user_features, int64_t n,
                                                   float* out) {
  HNM_REQUIRE(ctx && w && user_ids && item_ids && out, HNM_EINVAL, "widedeep_pair: NULL argument");
  HNM_REQUIRE(w->l1 <= 512 && w->l2 <= 512 && w->l3 <= 512 && w->l1_in <= 512, HNM_EUNSUPPORTED,
              "widedeep_pair: widths must be <= 512");
  if (n <= 0) return HNM_OK;
  float* xu = nullptr;
  float* wide = nullptr;
  if (w->num_user_features > 0) {
    HNM_REQUIRE(user_features && w->duf_w, HNM_EINVAL, "widedeep_pair: user_features required");
    const int F = w->num_user_features;
    const size_t szx = hnm_align((size_t)n * w->d * 4), szf = hnm_align((size_t)n * F * 4);
    void* wsp;
    hnm_status st = hnm_workspace(ctx, szx + szf + hnm_align((size_t)n * 4), &wsp);
    if (st) return st;
    xu = (float*)wsp;
    float* wf = (float*)((char*)wsp + szx);
    wide = (float*)((char*)wsp + szx + szf);
    st = hnm_linear_rows_f32(ctx, user_features, F, nullptr, n, n, F, w->duf_w, F, w->duf_b,
                             w->d, xu, w->d, 0);
    if (st) return st;
    if (w->wuf_w && w->wide_feat) {
      st = hnm_linear_rows_f32(ctx, user_features, F, nullptr, n, n, F, w->wuf_w, F, w->wuf_b, F,
                               wf, F, 0);
      if (st) return st;
      // wide feature term = wf . final_w[U + I : U + I + F]
      st = hnm_linear_rows_f32(ctx, wf, F, nullptr, n, n, F, w->wide_feat, F, nullptr, 1, wide, 1, 0);
      if (st) return st;
    } else {
      wide = nullptr;
    }
  }
  hipLaunchKernelGGL(widedeep_pair_kernel, dim3((unsigned)n), dim3(256), 0, ctx->stream, *w,
                     user_ids, item_ids, n, xu, wide, out, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
