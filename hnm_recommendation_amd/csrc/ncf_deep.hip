// NeuralCF with an MLP tower of any depth, exact fp32 (reference `_build_mlp`,
// neural_cf.py:75-90: Linear -> ReLU -> Dropout for every consecutive pair of mlp_dims; eval
// mode, so Dropout is the identity).  The fused certified kernels (ncf.hip, ncf_cert.hip) cover
// the reference's default two-layer tower; every other tower takes this file:
//
//   layer 1 decomposed per row (hnm_linear_rows_f32): P_u = W1[:, :h] m_u + b1 once per user,
//   Q_i = W1[:, h:] m_i once per item, so a pair's first activation is relu(P_u + Q_i);
//   score = sum_j wp[j] g_u[j] g_i[j] + sum_j wp[mf + j] x_L[j] + bp (neural_cf.py:131-141),
//   ONE fmaf chain in that order.
// Two kernels compute it, bitwise alike:
//   * ncf_deep_mfma_kernel (widths <= 64, mf <= 128): 32-item tiles through f32 MFMA chains,
//     dense rows or fused per-partition top-k lists (hnm_ncf_deep_topk_f32) -- see below;
//   * ncf_deep_kernel (any width <= 512, and the pair forward): per pair, a workgroup holds TP
//     pairs' activations in LDS (k-major, so the TP lanes of a pair group read consecutive
//     words) and 256 / TP lane groups share each layer's output units (the weights are
//     wave-uniform loads).  DENSE: pairs (b, i) for every item; else pairs (user_ids[n],
//     item_ids[n]) (forward).
#include <vector>

#include "hnm_device.h"
#include "hnm_internal.h"
#include "ncf_internal.h"

hnm_status hnm_topk_merge_i32(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                              int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                              float* ov, int64_t* oi);

struct DeepArgs {
  const float* P;        // [B, d1]   user halves of layer 1 (+ b1)
  const float* Q;        // [nq, d1]  item halves (all items, or the pairs' items)
  const float* gu;       // gmf_user [num_users, mf]
  const float* gi;       // gmf_item [num_items, mf]
  const int64_t* uids;   // [B] (gmf gather)
  const int64_t* iids;   // [B] pair mode, NULL dense
  const float* w[8];
  const float* b[8];
  const float* wp;
  const float* bp;
  int64_t num_users, num_items, B, nq;
  int mf, nl, d1;
  int dims[9];
  float* out;
  int64_t ldo;
};

// dynamic LDS: two activation buffers of TP x maxw floats
template <int TP, bool DENSE>
__global__ __launch_bounds__(256) void ncf_deep_kernel(DeepArgs a, int maxw, unsigned* err) {
  extern __shared__ float lds[];
  float* X = lds;
  float* Y = lds + (size_t)TP * maxw;
  constexpr int NGR = 256 / TP;
  const int t = threadIdx.x, p = t % TP, grp = t / TP;
  // pair -> (row of P / user, row of Q, gmf item row, output slot)
  int64_t b, q, item, o;
  bool ok;
  if (DENSE) {
    b = blockIdx.y;
    item = (int64_t)blockIdx.x * TP + p;
    ok = item < a.num_items;
    q = item;
    o = b * a.ldo + item;
  } else {
    b = (int64_t)blockIdx.x * TP + p;
    ok = b < a.B;
    q = b;
    item = ok ? a.iids[b] : 0;
    o = b;
  }
  const int64_t u = (DENSE || ok) ? a.uids[b] : 0;
  const bool good = ok && u >= 0 && u < a.num_users && item >= 0 && item < a.num_items;
  if (ok && !good && grp == 0) hnm_flag(err, HNM_ERR_OOB);
  // layer 1: x = relu(P_b + Q_q)
  for (int k = grp; k < a.d1; k += NGR) {
    float v = 0.f;
    if (good) v = fmaxf(a.P[b * a.d1 + k] + a.Q[q * a.d1 + k], 0.f);
    X[k * TP + p] = v;
  }
  __syncthreads();
  // layers 2..nl: y_j = relu(b_j + sum_k W[j, k] x_k), fma chain in k order
  for (int l = 1; l < a.nl; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1];
    const float* __restrict__ W = a.w[l];
    const float* __restrict__ bl = a.b[l];
    for (int j = grp; j < dout; j += NGR) {
      const float* wr = W + (int64_t)j * din;
      float acc = 0.f;
      int k = 0;
      for (; k + 3 < din; k += 4) {
        acc = fmaf(wr[k], X[k * TP + p], acc);
        acc = fmaf(wr[k + 1], X[(k + 1) * TP + p], acc);
        acc = fmaf(wr[k + 2], X[(k + 2) * TP + p], acc);
        acc = fmaf(wr[k + 3], X[(k + 3) * TP + p], acc);
      }
      for (; k < din; ++k) acc = fmaf(wr[k], X[k * TP + p], acc);
      Y[j * TP + p] = fmaxf(acc + bl[j], 0.f);
    }
    __syncthreads();
    float* s = X;
    X = Y;
    Y = s;
  }
  if (grp != 0 || !ok) return;
  if (!good) {
    a.out[o] = __builtin_nanf("");
    return;
  }
  // prediction layer over [gmf ; mlp]
  const float* g0 = a.gu + u * a.mf;
  const float* g1 = a.gi + item * a.mf;
  float s = 0.f;
  for (int j = 0; j < a.mf; ++j) s = fmaf(a.wp[j], g0[j] * g1[j], s);
  const int dl = a.dims[a.nl];
  for (int j = 0; j < dl; ++j) s = fmaf(a.wp[a.mf + j], X[j * TP + p], s);
  a.out[o] = s + a.bp[0];
}

// ------------------------------------------------------------------ fp32-MFMA tower tiles
// Towers whose widths dims[1..nl] are all <= 64 (and mf <= 128): every layer after the first is
// a chain of v_mfma_f32_32x32x2f32 over 32-item tiles -- A = the layer's weights (32 output
// units x 2 k), B = the pairs' activations (2 k x 32 items).  The f32 MFMA accumulates each
// output as the fmaf chain over k in order (MI355X_MICROARCH.md: exact f32, bitwise the chain),
// so scores are bitwise those of ncf_deep_kernel (HNM_OPT_DEEP_MFMA = 0) at 16x its FLOP rate
// with no per-FMA LDS read.
//   * unit placement: A row m of tile t carries unit 32t + 2r + h where m = mfma32_row(r, h),
//     so the accumulator register r of lane half h holds exactly the unit the next layer's
//     step s = 16t + r reads as its k = 2s + h operand -- layer outputs feed the next layer from
//     registers, no LDS round trip;
//   * layer 1 (relu(P_u + Q_i), both pair-permuted to the same lane-half order) is computed
//     from the LDS item tile as the B operand of layer 2;
//   * prediction: each lane half finishes the serial chain of one of the wave's two users
//     (half 0 user A, half 1 user B) after one permlane32 swap of the last layer's units:
//     s = fma over GMF terms (g_u[j] g_i[j]), then over the MLP units, + bp (ncf_deep_kernel's
//     order);
//   * workgroup = 4 waves x WU users (two at a time, one MFMA chain each) over one item
//     partition; the 32-item tile (Q rows, GMF rows) is staged once in LDS for all 4 WU users;
//   * top-k: a wave-resident list per (user, partition), merged across partitions afterwards
//     (the exact NCF path's scheme, ncf.hip); DENSE writes the score rows instead.
#define DM_W 64               // P / Q row width (pair-permuted, zero padded)
#define DM_QRS (DM_W + 4)     // LDS row stride of the Q tile (b128 reads conflict-free)
#define DM_WU 4               // users per wave (two MFMA chains at a time)
#define DM_NU (4 * DM_WU)     // users per workgroup

struct DeepMArgs {
  const float* P;      // [B, 64]
  const float* Q;      // [I, 64]
  const float* gu;     // gmf_user [num_users, mf]
  const float* G;      // [I, MFP] GMF item rows, zero padded, 16-B aligned
  const int64_t* uids;
  const float* img;    // deep_pack_kernel image: per MFMA layer A operands, then biases
  const float* wp;     // [mf + dl]
  const float* bp;
  int64_t num_users, num_items, B, ipp;
  int mf, nl, dl, img_n;
  int last16;   // the last layer (l = nl - 1 >= 2, <= 16 outputs) on v_mfma_f32_16x16x4f32
  int meta[8];  // MFMA layer l >= 1: A image offset | 4-step groups << 16 | 32-unit tiles << 20
  const int64_t* mptr;
  const int32_t* midx;
  int K;
  float* cv;
  int32_t* ci;
  int NP;
  float* out;
  int64_t ldo;
  unsigned* err;
};

struct DeepPack {
  const float* w[8];
  const float* b[8];
  int dims[9];
  int nl, img_n, last16;
  int ks4[8], nt[8], aoff[8], boff[8];
};

__device__ __forceinline__ int dm_unit(int t, int m) {  // unit at A row m of tile t
  return 32 * t + 2 * ((m & 3) + 4 * (m >> 3)) + ((m >> 2) & 1);
}

__global__ __launch_bounds__(256) void deep_pack_kernel(DeepPack pk, float* __restrict__ img) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < pk.img_n; e += gridDim.x * 256) {
    int l = 1;
    while (l + 1 < pk.nl && e >= pk.aoff[l + 1]) ++l;
    const int din = pk.dims[l], dout = pk.dims[l + 1];
    float v = 0.f;
    if (pk.last16 && l == pk.nl - 1) {
      // 16x16x4 layer: A[m = lane & 15][k = lane >> 4] of step s = 4 * group + (e & 3)
      // (input units 4s .. 4s + 3); then the bias, 16 plain floats
      if (e < pk.boff[l]) {
        const int rel = e - pk.aoff[l];
        const int lane = (rel >> 2) & 63, s = 4 * (rel >> 8) + (rel & 3);
        const int m = lane & 15, k = 4 * s + (lane >> 4);
        if (m < dout && k < din) v = pk.w[l][(int64_t)m * din + k];
      } else {
        const int unit = e - pk.boff[l];
        if (unit < dout) v = pk.b[l][unit];
      }
    } else if (e < pk.boff[l]) {
      const int rel = e - pk.aoff[l];
      const int lane = (rel >> 2) & 63, grp = rel >> 8;
      const int t = grp / pk.ks4[l], s = 4 * (grp % pk.ks4[l]) + (rel & 3);
      const int unit = dm_unit(t, lane & 31), k = 2 * s + (lane >> 5);
      if (unit < dout && k < din) v = pk.w[l][(int64_t)unit * din + k];
    } else {
      const int rel = e - pk.boff[l];
      const int unit = 32 * (rel >> 5) + 2 * (rel & 15) + ((rel >> 4) & 1);
      if (unit < dout) v = pk.b[l][unit];
    }
    img[e] = v;
  }
}

// acc{A,B}{0,1} = W_l (tiles 0/1) x b{A,B} + C for one k step of a 4-step group
#define DM_STEP(W0, W1, BA, BB, CA0, CA1, CB0, CB1)       \
  do {                                                    \
    cA0 = mfma32x32x2((W0), (BA), CA0);                   \
    cB0 = mfma32x32x2((W0), (BB), CB0);                   \
    if (two) {                                            \
      cA1 = mfma32x32x2((W1), (BA), CA1);                 \
      cB1 = mfma32x32x2((W1), (BB), CB1);                 \
    }                                                     \
  } while (0)
#define DM_ACC(W0, W1, BA, BB) DM_STEP(W0, W1, BA, BB, cA0, cA1, cB0, cB1)

template <int NT, int MFP, bool DENSE>
__global__ __launch_bounds__(256, NT == 1 ? 3 : 2) void ncf_deep_mfma_kernel(DeepMArgs a) {
  constexpr int WU = DM_WU, NU = DM_NU;
  constexpr int GRS = MFP + 4;       // LDS row stride of the GMF tile
  constexpr int GF4 = MFP / 32;      // GMF tile float4 a thread (32 rows x MFP / 4)
  extern __shared__ float4 dm_lds4[];
  float* img = (float*)dm_lds4;
  float* qs = img + a.img_n;              // [TILE][DM_QRS] (one buffer: three workgroups a CU)
  float* gs = qs + TILE * DM_QRS;         // [TILE][GRS]
  float* ps = gs + TILE * GRS;            // [NU][DM_W]
  float* us = ps + NU * DM_W;             // [NU][MFP]  g_u rows (zero padded)
  float* wps = us + NU * MFP;             // [MFP + 64] wp: GMF part, MLP part (zero padded)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int64_t B = a.B, I = a.num_items;
  const int64_t ublk = (int64_t)blockIdx.x * NU;
  const int p = blockIdx.y;
  const int64_t part_start = (int64_t)p * a.ipp;
  const int64_t part_end = std::min<int64_t>(I, part_start + a.ipp);

  for (int e = tid; e < a.img_n / 4; e += 256) dm_lds4[e] = reinterpret_cast<const float4*>(a.img)[e];
  for (int e = tid; e < NU * DM_W / 4; e += 256) {
    const int64_t b = ublk + e / (DM_W / 4);
    reinterpret_cast<float4*>(ps)[e] =
        b < B ? reinterpret_cast<const float4*>(a.P + b * DM_W)[e % (DM_W / 4)]
              : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int e = tid; e < NU * MFP; e += 256) {
    const int c = e % MFP;
    const int64_t b = ublk + e / MFP;
    const int64_t u = b < B ? a.uids[b] : -1;
    us[e] = (u >= 0 && u < a.num_users && c < a.mf) ? a.gu[u * a.mf + c] : 0.f;
  }
  for (int e = tid; e < MFP + 64; e += 256)
    wps[e] = e < a.mf ? a.wp[e] : (e >= MFP && e - MFP < a.dl) ? a.wp[a.mf + e - MFP] : 0.f;

  WaveTopK<1> L[WU];
  int nm[WU], mpos[WU], mend[WU];  // wave-uniform mask cursors (mask nnz < 2^31)
  bool uok[WU];
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    L[u].init();
    nm[u] = INT_BIG;
    mpos[u] = 0;
    mend[u] = 0;
    const int64_t b = ublk + wave * WU + u;
    const int64_t id = b < B ? a.uids[b] : 0;
    uok[u] = id >= 0 && id < a.num_users;
    if (b < B && !uok[u] && p == 0 && lane == 0) hnm_flag(a.err, HNM_ERR_OOB);
    if (!DENSE && a.mptr && b < B) {
      const int64_t lo = a.mptr[b], hi = a.mptr[b + 1];
      mpos[u] = (int)mask_lower_bound(a.midx, lo, hi, (int)part_start);
      mend[u] = (int)hi;
      nm[u] = mpos[u] < mend[u] ? a.midx[mpos[u]] : INT_BIG;
    }
  }

  // item tile staging through registers: issued before a tile's compute, written to the other
  // LDS buffer after it
  float4 qst[2], gst[GF4];
  auto load_tile = [&](int64_t base) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f = tid + 256 * q;
      const int64_t item = base + (f >> 4);
      qst[q] = item < part_end ? reinterpret_cast<const float4*>(a.Q + item * DM_W)[f & 15]
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < GF4; ++q) {
      const int f = tid + 256 * q;
      const int64_t item = base + f / (MFP / 4);
      gst[q] = item < part_end ? reinterpret_cast<const float4*>(a.G + item * MFP)[f % (MFP / 4)]
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f = tid + 256 * q;
      *reinterpret_cast<float4*>(&qs[(buf * TILE + (f >> 4)) * DM_QRS + 4 * (f & 15)]) = qst[q];
    }
#pragma unroll
    for (int q = 0; q < GF4; ++q) {
      const int f = tid + 256 * q;
      *reinterpret_cast<float4*>(&gs[(buf * TILE + f / (MFP / 4)) * GRS + 4 * (f % (MFP / 4))]) =
          gst[q];
    }
  };

  const int64_t ntiles = part_end > part_start ? hnm_cdiv(part_end - part_start, TILE) : 0;
  if (ntiles > 0) {
    load_tile(part_start);
    store_tile(0);
  }
  __syncthreads();

  const float bpv = a.bp[0];
  const float* wm = wps + MFP;
  const int meta1 = a.meta[1];
  const f32x16 zero16 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                         0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t tt = 0; tt < ntiles; ++tt) {
    const int buf = 0;
    const int64_t base = part_start + tt * TILE;
    if (tt + 1 < ntiles) load_tile(base + TILE);
    const float* qrow = &qs[(buf * TILE + j) * DM_QRS];
    const float* grow = &gs[(buf * TILE + j) * GRS];
    const int64_t item = base + j;
    const bool ivalid = item < part_end;
    const int64_t tile_end = std::min<int64_t>(base + TILE, part_end);

#pragma unroll
    for (int up = 0; up < WU; up += 2) {
      const int urA = wave * WU + up, urB = urA + 1;
      const int64_t bA = ublk + urA, bB = bA + 1;
      if (bA >= B) break;
      const float* ur = &us[(h ? urB : urA) * MFP];
      // the chain of this half's user: GMF terms first, s = fma(wp[c], g_u[c] * g_i[c], s),
      // eight terms at a time (interleaved with layer 2's MFMAs below)
      float s = 0.f;
      auto gmf8 = [&](int g) {
#pragma unroll
        for (int c = 8 * g; c < 8 * g + 8; c += 4) {
          const float4 gv = *reinterpret_cast<const float4*>(grow + c);
          const float4 xv = *reinterpret_cast<const float4*>(ur + c);
          const float4 wv = *reinterpret_cast<const float4*>(wps + c);
          s = fmaf(wv.x, xv.x * gv.x, s);
          s = fmaf(wv.y, xv.y * gv.y, s);
          s = fmaf(wv.z, xv.z * gv.z, s);
          s = fmaf(wv.w, xv.w * gv.w, s);
        }
      };
      if (a.nl == 1) {
#pragma unroll
        for (int g = 0; g < MFP / 8; ++g) gmf8(g);
        // single Linear: the MLP output is relu(P + Q) itself, unit jj at pair-permuted column
        const float* pr = &ps[(h ? urB : urA) * DM_W];
        for (int jj = 0; jj < a.dl; ++jj) {
          const int c = (jj & 1) * (DM_W / 2) + (jj >> 1);
          s = fmaf(wm[jj], fmaxf(pr[c] + qrow[c], 0.f), s);
        }
      } else {
        // layer 2 (the first MFMA layer): B operand relu(P + Q) from the LDS tile
        f32x16 cA0, cA1, cB0, cB1;
        {
          const float* pA = &ps[urA * DM_W + h * (DM_W / 2)];
          const float* pB = &ps[urB * DM_W + h * (DM_W / 2)];
          const float* qh = qrow + h * (DM_W / 2);
          const int ks4 = (meta1 >> 16) & 15;
          const bool two = NT > 1 && (meta1 >> 20) > 1;
          const float* A0 = img + (meta1 & 0xffff) + 4 * lane;
          const float* A1 = A0 + ks4 * 256;
          const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
          {  // group 0: the accumulators start from 0
            const float4 q = *reinterpret_cast<const float4*>(qh);
            const float4 pa = *reinterpret_cast<const float4*>(pA);
            const float4 pb = *reinterpret_cast<const float4*>(pB);
            const float4 w0 = *reinterpret_cast<const float4*>(A0);
            const float4 w1 = two ? *reinterpret_cast<const float4*>(A1) : z4;
            DM_STEP(w0.x, w1.x, fmaxf(pa.x + q.x, 0.f), fmaxf(pb.x + q.x, 0.f), zero16, zero16,
                    zero16, zero16);
            DM_ACC(w0.y, w1.y, fmaxf(pa.y + q.y, 0.f), fmaxf(pb.y + q.y, 0.f));
            DM_ACC(w0.z, w1.z, fmaxf(pa.z + q.z, 0.f), fmaxf(pb.z + q.z, 0.f));
            DM_ACC(w0.w, w1.w, fmaxf(pa.w + q.w, 0.f), fmaxf(pb.w + q.w, 0.f));
            gmf8(0);
          }
          for (int s4 = 1; s4 < ks4; ++s4) {
            const float4 q = *reinterpret_cast<const float4*>(qh + 4 * s4);
            const float4 pa = *reinterpret_cast<const float4*>(pA + 4 * s4);
            const float4 pb = *reinterpret_cast<const float4*>(pB + 4 * s4);
            const float4 w0 = *reinterpret_cast<const float4*>(A0 + 256 * s4);
            const float4 w1 = two ? *reinterpret_cast<const float4*>(A1 + 256 * s4) : z4;
            DM_ACC(w0.x, w1.x, fmaxf(pa.x + q.x, 0.f), fmaxf(pb.x + q.x, 0.f));
            DM_ACC(w0.y, w1.y, fmaxf(pa.y + q.y, 0.f), fmaxf(pb.y + q.y, 0.f));
            DM_ACC(w0.z, w1.z, fmaxf(pa.z + q.z, 0.f), fmaxf(pb.z + q.z, 0.f));
            DM_ACC(w0.w, w1.w, fmaxf(pa.w + q.w, 0.f), fmaxf(pb.w + q.w, 0.f));
            if (s4 < MFP / 8) gmf8(s4);
          }
          for (int g = ks4; g < MFP / 8; ++g) gmf8(g);
        }
        f32x16 xA0, xA1, xB0, xB1;
        auto epilogue = [&](int meta) {  // x = relu(acc + b): fmaxf(acc + b, 0), the chain's
          const int ks4 = (meta >> 16) & 15, nt = meta >> 20;
          const float* bi = img + (meta & 0xffff) + nt * ks4 * 256 + 16 * h;
          const bool two = NT > 1 && nt > 1;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float b0 = bi[r];
            xA0[r] = fmaxf(cA0[r] + b0, 0.f);
            xB0[r] = fmaxf(cB0[r] + b0, 0.f);
            if (NT > 1) {
              const float b1 = two ? bi[32 + r] : 0.f;
              xA1[r] = two ? fmaxf(cA1[r] + b1, 0.f) : 0.f;
              xB1[r] = two ? fmaxf(cB1[r] + b1, 0.f) : 0.f;
            }
          }
        };
        epilogue(meta1);
        // layers 3..: B operand of step s = 16t + r is x_t[r] (unit 2s + h), from registers
        for (int l = 2; l < a.nl - a.last16; ++l) {
          const int meta = a.meta[l];
          const int ks4 = (meta >> 16) & 15;
          const bool two = NT > 1 && (meta >> 20) > 1;
          const float* A0 = img + (meta & 0xffff) + 4 * lane;
          const float* A1 = A0 + ks4 * 256;
#pragma unroll
          for (int s4 = 0; s4 < 4 * NT; ++s4) {
            if (s4 < ks4) {
              const float4 w0 = *reinterpret_cast<const float4*>(A0 + 256 * s4);
              const float4 w1 = two ? *reinterpret_cast<const float4*>(A1 + 256 * s4)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
              const int r0 = (4 * s4) & 15;
              const f32x16& vA = s4 < 4 ? xA0 : xA1;
              const f32x16& vB = s4 < 4 ? xB0 : xB1;
              if (s4 == 0)
                DM_STEP(w0.x, w1.x, vA[r0], vB[r0], zero16, zero16, zero16, zero16);
              else
                DM_ACC(w0.x, w1.x, vA[r0], vB[r0]);
              DM_ACC(w0.y, w1.y, vA[r0 + 1], vB[r0 + 1]);
              DM_ACC(w0.z, w1.z, vA[r0 + 2], vB[r0 + 2]);
              DM_ACC(w0.w, w1.w, vA[r0 + 3], vB[r0 + 3]);
            }
          }
          epilogue(meta);
        }
        if (a.last16) {
          // last layer (<= 16 outputs) on v_mfma_f32_16x16x4f32: half the matrix cycles of a
          // 32-unit tile.  Step s takes input units 4s .. 4s + 3 = registers (2s, 2s + 1) of x
          // (units 2r + h); a permlane32 then a permlane16 swap turn the register pair into the
          // B operands of the two 16-item blocks (lane l: item l & 15 of the block, unit
          // 4s + (l >> 4)).
          const int meta = a.meta[a.nl - 1];
          const int g4 = (meta >> 16) & 15;
          const float* A16 = img + (meta & 0xffff) + 4 * lane;
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          f32x4 dA0 = z, dA1 = z, dB0 = z, dB1 = z;  // (user, item block)
          float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int st = 0; st < 8 * NT; ++st) {
            if (st < 4 * g4) {
              // one conflict-free ds_read_b128 per 4 steps (lane-contiguous 16 B)
              if ((st & 3) == 0) w4 = *reinterpret_cast<const float4*>(A16 + 256 * (st >> 2));
              const float w = (st & 3) == 0 ? w4.x : (st & 3) == 1 ? w4.y : (st & 3) == 2 ? w4.z : w4.w;
              const int t = st >> 3, r = (2 * st) & 15;
              const auto pa = __builtin_amdgcn_permlane32_swap(
                  __float_as_uint(t ? xA1[r] : xA0[r]), __float_as_uint(t ? xA1[r + 1] : xA0[r + 1]),
                  false, false);
              const auto qa = __builtin_amdgcn_permlane16_swap(pa[0], pa[1], false, false);
              const auto pb = __builtin_amdgcn_permlane32_swap(
                  __float_as_uint(t ? xB1[r] : xB0[r]), __float_as_uint(t ? xB1[r + 1] : xB0[r + 1]),
                  false, false);
              const auto qb = __builtin_amdgcn_permlane16_swap(pb[0], pb[1], false, false);
              dA0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w, __uint_as_float(qa[0]), dA0, 0, 0, 0);
              dA1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w, __uint_as_float(qa[1]), dA1, 0, 0, 0);
              dB0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w, __uint_as_float(qb[0]), dB0, 0, 0, 0);
              dB1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w, __uint_as_float(qb[1]), dB1, 0, 0, 0);
            }
          }
          // lane l holds units 4 (l >> 4) + i of item (l & 15) of its block; a 4 x 4 transpose
          // of (block set, 16-lane row) by permlane32 + permlane16 swaps brings all 16 units
          // of (user h, item l & 31) into lane l, the lane that holds that pair's chain
          const float* b16 = img + (meta & 0xffff) + g4 * 256;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const auto x02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(dA0[i]),
                                                              __float_as_uint(dB0[i]), false, false);
            const auto x13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(dA1[i]),
                                                              __float_as_uint(dB1[i]), false, false);
            const auto y01 = __builtin_amdgcn_permlane16_swap(x02[0], x13[0], false, false);
            const auto y23 = __builtin_amdgcn_permlane16_swap(x02[1], x13[1], false, false);
            dA0[i] = __uint_as_float(y01[0]);  // unit i
            dA1[i] = __uint_as_float(y01[1]);  // unit 4 + i
            dB0[i] = __uint_as_float(y23[0]);  // unit 8 + i
            dB1[i] = __uint_as_float(y23[1]);  // unit 12 + i
          }
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            if (u < a.dl) {
              const float v = (u < 4 ? dA0 : u < 8 ? dA1 : u < 12 ? dB0 : dB1)[u & 3];
              s = fmaf(wm[u], fmaxf(v + b16[u], 0.f), s);
            }
          }
        } else {
        // MLP terms of the chain: one permlane32 swap of (x_A, x_B) gives every lane of half 0
        // user A's even (r[0]) and odd (r[1]) units, and every lane of half 1 user B's
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int jj = 32 * t + 2 * r;
            if (jj < a.dl) {
              const auto sw = __builtin_amdgcn_permlane32_swap(
                  __float_as_uint(t ? xA1[r] : xA0[r]), __float_as_uint(t ? xB1[r] : xB0[r]),
                  false, false);
              s = fmaf(wm[jj], __uint_as_float(sw[0]), s);
              s = fmaf(wm[jj + 1], __uint_as_float(sw[1]), s);  // wm zero past dl: exact
            }
          }
        }
        }
      }
      float score = s + bpv;
      const int64_t bM = h ? bB : bA;
      const bool okM = ivalid && bM < B;
      if (!(h ? uok[up + 1] : uok[up])) score = __builtin_nanf("");
      if (DENSE) {
        if (okM) a.out[bM * a.ldo + item] = score;
      } else {
        while (nm[up] < tile_end) {  // wave-uniform mask cursors
          if (h == 0 && item == nm[up]) score = -__builtin_inff();
          ++mpos[up];
          nm[up] = mpos[up] < mend[up] ? a.midx[mpos[up]] : INT_BIG;
        }
        while (nm[up + 1] < tile_end) {
          if (h == 1 && item == nm[up + 1]) score = -__builtin_inff();
          ++mpos[up + 1];
          nm[up + 1] = mpos[up + 1] < mend[up + 1] ? a.midx[mpos[up + 1]] : INT_BIG;
        }
        L[up].offer(score, (int)item, okM && h == 0, a.K);
        L[up + 1].offer(score, (int)item, okM && h == 1, a.K);
      }
    }

    // tile t + 1 into the other buffer (every wave finished reading it before the last barrier)
    if (tt + 1 < ntiles) {
      __syncthreads();
      store_tile(0);
    }
    __syncthreads();
  }

  if (!DENSE) {
#pragma unroll
    for (int u = 0; u < WU; ++u) {
      const int64_t b = ublk + wave * WU + u;
      if (b < B) L[u].store(a.cv + (b * a.NP + p) * a.K, a.ci + (b * a.NP + p) * a.K, a.K);
    }
  }
}
#undef DM_ACC
#undef DM_STEP

// ------------------------------------------------------------------ host side
static hnm_status deep_check(const hnm_ncf_deep_weights* w) {
  HNM_REQUIRE(w && w->gmf_user && w->gmf_item && w->mlp_user && w->mlp_item && w->wp && w->bp,
              HNM_EINVAL, "ncf_deep: NULL weight");
  HNM_REQUIRE(w->nl >= 1 && w->nl <= 8, HNM_EUNSUPPORTED, "ncf_deep: 1 <= layers <= 8 (got %d)",
              (int)w->nl);
  HNM_REQUIRE(w->mf >= 1 && w->num_users > 0 && w->num_items > 0, HNM_EINVAL,
              "ncf_deep: bad sizes");
  HNM_REQUIRE(w->dims[0] >= 2 && w->dims[0] % 2 == 0, HNM_EINVAL,
              "ncf_deep: mlp_dims[0] must be even (two embedding halves)");
  for (int l = 0; l < w->nl; ++l) {
    HNM_REQUIRE(w->w[l] && w->b[l], HNM_EINVAL, "ncf_deep: layer %d NULL", l);
    HNM_REQUIRE(w->dims[l + 1] >= 1 && w->dims[l + 1] <= 512, HNM_EUNSUPPORTED,
                "ncf_deep: layer widths 1..512 (got %d)", (int)w->dims[l + 1]);
  }
  return HNM_OK;
}

// MFMA tile layout of a tower; false when it does not fit (widths > 64, mf > 128, an LDS
// image beyond a CU's 160 KB)
struct DeepMLayout {
  DeepPack pk;
  int mfp;     // GMF width padded to 32, 64 or 128
  int nt;      // max 32-unit tiles of an MFMA layer (1 or 2)
  size_t lds;  // dynamic LDS bytes
};
static bool deep_mfma_layout(const hnm_ctx* ctx, const hnm_ncf_deep_weights* w, DeepMLayout* o) {
  if (!ctx->deep_mfma || w->mf > 128 || w->num_items >= INT_BIG) return false;
  for (int l = 1; l <= w->nl; ++l)
    if (w->dims[l] > 64) return false;
  DeepPack& pk = o->pk;
  pk = DeepPack{};
  pk.nl = w->nl;
  for (int l = 0; l <= w->nl; ++l) pk.dims[l] = w->dims[l];
  int off = 0;
  o->nt = 1;
  pk.last16 = w->nl >= 3 && w->dims[w->nl] <= 16;
  for (int l = 1; l < w->nl; ++l) {
    pk.w[l] = w->w[l];
    pk.b[l] = w->b[l];
    pk.aoff[l] = off;
    if (pk.last16 && l == w->nl - 1) {  // 16x16x4 steps of 4 input units, bias 16 floats
      pk.ks4[l] = (int)hnm_cdiv(hnm_cdiv(w->dims[l], 4), 4);
      pk.nt[l] = 1;
      pk.boff[l] = off + pk.ks4[l] * 256;
      off = pk.boff[l] + 16;
      continue;
    }
    pk.ks4[l] = (int)hnm_cdiv(hnm_cdiv(w->dims[l], 2), 4);
    pk.nt[l] = (int)hnm_cdiv(w->dims[l + 1], 32);
    pk.boff[l] = off + pk.nt[l] * pk.ks4[l] * 256;
    off = pk.boff[l] + pk.nt[l] * 32;
    o->nt = std::max(o->nt, pk.nt[l]);
  }
  pk.img_n = off;
  o->mfp = w->mf <= 32 ? 32 : w->mf <= 64 ? 64 : 128;
  o->lds = (size_t)4 * (off + TILE * DM_QRS + TILE * (o->mfp + 4) + DM_NU * DM_W +
                        DM_NU * o->mfp + o->mfp + 64);
  return o->lds <= 160 * 1024 && off < 65536;
}

// Workspace: P [B, 64] and Q [I, 64] (pair-permuted, zero padded), the packed weight image,
// the GMF item rows padded to mfp columns when the table is not already so, then `extra`
// bytes for the caller.
static hnm_status deep_mfma_tables(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                   const DeepMLayout& lay, const int64_t* ids, int64_t B,
                                   size_t extra, DeepMArgs* a, void** extra_out) {
  const int64_t I = w->num_items;
  const int h = w->dims[0] / 2, d1 = w->dims[1];
  const bool gcopy = w->mf != lay.mfp || (uintptr_t)w->gmf_item % 16 != 0;
  const size_t szP = hnm_align((size_t)B * DM_W * 4), szQ = hnm_align((size_t)I * DM_W * 4);
  const size_t szI = hnm_align((size_t)std::max(lay.pk.img_n, 4) * 4);
  const size_t szG = gcopy ? hnm_align((size_t)I * lay.mfp * 4) : 0;
  void* ws;
  hnm_status st = hnm_workspace(ctx, szP + szQ + szI + szG + extra, &ws);
  if (st) return st;
  char* cur = (char*)ws;
  float* P = (float*)cur; cur += szP;
  float* Q = (float*)cur; cur += szQ;
  float* img = (float*)cur; cur += szI;
  float* Gc = (float*)cur; cur += szG;
  *extra_out = cur;
  if (d1 < DM_W) {
    HNM_HIP_CHECK(hipMemsetAsync(P, 0, szP + szQ, ctx->stream));
  }
  st = hnm_linear_rows_f32(ctx, w->mlp_user, h, ids, w->num_users, B, h, w->w[0], 2 * h,
                           w->b[0], d1, P, DM_W, 1);
  if (st) return st;
  st = hnm_linear_rows_f32(ctx, w->mlp_item, h, nullptr, I, I, h, w->w[0] + h, 2 * h, nullptr,
                           d1, Q, DM_W, 1);
  if (st) return st;
  if (gcopy) {
    HNM_HIP_CHECK(hipMemsetAsync(Gc, 0, szG, ctx->stream));
    HNM_HIP_CHECK(hipMemcpy2DAsync(Gc, lay.mfp * 4, w->gmf_item, w->mf * 4, w->mf * 4, I,
                                   hipMemcpyDeviceToDevice, ctx->stream));
  }
  if (lay.pk.img_n > 0) {
    hipLaunchKernelGGL(deep_pack_kernel, dim3((unsigned)std::min<int64_t>(
                                             256, hnm_cdiv(lay.pk.img_n, 256))),
                       dim3(256), 0, ctx->stream, lay.pk, img);
    HNM_LAUNCH_CHECK();
  }
  DeepMArgs& m = *a;
  m = DeepMArgs{};
  m.P = P;
  m.Q = Q;
  m.gu = w->gmf_user;
  m.G = gcopy ? Gc : w->gmf_item;
  m.uids = ids;
  m.img = img;
  m.wp = w->wp;
  m.bp = w->bp;
  m.num_users = w->num_users;
  m.num_items = I;
  m.B = B;
  m.mf = w->mf;
  m.nl = w->nl;
  m.dl = w->dims[w->nl];
  m.img_n = lay.pk.img_n;
  m.last16 = lay.pk.last16;
  for (int l = 1; l < w->nl; ++l)
    m.meta[l] = lay.pk.aoff[l] | lay.pk.ks4[l] << 16 | lay.pk.nt[l] << 20;
  m.K = 1;
  m.err = ctx->err_dev;
  return HNM_OK;
}

template <int NT, int MFP, bool DENSE>
static hnm_status deep_mfma_launch1(hnm_ctx* ctx, DeepMArgs a, const DeepMLayout& lay) {
  const int64_t ublocks = hnm_cdiv(a.B, DM_NU);
  const Partition part = choose_partition(a.num_items, ublocks, ctx->num_cus, TILE, NT == 1 ? 3 : 2);
  a.ipp = part.ipp;
  a.NP = part.np;
  HNM_REQUIRE(ublocks < ((int64_t)1 << 31), HNM_EUNSUPPORTED, "ncf_deep: batch too large");
  if (lay.lds > 64 * 1024)  // e.g. two 64-wide MFMA layers: one workgroup a CU
    (void)hipFuncSetAttribute((const void*)ncf_deep_mfma_kernel<NT, MFP, DENSE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lay.lds);
  hnm_timer_begin(ctx, HNM_TIME_SCORE);
  hipLaunchKernelGGL((ncf_deep_mfma_kernel<NT, MFP, DENSE>),
                     dim3((unsigned)ublocks, (unsigned)part.np), dim3(256), lay.lds, ctx->stream, a);
  hnm_timer_end(ctx, HNM_TIME_SCORE);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

// NT = 1 when every MFMA layer has <= 32 outputs (one 32-unit tile: half the registers), else 2
template <bool DENSE>
static hnm_status deep_mfma_launch(hnm_ctx* ctx, const DeepMArgs& a, const DeepMLayout& lay) {
#define HNM_DEEP_MFP(NTV)                                                  \
  return lay.mfp == 32   ? deep_mfma_launch1<NTV, 32, DENSE>(ctx, a, lay)  \
         : lay.mfp == 64 ? deep_mfma_launch1<NTV, 64, DENSE>(ctx, a, lay)  \
                         : deep_mfma_launch1<NTV, 128, DENSE>(ctx, a, lay);
  if (lay.nt > 1) {
    HNM_DEEP_MFP(2)
  }
  HNM_DEEP_MFP(1)
#undef HNM_DEEP_MFP
}

// the per-pair LDS kernel (any width <= 512): P [B, d1] and Q [nq, d1] in the workspace
// (natural order), then `extra` bytes
static hnm_status deep_scalar_tables(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                     const int64_t* ids, int64_t B, const int64_t* item_ids,
                                     size_t extra, DeepArgs* a, void** extra_out) {
  const bool dense = item_ids == nullptr;
  const int h = w->dims[0] / 2, d1 = w->dims[1];
  const int64_t nq = dense ? w->num_items : B;
  const size_t szP = hnm_align((size_t)B * d1 * 4), szQ = hnm_align((size_t)nq * d1 * 4);
  void* ws;
  hnm_status st = hnm_workspace(ctx, szP + szQ + extra, &ws);
  if (st) return st;
  float* P = (float*)ws;
  float* Q = (float*)((char*)ws + szP);
  if (extra_out) *extra_out = (char*)ws + szP + szQ;
  st = hnm_linear_rows_f32(ctx, w->mlp_user, h, ids, w->num_users, B, h, w->w[0], 2 * h,
                           w->b[0], d1, P, d1, 0);
  if (st) return st;
  st = hnm_linear_rows_f32(ctx, w->mlp_item, h, item_ids, w->num_items, nq, h, w->w[0] + h,
                           2 * h, nullptr, d1, Q, d1, 0);
  if (st) return st;
  *a = DeepArgs{};
  a->P = P;
  a->Q = Q;
  a->gu = w->gmf_user;
  a->gi = w->gmf_item;
  a->uids = ids;
  a->iids = item_ids;
  for (int l = 0; l < w->nl; ++l) {
    a->w[l] = w->w[l];
    a->b[l] = w->b[l];
  }
  a->wp = w->wp;
  a->bp = w->bp;
  a->num_users = w->num_users;
  a->num_items = w->num_items;
  a->B = B;
  a->nq = nq;
  a->mf = w->mf;
  a->nl = w->nl;
  a->d1 = d1;
  for (int l = 0; l <= w->nl; ++l) a->dims[l] = w->dims[l];
  return HNM_OK;
}

// dense rows of users [b0, b0 + nb) of the tables `all` into out (row stride ldo)
static hnm_status deep_scalar_dense(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                    const DeepArgs& all, int64_t b0, int64_t nb, float* out,
                                    int64_t ldo) {
  int maxw = 1;
  for (int l = 1; l <= w->nl; ++l) maxw = std::max(maxw, (int)w->dims[l]);
  const int TP = maxw <= 128 ? 64 : maxw <= 256 ? 32 : 16;
  const size_t lds = (size_t)2 * TP * maxw * 4;
  // grid.y = the chunk's users (< 65536 per launch): any B
  for (int64_t c0 = 0; c0 < nb; c0 += 65535) {
    const int64_t n = std::min<int64_t>(65535, nb - c0);
    DeepArgs a = all;
    a.P = all.P + (b0 + c0) * all.d1;
    a.uids = all.uids + b0 + c0;
    a.out = out + c0 * ldo;
    a.ldo = ldo;
    a.B = n;
    const dim3 g((unsigned)hnm_cdiv(w->num_items, TP), (unsigned)n);
    if (TP == 64)
      hipLaunchKernelGGL((ncf_deep_kernel<64, true>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
    else if (TP == 32)
      hipLaunchKernelGGL((ncf_deep_kernel<32, true>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
    else
      hipLaunchKernelGGL((ncf_deep_kernel<16, true>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
    HNM_LAUNCH_CHECK();
  }
  return HNM_OK;
}

extern "C" hnm_status hnm_ncf_deep_scores_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                              const int64_t* user_ids, int64_t B,
                                              const int64_t* item_ids, float* out, int64_t ldo) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = deep_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ((user_ids && out) || B == 0), HNM_EINVAL, "ncf_deep: NULL argument");
  const bool dense = item_ids == nullptr;
  HNM_REQUIRE(!dense || ldo >= w->num_items, HNM_EINVAL, "ncf_deep: ldo < num_items");
  if (B <= 0) return HNM_OK;
  DeepMLayout lay;
  if (dense && deep_mfma_layout(ctx, w, &lay)) {
    DeepMArgs m;
    void* extra;
    if ((st = deep_mfma_tables(ctx, w, lay, user_ids, B, 0, &m, &extra))) return st;
    m.out = out;
    m.ldo = ldo;
    return deep_mfma_launch<true>(ctx, m, lay);
  }
  DeepArgs a;
  if ((st = deep_scalar_tables(ctx, w, user_ids, B, item_ids, 0, &a, nullptr))) return st;
  if (dense) {
    hnm_timer_begin(ctx, HNM_TIME_SCORE);
    st = deep_scalar_dense(ctx, w, a, 0, B, out, ldo);
    hnm_timer_end(ctx, HNM_TIME_SCORE);
    return st;
  }
  a.out = out;
  a.ldo = ldo;
  int maxw = 1;
  for (int l = 1; l <= w->nl; ++l) maxw = std::max(maxw, (int)w->dims[l]);
  const int TP = maxw <= 128 ? 64 : maxw <= 256 ? 32 : 16;
  const size_t lds = (size_t)2 * TP * maxw * 4;
  const dim3 g((unsigned)hnm_cdiv(B, TP));
  if (TP == 64)
    hipLaunchKernelGGL((ncf_deep_kernel<64, false>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
  else if (TP == 32)
    hipLaunchKernelGGL((ncf_deep_kernel<32, false>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
  else
    hipLaunchKernelGGL((ncf_deep_kernel<16, false>), g, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}

static hnm_status deep_topk_exact(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                  const int64_t* ids, int64_t B, const int64_t* mptr,
                                  const int32_t* midx, int K, float* ov, int64_t* oi) {
  const int64_t I = w->num_items;
  DeepMLayout lay;
  hnm_status st;
  if (deep_mfma_layout(ctx, w, &lay)) {
    const Partition part = choose_partition(I, hnm_cdiv(B, DM_NU), ctx->num_cus, TILE, lay.nt == 1 ? 3 : 2);
    const size_t szC = hnm_align((size_t)B * part.np * K * 4);
    DeepMArgs m;
    void* extra;
    if ((st = deep_mfma_tables(ctx, w, lay, ids, B, 2 * szC, &m, &extra))) return st;
    m.cv = (float*)extra;
    m.ci = (int32_t*)((char*)extra + szC);
    m.mptr = mptr;
    m.midx = midx;
    m.K = K;
    st = deep_mfma_launch<false>(ctx, m, lay);
    if (st) return st;
    return hnm_topk_merge_i32(ctx, m.cv, m.ci, B, 1, 0, (int64_t)part.np * K, part.np * K, K, ov,
                              oi);
  }
  // wide towers: dense rows of <= 256 MB per user chunk in the workspace + the row top-k
  const int64_t step = std::max<int64_t>(1, std::min<int64_t>(B, ((int64_t)1 << 26) / I));
  DeepArgs a;
  void* extra;
  if ((st = deep_scalar_tables(ctx, w, ids, B, nullptr, hnm_align((size_t)step * I * 4), &a,
                               &extra)))
    return st;
  float* buf = (float*)extra;
  for (int64_t b0 = 0; b0 < B; b0 += step) {
    const int64_t nb = std::min<int64_t>(step, B - b0);
    hnm_timer_begin(ctx, HNM_TIME_SCORE);
    st = deep_scalar_dense(ctx, w, a, b0, nb, buf, I);
    hnm_timer_end(ctx, HNM_TIME_SCORE);
    if (st) return st;
    st = hnm_topk_rows_strided(ctx, buf, I, nb, I, mptr ? mptr + b0 : nullptr, midx, K,
                               ov ? ov + b0 * K : nullptr, oi + b0 * K, 1);
    if (st) return st;
  }
  return HNM_OK;
}

__global__ void deep_stats_kernel(unsigned long long* stats, int64_t B) {
  atomicAdd(&stats[0], (unsigned long long)B);
  atomicAdd(&stats[2], (unsigned long long)B);
}

__global__ void deep_scatter_rows_kernel(const int32_t* __restrict__ rows, int n, int K,
                                        const float* __restrict__ tv, const int64_t* __restrict__ ti,
                                        float* __restrict__ ov, int64_t* __restrict__ oi) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= (int64_t)n * K) return;
  const int64_t o = (int64_t)rows[x / K] * K + x % K;
  if (ov) ov[o] = tv[o];
  oi[o] = ti[o];
}

// Round 6: towers [2 h0, h1 <= 64, h2 <= 32, h3 <= 16] (the bench's [128, 64, 32, 16]) take the
// certified f16 pre-filter (ncf_cert.hip: the two-layer scan with a layer-3 matrix epilogue, exact
// deep re-scoring -- results bitwise the exact path's); the rows it queues (unusable bound,
// overflowing segments) take the exact deep scan: one B = 1 call each for a few rows, else the
// whole chunk exactly with those rows' lists copied over (the count is read back: one sync).
// When the proxy rows predict that the bound cannot prune (a worst-case bound through two
// absolute-value layers wider than the score spread: init-like weights, tests/test_gpu_ncf_deep.py
// prints the ratio) the whole call takes the exact kernels after the begin phase.
static hnm_status deep_topk_chunk(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                  const int64_t* ids, int64_t B, const int64_t* mptr,
                                  const int32_t* midx, int K, float* ov, int64_t* oi) {
  if (!(ctx->prefilter && B >= 16 && ncf_deep_cert_eligible(w, K)))
    return deep_topk_exact(ctx, w, ids, B, mptr, midx, K, ov, oi);
  int32_t *orows = nullptr, *ocnt = nullptr;
  bool pruned = false;
  hnm_status st = ncf_deep_cert(ctx, w, ids, B, mptr, midx, K, ov, oi, &orows, &ocnt, &pruned);
  if (st) return st;
  if (!pruned) {  // the bound is wider than the rows' spread: the exact kernels for every row
    if (ctx->stats_on) {  // counted as B rows scored, all B on the exact fallback
      hipLaunchKernelGGL(deep_stats_kernel, dim3(1), dim3(1), 0, ctx->stream, ctx->stats_dev, B);
      HNM_LAUNCH_CHECK();
    }
    return deep_topk_exact(ctx, w, ids, B, mptr, midx, K, ov, oi);
  }
  int32_t n = 0;
  HNM_HIP_CHECK(hipMemcpyAsync(&n, ocnt, 4, hipMemcpyDeviceToHost, ctx->stream));
  HNM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  if (n <= 0) return HNM_OK;
  if (n <= 16) {  // the rows' list is read before the exact calls reuse the workspace
    std::vector<int32_t> rows((size_t)n);
    HNM_HIP_CHECK(hipMemcpy(rows.data(), orows, (size_t)n * 4, hipMemcpyDeviceToHost));
    for (int32_t r : rows) {
      st = deep_topk_exact(ctx, w, ids + r, 1, mptr ? mptr + r : nullptr, midx, K,
                           ov ? ov + (int64_t)r * K : nullptr, oi + (int64_t)r * K);
      if (st) return st;
    }
    return HNM_OK;
  }
  int32_t* drows = nullptr;
  float* tv = nullptr;
  int64_t* ti = nullptr;
  if (hipMallocAsync((void**)&drows, (size_t)n * 4, ctx->stream) != hipSuccess ||
      hipMallocAsync((void**)&tv, (size_t)B * K * 4, ctx->stream) != hipSuccess ||
      hipMallocAsync((void**)&ti, (size_t)B * K * 8, ctx->stream) != hipSuccess) {
    if (drows) (void)hipFreeAsync(drows, ctx->stream);
    if (tv) (void)hipFreeAsync(tv, ctx->stream);
    hnm_set_error("ncf_deep_topk: fallback buffers: hipMallocAsync failed");
    return HNM_ENOMEM;
  }
  HNM_HIP_CHECK(hipMemcpyAsync(drows, orows, (size_t)n * 4, hipMemcpyDeviceToDevice, ctx->stream));
  st = deep_topk_exact(ctx, w, ids, B, mptr, midx, K, tv, ti);
  if (!st) {
    hipLaunchKernelGGL(deep_scatter_rows_kernel, dim3((unsigned)hnm_cdiv((int64_t)n * K, 256)),
                       dim3(256), 0, ctx->stream, drows, n, K, tv, ti, ov, oi);
    if (hipGetLastError() != hipSuccess) st = HNM_EHIP;
  }
  (void)hipFreeAsync(drows, ctx->stream);
  (void)hipFreeAsync(tv, ctx->stream);
  (void)hipFreeAsync(ti, ctx->stream);
  if (st == HNM_EHIP) hnm_set_error("ncf_deep_topk: fallback scatter launch failed");
  return st;
}

// Diagnostics of the deep certified pre-filter (no reference counterpart): approx[b, i] = the f16
// scan's score without bp, bound[b, i] its certified bound (real units): |approx + bp - exact| <=
// bound for every pair (tests check it on the full catalogue).
extern "C" hnm_status hnm_ncf_deep_prefilter_debug_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                                       const int64_t* user_ids, int64_t B,
                                                       float* approx, int64_t lda, float* bound) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = deep_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && user_ids && approx && bound && lda >= w->num_items, HNM_EINVAL,
              "ncf_deep_prefilter_debug: bad argument");
  HNM_REQUIRE(w->nl == 3 && w->dims[1] <= 64 && w->dims[2] <= 32 && w->dims[3] <= 16 &&
                  w->mf <= 64 && w->mf % 4 == 0 && w->num_items * 64 < ((int64_t)1 << 31),
              HNM_EUNSUPPORTED,
              "ncf_deep_prefilter_debug: the deep pre-filter covers towers [2 h0, <= 64, <= 32, "
              "<= 16], mf <= 64 (a multiple of 4), < 2^25 items");
  if (B <= 0) return HNM_OK;
  return ncf_deep_cert_debug(ctx, w, user_ids, B, approx, lda, bound);
}

extern "C" hnm_status hnm_ncf_deep_topk_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                            const int64_t* user_ids, int64_t B,
                                            const int64_t* mask_ptr, const int32_t* mask_idx,
                                            int k, float* out_val, int64_t* out_idx) {
  HNM_CTX_DEVICE(ctx);
  hnm_status st = deep_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ((user_ids && out_idx) || B == 0), HNM_EINVAL, "ncf_deep_topk: NULL argument");
  HNM_REQUIRE(k >= 1 && k <= 64 && k <= w->num_items, HNM_EINVAL,
              "ncf_deep_topk: 1 <= k <= min(64, num_items)");
  HNM_REQUIRE(w->num_items < INT_BIG, HNM_EUNSUPPORTED, "ncf_deep_topk: too many items");
  // chunks of rows bound the per-(row, partition) candidate lists
  constexpr int64_t CHUNK = 32768;
  for (int64_t b0 = 0; b0 < B; b0 += CHUNK) {
    const int64_t nb = std::min<int64_t>(CHUNK, B - b0);
    st = deep_topk_chunk(ctx, w, user_ids + b0, nb, mask_ptr ? mask_ptr + b0 : nullptr, mask_idx,
                         k, out_val ? out_val + b0 * k : nullptr, out_idx + b0 * k);
    if (st) return st;
  }
  return HNM_OK;
}
