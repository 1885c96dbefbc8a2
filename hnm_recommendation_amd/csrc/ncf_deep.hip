// NeuralCF with an MLP tower of any depth, exact fp32 (reference `_build_mlp`,
// neural_cf.py:75-90: Linear -> ReLU -> Dropout for every consecutive pair of mlp_dims; eval
// mode, so Dropout is the identity).  The fused certified kernels (ncf.hip, ncf_cert.hip) cover
// the reference's default two-layer tower; every other tower takes this path:
//
//   layer 1 decomposed per row (hnm_linear_rows_f32): P_u = W1[:, :h] m_u + b1 once per user,
//   Q_i = W1[:, h:] m_i once per item, so a pair's first activation is relu(P_u + Q_i);
//   layers 2.. per pair: a workgroup holds TP pairs' activations in LDS (k-major, so the TP
//   lanes of a pair group read consecutive words) and 256 / TP lane groups share each layer's
//   output units (the weights are wave-uniform loads: one cache line serves the wave);
//   score = sum_j wp[j] g_u[j] g_i[j] + sum_j wp[mf + j] x_L[j] + bp (neural_cf.py:131-141).
// DENSE: pairs (b, i) for every item (predict_all_items, and recommend via the row top-k
// kernel); else pairs (user_ids[n], item_ids[n]) (forward).
#include "hnm_device.h"
#include "hnm_internal.h"

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

extern "C" hnm_status hnm_ncf_deep_scores_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                              const int64_t* user_ids, int64_t B,
                                              const int64_t* item_ids, float* out, int64_t ldo) {
  hnm_status st = deep_check(w);
  if (st) return st;
  HNM_REQUIRE(ctx && ((user_ids && out) || B == 0), HNM_EINVAL, "ncf_deep: NULL argument");
  const bool dense = item_ids == nullptr;
  HNM_REQUIRE(!dense || ldo >= w->num_items, HNM_EINVAL, "ncf_deep: ldo < num_items");
  if (B <= 0) return HNM_OK;
  const int h = w->dims[0] / 2, d1 = w->dims[1];
  const int64_t nq = dense ? w->num_items : B;
  const size_t szP = hnm_align((size_t)B * d1 * 4), szQ = hnm_align((size_t)nq * d1 * 4);
  void* ws;
  st = hnm_workspace(ctx, szP + szQ, &ws);
  if (st) return st;
  float* P = (float*)ws;
  float* Q = (float*)((char*)ws + szP);
  st = hnm_linear_rows_f32(ctx, w->mlp_user, h, user_ids, w->num_users, B, h, w->w[0], 2 * h,
                           w->b[0], d1, P, d1, 0);
  if (st) return st;
  st = hnm_linear_rows_f32(ctx, w->mlp_item, h, item_ids, w->num_items, nq, h, w->w[0] + h, 2 * h,
                           nullptr, d1, Q, d1, 0);
  if (st) return st;
  DeepArgs a{};
  a.P = P;
  a.Q = Q;
  a.gu = w->gmf_user;
  a.gi = w->gmf_item;
  a.uids = user_ids;
  a.iids = item_ids;
  for (int l = 0; l < w->nl; ++l) {
    a.w[l] = w->w[l];
    a.b[l] = w->b[l];
  }
  a.wp = w->wp;
  a.bp = w->bp;
  a.num_users = w->num_users;
  a.num_items = w->num_items;
  a.B = B;
  a.nq = nq;
  a.mf = w->mf;
  a.nl = w->nl;
  a.d1 = d1;
  for (int l = 0; l <= w->nl; ++l) a.dims[l] = w->dims[l];
  a.out = out;
  a.ldo = ldo;
  int maxw = 1;
  for (int l = 1; l <= w->nl; ++l) maxw = std::max(maxw, (int)w->dims[l]);
  const int TP = maxw <= 128 ? 64 : maxw <= 256 ? 32 : 16;
  const size_t lds = (size_t)2 * TP * maxw * 4;
  auto launch = [&](auto kern, dim3 grid) {
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, ctx->stream, a, maxw, ctx->err_dev);
  };
  if (dense) {
    // grid.y = the chunk's users (< 65536 per launch): any B
    const DeepArgs all = a;
    for (int64_t b0 = 0; b0 < B; b0 += 65535) {
      const int64_t nb = std::min<int64_t>(65535, B - b0);
      a = all;
      a.P = all.P + b0 * d1;
      a.uids = all.uids + b0;
      a.out = all.out + b0 * ldo;
      a.B = nb;
      const dim3 g((unsigned)hnm_cdiv(w->num_items, TP), (unsigned)nb);
      if (TP == 64) launch(ncf_deep_kernel<64, true>, g);
      else if (TP == 32) launch(ncf_deep_kernel<32, true>, g);
      else launch(ncf_deep_kernel<16, true>, g);
      HNM_LAUNCH_CHECK();
    }
  } else {
    const dim3 g((unsigned)hnm_cdiv(B, TP));
    if (TP == 64) launch(ncf_deep_kernel<64, false>, g);
    else if (TP == 32) launch(ncf_deep_kernel<32, false>, g);
    else launch(ncf_deep_kernel<16, false>, g);
  }
  HNM_LAUNCH_CHECK();
  return HNM_OK;
}
