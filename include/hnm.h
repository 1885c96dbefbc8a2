/* libhnm_mi355x — C ABI of the MI355X-native top-N scoring hot path.
 *
 * Drop-in boundary for hyunlord/hnm_recommendation @ 2025-07-25 (reference paths below are
 * relative to that repo).  The reference has no FFI: its boundary is the PyTorch module
 * surface `NeuralCF` / `LightGCN` / `WideDeep` / `MatrixFactorization` with `forward`,
 * `predict_all_items`, `recommend` and `set_graph`.  Each entry point
 * below replaces the ATen / torch_sparse work one of those methods does; the Python
 * mirror in `hnm_recommendation_amd/models/` binds them with ctypes.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer owned by the caller (the torch caching
 *    allocator); the library never frees caller memory.  Shapes are row-major, fp32
 *    tables with an explicit leading dimension, int64 ids.  An empty batch (B == 0 or
 *    n == 0) is a no-op whose per-row pointers (ids, outputs, bounds) may be NULL -- what
 *    torch hands over for an empty tensor.
 *  - Calls are asynchronous and stream-ordered on the ctx stream (hnm_ctx_set_stream:
 *    torch's current stream).  A ctx is not re-entrant: use one per (device, thread)
 *    (the Python layer does: one per thread, destroyed when the thread exits).  Switching
 *    a ctx to another stream queues the new stream behind the work already issued on the
 *    old one (an event recorded on the old stream, waited on by the new one; no host sync),
 *    so the ctx workspace is never reused while a kernel on the previous stream still reads
 *    it.  A stream handed to hnm_ctx_set_stream must therefore stay alive until the ctx has
 *    been switched away from it (torch's pooled streams always do; a caller-owned
 *    hipStream_t / torch.cuda.ExternalStream must outlive that switch).
 *  - Device binding: a ctx belongs to the device it was created on.  Every entry that takes
 *    a ctx switches the calling thread to ctx->device for its duration (workspace allocation,
 *    events, launches, the null stream when no stream was set) and restores the caller's
 *    current device before returning; hnm_ctx_create leaves the current device unchanged.  So
 *    one host thread may drive ctxs of several GPUs; the pointers passed to a call must live on
 *    that ctx's device, and a stream set with hnm_ctx_set_stream must belong to it.
 *  - Status: 0 on success, negative on error; hnm_last_error() holds a thread-local
 *    message.  No C++ exception crosses the ABI.
 *  - Out-of-range user/item ids never fault: the row is skipped (index -1 / NaN) and the
 *    ctx error word records it; hnm_ctx_check() synchronizes and returns HNM_EOOB, which
 *    the Python layer raises as IndexError (reference: nn.Embedding IndexError).
 *  - Top-K order is (score desc, item index asc); -inf (filtered) items rank last and are
 *    returned only when fewer than k finite scores exist (torch.topk semantics).
 */
#ifndef HNM_H_
#define HNM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HNM_ABI_VERSION 1

typedef int32_t hnm_status;
enum {
  HNM_OK = 0,
  HNM_EINVAL = -1,       /* bad argument / shape */
  HNM_EOOB = -2,         /* an id was out of range (reported by hnm_ctx_check) */
  HNM_EHIP = -3,         /* HIP runtime error */
  HNM_ENOMEM = -4,       /* workspace allocation failed */
  HNM_EUNSUPPORTED = -5, /* shape outside what the kernels are built for */
  HNM_ECOLL = -6         /* RCCL error (hnm_ctx_rccl_init, hnm_topk_allgather_merge_f32) */
};

typedef struct hnm_ctx hnm_ctx;
typedef struct hnm_spmm_plan hnm_spmm_plan;

int hnm_abi_version(void);
const char* hnm_last_error(void);

/* ---- context ------------------------------------------------------------------------ */
hnm_status hnm_ctx_create(int device, hnm_ctx** out);
hnm_status hnm_ctx_destroy(hnm_ctx* ctx);
hnm_status hnm_ctx_set_stream(hnm_ctx* ctx, void* hip_stream);
hnm_status hnm_ctx_reserve(hnm_ctx* ctx, size_t bytes);   /* pre-grow workspace */
hnm_status hnm_ctx_check(hnm_ctx* ctx);                   /* sync; HNM_EOOB if flagged */
hnm_status hnm_ctx_num_cus(hnm_ctx* ctx, int* out);
/* Close an open two-phase top-K call (hnm_*_topk_begin_f32 without its _finish), e.g.
 * after a failed cross-shard exchange; the begin phase's tables are discarded. */
hnm_status hnm_ctx_abort_pending(hnm_ctx* ctx);
/* Options.  HNM_OPT_PREFILTER (default 1): NCF and dot-product top-K scan the catalogue
 * with the certified f16 pre-filter and re-score the surviving candidates in exact fp32
 * (results identical to the fp32 scan); 0 = exact fp32 scan of every item.  Calls outside
 * the pre-filter's range take the exact scan whatever the option: fewer than 8,192 items or
 * than 64 k, k > 64, the dot path with d > 128 or with an f16 item copy of 2 GiB or more
 * (16.7M items at d <= 64, 8.3M at d <= 128), NCF layer widths beyond 64 / 32 or 33.5M items. */
enum { HNM_OPT_PREFILTER = 1,
       HNM_OPT_STATS = 3,      /* 1: count pre-filter candidates / fallback rows (diagnostics) */
       HNM_OPT_STRIDED = 4,    /* NeuralCF certified top-K: 1 = the gated per-user strided
                                  sample may run (weights whose best items are user-specific:
                                  bench "norms" 3.68 -> 3.09 ms a step); 0 (default) = the
                                  champion sample alone (the gate costs ~2 % of the init-weight
                                  step) */
       HNM_OPT_DEEP_MFMA = 5   /* deep NeuralCF towers (hnm_ncf_deep_*): 1 (default) = the
                                  fp32-MFMA tile kernel where the tower fits it (widths <= 64,
                                  mf <= 128); 0 = the per-pair LDS kernel everywhere (same
                                  scores bitwise: the A/B and parity switch) */,
       HNM_OPT_LINEAR_MFMA = 6 /* hnm_linear_rows_f32 (every per-call layer-1 projection): 1
                                  (default) = the fp32-MFMA kernel where K % 32 == 0 (exact fp32
                                  fma chain in k order: bitwise the VALU kernel); 0 = the VALU
                                  kernel everywhere (the A/B and parity switch) */ };
hnm_status hnm_ctx_set_option(hnm_ctx* ctx, int option, int64_t value);
/* Pre-filter counters since the last reset (counted only while HNM_OPT_STATS is 1): out[0]
 * rows scored, out[1] candidates re-scored in fp32, out[2] rows that took the exact fallback
 * scan.  Synchronizes the whole DEVICE (not the ctx stream), so it may be called on a ctx
 * another thread owns; counts of calls that thread issues while this runs may land before or
 * after a reset (totals are exact for threads that are idle meanwhile). */
hnm_status hnm_ctx_prefilter_stats(hnm_ctx* ctx, int64_t* out, int reset);
/* The same counters, the first n of 6: out[3] = rows whose bound also used the per-user strided
 * sample (NeuralCF: gated on when it is predicted to save re-scoring); out[4] / out[5] = the
 * last NeuralCF call's gate inputs: candidates its proxy rows would re-score with the champion
 * bound alone / with the strided sample's bound too (diagnostics). */
hnm_status hnm_ctx_prefilter_stats_ex(hnm_ctx* ctx, int64_t* out, int n, int reset);
/* Dominant-kernel timer: while on, calls record HIP events on the ctx stream around their
 * main kernel; `mask` selects the class: 1 = the scoring / scan kernel of every top-K or
 * dense call, 2 = each LightGCN propagation layer (SpMM), 3 = both.  hnm_ctx_timing()
 * syncs, returns the summed kernel time and the number of timed launches, and resets.
 * Enabling creates 1,024 event pairs up front (more are created only past that many timed
 * launches), so a timed loop records without creating events.  (bench.py's live roofline
 * figures.) */
hnm_status hnm_ctx_enable_timing(hnm_ctx* ctx, int mask);
hnm_status hnm_ctx_timing(hnm_ctx* ctx, double* total_ms, int64_t* launches);

/* ---- a1: embedding row gather ------------------------------------------------------
 * out[b, :d] = table[ids[b], :d].  Replaces nn.Embedding.__call__ at
 * neural_cf.py:155-156, lightgcn.py:199, wide_deep.py:207. */
hnm_status hnm_gather_rows_f32(hnm_ctx* ctx, const float* table, int64_t rows, int64_t ld,
                               int d, const int64_t* ids, int64_t n, float* out,
                               int64_t ldo);

/* ---- per-row projection used to decompose the first MLP layer --------------------
 * Y[r, c(n)] = sum_k X[x(r), k] * W[n, k] (+ bias[n]),  n < N, k < K.
 * x(r) = ids ? ids[r] : r (ids bounded by x_rows);  c(n) = n, or with pair_permute
 * c(n) = (n & 1) * (ldy / 2) + (n >> 1) — the lane-half layout the MFMA kernels read.
 * W has leading dimension ldw (a column slice of a Linear weight, e.g. the user or the
 * item half of mlp_layers.0.weight, neural_cf.py:85-87 / wide_deep.py:128). */
hnm_status hnm_linear_rows_f32(hnm_ctx* ctx, const float* X, int64_t ldx, const int64_t* ids,
                               int64_t x_rows, int64_t M, int K, const float* W,
                               int64_t ldw, const float* bias, int N, float* Y, int64_t ldy,
                               int pair_permute);

/* ---- a7 + a11 + a12: dot-product scoring fused with filter and top-K ---------------
 * s[b, i] = user_tab[user_ids[b]] . item_tab[i] (+ user_bias[user_ids[b]]) (+ item_bias[i])
 *           (+ const_bias[0]); masked (b, i) -> -inf; top-k per row.
 * LightGCN.predict_all_items + recommend (lightgcn.py:188-204, 332-358) and
 * MatrixFactorization (matrix_factorization.py:108-131, 220-246).
 * mask: CSR over the batch rows (mask_ptr[B+1], mask_idx sorted ascending per row) or NULL.
 * d <= 128, d % 4 == 0, 16-B aligned tables.  Fused path: k <= 64 (larger k: dense
 * scores + hnm_topk_rows_f32). */
hnm_status hnm_dot_topk_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                            int64_t ldu, const int64_t* user_ids, int64_t B,
                            const float* item_tab, int64_t num_items, int64_t ldi, int d,
                            const float* user_bias, const float* item_bias,
                            const float* const_bias, const int64_t* mask_ptr,
                            const int32_t* mask_idx, int k, float* out_val,
                            int64_t* out_idx);
/* Two-phase hnm_dot_topk_f32 for item-sharded serving: as hnm_ncf_topk_begin_f32 /
 * _finish_f32 (lower bounds in real score units, biases included). */
hnm_status hnm_dot_topk_begin_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                  int64_t ldu, const int64_t* user_ids, int64_t B,
                                  const float* item_tab, int64_t num_items, int64_t ldi, int d,
                                  const float* user_bias, const float* item_bias,
                                  const float* const_bias, const int64_t* mask_ptr,
                                  const int32_t* mask_idx, int k, float* lower_bound);
/* The begin phase with each row's k best certified sample lower bounds [B, k] (distinct
 * items, real units, descending, -inf padded; as hnm_ncf_topk_begin_lists_f32): the caller
 * all-gathers them over the item shards and passes the k-th best of the union to finish. */
hnm_status hnm_dot_topk_begin_lists_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                        int64_t ldu, const int64_t* user_ids, int64_t B,
                                        const float* item_tab, int64_t num_items, int64_t ldi,
                                        int d, const float* user_bias, const float* item_bias,
                                        const float* const_bias, const int64_t* mask_ptr,
                                        const int32_t* mask_idx, int k, float* lower_lists);
hnm_status hnm_dot_topk_finish_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                   int64_t ldu, const int64_t* user_ids, int64_t B,
                                   const float* item_tab, int64_t num_items, int64_t ldi, int d,
                                   const float* user_bias, const float* item_bias,
                                   const float* const_bias, const int64_t* mask_ptr,
                                   const int32_t* mask_idx, int k, const float* lower_bound,
                                   int short_ok, float* out_val, int64_t* out_idx);
/* Diagnostics of the certified f16 pre-filter of hnm_dot_topk_f32 (no reference
 * counterpart): approx[b, i] = the f16 scan's score (biases included), bound[b] = the
 * row's error bound; |approx - exact| <= bound for every item (tests check it). */
hnm_status hnm_dot_prefilter_debug_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                                       int64_t ldu, const int64_t* user_ids, int64_t B,
                                       const float* item_tab, int64_t num_items, int64_t ldi,
                                       int d, const float* user_bias, const float* item_bias,
                                       const float* const_bias, float* approx, int64_t lda,
                                       float* bound);
/* Dense variant: out[b, i] (ldo >= num_items), the predict_all_items matrix. */
hnm_status hnm_dot_scores_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                              int64_t ldu, const int64_t* user_ids, int64_t B,
                              const float* item_tab, int64_t num_items, int64_t ldi, int d,
                              const float* user_bias, const float* item_bias,
                              const float* const_bias, float* out, int64_t ldo);

/* Pairwise variant: out[n] = user_tab[user_ids[n]] . item_tab[item_ids[n]] + biases
 * (LightGCN.predict lightgcn.py:166-186, MatrixFactorization.forward :80-106). */
hnm_status hnm_pair_dot_f32(hnm_ctx* ctx, const float* user_tab, int64_t num_users,
                            int64_t ldu, const float* item_tab, int64_t num_items, int64_t ldi,
                            int d, const int64_t* user_ids, const int64_t* item_ids, int64_t n,
                            const float* user_bias, const float* item_bias,
                            const float* const_bias, float* out);

/* ---- a3 + a4: NeuralCF --------------------------------------------------------------
 * Reference layout (state_dict of neural_cf.py:56-67):  mlp_dims = [2*h0, h1, h2].
 *   s = wp[:mf].(g_u * g_i) + wp[mf:].relu(W2 relu(W1 [m_u; m_i] + b1) + b2) + bp
 * Requires mf <= 128, h1 <= 128, h2 <= 32 (the default 64 / [128,64,32] config). */
typedef struct {
  const float* gmf_user;   /* [num_users, mf] */
  const float* gmf_item;   /* [num_items, mf] */
  const float* mlp_user;   /* [num_users, h0] */
  const float* mlp_item;   /* [num_items, h0] */
  const float* w1;         /* [h1, 2*h0]  mlp_layers.0.weight */
  const float* b1;         /* [h1] */
  const float* w2;         /* [h2, h1]    mlp_layers.3.weight */
  const float* b2;         /* [h2] */
  const float* wp;         /* [mf + h2]   prediction_layer.weight */
  const float* bp;         /* [1]         prediction_layer.bias */
  int64_t num_users;
  int64_t num_items;
  int32_t mf;
  int32_t h0;
  int32_t h1;
  int32_t h2;
  /* Optional (NULL: computed per call; ZERO-INITIALISE the struct so an unset field is NULL --
   * a non-NULL pointer is used as the table, and one that is not 16-B aligned is refused with
   * HNM_EINVAL): the item half of layer 1 for THESE num_items rows,
   * W1[:, h0:] m_i pair-permuted, [num_items, 64] (h1 <= 64 and mf <= 64) or [num_items, 128],
   * as hnm_ncf_item_proj_f32 writes it -- for callers whose item tables and W1 stay fixed
   * between calls (a server); a row shard points at its first row. */
  const float* item_proj;
} hnm_ncf_weights;

/* out = the item projection hnm_ncf_weights.item_proj takes (zero padded columns). */
hnm_status hnm_ncf_item_proj_f32(hnm_ctx* ctx, const hnm_ncf_weights* w, float* out);

hnm_status hnm_ncf_topk_f32(hnm_ctx* ctx, const hnm_ncf_weights* w, const int64_t* user_ids,
                            int64_t B, const int64_t* mask_ptr, const int32_t* mask_idx,
                            int k, float* out_val, int64_t* out_idx);
/* Two-phase hnm_ncf_topk_f32 for item-sharded serving (no reference counterpart: the
 * reference is single-device).  begin: per-call tables + each row's
 * certified lower bound of its exact k-th best score over this call's items, lower_bound[B]
 * (real score units; -inf when unknown, e.g. with the pre-filter off).  The caller may
 * replace the bounds by any valid lower bounds -- the max over the item shards of a node --
 * then finish completes the fused top-k with them; short_ok = 1 lets a row keep fewer than
 * k entries (padded with -inf / -1: another shard holds its better items).  Nothing else may
 * use the ctx between begin and finish (HNM_EINVAL otherwise). */
hnm_status hnm_ncf_topk_begin_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                  const int64_t* user_ids, int64_t B, const int64_t* mask_ptr,
                                  const int32_t* mask_idx, int k, float* lower_bound);
/* As hnm_ncf_topk_begin_f32, but for each row the k best certified lower bounds of the
 * sample's items, lower_lists[B, k] (real units, descending, -inf padded; all -inf when
 * unknown): bounds of k DISTINCT items' exact scores, so the k-th best of the union of every
 * item shard's lists is a lower bound of the row's global k-th best -- as tight as a
 * single-device call's -- where the max of the shards' single bounds is only each shard's own
 * k-th.  finish then takes that merged bound. */
hnm_status hnm_ncf_topk_begin_lists_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                        const int64_t* user_ids, int64_t B,
                                        const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                                        float* lower_lists);
hnm_status hnm_ncf_topk_finish_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                   const int64_t* user_ids, int64_t B, const int64_t* mask_ptr,
                                   const int32_t* mask_idx, int k, const float* lower_bound,
                                   int short_ok, float* out_val, int64_t* out_idx);
hnm_status hnm_ncf_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                              const int64_t* user_ids, int64_t B, float* out, int64_t ldo);
/* Diagnostics of the certified pre-filter (no reference counterpart): approx[b, i] = the
 * f16 scan's score of item i without the output bias bp, bound[b, i] = the pair's error
 * bound (both [B, lda]); |approx + bp - exact| <= bound holds for every pair (tests check
 * it on the full catalogue). */
hnm_status hnm_ncf_prefilter_debug_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                       const int64_t* user_ids, int64_t B, float* approx,
                                       int64_t lda, float* bound);
/* NeuralCF.forward(user_ids, item_ids) (neural_cf.py:112-141): out[n]. */
hnm_status hnm_ncf_pair_scores_f32(hnm_ctx* ctx, const hnm_ncf_weights* w,
                                   const int64_t* user_ids, const int64_t* item_ids,
                                   int64_t n, float* out);

/* NeuralCF with an MLP tower of any depth (neural_cf.py:75-90: one Linear -> ReLU per
 * consecutive pair of mlp_dims, any length >= 2), exact fp32 -- the path for towers the fused
 * kernels above do not cover (they take the default two-layer tower).  w[l] / b[l] =
 * mlp_layers.{3l}.weight [dims[l+1], dims[l]] / bias; dims[0] = 2 x the MLP embedding width;
 * widths dims[1..nl] <= 512, nl <= 8.
 * item_ids NULL: dense scores out[b * ldo + i] for every item (ldo >= num_items:
 * predict_all_items; recommend = hnm_ncf_deep_topk_f32).  item_ids set: pair scores
 * out[n] = s(user_ids[n], item_ids[n]), n < B (forward).  Out-of-range ids flag HNM_EOOB
 * (hnm_ctx_check) and score NaN. */
typedef struct {
  const float* gmf_user;   /* [num_users, mf] */
  const float* gmf_item;   /* [num_items, mf] */
  const float* mlp_user;   /* [num_users, dims[0] / 2] */
  const float* mlp_item;   /* [num_items, dims[0] / 2] */
  const float* w[8];
  const float* b[8];
  const float* wp;         /* [mf + dims[nl]] prediction_layer.weight */
  const float* bp;         /* [1] */
  int64_t num_users;
  int64_t num_items;
  int32_t mf;
  int32_t nl;              /* Linear layers = len(mlp_dims) - 1 */
  int32_t dims[9];
} hnm_ncf_deep_weights;

hnm_status hnm_ncf_deep_scores_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                   const int64_t* user_ids, int64_t B, const int64_t* item_ids,
                                   float* out, int64_t ldo);
/* Fused top-k of a deep tower (NeuralCF.recommend, neural_cf.py:300-326, with the -inf filter
 * and torch.topk of neural_cf.py:316-324): (score desc, item asc), scores bitwise those of
 * hnm_ncf_deep_scores_f32, 1 <= k <= 64, mask as hnm_ncf_topk_f32.  Three-layer towers
 * [2 h0, h1 <= 64, h2 <= 32, h3 <= 16] with mf <= 64 (a multiple of 4) take the certified f16
 * pre-filter when HNM_OPT_PREFILTER is on and the call is in its range (B >= 16, >= 8,192 items,
 * >= 64 k): the two-layer tower's f16 scan with a third layer on the matrix pipe, its worst-case
 * bound carried through |wp3|^T |W3| |W2|, exact fp32 re-scoring of the survivors by the deep
 * chain (outputs bitwise the exact path's); rows the bound cannot serve take the exact scan
 * (their count is read back: the call synchronizes its stream).  Otherwise towers with every
 * width dims[1..nl] <= 64 and mf <= 128 take the fp32-MFMA scan that keeps per-partition top-k
 * lists (no [B, I] score matrix); wider towers score dense rows per user chunk in the
 * workspace and take the row top-k kernel. */
hnm_status hnm_ncf_deep_topk_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                 const int64_t* user_ids, int64_t B, const int64_t* mask_ptr,
                                 const int32_t* mask_idx, int k, float* out_val,
                                 int64_t* out_idx);
/* Diagnostics of that pre-filter (no reference counterpart): approx[b, i] = the f16 scan's score
 * of item i without bp, bound[b, i] its certified bound ([B, lda], real units); |approx + bp -
 * exact| <= bound for every pair (tests check it on the full catalogue). */
hnm_status hnm_ncf_deep_prefilter_debug_f32(hnm_ctx* ctx, const hnm_ncf_deep_weights* w,
                                            const int64_t* user_ids, int64_t B, float* approx,
                                            int64_t lda, float* bound);

/* ---- a9 + a10: Wide&Deep ------------------------------------------------------------
 * Reference layout (wide_deep.py:92-134): deep tower Linear -> ReLU -> BatchNorm1d (eval:
 * running stats, eps) per layer; final_layer over [wide (one-hot u, one-hot i, wide user
 * features) ; deep].  wide_user/item_embedding are unused by the reference forward.
 *   s = wide_user[u] + wide_item[i] (+ wide_user_features(f_u) . wide_feat)
 *       + final_deep . deep(u, i) + final_b
 * where wide_user / wide_item / wide_feat / final_deep are the segments [0, U), [U, U+I),
 * [U+I, U+I+F) and [wide_dim, ...) of final_layer.weight[0] (item rows may be a shard).
 * Towers of 2 (w3 == NULL, l3 == 0) or 3 layers, widths <= 512 / 256 / 128; deep input
 * [e_u; e_i] (+ deep_user_features(f_u) when num_user_features > 0). */
typedef struct {
  const float* deep_user;  /* [num_users, d] */
  const float* deep_item;  /* [num_items, d] */
  const float* w1;         /* [l1, l1_in]  deep_network.0 */
  const float* b1;
  const float* bn1_w;      /* deep_network.2 weight / bias / running_mean / running_var */
  const float* bn1_b;
  const float* bn1_mean;
  const float* bn1_var;
  const float* w2;         /* [l2, l1]  deep_network.4 */
  const float* b2;
  const float* bn2_w;
  const float* bn2_b;
  const float* bn2_mean;
  const float* bn2_var;
  const float* w3;         /* [l3, l2]  deep_network.8 (NULL for a two-layer tower) */
  const float* b3;
  const float* bn3_w;
  const float* bn3_b;
  const float* bn3_mean;
  const float* bn3_var;
  const float* wide_user;  /* final_layer.weight[0, 0:U] */
  const float* wide_item;  /* final_layer.weight[0, U:U+I] */
  const float* wide_feat;  /* final_layer.weight[0, U+I:U+I+F] or NULL */
  const float* final_deep; /* final_layer.weight[0, wide_dim:] (last hidden width) */
  const float* final_b;    /* [1] */
  const float* duf_w;      /* [d, F] deep_user_features or NULL */
  const float* duf_b;
  const float* wuf_w;      /* [F, F] wide_user_features or NULL */
  const float* wuf_b;
  int64_t num_users;
  int64_t num_items;
  int32_t d;
  int32_t l1_in;
  int32_t l1;
  int32_t l2;
  int32_t l3;
  int32_t num_user_features;
  float eps;
} hnm_widedeep_weights;

hnm_status hnm_widedeep_topk_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                 const int64_t* user_ids, int64_t B, const float* user_features,
                                 const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                                 float* out_val, int64_t* out_idx);
hnm_status hnm_widedeep_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                   const int64_t* user_ids, int64_t B, const float* user_features,
                                   float* out, int64_t ldo);
/* WideDeep.forward(user_ids, item_ids, user_features) (wide_deep.py:157-230): out[n]. */
hnm_status hnm_widedeep_pair_scores_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                        const int64_t* user_ids, const int64_t* item_ids,
                                        const float* user_features, int64_t n, float* out);
/* Item-side feature weights of WideDeep(num_item_features > 0) (wide_deep.py:101-103,
 * 116-117): deep_item_features [d, Fi] + bias, wide_item_features [Fi, Fi] + bias (NULL
 * when use_wide_features=False) and its slice of final_layer.weight. */
typedef struct {
  const float* dif_w;
  const float* dif_b;
  const float* wif_w;
  const float* wif_b;
  const float* wide_feat;
  int32_t num_item_features;
} hnm_widedeep_item_features;
/* WideDeep.forward(user_ids, item_ids, user_features, item_features): pairwise scores with
 * per-pair item features [n, Fi] (wide_deep.py:190-195, 214-217).  itf may be NULL (no
 * item features).  A NULL w->wide_user / w->wide_item means use_wide_user_item=False. */
hnm_status hnm_widedeep_pair_scores_ex_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                           const hnm_widedeep_item_features* itf,
                                           const int64_t* user_ids, const int64_t* item_ids,
                                           const float* user_features, const float* item_features,
                                           int64_t n, float* out);

/* ---- top-K merge (item partitions, item shards across GPUs) ------------------------
 * Candidates of row b: for g < G: cand[g*gstride + b*bstride + j], j < kc (value, global
 * item index; index < 0 = empty).  out: the best k of them per row, sorted. */
hnm_status hnm_topk_merge_f32(hnm_ctx* ctx, const float* cand_val, const int64_t* cand_idx,
                              int64_t B, int64_t G, int64_t gstride, int64_t bstride,
                              int kc, int k, float* out_val, int64_t* out_idx);

/* ---- (e) item-sharded exchange from the C ABI, over RCCL (SURVEY §8(b) hnm_topk_allgather_merge)
 * Every rank scores the SAME B users against its own item shard (global item ids) into [B, k]
 * lists; hnm_topk_allgather_merge_f32 all-gathers the lists of the communicator's ranks on the
 * ctx stream and merges them into the global top-k (score desc, item asc), identical on every
 * rank.  Every rank must call it (B and k equal on all).  The communicator: hnm_rccl_unique_id
 * on one rank (size >= 128 bytes), the bytes shared by the host, hnm_ctx_rccl_init on every
 * rank (owned by the ctx); or hnm_ctx_set_rccl_comm with the host's own ncclComm_t (borrowed;
 * NULL detaches).  The Python mirror's exchange (sharding.py, torch.distributed) adds a
 * certified bound exchange before the shard scans; this is the single-phase form. */
hnm_status hnm_rccl_unique_id(void* out, int64_t size);
hnm_status hnm_ctx_rccl_init(hnm_ctx* ctx, int world, int rank, const void* unique_id,
                             int64_t size);
hnm_status hnm_ctx_set_rccl_comm(hnm_ctx* ctx, void* comm);
/* Abort the ctx's own communicator (ncclCommAbort; a borrowed one is only detached).  When
 * hnm_topk_allgather_merge_f32 returns an error on one rank (argument check, open two-phase
 * call, workspace ENOMEM -- all checked before the collective), that rank never entered the
 * collective its peers are waiting in: the host aborts the communicator on every rank and
 * creates a new one (hnm_ctx_rccl_init). */
hnm_status hnm_ctx_rccl_abort(hnm_ctx* ctx);
hnm_status hnm_topk_allgather_merge_f32(hnm_ctx* ctx, const float* local_val,
                                        const int64_t* local_idx, int64_t B, int k,
                                        float* out_val, int64_t* out_idx);

/* The item-shard exchange's candidate lists as int32 pairs (one all_to_all): pairs[2e] = the
 * bits of val[e], pairs[2e+1] = idx[e] + offset (idx < 0 stays; global ids < 2^31); pairs
 * 8-byte aligned. */
hnm_status hnm_pack_candidates_i32(hnm_ctx* ctx, const float* val, const int64_t* idx, int64_t n,
                                   int64_t offset, int32_t* pairs);
/* Merge of received pairs [G][B][kc][2] (G <= 16), each list sorted in the top-K order (score
 * desc, id asc; id < 0 = empty, at the tail) -> out [B, k] sorted, empty slots (-inf, -1):
 * the same result as hnm_topk_merge_f32 over the unpacked candidates. */
hnm_status hnm_topk_merge_sorted_pairs_i32(hnm_ctx* ctx, const int32_t* pairs, int64_t B,
                                           int64_t G, int kc, int k, float* out_val,
                                           int64_t* out_idx);
/* The item-shard bound exchange's merge: lists[g*B*kc + b*kc + j] (g < G <= 16, j < kc), each
 * row of each list in descending order (hnm_{ncf,dot}_topk_begin_lists_f32's output,
 * all-gathered); out[b] = the k-th best value of row b's union of the G lists (k <= G*kc).
 * New (the reference has no multi-GPU path): sharding.py's exchange calls it. */
hnm_status hnm_topk_lists_kth_f32(hnm_ctx* ctx, const float* lists, int64_t B, int64_t G,
                                  int kc, int k, float* out);

/* Diagnostics of the certified split-f16 pre-filter of hnm_widedeep_topk_f32 (no reference
 * counterpart): approx[b, i] = the scan's score, bound[b, i] = its certified error bound;
 * |approx - exact| <= bound for every pair (tests check it on the full catalogue). */
hnm_status hnm_widedeep_prefilter_debug_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                            const int64_t* user_ids, int64_t B,
                                            const float* user_features, float* approx,
                                            int64_t lda, float* bound);
/* The re-scoring cascade's refining stage (round 5) over the WHOLE catalogue: approx[b*lda + i]
 * = the three-pass split-f16 score of (user b, item i), bound[b*lda + i] its certified bound
 * (|approx - exact| <= bound, exact = hnm_widedeep_pair_scores_f32's arithmetic); the top-K path
 * runs it only on the scan's survivors.  Diagnostics / tests; B * num_items < 2^31. */
hnm_status hnm_widedeep_refine_debug_f32(hnm_ctx* ctx, const hnm_widedeep_weights* w,
                                         const int64_t* user_ids, int64_t B,
                                         const float* user_features, float* approx, int64_t lda,
                                         float* bound);

/* ---- a11: batch mask from a device-resident history CSR --------------------------------
 * The purchase-history filter (serve.py:350-352; the filter_items loop of every recommend,
 * neural_cf.py:316-321) without a host round trip: hist_ptr[num_users + 1] / hist_idx (per
 * user, sorted ascending, unique, in [0, num_items)) stay on the device; for a batch of
 * user_ids[B] this writes the CSR mask the top-K entry points take: mask_ptr[B + 1] and
 * mask_idx[mask_ptr[B]] with row b = the history ids i of user_ids[b] with
 * item_lo <= i < item_hi, as i - item_lo (an item shard's local ids; pass 0 / INT64_MAX for
 * the whole catalogue).  Users outside [0, num_users) get empty rows (the scoring call flags
 * them).  capacity = the mask_idx length (B x the longest history always suffices); beyond
 * it rows are truncated and hnm_ctx_check() returns HNM_EINVAL.  Asynchronous, two launches. */
hnm_status hnm_mask_gather_csr(hnm_ctx* ctx, const int64_t* hist_ptr, const int32_t* hist_idx,
                               int64_t num_users, const int64_t* user_ids, int64_t B,
                               int64_t item_lo, int64_t item_hi, int64_t capacity,
                               int64_t* mask_ptr, int32_t* mask_idx);

/* ---- torch.topk over a dense score matrix (serve.py:350-355, k up to 100) ----------
 * Row top-k of scores[b, :I] (leading dim ld) with the optional CSR -inf mask, 1 <= k <= I
 * (torch.topk's range).  k <= 128: row-select kernels; larger k: a stable segmented radix
 * sort of whole rows in chunks (same (score desc, item asc) order; workspace ~512 MB). */
hnm_status hnm_topk_rows_f32(hnm_ctx* ctx, const float* scores, int64_t ld, int64_t B,
                             int64_t I, const int64_t* mask_ptr, const int32_t* mask_idx,
                             int k, float* out_val, int64_t* out_idx);

/* ---- a5: LightGCN.set_graph ----------------------------------------------------------
 * A_hat = D^-1/2 (A + I) D^-1/2 (lightgcn.py:81-134) as CSR with E + N entries:
 * self-loops appended, deg = row sums of the weights (edge_weight NULL -> 1), deg^-1/2
 * with inf -> 0, val = dinv[row] * w * dinv[col]; duplicates kept (summed by the SpMM). */
hnm_status hnm_csr_build_norm(hnm_ctx* ctx, const int64_t* edge_index, const float* edge_weight,
                              int64_t E, int64_t N, int64_t* rowptr, int32_t* col, float* val);

/* ---- a6: LightGCN.forward propagation -----------------------------------------------
 * Y = A_hat X (graph @ all_embeddings, lightgcn.py:152), with the layer combine fused:
 * acc_out = acc_in + alpha * Y (lightgcn.py:156-158).  Y and acc_out may be NULL.
 * d in {4, 8, 16, 32, 64, 128, 256}.  With a plan on a graph of N <= 2^22 nodes (the "walk
 * plan"; rowptr[0] == 0): every row's entries are summed in (col, CSR position) order -- rows
 * of at most 128 entries (the user rows) as one fp32 fma chain each by the column-ordered short
 * walk; longer rows (the item rows: ~300 neighbours each, power-law up to ~1e6) by the
 * user-ordered walk: cut into pieces of at most `cap` entries (piece j = sorted entries
 * j, j + n, ...), each piece one fp32 fma chain, several pieces summed in 256/(d/4)
 * interleaved slices and a fixed pairwise tree -- deterministic.  Larger graphs: short rows one
 * 16-lane group each, long rows one wave, rows over 2,048 entries in 2,048-entry segments + a
 * fixed tree, all in CSR order.  Without a plan: one wave per row, CSR order (deterministic,
 * slower on power-law rows).
 * BINDING: a plan is bound to the col / val pointers of its first prepare / SpMM /
 * rows_combine call and snapshots their values then (a walk plan keeps a sorted copy and
 * per-d schedules); a later call with other col / val pointers fails with HNM_EINVAL, and
 * values changed in place behind the same pointers are NOT seen -- create a new plan.
 * PREPARATION: binding and the first use of each d do one-time host work that synchronizes the
 * ctx stream (a D2H copy of col / val, host sorts, synchronous uploads of ~8 B per entry per
 * schedule; seconds on the 65M-entry H&M graph) and cannot be captured in a hipGraph: call
 * hnm_spmm_plan_prepare(ctx, plan, col, val, d) up front (d = 0: bind only).  After it every
 * SpMM / rows_combine call is asynchronous; an SpMM over split rows needs n_part * d * 4 bytes
 * of ctx workspace (a few MB; hnm_ctx_reserve covers it).
 * ROW RANGES: a range call launches only the short-walk blocks holding rows of the range, but
 * the whole long-row walk whenever one of its rows is in the range (outputs restricted to the
 * range): chunking [0, N) into many ranges repeats the item half's gathers per chunk. */
hnm_status hnm_spmm_plan_create(hnm_ctx* ctx, int64_t N, const int64_t* rowptr,
                                hnm_spmm_plan** out);
hnm_status hnm_spmm_plan_prepare(hnm_ctx* ctx, hnm_spmm_plan* plan, const int32_t* col,
                                 const float* val, int d);
hnm_status hnm_spmm_plan_destroy(hnm_spmm_plan* plan);
/* A row-restricted copy of a BOUND plan (no reference counterpart: the item-sharded LightGCN
 * propagation of SURVEY §8(e)).  The new plan computes only the rows inside the n_ranges host
 * ranges [ranges[2j], ranges[2j+1]) (ascending, disjoint, within [0, N)); SpMM calls on it never
 * write other rows of Y or acc.  Every kept row is summed exactly as the base plan sums it (same
 * pieces and order: bitwise equal rows), and a walk plan's schedules hold only the kept rows'
 * entries, so a layer costs what its kept rows cost (one rank: all user rows + its item shard).
 * The copy is bound to the base's col / val, owns its own sorted copy and schedules (destroy it
 * separately; its per-d schedules are built on first use / prepare as for any plan);
 * rows_combine on it equals rows_combine on the base.  The base itself must not be restricted. */
hnm_status hnm_spmm_plan_restrict(hnm_ctx* ctx, const hnm_spmm_plan* base, const int64_t* ranges,
                                  int n_ranges, hnm_spmm_plan** out);
hnm_status hnm_spmm_csr_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                            const int64_t* rowptr, const int32_t* col, const float* val,
                            const float* X, int d, float* Y, float alpha,
                            const float* acc_in, float* acc_out);
/* Row-range form: rows [row_begin, row_end) only.  Accumulators exist for rows >= acc_row0
 * and are stored from there on (acc[(r - acc_row0) * d]); acc_in NULL means beta * X[r]
 * (the alpha_0 * E_0 term folded into layer 1: acc_out = fma(alpha, Y, beta * X)).
 * hnm_spmm_csr_f32 == range [0, N), acc_row0 0, beta 0. */
hnm_status hnm_spmm_csr_range_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                                  const int64_t* rowptr, const int32_t* col, const float* val,
                                  const float* X, int d, float* Y, float alpha,
                                  const float* acc_in, float* acc_out, float beta,
                                  int64_t row_begin, int64_t row_end, int64_t acc_row0);
/* Final embeddings of `n` listed rows (ids < N) after L layers, given the layer inputs
 * E_0 .. E_{L-1} (host array `layers` of L device pointers, each [N, d]) and alphas[0..L]
 * (host): out[b] = sum_l alphas[l] E_l[rows[b]] with E_L[r] = (A_hat E_{L-1})[r] computed
 * for the listed rows only -- the last layer of LightGCN.forward restricted to the users a
 * recommend() call reads (lightgcn.py:197-199).  Same operations and order as the fused
 * combine of hnm_spmm_csr_f32 with the same plan (bitwise equal: every row is summed in the
 * order that plan's SpMM uses for it; plan NULL: the plan-less SpMM's order).  An id out of
 * range flags HNM_EOOB and writes NaN.  1 <= L <= 8. */
hnm_status hnm_spmm_rows_combine_f32(hnm_ctx* ctx, const hnm_spmm_plan* plan, int64_t N,
                                     const int64_t* rowptr,
                                     const int32_t* col, const float* val, const int64_t* rows,
                                     int64_t n, int d, const float* const* layers,
                                     const float* alphas, int L, float* out);
/* out = alpha * x + beta * y (y may be NULL): the alpha_0 * E_0 term of the combine. */
hnm_status hnm_axpby_f32(hnm_ctx* ctx, int64_t n, float alpha, const float* x, float beta,
                         const float* y, float* out);

/* ---- (f)4: ranking metrics over top-K lists (src/evaluation/metrics.py) ---------------
 * Per user r: predicted ids pred[r*ldp + j], j < min(pred_len ? pred_len[r] : ldp, k);
 * truth ids either CSR (truth_ptr[B+1] non-NULL: truth_idx[truth_ptr[r] .. truth_ptr[r+1]))
 * or dense rows truth_idx[r*ldt + j], j < ldt, kept where truth_mask == NULL ||
 * truth_mask[r*ldt + j] != 0 (the torchmetrics classes' `target[i][mask[i]]`).
 * n_true = the kept-entry count (pass unique ids for evaluate_recommendations' set
 * semantics, metrics.py:212).  inv_log2[i] = 1.0 / np.log2(i + 2), i < k (device, float64).
 * per_user[r*4 + 0..3] = AP@k, Recall@k, Precision@k, NDCG@k: the reference's float64
 * formulas in its summation order (evaluate_recommendations :218-247, MeanAveragePrecision
 * :49-62, RecallAtK :95-100, PrecisionAtK :133-137, NDCGAtK :176-186), zero denominators
 * -> 0.0.  sums[0..3] = sum over all rows of each metric, sums[4..7] = the same over rows
 * with n_true > 0, sums[8] = that row count (deterministic fixed-order reduction).
 * per_user, n_true and sums may each be NULL (not all three).  k <= 128. */
hnm_status hnm_rank_metrics_f64(hnm_ctx* ctx, const int64_t* pred, int64_t B, int64_t ldp,
                                const int64_t* pred_len, int k, const int64_t* truth_ptr,
                                const int64_t* truth_idx, int64_t ldt, const uint8_t* truth_mask,
                                const double* inv_log2, double* per_user, int64_t* n_true,
                                double* sums);

#ifdef __cplusplus
}
#endif
#endif /* HNM_H_ */
