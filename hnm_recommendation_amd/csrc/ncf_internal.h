// Shared between ncf.hip (exact fp32 kernels) and ncf_cert.hip (certified f16 pre-filter).
#pragma once
#include "hnm_internal.h"

// Per-call device tables built by ncf_common (layer-1 projections and the GMF operands).
struct NcfTabs {
  const float* Pu;   // [B, 64]  pair-permuted  W1u m_u + b1
  const float* WGu;  // [B, 64]  pair-permuted  wp_gmf * g_u
  const float* Qi;   // [I, 64]  pair-permuted  W1i m_i
  const float* G;    // [I, ldg] natural order, ldg % 4 == 0, 16-byte aligned, zero-padded
  int64_t ldg;
};

// Exact fp32 top-K over all items (ncf32_kernel LIST mode + partition merge) for the
// request rows rows[0 .. *nrows) (device pointers; rows == nullptr: rows 0 .. B).
// cv/ci: candidate scratch of ncf_list_bytes(B, I, K, num_cus) bytes each.
hnm_status ncf_list_rows(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                         const int64_t* mptr, const int32_t* midx, int K, const int32_t* rows,
                         const int32_t* nrows, float* cv, int32_t* ci, float* ov, int64_t* oi);
size_t ncf_list_bytes(int64_t B, int64_t I, int K, int num_cus);

// Deep NeuralCF towers [2 h0, h1 <= 64, h2 <= 32, h3 <= 16] on the certified path (round 6): the
// two-layer tower's tables (hnm_ncf_weights view: w1/b1, w2/b2 = layers 1 and 2) plus layer 3
// and the prediction weights of its units.  W3 == nullptr: the two-layer tower.
struct CertDeep {
  const float* W3;   // [h3, h2]  mlp_layers.6.weight
  const float* b3;   // [h3]
  const float* wp3;  // [h3]      prediction_layer.weight[mf:]
  int h3;
  // re-scoring (the exact deep chain, ncf_deep_kernel's order): raw GMF rows and weights
  const float* gmf_user;  // [num_users, mf]
  const float* gmf_item;  // [num_items, mf]
  const float* wp;        // [mf + h3]
  const int64_t* ids;     // [B] the call's user ids
};

// Deep towers on the certified path (ncf.hip): eligible for nl == 3 with widths <= 64 / 32 / 16,
// mf <= 64 (a multiple of 4, 16-B aligned GMF item rows) and the two-layer path's catalogue
// conditions; ncf_deep_cert = tables + ncf_deep_cert_topk (fallback rows listed on the device).
bool ncf_deep_cert_eligible(const hnm_ncf_deep_weights* dw, int K);
hnm_status ncf_deep_cert(hnm_ctx* ctx, const hnm_ncf_deep_weights* dw, const int64_t* ids,
                         int64_t B, const int64_t* mptr, const int32_t* midx, int K, float* ov,
                         int64_t* oi, int32_t** ovf_rows, int32_t** ovf_cnt, bool* pruned);
hnm_status ncf_deep_cert_debug(hnm_ctx* ctx, const hnm_ncf_deep_weights* dw, const int64_t* ids,
                               int64_t B, float* approx, int64_t lda, float* bound);

// Certified pre-filter path (ncf_cert.hip): eligible when h1 <= 64, mf <= 64, K <= 64 and
// the catalogue is large enough for the sample pass to pay.
bool ncf_cert_eligible(const hnm_ncf_weights* w, int K);
// strided: the call may run the gated strided sample (HNM_OPT_STRIDED), whose per-row scratch
// ([B, I / 8] values) is carved only then; begin and finish of one call must agree on it
size_t ncf_cert_bytes(int64_t B, int64_t I, int K, int num_cus, int wg, bool strided);
int ncf_cert_wg(const hnm_ctx* ctx);  // scan workgroups per CU of the selected variant
hnm_status ncf_cert_topk(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                         const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                         bool strided, float* ov, int64_t* oi);
// The two phases of ncf_cert_topk: begin writes each row's certified lower bound of the
// exact K-th best score (real units) to lb (nullptr: kept in the scratch); finish takes any
// lower bounds (e.g. the max over item shards) and completes the top-K.
// lists (nullable): each row's K best certified sample lower bounds [B, K], real units.
hnm_status ncf_cert_begin(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                          const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                          bool strided, float* lb, float* lists = nullptr,
                          const CertDeep* dp = nullptr);
hnm_status ncf_cert_finish(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                           const int64_t* mptr, const int32_t* midx, int K, void* scratch,
                           bool strided, const float* lb, int short_ok, float* ov, int64_t* oi,
                           const CertDeep* dp = nullptr, int32_t** ovf_rows = nullptr,
                           int32_t** ovf_cnt = nullptr);
// Deep towers (CertDeep): the one-shot certified top-K with the deep scan and the exact deep
// re-scoring; rows that need the exact scan of the whole catalogue (unusable bound, overflowing
// segments, fewer than K candidates) are listed on the device at *ovf_rows[0 .. *ovf_cnt) for the
// caller (the deep exact kernels live in ncf_deep.hip).  The strided sample is not used.
// *pruned = false: the proxy rows predict that the bound cannot prune (more than 1/16 of the
// catalogue a row): nothing is written, the caller runs the exact kernels.
hnm_status ncf_deep_cert_topk(hnm_ctx* ctx, const hnm_ncf_weights* w, const CertDeep& dp,
                              const NcfTabs& t, int64_t B, const int64_t* mptr,
                              const int32_t* midx, int K, void* scratch, float* ov, int64_t* oi,
                              int32_t** ovf_rows, int32_t** ovf_cnt, bool* pruned);
// Diagnostics: the pre-filter's approximate scores (real units, bp excluded) for every
// item and its per-user error bound E_u: |approx + bp - exact| <= E_u is what the path
// relies on (tests check it on the full catalogue).
hnm_status ncf_cert_debug(hnm_ctx* ctx, const hnm_ncf_weights* w, const NcfTabs& t, int64_t B,
                          void* scratch, float* approx, int64_t lda, float* bound,
                          const CertDeep* dp = nullptr);
