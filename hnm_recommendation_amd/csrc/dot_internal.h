// Shared between score.hip (exact fp32 dot kernels) and dot_cert.hip (certified f16
// pre-filter for the dot-product models: LightGCN, MatrixFactorization).
#pragma once
#include "hnm_internal.h"

enum { DOT_LIST = 0, DOT_DENSE = 1, DOT_THRESH = 2 };

struct DotArgs {
  const float* ut;         // user table [U, ldu]
  int64_t num_users, ldu;
  const int64_t* uids;     // [B] user ids of the request rows
  int64_t B;
  const float* it;         // item table; item i is row i * istride
  int64_t I, ldi, istride;
  int d;
  const float *ubias, *ibias, *cbias;
  int64_t ipp;             // items per partition (blockIdx.y)
  const int64_t* mptr;     // CSR mask over request rows (real item ids)
  const int32_t* midx;
  int K;
  float* cand_v;           // LIST: [launch rows, NP, K]
  int32_t* cand_i;
  int NP;
  float* dense;            // DENSE: [B, ldo]
  int64_t ldo;
  const float* tau;        // THRESH: tau of request row r at tau[r * tau_ld]
  int64_t tau_ld;
  int* cnt;                // THRESH: [B] append counters
  float* buf_v;            // THRESH: [B, cap]
  int32_t* buf_i;
  int cap;
  const int32_t* rows;     // optional: launch row b serves request row rows[b] ...
  const int32_t* nrows;    // ... for b < *nrows (device count)
  int dyn_cus;             // LIST with rows: > 0 = partitions follow *nrows (list_rows_np)
  unsigned* err;
};


DotArgs dot_args(hnm_ctx* ctx, const float* ut, int64_t U, int64_t ldu, const int64_t* ids,
                 int64_t B, const float* it, int64_t I, int64_t ldi, int d, const float* ub,
                 const float* ib, const float* cb, const int64_t* mptr, const int32_t* midx,
                 int K);
// LIST pass over `a` -> merged top-K into ov/oi rows (remapped through a.rows when set).
hnm_status dot_list_pass(hnm_ctx* ctx, DotArgs a, bool bias, float* cv, int32_t* ci, float* ov,
                         int64_t* oi);
size_t list_cand_bytes(int64_t B, int64_t I, int K, int num_cus);

// Certified f16 pre-filter + exact fp32 re-scoring (dot_cert.hip).
bool dot_cert_eligible(int d, int64_t I, int K);
size_t dot_cert_bytes(int64_t B, int64_t I, int d, int K, int num_cus);
hnm_status dot_cert_topk(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch, float* ov,
                         int64_t* oi);
// The two phases of dot_cert_topk (see ncf_cert_begin / ncf_cert_finish).
hnm_status dot_cert_begin(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch, float* lb,
                          float* lists = nullptr);
hnm_status dot_cert_finish(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                           const float* lb, int short_ok, float* ov, int64_t* oi);
// Diagnostics: approx[b, i] = the f16 scan's score (biases included), bound[b] = the row's
// error bound; |approx - exact| <= bound for every item.
hnm_status dot_cert_debug(hnm_ctx* ctx, const DotArgs& a, bool bias, void* scratch,
                          float* approx, int64_t lda, float* bound);
