// Host-side internals of libhnm_mi355x: the context object, error plumbing, workspace.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>

#include "../../include/hnm.h"

struct hnm_ctx {
  int device;
  hipStream_t stream;   // borrowed from the caller (torch's current stream); 0 = null stream
  hipEvent_t chain_ev;  // stream switch: recorded on the old stream, waited on by the new one,
                        // so all work of this ctx (and its workspace reuse) stays ordered
  hipStream_t side;     // owned side stream: independent work overlapped with the ctx stream
  hipEvent_t side_in, side_out;  // fork (ctx stream -> side) / join (side -> ctx stream)
  void* ws;             // grow-only device workspace owned by the ctx
  size_t ws_size;
  unsigned* err_dev;    // device error word (HNM_ERR_* bits), read by hnm_ctx_check
  int num_cus;
  // dominant-kernel timer (hnm_ctx_enable_timing): HIP events recorded on the ctx stream
  // immediately before/after the main kernel of each call
  int timing;
  int nev;
  int cap;
  hipEvent_t* ev0;
  hipEvent_t* ev1;
  int prefilter;                   // HNM_OPT_PREFILTER (default 1)
  unsigned long long* stats_dev;   // pre-filter counters: rows, candidates, fallback rows
  int stats_on;                    // HNM_OPT_STATS (default 0: counting costs same-address atomics)
  // open two-phase top-K call (hnm_*_topk_begin_f32 ... hnm_*_topk_finish_f32): the
  // workspace holds the begin phase's tables until the matching finish, so every other
  // workspace user is refused meanwhile
  struct {
    int kind;               // 0 none; HNM_PEND_* below
    int64_t B, I;
    int K;
    const void* ids;
    const void* items;      // the item table the begin phase read
  } pend;
};
#define HNM_PEND_NCF_CERT 1
#define HNM_PEND_NCF_EXACT 2
#define HNM_PEND_DOT_CERT 3
#define HNM_PEND_DOT_EXACT 4

// dominant-kernel timer classes (hnm_ctx_enable_timing mask)
#define HNM_TIME_SCORE 1  // the scoring / scan kernel of each top-K or dense call
#define HNM_TIME_SPMM 2   // one LightGCN propagation layer (light + segment + finish kernels)
void hnm_timer_begin(hnm_ctx* ctx, int cls);
void hnm_timer_end(hnm_ctx* ctx, int cls);

void hnm_set_error(const char* fmt, ...);

#define HNM_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      hnm_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                    __LINE__);                                                     \
      return HNM_EHIP;                                                             \
    }                                                                              \
  } while (0)

#define HNM_REQUIRE(cond, code, ...)  \
  do {                                \
    if (!(cond)) {                    \
      hnm_set_error(__VA_ARGS__);     \
      return (code);                  \
    }                                 \
  } while (0)

#define HNM_LAUNCH_CHECK()                                                          \
  do {                                                                              \
    hipError_t _e = hipGetLastError();                                              \
    if (_e != hipSuccess) {                                                         \
      hnm_set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e),      \
                    __FILE__, __LINE__);                                            \
      return HNM_EHIP;                                                              \
    }                                                                               \
  } while (0)

// Returns a device pointer to at least `bytes` of workspace (aligned to 256 B), growing
// the ctx workspace if needed.  Growth synchronizes the stream (the old buffer may still
// be read by queued kernels); call hnm_ctx_reserve() before graph capture.
hnm_status hnm_workspace(hnm_ctx* ctx, size_t bytes, void** out);
// row top-k for k > 128 by a stable segmented radix sort of whole rows (topk_sort.hip)
hnm_status hnm_topk_rows_sort(hnm_ctx* ctx, const float* scores, int64_t ld, int64_t B,
                              int64_t I, const int64_t* mask_ptr, const int32_t* mask_idx, int k,
                              float* out_val, int64_t* out_idx);

static inline size_t hnm_align(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }
__host__ __device__ static inline int64_t hnm_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Item partitions for the fused scoring kernels: ~`wg_per_cu` workgroups per CU (the
// kernel's occupancy, so the whole grid is resident in one wave of workgroups), >= 4
// tiles of `tile` items per partition.
struct Partition {
  int np;
  int64_t ipp;
};
static inline Partition choose_partition(int64_t I, int64_t ublocks, int num_cus,
                                         int64_t tile = 32, int wg_per_cu = 2) {
  const int64_t want = std::max<int64_t>(
      1, (int64_t)wg_per_cu * num_cus / std::max<int64_t>(ublocks, 1));
  const int64_t maxp = std::max<int64_t>(1, hnm_cdiv(I, 4 * tile));
  int64_t np = std::min(want, maxp);
  int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), tile) * tile;
  np = hnm_cdiv(I, ipp);
  return {(int)np, ipp};
}

// torch.topk over a dense [B, I] score matrix whose column c is item c * istride, with the
// optional CSR mask in real item ids (score.hip).  K <= 64.
hnm_status hnm_topk_rows_strided(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t I,
                                 const int64_t* mptr, const int32_t* midx, int K, float* ov,
                                 int64_t* oi, int64_t istride);
// Lower bound of the K-th best value of each sample row (score.hip sample_kth_kernel),
// written at out[b * K + K - 1].
hnm_status hnm_sample_kth(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t Ns,
                          const int64_t* mptr, const int32_t* midx, int K, int64_t grp,
                          int64_t period, const int32_t* sidx, float* out);

// p[0, n) = v on the ctx stream
hnm_status hnm_fill_f32(hnm_ctx* ctx, float* p, int64_t n, float v);
