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
  int strided;                     // HNM_OPT_STRIDED (default 0)
  int deep_mfma;                   // HNM_OPT_DEEP_MFMA (default 1)
  int linear_mfma;                 // HNM_OPT_LINEAR_MFMA (default 1)
  void* comm;                      // RCCL communicator (ncclComm_t) of the C-side exchange
  int comm_owned;                  // 1: created by hnm_ctx_rccl_init, destroyed with the ctx
  unsigned long long* stats_dev;   // pre-filter counters: rows, candidates, fallback rows,
                                   // rows whose bound used the gated strided sample, and
                                   // (last NCF call) the gate's predicted proxy candidates
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
    int flags;              // HNM_PEND_STRIDED: the begin carved the strided sample's scratch
  } pend;
};
// Device binding: every entry point that takes a ctx runs on ctx->device --
// its workspace hipMalloc, events, null stream and launches -- and leaves the calling thread's
// current device as it found it, so one host thread may drive ctxs of several GPUs.
struct HnmDeviceGuard {
  int prev = -1;
  explicit HnmDeviceGuard(int device) {
    int cur = -1;
    if (device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != device &&
        hipSetDevice(device) == hipSuccess)
      prev = cur;
  }
  ~HnmDeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  HnmDeviceGuard(const HnmDeviceGuard&) = delete;
  HnmDeviceGuard& operator=(const HnmDeviceGuard&) = delete;
};
#define HNM_CTX_DEVICE(c) const HnmDeviceGuard hnm_device_guard_((c) ? (c)->device : -1)
#define HNM_STATS_N 6  // pre-filter counters (hnm_ctx_prefilter_stats_ex)
#define HNM_PEND_NCF_CERT 1
#define HNM_PEND_NCF_EXACT 2
#define HNM_PEND_DOT_CERT 3
#define HNM_PEND_DOT_EXACT 4
#define HNM_PEND_STRIDED 1  // pend.flags

// dominant-kernel timer classes (hnm_ctx_enable_timing mask)
#define HNM_TIME_SCORE 1  // the scoring / scan kernel of each top-K or dense call
#define HNM_TIME_SPMM 2   // one LightGCN propagation layer (light + segment + finish kernels)
void hnm_timer_begin(hnm_ctx* ctx, int cls);
void hnm_timer_end(hnm_ctx* ctx, int cls);

void hnm_set_error(const char* fmt, ...);
void hnm_rccl_release(hnm_ctx* ctx);  // collective.hip

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
__host__ __device__ static inline Partition choose_partition(int64_t I, int64_t ublocks,
                                                             int num_cus, int64_t tile = 32,
                                                             int wg_per_cu = 2) {
  int64_t want = (int64_t)wg_per_cu * num_cus / (ublocks > 1 ? ublocks : 1);
  if (want < 1) want = 1;
  int64_t maxp = hnm_cdiv(I, 4 * tile);
  if (maxp < 1) maxp = 1;
  int64_t np = want < maxp ? want : maxp;
  int64_t ipp = hnm_cdiv(hnm_cdiv(I, np), tile) * tile;
  np = hnm_cdiv(I, ipp);
  return {(int)np, ipp};
}

// Row-list launches -- the certified paths' exact fallback, whose queued rows are known only
// on the device (rows[0, *nrows)): a FLAT grid of list_rows_grid(B, I, num_cus) workgroups;
// each derives the partition actually used from *nrows, np = choose_partition(I, nb =
// cdiv(nrows, 128), num_cus).np, and takes (user block w / np, item partition w % np) for
// w < nb * np (the rest exit), so that a handful of queued rows still spreads over the whole
// chip.  (A (blocks, partitions) grid sized for the worst case launched ~15k mostly empty
// workgroups of 78 KB LDS: 12.5 ms of dispatch for 19 queued rows, round 5.)  Candidates of list
// row b sit at [b][p][K] with row stride np * K; the merge derives np the same way
// (topk_merge_kernel's dyn_cus).
static inline int64_t list_rows_grid(int64_t B, int64_t I, int num_cus) {
  int64_t best = 1;
  for (int64_t nb = 1; nb <= hnm_cdiv(B, 128); ++nb) {
    const int np = choose_partition(I, nb, num_cus).np;
    best = std::max<int64_t>(best, nb * np);
    if (np == 1) {
      best = std::max<int64_t>(best, hnm_cdiv(B, 128));
      break;
    }
  }
  return best;
}
// candidate slots (rows x partitions) a row-list launch over <= B queued rows can write
static inline int64_t list_rows_slots(int64_t B, int64_t I, int num_cus) {
  int64_t best = 0;
  // rows * np(rows) peaks at the largest row count of each user-block count
  for (int64_t nb = 1; nb <= hnm_cdiv(B, 128); ++nb) {
    const int64_t n = std::min<int64_t>(B, nb * 128);
    best = std::max<int64_t>(best, n * choose_partition(I, nb, num_cus).np);
    if (choose_partition(I, nb, num_cus).np == 1) {
      best = std::max<int64_t>(best, B);
      break;
    }
  }
  return best;
}

// torch.topk over a dense [B, I] score matrix whose column c is item c * istride, with the
// optional CSR mask in real item ids (score.hip).  K <= 64.
hnm_status hnm_topk_rows_strided(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t I,
                                 const int64_t* mptr, const int32_t* midx, int K, float* ov,
                                 int64_t* oi, int64_t istride);
// Per sample row (score.hip sample_kth_kernel): out is [B, K], slot r = a lower bound of the
// row's (r+1)-th best value (the row's K best sampled survivors in descending order), -inf past
// the survivors; every slot NaN when the row holds a NaN.  All K slots are written (the
// bound-lists kernels read them), so callers must allocate B * K floats.  gate (optional,
// device): *gate == 0 skips the launch's work (a sample pass that was gated off).
hnm_status hnm_sample_kth(hnm_ctx* ctx, const float* s, int64_t ld, int64_t B, int64_t Ns,
                          const int64_t* mptr, const int32_t* midx, int K, int64_t grp,
                          int64_t period, const int32_t* sidx, float* out,
                          const int* gate = nullptr);

// Top-k merge of kc candidates per row (G groups), one wave per row (api.hip).  rows/nrows: list
// row b is output row rows[b], b < *nrows.  dyn_cus > 0: a row-list launch's candidates, whose
// partition count np follows *nrows (list_rows_np): kc and bstride are then np * kc.
hnm_status hnm_topk_merge_rows(hnm_ctx* ctx, const float* cv, const int32_t* ci, int64_t B,
                               int64_t G, int64_t gstride, int64_t bstride, int kc, int k,
                               float* ov, int64_t* oi, const int32_t* rows,
                               const int32_t* nrows, int64_t dyn_items = 0, int dyn_cus = 0);

// p[0, n) = v on the ctx stream
hnm_status hnm_fill_f32(hnm_ctx* ctx, float* p, int64_t n, float v);
