// Item-sharded top-k exchange over RCCL from the C ABI (SURVEY §8(b)'s
// `hnm_topk_allgather_merge`, §8(e)): for callers of include/hnm.h that are not Python.  The
// Python mirror runs its exchange through torch.distributed (sharding.py: a certified two-phase
// bound exchange + one packed all_to_all); this entry is the single-phase form a C / cgo / JNI
// host can drive on its own:
//
//   every rank scores the SAME batch of B users against its own contiguous item shard
//   (hnm_*_topk_f32 on the shard's tables, ids made global by the shard offset), then
//   hnm_topk_allgather_merge_f32 all-gathers the [B, k] lists of the `world` ranks over the
//   ctx's RCCL communicator (one ncclAllGather of the values and one of the ids, grouped, on the
//   ctx stream) and merges the world * k candidates of each row on the device
//   (hnm_topk_merge_f32: score desc, item asc) -- the global top-k, identical on every rank.
//
// The communicator is either created here (hnm_rccl_unique_id on one rank, the 128 id bytes
// shared by the host's own means, hnm_ctx_rccl_init on every rank; the ctx owns and destroys it)
// or borrowed from the host (hnm_ctx_set_rccl_comm with an existing ncclComm_t).
#include <rccl/rccl.h>
#include <string.h>

#include "hnm_internal.h"

#define HNM_RCCL_CHECK(expr)                                                             \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess) {                                                             \
      hnm_set_error("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__,     \
                    __LINE__);                                                           \
      return HNM_ECOLL;                                                                  \
    }                                                                                    \
  } while (0)

extern "C" hnm_status hnm_rccl_unique_id(void* out, int64_t size) {
  HNM_REQUIRE(out && size >= (int64_t)sizeof(ncclUniqueId), HNM_EINVAL,
              "rccl_unique_id: needs a buffer of %d bytes", (int)sizeof(ncclUniqueId));
  ncclUniqueId id;
  HNM_RCCL_CHECK(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return HNM_OK;
}

void hnm_rccl_release(hnm_ctx* ctx) {  // hnm_ctx_destroy / a replaced communicator
  if (ctx->comm && ctx->comm_owned) (void)ncclCommDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  ctx->comm_owned = 0;
}

extern "C" hnm_status hnm_ctx_rccl_init(hnm_ctx* ctx, int world, int rank, const void* unique_id,
                                        int64_t size) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && unique_id && size >= (int64_t)sizeof(ncclUniqueId) && world >= 1 &&
                  rank >= 0 && rank < world,
              HNM_EINVAL, "ctx_rccl_init: bad argument (world %d, rank %d)", world, rank);
  // RCCL binds the communicator to the current device: the ctx's, for this call only (the
  // entry's device guard restores the caller's current device on every exit path)
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ncclComm_t comm;
  HNM_RCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
  hnm_rccl_release(ctx);
  ctx->comm = comm;
  ctx->comm_owned = 1;
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_set_rccl_comm(hnm_ctx* ctx, void* comm) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  hnm_rccl_release(ctx);
  ctx->comm = comm;  // borrowed (NULL detaches)
  return HNM_OK;
}

extern "C" hnm_status hnm_ctx_rccl_abort(hnm_ctx* ctx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx, HNM_EINVAL, "ctx is NULL");
  // a communicator whose ranks disagree (one rank returned before the collective): abort
  // releases the peers blocked in it; the ctx no longer has a communicator afterwards
  if (ctx->comm && ctx->comm_owned) HNM_RCCL_CHECK(ncclCommAbort((ncclComm_t)ctx->comm));
  ctx->comm = nullptr;
  ctx->comm_owned = 0;
  return HNM_OK;
}

extern "C" hnm_status hnm_topk_allgather_merge_f32(hnm_ctx* ctx, const float* lval,
                                                   const int64_t* lidx, int64_t B, int k,
                                                   float* gval, int64_t* gidx) {
  HNM_CTX_DEVICE(ctx);
  HNM_REQUIRE(ctx && ((lval && lidx && gidx) || B == 0), HNM_EINVAL,
              "topk_allgather_merge: NULL argument");
  HNM_REQUIRE(ctx->comm, HNM_EINVAL,
              "topk_allgather_merge: no RCCL communicator (hnm_ctx_rccl_init / _set_rccl_comm)");
  HNM_REQUIRE(k >= 1 && k <= 128, HNM_EINVAL, "topk_allgather_merge: 1 <= k <= 128");
  HNM_REQUIRE(!ctx->pend.kind, HNM_EINVAL,
              "topk_allgather_merge: a two-phase top-k call is open on this ctx");
  ncclComm_t comm = (ncclComm_t)ctx->comm;
  int world = 0;
  HNM_RCCL_CHECK(ncclCommCount(comm, &world));
  // every rank takes part in the collective, B == 0 included (the counts must agree).  All local
  // checks -- the arguments, an open two-phase call, the workspace (the merge after the
  // collective needs none) -- run before it, so a rank that fails here returns before entering
  // the collective its peers are blocked in: the host then aborts the communicator on every
  // rank (hnm_ctx_rccl_abort).
  const size_t n = (size_t)std::max<int64_t>(B, 0) * k;
  const size_t szV = hnm_align(std::max<size_t>(n, 1) * world * 4);
  void* ws;
  hnm_status st = hnm_workspace(ctx, szV + std::max<size_t>(n, 1) * world * 8, &ws);
  if (st) return st;
  float* av = (float*)ws;
  int64_t* ai = (int64_t*)((char*)ws + szV);
  HNM_RCCL_CHECK(ncclGroupStart());
  // the group is closed on every path, a failed enqueue included
  const ncclResult_t r0 = ncclAllGather(lval, av, n, ncclFloat32, comm, ctx->stream);
  const ncclResult_t r1 =
      r0 == ncclSuccess ? ncclAllGather(lidx, ai, n, ncclInt64, comm, ctx->stream) : r0;
  const ncclResult_t r2 = ncclGroupEnd();
  HNM_RCCL_CHECK(r1 != ncclSuccess ? r1 : r2);
  if (B <= 0) return HNM_OK;
  // gathered [world][B][k]: group g = rank g's lists
  return hnm_topk_merge_f32(ctx, av, ai, B, world, (int64_t)n, k, k, k, gval, gidx);
}
