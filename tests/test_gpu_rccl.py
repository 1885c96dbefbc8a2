"""GPU: the multi-GPU exchange branch of `ItemShardedRecommender` through a REAL RCCL
process group (backend "nccl" = RCCL on ROCm) -- a 1-rank group on the box's one GPU, with
`exchange=True` forcing the collective path.  This executes, on device tensors, exactly the
calls the 8-GPU run makes (sharding.py: `all_gather_into_tensor` of user ids and of the
certified bound lists, `all_to_all_single` of packed candidates) plus the HIP merge, and checks the result bit for bit against single-GPU
`recommend_with_scores` for NCF (two-phase certified), the dot scorer on LightGCN d=128
propagated tables (two-phase certified) and Wide&Deep (one-shot certified).  An exception
injected into either bound exchange must abort the open two-phase call so the next recommend
on the same ctx works.

The group runs in a spawned child (RCCL state stays out of the pytest process); any
assertion in the child fails `mp.spawn`.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hnm_recommendation_amd import LightGCN, NeuralCF, WideDeep
from hnm_recommendation_amd import _lib
from hnm_recommendation_amd import sharding as S
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
K = 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _load(m, sd):
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to("cuda:0").eval()


def _same(a, b, what):
    (av, ai), (bv, bi) = a, b
    assert torch.equal(ai, bi), f"{what}: item ids differ from single-GPU"
    assert torch.equal(av.view(torch.int32), bv.view(torch.int32)), f"{what}: score bits differ"


def _rccl_worker(rank, port):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        # ---- NeuralCF, full catalogue (certified two-phase path engages at I >= 8192)
        U, I = 20_000, syn.HM_ITEMS
        m = _load(NeuralCF(U, I), syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=5))
        users = torch.from_numpy(syn.user_batch(U, 1000, seed=9)).to(dev)
        sc = S.ncf_shard_topk(m, 0, I, K)
        rec = S.ItemShardedRecommender(sc, S.hip_merge, K, 0, exchange=True)
        ref = m.recommend_with_scores(users)
        _same(rec.recommend(users), ref, "ncf rccl exchange")

        # the purchase-history filter through the exchange (device-gathered per-shard mask)
        from hnm_recommendation_amd import UserHistory
        hist_d = syn.filter_dict(users.cpu().numpy(), I, per_user=23, seed=4)
        frec = S.ItemShardedRecommender(S.ncf_shard_topk(m, 0, I, K, UserHistory(hist_d, U, I, dev)),
                                        S.hip_merge, K, 0, exchange=True)
        _same(frec.recommend(users), m.recommend_with_scores(users, filter_items=hist_d),
              "ncf rccl exchange, filtered")

        # injected failure inside the exchange (NCF: the bound lists' all_gather, the call after
        # the user ids'): the open two-phase call is aborted, the error propagates, and the
        # same thread's ctx serves the next call
        real = dist.all_gather_into_tensor
        calls = {"n": 0}

        def failing(*a, **kw):
            calls["n"] += 1
            if calls["n"] == 2:
                raise RuntimeError("injected all_gather failure")
            return real(*a, **kw)
        S.dist.all_gather_into_tensor = failing
        try:
            with pytest.raises(RuntimeError, match="injected"):
                rec.recommend(users)
        finally:
            S.dist.all_gather_into_tensor = real
        assert calls["n"] == 2 and sc._open is None
        _same(rec.recommend(users), ref, "ncf rccl exchange after abort")
        _same(m.recommend_with_scores(users), ref, "ncf single-GPU after abort")

        # ---- dot scorer on LightGCN d=128 propagated tables
        LU, LE = 30_000, 600_000
        lg = LightGCN(LU, I, embedding_dim=128, num_layers=3)
        lg.set_graph(torch.from_numpy(syn.bipartite_edge_index(LU, I, LE, seed=2)))
        lg = _load(lg, syn.lightgcn_state_dict(LU, I, 128, seed=0))
        fu, fi = lg.forward()
        lusers = torch.from_numpy(syn.user_batch(LU, 777, seed=11)).to(dev)
        drec = S.ItemShardedRecommender(S.dot_shard_topk(fu, fi, 0, I, K), S.hip_merge, K, 0,
                                        exchange=True)
        _same(drec.recommend(lusers), lg.recommend_with_scores(lusers), "lightgcn128 rccl")
        # the dot scorer's bound lists exchange: a failure there aborts too
        calls["n"] = 0
        S.dist.all_gather_into_tensor = failing
        try:
            with pytest.raises(RuntimeError, match="injected"):
                drec.recommend(lusers)
        finally:
            S.dist.all_gather_into_tensor = real
        assert calls["n"] == 2 and drec.local_topk._open is None
        _same(drec.recommend(lusers), lg.recommend_with_scores(lusers), "lightgcn128 after abort")
        # the per-call-propagation scorer (what bench.py's LightGCN step runs)
        prec = S.ItemShardedRecommender(S.lightgcn_shard_topk(lg, 0, I, K), S.hip_merge, K, 0,
                                        exchange=True)
        _same(prec.recommend(lusers), lg.recommend_with_scores(lusers), "lightgcn128 per-call")

        # ---- Wide&Deep (one-shot certified scorer, full K-lists exchanged)
        WU, WI = 5_000, 20_000
        wd = _load(WideDeep(WU, WI), syn.widedeep_state_dict(WU, WI, 64, (512, 256, 128), seed=3))
        wusers = torch.from_numpy(syn.user_batch(WU, 96, seed=12)).to(dev)
        wrec = S.ItemShardedRecommender(S.widedeep_shard_topk(wd, 0, WI, K), S.hip_merge, K, 0,
                                        exchange=True)
        _same(wrec.recommend(wusers), wd.recommend_with_scores(wusers), "widedeep rccl")
        _lib.sync_check(dev)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_exchange_matches_single_gpu():
    mp.spawn(_rccl_worker, args=(_free_port(),), nprocs=1, join=True)


def _c_exchange_worker(rank):
    """hnm_topk_allgather_merge_f32 (the C-ABI exchange, csrc/collective.hip) on a 1-rank RCCL
    communicator the library creates itself: unsorted lists with ties and empty slots come back
    as the (score desc, item asc) top-k; the dot top-k of a 3-shard split merged by the library
    equals the unsharded call; no communicator -> ValueError; B = 0 is a no-op."""
    import ctypes as C
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    c = _lib.ctx(dev)
    f = _lib.fn
    B, k = 300, 12
    # without a communicator the entry refuses
    v = torch.zeros(B, k, device=dev)
    i = torch.zeros(B, k, dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        _lib.check(f("hnm_topk_allgather_merge_f32")(c, _lib.ptr(v), _lib.ptr(i), B, k,
                                                     _lib.ptr(v), _lib.ptr(i)), "merge")
    uid = (C.c_char * 128)()
    _lib.check(f("hnm_rccl_unique_id")(uid, 128), "unique_id")
    _lib.check(f("hnm_ctx_rccl_init")(c, 1, 0, uid, 128), "rccl_init")
    # (1) unsorted lists, ties, empty (-inf, -1) slots
    g = torch.Generator().manual_seed(3)
    lv = torch.randint(0, 6, (B, k), generator=g).float().to(dev)
    li = torch.stack([torch.randperm(1000, generator=g)[:k] for _ in range(B)]).to(dev)
    lv[:, -2:] = -float("inf")
    li[:, -2:] = -1
    ov = torch.empty(B, k, device=dev)
    oi = torch.empty(B, k, dtype=torch.int64, device=dev)
    _lib.check(f("hnm_topk_allgather_merge_f32")(c, _lib.ptr(lv), _lib.ptr(li), B, k,
                                                 _lib.ptr(ov), _lib.ptr(oi)), "merge")
    torch.cuda.synchronize()
    ref_i = li.cpu().numpy().copy()
    ref_v = lv.cpu().numpy().copy()
    for b in range(B):
        key = np.lexsort((np.where(ref_i[b] < 0, 1 << 40, ref_i[b]), -ref_v[b].astype(np.float64)))
        ref_i[b], ref_v[b] = ref_i[b][key], ref_v[b][key]
    np.testing.assert_array_equal(oi.cpu().numpy(), ref_i)
    np.testing.assert_array_equal(ov.cpu().numpy(), ref_v)
    # (2) three item shards of a dot-product model, scored with global ids, merged
    U, I, d = 5000, 30_001, 64
    sd = syn.lightgcn_state_dict(U, I, d, seed=4)
    ut = torch.from_numpy(sd["embeddings.weight"][:U]).to(dev)
    it = torch.from_numpy(sd["embeddings.weight"][U:]).to(dev)
    users = torch.from_numpy(syn.user_batch(U, B, seed=2)).to(dev)
    full = S.dot_shard_topk(ut, it, 0, I, k)(users)
    parts = []
    for r in range(3):
        lo, hi = S.shard_range(I, r, 3)
        pv, pi = S.dot_shard_topk(ut, it, lo, hi, k)(users)
        parts.append((pv, torch.where(pi >= 0, pi + lo, pi)))
    # world 1: the three shards' lists side by side as one rank's k' = 3k candidates
    cv = torch.cat([p[0] for p in parts], 1).contiguous()
    ci = torch.cat([p[1] for p in parts], 1).contiguous()
    mv = torch.empty(B, 3 * k, device=dev)
    mi = torch.empty(B, 3 * k, dtype=torch.int64, device=dev)
    _lib.check(f("hnm_topk_allgather_merge_f32")(c, _lib.ptr(cv), _lib.ptr(ci), B, 3 * k,
                                                 _lib.ptr(mv), _lib.ptr(mi)), "merge shards")
    _same((mv[:, :k].contiguous(), mi[:, :k].contiguous()), full, "C exchange, 3 shards")
    # (3) B = 0
    _lib.check(f("hnm_topk_allgather_merge_f32")(c, None, None, 0, k, None, None), "merge B=0")
    torch.cuda.synchronize()
    _lib.check(f("hnm_ctx_set_rccl_comm")(c, None), "detach")


def test_c_abi_rccl_exchange_one_rank():
    mp.spawn(_c_exchange_worker, nprocs=1, join=True)


def _device_binding_worker(rank):
    """hnm.h "Device binding": hnm_ctx_create leaves the caller's current device unchanged (also
    for a refused device id); with two or more GPUs, a ctx of device 0 driven from a thread whose
    current device is 1 runs a fused top-k and the C-ABI exchange on device 0 (results equal to
    the same calls made from device 0) and leaves device 1 current; hnm_ctx_rccl_abort releases
    the ctx's communicator (the exchange is then refused)."""
    import ctypes as C
    f = _lib.fn
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(0)
    h = C.c_void_p()
    assert f("hnm_ctx_create")(ndev + 3, C.byref(h)) == _lib.HNM_EINVAL
    assert torch.cuda.current_device() == 0
    other = 1 if ndev > 1 else 0
    torch.cuda.set_device(other)
    _lib.check(f("hnm_ctx_create")(0, C.byref(h)), "ctx_create")
    assert torch.cuda.current_device() == other
    dev = torch.device("cuda", 0)
    U, I, d, B, k = 3000, 20_000, 64, 200, 12
    sd = syn.lightgcn_state_dict(U, I, d, seed=6)
    ut = torch.from_numpy(sd["embeddings.weight"][:U]).to(dev)
    it = torch.from_numpy(sd["embeddings.weight"][U:]).to(dev)
    users = torch.from_numpy(syn.user_batch(U, B, seed=4)).to(dev)
    torch.cuda.synchronize(dev)
    ov = torch.empty(B, k, device=dev)
    oi = torch.empty(B, k, dtype=torch.int64, device=dev)
    try:
        _lib.check(f("hnm_dot_topk_f32")(h, _lib.ptr(ut), U, d, _lib.ptr(users), B, _lib.ptr(it), I, d,
                                         d, None, None, None, None, None, k, _lib.ptr(ov),
                                         _lib.ptr(oi)), "dot_topk")
        assert torch.cuda.current_device() == other
        uid = (C.c_char * 128)()
        _lib.check(f("hnm_rccl_unique_id")(uid, 128), "unique_id")
        _lib.check(f("hnm_ctx_rccl_init")(h, 1, 0, uid, 128), "rccl_init")
        mv = torch.empty(B, k, device=dev)
        mi = torch.empty(B, k, dtype=torch.int64, device=dev)
        _lib.check(f("hnm_topk_allgather_merge_f32")(h, _lib.ptr(ov), _lib.ptr(oi), B, k,
                                                     _lib.ptr(mv), _lib.ptr(mi)), "merge")
        assert torch.cuda.current_device() == other
        _lib.check(f("hnm_ctx_check")(h), "check")
        torch.cuda.set_device(0)
        ref = S.dot_shard_topk(ut, it, 0, I, k)(users)
        _same((ov, oi), ref, "dot top-k from another current device")
        _same((mv, mi), ref, "C exchange from another current device")
        _lib.check(f("hnm_ctx_rccl_abort")(h), "rccl_abort")
        with pytest.raises(ValueError):
            _lib.check(f("hnm_topk_allgather_merge_f32")(h, _lib.ptr(ov), _lib.ptr(oi), B, k,
                                                         _lib.ptr(mv), _lib.ptr(mi)), "merge")
        print(f"device binding checked with {ndev} visible device(s)")
    finally:
        f("hnm_ctx_destroy")(h)
    assert torch.cuda.current_device() == 0


def test_c_abi_device_binding():
    mp.spawn(_device_binding_worker, nprocs=1, join=True)
