"""GPU: the item-sharded multi-GPU path with the real HIP kernels (per-shard fused top-K +
HIP merge), rehearsed as 2 gloo ranks on one GPU (the collectives are staged through host
memory; on a node they are RCCL).  The sharded top-K must equal the single-GPU top-K
bit for bit: the (score desc, item asc) order is total.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hnm_recommendation_amd import NeuralCF
from hnm_recommendation_amd import sharding as S
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
U, I, B, K = 6000, 40000, 300, 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=21, bias_scale=0.05, emb_scale=20.0)
    m = NeuralCF(U, I)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to("cuda:0").eval()


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model()
        lo, hi = S.shard_range(I, rank, world)
        users = torch.from_numpy(syn.user_batch(U, B, seed=50 + rank)).cuda()
        # both scorers run the bound-lists exchange (begin_lists -> all_gather -> k-th of the
        # union -> finish) and the packed pair all_to_all + sorted merge
        assert hasattr(S.ncf_shard_topk, "begin_lists") and hasattr(S.dot_shard_topk, "begin_lists")
        ncf = S.ItemShardedRecommender(S.ncf_shard_topk(m, lo, hi, K), S.hip_merge, K, lo, rank, world)
        v, i = ncf.recommend(users)
        gu = m.gmf_user_embedding.weight.detach().contiguous()
        gi = m.gmf_item_embedding.weight.detach().contiguous()
        dot = S.ItemShardedRecommender(S.dot_shard_topk(gu, gi, lo, hi, K), S.hip_merge, K, lo,
                                       rank, world)
        dv, di = dot.recommend(users)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), users=users.cpu().numpy(),
                 v=v.cpu().numpy(), i=i.cpu().numpy(), dv=dv.cpu().numpy(), di=di.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_item_sharding_matches_single_gpu(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    m = _model()
    gu = m.gmf_user_embedding.weight.detach().contiguous()
    gi = m.gmf_item_embedding.weight.detach().contiguous()
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        users = torch.from_numpy(z["users"]).cuda()
        v, i = m.recommend_with_scores(users, k=K)
        assert np.array_equal(z["i"], i.cpu().numpy())
        assert np.array_equal(z["v"].view(np.uint32), v.cpu().numpy().view(np.uint32))
        sv, si = S.dot_shard_topk(gu, gi, 0, I, K)(users)
        assert np.array_equal(z["di"], si.cpu().numpy())
        assert np.array_equal(z["dv"].view(np.uint32), sv.cpu().numpy().view(np.uint32))


def test_two_phase_contract():
    """begin/finish with the call's own bounds == the one-shot top-K (bitwise); the ctx
    refuses other work while a pair is open; finish without a matching begin raises."""
    m = _model()
    users = torch.from_numpy(syn.user_batch(U, 777, seed=3)).cuda()
    gu = m.gmf_user_embedding.weight.detach().contiguous()
    gi = m.gmf_item_embedding.weight.detach().contiguous()
    for scorer in (S.ncf_shard_topk(m, 0, I, K), S.dot_shard_topk(gu, gi, 0, I, K)):
        v1, i1 = scorer(users)
        lb = scorer.begin(users)
        assert torch.isfinite(lb).all()
        assert (v1[:, K - 1] >= lb).all()  # a lower bound of the exact k-th best score
        with pytest.raises(ValueError):
            scorer(users)  # the ctx's workspace is held by the open pair
        v2, i2 = scorer.finish(users, lb)
        assert torch.equal(i1, i2) and torch.equal(v1.view(torch.int32), v2.view(torch.int32))
    sc = S.dot_shard_topk(gu, gi, 0, I, K)
    sc._open = (users.to(torch.int64).contiguous(), K)  # no begin on the ctx
    with pytest.raises(ValueError):
        sc.finish(users, torch.zeros(users.numel(), device="cuda"))


# ------------------------------------------------------------------ BASELINE configs[4]
# LightGCN d=128 at the full H&M shape (65M-nnz graph): propagation item rows and the item
# table row-sharded, the bound and candidate exchanges -- rehearsed with 2 gloo ranks on one GPU.
LU, LI = syn.HM_USERS, syn.HM_ITEMS
LB = 512


def _lightgcn128(ei=None):
    from hnm_recommendation_amd import LightGCN
    if ei is None:
        ei = torch.from_numpy(syn.bipartite_edge_index(LU, LI, syn.HM_INTERACTIONS, seed=2))
    m = LightGCN(LU, LI, embedding_dim=128, num_layers=3)
    m.set_graph(ei)
    sd = syn.lightgcn_state_dict(LU, LI, 128, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.to("cuda:0").eval()


def _lgcn_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _lightgcn128()
        lo, hi = S.shard_range(LI, rank, world)
        users = torch.from_numpy(syn.user_batch(LU, LB, seed=70 + rank)).cuda()
        # the propagation recomputed per call with its item rows sharded over the ranks
        # (restricted plans + one all_gather of the [I, d] item rows after layers 1 and 2)
        ex = S.ItemRowExchange(LU, LI, rank, world)
        rec = S.ItemShardedRecommender(S.lightgcn_shard_topk(m, lo, hi, K, exchange=ex),
                                       S.hip_merge, K, lo, rank, world)
        v, i = rec.recommend(users)
        assert ex.calls == 2
        np.savez(os.path.join(out_dir, f"l{rank}.npz"), users=users.cpu().numpy(),
                 v=v.cpu().numpy(), i=i.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_lightgcn128_full_shape_two_rank_sharding(tmp_path):
    """configs[4] rehearsal: sharded result == single-GPU recommend_with_scores bitwise,
    and sampled rows == the CPU restatement of the reference (oracle/torch_cpu.py)."""
    world = 2
    mp.spawn(_lgcn_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ei = torch.from_numpy(syn.bipartite_edge_index(LU, LI, syn.HM_INTERACTIONS, seed=2))
    m = _lightgcn128(ei)
    rows = {}
    for r in range(world):
        z = np.load(tmp_path / f"l{r}.npz")
        users = torch.from_numpy(z["users"]).cuda()
        v, i = m.recommend_with_scores(users, k=K)
        assert np.array_equal(z["i"], i.cpu().numpy()), f"rank {r}: sharded != single-GPU"
        assert np.array_equal(z["v"].view(np.uint32), v.cpu().numpy().view(np.uint32))
        rows[r] = (z["users"][:4], z["i"][:4], z["v"][:4])
    # sampled rows against the reference's torch path restated on CPU
    from oracle import torch_cpu as T
    from parity import assert_topk_equivalent
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g = T.lightgcn_graph(ei, LU + LI)
    del ei, m
    w = torch.from_numpy(syn.lightgcn_state_dict(LU, LI, 128, seed=0)["embeddings.weight"])
    fu, fi = T.lightgcn_forward(w, g, LU)
    for r, (u, i, v) in rows.items():
        dense = (fu[torch.from_numpy(u)] @ fi.t()).numpy()
        assert_topk_equivalent(i, dense, K, what=f"lightgcn128 sharded rank {r} vs CPU ref")
        np.testing.assert_allclose(v, np.take_along_axis(dense, i, 1), rtol=1e-4,
                                   atol=1e-4 * float(np.abs(dense).max()))


# ------------------------------------------------------------------ N = 8 per-rank shape
# What one rank runs in the driver's 8-GPU scaling bench (bench.py --gpus 8, NCF default):
# the all-gathered 8 x 4,096 users against its 1/8 item shard of the full catalogue.  One
# process, no collective: the two-phase call with the rank's own bounds (the exchanged
# bound of 8 ranks only raises them) and the one-shot call must both equal the exact fp32 scan
# of the shard bit for bit, with no fallback rows.
def test_ncf_eight_way_rank_shape_certified_equals_exact():
    from hnm_recommendation_amd import _lib
    UU, II, world, rank = 200_000, syn.HM_ITEMS, 8, 7
    sd = syn.ncf_state_dict(UU, II, 64, (128, 64, 32), seed=0)
    m = NeuralCF(UU, II)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to("cuda:0").eval()
    lo, hi = S.shard_range(II, rank, world)
    users = torch.from_numpy(syn.user_batch(UU, world * 4096, seed=81)).cuda()
    sc = S.ncf_shard_topk(m, lo, hi, K)
    _lib.set_prefilter(users.device, False)
    try:
        ev, ei = sc(users)
    finally:
        _lib.set_prefilter(users.device, True)
    _lib.prefilter_stats(users.device, reset=True)
    _lib.set_option(users.device, _lib.HNM_OPT_STATS, 1)
    v1, i1 = sc(users)
    lb = sc.begin(users)
    v2, i2 = sc.finish(users, lb)
    _lib.set_option(users.device, _lib.HNM_OPT_STATS, 0)
    rows, cands, fallback = _lib.prefilter_stats(users.device, reset=True)
    print(f"rank shape {users.numel()} x {hi - lo}: candidates/row "
          f"{cands / max(rows - fallback, 1):.1f}, fallback rows {fallback} of {rows}")
    assert fallback == 0
    for v, i in ((v1, i1), (v2, i2)):
        assert torch.equal(i, ei)
        assert torch.equal(v.view(torch.int32), ev.view(torch.int32))


def test_mf_shard_scorer_with_biases():
    """The per-shard dot scorer with MatrixFactorization's user / item / global biases
    (matrix_factorization.py:108-131; what bench.py's `mf` step runs): each shard's top-K
    (certified path) equals the exact dense scores of that item slice, ordered (score desc,
    item asc), bit for bit -- the whole catalogue and a middle shard of three."""
    from hnm_recommendation_amd import MatrixFactorization
    U2, I2 = 5000, 30000
    sd = syn.mf_state_dict(U2, I2, 64, seed=4, bias_scale=0.05)
    m = MatrixFactorization(U2, I2, sparse=False)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to("cuda:0").eval()
    users = torch.from_numpy(syn.user_batch(U2, 257, seed=8)).cuda()
    dense = m.predict_all_items(users).cpu().numpy()
    for lo, hi in ((0, I2), S.shard_range(I2, 1, 3)):
        sc = S.dot_shard_topk(m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(),
                              lo, hi, K, user_bias=m.user_bias.weight.detach(),
                              item_bias=m.item_bias.weight.detach(),
                              const_bias=m.global_bias.detach())
        v, i = sc(users)
        v, i = v.cpu().numpy(), i.cpu().numpy()
        for r in range(users.numel()):
            s = dense[r, lo:hi]
            order = np.lexsort((np.arange(hi - lo), -s))[:K]
            assert np.array_equal(i[r], order), r
            assert np.array_equal(v[r].view(np.uint32), s[order].view(np.uint32)), r


def test_ncf_bound_lists():
    """hnm_ncf_topk_begin_lists_f32: each row's k certified sample lower bounds, descending;
    the r-th is <= the row's exact r-th best score over the shard, and the k-th equals
    begin's single bound bitwise.  Then the sharded protocol in one process: 4 shards' lists
    merged (k-th of the union) and every shard finished with that bound (short rows allowed)
    -> the merged top-k equals the single-GPU top-k bit for bit, and the merged bound is at
    least the max of the shards' single bounds (the all_reduce protocol's)."""
    m = _model()
    users = torch.from_numpy(syn.user_batch(U, 333, seed=12)).cuda()
    sc = S.ncf_shard_topk(m, 0, I, K)
    lists = sc.begin_lists(users)
    sc.abort()
    lb = sc.begin(users)
    sc.abort()
    assert lists.shape == (users.numel(), K)
    assert torch.equal(lists[:, K - 1].view(torch.int32), lb.view(torch.int32))
    assert (lists[:, :-1] >= lists[:, 1:]).all()
    exact = torch.sort(m.predict_all_items(users), dim=1, descending=True).values[:, :K]
    assert (lists <= exact).all()
    G = 4
    shards = [S.ncf_shard_topk(m, *S.shard_range(I, r, G), K) for r in range(G)]
    allv, singles = [], []
    for s in shards:
        allv.append(s.begin_lists(users))
        s.abort()
        singles.append(s.begin(users))
        s.abort()
    merged = torch.topk(torch.cat(allv, dim=1), K, dim=1).values[:, K - 1]
    assert (merged >= torch.stack(singles).amax(0)).all()
    vs, ids = [], []
    for r, s in enumerate(shards):
        s.begin_lists(users)
        v, i = s.finish(users, merged)
        lo = S.shard_range(I, r, G)[0]
        vs.append(v)
        ids.append(torch.where(i >= 0, i + lo, i))
    gv, gi = S.hip_merge(torch.stack(vs), torch.stack(ids), K)
    v1, i1 = m.recommend_with_scores(users, k=K)
    assert torch.equal(gi, i1) and torch.equal(gv.view(torch.int32), v1.view(torch.int32))


def test_dot_bound_lists():
    """hnm_dot_topk_begin_lists_f32 on MF with biases: descending certified lists, the r-th
    <= the row's exact r-th best score, the k-th equal to begin's single bound bitwise; 3
    shards' lists merged and every shard finished with the merged bound -> the merged top-k
    equals the exact dense top-k (score desc, item asc) bit for bit."""
    from hnm_recommendation_amd import MatrixFactorization
    U2, I2, G = 5000, 30000, 3
    sd = syn.mf_state_dict(U2, I2, 64, seed=5, bias_scale=0.05)
    m = MatrixFactorization(U2, I2, sparse=False)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to("cuda:0").eval()
    users = torch.from_numpy(syn.user_batch(U2, 301, seed=9)).cuda()

    def scorer(lo, hi):
        return S.dot_shard_topk(m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(),
                                lo, hi, K, user_bias=m.user_bias.weight.detach(),
                                item_bias=m.item_bias.weight.detach(),
                                const_bias=m.global_bias.detach())
    dense = m.predict_all_items(users)
    sc = scorer(0, I2)
    lists = sc.begin_lists(users)
    sc.abort()
    lb = sc.begin(users)
    sc.abort()
    assert lists.shape == (users.numel(), K)
    assert torch.equal(lists[:, K - 1].view(torch.int32), lb.view(torch.int32))
    assert (lists[:, :-1] >= lists[:, 1:]).all()
    assert (lists <= torch.sort(dense, dim=1, descending=True).values[:, :K]).all()
    assert torch.isfinite(lists).all()
    shards = [scorer(*S.shard_range(I2, r, G)) for r in range(G)]
    allv = []
    for s_ in shards:
        allv.append(s_.begin_lists(users))
        s_.abort()
    merged = torch.topk(torch.cat(allv, dim=1), K, dim=1).values[:, K - 1].contiguous()
    vs, ids = [], []
    for r, s_ in enumerate(shards):
        s_.begin_lists(users)
        v, i = s_.finish(users, merged)
        lo = S.shard_range(I2, r, G)[0]
        vs.append(v)
        ids.append(torch.where(i >= 0, i + lo, i))
    gv, gi = S.hip_merge(torch.stack(vs), torch.stack(ids), K)
    gv, gi, dn = gv.cpu().numpy(), gi.cpu().numpy(), dense.cpu().numpy()
    for r in range(users.numel()):
        order = np.lexsort((np.arange(I2), -dn[r]))[:K]
        assert np.array_equal(gi[r], order), r
        assert np.array_equal(gv[r].view(np.uint32), dn[r][order].view(np.uint32)), r


def test_bound_lists_exact_mode_and_tiny_shard():
    """Bound lists where no certified bound exists: a shard of 10 items (< K, exact path: -inf
    lists padded to K) beside a certified 8,990-item shard, and the whole protocol with the
    pre-filter off (every list -inf, finish = the exact scan) -> the merged top-k equals the
    exact dense top-k bit for bit in both."""
    from hnm_recommendation_amd import MatrixFactorization, _lib
    U2, I2, cut = 2000, 9000, 8990
    sd = syn.mf_state_dict(U2, I2, 64, seed=6, bias_scale=0.05)
    m = MatrixFactorization(U2, I2, sparse=False)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to("cuda:0").eval()
    users = torch.from_numpy(syn.user_batch(U2, 130, seed=3)).cuda()
    dn = m.predict_all_items(users).cpu().numpy()

    def scorer(lo, hi):
        return S.dot_shard_topk(m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(),
                                lo, hi, K, user_bias=m.user_bias.weight.detach(),
                                item_bias=m.item_bias.weight.detach(),
                                const_bias=m.global_bias.detach())

    def protocol():
        shards = [(0, cut), (cut, I2)]
        scs = [scorer(lo, hi) for lo, hi in shards]
        allv = []
        for sc in scs:
            allv.append(sc.begin_lists(users))
            sc.abort()
        merged = torch.topk(torch.cat(allv, dim=1), K, dim=1).values[:, K - 1].contiguous()
        vs, ids = [], []
        for (lo, _), sc in zip(shards, scs):
            sc.begin_lists(users)
            v, i = sc.finish(users, merged)
            vs.append(v)
            ids.append(torch.where(i >= 0, i + lo, i))
        gv, gi = S.hip_merge(torch.stack(vs), torch.stack(ids), K)
        gv, gi = gv.cpu().numpy(), gi.cpu().numpy()
        for r in range(users.numel()):
            order = np.lexsort((np.arange(I2), -dn[r]))[:K]
            assert np.array_equal(gi[r], order), r
            assert np.array_equal(gv[r].view(np.uint32), dn[r][order].view(np.uint32)), r
        return allv

    allv = protocol()
    assert allv[1].shape == (users.numel(), K) and torch.isneginf(allv[1]).all()
    assert torch.isfinite(allv[0]).all()
    _lib.set_prefilter(users.device, False)
    try:
        allv = protocol()
    finally:
        _lib.set_prefilter(users.device, True)
    assert all(torch.isneginf(a).all() for a in allv)


def test_kth_of_lists_matches_torch_topk():
    """The exchange's k-th best of G descending bound lists (hnm_topk_lists_kth_f32) equals
    torch.topk over their concatenation bit for bit, with -inf tails, ties, G = 1 and 16."""
    g = torch.Generator().manual_seed(5)
    for G, B, kk in ((8, 1000, K), (1, 77, K), (3, 513, 64), (16, 300, 5)):
        v = torch.randn(G, B, kk, generator=g)
        v[v < -1.2] = float("-inf")                     # short rows' padding
        v[:, ::7, :] = torch.round(v[:, ::7, :] * 4) / 4  # ties across shards
        v = torch.sort(v, dim=2, descending=True).values.cuda()
        got = S._kth_of_lists(v, kk)
        ref = torch.topk(v.permute(1, 0, 2).reshape(B, G * kk), kk, dim=1).values[:, kk - 1]
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), (G, B, kk)


def test_packed_pairs_merge_matches_hip_merge():
    """The exchange's pack (score bits + global id) and G-way merge of sorted lists equal the
    unpacked candidates through hnm_topk_merge_f32 bit for bit: ties across shards (id
    order), short lists padded (-inf, -1), G = 1, 8 and 16, k below / equal / above kc."""
    g = torch.Generator().manual_seed(9)
    for G, B, kc, k in ((8, 700, K, K), (1, 50, K, K), (16, 129, 5, 12), (3, 64, 20, 7)):
        vs, ids, offs = [], [], []
        for s in range(G):
            n = 40
            sc = torch.round(torch.randn(B, n, generator=g) * 3) / 3   # many ties
            order = torch.argsort(-sc, dim=1, stable=True)[:, :kc]      # (score desc, id asc)
            v = torch.gather(sc, 1, order)
            i = order.clone()
            short = torch.rand(B, generator=g) < 0.2                    # short rows
            v[short, kc // 2:] = float("-inf")
            i[short, kc // 2:] = -1
            vs.append(v)
            ids.append(i)
            offs.append(s * n)
        packed = torch.stack([S._pack_pairs(v.cuda(), i.cuda(), o) for v, i, o in zip(vs, ids, offs)])
        got_v, got_i = S._merge_pairs(packed, k)
        rv = torch.stack(vs).cuda()
        ri = torch.stack([torch.where(i >= 0, i + o, i) for i, o in zip(ids, offs)]).cuda()
        ref_v, ref_i = S.hip_merge(rv, ri, k)
        assert torch.equal(got_i, ref_i), (G, B, kc, k)
        assert torch.equal(got_v.view(torch.int32), ref_v.view(torch.int32)), (G, B, kc, k)
