"""World-size-2 gloo test (CPU) of the item-sharded recommend path's host logic:
shard ranges, all_gather of user ids, global index offsets, all_to_all layout and the
(score desc, item asc) merge.  The per-shard scorer and the merge are the oracle here
(the product wires the HIP kernels, covered by the GPU tests); the result must equal the
single-process top-k over all items exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import hnm_oracle as O
from hnm_recommendation_amd import sharding as S
from hnm_recommendation_amd import synthetic as syn

U, I, B, K = 300, 257, 16, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_merge(cv, ci, k):
    G, Bn, kc = cv.shape
    v = cv.permute(1, 0, 2).reshape(Bn, G * kc).numpy().astype(np.float64)
    i = ci.permute(1, 0, 2).reshape(Bn, G * kc).numpy()
    out_v = np.empty((Bn, k), np.float32)
    out_i = np.empty((Bn, k), np.int64)
    for b in range(Bn):
        order = sorted(range(G * kc), key=lambda q: (-v[b, q], i[b, q]))[:k]
        out_v[b] = v[b, order]
        out_i[b] = i[b, order]
    return torch.from_numpy(out_v), torch.from_numpy(out_i)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0, bias_scale=0.05, emb_scale=20.0)
    lo, hi = S.shard_range(I, rank, world)

    def local_topk(all_ids):
        ids = all_ids.numpy()
        sub = dict(sd)
        sub["gmf_item_embedding.weight"] = sd["gmf_item_embedding.weight"][lo:hi]
        sub["mlp_item_embedding.weight"] = sd["mlp_item_embedding.weight"][lo:hi]
        scores = O.ncf_predict_all_items(sub, ids)
        v, i = O.topk(scores, K)
        return torch.from_numpy(v.astype(np.float32)), torch.from_numpy(i)

    class TwoPhase:
        """The certified scorer's protocol: begin -> lower bounds of each user's k-th best
        score (here: the shard's exact k-th), finish -> only items >= the all-reduced bound
        (short rows padded with -inf / -1)."""
        def __call__(self, all_ids):
            return local_topk(all_ids)

        def begin(self, all_ids):
            v, _ = local_topk(all_ids)
            return v[:, K - 1].clone()

        def finish(self, all_ids, lb):
            v, i = local_topk(all_ids)
            keep = v >= lb[:, None]
            return torch.where(keep, v, torch.tensor(-np.inf)), torch.where(keep, i, torch.tensor(-1))

    class TwoPhaseLists(TwoPhase):
        """NCF's protocol: begin_lists -> each row's k best lower bounds of distinct shard
        items (here: the shard's exact top-K values), all_gathered; the k-th best of the
        union is the bound finish filters with."""
        def begin_lists(self, all_ids):
            return local_topk(all_ids)[0].clone()

    users = torch.from_numpy(syn.user_batch(U, B, seed=10 + rank))
    out = []
    for scorer in (local_topk, TwoPhase(), TwoPhaseLists()):
        rec = S.ItemShardedRecommender(scorer, _np_merge, K, lo, rank, world)
        v, i = rec.recommend(users)
        out.append((v.numpy(), i.numpy()))
    for o in out[1:]:
        assert np.array_equal(out[0][1], o[1]) and np.array_equal(out[0][0], o[0])
    q.put((rank, users.numpy(), out[1][0], out[1][1]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_item_sharded_recommend_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0, bias_scale=0.05, emb_scale=20.0)
    for rank, users, v, i in results:
        full = O.ncf_predict_all_items(sd, users)
        rv, ri = O.topk(full, K)
        assert np.array_equal(i, ri), f"rank {rank}"
        np.testing.assert_array_equal(v, rv.astype(np.float32))


def test_shard_ranges_cover_items():
    for G in (1, 2, 3, 8):
        r = [S.shard_range(105542, g, G) for g in range(G)]
        assert r[0][0] == 0 and r[-1][1] == 105542
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


def _one_rank_worker(rank, port, q):
    """exchange=True on a 1-rank group: the collective branch at world 1 (the shape of the
    GPU RCCL test), and an exception injected into the bound all_reduce aborts the open
    two-phase call before it propagates."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0, bias_scale=0.05, emb_scale=20.0)

        class TwoPhase:
            def __init__(self):
                self.open, self.aborts = False, 0

            def _topk(self, all_ids):
                v, i = O.topk(O.ncf_predict_all_items(sd, all_ids.numpy()), K)
                return torch.from_numpy(v.astype(np.float32)), torch.from_numpy(i)

            def begin(self, all_ids):
                assert not self.open
                self.open = True
                return self._topk(all_ids)[0][:, K - 1].clone()

            def finish(self, all_ids, lb):
                assert self.open
                self.open = False
                return self._topk(all_ids)

            def abort(self):
                self.open = False
                self.aborts += 1

        users = torch.from_numpy(syn.user_batch(U, B, seed=31))
        sc = TwoPhase()
        rec = S.ItemShardedRecommender(sc, _np_merge, K, 0, exchange=True)
        v, i = rec.recommend(users)
        real = dist.all_reduce

        def failing(*a, **kw):
            raise RuntimeError("injected")
        S.dist.all_reduce = failing
        try:
            rec.recommend(users)
            raise AssertionError("the injected failure did not propagate")
        except RuntimeError as e:
            assert "injected" in str(e)
        finally:
            S.dist.all_reduce = real
        assert sc.aborts == 1 and not sc.open
        v2, i2 = rec.recommend(users)
        assert torch.equal(i, i2) and torch.equal(v, v2)
        q.put((users.numpy(), v.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


def test_forced_exchange_one_rank_and_abort():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank_worker, args=(0, _free_port(), q))
    p.start()
    users, v, i = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0, bias_scale=0.05, emb_scale=20.0)
    rv, ri = O.topk(O.ncf_predict_all_items(sd, users), K)
    assert np.array_equal(i, ri)
    np.testing.assert_array_equal(v, rv.astype(np.float32))


def test_exchange_requires_process_group():
    if dist.is_initialized():
        pytest.skip("a process group is live in this process")
    with pytest.raises(RuntimeError, match="process group"):
        S.ItemShardedRecommender(lambda u: u, _np_merge, K, 0, exchange=True)
