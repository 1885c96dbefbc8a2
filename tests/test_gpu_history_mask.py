"""GPU: the device-resident purchase-history filter (`UserHistory` + hnm_mask_gather_csr).

The reference masks `filter_items[user_id]` per row with `scores[i, items] = -inf`
(neural_cf.py:316-321, same loop in lightgcn.py / wide_deep.py / matrix_factorization.py;
serve.py:350-352 for the server's purchase history).  A `UserHistory` holds that history
as a CSR on the GPU and gathers each batch's rows there; the result must be bit-identical
to the `filter_items` dict path (whose mask the oracle / reference goldens pin: the filtered
cases of test_gpu_golden_full.py and test_gpu_parity.py) for every model, on the certified
and the exact scans, including users without history, repeated users, negative history ids
(wrap like torch indexing) and histories that filter a user's whole top-K.
"""
import numpy as np
import pytest
import torch

from hnm_recommendation_amd import LightGCN, MatrixFactorization, NeuralCF, UserHistory, WideDeep
from hnm_recommendation_amd import _lib
from hnm_recommendation_amd import synthetic as syn
from hnm_recommendation_amd.models.base import filter_csr

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _load(m, sd):
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval()


def _history(users, I, seed):
    h = syn.filter_dict(users, I, per_user=23, seed=seed)
    us = sorted(h)
    del h[us[0]]                            # a batch user without history
    h[us[1]] = set()                        # an empty set
    h[us[2]] = {-1, -2, 5, 5 - I}           # negative ids wrap (5 - I == 5)
    h[us[3]] = set(range(0, I, max(1, I // 3000)))   # a long row
    h[10**9] = {1, 2}                       # a user outside [0, U): ignored
    return h


def _same(a, b, what):
    assert torch.equal(a[1], b[1]), f"{what}: ids differ"
    assert torch.equal(a[0].view(torch.int32), b[0].view(torch.int32)), f"{what}: score bits differ"


def test_mask_gather_matches_host_csr():
    U, I = 5000, 3000
    users = syn.user_batch(U, 700, seed=5)
    users = np.concatenate([users, users[:9]])       # repeated users
    h = _history(users, I, 6)
    hist = UserHistory(h, U, I, DEV)
    u = torch.from_numpy(users).to(DEV)
    mp, mi = hist.mask_for(u)
    hp, hi = filter_csr(u, h, I, DEV)
    n = int(hp[-1])
    assert torch.equal(mp, hp) and torch.equal(mi[:n], hi)
    assert hist.max_len == max(len({x % I for x in s}) for s in h.values() if s)
    _lib.sync_check(DEV)


@pytest.mark.parametrize("model", ["ncf", "mf", "lightgcn", "widedeep"])
def test_history_filter_equals_dict_filter(model):
    I = 20_000 if model == "widedeep" else syn.HM_ITEMS
    U = 6000
    if model == "ncf":
        m = _load(NeuralCF(U, I), syn.ncf_state_dict(U, I, seed=3, bias_scale=0.05, emb_scale=20.0))
    elif model == "mf":
        m = _load(MatrixFactorization(U, I, sparse=False), syn.mf_state_dict(U, I, seed=3,
                                                                             bias_scale=0.05))
    elif model == "lightgcn":
        m = LightGCN(U, I, embedding_dim=64)
        m.set_graph(torch.from_numpy(syn.bipartite_edge_index(U, I, 120_000, seed=2)))
        m = _load(m, syn.lightgcn_state_dict(U, I, 64, seed=3))
    else:
        m = _load(WideDeep(U, I), syn.widedeep_state_dict(U, I, 64, (512, 256, 128), seed=3))
    B = 64 if model == "widedeep" else 777
    users = syn.user_batch(U, B, seed=8)
    h = _history(users, I, 9)
    # filter a user's entire unfiltered top-12 (the next 12 must come back)
    u_dev = torch.from_numpy(users).to(DEV)
    top = m.recommend_with_scores(u_dev[:1])[1][0].cpu().tolist()
    h[int(users[0])] = set(top)
    hist = UserHistory(h, U, I, DEV)
    for prefilter in (True, False):
        _lib.set_prefilter(DEV, prefilter)
        try:
            for k in (12, 100):
                a = m.recommend_with_scores(u_dev, filter_items=h, k=k)
                b = m.recommend_with_scores(u_dev, filter_items=hist, k=k)
                _same(a, b, f"{model} k={k} prefilter={prefilter}")
                # host ids: checked on the host, no device-side check; same answer
                c = m.recommend_with_scores(torch.from_numpy(users), filter_items=hist, k=k)
                _same(a, c, f"{model} host ids k={k}")
        finally:
            _lib.set_prefilter(DEV, True)
    assert not set(b[1][0].tolist()) & set(top)


def test_recommender_uses_device_history():
    from hnm_recommendation_amd.serving import Recommender
    U, I = 4000, 12_000
    m = _load(NeuralCF(U, I), syn.ncf_state_dict(U, I, seed=4))
    users = syn.user_batch(U, 50, seed=2)
    h = _history(users, I, 3)
    rec = Recommender(U, I, models={"neural_cf": m}, user_history=h, device=DEV)
    out = rec.get_batch_recommendations([int(x) for x in users] + [U + 5], num_items=12,
                                        include_scores=True)
    assert rec._history_dev is not None and rec._history_dev.nnz > 0
    assert out[-1]["error"].endswith("not found")
    v, i = m.recommend_with_scores(torch.from_numpy(users).to(DEV), filter_items=h, k=12)
    for r, row in enumerate(out[:-1]):
        assert [int(x["article_id"]) for x in row["recommendations"]] == i[r].tolist()
        assert [x["score"] for x in row["recommendations"]] == v[r].tolist()
    rec.set_user_history({})
    one = rec.get_recommendations(int(users[0]), num_items=5)
    assert [int(x["article_id"]) for x in one["recommendations"]] == \
        m.recommend_with_scores(torch.from_numpy(users[:1]).to(DEV), k=5)[1][0].tolist()


def test_host_ids_skip_sync_and_device_ids_still_raise():
    U, I = 300, 9000
    m = _load(NeuralCF(U, I), syn.ncf_state_dict(U, I, seed=1))
    with pytest.raises(IndexError):
        m.recommend(torch.tensor([0, U]))                      # host: raised before launch
    with pytest.raises(IndexError):
        m.recommend(torch.tensor([0, U], device=DEV))          # device: error word + sync
    v, i = m.recommend_with_scores(torch.tensor([1, 2, 3]))
    assert i.shape == (3, 12) and torch.isfinite(v).all()


def test_sharded_history_masks_merge_to_full():
    """Per-item-shard masks (history ids in [lo, hi), renumbered) through the sharded
    scorers: 3 shards' top-K merged with the HIP merge == the whole-catalogue filtered
    top-K, bitwise (NCF, dot/MF tables, LightGCN per-call propagation)."""
    from hnm_recommendation_amd import sharding as S
    U, I, K = 6000, syn.HM_ITEMS, 12
    users = syn.user_batch(U, 400, seed=18)
    h = _history(users, I, 19)
    hist = UserHistory(h, U, I, DEV)
    u = torch.from_numpy(users).to(DEV)
    ncf = _load(NeuralCF(U, I), syn.ncf_state_dict(U, I, seed=7, bias_scale=0.05, emb_scale=20.0))
    lg = LightGCN(U, I, embedding_dim=64)
    lg.set_graph(torch.from_numpy(syn.bipartite_edge_index(U, I, 150_000, seed=2)))
    lg = _load(lg, syn.lightgcn_state_dict(U, I, 64, seed=7))
    fu, fi = lg.forward()
    cases = [("ncf", lambda lo, hi: S.ncf_shard_topk(ncf, lo, hi, K, hist),
              ncf.recommend_with_scores(u, filter_items=h)),
             ("lightgcn", lambda lo, hi: S.lightgcn_shard_topk(lg, lo, hi, K, hist),
              lg.recommend_with_scores(u, filter_items=h)),
             ("dot", lambda lo, hi: S.dot_shard_topk(fu, fi, lo, hi, K, hist),
              lg.recommend_with_scores(u, filter_items=h))]
    for name, make, ref in cases:
        cv, ci = [], []
        for g in range(3):
            lo, hi = S.shard_range(I, g, 3)
            v, i = make(lo, hi)(u)
            cv.append(v)
            ci.append(torch.where(i >= 0, i + lo, i))
        got = S.hip_merge(torch.stack(cv), torch.stack(ci), K)
        _same(got, ref, f"{name} 3-shard filtered")
    # the shard scorers shift copies of the module's (cached) weight struct, never the struct
    _same(ncf.recommend_with_scores(u, filter_items=h), cases[0][2], "ncf module after shards")
