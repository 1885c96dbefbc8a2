"""GPU: edge cases of the drop-in surface, against torch.topk's semantics.

The reference's recommend() ends in `torch.topk(scores, self.top_k, dim=1)`
(neural_cf.py:324, lightgcn.py:356, wide_deep.py:433, matrix_factorization.py:244) and the
server in `torch.topk(scores[0], num_items)` (serve.py:355).  Covered here:

* empty batches (B = 0): forward / predict_all_items / recommend / recommend_with_scores
  (fused k and dense k, with a filter dict and a UserHistory) on all four models, on the
  certified scans (I >= 8192) and the small-catalogue kernels -> shapes [0], [0, I], [0, k];
* k beyond the fused kernels (129 <= k <= I): the whole-row stable sort path
  (csrc/topk_sort.hip) returns exactly the first k of the stable (score desc, item asc) order
  of the model's own dense scores, masked entries -inf, over several row chunks;
* recommend() with top_k > num_items raises RuntimeError as torch.topk does; k = 0 -> [B, 0];
* a repeated user gets identical rows.
"""
import numpy as np
import pytest
import torch

from hnm_recommendation_amd import LightGCN, MatrixFactorization, NeuralCF, UserHistory, WideDeep
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _load(m, sd):
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval()


def _model(name, U, I, **kw):
    if name == "ncf":
        return _load(NeuralCF(U, I, **kw), syn.ncf_state_dict(U, I, seed=3, bias_scale=0.05,
                                                              emb_scale=20.0))
    if name == "mf":
        return _load(MatrixFactorization(U, I, sparse=False, **kw),
                     syn.mf_state_dict(U, I, seed=3, bias_scale=0.05))
    if name == "lightgcn":
        m = LightGCN(U, I, embedding_dim=64, **kw)
        m.set_graph(torch.from_numpy(syn.bipartite_edge_index(U, I, 8 * U, seed=2)))
        return _load(m, syn.lightgcn_state_dict(U, I, 64, seed=3))
    return _load(WideDeep(U, I, **kw), syn.widedeep_state_dict(U, I, 64, (512, 256, 128), seed=3))


def _stable_topk(dense, k, masks=None):
    """First k of the stable (score desc, item asc) order of each row; masked -> -inf."""
    d = dense.copy()
    if masks:
        for r, items in masks.items():
            d[r, sorted({x % d.shape[1] for x in items})] = -np.inf
    order = np.argsort(-d, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(d, order, 1), order


@pytest.mark.parametrize("name,I", [("ncf", 1500), ("ncf", 9000), ("mf", 9000),
                                    ("lightgcn", 9000), ("widedeep", 9000)])
def test_empty_batch(name, I):
    U = 2000
    m = _model(name, U, I)
    for ids in (torch.empty(0, dtype=torch.int64, device=DEV), torch.empty(0, dtype=torch.int64)):
        assert m.predict_all_items(ids).shape == (0, I)
        pairs = m.predict if name == "lightgcn" else m.forward
        assert pairs(ids, ids).numel() == 0
        assert m.recommend(ids).shape == (0, m.top_k)
        hist = UserHistory({1: {2, 3}}, U, I, DEV)
        for k in (12, 100, 300):
            for f in (None, {1: {2}}, hist):
                v, i = m.recommend_with_scores(ids, filter_items=f, k=k)
                assert v.shape == (0, k) and i.shape == (0, k) and i.dtype == torch.int64


@pytest.mark.parametrize("name", ["ncf", "mf", "lightgcn", "widedeep"])
def test_large_k_stable_sort_path(name):
    U, I = 3000, 2345 if name != "widedeep" else 9000
    m = _model(name, U, I)
    users = syn.user_batch(U, 97, seed=5)
    users[5] = users[4]                               # a repeated user
    u = torch.from_numpy(users).to(DEV)
    masks = {2: set(range(0, I, 7)), 4: {1, 2, 3, -1}, 5: {1, 2, 3, -1}}
    filt = {int(users[r]): s for r, s in masks.items() if r != 5}
    dense = m.predict_all_items(u).cpu().numpy()
    for k in (129, 700, I):
        v, i = m.recommend_with_scores(u, filter_items=filt, k=k)
        ev, ei = _stable_topk(dense, k, masks)
        np.testing.assert_array_equal(i.cpu().numpy(), ei, err_msg=f"{name} k={k} ids")
        np.testing.assert_array_equal(v.cpu().numpy().view(np.int32), ev.astype(np.float32).view(np.int32),
                                      err_msg=f"{name} k={k} score bits")
        assert torch.equal(i[4], i[5]) and torch.equal(v[4], v[5])
    # k > I clamps to the catalogue on recommend_with_scores (the serve path)
    assert m.recommend_with_scores(u, k=I + 5)[1].shape == (97, I)


def test_large_k_sort_path_row_chunks_full_catalogue():
    """B = 400 rows at I = 105,542: the sort path runs in several row chunks (~318 rows each)."""
    U, I = 20_000, syn.HM_ITEMS
    m = _model("mf", U, I)
    users = syn.user_batch(U, 400, seed=9)
    u = torch.from_numpy(users).to(DEV)
    masks = {r: set(syn.filter_dict(users[r:r + 1], I, per_user=23, seed=r)[int(users[r])])
             for r in (0, 317, 318, 399)}
    hist = UserHistory({int(users[r]): s for r, s in masks.items()}, U, I, DEV)
    dense = m.predict_all_items(u).cpu().numpy()
    v, i = m.recommend_with_scores(u, filter_items=hist, k=300)
    ev, ei = _stable_topk(dense, 300, masks)
    np.testing.assert_array_equal(i.cpu().numpy(), ei)
    np.testing.assert_array_equal(v.cpu().numpy(), ev)


@pytest.mark.parametrize("name", ["ncf", "mf", "lightgcn", "widedeep"])
def test_top_k_range_like_torch_topk(name):
    U, I = 500, 40
    m = _model(name, U, I, top_k=41)
    u = torch.tensor([0, 1, 2], device=DEV)
    with pytest.raises(RuntimeError, match="out of range"):
        m.recommend(u)
    m.top_k = 40                                      # k == I is legal: the full order
    dense = m.predict_all_items(u).cpu().numpy()
    np.testing.assert_array_equal(m.recommend(u).cpu().numpy(), _stable_topk(dense, 40)[1])
    v, i = m.recommend_with_scores(u, k=0)
    assert v.shape == (3, 0) and i.shape == (3, 0)
    with pytest.raises(RuntimeError, match="out of range"):
        m.recommend_with_scores(u, k=-1)
