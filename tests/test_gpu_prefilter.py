"""GPU: the certified f16 pre-filter of NCF top-K (ncf_cert.hip).

The pre-filter only prunes; returned scores are recomputed in exact fp32.  These tests pin
(1) the error bound the pruning relies on, |approx + bp - exact| <= E_u, on the full H&M
catalogue; (2) that top-K with the pre-filter is IDENTICAL (indices and score bits) to the
exact fp32 scan of every item; (3) the on-device fallback rows (overflowing candidate
lists, heavily filtered users, unusable bounds).
"""
import numpy as np
import pytest
import torch

from hnm_recommendation_amd import NeuralCF, _lib
from hnm_recommendation_amd import synthetic as syn
from oracle import hnm_oracle as O
from parity import assert_topk_equivalent

pytestmark = pytest.mark.gpu
DEV = "cuda"


def to_module(m, sd):
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval()


def prefilter_debug(m, users):
    w, keep = m._weights()
    B, I = users.numel(), m.num_items
    approx = torch.empty(B, I, device=DEV)
    bound = torch.empty(B, I, device=DEV)
    _lib.check(_lib.fn("hnm_ncf_prefilter_debug_f32")(_lib.ctx(users.device), w, _lib.ptr(users),
                                                      B, _lib.ptr(approx), I, _lib.ptr(bound)),
               "hnm_ncf_prefilter_debug_f32")
    _lib.sync_check(users.device)
    return approx, bound


def topk_both(m, users, filter_items=None, k=12):
    _lib.set_prefilter(users.device, False)
    try:
        ev, ei = m.recommend_with_scores(users, filter_items=filter_items, k=k)
    finally:
        _lib.set_prefilter(users.device, True)
    _lib.prefilter_stats(users.device, reset=True)
    pv, pi = m.recommend_with_scores(users, filter_items=filter_items, k=k)
    stats = _lib.prefilter_stats(users.device, reset=True)
    return (ev.cpu().numpy(), ei.cpu().numpy()), (pv.cpu().numpy(), pi.cpu().numpy()), stats


def full_model(seed=0, **kw):
    U, I = syn.HM_USERS, syn.HM_ITEMS
    return to_module(NeuralCF(U, I), syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=seed, **kw))


@pytest.mark.parametrize("kw", [{}, {"bias_scale": 0.1, "emb_scale": 30.0}])
def test_bound_holds_full_catalogue(kw):
    m = full_model(**kw)
    users = torch.from_numpy(syn.user_batch(syn.HM_USERS, 48, seed=5)).to(DEV)
    approx, bound = prefilter_debug(m, users)
    exact = m.predict_all_items(users)
    bp = float(m.prediction_layer.bias.detach())
    err = (approx + bp - exact).abs()
    ratio = (err / bound).max().item()
    print(f"max |approx + bp - exact| / bound = {ratio:.4f}; mean bound / score std = "
          f"{(bound.mean(1) / exact.std(1)).mean().item():.3f}")
    assert torch.isfinite(bound).all()
    assert ratio <= 1.0, ratio


@pytest.mark.parametrize("kw", [{}, {"bias_scale": 0.1, "emb_scale": 30.0}])
def test_prefilter_identical_to_exact_scan(kw):
    m = full_model(seed=3, **kw)
    users_np = syn.user_batch(syn.HM_USERS, 1024, seed=9)
    users = torch.from_numpy(users_np).to(DEV)
    (ev, ei), (pv, pi), stats = topk_both(m, users)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))  # bit-identical scores
    rows, cands, fallback = stats
    print(f"candidates/row {cands / max(rows - fallback, 1):.1f}, fallback rows {fallback}")
    assert rows == 1024 and fallback == 0
    # and against the CPU oracle on a few rows
    ref = O.ncf_predict_all_items(syn.ncf_state_dict(syn.HM_USERS, syn.HM_ITEMS, 64,
                                                     (128, 64, 32), seed=3, **kw), users_np[:3])
    assert_topk_equivalent(pi[:3], ref, 12, what="prefilter vs oracle")


def test_prefilter_with_filters_and_k():
    m = full_model(seed=4)
    users_np = syn.user_batch(syn.HM_USERS, 200, seed=2)
    users = torch.from_numpy(users_np).to(DEV)
    # filter each user's exact top-30 partially, plus random history
    _lib.set_prefilter(users.device, False)
    _, top = m.recommend_with_scores(users, k=30)
    _lib.set_prefilter(users.device, True)
    rng = np.random.default_rng(0)
    top = top.cpu().numpy()
    f = {int(u): set(top[r, ::2].tolist()) | set(rng.integers(0, syn.HM_ITEMS, 50).tolist())
         for r, u in enumerate(users_np)}
    for k in (1, 12, 64):
        (ev, ei), (pv, pi), stats = topk_both(m, users, f, k=k)
        assert np.array_equal(ei, pi), k
        assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32)), k
        for r, u in enumerate(users_np):
            assert not (set(pi[r].tolist()) & f[int(u)])


def test_fallback_rows_exact():
    """All-tied rows overflow the candidate list; a user whose catalogue is filtered down
    to < K items has no finite sample threshold; both take the exact on-device scan."""
    U, I = 5000, 40000
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=6)
    sd["gmf_item_embedding.weight"] = np.zeros_like(sd["gmf_item_embedding.weight"])
    sd["mlp_item_embedding.weight"][:] = sd["mlp_item_embedding.weight"][:1]  # identical items
    m = to_module(NeuralCF(U, I), sd)
    users = torch.tensor([1, 2, 3, 4, 5], device=DEV)
    f = {3: set(range(I)) - {7, 9000}}
    (ev, ei), (pv, pi), stats = topk_both(m, users, f)
    assert np.array_equal(ei, pi) and np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    assert pi[0].tolist() == list(range(12))  # ties -> lowest item ids
    assert pi[2, :2].tolist() == [7, 9000] and np.isneginf(pv[2, 2:]).all()
    assert stats[2] == 5


def test_unusable_bound_falls_back():
    """A non-finite weight makes the bound unusable: every row takes the exact scan."""
    U, I = 3000, 20000
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=7)
    sd["mlp_item_embedding.weight"][123, 5] = np.inf
    m = to_module(NeuralCF(U, I), sd)
    users = torch.arange(0, 300, device=DEV)
    (ev, ei), (pv, pi), stats = topk_both(m, users)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    assert stats[2] == 300
