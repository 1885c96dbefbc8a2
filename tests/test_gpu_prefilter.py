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
    _lib.set_option(users.device, _lib.HNM_OPT_STATS, 1)
    pv, pi = m.recommend_with_scores(users, filter_items=filter_items, k=k)
    _lib.set_option(users.device, _lib.HNM_OPT_STATS, 0)
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
    users_np = syn.user_batch(syn.HM_USERS, 1024 - 23, seed=9)  # odd users in the last wave
    users = torch.from_numpy(users_np).to(DEV)
    (ev, ei), (pv, pi), stats = topk_both(m, users)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))  # bit-identical scores
    rows, cands, fallback = stats
    print(f"candidates/row {cands / max(rows - fallback, 1):.1f}, fallback rows {fallback}")
    assert rows == users_np.size and fallback == 0
    # and against the CPU oracle on every 64th row
    rows = np.arange(0, users_np.size, 64)
    ref = O.ncf_predict_all_items(syn.ncf_state_dict(syn.HM_USERS, syn.HM_ITEMS, 64,
                                                     (128, 64, 32), seed=3, **kw), users_np[rows])
    assert_topk_equivalent(pi[rows], ref, 12, what="prefilter vs oracle")


def test_prefilter_with_filters_and_k():
    m = full_model(seed=4)
    users_np = syn.user_batch(syn.HM_USERS, 201, seed=2)
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
    # 16 rows: below that the library routes the batch to the exact scan (ncf.hip, serve path)
    users = torch.arange(1, 17, device=DEV)
    f = {3: set(range(I)) - {7, 9000}}
    (ev, ei), (pv, pi), stats = topk_both(m, users, f)
    assert np.array_equal(ei, pi) and np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    assert pi[0].tolist() == list(range(12))  # ties -> lowest item ids
    assert pi[2, :2].tolist() == [7, 9000] and np.isneginf(pv[2, 2:]).all()
    assert stats[2] == 16


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


# ------------------------------------------------------------------ dot models (LightGCN / MF)
def dot_topk(ut, ids, it, k, ub=None, ib=None, cb=None, mptr=None, midx=None):
    B = ids.numel()
    ov = torch.empty(B, k, device=DEV)
    oi = torch.empty(B, k, dtype=torch.int64, device=DEV)
    _lib.check(_lib.fn("hnm_dot_topk_f32")(
        _lib.ctx(ids.device), _lib.ptr(ut), ut.shape[0], ut.stride(0), _lib.ptr(ids), B,
        _lib.ptr(it), it.shape[0], it.stride(0), ut.shape[1], _lib.ptr(ub), _lib.ptr(ib),
        _lib.ptr(cb), _lib.ptr(mptr), _lib.ptr(midx), k, _lib.ptr(ov), _lib.ptr(oi)), "dot_topk")
    _lib.sync_check(ids.device)
    return ov.cpu().numpy(), oi.cpu().numpy()


def dot_both(*args, **kw):
    dev = args[1].device
    _lib.set_prefilter(dev, False)
    try:
        ex = dot_topk(*args, **kw)
    finally:
        _lib.set_prefilter(dev, True)
    _lib.prefilter_stats(dev, reset=True)
    _lib.set_option(dev, _lib.HNM_OPT_STATS, 1)
    pf = dot_topk(*args, **kw)
    _lib.set_option(dev, _lib.HNM_OPT_STATS, 0)
    return ex, pf, _lib.prefilter_stats(dev, reset=True)


def dot_tables(d, U=50000, I=syn.HM_ITEMS, seed=0, bias=False):
    g = torch.Generator().manual_seed(seed)
    ut = (torch.randn(U, d, generator=g) * 0.1).to(DEV)
    it = (torch.randn(I, d, generator=g) * 0.1 * (1 + torch.rand(I, 1, generator=g))).to(DEV)
    b = None
    if bias:
        b = ((torch.randn(U, generator=g) * 0.05).to(DEV), (torch.randn(I, generator=g) * 0.05).to(DEV),
             torch.tensor([0.3], device=DEV))
    return ut, it, b


@pytest.mark.parametrize("d,bias", [(64, False), (128, False), (64, True), (32, True)])
def test_dot_bound_holds(d, bias):
    ut, it, b = dot_tables(d, bias=bias)
    ids = torch.from_numpy(syn.user_batch(ut.shape[0], 40, seed=3)).to(DEV)
    ub, ib, cb = b if b else (None, None, None)
    I = it.shape[0]
    approx = torch.empty(40, I, device=DEV)
    bound = torch.empty(40, device=DEV)
    _lib.check(_lib.fn("hnm_dot_prefilter_debug_f32")(
        _lib.ctx(ids.device), _lib.ptr(ut), ut.shape[0], ut.stride(0), _lib.ptr(ids), 40,
        _lib.ptr(it), I, it.stride(0), d, _lib.ptr(ub), _lib.ptr(ib), _lib.ptr(cb),
        _lib.ptr(approx), I, _lib.ptr(bound)), "dot_prefilter_debug")
    _lib.sync_check(ids.device)
    exact = ut[ids] @ it.T
    if b:
        exact = exact + ub[ids][:, None] + cb + ib[None, :]
    ratio = ((approx - exact).abs().amax(1) / bound).max().item()
    print(f"d={d} bias={bias}: max err / bound = {ratio:.4f}, bound / std = "
          f"{(bound / exact.std(1)).mean().item():.2e}")
    assert ratio <= 1.0


@pytest.mark.parametrize("d,bias,B", [(64, False, 4096), (128, False, 1000), (64, True, 777),
                                      (32, True, 5)])
def test_dot_prefilter_identical(d, bias, B):
    ut, it, b = dot_tables(d, bias=bias, seed=d + B)
    ids = torch.from_numpy(syn.user_batch(ut.shape[0], B, seed=B)).to(DEV)
    kw = dict(zip(("ub", "ib", "cb"), b)) if b else {}
    (ev, ei), (pv, pi), stats = dot_both(ut, ids, it, 12, **kw)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    rows, cands, fallback = stats
    print(f"d={d} B={B}: candidates/row {cands / max(rows - fallback, 1):.1f}, fallback {fallback}")
    assert rows == B and fallback == 0


@pytest.mark.parametrize("B,I,k", [(32768, 13192, 12), (20000, 8200, 12), (50000, 9000, 40)])
def test_dot_prefilter_many_rows_small_shard(B, I, k):
    """An 8-rank item shard's shape on one GPU (round 5): many rows over few items, so the
    sample K-th pops 2 or 4 rows per wave (sample_kth_kernel<R>, lossless at <= 4 columns a
    lane) and most rows re-score a handful of candidates in one sorting round
    (dcert_rescore_kernel's 16 / 32 / 64-lane sort) -- bitwise the exact scan's top-K."""
    ut, it, b = dot_tables(64, U=60000, I=I, seed=7, bias=True)
    ids = torch.from_numpy(syn.user_batch(ut.shape[0], B, seed=13)).to(DEV)
    ub, ib, cb = b
    (ev, ei), (pv, pi), stats = dot_both(ut, ids, it, k, ub=ub, ib=ib, cb=cb)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    rows, cands, fallback = stats
    print(f"dot B={B} I={I} k={k}: candidates/row {cands / max(rows - fallback, 1):.1f}, "
          f"fallback {fallback}")
    assert rows == B


def test_dot_prefilter_masks_ties_fallback():
    d, I = 64, 30000
    ut, it, _ = dot_tables(d, U=2000, I=I, seed=5)
    it[100:200] = it[100]  # 100 exact ties
    ids = torch.arange(0, 300, device=DEV)
    rng = np.random.default_rng(1)
    f = {u: set(rng.integers(0, I, 40).tolist()) | set(range(100, 150)) for u in range(0, 300, 3)}
    f[7] = set(range(I)) - {5, 17}  # < K unfiltered items -> fallback row
    from hnm_recommendation_amd.models.base import filter_csr
    mptr, midx = filter_csr(ids, f, I, ids.device)
    (ev, ei), (pv, pi), stats = dot_both(ut, ids, it, 12, mptr=mptr, midx=midx)
    assert np.array_equal(ei, pi) and np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    assert sorted(pi[7, :2].tolist()) == [5, 17] and np.isneginf(pv[7, 2:]).all()
    assert stats[2] >= 1
    # degenerate user (zero row): every item ties -> overflow -> exact fallback
    ut[11] = 0
    (ev, ei), (pv, pi), stats = dot_both(ut, ids, it, 12)
    assert np.array_equal(ei, pi) and pi[11].tolist() == list(range(12))


# ------------------------------------------------------------------ Wide&Deep (split-f16)
def wd_model(U, I, seed=0, layers=(512, 256, 128), d=64, **kw):
    from hnm_recommendation_amd import WideDeep
    sd = syn.widedeep_state_dict(U, I, d, layers, seed=seed, **kw)
    m = WideDeep(U, I, embedding_dim=d, deep_layers=list(layers),
                 num_user_features=kw.get("num_user_features", 0))
    return to_module(m, sd), sd


def wd_prefilter_debug(m, users, feats=None):
    w, keep = m._weights()
    B, I = users.numel(), m.num_items
    approx = torch.empty(B, I, device=DEV)
    bound = torch.empty(B, I, device=DEV)
    _lib.check(_lib.fn("hnm_widedeep_prefilter_debug_f32")(
        _lib.ctx(users.device), w, _lib.ptr(users), B, _lib.ptr(feats), _lib.ptr(approx), I,
        _lib.ptr(bound)), "hnm_widedeep_prefilter_debug_f32")
    _lib.sync_check(users.device)
    return approx, bound


def wd_refine_debug(m, users, feats=None):
    """The re-scoring cascade's three-pass refining stage over the whole catalogue."""
    w, keep = m._weights()
    B, I = users.numel(), m.num_items
    approx = torch.empty(B, I, device=DEV)
    bound = torch.empty(B, I, device=DEV)
    _lib.check(_lib.fn("hnm_widedeep_refine_debug_f32")(
        _lib.ctx(users.device), w, _lib.ptr(users), B, _lib.ptr(feats), _lib.ptr(approx), I,
        _lib.ptr(bound)), "hnm_widedeep_refine_debug_f32")
    _lib.sync_check(users.device)
    return approx, bound


@pytest.mark.parametrize("kw", [{}, {"bias_scale": 0.05, "randomize_bn": True, "emb_scale": 10.0}])
def test_wd_refine_bound_holds_full_catalogue(kw):
    """The cascade's refined bound (widedeep.hip wdc_refine_kernel, round 5): |approx - exact|
    <= bound for every pair of 16 users x the H&M catalogue, and much tighter than the scan's."""
    m, _ = wd_model(20000, syn.HM_ITEMS, seed=1, **kw)
    users = torch.from_numpy(syn.user_batch(20000, 16, seed=5)).to(DEV)
    approx, bound = wd_refine_debug(m, users)
    exact = m.predict_all_items(users)
    ratio = ((approx - exact).abs() / bound).max().item()
    _, scan_bound = wd_prefilter_debug(m, users)
    tight = (bound / scan_bound).median().item()
    print(f"W&D refine: max |approx - exact| / bound = {ratio:.4f}; median bound / scan bound = "
          f"{tight:.4f}")
    assert torch.isfinite(bound).all()
    assert ratio <= 1.0, ratio
    assert tight < 0.5, tight


@pytest.mark.parametrize("kw", [{}, {"bias_scale": 0.05, "randomize_bn": True, "emb_scale": 10.0}])
def test_wd_bound_holds_full_catalogue(kw):
    """|approx - exact| <= bound for every pair of 16 users x the H&M catalogue."""
    m, _ = wd_model(20000, syn.HM_ITEMS, seed=1, **kw)
    users = torch.from_numpy(syn.user_batch(20000, 16, seed=5)).to(DEV)
    approx, bound = wd_prefilter_debug(m, users)
    exact = m.predict_all_items(users)
    ratio = ((approx - exact).abs() / bound).max().item()
    print(f"W&D: max |approx - exact| / bound = {ratio:.4f}; mean bound / score std = "
          f"{(bound.mean(1) / exact.std(1)).mean().item():.4f}")
    assert torch.isfinite(bound).all()
    assert ratio <= 1.0, ratio


@pytest.mark.parametrize("kw", [{}, {"bias_scale": 0.05, "randomize_bn": True, "emb_scale": 10.0}])
def test_wd_prefilter_identical_to_exact(kw):
    m, _ = wd_model(20000, syn.HM_ITEMS, seed=2, **kw)
    users_np = syn.user_batch(20000, 64 + 3, seed=9)
    users = torch.from_numpy(users_np).to(DEV)
    (ev, ei), (pv, pi), stats = topk_both(m, users)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    rows, cands, fallback = stats
    print(f"W&D candidates/row {cands / max(rows - fallback, 1):.1f}, fallback rows {fallback}")
    assert rows == users_np.size and fallback == 0


def test_wd_prefilter_filters_k_fallback():
    m, _ = wd_model(5000, 12000, seed=3, bias_scale=0.05, randomize_bn=True)
    users_np = syn.user_batch(5000, 37, seed=2)
    users = torch.from_numpy(users_np).to(DEV)
    _lib.set_prefilter(users.device, False)
    _, top = m.recommend_with_scores(users, k=30)
    _lib.set_prefilter(users.device, True)
    top = top.cpu().numpy()
    rng = np.random.default_rng(1)
    f = {int(u): set(top[r, ::2].tolist()) | set(rng.integers(0, 12000, 50).tolist())
         for r, u in enumerate(users_np)}
    f[int(users_np[5])] = set(range(12000)) - {11, 7000}  # < K items left: exact fallback
    for k in (1, 12, 64):
        (ev, ei), (pv, pi), stats = topk_both(m, users, f, k=k)
        assert np.array_equal(ei, pi), k
        assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32)), k
        assert stats[2] >= (1 if k > 2 else 0)
        for r, u in enumerate(users_np):
            assert not (set(pi[r][np.isfinite(pv[r])].tolist()) & f[int(u)])
    assert pi[5, :2].tolist() == [11, 7000] and np.isneginf(pv[5, 2:]).all()


def test_wd_prefilter_small_towers_and_bad_bound():
    # two-layer tower (RB2 = 1, no layer 3) with user features
    from hnm_recommendation_amd import WideDeep
    U, I, F = 3000, 9000, 10
    sd = syn.widedeep_state_dict(U, I, 16, (64, 32), num_user_features=F, seed=4,
                                 bias_scale=0.05, randomize_bn=True, emb_scale=10.0)
    m = to_module(WideDeep(U, I, num_user_features=F, embedding_dim=16, deep_layers=[64, 32]), sd)
    users = torch.from_numpy(syn.user_batch(U, 21, seed=8)).to(DEV)
    feats = torch.from_numpy(np.random.default_rng(9).standard_normal((21, F)).astype(np.float32)).to(DEV)
    _lib.set_prefilter(users.device, False)
    ev, ei = m.recommend_with_scores(users, feats, k=12)
    _lib.set_prefilter(users.device, True)
    pv, pi = m.recommend_with_scores(users, feats, k=12)
    assert torch.equal(ei, pi) and torch.equal(ev, pv)
    approx, bound = wd_prefilter_debug(m, users, feats)
    exact = m.predict_all_items(users, feats)
    assert ((approx - exact).abs() <= bound).all()
    # a non-finite weight: the bound is unusable, every row takes the exact kernel
    m2, _ = wd_model(3000, 8192, seed=5, layers=(128, 64, 32), d=32)
    with torch.no_grad():
        m2.deep_item_embedding.weight[17, 3] = float("inf")
    users = torch.arange(0, 40, device=DEV)
    (ev, ei), (pv, pi), stats = topk_both(m2, users)
    assert np.array_equal(ei, pi)
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    assert stats[2] == 40
