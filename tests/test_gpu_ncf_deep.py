"""GPU: NeuralCF towers other than the fused two-layer one (neural_cf.py:75-90 `_build_mlp`,
scored as neural_cf.py:131-141 and ranked as neural_cf.py:300-326).

* The fp32-MFMA tile kernel (ncf_deep.hip `ncf_deep_mfma_kernel`, widths <= 64) scores bitwise
  what the per-pair LDS kernel scores (HNM_OPT_DEEP_MFMA = 0): the f32 MFMA is the fmaf chain.
* Its fused top-k (hnm_ncf_deep_topk_f32, per-partition wave lists + merge) equals the
  (score desc, item asc) order of those dense rows exactly, filtered and unfiltered, at both
  users-per-wave variants and on towers with one and two 32-unit tiles, odd widths, a single
  Linear, mf not a multiple of 8 and 7 layers; the wide-tower route (dense chunk + row top-k
  inside the library) gives the same lists; item shards (sharding.ncf_deep_shard_topk) merge to
  the unsharded lists.
* Rows against the CPU oracle (oracle/hnm_oracle.py ncf_predict_all_items) within the fp32
  tolerance of tests/parity.py: every row at B = 37, every 4th at B = 300, 17 full-catalogue rows.
"""
import numpy as np
import pytest
import torch

from oracle import hnm_oracle as O
from parity import assert_scores_close
from hnm_recommendation_amd import NeuralCF, _lib
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"

TOWERS = [  # (mf, mlp_dims)
    (64, (128, 64, 32, 16)),          # one 32-unit MFMA tile a layer
    (32, (64, 32)),                   # a single Linear: no MFMA layer
    (20, (96, 48, 40, 24, 12)),       # odd widths; mf padded to 24
    (64, (128, 64, 64, 8)),           # a 64-wide MFMA layer (two tiles)
    (128, (64, 32, 16, 8, 4, 2, 1)),  # 6 Linear layers, mf 128
]


def model(U, I, mf, dims, seed):
    sd = syn.ncf_state_dict(U, I, mf, dims, seed=seed, bias_scale=0.05, emb_scale=8.0)
    m = NeuralCF(U, I, mf_dim=mf, mlp_dims=list(dims))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval(), sd


def per_pair(fn):
    """Run fn with the per-pair LDS kernel (and the dense-chunk top-k) forced."""
    _lib.set_option(DEV, _lib.HNM_OPT_DEEP_MFMA, 0)
    try:
        return fn()
    finally:
        _lib.set_option(DEV, _lib.HNM_OPT_DEEP_MFMA, 1)


def topk_order(scores, k):
    """(score desc, item asc) per row -- the library's total order."""
    idx = np.empty((scores.shape[0], k), np.int64)
    items = np.arange(scores.shape[1])
    for b in range(scores.shape[0]):
        idx[b] = np.lexsort((items, -scores[b].astype(np.float64)))[:k]
    return idx, np.take_along_axis(scores, idx, 1)


@pytest.mark.parametrize("mf,dims", TOWERS)
@pytest.mark.parametrize("B", [37, 300])
def test_deep_mfma_bitwise_and_fused_topk(mf, dims, B):
    U, I, K = 700, 3001, 12
    m, sd = model(U, I, mf, dims, seed=len(dims) + mf)
    assert not m._fused()
    users_np = syn.user_batch(U, B, seed=B)
    users = torch.from_numpy(users_np).to(DEV)
    fast = m.predict_all_items(users)
    slow = per_pair(lambda: m.predict_all_items(users))
    assert torch.equal(fast.view(torch.int32), slow.view(torch.int32)), "MFMA vs per-pair"
    dense = fast.cpu().numpy()
    # every row (B = 37) / every 4th row and the last (B = 300) against the oracle
    rows = list(range(B)) if B <= 64 else list(range(0, B, 4)) + [B - 1]
    assert_scores_close(dense[rows], O.ncf_predict_all_items(sd, users_np[rows]), "deep oracle")

    ref_i, ref_v = topk_order(dense, K)
    v, i = m.recommend_with_scores(users, k=K)
    np.testing.assert_array_equal(i.cpu().numpy(), ref_i)
    np.testing.assert_array_equal(v.cpu().numpy().view(np.int32), ref_v.view(np.int32))
    v2, i2 = per_pair(lambda: m.recommend_with_scores(users, k=K))
    assert torch.equal(i2, i) and torch.equal(v2.view(torch.int32), v.view(torch.int32))

    # history filter: each row's current top-3 plus random items, every 3rd row
    rng = np.random.default_rng(B)
    filt = {}
    for b in range(0, B, 3):
        u = int(users_np[b])
        filt.setdefault(u, set()).update(int(x) for x in ref_i[b, :3])
        filt[u].update(int(x) for x in rng.integers(0, I, 40))
    masked = dense.copy()
    for b in range(B):
        for it in filt.get(int(users_np[b]), ()):
            masked[b, it] = -np.inf
    ref_i, ref_v = topk_order(masked, K)
    v, i = m.recommend_with_scores(users, filter_items=filt, k=K)
    np.testing.assert_array_equal(i.cpu().numpy(), ref_i)
    np.testing.assert_array_equal(v.cpu().numpy(), ref_v)
    # k = 64, the fused path's maximum
    ref_i, _ = topk_order(dense, 64)
    np.testing.assert_array_equal(m.recommend_with_scores(users, k=64)[1].cpu().numpy(), ref_i)


def exact(fn):
    """Run fn with the certified pre-filter off (the exact deep kernels everywhere)."""
    _lib.set_prefilter(DEV, False)
    try:
        return fn()
    finally:
        _lib.set_prefilter(DEV, True)


def test_deep_mfma_full_catalogue_topk():
    """[128,64,32,16] over the full H&M catalogue (105,542 items, many partitions) at B = 512:
    the fused exact top-12 (pre-filter off) equals the per-pair route's lists bitwise, and so does
    the default (certified, round 6) call; oracle rows agree."""
    U, I = 3000, syn.HM_ITEMS
    m, sd = model(U, I, 64, (128, 64, 32, 16), seed=21)
    users_np = syn.user_batch(U, 512, seed=4)
    users = torch.from_numpy(users_np).to(DEV)
    v, i = exact(lambda: m.recommend_with_scores(users))
    v2, i2 = exact(lambda: per_pair(lambda: m.recommend_with_scores(users)))
    assert torch.equal(i, i2) and torch.equal(v.view(torch.int32), v2.view(torch.int32))
    v3, i3 = m.recommend_with_scores(users)
    assert torch.equal(i, i3) and torch.equal(v.view(torch.int32), v3.view(torch.int32))
    rows = list(range(0, 512, 32)) + [511]  # 17 rows x 105,542 items
    ref = O.ncf_predict_all_items(sd, users_np[rows])
    got = m.predict_all_items(users[rows]).cpu().numpy()
    assert_scores_close(got, ref, "deep full-catalogue rows")


def test_deep_item_shards_merge_to_the_unsharded_topk():
    """Item-sharded deep towers (sharding.ncf_shard_topk -> ncf_deep_shard_topk on shard tables,
    ragged shards, with the history filter): the shards' lists merged by hnm_topk_merge_f32 are
    bitwise the unsharded fused top-k."""
    from hnm_recommendation_amd import sharding as S
    from hnm_recommendation_amd import UserHistory
    U, I, K, B = 900, 7001, 12, 260
    m, _ = model(U, I, 64, (128, 64, 32, 16), seed=8)
    users_np = syn.user_batch(U, B, seed=5)
    users = torch.from_numpy(users_np).to(DEV)
    rng = np.random.default_rng(2)
    filt = {int(u): set(int(x) for x in rng.integers(0, I, 30)) for u in users_np[::4]}
    hist = UserHistory(filt, U, I, torch.device(DEV))
    for f, h in ((None, None), (filt, hist)):
        full_v, full_i = m.recommend_with_scores(users, filter_items=f, k=K)
        vs, is_ = [], []
        for r in range(3):
            lo, hi = S.shard_range(I, r, 3)
            sc = S.ncf_shard_topk(m, lo, hi, K, history=h)
            assert isinstance(sc, S.ncf_deep_shard_topk)
            v, i = sc(users)
            vs.append(v)
            is_.append(torch.where(i >= 0, i + lo, i))
        mv, mi = S.hip_merge(torch.stack(vs).contiguous(), torch.stack(is_).contiguous(), K)
        assert torch.equal(mi, full_i)
        assert torch.equal(mv.view(torch.int32), full_v.view(torch.int32))



# ------------------------------------------------------------------ certified deep pre-filter
# Round 6: three-layer towers take the two-layer tower's certified f16 scan with a
# third layer on the matrix pipe and a worst-case bound carried through |wp3|^T |W3| |W2|
# (ncf_cert.hip); survivors are re-scored by the exact deep chain.  The bound must hold pair by
# pair over the full catalogue, and the top-k must be bitwise the exact path's, for weights unlike
# the init too (synthetic.stress_state_dict) -- and rows the bound cannot serve must come back
# exact through both fallback routes.
DEEP_DIMS = (128, 64, 32, 16)
DEEP_WEIGHTS = ["init", "personal", "norms", "student_t"]


def deep_weights_model(U, I, kind, seed=3):
    kw = ({} if kind == "init" else dict(bias_scale=0.05, emb_scale=20.0) if kind == "personal"
          else dict(bias_scale=0.05))
    sd = syn.ncf_state_dict(U, I, 64, DEEP_DIMS, seed=seed, **kw)
    if kind not in ("init", "personal"):
        sd = syn.stress_state_dict(sd, kind, syn.NCF_EMB_KEYS, "mlp_item_embedding.weight")
    m = NeuralCF(U, I, mf_dim=64, mlp_dims=list(DEEP_DIMS))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval()


def deep_debug(m, users):
    import ctypes as C
    w, keep = m._deep_weights()
    I = m.num_items
    approx = torch.empty(users.numel(), I, device=DEV)
    bound = torch.empty_like(approx)
    _lib.check(_lib.fn("hnm_ncf_deep_prefilter_debug_f32")(
        _lib.ctx(users.device), C.byref(w), _lib.ptr(users), users.numel(), _lib.ptr(approx), I,
        _lib.ptr(bound)), "hnm_ncf_deep_prefilter_debug_f32")
    return approx, bound


@pytest.mark.parametrize("kind", DEEP_WEIGHTS)
def test_deep_bound_holds_full_catalogue(kind):
    U, I = 4000, syn.HM_ITEMS
    m = deep_weights_model(U, I, kind)
    users = torch.from_numpy(syn.user_batch(U, 16, seed=9)).to(DEV)
    approx, bound = deep_debug(m, users)
    ex = m.predict_all_items(users)
    bp = float(m.prediction_layer.bias.detach())
    err = (approx + bp - ex).abs()
    ratio = (err / bound).max().item()
    spread = ex.std(1, keepdim=True)
    print(f"deep bound [{kind}]: max |approx - exact| / bound {ratio:.4f}, "
          f"mean bound / score std {(bound / spread).mean().item():.4f}")
    assert torch.isfinite(bound).all()
    assert (err <= bound).all(), ratio


@pytest.mark.parametrize("kind", DEEP_WEIGHTS)
def test_deep_certified_topk_bitwise(kind):
    U, I, B = 6000, syn.HM_ITEMS, 700
    m = deep_weights_model(U, I, kind, seed=5)
    users_np = syn.user_batch(U, B, seed=11)
    users = torch.from_numpy(users_np).to(DEV)
    ks = (12, 64) if kind == "init" else (12,)
    for k in ks:
        _lib.prefilter_stats(DEV, reset=True)
        _lib.set_option(DEV, _lib.HNM_OPT_STATS, 1)
        v, i = m.recommend_with_scores(users, k=k)
        _lib.set_option(DEV, _lib.HNM_OPT_STATS, 0)
        rows, cands, fb = _lib.prefilter_stats(DEV, reset=True)
        ev, ei = exact(lambda: m.recommend_with_scores(users, k=k))
        print(f"deep certified [{kind}, k={k}]: {cands / max(rows - fb, 1):.1f} candidates a row, "
              f"{fb} fallback rows of {rows}")
        assert rows == B
        assert torch.equal(i, ei), kind
        assert torch.equal(v.view(torch.int32), ev.view(torch.int32)), kind
    if kind == "init":  # the history filter (every 3rd row: its top-3 and 40 random items)
        rng = np.random.default_rng(1)
        filt = {}
        top = ei.cpu().numpy()
        for b in range(0, B, 3):
            u = int(users_np[b])
            filt.setdefault(u, set()).update(int(x) for x in top[b, :3])
            filt[u].update(int(x) for x in rng.integers(0, I, 40))
        v, i = m.recommend_with_scores(users, filter_items=filt, k=12)
        ev, ei = exact(lambda: m.recommend_with_scores(users, filter_items=filt, k=12))
        assert torch.equal(i, ei) and torch.equal(v.view(torch.int32), ev.view(torch.int32))


@pytest.mark.parametrize("B", [16, 40])
def test_deep_certified_fallback_rows(B):
    """One item row at 1e13 makes the bound unusable (maxima above the 2^40 guard): every row is
    queued for the exact scan -- B = 16 through one exact call per row, B = 40 through the whole
    batch exactly with the queued rows' lists copied over -- and the lists equal the exact path's."""
    U, I = 3000, syn.HM_ITEMS
    m = deep_weights_model(U, I, "huge", seed=7)
    users = torch.from_numpy(syn.user_batch(U, B, seed=B)).to(DEV)
    _lib.prefilter_stats(DEV, reset=True)
    _lib.set_option(DEV, _lib.HNM_OPT_STATS, 1)
    v, i = m.recommend_with_scores(users)
    _lib.set_option(DEV, _lib.HNM_OPT_STATS, 0)
    rows, cands, fb = _lib.prefilter_stats(DEV, reset=True)
    assert fb == B, (rows, fb)
    ev, ei = exact(lambda: m.recommend_with_scores(users))
    assert torch.equal(i, ei) and torch.equal(v.view(torch.int32), ev.view(torch.int32))
