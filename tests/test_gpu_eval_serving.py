"""GPU parity of the top-K consumers: the metrics kernel
(`hnm_rank_metrics_f64`) against the reference's own metrics.py outputs (golden fixture)
and the oracle, and the batched serving path against the oracle's per-user serve loop.

Bars: per-user metric values bitwise equal to the reference's float64 loop (same
formulas, same order, numpy's own 1/log2 terms); means within 1e-13 relative (the
reference averages with np.mean's pairwise sum, we with a fixed-order device tree; the
torchmetrics classes accumulate in float32: 2e-6).  Serving: top-K sets per the scoring
bar (parity.assert_topk_equivalent), scores within 1e-4 relative.
"""
import numpy as np
import pytest
import torch

from parity import assert_scores_close, assert_topk_equivalent, load_golden
from oracle import hnm_oracle as O
from hnm_recommendation_amd import NeuralCF, MatrixFactorization
from hnm_recommendation_amd import evaluation as EV
from hnm_recommendation_amd import synthetic as syn
from hnm_recommendation_amd.serving import Recommender, create_model_from_checkpoint

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lists(keys, ptr, idx):
    return {int(k): idx[ptr[j]:ptr[j + 1]].tolist() for j, k in enumerate(keys)}


def test_evaluate_recommendations_golden():
    g = load_golden("metrics_small.npz")
    k = int(g["k"])
    preds = _lists(g["pred_keys"], g["pred_ptr"], g["pred_idx"])
    truth = _lists(g["truth_keys"], g["truth_ptr"], g["truth_idx"])
    res, per = EV.evaluate_recommendations(preds, truth, k, device=DEV, per_user=True)
    assert np.array_equal(per.cpu().numpy(), g["per_user"])  # bitwise per user
    got = [res[f"map@{k}"], res[f"recall@{k}"], res[f"precision@{k}"], res[f"ndcg@{k}"]]
    np.testing.assert_allclose(got, g["agg"], rtol=1e-13)
    with pytest.raises(ZeroDivisionError):
        EV.evaluate_recommendations({0: [1]}, {0: []}, k, device=DEV)


def test_metric_classes_golden():
    g = load_golden("metrics_small.npz")
    k = int(g["k"])
    s, tg, mk = (torch.from_numpy(g[n]).to(DEV) for n in ("scores", "target", "mask"))
    for name, C in (("map", EV.MeanAveragePrecision), ("recall", EV.RecallAtK),
                    ("precision", EV.PrecisionAtK), ("ndcg", EV.NDCGAtK)):
        m = C(k=k)
        m.update(s[:50], tg[:50], mk[:50])  # two updates accumulate like one
        m.update(s[50:], tg[50:], mk[50:])
        np.testing.assert_allclose(float(m.compute()), g[f"cls_{name}"], rtol=2e-6)
        for b in (0, 3, 17):
            m1 = C(k=k)
            m1.update(s[b:b + 1], tg[b:b + 1], mk[b:b + 1])
            assert np.float32(m1.compute()) == np.float32(g[f"cls_{name}_rows"][b])


@pytest.mark.parametrize("k", [1, 12, 100, 128])
def test_rank_metrics_vs_oracle(k):
    """Random lists: long truth rows (> 64, several chunks), repeats in predictions,
    predictions longer than k, empty truth rows, dense truth with a mask."""
    rng = np.random.Generator(np.random.PCG64(100 + k))
    B, I = 700, 500
    L = k + 7
    pred = rng.integers(0, I, (B, L)).astype(np.int64)
    lens = rng.integers(0, 300, B)
    lens[:5] = 0
    truth = [np.unique(rng.integers(0, I, n)) for n in lens]
    ptr = np.concatenate([[0], np.cumsum([t.size for t in truth])]).astype(np.int64)
    idx = np.concatenate(truth).astype(np.int64)
    per, nt, sums = EV.rank_metrics(torch.from_numpy(pred).to(DEV), k,
                                    truth_ptr=torch.from_numpy(ptr).to(DEV),
                                    truth_idx=torch.from_numpy(idx).to(DEV))
    ref = np.asarray([O.user_metrics(pred[b].tolist(), set(truth[b].tolist()), k)
                      for b in range(B)])
    assert np.array_equal(per.cpu().numpy(), ref)
    assert np.array_equal(nt.cpu().numpy(), np.asarray([t.size for t in truth]))
    s = sums.cpu().numpy()
    np.testing.assert_allclose(s[:4], ref.sum(0), rtol=1e-12)
    has = lens > 0
    np.testing.assert_allclose(s[4:8], ref[has].sum(0), rtol=1e-12)
    assert s[8] == has.sum()

    # dense truth + mask (torchmetrics layout), duplicates counted in n_true
    T = 90
    dense = rng.integers(0, I, (B, T)).astype(np.int64)
    mask = rng.random((B, T)) < 0.4
    per2, nt2, _ = EV.rank_metrics(torch.from_numpy(pred).to(DEV), k,
                                   truth=torch.from_numpy(dense).to(DEV),
                                   truth_mask=torch.from_numpy(mask).to(DEV))
    p2 = per2.cpu().numpy()
    for b in range(0, B, 7):
        tb = dense[b][mask[b]]
        n = len(tb)
        ts = set(tb.tolist())
        pr = pred[b][:k].tolist()
        hits = [p in ts for p in pr]
        ap, nh, dcg = 0.0, 0.0, 0.0
        for i, h in enumerate(hits):
            if h:
                nh += 1.0
                ap += nh / (i + 1.0)
                dcg += 1.0 / np.log2(i + 2)
        idcg = sum(1.0 / np.log2(i + 2) for i in range(min(n, k)))
        exp = (ap / min(n, k) if n else 0.0, nh / n if n else 0.0, nh / len(pr),
               dcg / idcg if idcg > 0 else 0.0)
        assert tuple(p2[b]) == exp, b
        assert int(nt2[b]) == n


def _ncf_model():
    g = load_golden("ncf_small.npz")
    m = NeuralCF(int(g["U"]), int(g["I"]), top_k=int(g["K"]))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in g["sd"].items()})
    return g, m.to(DEV).eval()


def test_evaluate_model_matches_oracle():
    """Offline evaluation: fused top-K -> metrics on the device vs oracle top-K + metrics."""
    g, m = _ncf_model()
    U = int(g["U"])
    users = np.arange(U, dtype=np.int64)
    rng = np.random.Generator(np.random.PCG64(5))
    truth = {u: set(rng.integers(0, int(g["I"]), int(rng.integers(1, 30))).tolist())
             for u in range(U)}
    dense = O.ncf_predict_all_items(g["sd"], users)
    _, top = O.topk(dense, 12)
    ref, _ = O.evaluate_recommendations({u: top[u].tolist() for u in range(U)}, truth, 12)
    tp, ti = EV.truth_csr(users.tolist(), truth, DEV)
    got = EV.evaluate_model(m, torch.from_numpy(users), tp, ti, k=12, batch_size=256)
    for key in ref:
        np.testing.assert_allclose(got[key], ref[key], rtol=1e-9)


def test_serving_batch_matches_oracle():
    g, m = _ncf_model()
    U, I = int(g["U"]), int(g["I"])
    hist = syn.filter_dict(np.arange(U), I, per_user=23, seed=3)
    srv = Recommender(U, I, models={"neural_cf": m}, user_history=hist,
                      model_metrics={"neural_cf": {"test_map": 0.1}}, device=DEV)
    ids = [5, 17, U + 3, 17, 0, U - 1, "not-a-customer"]
    for n_items, scores in ((12, True), (100, True), (7, False)):
        out = srv.get_batch_recommendations(ids, num_items=n_items, include_scores=scores)
        assert [r["user_id"] for r in out] == ids
        assert "error" in out[2] and "error" in out[6]
        good = [j for j in range(len(ids)) if "error" not in out[j]]
        uidx = np.asarray([ids[j] for j in good], np.int64)
        dense = O.ncf_predict_all_items(g["sd"], uidx)
        masked = O.apply_filter(dense, uidx, hist)  # serve.py:350-352
        got = np.asarray([[int(r["article_id"]) for r in out[j]["recommendations"]]
                          for j in good])
        assert_topk_equivalent(got, masked, n_items, what=f"serve batch k={n_items}")
        if scores:
            sv = np.asarray([[r["score"] for r in out[j]["recommendations"]] for j in good])
            assert_scores_close(sv, np.take_along_axis(masked, got, 1), "serve scores")
        else:
            assert all(r["score"] is None for j in good for r in out[j]["recommendations"])
        assert all(out[j]["model_name"] == "neural_cf" for j in good)
    one = srv.get_recommendations(5, num_items=12, filter_purchased=False)
    dense = O.ncf_predict_all_items(g["sd"], np.asarray([5]))
    assert_topk_equivalent(np.asarray([[int(r["article_id"]) for r in one["recommendations"]]]),
                           dense, 12, what="serve single unfiltered")
    with pytest.raises(ValueError):
        srv.get_recommendations(U + 1)
    with pytest.raises(ValueError):
        srv.get_recommendations(1, model_name="lightgcn")


def test_checkpoint_ingestion_roundtrip(tmp_path):
    """A Lightning-style .ckpt (state_dict + hyper_parameters) -> module on the GPU,
    dispatched by directory name; recommendations equal the source module's."""
    U, I = 500, 300
    sd = syn.mf_state_dict(U, I, 64, seed=0, bias_scale=0.05)
    src = MatrixFactorization(num_users=U, num_items=I, embedding_dim=64, top_k=12)
    src.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    d = tmp_path / "matrix_factorization_v1"
    d.mkdir()
    torch.save({"state_dict": src.state_dict(), "hyper_parameters": dict(src.hparams),
                "metrics": {"test_map": 0.2}}, d / "best.ckpt")
    srv = Recommender(U, I, device=DEV)
    assert srv.load_checkpoints(str(tmp_path)) == ["matrix_factorization_v1"]
    users = torch.arange(0, 64, device=DEV)
    got = srv.models["matrix_factorization_v1"].recommend(users).cpu().numpy()
    dense = O.mf_predict_all_items(sd, np.arange(64))
    assert_topk_equivalent(got, dense, 12, what="ckpt mf")
    assert create_model_from_checkpoint("unknown_model", {"state_dict": {}}, U, I, DEV) is None


def test_recommendation_metrics_formulas():
    from hnm_recommendation_amd import RecommendationMetrics
    m = RecommendationMetrics(top_k=3)
    m.update(torch.tensor([[1, 2, 3], [4, 5, 6]], device=DEV), [[2, 9], [7]])
    r = m.compute()
    # user 0: hit at rank 2 -> AP = (1/2)/min(2,3) = 0.25; user 1: 0
    assert abs(float(r["map_at_k"]) - 0.125) < 1e-12
    assert abs(float(r["recall_at_k"]) - 0.25) < 1e-12
    assert abs(float(r["precision_at_k"]) - (1 / 3) / 2) < 1e-12
    idcg = 1 + 1 / np.log2(3)
    assert abs(float(r["ndcg_at_k"]) - (1 / np.log2(3)) / idcg / 2) < 1e-12


def test_lightning_checkpoint_fixture_serves_on_gpu():
    """The committed Lightning-2.x-shaped .ckpt fixtures (tests/golden/lightning/) loaded by
    Recommender.load_checkpoints onto the GPU serve the same top-K as the oracle run on
    the checkpoint's own state_dict (NeuralCF and LightGCN with its graph)."""
    import os
    from hnm_recommendation_amd.serving import load_checkpoint
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lightning")
    U, I = 60, 40
    ei = syn.bipartite_edge_index(U, I, 300, seed=23)
    srv = Recommender(U, I, device=DEV)
    assert srv.load_checkpoints(root, graph=(torch.from_numpy(ei), None)) == ["lightgcn", "neural_cf"]
    users = np.arange(0, 50)
    sd = {k: v.numpy() for k, v in load_checkpoint(
        os.path.join(root, "neural_cf", "epoch=3-step=1200.ckpt"))["state_dict"].items()}
    got = srv.models["neural_cf"].recommend(torch.from_numpy(users).to(DEV)).cpu().numpy()
    assert_topk_equivalent(got, O.ncf_predict_all_items(sd, users), 12, what="ckpt ncf")
    lsd = load_checkpoint(os.path.join(root, "lightgcn", "epoch=3-step=1200.ckpt"))["state_dict"]
    fu, fi = O.lightgcn_forward(lsd["embeddings.weight"].numpy(),
                                O.lightgcn_set_graph(ei, None, U + I), U, 3)
    got = srv.models["lightgcn"].recommend(torch.from_numpy(users).to(DEV)).cpu().numpy()
    assert_topk_equivalent(got, O.lightgcn_predict_all_items(fu, fi, users), 12, what="ckpt lgcn")
    one = srv.get_recommendations(3, model_name="neural_cf", num_items=5, include_scores=True)
    assert len(one["recommendations"]) == 5
    with pytest.raises(ValueError):
        srv.get_recommendations(3, model_name="neural_cf", num_items=101)  # serve.py:56 le=100


def _hook_model(name):
    """(module, golden) for the Lightning-hook test, built like the golden tests build them."""
    from hnm_recommendation_amd import LightGCN, WideDeep
    if name == "ncf":
        g = load_golden("ncf_small.npz")
        m = NeuralCF(int(g["U"]), int(g["I"]), top_k=int(g["K"]))
    elif name == "mf":
        g = load_golden("mf_small.npz")
        m = MatrixFactorization(int(g["U"]), int(g["I"]), top_k=int(g["K"]), sparse=False)
    elif name == "lightgcn":
        g = load_golden("lightgcn_d64.npz")
        m = LightGCN(int(g["U"]), int(g["I"]), embedding_dim=int(g["d"]), num_layers=3,
                     top_k=int(g["K"]))
        m.set_graph(torch.from_numpy(g["edge_index"]))
    elif name == "widedeep_feat":
        g = load_golden("widedeep_feat.npz")
        m = WideDeep(int(g["U"]), int(g["I"]), num_user_features=int(g["F"]), embedding_dim=16,
                     deep_layers=[64, 32], top_k=int(g["K"]))
    else:
        g = load_golden("widedeep_small.npz")
        m = WideDeep(int(g["U"]), int(g["I"]), embedding_dim=64, deep_layers=[512, 256, 128],
                     top_k=int(g["K"]))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in g["sd"].items()})
    return m.to(DEV).eval(), g


@pytest.mark.parametrize("name", ["ncf", "mf", "lightgcn", "widedeep", "widedeep_feat"])
def test_lightning_eval_hooks(name):
    """validation_step / on_validation_epoch_end / test_step / on_test_epoch_end on the four
    mirrors (neural_cf.py:235-272, lightgcn.py:267-294, wide_deep.py:314-342,
    matrix_factorization.py:158-185) over {'user_ids', 'ground_truth'} batches (truth padded
    with -1, some users with none): the logged val_* / test_* values equal the reference's
    formulas (oracle.user_metrics, float64) over the module's top-K -- itself checked against
    the REFERENCE's own dense scores (golden) -- MAP and Precision over every row, Recall and
    NDCG over rows with truth."""
    m, g = _hook_model(name)
    K, I = int(g["K"]), int(g["I"])
    users = np.asarray(g["user_ids"])
    rng = np.random.Generator(np.random.PCG64(7))
    T = 20
    truth = np.full((len(users), T), -1, np.int64)
    for r in range(len(users)):
        n = int(rng.integers(0, T + 1)) if r % 5 else 0
        truth[r, :n] = rng.integers(0, I, n)
    # half the truth rows hold an item of the reference's own top-K, so hits are frequent
    ref_top = O.topk(g["dense"], K)[1]
    truth[1::2, 0] = ref_top[1::2, 3]
    feats = g["user_features"] if "user_features" in g else None
    halves = [slice(0, len(users) // 2), slice(len(users) // 2, len(users))]
    for hook, end, prefix in ((m.validation_step, m.on_validation_epoch_end, "val"),
                              (m.test_step, m.on_test_epoch_end, "test")):
        for j, sl in enumerate(halves):
            batch = {"user_ids": torch.from_numpy(users[sl]).to(DEV),
                     "ground_truth": torch.from_numpy(truth[sl]).to(DEV)}
            if feats is not None:
                batch["user_features"] = torch.from_numpy(feats[sl]).to(DEV)
            hook(batch, j)
        end()
        got = {k: float(m.logged_metrics[f"{prefix}_{k}"])
               for k in ("map_at_k", "recall_at_k", "precision_at_k", "ndcg_at_k")}
        uid = torch.from_numpy(users).to(DEV)
        ours = (m.recommend(uid) if feats is None else
                m.recommend(uid, torch.from_numpy(feats).to(DEV))).cpu().numpy()
        assert_topk_equivalent(ours, g["dense"], K, what=f"{name} hook top-K")
        rows = [O.user_metrics(ours[r].tolist(), set(int(x) for x in truth[r] if x >= 0), K)
                for r in range(len(users))]
        a = np.asarray(rows)
        has = np.array([(truth[r] >= 0).any() for r in range(len(users))])
        want = {"map_at_k": a[:, 0].mean(), "recall_at_k": a[has, 1].mean(),
                "precision_at_k": a[:, 2].mean(), "ndcg_at_k": a[has, 3].mean()}
        for k in want:
            np.testing.assert_allclose(got[k], want[k], rtol=1e-12, err_msg=f"{name} {prefix} {k}")
        assert got["map_at_k"] > 0
    # metrics were reset at each epoch end
    assert m.metrics._n_all == 0
    if name == "ncf":
        m.top_k = I + 1
        with pytest.raises(RuntimeError):
            m.validation_step({"user_ids": torch.from_numpy(users[:2]).to(DEV),
                               "ground_truth": torch.from_numpy(truth[:2]).to(DEV)}, 0)
