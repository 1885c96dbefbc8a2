"""Pin the CPU oracle against the golden fixtures produced by the reference itself.

These run on CPU (no GPU) and prove that `oracle/hnm_oracle.py` restates the reference
arithmetic before it is trusted as the checker for the HIP path.
"""
import numpy as np
import pytest

from parity import (assert_scores_close, assert_topk_equivalent, filter_from_arrays,
                    load_golden)
from oracle import hnm_oracle as O
from hnm_recommendation_amd import synthetic as syn


def test_ncf_small_matches_reference():
    g = load_golden("ncf_small.npz")
    dense = O.ncf_predict_all_items(g["sd"], g["user_ids"])
    assert_scores_close(dense, g["dense"], "ncf dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    assert_topk_equivalent(O.recommend(dense, g["user_ids"], int(g["K"])), g["dense"], int(g["K"]))
    f = filter_from_arrays(g["filter_keys"], g["filter_ptr"], g["filter_idx"])
    masked = O.apply_filter(dense, g["user_ids"], f)
    assert_topk_equivalent(g["topk_filtered"], masked, int(g["K"]))
    pair = O.ncf_forward(g["sd"], g["pair_users"], g["pair_items"])
    assert_scores_close(pair, g["pair_scores"], "ncf pair")


@pytest.mark.parametrize("name", ["ncf_deep_d4.npz", "ncf_deep_d2.npz", "ncf_deep_wide.npz"])
def test_ncf_deep_towers_match_reference(name):
    """NeuralCF towers of other depths (neural_cf.py:75-90): [128,64,32,16], [64,32] (mf 32),
    [256,128,64] -- the oracle's layer loop against the reference's own outputs."""
    g = load_golden(name)
    dense = O.ncf_predict_all_items(g["sd"], g["user_ids"])
    assert_scores_close(dense, g["dense"], name)
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    f = filter_from_arrays(g["filter_keys"], g["filter_ptr"], g["filter_idx"])
    assert_topk_equivalent(g["topk_filtered"], O.apply_filter(dense, g["user_ids"], f), int(g["K"]))
    pair = O.ncf_forward(g["sd"], g["pair_users"], g["pair_items"])
    assert_scores_close(pair, g["pair_scores"], name + " pair")


def test_ncf_config1_matches_reference():
    """BASELINE configs[0]: 10k users x 5k items, weights regenerated from seed 0."""
    g = load_golden("ncf_config1.npz")
    sd = syn.ncf_state_dict(int(g["U"]), int(g["I"]), 64, (128, 64, 32), seed=int(g["seed"]))
    users = g["user_ids"][:64]
    dense = O.ncf_predict_all_items(sd, users)
    assert_topk_equivalent(g["topk"][:64], dense, 12)
    np.testing.assert_allclose(dense.astype(np.float64).sum(1), g["row_sums"][:64], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ["lightgcn_d64.npz", "lightgcn_d128.npz", "lightgcn_d64_alpha.npz"])
def test_lightgcn_matches_reference(name):
    g = load_golden(name)
    U, I = int(g["U"]), int(g["I"])
    alpha = None if float(g["alpha"]) < 0 else float(g["alpha"])
    np.testing.assert_allclose(O.lightgcn_alphas(3, alpha), g["alphas"], rtol=1e-12)
    graph = O.lightgcn_set_graph(g["edge_index"], g.get("edge_weight"), U + I)
    fu, fi = O.lightgcn_forward(g["sd"]["embeddings.weight"], graph, U, 3, alpha)
    assert_scores_close(fu, g["F_U"], "F_U")
    assert_scores_close(fi, g["F_I"], "F_I")
    dense = O.lightgcn_predict_all_items(fu, fi, g["user_ids"])
    assert_scores_close(dense, g["dense"], "lightgcn dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    f = filter_from_arrays(g["filter_keys"], g["filter_ptr"], g["filter_idx"])
    assert_topk_equivalent(g["topk_filtered"], O.apply_filter(dense, g["user_ids"], f), int(g["K"]))


def test_widedeep_matches_reference():
    g = load_golden("widedeep_small.npz")
    dense = O.widedeep_predict_all_items(g["sd"], g["user_ids"])
    assert_scores_close(dense, g["dense"], "wd dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    f = filter_from_arrays(g["filter_keys"], g["filter_ptr"], g["filter_idx"])
    assert_topk_equivalent(g["topk_filtered"], O.apply_filter(dense, g["user_ids"], f), int(g["K"]))
    pair = O.widedeep_forward(g["sd"], g["pair_users"], g["pair_items"])
    assert_scores_close(pair, g["pair_scores"], "wd pair")


def test_widedeep_user_features_match_reference():
    g = load_golden("widedeep_feat.npz")
    dense = O.widedeep_predict_all_items(g["sd"], g["user_ids"], g["user_features"])
    assert_scores_close(dense, g["dense"], "wd feat dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))


def test_mf_matches_reference():
    g = load_golden("mf_small.npz")
    dense = O.mf_predict_all_items(g["sd"], g["user_ids"])
    assert_scores_close(dense, g["dense"], "mf dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    f = filter_from_arrays(g["filter_keys"], g["filter_ptr"], g["filter_idx"])
    assert_topk_equivalent(g["topk_filtered"], O.apply_filter(dense, g["user_ids"], f), int(g["K"]))


def test_oracle_topk_tie_order_is_index_ascending():
    s = np.array([[1.0, 3.0, 3.0, 2.0, 3.0, -np.inf]], np.float32)
    v, i = O.topk(s, 4)
    assert i.tolist() == [[1, 2, 4, 3]]
    m = O.apply_filter(s, [7], {7: {1, 2, 4, 3, 0}})
    assert O.topk(m, 2)[1].tolist() == [[0, 1]]  # all -inf: lowest indices first


def _lists(keys, ptr, idx):
    return {int(k): idx[ptr[j]:ptr[j + 1]].tolist() for j, k in enumerate(keys)}


def test_metrics_match_reference():
    """metrics.py (evaluate_recommendations + the four Metric classes) on the fixture."""
    g = load_golden("metrics_small.npz")
    k = int(g["k"])
    preds = _lists(g["pred_keys"], g["pred_ptr"], g["pred_idx"])
    truth = _lists(g["truth_keys"], g["truth_ptr"], g["truth_idx"])
    agg, per = O.evaluate_recommendations(preds, truth, k)
    assert np.array_equal(per, g["per_user"])  # bitwise: same float64 ops, same order
    np.testing.assert_allclose([agg[f"map@{k}"], agg[f"recall@{k}"], agg[f"precision@{k}"],
                                agg[f"ndcg@{k}"]], g["agg"], rtol=1e-13)
    with pytest.raises(ZeroDivisionError):
        O.evaluate_recommendations({0: [1]}, {0: []}, k)
    means, rows = O.metric_classes(g["scores"], g["target"], g["mask"], k)
    for j, name in enumerate(("map", "recall", "precision", "ndcg")):
        # the reference accumulates in float32 tensors (metrics.py:16): 1e-6 relative
        np.testing.assert_allclose(means[name], g[f"cls_{name}"], rtol=2e-6)
        np.testing.assert_array_equal(rows[:, j].astype(np.float32),
                                      g[f"cls_{name}_rows"].astype(np.float32))


# ------------------------------------------------------------------ full catalogue
# I = 105,542 fixtures (tests/golden/make_golden.py `full`): the oracle reproduces the
# reference's stored top-K on a few users (the GPU tests check all of them).
from parity import assert_topk_matches_reference  # noqa: E402


def _rows(g, n, prefix=""):
    keys = ("topk", "topk_scores", "kth", "kth_gap", "row_absmax")
    return {prefix + k: g[prefix + k][:n] for k in keys}


@pytest.mark.parametrize("name", ["ncf_full.npz", "ncf_full_personal.npz"])
def test_ncf_full_catalogue_oracle(name):
    g = load_golden(name)
    sd = syn.ncf_state_dict(int(g["U"]), int(g["I"]), 64, (128, 64, 32), seed=int(g["seed"]),
                            bias_scale=float(g["bias_scale"]), emb_scale=float(g["emb_scale"]))
    dense = O.ncf_predict_all_items(sd, g["user_ids"][:4])
    v, i = O.topk(dense, 12)
    assert_topk_matches_reference(i, v, _rows(g, 4), what=name)
    np.testing.assert_allclose(dense[:, ::int(g["slice_step"])], g["dense_slice"][:4], rtol=1e-4,
                               atol=1e-4 * float(np.abs(g["dense_slice"]).max()))


def test_mf_full_catalogue_oracle():
    g = load_golden("mf_full.npz")
    sd = syn.mf_state_dict(int(g["U"]), int(g["I"]), 64, seed=int(g["seed"]),
                           bias_scale=float(g["bias_scale"]))
    v, i = O.topk(O.mf_predict_all_items(sd, g["user_ids"][:16]), 12)
    assert_topk_matches_reference(i, v, _rows(g, 16), what="mf full")


def test_lightgcn_full_catalogue_oracle():
    g = load_golden("lightgcn_full_d64.npz")
    U, I, E = int(g["U"]), int(g["I"]), int(g["E"])
    w = syn.lightgcn_state_dict(U, I, 64, seed=int(g["seed"]))["embeddings.weight"]
    graph = O.lightgcn_set_graph(syn.bipartite_edge_index(U, I, E, seed=int(g["graph_seed"])),
                                 None, U + I)
    fu, fi = O.lightgcn_forward(w, graph, U)
    assert_scores_close(fu[g["user_ids"][:16]], g["F_U_rows"], "F_U rows")
    assert_scores_close(fi[g["F_I_sample_ids"]], g["F_I_rows"], "F_I rows")
    v, i = O.topk(O.lightgcn_predict_all_items(fu, fi, g["user_ids"][:16]), 12)
    assert_topk_matches_reference(i, v, _rows(g, 16), what="lightgcn full")


def test_widedeep_item_features_pair_matches_reference():
    g = load_golden("widedeep_itemfeat.npz")
    pair = O.widedeep_forward(g["sd"], g["pair_users"], g["pair_items"], g["user_features"],
                              item_features=g["item_features"])
    assert_scores_close(pair, g["pair_scores"], "wd item-feature pair")


def test_widedeep_no_wide_user_item_matches_reference():
    g = load_golden("widedeep_nowide.npz")
    dense = O.widedeep_predict_all_items(g["sd"], g["user_ids"])
    assert_scores_close(dense, g["dense"], "wd no-wide dense")
    assert_topk_equivalent(g["topk"], dense, int(g["K"]))
    pair = O.widedeep_forward(g["sd"], g["pair_users"], g["pair_items"])
    assert_scores_close(pair, g["pair_scores"], "wd no-wide pair")
