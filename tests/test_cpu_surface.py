"""CPU-side checks (no GPU): library exports, module surface vs the reference, host logic,
error behaviour."""
import os
import re

import numpy as np
import pytest
import torch

from parity import load_golden
from hnm_recommendation_amd import (LightGCN, MatrixFactorization, NeuralCF,
                                    RecommendationMetrics, WideDeep)
from hnm_recommendation_amd import _lib
from hnm_recommendation_amd import synthetic as syn
from hnm_recommendation_amd.models.base import filter_csr

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "hnm.h")).read()
    return sorted(set(re.findall(r"^\s*(?:hnm_status|int|const char\*)\s+(hnm_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.hnm_abi_version() == 1
    # every header symbol has a ctypes signature
    assert set(syms) <= set(_lib.declared_symbols()), set(syms) - set(_lib.declared_symbols())


@pytest.mark.parametrize("cls,golden,kw", [
    (NeuralCF, "ncf_small.npz", {}),
    (LightGCN, "lightgcn_d64.npz", {}),
    (LightGCN, "lightgcn_d128.npz", {"embedding_dim": 128}),
    (MatrixFactorization, "mf_small.npz", {"sparse": False}),
    (WideDeep, "widedeep_small.npz", {}),
    (WideDeep, "widedeep_feat.npz", {"num_user_features": 10, "embedding_dim": 16,
                                      "deep_layers": [64, 32]}),
    (WideDeep, "widedeep_itemfeat.npz", {"num_user_features": 6, "num_item_features": 5,
                                          "embedding_dim": 16, "deep_layers": [64, 32]}),
    (WideDeep, "widedeep_nowide.npz", {"use_wide_user_item": False, "embedding_dim": 32,
                                        "deep_layers": [128, 64]}),
])
def test_state_dict_keys_match_reference(cls, golden, kw):
    g = load_golden(golden)
    m = cls(int(g["U"]), int(g["I"]), **kw)
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ref = {k: tuple(np.asarray(v).shape) for k, v in g["sd"].items()}
    assert ours == ref
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in g["sd"].items()})


def test_hparams_and_signature_mirror_reference():
    m = NeuralCF(num_users=100, num_items=50, mf_dim=32, mlp_dims=[64, 32, 16], top_k=5)
    assert m.hparams["mf_dim"] == 32 and m.hparams["top_k"] == 5
    # reference tests/test_models.py:75 passes embedding_dim to NeuralCF -> TypeError there too
    with pytest.raises(TypeError):
        NeuralCF(num_users=100, num_items=50, embedding_dim=16, top_k=5)
    lg = LightGCN(num_users=100, num_items=50, embedding_dim=16, num_layers=3, top_k=5)
    assert len(lg.alpha) == 4 and abs(sum(lg.alpha) - 1) < 1e-6
    lg2 = LightGCN(100, 50, alpha=0.5)
    np.testing.assert_allclose(lg2.alpha, np.array([1, .5, .25, .125]) / 1.875)


def test_lightgcn_errors_like_reference():
    m = LightGCN(100, 50, embedding_dim=16)
    with pytest.raises(RuntimeError, match="Graph not set"):
        m.forward()
    users = torch.randint(0, 100, (200,))
    items = torch.randint(0, 50, (200,)) + 100
    m.set_graph(torch.stack([torch.cat([users, items]), torch.cat([items, users])]))
    assert m.graph is not None


def test_no_cpu_fallback():
    m = NeuralCF(100, 50)
    with pytest.raises(RuntimeError, match="no CPU path|GPU"):
        m.recommend(torch.tensor([0, 1]))
    with pytest.raises(RuntimeError, match="no CPU path|GPU"):
        m.predict_all_items(torch.tensor([0, 1]))


def test_filter_csr_host_logic():
    ids = torch.tensor([5, 7, 5, 9])
    mptr, midx = filter_csr(ids, {5: {3, 1, 1}, 9: {-1}, 11: {2}}, 10, torch.device("cpu"))
    assert mptr.tolist() == [0, 2, 2, 4, 5]
    assert midx.tolist() == [1, 3, 1, 3, 9]
    assert filter_csr(ids, None, 10, torch.device("cpu")) == (None, None)
    assert filter_csr(ids, {}, 10, torch.device("cpu")) == (None, None)
    with pytest.raises(IndexError):
        filter_csr(ids, {7: {10}}, 10, torch.device("cpu"))


def test_user_history_csr_host_logic():
    """UserHistory's host-side CSR (the device gather itself is a GPU test): per user sorted,
    de-duplicated, negative ids wrapped, users outside [0, U) and empty sets ignored; the
    interaction-array builder gives the same CSR as the dict builder."""
    from hnm_recommendation_amd import UserHistory
    U, I = 6, 10
    h = {1: {3, 1, 1, -1}, 4: {2}, 5: set(), 9: {1}}
    uh = UserHistory(h, U, I, "cpu")
    assert uh.hist_ptr.tolist() == [0, 0, 3, 3, 3, 4, 4]
    assert uh.hist_idx.tolist() == [1, 3, 9, 2]
    assert uh.max_len == 3 and uh.nnz == 4
    u = np.array([1, 1, 1, 1, 4])
    i = np.array([3, 1, 1, 9, 2])
    ui = UserHistory.from_interactions(u, i, U, I, "cpu")
    assert torch.equal(ui.hist_ptr, uh.hist_ptr) and torch.equal(ui.hist_idx, uh.hist_idx)
    with pytest.raises(IndexError):
        UserHistory({0: {10}}, U, I, "cpu")
    with pytest.raises(IndexError):
        UserHistory.from_interactions(np.array([0]), np.array([I]), U, I, "cpu")
    assert UserHistory({}, U, I, "cpu").mask_for(torch.tensor([0])) == (None, None)


# ------------------------------------------------------------------ serving / checkpoints
def test_checkpoint_dispatch_on_cpu(tmp_path):
    """serve.py:216-258: directory-name substring -> class, hparams override, state load
    (module construction and state loading need no GPU; scoring does)."""
    from hnm_recommendation_amd.serving import create_model_from_checkpoint, load_checkpoint
    from hnm_recommendation_amd import synthetic as syn
    U, I = 50, 40
    cases = [("exp1/neural_cf", NeuralCF(U, I)), ("wide_deep_run", WideDeep(U, I)),
             ("matrix_factorization", MatrixFactorization(U, I)),
             ("lightgcn_best", LightGCN(U, I))]
    graph = (torch.from_numpy(syn.bipartite_edge_index(U, I, 200, seed=2)), None)
    for name, src in cases:
        with torch.no_grad():
            for p in src.parameters():
                p.copy_(torch.randn_like(p))
        path = tmp_path / (name.replace("/", "_") + ".ckpt")
        hp = dict(src.hparams)
        hp["num_users"], hp["num_items"] = 1, 1  # overridden by the server (serve.py:233-234)
        torch.save({"state_dict": src.state_dict(), "hyper_parameters": hp}, path)
        m = create_model_from_checkpoint(name, load_checkpoint(str(path)), U, I, "cpu", graph)
        assert type(m) is type(src) and not m.training
        for (ka, a), (kb, b) in zip(m.state_dict().items(), src.state_dict().items()):
            assert ka == kb and torch.equal(a, b)
    ck = {"state_dict": LightGCN(U, I).state_dict(), "hyper_parameters": {}}
    assert create_model_from_checkpoint("lightgcn", ck, U, I, "cpu", None) is None  # no graph
    assert create_model_from_checkpoint("popularity", ck, U, I, "cpu") is None
    assert create_model_from_checkpoint("neural_cf", ck, U, I, "cpu") is None  # wrong keys


def test_recommender_host_logic():
    from hnm_recommendation_amd.serving import Recommender
    srv = Recommender(100, 50, device="cpu", customer_index={"abc": 7})
    assert srv.get_user_idx(5) == 5 and srv.get_user_idx(100) is None
    assert srv.get_user_idx("abc") == 7 and srv.get_user_idx("zzz") is None
    with pytest.raises(ValueError):
        srv._get_best_model()
    srv.add_model("neural_cf", NeuralCF(100, 50), {"test_map": 0.1})
    srv.add_model("lightgcn", LightGCN(100, 50), {"test_map": 0.3})
    srv.add_model("mf", MatrixFactorization(100, 50))
    assert srv._get_best_model() == "lightgcn"
    with pytest.raises(ValueError):
        srv.get_recommendations(1, model_name="nope")
    with pytest.raises(RuntimeError):  # scoring needs the GPU: no CPU path
        srv.get_recommendations(1, model_name="mf")


def test_recommend_top_k_range_like_torch_topk():
    """recommend() ends in torch.topk(scores, top_k) (neural_cf.py:324 and the other models):
    top_k > num_items raises RuntimeError -- checked before any launch, so also here on CPU."""
    for m in (NeuralCF(10, 5), MatrixFactorization(10, 5), WideDeep(10, 5)):
        with pytest.raises(RuntimeError, match="out of range"):
            m.recommend(torch.tensor([0]))


def test_metrics_need_gpu():
    from hnm_recommendation_amd import evaluation as EV
    with pytest.raises(RuntimeError):
        EV.rank_metrics(torch.zeros(2, 12, dtype=torch.int64), 12,
                        truth=torch.zeros(2, 3, dtype=torch.int64))


LIGHTNING = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lightning")


def _lightning_graph():
    return torch.from_numpy(syn.bipartite_edge_index(60, 40, 300, seed=23)), None


def test_lightning_checkpoint_fixture_loads_like_serve_py():
    """The Lightning-2.x-shaped .ckpt fixtures (tests/golden/make_lightning_ckpt.py) go
    through the safe loader and the serve.py dispatch: name = parent directory
    (serve.py:184-186), hparams from `hyper_parameters` with num_users/num_items overridden
    (:227-232), `metrics` kept (:203)."""
    from hnm_recommendation_amd.serving import Recommender, load_checkpoint
    ck = load_checkpoint(os.path.join(LIGHTNING, "neural_cf", "epoch=3-step=1200.ckpt"))
    assert {"epoch", "global_step", "pytorch-lightning_version", "state_dict", "loops",
            "callbacks", "optimizer_states", "lr_schedulers", "hparams_name",
            "hyper_parameters"} <= set(ck)
    srv = Recommender(60, 40, device="cpu")
    assert srv.load_checkpoints(LIGHTNING, graph=_lightning_graph()) == ["lightgcn", "neural_cf"]
    m = srv.models["neural_cf"]
    assert type(m).__name__ == "NeuralCF" and m.mf_dim == 16 and m.mlp_dims == [32, 16, 8]
    for k, v in ck["state_dict"].items():
        assert torch.equal(m.state_dict()[k], v), k
    assert srv.model_metrics["neural_cf"]["test_map"] == pytest.approx(0.0123)
    assert type(srv.models["lightgcn"]).__name__ == "LightGCN"
    assert srv.models["lightgcn"].embedding_dim == 16


def test_build_tracks_every_csrc_header():
    """Incremental builds rebuild every object when any csrc header changes (a header left
    out of build.HEADERS once left stale objects calling an old signature)."""
    import glob
    from hnm_recommendation_amd import build
    hdrs = {os.path.basename(p) for p in glob.glob(os.path.join(build.CSRC, "*.h"))}
    assert hdrs <= set(build.HEADERS), sorted(hdrs - set(build.HEADERS))


def test_ncf_shard_scorer_dispatch():
    """sharding.ncf_shard_topk gives the fused two-phase scorer for the default tower and
    ncf_deep_shard_topk (single-phase, k <= 64) for any other tower (no GPU work at
    construction)."""
    from hnm_recommendation_amd import NeuralCF
    from hnm_recommendation_amd import sharding as S
    fused = S.ncf_shard_topk(NeuralCF(50, 40), 0, 40, 12)
    assert type(fused) is S.ncf_shard_topk and hasattr(fused, "begin_lists")
    deep = S.ncf_shard_topk(NeuralCF(50, 40, mlp_dims=[128, 64, 32, 16]), 10, 40, 12)
    assert type(deep) is S.ncf_deep_shard_topk and not hasattr(deep, "begin_lists")
    assert (deep.lo, deep.hi, deep.k) == (10, 40, 12)
    with pytest.raises(ValueError):
        S.ncf_shard_topk(NeuralCF(50, 40, mlp_dims=[64, 32]), 0, 40, 100)
