"""GPU: the certified f16 pre-filters (ncf_cert.hip, dot_cert.hip, widedeep.hip) under weight
distributions unlike the synthetic init -- what trained models look like, not what the
generator draws (VERDICT r3 "Weak #6").

Each case checks, over the FULL H&M catalogue (105,542 items):
  * pair by pair, |approx - exact| <= bound (the worst-case bound every pruning step relies on);
  * top-K with the pre-filter is bitwise equal (ids and score bits) to HNM_OPT_PREFILTER=0;
  * the unusable-bound guard: the scans scale every operand by a power of two before the f16
    conversion (so no operand can overflow f16's 6.5e4), and refuse a call whose maxima exceed
    2^40 or are not finite -- such calls must report every row on the exact fallback.

Stress kinds:
  norms      every embedding row rescaled to a norm drawn uniformly from [50, 200];
  student_t  every weight (embeddings, Linear weights AND biases) Student-t(nu = 3), heavy
             tailed, at the init's spread;
  bn         (W&D) BatchNorm with running_var down to 1e-4 and gamma up to 10 (|scale| ~ 1e3);
  big        one item's embedding row at 1e6 (dynamic range 1e8 against the rest);
  huge       one item's embedding row at 1e13 (> 2^40): NCF / dot bounds are unusable, every
             row falls back to the exact scan; W&D (guard 1e30) keeps a valid bound that admits
             every item, so every row is re-scored exactly over the whole catalogue.
(reference: neural_cf.py:143-208, lightgcn.py:188-204, matrix_factorization.py:108-131,
wide_deep.py:157-285)
"""
import numpy as np
import pytest
import torch

from hnm_recommendation_amd import NeuralCF, WideDeep, _lib
from hnm_recommendation_amd import synthetic as syn

from test_gpu_prefilter import (dot_both, prefilter_debug, to_module, topk_both,
                                wd_prefilter_debug, wd_refine_debug)

pytestmark = pytest.mark.gpu
DEV = "cuda"
I_FULL = syn.HM_ITEMS


def stress(sd, kind, emb_keys, item_key, seed):
    return syn.stress_state_dict(sd, kind, emb_keys, item_key, seed)


def _check_bitwise(ex, pf, stats, B, kind, what, I=I_FULL):
    (ev, ei), (pv, pi) = ex, pf
    assert np.array_equal(ei, pi), what
    assert np.array_equal(ev.view(np.uint32), pv.view(np.uint32)), what
    rows, cands, fallback = stats
    print(f"{what} {kind}: candidates/row {cands / max(rows - fallback, 1):.1f}, "
          f"fallback rows {fallback} of {rows}")
    assert rows == B
    if kind == "huge" and what == "W&D":
        # the split-f16 scan's guard is at 1e30 (its operands are scaled to 2^14 and its
        # slack terms are exact), so 1e13 stays usable: the scan's bound then covers every
        # other item, and the re-scoring cascade's three-pass stage (round 5) still leaves
        # (nearly) the whole catalogue to the exact fp32 stage -- or the rows fall back
        assert fallback == B or cands >= B * (I - 2), (fallback, cands)
    elif kind == "huge":
        assert fallback == B  # unusable bound (> 2^40): every row on the exact scan


# ------------------------------------------------------------------ NeuralCF
NCF_EMB = ["gmf_user_embedding.weight", "gmf_item_embedding.weight",
           "mlp_user_embedding.weight", "mlp_item_embedding.weight"]


def ncf_stress(kind, U=50_000, seed=0):
    sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=seed, bias_scale=0.05)
    sd = stress(sd, kind, NCF_EMB, "mlp_item_embedding.weight", seed)
    return to_module(NeuralCF(U, I_FULL), sd)


@pytest.mark.parametrize("kind", ["norms", "student_t", "big"])
def test_ncf_bound_stress(kind):
    m = ncf_stress(kind)
    users = torch.from_numpy(syn.user_batch(m.num_users, 32, seed=5)).to(DEV)
    approx, bound = prefilter_debug(m, users)
    exact = m.predict_all_items(users)
    bp = float(m.prediction_layer.bias.detach())
    ratio = ((approx + bp - exact).abs() / bound).max().item()
    print(f"NCF {kind}: max |approx + bp - exact| / bound = {ratio:.4f}")
    assert torch.isfinite(bound).all()
    assert ratio <= 1.0, ratio


@pytest.mark.parametrize("kind", ["norms", "student_t", "big", "huge"])
def test_ncf_topk_stress_bitwise(kind):
    m = ncf_stress(kind, seed=1)
    B = 300
    users = torch.from_numpy(syn.user_batch(m.num_users, B, seed=9)).to(DEV)
    ex, pf, stats = topk_both(m, users)
    _check_bitwise(ex, pf, stats, B, kind, "NCF")


# ------------------------------------------------------------------ dot models (MF / LightGCN)
def dot_stress(kind, d=64, U=50_000, seed=0):
    rng = np.random.Generator(np.random.PCG64(2000 + seed))
    ut = (rng.standard_normal((U, d)) * 0.1).astype(np.float32)
    it = (rng.standard_normal((I_FULL, d)) * 0.1).astype(np.float32)
    ub = (rng.standard_normal(U) * 0.05).astype(np.float32)
    ib = (rng.standard_normal(I_FULL) * 0.05).astype(np.float32)
    sd = stress({"u": ut, "i": it, "ub": ub, "ib": ib}, kind, ["u", "i"], "i", seed)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in sd.items()}
    return t["u"], t["i"], (t["ub"], t["ib"], torch.tensor([0.2], device=DEV))


@pytest.mark.parametrize("kind", ["norms", "student_t", "big"])
def test_dot_bound_stress(kind):
    ut, it, (ub, ib, cb) = dot_stress(kind)
    d = ut.shape[1]
    ids = torch.from_numpy(syn.user_batch(ut.shape[0], 40, seed=3)).to(DEV)
    approx = torch.empty(40, I_FULL, device=DEV)
    bound = torch.empty(40, device=DEV)
    _lib.check(_lib.fn("hnm_dot_prefilter_debug_f32")(
        _lib.ctx(ids.device), _lib.ptr(ut), ut.shape[0], ut.stride(0), _lib.ptr(ids), 40,
        _lib.ptr(it), I_FULL, it.stride(0), d, _lib.ptr(ub), _lib.ptr(ib), _lib.ptr(cb),
        _lib.ptr(approx), I_FULL, _lib.ptr(bound)), "dot_prefilter_debug")
    _lib.sync_check(ids.device)
    exact = ut[ids] @ it.T + ub[ids][:, None] + cb + ib[None, :]
    ratio = ((approx - exact).abs().amax(1) / bound).max().item()
    print(f"dot {kind}: max err / bound = {ratio:.4f}")
    assert torch.isfinite(bound).all()
    assert ratio <= 1.0, ratio


@pytest.mark.parametrize("kind,d", [("norms", 64), ("student_t", 64), ("student_t", 128),
                                    ("big", 64), ("huge", 64)])
def test_dot_topk_stress_bitwise(kind, d):
    ut, it, (ub, ib, cb) = dot_stress(kind, d=d, seed=1)
    B = 777
    ids = torch.from_numpy(syn.user_batch(ut.shape[0], B, seed=4)).to(DEV)
    ex, pf, stats = dot_both(ut, ids, it, 12, ub=ub, ib=ib, cb=cb)
    _check_bitwise(ex, pf, stats, B, kind, f"dot d={d}")


# ------------------------------------------------------------------ Wide&Deep
WD_EMB = ["deep_user_embedding.weight", "deep_item_embedding.weight"]


def wd_stress(kind, U=20_000, seed=0):
    sd = syn.widedeep_state_dict(U, I_FULL, 64, (512, 256, 128), seed=seed, bias_scale=0.05,
                                 randomize_bn=True)
    sd = stress(sd, kind, WD_EMB, "deep_item_embedding.weight", seed)
    return to_module(WideDeep(U, I_FULL, embedding_dim=64, deep_layers=[512, 256, 128]), sd)


@pytest.mark.parametrize("kind", ["norms", "student_t", "bn", "big"])
def test_wd_bound_stress(kind):
    m = wd_stress(kind)
    users = torch.from_numpy(syn.user_batch(m.num_users, 16, seed=5)).to(DEV)
    exact = m.predict_all_items(users)
    for what, fn in (("scan", wd_prefilter_debug), ("refine", wd_refine_debug)):
        approx, bound = fn(m, users)
        ratio = ((approx - exact).abs() / bound).max().item()
        print(f"W&D {kind} {what}: max |approx - exact| / bound = {ratio:.4f}")
        assert torch.isfinite(bound).all()
        assert ratio <= 1.0, (what, ratio)


@pytest.mark.parametrize("kind", ["norms", "student_t", "bn", "big", "huge"])
def test_wd_topk_stress_bitwise(kind):
    m = wd_stress(kind, seed=1)
    B = 48
    users = torch.from_numpy(syn.user_batch(m.num_users, B, seed=9)).to(DEV)
    ex, pf, stats = topk_both(m, users)
    _check_bitwise(ex, pf, stats, B, kind, "W&D")


@pytest.mark.parametrize("kind", ["init", "personal", "norms", "student_t"])
def test_ncf_strided_sample_gate(kind):
    """The certified NCF path's gated per-user strided sample (ncf_cert.hip CERT_STRIDE, round
    5; opt-in, HNM_OPT_STRIDED = 1): whether it runs is predicted on the proxy rows (candidates saved vs. the pass's cost);
    either way the top-K is bitwise the exact scan's (rows whose segments overflow take the
    exact fallback, now spread over the whole chip), and the count of rows that used it is
    all-or-nothing per call.  At U = 60,000 the init weights' user embeddings are 5x larger
    than at the H&M shape (xavier bounds scale with 1/sqrt(U)).  Measured (round 5, B = 512):
    init 1,158 candidates a row, bound-limited (the gate correctly predicts no saving: off);
    personal 413 and norms 106 with the pass on (norms: 598 + overflow rows before it at the
    H&M shape)."""
    U, B = 60_000, 512
    if kind == "init":
        sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=3)
    elif kind == "personal":
        sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=3, bias_scale=0.05,
                                emb_scale=20.0)
    else:
        sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=3, bias_scale=0.05)
        sd = stress(sd, kind, NCF_EMB, "mlp_item_embedding.weight", 3)
    m = to_module(NeuralCF(U, I_FULL), sd)
    users = torch.from_numpy(syn.user_batch(U, B, seed=11)).to(DEV)
    dev = users.device
    _lib.set_prefilter(dev, False)
    try:
        ev, ei = m.recommend_with_scores(users)
    finally:
        _lib.set_prefilter(dev, True)
    _lib.prefilter_stats(dev, reset=True)
    _lib.set_option(dev, _lib.HNM_OPT_STATS, 1)
    _lib.set_option(dev, _lib.HNM_OPT_STRIDED, 1)  # opt-in (default 0)
    try:
        pv, pi = m.recommend_with_scores(users)
    finally:
        _lib.set_option(dev, _lib.HNM_OPT_STATS, 0)
        _lib.set_option(dev, _lib.HNM_OPT_STRIDED, 0)
    rows, cands, fallback, sampled = _lib.prefilter_stats(dev, reset=True, extended=True)
    print(f"NCF {kind}: candidates/row {cands / max(rows - fallback, 1):.1f}, fallback {fallback}, "
          f"strided-sample rows {sampled}")
    assert torch.equal(ei, pi) and torch.equal(ev.view(torch.int32), pv.view(torch.int32))
    assert rows == B
    assert sampled in (0, B)
    if kind in ("personal", "norms"):
        # the gate fires on these weights, so the bitwise check above covers a call whose bound
        # took the strided sample's kth2
        assert sampled == B, (kind, sampled)


@pytest.mark.parametrize("kind", ["personal", "norms"])
def test_ncf_best_first_rescoring(kind):
    """Rows whose scan bound came from a poor sample append hundreds of candidates; the
    re-scoring scores the 64 best (by the scan's test value) first and then only candidates
    that pass against their exact K-th (ncf_cert.hip ncf_rescore_kernel, round 5).  Bitwise the
    exact scan's top-K, with far fewer exact re-scores than appended candidates (the bench's
    weight sets at the H&M shape: personal 306 appended / 64 re-scored a row, norms 598 / 64)."""
    U, B = syn.HM_USERS, 512
    if kind == "personal":
        sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=4, bias_scale=0.05,
                                emb_scale=20.0)
    else:
        sd = syn.ncf_state_dict(U, I_FULL, 64, (128, 64, 32), seed=4, bias_scale=0.05)
        sd = stress(sd, kind, NCF_EMB, "mlp_item_embedding.weight", 4)
    m = to_module(NeuralCF(U, I_FULL), sd)
    users = torch.from_numpy(syn.user_batch(U, B, seed=21)).to(DEV)
    ex, pf, stats = topk_both(m, users)
    (ev, ei), (pv, pi) = ex, pf
    assert np.array_equal(ei, pi) and np.array_equal(ev.view(np.uint32), pv.view(np.uint32))
    rows, cands, fallback = stats
    per_row = cands / max(rows - fallback, 1)
    print(f"NCF {kind}: exact re-scores / row {per_row:.1f}, fallback rows {fallback}")
    assert rows == B
    assert per_row <= 128, per_row  # 64 + the few that pass against the exact K-th

