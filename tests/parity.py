"""Parity helpers shared by the CPU and GPU test suites.

The bar (BASELINE.json north_star): identical top-K index SETS for the integer work and
scores within 1e-4 relative fp32.  torch.topk's tie order is unspecified, so a near-tie
at the K-th position (gap below the tolerance) makes the boundary items interchangeable:
`assert_topk_equivalent` accepts exactly those swaps and nothing else.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

RTOL = 1e-4  # north_star: scores within 1e-4 relative fp32


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    out = {k: z[k] for k in z.files}
    out["sd"] = {k[3:]: out[k] for k in z.files if k.startswith("sd/")}
    return out


def filter_from_arrays(keys, ptr, idx):
    return {int(k): set(int(x) for x in idx[ptr[i]:ptr[i + 1]]) for i, k in enumerate(keys)}


def score_tol(ref_scores):
    """Absolute tolerance per row: 1e-4 relative to the row's score scale."""
    s = np.asarray(ref_scores, np.float64)
    finite = np.where(np.isfinite(s), np.abs(s), 0.0)
    return RTOL * np.maximum(finite.max(axis=-1, keepdims=True), 1e-30)


def assert_scores_close(got, ref, what="scores"):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    both_inf = np.isinf(got) & np.isinf(ref) & (np.sign(got) == np.sign(ref))
    tol = score_tol(ref) if ref.ndim == 2 else RTOL * max(np.abs(ref[np.isfinite(ref)]).max(), 1e-30)
    err = np.where(both_inf, 0.0, np.abs(got - ref))
    bad = err > tol + RTOL * np.abs(np.where(np.isfinite(ref), ref, 0))
    assert not bad.any(), f"{what}: {bad.sum()} elements off, max err {err.max():.3e}"


def assert_topk_equivalent(got_idx, ref_scores, k, filter_rows=None, what="topk"):
    """got_idx [B, k] must be a valid top-k of ref_scores [B, I] up to near-ties.

    * indices distinct and in range,
    * every returned item scores >= (true k-th score - tol),
    * every item scoring > (true k-th score + tol) is returned,
    * returned order is non-increasing within tol.
    """
    got_idx = np.asarray(got_idx, np.int64)
    s = np.asarray(ref_scores, np.float64)
    B, I = s.shape
    assert got_idx.shape == (B, min(k, I)), (what, got_idx.shape)
    tol = score_tol(s)[:, 0]
    for b in range(B):
        row = s[b]
        g = got_idx[b]
        assert len(set(g.tolist())) == len(g), f"{what}: duplicate idx row {b}"
        assert g.min() >= 0 and g.max() < I, f"{what}: idx out of range row {b}"
        kth = np.sort(row)[::-1][len(g) - 1]
        gs = row[g]
        if np.isfinite(kth):
            assert (gs >= kth - tol[b]).all(), f"{what}: row {b} returned a non-top item"
            must = np.nonzero(row > kth + tol[b])[0]
            missing = set(must.tolist()) - set(g.tolist())
            assert not missing, f"{what}: row {b} missing {sorted(missing)[:5]}"
        else:
            # fewer than k finite candidates: every finite item must be present
            must = np.nonzero(np.isfinite(row))[0]
            assert set(must.tolist()) <= set(g.tolist()), f"{what}: row {b} missing finite"
        fin = np.isfinite(gs)
        d = np.diff(gs[fin])
        assert (d <= tol[b]).all(), f"{what}: row {b} not sorted desc"


def same_topk_sets(a, b):
    return all(set(x.tolist()) == set(y.tolist()) for x, y in zip(np.asarray(a), np.asarray(b)))


def assert_topk_matches_reference(got_idx, got_vals, ref, prefix="", what="topk"):
    """Our top-K against the REFERENCE's stored top-K (a `_topk_record` of
    tests/golden/make_golden.py: topk, topk_scores, kth, kth_gap, row_absmax).

    * returned scores equal the reference's top-K scores position by position within
      1e-4 of the row's score scale (both lists are sorted desc);
    * when the reference's K-th and (K+1)-th scores are separated by more than that
      tolerance the index SETS are identical; otherwise only items tied with the K-th
      (within tolerance) may differ, and everything above it must be present."""
    got_idx = np.asarray(got_idx, np.int64)
    got_vals = np.asarray(got_vals, np.float64)
    r_idx = np.asarray(ref[prefix + "topk"], np.int64)
    r_val = np.asarray(ref[prefix + "topk_scores"], np.float64)
    kth = np.asarray(ref[prefix + "kth"], np.float64)
    gap = np.asarray(ref[prefix + "kth_gap"], np.float64)
    scale = np.asarray(ref[prefix + "row_absmax"], np.float64)
    assert got_idx.shape == r_idx.shape, (what, got_idx.shape, r_idx.shape)
    n_exact = 0
    for b in range(r_idx.shape[0]):
        tol = RTOL * max(scale[b], 1e-30)
        fin = np.isfinite(r_val[b])
        assert np.array_equal(np.isfinite(got_vals[b]), fin), f"{what}: row {b} finiteness"
        err = np.abs(got_vals[b][fin] - r_val[b][fin])
        assert (err <= tol).all(), f"{what}: row {b} scores off by {err.max():.3e} (tol {tol:.3e})"
        g, r = set(got_idx[b].tolist()), set(r_idx[b].tolist())
        if not np.isfinite(kth[b]) or gap[b] > tol:
            assert g == r, f"{what}: row {b} set differs: {sorted(g - r)} vs {sorted(r - g)}"
            n_exact += 1
        else:
            must = {int(i) for i, v in zip(r_idx[b], r_val[b]) if v > kth[b] + tol}
            assert must <= g, f"{what}: row {b} missing {sorted(must - g)}"
            assert (got_vals[b] >= kth[b] - tol).all(), f"{what}: row {b} non-top item"
    return n_exact
