"""GPU: the row-level C-ABI entries of include/hnm.h, called directly through ctypes against
numpy restatements of the reference operations they replace:

* hnm_gather_rows_f32  -- nn.Embedding.__call__ (neural_cf.py:155-156, lightgcn.py:199,
  wide_deep.py:207): out[b] = table[ids[b]], bitwise; an out-of-range id writes NaN and
  flags HNM_EOOB (IndexError at hnm_ctx_check, like nn.Embedding);
* hnm_linear_rows_f32  -- the user / item half of a first Linear layer (neural_cf.py:85-87,
  wide_deep.py:128): Y[r] = X[ids[r]] @ W[:, slice]^T + b, plain and pair-permuted layouts;
* hnm_axpby_f32        -- the alpha_0 E_0 term of the LightGCN layer combine
  (lightgcn.py:156-158): out = alpha x + beta y.
"""
import numpy as np
import pytest
import torch

from hnm_recommendation_amd import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _c(t):
    return _lib.ctx(t.device)


@pytest.mark.parametrize("d,ld,ldo", [(64, 64, 64), (128, 132, 128), (13, 17, 20), (300, 300, 304)])
def test_gather_rows(d, ld, ldo):
    rng = np.random.default_rng(d)
    R = 5000
    tab = rng.standard_normal((R, ld)).astype(np.float32)
    ids = np.concatenate([rng.integers(0, R, 997), [0, R - 1, 5, 5]]).astype(np.int64)
    T, I = torch.from_numpy(tab).to(DEV), torch.from_numpy(ids).to(DEV)
    out = torch.full((ids.size, ldo), -7.0, device=DEV)
    _lib.check(_lib.fn("hnm_gather_rows_f32")(_c(T), _lib.ptr(T), R, ld, d, _lib.ptr(I), ids.size,
                                              _lib.ptr(out), ldo), "gather")
    _lib.sync_check(T.device)
    got = out.cpu().numpy()
    assert np.array_equal(got[:, :d].view(np.uint32), tab[ids, :d].view(np.uint32))
    assert (got[:, d:] == -7.0).all()  # padding columns untouched
    # out-of-range ids: NaN rows + IndexError at the check; other rows still gathered
    bad = torch.tensor([3, R, -1, 4], dtype=torch.int64, device=DEV)
    o2 = torch.zeros(4, ldo, device=DEV)
    _lib.check(_lib.fn("hnm_gather_rows_f32")(_c(T), _lib.ptr(T), R, ld, d, _lib.ptr(bad), 4,
                                              _lib.ptr(o2), ldo), "gather")
    with pytest.raises(IndexError):
        _lib.sync_check(T.device)
    g2 = o2.cpu().numpy()
    assert np.isnan(g2[1, :d]).all() and np.isnan(g2[2, :d]).all()
    assert np.array_equal(g2[0, :d], tab[3, :d]) and np.array_equal(g2[3, :d], tab[4, :d])
    # empty batch: NULL ids / out accepted
    assert _lib.fn("hnm_gather_rows_f32")(_c(T), _lib.ptr(T), R, ld, d, None, 0, None, ldo) == 0


@pytest.mark.parametrize("K,N,permute,with_ids,M", [(64, 64, 0, True, 4096), (64, 64, 1, True, 37),
                                                    (32, 96, 1, False, 20000), (13, 10, 0, True, 300),
                                                    (256, 512, 0, False, 777)])
def test_linear_rows(K, N, permute, with_ids, M):
    """Y[r, c(n)] = sum_k X[x(r), k] W[n, k] + b[n] with W a column slice (ldw = 2K, the item
    half) of a wider Linear weight; fp32 fma chain vs float64 (error <= K 2^-24 sum |x w|)."""
    rng = np.random.default_rng(K + N)
    R = 6000
    X = rng.standard_normal((R, K)).astype(np.float32)
    W = rng.standard_normal((N, 2 * K)).astype(np.float32) * 0.1
    b = rng.standard_normal(N).astype(np.float32)
    ids = rng.integers(0, R, M).astype(np.int64) if with_ids else None
    ldy = N + (N % 2) + (4 if permute else 2)
    Xt, Wt, bt = (torch.from_numpy(a).to(DEV) for a in (X, W, b))
    It = torch.from_numpy(ids).to(DEV) if with_ids else None
    rows = M if with_ids else min(M, R)
    Y = torch.full((rows, ldy), -3.0, device=DEV)
    _lib.check(_lib.fn("hnm_linear_rows_f32")(_c(Xt), _lib.ptr(Xt), K, _lib.ptr(It), R, rows, K,
                                              _lib._p(Wt.data_ptr() + 4 * K),
                                              2 * K, _lib.ptr(bt), N, _lib.ptr(Y), ldy, permute),
               "linear_rows")
    _lib.sync_check(Xt.device)
    src = X[ids] if with_ids else X[:rows]
    Wi = W[:, K:].astype(np.float64)
    ref = src.astype(np.float64) @ Wi.T + b
    mag = np.abs(src.astype(np.float64)) @ np.abs(Wi).T + np.abs(b)
    got = Y.cpu().numpy()
    cols = np.arange(N)
    pos = (cols & 1) * (ldy // 2) + (cols >> 1) if permute else cols
    err = np.abs(got[:, pos] - ref)
    assert (err <= (K + 2) * 2.0 ** -24 * mag + 1e-30).all(), float((err / mag).max())
    untouched = np.setdiff1d(np.arange(ldy), pos)
    assert (got[:, untouched] == -3.0).all()


@pytest.mark.parametrize("K,N,permute,with_ids,M", [(64, 64, 1, True, 40000), (64, 512, 0, False, 33000),
                                                    (32, 96, 1, True, 35001), (128, 64, 0, True, 40000)])
def test_linear_rows_mfma_bitwise_valu(K, N, permute, with_ids, M):
    """The fp32-MFMA projection (linear_rows_mfma_kernel, HNM_OPT_LINEAR_MFMA, taken for
    K % 32 == 0 at >= 2 row blocks a CU) is bitwise the VALU kernel's k-ordered fmaf chain --
    incl. rows of zeros, -0, fp32 denormals and an out-of-range id (NaN row)."""
    rng = np.random.default_rng(K * N + M)
    R = 50000
    X = rng.standard_normal((R, K)).astype(np.float32)
    X[7] = 0.0
    X[8] = -0.0
    X[9] = np.float32(1e-40) * rng.standard_normal(K).astype(np.float32)  # denormals
    X[10, ::3] = 0.0
    W = rng.standard_normal((N, 2 * K)).astype(np.float32) * 0.1
    W[3] = -0.0
    W[4, :] = np.float32(3e-39)
    b = rng.standard_normal(N).astype(np.float32)
    ids = rng.integers(0, R, M).astype(np.int64) if with_ids else None
    if with_ids:
        ids[:6] = [7, 8, 9, 10, 7, 8]
        ids[100] = R  # out of range: NaN row, IndexError at the check
    ldy = N + (4 if permute else 2)
    Xt, Wt, bt = (torch.from_numpy(a).to(DEV) for a in (X, W, b))
    It = torch.from_numpy(ids).to(DEV) if with_ids else None
    rows = M if with_ids else min(M, R)
    outs = []
    try:
        for opt in (0, 1):
            _lib.set_option(Xt.device, _lib.HNM_OPT_LINEAR_MFMA, opt)
            Y = torch.full((rows, ldy), -3.0, device=DEV)
            _lib.check(_lib.fn("hnm_linear_rows_f32")(_c(Xt), _lib.ptr(Xt), K, _lib.ptr(It), R, rows,
                                                      K, _lib._p(Wt.data_ptr() + 4 * K), 2 * K,
                                                      _lib.ptr(bt), N, _lib.ptr(Y), ldy, permute),
                       "linear_rows")
            if with_ids:
                with pytest.raises(IndexError):
                    _lib.sync_check(Xt.device)
            else:
                _lib.sync_check(Xt.device)
            outs.append(Y.cpu().numpy())
    finally:
        _lib.set_option(Xt.device, _lib.HNM_OPT_LINEAR_MFMA, 1)
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    if with_ids:
        assert np.isnan(outs[1][100, :N if not permute else N // 2]).all()


def test_linear_rows_oob():
    X = torch.randn(100, 16, device=DEV)
    W = torch.randn(8, 16, device=DEV)
    ids = torch.tensor([1, 100, 2], dtype=torch.int64, device=DEV)
    Y = torch.zeros(3, 8, device=DEV)
    _lib.check(_lib.fn("hnm_linear_rows_f32")(_c(X), _lib.ptr(X), 16, _lib.ptr(ids), 100, 3, 16,
                                              _lib.ptr(W), 16, None, 8, _lib.ptr(Y), 8, 0), "lin")
    with pytest.raises(IndexError):
        _lib.sync_check(X.device)
    y = Y.cpu().numpy()
    assert np.isnan(y[1]).all() and np.isfinite(y[[0, 2]]).all()
    # shape errors are refused before any launch
    assert _lib.fn("hnm_linear_rows_f32")(_c(X), _lib.ptr(X), 8, None, 100, 3, 16, _lib.ptr(W),
                                          16, None, 8, _lib.ptr(Y), 8, 0) == _lib.HNM_EINVAL


@pytest.mark.parametrize("n,with_y", [(1, True), (1_000_003, True), (4096 * 64, False)])
def test_axpby(n, with_y):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    a, bb = np.float32(0.25), np.float32(-1.75)
    xt, yt = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    out = torch.empty_like(xt)
    _lib.check(_lib.fn("hnm_axpby_f32")(_c(xt), n, float(a), _lib.ptr(xt), float(bb),
                                        _lib.ptr(yt) if with_y else None, _lib.ptr(out)), "axpby")
    torch.cuda.synchronize()
    ref = a.astype(np.float64) * x + (bb.astype(np.float64) * y if with_y else 0.0)
    got = out.cpu().numpy().astype(np.float64)
    # a x rounded once, then (fused or not) one more rounding: <= 2 ulp of the magnitudes
    tol = 2.0 ** -23 * (np.abs(a * x) + (np.abs(bb * y) if with_y else 0.0)) + 1e-45
    assert (np.abs(got - ref) <= tol).all()
    if not with_y:
        assert np.array_equal(out.cpu().numpy(), (a * x).astype(np.float32))
