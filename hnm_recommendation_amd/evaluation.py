"""Ranking metrics over the top-K output on the GPU.

Mirrors `src/evaluation/metrics.py` of the reference:

* `evaluate_recommendations(predictions, ground_truth, k)` (`metrics.py:193-255`),
* the torchmetrics classes `MeanAveragePrecision` (`:10-66`), `RecallAtK` (`:69-105`),
  `PrecisionAtK` (`:108-142`), `NDCGAtK` (`:145-190`) with `update(preds, target, mask)`
  / `compute()`,
* `RecommendationMetrics`, the class every reference model imports (`neural_cf.py:6`,
  `lightgcn.py:10`, `wide_deep.py:6`, `matrix_factorization.py:7`) but the published
  snapshot does not define; keys follow its callers
  (`benchmark_models.py:203-206`, `train.py:257-260`).

The per-user loops run in one HIP kernel (`csrc/eval.hip`, `hnm_rank_metrics_f64`): one
wave per user, the reference's float64 formulas in its summation order, so every user's
AP / Recall / Precision / NDCG is bitwise the value the Python loop computes; means come
from a fixed-order device reduction.  `evaluate_model` chains a model's fused top-K and
the metrics kernel batch by batch on the device -- full-catalogue offline evaluation with
only four sums crossing PCIe.  There is no CPU path: inputs go to the GPU (or raise).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import numpy as np
import torch

from . import _lib

_INV_LOG2: dict = {}


def _inv_log2(k: int, device) -> torch.Tensor:
    """[1.0 / np.log2(i + 2)] for i < k, formed term by term as the reference does
    (`metrics.py:180`, `:243`), cached per device."""
    key = (k, str(device))
    t = _INV_LOG2.get(key)
    if t is None:
        tab = np.asarray([1.0 / np.log2(i + 2) for i in range(k)], np.float64)
        t = torch.from_numpy(tab).to(device)
        _INV_LOG2[key] = t
    return t


def _device(device=None) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        _lib.require_gpu(torch.empty(0))  # raises: no CPU path
    return torch.device("cuda", torch.cuda.current_device())


def rank_metrics(pred: torch.Tensor, k: int, *, truth_ptr: Optional[torch.Tensor] = None,
                 truth_idx: Optional[torch.Tensor] = None, truth: Optional[torch.Tensor] = None,
                 truth_mask: Optional[torch.Tensor] = None,
                 pred_len: Optional[torch.Tensor] = None, per_user: bool = True):
    """Per-user metrics of top-K lists on the GPU (`hnm_rank_metrics_f64`).

    pred [B, L] int64 predicted item ids (first min(L, k) or pred_len[b] used); truth as a
    CSR (`truth_ptr` [B+1], `truth_idx`) or dense `truth` [B, T] with optional bool
    `truth_mask`.  Returns (per_user [B, 4] float64 (AP, Recall, Precision, NDCG) or None,
    n_true [B] int64 or None, sums [9] float64: metric sums over all rows, over rows with
    truth, and that row count).
    """
    _lib.require_gpu(pred)
    dev = pred.device
    if pred.dim() != 2:
        raise ValueError("pred must be [B, L]")
    if not 1 <= k <= 128:
        raise ValueError("k must be in [1, 128]")
    B = pred.shape[0]
    p = pred.to(torch.int64).contiguous()
    if truth_ptr is not None:
        if truth is not None or truth_mask is not None:
            raise ValueError("give the truth either as CSR or dense, not both")
        tp = truth_ptr.to(device=dev, dtype=torch.int64).contiguous()
        ti = truth_idx.to(device=dev, dtype=torch.int64).contiguous()
        if tp.numel() != B + 1:
            raise ValueError("truth_ptr must have B + 1 entries")
        ldt, tm = 0, None
    else:
        if truth is None or truth.dim() != 2 or truth.shape[0] != B:
            raise ValueError("dense truth must be [B, T]")
        tp = None
        ti = truth.to(device=dev, dtype=torch.int64).contiguous()
        ldt = ti.shape[1]
        tm = None
        if truth_mask is not None:
            if truth_mask.shape != truth.shape:
                raise ValueError("truth_mask must match truth")
            tm = truth_mask.to(device=dev, dtype=torch.bool).contiguous().view(torch.uint8)
    pl = None if pred_len is None else pred_len.to(device=dev, dtype=torch.int64).contiguous()
    out = torch.empty(B, 4, dtype=torch.float64, device=dev) if per_user else None
    nt = torch.empty(B, dtype=torch.int64, device=dev) if per_user else None
    sums = torch.empty(9, dtype=torch.float64, device=dev)
    c = _lib.ctx(dev)
    _lib.check(_lib.fn("hnm_rank_metrics_f64")(
        c, _lib.ptr(p), B, p.shape[1], _lib.ptr(pl), int(k), _lib.ptr(tp), _lib.ptr(ti), ldt,
        _lib.ptr(tm), _lib.ptr(_inv_log2(k, dev)), _lib.ptr(out), _lib.ptr(nt),
        _lib.ptr(sums)), "hnm_rank_metrics_f64")
    return out, nt, sums


def truth_csr(users: Iterable[int], ground_truth: Dict[int, Iterable[int]], device):
    """CSR (ptr, idx) of `set(ground_truth[u])` for each u (sorted unique ids: the set
    semantics of `metrics.py:212`); users absent from the dict get empty rows."""
    ptr = [0]
    rows = []
    for u in users:
        t = ground_truth.get(u, ())
        a = np.unique(np.fromiter((int(x) for x in t), dtype=np.int64))
        rows.append(a)
        ptr.append(ptr[-1] + a.size)
    idx = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    return (torch.from_numpy(np.asarray(ptr, np.int64)).to(device),
            torch.from_numpy(idx.astype(np.int64)).to(device))


def evaluate_recommendations(predictions: Dict[int, list], ground_truth: Dict[int, list],
                             k: int = 12, device=None, per_user: bool = False):
    """`evaluate_recommendations` (`metrics.py:193-255`) with the per-user loop on the GPU.

    Mean over the ground-truth users of MAP@k, Recall@k, Precision@k, NDCG@k; users with
    no predictions contribute zeros (`:214-220`); a predicted user whose truth list is
    empty raises ZeroDivisionError as the reference's `ap / min(0, k)` does (`:229`).
    Returns {'map@k', 'recall@k', 'precision@k', 'ndcg@k'} (and the [U, 4] per-user
    float64 tensor when per_user=True).
    """
    dev = _device(device)
    users = list(ground_truth)
    for u in users:
        if u in predictions and len(set(ground_truth[u])) == 0:
            raise ZeroDivisionError("float division by zero")
    U = len(users)
    pred = np.zeros((U, k), np.int64)
    plen = np.zeros(U, np.int64)
    for r, u in enumerate(users):
        lst = predictions.get(u)
        if lst is None:
            continue
        lst = [int(x) for x in list(lst)[:k]]
        pred[r, :len(lst)] = lst
        plen[r] = len(lst)
    if U == 0:  # np.mean of an empty list: nan (with a RuntimeWarning in the reference)
        nan = np.float64("nan")
        res = {f"map@{k}": nan, f"recall@{k}": nan, f"precision@{k}": nan, f"ndcg@{k}": nan}
        return (res, torch.zeros(0, 4, dtype=torch.float64, device=dev)) if per_user else res
    tp, ti = truth_csr(users, ground_truth, dev)
    pu, _, sums = rank_metrics(torch.from_numpy(pred).to(dev), k, truth_ptr=tp, truth_idx=ti,
                               pred_len=torch.from_numpy(plen).to(dev), per_user=per_user)
    s = sums.cpu().numpy()
    res = {f"map@{k}": np.float64(s[0] / U), f"recall@{k}": np.float64(s[1] / U),
           f"precision@{k}": np.float64(s[2] / U), f"ndcg@{k}": np.float64(s[3] / U)}
    return (res, pu) if per_user else res


class _RankMetric:
    """Shared body of the four torchmetrics classes (`metrics.py:10-190`).

    `update(preds, target, mask=None)`: preds [B, n_items] are scores (2-D preds are
    always top-k'ed by the reference, `:31-35`; here by the HIP row top-K kernel, ties
    (score desc, index asc) where torch.topk leaves them unspecified); truth =
    `target[i][mask[i]]`, duplicates counted by len() (`:41-44`).  States accumulate in
    float64 (the reference's are float32 tensors, `:16`)."""

    _col = 0
    _only_with_truth = False

    def __init__(self, k: int = 12):
        self.k = k
        self.reset()

    def reset(self):
        self._sum = 0.0
        self._count = 0

    def update(self, preds: torch.Tensor, target: torch.Tensor, mask: Optional[torch.Tensor] = None):
        from .models.base import dense_topk
        _lib.require_gpu(preds)
        if preds.dim() != 2:
            raise ValueError("preds must be [batch_size, n_items] scores")
        kk = min(self.k, preds.shape[1])
        scores = preds.detach().to(torch.float32).contiguous()
        _, top = dense_topk(scores, kk)
        tgt = target.to(preds.device)
        if tgt.dim() == 1:
            tgt = tgt.reshape(-1, 1)
        _, _, sums = rank_metrics(top, self.k, truth=tgt, truth_mask=mask, per_user=False)
        s = sums.cpu().numpy()
        if self._only_with_truth:
            self._sum += float(s[4 + self._col])
            self._count += int(s[8])
        else:
            self._sum += float(s[self._col])
            self._count += preds.shape[0]

    def compute(self) -> torch.Tensor:
        return torch.tensor(self._sum / self._count if self._count > 0 else 0.0,
                            dtype=torch.float32)


class MeanAveragePrecision(_RankMetric):
    """MAP@k (`metrics.py:10-66`): every row counted, 0 for rows without truth."""
    _col = 0


class RecallAtK(_RankMetric):
    """Recall@k (`metrics.py:69-105`): rows with truth only."""
    _col = 1
    _only_with_truth = True


class PrecisionAtK(_RankMetric):
    """Precision@k (`metrics.py:108-142`): every row counted."""
    _col = 2


class NDCGAtK(_RankMetric):
    """NDCG@k (`metrics.py:145-190`): rows with truth only."""
    _col = 3
    _only_with_truth = True


def _rows(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    out = []
    for r in x:
        r = np.asarray(r).reshape(-1)
        out.append([int(v) for v in r if v >= 0])
    return out


class RecommendationMetrics:
    """Accumulates MAP / Recall / Precision / NDCG @ top_k over top-K index rows and
    ground-truth rows (negative ids = padding).  Truth rows are de-duplicated (set
    semantics, `metrics.py:212`); MAP and Precision average over every row, Recall and
    NDCG over rows with truth (the torchmetrics classes' counting)."""

    def __init__(self, top_k: int = 12):
        self.top_k = top_k
        self.reset()

    def reset(self):
        self._s = np.zeros(4)
        self._n_all = 0
        self._n_truth = 0

    def update(self, top_k_items, ground_truth, device=None):
        dev = top_k_items.device if isinstance(top_k_items, torch.Tensor) and \
            top_k_items.is_cuda else _device(device)
        preds = _rows(top_k_items)
        truth = _rows(ground_truth)
        if len(preds) != len(truth):
            raise ValueError("top_k_items and ground_truth must have the same number of rows")
        B = len(preds)
        if B == 0:
            return
        k = self.top_k
        pred = np.zeros((B, k), np.int64)
        plen = np.zeros(B, np.int64)
        for r, p in enumerate(preds):
            p = p[:k]
            pred[r, :len(p)] = p
            plen[r] = len(p)
        tp, ti = truth_csr(range(B), dict(enumerate(truth)), dev)
        _, _, sums = rank_metrics(torch.from_numpy(pred).to(dev), k, truth_ptr=tp, truth_idx=ti,
                                  pred_len=torch.from_numpy(plen).to(dev), per_user=False)
        s = sums.cpu().numpy()
        self._s += np.array([s[0], s[5], s[2], s[7]])
        self._n_all += B
        self._n_truth += int(s[8])

    def compute(self):
        def avg(s, n):
            return torch.tensor(s / n if n else 0.0)
        return {"map_at_k": avg(self._s[0], self._n_all),
                "recall_at_k": avg(self._s[1], self._n_truth),
                "precision_at_k": avg(self._s[2], self._n_all),
                "ndcg_at_k": avg(self._s[3], self._n_truth)}


def evaluate_model(model, user_ids: torch.Tensor, truth_ptr: torch.Tensor,
                   truth_idx: torch.Tensor, k: int = 12, batch_size: int = 4096,
                   filter_items: Optional[Dict[int, set]] = None) -> Dict[str, float]:
    """Offline evaluation of a model over many users, entirely on the device: per batch
    the model's fused top-k (`recommend_with_scores`) feeds the metrics kernel, sums stay
    on the GPU.  `truth_ptr`/`truth_idx`: CSR of each user's unique truth ids (row b
    belongs to user_ids[b]; `truth_csr` builds it from a dict).  Returns the means of
    `evaluate_recommendations` over all users (the `benchmark_models.py:151-167` loop:
    predict, top-12, metrics)."""
    dev = model.device
    _lib.require_gpu(next(model.parameters()))
    u = torch.as_tensor(user_ids).to(device=dev, dtype=torch.int64)
    tp = truth_ptr.to(device=dev, dtype=torch.int64)
    ti = truth_idx.to(device=dev, dtype=torch.int64)
    n = u.numel()
    if tp.numel() != n + 1:
        raise ValueError("truth_ptr must have len(user_ids) + 1 entries")
    tot = torch.zeros(9, dtype=torch.float64, device=dev)
    model.eval()
    with torch.no_grad():
        for b0 in range(0, n, batch_size):
            b1 = min(n, b0 + batch_size)
            _, top = model.recommend_with_scores(u[b0:b1], filter_items=filter_items, k=k)
            _, _, s = rank_metrics(top, k, truth_ptr=tp[b0:b1 + 1], truth_idx=ti, per_user=False)
            tot += s
    s = tot.cpu().numpy()
    nn_ = max(n, 1)
    return {f"map@{k}": float(s[0] / nn_), f"recall@{k}": float(s[1] / nn_),
            f"precision@{k}": float(s[2] / nn_), f"ndcg@{k}": float(s[3] / nn_)}
