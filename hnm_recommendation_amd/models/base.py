"""Shared host logic of the drop-in model modules.

The reference models are `pytorch_lightning.LightningModule`s (e.g. `neural_cf.py:9`);
Lightning is not part of the scoring hot path and is not installed here, so the mirror
modules are plain `nn.Module`s that keep what the serving/eval callers rely on:
constructor kwargs, `hparams` (what `save_hyperparameters()` records and `serve.py:228`
reads back from `.ckpt` files), submodule names (state_dict keys), `eval()/to()`.
"""
from __future__ import annotations

import inspect
import itertools
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from .. import _lib


class RecModule(nn.Module):
    """nn.Module + the LightningModule bits the hot path's callers use."""

    def save_hyperparameters(self):
        frame = inspect.currentframe().f_back
        info = inspect.getargvalues(frame)
        self.hparams = {k: info.locals[k] for k in info.args if k != "self"}

    def log(self, name, value, *args, **kwargs):
        """LightningModule.log stand-in: the last value per name lands in `logged_metrics`
        (what a Trainer's callback_metrics would hold)."""
        if not hasattr(self, "logged_metrics"):
            self.logged_metrics = {}
        self.logged_metrics[name] = value

    # ------------------------------------------------------ Lightning evaluation hooks
    # The reference's offline-evaluation stack (`trainer.validate` / `trainer.test(ckpt_path=
    # "best")`, scripts/train.py:252): validation_step -> predict_all_items -> torch.topk ->
    # metrics.update, then on_*_epoch_end logs metrics.compute() and resets (neural_cf.py:235-272,
    # lightgcn.py:267-294, wide_deep.py:314-342, matrix_factorization.py:158-185).  Here the
    # dense score matrix + torch.topk is the fused top-K (`recommend_with_scores`, same
    # (score desc, item asc) order), so a step never materialises the [B, num_items] scores.
    def _validation_topk(self, batch):
        return self.recommend_with_scores(batch["user_ids"], k=self.top_k)[1]

    def validation_step(self, batch, batch_idx):
        """batch: {'user_ids': [B], 'ground_truth': [B, T] item ids (negative = padding) or a
        list of id lists}."""
        self._check_top_k()  # torch.topk(scores, self.top_k) raises for top_k > num_items
        with torch.no_grad():
            top = self._validation_topk(batch)
        self.metrics.update(top, batch["ground_truth"])

    def _epoch_end(self, prefix, **kw):
        metrics = self.metrics.compute()
        self.metrics.reset()
        for name, value in metrics.items():
            self.log(f"{prefix}_{name}", value, **kw)
        return metrics

    def on_validation_epoch_end(self):
        return self._epoch_end("val", prog_bar=True)

    def test_step(self, batch, batch_idx):
        self.validation_step(batch, batch_idx)

    def on_test_epoch_end(self):
        return self._epoch_end("test")

    # ------------------------------------------------------------------ helpers
    @property
    def device(self) -> torch.device:
        return next(self.parameters()).device

    def _ids(self, ids: torch.Tensor, bound: int, what: str = "user_ids"):
        """(int64 contiguous ids on the module device, host_checked).  Host ids are
        range-checked here for free (IndexError before any launch), so the call needs no
        device-side check; device ids are checked by the kernels' error word, which costs a
        stream sync after the call (`_check`)."""
        if not isinstance(ids, torch.Tensor):
            ids = torch.as_tensor(ids)
        if ids.dim() == 0:
            ids = ids.reshape(1)
        dev = self.device
        _lib.require_gpu(next(self.parameters()))
        host = not ids.is_cuda
        if host and ids.numel() > 0:
            lo, hi = int(ids.min()), int(ids.max())
            if lo < 0 or hi >= bound:
                raise IndexError(f"index out of range in self ({what} must be in [0, {bound}))")
        return ids.to(device=dev, dtype=torch.int64).contiguous(), host

    def _check_top_k(self):
        """`recommend()` ends in `torch.topk(scores, self.top_k, dim=1)` (e.g. neural_cf.py:324),
        which raises for top_k outside [0, num_items]; so does the mirror, before any launch.
        `recommend_with_scores(k=...)` (the serve path's per-request k) clamps k instead."""
        if not 0 <= self.top_k <= self.num_items:
            raise RuntimeError("selected index k out of range")

    @staticmethod
    def _check(device, *host_checked):
        """Raise IndexError for out-of-range device ids (syncs the stream) -- skipped when
        every id of the call was range-checked on the host."""
        if not all(host_checked):
            _lib.sync_check(device)


def _history_arrays(keys, sets, num_items: int):
    """Vectorized CSR of `{key: iterable of item ids}` rows in `keys` order: negative ids
    wrap like torch indexing, ids outside [-num_items, num_items) raise IndexError as
    `scores[i, items] = -inf` would, rows sorted ascending and de-duplicated (one
    lexicographic np.unique over (row, item), no per-row numpy calls)."""
    lens = np.fromiter((len(x) for x in sets), dtype=np.int64, count=len(sets))
    total = int(lens.sum())
    flat = np.fromiter(itertools.chain.from_iterable(sets), dtype=np.int64, count=total)
    bad = (flat >= num_items) | (flat < -num_items)
    if bad.any():
        raise IndexError(f"index {int(flat[bad][0])} is out of bounds for dimension 1 "
                         f"with size {num_items}")
    flat = np.where(flat < 0, flat + num_items, flat)
    rows = np.repeat(np.arange(len(sets), dtype=np.int64), lens)
    key = np.unique(rows * num_items + flat)          # sorted by (row, item), unique
    r, items = np.divmod(key, num_items)
    ptr = np.zeros(len(sets) + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=len(sets)), out=ptr[1:])
    return ptr, items.astype(np.int32)


class UserHistory:
    """Device-resident per-user item history (CSR over user ids), built ONCE, for the
    -inf filter of batched recommend calls without a host round trip per batch.

    `recommend_with_scores(user_ids, filter_items=history)` (every model) gathers the
    batch's rows on the GPU (hnm_mask_gather_csr) and passes them to the fused top-K kernels
    as the same CSR mask a `filter_items` dict produces -- identical results (tests), but the
    per-call cost is two small kernel launches instead of a Python/numpy pass over the batch.
    This is what `serving.Recommender` holds for its purchase history (serve.py:166-168,
    350-352); the item-sharded scorers take it too (`mask_for(ids, item_range)`)."""

    def __init__(self, history: Dict[int, set], num_users: int, num_items: int, device):
        users = sorted(u for u in history if 0 <= int(u) < num_users and history[u])
        ptr_rows, idx = _history_arrays(users, [history[u] for u in users], num_items)
        full = np.zeros(int(num_users) + 1, np.int64)
        if users:
            full[np.asarray(users, np.int64) + 1] = np.diff(ptr_rows)
        np.cumsum(full, out=full)
        self._set(full, idx, num_users, num_items, device)

    @classmethod
    def from_interactions(cls, user_ids, item_ids, num_users: int, num_items: int, device):
        """From (user, item) interaction arrays -- e.g. the training transactions that are a
        customer's purchase history (serve.py:166-168) -- de-duplicated and sorted per user."""
        u = np.asarray(user_ids, np.int64)
        i = np.asarray(item_ids, np.int64)
        if u.shape != i.shape:
            raise ValueError("user_ids and item_ids must have the same shape")
        if u.size and (u.min() < 0 or u.max() >= num_users or i.min() < 0 or i.max() >= num_items):
            raise IndexError("interaction ids out of range")
        key = np.unique(u * num_items + i)
        r, items = np.divmod(key, num_items)
        full = np.zeros(int(num_users) + 1, np.int64)
        np.cumsum(np.bincount(r, minlength=num_users), out=full[1:])
        obj = cls.__new__(cls)
        obj._set(full, items.astype(np.int32), num_users, num_items, device)
        return obj

    def _set(self, ptr, idx, num_users, num_items, device):
        self.num_users, self.num_items = int(num_users), int(num_items)
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        lens = np.diff(ptr)
        self.max_len = int(lens.max()) if lens.size else 0
        self.nnz = int(ptr[-1])
        self.hist_ptr = torch.from_numpy(ptr).to(self.device)
        self.hist_idx = torch.from_numpy(idx if idx.size else np.zeros(1, np.int32)).to(self.device)

    def mask_for(self, user_ids: torch.Tensor, item_range=None):
        """(mask_ptr int64[B+1], mask_idx int32) for a batch of device user ids -- with
        item_range = (lo, hi): only history items in [lo, hi), renumbered i - lo (an item
        shard) -- or (None, None) when no history row can be non-empty."""
        if self.nnz == 0:
            return None, None
        u = user_ids
        if u.device != self.device:
            raise ValueError(f"history lives on {self.device}, user ids on {u.device}")
        lo, hi = (0, 2 ** 63 - 1) if item_range is None else (int(item_range[0]), int(item_range[1]))
        B = u.numel()
        cap = max(B * self.max_len, 1)
        mptr = torch.empty(B + 1, dtype=torch.int64, device=u.device)
        midx = torch.empty(cap, dtype=torch.int32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_mask_gather_csr")(c, _lib.ptr(self.hist_ptr), _lib.ptr(self.hist_idx),
                                                  self.num_users, _lib.ptr(u), B, lo, hi, cap,
                                                  _lib.ptr(mptr), _lib.ptr(midx)),
                   "hnm_mask_gather_csr")
        return mptr, midx


def filter_csr(user_ids: torch.Tensor, filter_items, num_items: int, device: torch.device):
    """Per-row CSR -inf mask for a batch: from a `UserHistory` (gathered on the device) or
    from the reference's `filter_items` dict.

    Mirrors the loop in every `recommend` (`neural_cf.py:316-321`): row i masks
    `filter_items[user_ids[i]]`; negative ids wrap like torch indexing; ids >= num_items
    raise IndexError as `scores[i, items] = -inf` would.
    Returns (mask_ptr int64[B+1], mask_idx int32[nnz]) on `device`, or (None, None).
    """
    if filter_items is None:
        return None, None
    if isinstance(filter_items, UserHistory):
        if filter_items.num_items != num_items:
            raise ValueError(f"history built for {filter_items.num_items} items, model has "
                             f"{num_items}")
        return filter_items.mask_for(user_ids)
    uids = user_ids.detach().cpu().tolist()
    empty = ()
    sets = [filter_items.get(u) or empty for u in uids]
    ptr, idx = _history_arrays(uids, sets, num_items)
    if ptr[-1] == 0:
        return None, None
    return (torch.from_numpy(ptr).to(device), torch.from_numpy(idx).to(device))


def empty_topk(k: int, u: torch.Tensor):
    """torch.topk's k = 0 result ([B, 0] scores and ids); k < 0 raises as torch.topk does."""
    if k < 0:
        raise RuntimeError("selected index k out of range")
    return (torch.empty(u.numel(), 0, dtype=torch.float32, device=u.device),
            torch.empty(u.numel(), 0, dtype=torch.int64, device=u.device))


def dense_topk(scores: torch.Tensor, k: int, mptr=None, midx=None):
    """torch.topk(scores, k) with the CSR mask, on the HIP row top-k kernel."""
    B, I = scores.shape
    k = min(k, I)
    out_v = torch.empty(B, k, dtype=torch.float32, device=scores.device)
    out_i = torch.empty(B, k, dtype=torch.int64, device=scores.device)
    c = _lib.ctx(scores.device)
    _lib.check(_lib.fn("hnm_topk_rows_f32")(c, _lib.ptr(scores), scores.stride(0), B, I,
                                            _lib.ptr(mptr), _lib.ptr(midx), k,
                                            _lib.ptr(out_v), _lib.ptr(out_i)),
               "hnm_topk_rows_f32")
    return out_v, out_i


def f32c(t: torch.Tensor) -> torch.Tensor:
    """fp32 contiguous view (no copy when already so)."""
    return t.detach().to(torch.float32).contiguous()
