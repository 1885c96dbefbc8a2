"""Shared host logic of the drop-in model modules.

The reference models are `pytorch_lightning.LightningModule`s (e.g. `neural_cf.py:9`);
Lightning is not part of the scoring hot path and is not installed here, so the mirror
modules are plain `nn.Module`s that keep what the serving/eval callers rely on:
constructor kwargs, `hparams` (what `save_hyperparameters()` records and `serve.py:228`
reads back from `.ckpt` files), submodule names (state_dict keys), `eval()/to()`.
"""
from __future__ import annotations

import inspect
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

    def log(self, *args, **kwargs):  # Lightning no-op (training is out of scope)
        pass

    # ------------------------------------------------------------------ helpers
    @property
    def device(self) -> torch.device:
        return next(self.parameters()).device

    def _ids(self, ids: torch.Tensor, bound: int, what: str = "user_ids") -> torch.Tensor:
        """int64 contiguous ids on the module device (host ids are range-checked for free)."""
        if not isinstance(ids, torch.Tensor):
            ids = torch.as_tensor(ids)
        if ids.dim() == 0:
            ids = ids.reshape(1)
        dev = self.device
        _lib.require_gpu(next(self.parameters()))
        if not ids.is_cuda and ids.numel() > 0:
            lo, hi = int(ids.min()), int(ids.max())
            if lo < 0 or hi >= bound:
                raise IndexError(f"index out of range in self ({what} must be in [0, {bound}))")
        return ids.to(device=dev, dtype=torch.int64).contiguous()


def filter_csr(user_ids: torch.Tensor, filter_items: Optional[Dict[int, set]], num_items: int,
               device: torch.device):
    """Build the per-row CSR -inf mask from the reference's `filter_items` dict.

    Mirrors the loop in every `recommend` (`neural_cf.py:316-321`): row i masks
    `filter_items[user_ids[i]]`; negative ids wrap like torch indexing; ids >= num_items
    raise IndexError as `scores[i, items] = -inf` would.
    Returns (mask_ptr int64[B+1], mask_idx int32[nnz]) on `device`, or (None, None).
    """
    if filter_items is None:
        return None, None
    uids = user_ids.detach().cpu().tolist()
    ptr = [0]
    idx = []
    for u in uids:
        items = filter_items.get(u)
        if items:
            arr = np.fromiter((int(x) for x in items), dtype=np.int64)
            bad = (arr >= num_items) | (arr < -num_items)
            if bad.any():
                raise IndexError(f"index {int(arr[bad][0])} is out of bounds for dimension 1 "
                                 f"with size {num_items}")
            arr = np.where(arr < 0, arr + num_items, arr)
            arr = np.unique(arr)
            idx.append(arr)
            ptr.append(ptr[-1] + arr.size)
        else:
            ptr.append(ptr[-1])
    if ptr[-1] == 0:
        return None, None
    mptr = torch.tensor(ptr, dtype=torch.int64).to(device)
    midx = torch.from_numpy(np.concatenate(idx).astype(np.int32)).to(device)
    return mptr, midx


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
