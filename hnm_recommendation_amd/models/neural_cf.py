"""NeuralCF drop-in (reference: `src/models/neural_cf.py`).

Same constructor, submodules and state_dict keys as the reference (`:18-73`); the
scoring methods run on the HIP library:

* `forward(user_ids, item_ids)` (`:112-141`)      -> hnm_ncf_pair_scores_f32
* `predict_all_items(user_ids)` (`:143-208`)      -> hnm_ncf_scores_f32 (dense [B, I])
* `recommend(user_ids, filter_items)` (`:300-326`) -> hnm_ncf_topk_f32 (fused pair-MLP +
  filter + top-K; never materializes [B, I])

Those fused kernels take the reference's default two-layer tower (mlp_dims of length 3 with
h1 <= 128, h2 <= 32, mf <= 128).  Any other tower `_build_mlp` accepts (`:75-90`: one
Linear -> ReLU per consecutive pair of mlp_dims, e.g. [64, 32] or [128, 64, 32, 16]) runs the
exact fp32 deep-tower kernels: pair scores for forward and dense rows for predict_all_items
(hnm_ncf_deep_scores_f32), and for recommend with k <= 64 the fused deep top-k
(hnm_ncf_deep_topk_f32: f32-MFMA layer chains over item tiles with per-partition top-k lists for
towers of widths <= 64, dense chunks + the row top-k inside the C entry for wider ones); k > 64
takes dense rows + the row top-k kernel.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import _lib
from ..evaluation import RecommendationMetrics
from .base import RecModule, dense_topk, empty_topk, f32c, filter_csr


class NeuralCF(RecModule):
    def __init__(
        self,
        num_users: int,
        num_items: int,
        mf_dim: int = 64,
        mlp_dims: List[int] = [128, 64, 32],
        dropout: float = 0.1,
        learning_rate: float = 0.001,
        weight_decay: float = 0.0001,
        top_k: int = 12,
        use_pretrain: bool = False,
    ):
        super().__init__()
        self.save_hyperparameters()
        self.num_users = num_users
        self.num_items = num_items
        self.mf_dim = mf_dim
        self.mlp_dims = mlp_dims
        self.dropout = dropout
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.top_k = top_k
        self.gmf_user_embedding = nn.Embedding(num_users, mf_dim)
        self.gmf_item_embedding = nn.Embedding(num_items, mf_dim)
        self.mlp_user_embedding = nn.Embedding(num_users, mlp_dims[0] // 2)
        self.mlp_item_embedding = nn.Embedding(num_items, mlp_dims[0] // 2)
        self.mlp_layers = self._build_mlp(mlp_dims, dropout)
        self.prediction_layer = nn.Linear(mf_dim + mlp_dims[-1], 1)
        self._init_weights()
        self.metrics = RecommendationMetrics(top_k=top_k)

    def _build_mlp(self, dims: List[int], dropout: float) -> nn.Sequential:
        """Linear -> ReLU -> Dropout per consecutive pair of dims (`neural_cf.py:75-90`)."""
        layers = []
        for i in range(len(dims) - 1):
            layers += [nn.Linear(dims[i], dims[i + 1]), nn.ReLU(), nn.Dropout(dropout)]
        return nn.Sequential(*layers)

    def _init_weights(self):
        """Reference init (`neural_cf.py:92-110`)."""
        nn.init.normal_(self.gmf_user_embedding.weight, std=0.01)
        nn.init.normal_(self.gmf_item_embedding.weight, std=0.01)
        nn.init.xavier_uniform_(self.mlp_user_embedding.weight)
        nn.init.xavier_uniform_(self.mlp_item_embedding.weight)
        for layer in self.mlp_layers:
            if isinstance(layer, nn.Linear):
                nn.init.xavier_uniform_(layer.weight)
                nn.init.zeros_(layer.bias)
        nn.init.xavier_uniform_(self.prediction_layer.weight)
        nn.init.zeros_(self.prediction_layer.bias)

    # ------------------------------------------------------------------ HIP plumbing
    def _linears(self):
        return [m for m in self.mlp_layers if isinstance(m, nn.Linear)]

    def _fused(self) -> bool:
        """Whether the fused (certified) kernels take this tower: two Linear layers within
        their register budget -- the reference default [128, 64, 32] with mf 64."""
        lin = self._linears()
        return (len(lin) == 2 and lin[0].out_features <= 128 and lin[1].out_features <= 32
                and 1 <= self.mf_dim <= 128)

    def _deep_weights(self):
        """(hnm_ncf_deep_weights, tensors it points into) for towers of any depth."""
        lin = self._linears()
        if not 1 <= len(lin) <= 8:
            raise ValueError(f"NeuralCF: 1..8 MLP layers supported, got mlp_dims={self.mlp_dims}")
        keep = [f32c(p) for p in (self.gmf_user_embedding.weight, self.gmf_item_embedding.weight,
                                  self.mlp_user_embedding.weight, self.mlp_item_embedding.weight)]
        ws = [f32c(m.weight) for m in lin]
        bs = [f32c(m.bias) for m in lin]
        wp, bp = f32c(self.prediction_layer.weight).reshape(-1), f32c(self.prediction_layer.bias)
        keep += ws + bs + [wp, bp]
        _lib.require_gpu(*keep)
        w = _lib.NcfDeepWeights()
        w.gmf_user, w.gmf_item, w.mlp_user, w.mlp_item = (t.data_ptr() for t in keep[:4])
        for j, (a, b) in enumerate(zip(ws, bs)):
            w.w[j], w.b[j] = a.data_ptr(), b.data_ptr()
        w.wp, w.bp = wp.data_ptr(), bp.data_ptr()
        w.num_users, w.num_items, w.mf, w.nl = self.num_users, self.num_items, self.mf_dim, len(lin)
        dims = [lin[0].in_features] + [m.out_features for m in lin]
        for j, v in enumerate(dims):
            w.dims[j] = v
        return w, keep

    def _deep_scores(self, u, items=None, out=None):
        w, keep = self._deep_weights()
        B = u.numel()
        if out is None:
            out = torch.empty(B, self.num_items if items is None else 1, dtype=torch.float32,
                              device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_ncf_deep_scores_f32")(
            c, C.byref(w), _lib.ptr(u), B, _lib.ptr(items), _lib.ptr(out),
            out.stride(0) if items is None else 1), "hnm_ncf_deep_scores_f32")
        return out

    def _weights(self):
        """(hnm_ncf_weights, tensors it points into).  When every parameter already is a
        contiguous fp32 GPU tensor the struct points at the parameters themselves and is reused
        while their storages are unchanged (keyed on the data pointers: the kernels read the
        values at call time, so in-place updates need no rebuild)."""
        if not self._fused():
            raise ValueError(
                "the fused NeuralCF kernels cover the reference's two-layer MLP tower "
                f"(h1 <= 128, h2 <= 32); mlp_dims={self.mlp_dims} runs the deep-tower path")
        l1, l2 = self._linears()
        params = (self.gmf_user_embedding.weight, self.gmf_item_embedding.weight,
                  self.mlp_user_embedding.weight, self.mlp_item_embedding.weight,
                  l1.weight, l1.bias, l2.weight, l2.bias, self.prediction_layer.weight,
                  self.prediction_layer.bias)
        key = tuple(p.data_ptr() for p in params)
        cached = getattr(self, "_wcache", None)
        if cached is not None and cached[0] == key:
            self._attach_item_proj(cached[1], cached[2])
            return cached[1], cached[2]
        keep = [f32c(p) for p in params]
        keep[8] = keep[8].reshape(-1)
        _lib.require_gpu(*keep)
        w = _lib.NcfWeights(*[t.data_ptr() for t in keep], self.num_users, self.num_items,
                            self.mf_dim, self.mlp_dims[0] // 2, l1.out_features,
                            l2.out_features)
        if all(t.data_ptr() == p.data_ptr() for t, p in zip(keep, params)):
            self._wcache = (key, w, keep)   # no conversion copies: safe to reuse
        self._attach_item_proj(w, keep)
        return w, keep

    def cache_item_tables(self, enabled: bool = True) -> "NeuralCF":
        """Keep the item half of layer 1 (W1[:, h0:] m_i for every item, 27 MB at the H&M
        catalogue) between calls instead of recomputing it in every recommend call (22 us of
        kernel time a call: most of a B = 1 request's scoring).  For frozen weights -- a server
        (`serving.Recommender` turns it on); the cache is keyed on the item table's and W1's
        storage and torch version counters, so in-place updates through the parameters
        (optimizer steps, load_state_dict) rebuild it, but writes through `.data` do not."""
        self._item_cache_on = bool(enabled)
        if not enabled:
            cached = getattr(self, "_wcache", None)
            if cached is not None:
                cached[1].item_proj = None      # the cached struct no longer points into it
            self._release_item_proj()
        return self

    def _release_item_proj(self):
        """Drop the cached projection once no stream can still read it: kernels of other
        threads' streams (or an open two-phase shard call) may hold its address, and the
        caching allocator would hand the block out again on the allocating stream alone."""
        old = getattr(self, "_item_proj", None)
        self._item_proj = None
        if old is not None:
            torch.cuda.synchronize(old[1].device)

    def _attach_item_proj(self, w, keep):
        if not getattr(self, "_item_cache_on", False):
            w.item_proj = None
            return
        mi, w1 = self.mlp_item_embedding.weight, self._linears()[0].weight
        key = (mi.data_ptr(), mi._version, w1.data_ptr(), w1._version, self.num_items)
        cached = getattr(self, "_item_proj", None)
        if cached is None or cached[0] != key:
            if cached is not None:
                self._release_item_proj()
            w.item_proj = None
            h1p = 128 if (w.h1 > 64 or w.mf > 64) else 64
            proj = torch.empty(self.num_items, h1p, dtype=torch.float32, device=keep[0].device)
            _lib.check(_lib.fn("hnm_ncf_item_proj_f32")(_lib.ctx(proj.device), C.byref(w),
                                                        _lib.ptr(proj)), "hnm_ncf_item_proj_f32")
            # other threads' streams read the cache as soon as it is published: complete it first
            torch.cuda.current_stream(proj.device).synchronize()
            cached = self._item_proj = (key, proj)
        w.item_proj = cached[1].data_ptr()

    # ------------------------------------------------------------------ reference API
    def forward(self, user_ids: torch.Tensor, item_ids: torch.Tensor) -> torch.Tensor:
        """Pairwise scores (`neural_cf.py:112-141`); `.squeeze()` semantics kept."""
        u, hu = self._ids(user_ids, self.num_users)
        i, hi = self._ids(item_ids, self.num_items, "item_ids")
        if u.numel() != i.numel():
            raise ValueError("user_ids and item_ids must have the same length")
        if not self._fused():
            out = self._deep_scores(u, i).reshape(-1)
            self._check(u.device, hu, hi)
            return out.squeeze()
        w, keep = self._weights()
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_ncf_pair_scores_f32")(c, w, _lib.ptr(u), _lib.ptr(i), u.numel(),
                                                      _lib.ptr(out)), "hnm_ncf_pair_scores_f32")
        self._check(u.device, hu, hi)
        return out.squeeze()

    def predict_all_items(self, user_ids: torch.Tensor) -> torch.Tensor:
        """Dense scores [B, num_items] (`neural_cf.py:143-208`)."""
        u, hu = self._ids(user_ids, self.num_users)
        if not self._fused():
            out = self._deep_scores(u)
            self._check(u.device, hu)
            return out
        w, keep = self._weights()
        out = torch.empty(u.numel(), self.num_items, dtype=torch.float32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_ncf_scores_f32")(c, w, _lib.ptr(u), u.numel(), _lib.ptr(out),
                                                 out.stride(0)), "hnm_ncf_scores_f32")
        self._check(u.device, hu)
        return out

    def recommend_with_scores(self, user_ids: torch.Tensor,
                              filter_items: Optional[Dict[int, set]] = None,
                              k: Optional[int] = None):
        """(scores [B, k], items [B, k]) sorted by score desc, item asc."""
        k = self.top_k if k is None else k
        u, hu = self._ids(user_ids, self.num_users)
        mptr, midx = filter_csr(u, filter_items, self.num_items, u.device)
        kk = min(k, self.num_items)
        if kk <= 0:
            return empty_topk(k, u)
        if not self._fused():
            return self._deep_topk(u, hu, kk, mptr, midx)
        w, keep = self._weights()
        if kk > 64:  # serve path k up to 100 (serve.py:56): dense + row top-k kernel
            scores = self.predict_all_items(u)
            return dense_topk(scores, kk, mptr, midx)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_ncf_topk_f32")(c, w, _lib.ptr(u), u.numel(), _lib.ptr(mptr),
                                               _lib.ptr(midx), kk, _lib.ptr(out_v),
                                               _lib.ptr(out_i)), "hnm_ncf_topk_f32")
        self._check(u.device, hu)
        return out_v, out_i

    def _deep_topk(self, u, hu, k, mptr, midx):
        """Deep towers: hnm_ncf_deep_topk_f32 for k <= 64 (the fp32-MFMA scan with fused
        per-partition top-k lists where the tower's widths are <= 64, else dense rows per user
        chunk in the library's workspace + the row top-k kernel); k > 64 (serve path, up to
        100): dense rows for a chunk of users (<= 256 MB of scores) + the row top-k kernel with
        the chunk's slice of the CSR mask (absolute offsets into mask_idx)."""
        B = u.numel()
        out_v = torch.empty(B, k, dtype=torch.float32, device=u.device)
        out_i = torch.empty(B, k, dtype=torch.int64, device=u.device)
        if k <= 64:
            w, keep = self._deep_weights()
            c = _lib.ctx(u.device)
            _lib.check(_lib.fn("hnm_ncf_deep_topk_f32")(
                c, C.byref(w), _lib.ptr(u), B, _lib.ptr(mptr), _lib.ptr(midx), k,
                _lib.ptr(out_v), _lib.ptr(out_i)), "hnm_ncf_deep_topk_f32")
            self._check(u.device, hu)
            return out_v, out_i
        step = max(1, min(B, 65535, (1 << 26) // max(self.num_items, 1)))
        buf = torch.empty(step, self.num_items, dtype=torch.float32, device=u.device)
        for b0 in range(0, B, step):
            b1 = min(B, b0 + step)
            sc = self._deep_scores(u[b0:b1], out=buf[: b1 - b0])
            v, i = dense_topk(sc, k, None if mptr is None else mptr[b0:b1 + 1], midx)
            out_v[b0:b1] = v
            out_i[b0:b1] = i
        self._check(u.device, hu)
        return out_v, out_i

    def recommend(self, user_ids: torch.Tensor,
                  filter_items: Optional[Dict[int, set]] = None) -> torch.Tensor:
        """Top-`top_k` item ids per user (`neural_cf.py:300-326`)."""
        self._check_top_k()
        self.eval()
        with torch.no_grad():
            return self.recommend_with_scores(user_ids, filter_items)[1]
