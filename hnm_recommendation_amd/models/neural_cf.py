"""NeuralCF drop-in (reference: `src/models/neural_cf.py`).

Same constructor, submodules and state_dict keys as the reference (`:18-73`); the
scoring methods run on the HIP library:

* `forward(user_ids, item_ids)` (`:112-141`)      -> hnm_ncf_pair_scores_f32
* `predict_all_items(user_ids)` (`:143-208`)      -> hnm_ncf_scores_f32 (dense [B, I])
* `recommend(user_ids, filter_items)` (`:300-326`) -> hnm_ncf_topk_f32 (fused pair-MLP +
  filter + top-K; never materializes [B, I])
"""
from __future__ import annotations

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
    def _weights(self):
        """(hnm_ncf_weights, tensors it points into).  When every parameter already is a
        contiguous fp32 GPU tensor the struct points at the parameters themselves and is reused
        while their storages are unchanged (keyed on the data pointers: the kernels read the
        values at call time, so in-place updates need no rebuild)."""
        lin = [m for m in self.mlp_layers if isinstance(m, nn.Linear)]
        if len(lin) != 2:
            raise ValueError(
                "the fused NeuralCF kernel covers the reference's two-layer MLP tower "
                f"(mlp_dims of length 3, e.g. [128, 64, 32]); got mlp_dims={self.mlp_dims}")
        l1, l2 = lin
        params = (self.gmf_user_embedding.weight, self.gmf_item_embedding.weight,
                  self.mlp_user_embedding.weight, self.mlp_item_embedding.weight,
                  l1.weight, l1.bias, l2.weight, l2.bias, self.prediction_layer.weight,
                  self.prediction_layer.bias)
        key = tuple(p.data_ptr() for p in params)
        cached = getattr(self, "_wcache", None)
        if cached is not None and cached[0] == key:
            return cached[1], cached[2]
        keep = [f32c(p) for p in params]
        keep[8] = keep[8].reshape(-1)
        _lib.require_gpu(*keep)
        w = _lib.NcfWeights(*[t.data_ptr() for t in keep], self.num_users, self.num_items,
                            self.mf_dim, self.mlp_dims[0] // 2, l1.out_features,
                            l2.out_features)
        if all(t.data_ptr() == p.data_ptr() for t, p in zip(keep, params)):
            self._wcache = (key, w, keep)   # no conversion copies: safe to reuse
        return w, keep

    # ------------------------------------------------------------------ reference API
    def forward(self, user_ids: torch.Tensor, item_ids: torch.Tensor) -> torch.Tensor:
        """Pairwise scores (`neural_cf.py:112-141`); `.squeeze()` semantics kept."""
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
        i, hi = self._ids(item_ids, self.num_items, "item_ids")
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_ncf_pair_scores_f32")(c, w, _lib.ptr(u), _lib.ptr(i), u.numel(),
                                                      _lib.ptr(out)), "hnm_ncf_pair_scores_f32")
        self._check(u.device, hu, hi)
        return out.squeeze()

    def predict_all_items(self, user_ids: torch.Tensor) -> torch.Tensor:
        """Dense scores [B, num_items] (`neural_cf.py:143-208`)."""
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
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
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
        mptr, midx = filter_csr(u, filter_items, self.num_items, u.device)
        kk = min(k, self.num_items)
        if kk <= 0:
            return empty_topk(k, u)
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

    def recommend(self, user_ids: torch.Tensor,
                  filter_items: Optional[Dict[int, set]] = None) -> torch.Tensor:
        """Top-`top_k` item ids per user (`neural_cf.py:300-326`)."""
        self._check_top_k()
        self.eval()
        with torch.no_grad():
            return self.recommend_with_scores(user_ids, filter_items)[1]
