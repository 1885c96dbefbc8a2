"""MatrixFactorization drop-in (reference: `src/models/matrix_factorization.py`).

SURVEY §8(f) row 1: the same fused dot-score + top-K kernel as LightGCN with the bias
epilogue s = u.i + b_u + b_i + g (`:108-131`).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .. import _lib
from ..evaluation import RecommendationMetrics
from .base import RecModule, dense_topk, empty_topk, f32c, filter_csr


class MatrixFactorization(RecModule):
    def __init__(
        self,
        num_users: int,
        num_items: int,
        embedding_dim: int = 64,
        learning_rate: float = 0.001,
        weight_decay: float = 0.01,
        top_k: int = 12,
        sparse: bool = True,
    ):
        super().__init__()
        self.save_hyperparameters()
        self.num_users = num_users
        self.num_items = num_items
        self.embedding_dim = embedding_dim
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.top_k = top_k
        self.user_embeddings = nn.Embedding(num_users, embedding_dim, sparse=sparse)
        self.item_embeddings = nn.Embedding(num_items, embedding_dim, sparse=sparse)
        self.user_bias = nn.Embedding(num_users, 1)
        self.item_bias = nn.Embedding(num_items, 1)
        self.global_bias = nn.Parameter(torch.zeros(1))
        self._init_weights()
        self.metrics = RecommendationMetrics(top_k=top_k)

    def _init_weights(self):
        """Reference init (`matrix_factorization.py:73-78`)."""
        nn.init.normal_(self.user_embeddings.weight, std=0.01)
        nn.init.normal_(self.item_embeddings.weight, std=0.01)
        nn.init.zeros_(self.user_bias.weight)
        nn.init.zeros_(self.item_bias.weight)

    def _tabs(self):
        t = (f32c(self.user_embeddings.weight), f32c(self.item_embeddings.weight),
             f32c(self.user_bias.weight).reshape(-1), f32c(self.item_bias.weight).reshape(-1),
             f32c(self.global_bias))
        _lib.require_gpu(*t)
        return t

    def forward(self, user_ids: torch.Tensor, item_ids: torch.Tensor) -> torch.Tensor:
        """u.i + b_u + b_i + g per pair (`matrix_factorization.py:80-106`)."""
        U, V, ub, ib, gb = self._tabs()
        u, hu = self._ids(user_ids, self.num_users)
        i, hi = self._ids(item_ids, self.num_items, "item_ids")
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_pair_dot_f32")(c, _lib.ptr(U), self.num_users, d, _lib.ptr(V),
                                               self.num_items, d, d, _lib.ptr(u), _lib.ptr(i),
                                               u.numel(), _lib.ptr(ub), _lib.ptr(ib),
                                               _lib.ptr(gb), _lib.ptr(out)), "hnm_pair_dot_f32")
        self._check(u.device, hu, hi)
        return out

    def predict_all_items(self, user_ids: torch.Tensor) -> torch.Tensor:
        U, V, ub, ib, gb = self._tabs()
        u, hu = self._ids(user_ids, self.num_users)
        out = torch.empty(u.numel(), self.num_items, dtype=torch.float32, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_dot_scores_f32")(c, _lib.ptr(U), self.num_users, d, _lib.ptr(u),
                                                 u.numel(), _lib.ptr(V), self.num_items, d, d,
                                                 _lib.ptr(ub), _lib.ptr(ib), _lib.ptr(gb),
                                                 _lib.ptr(out), out.stride(0)),
                   "hnm_dot_scores_f32")
        self._check(u.device, hu)
        return out

    def recommend_with_scores(self, user_ids, filter_items: Optional[Dict[int, set]] = None,
                              k: Optional[int] = None):
        k = self.top_k if k is None else k
        U, V, ub, ib, gb = self._tabs()
        u, hu = self._ids(user_ids, self.num_users)
        mptr, midx = filter_csr(u, filter_items, self.num_items, u.device)
        kk = min(k, self.num_items)
        if kk <= 0:
            return empty_topk(k, u)
        if kk > 64:
            return dense_topk(self.predict_all_items(u), kk, mptr, midx)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_dot_topk_f32")(c, _lib.ptr(U), self.num_users, d, _lib.ptr(u),
                                               u.numel(), _lib.ptr(V), self.num_items, d, d,
                                               _lib.ptr(ub), _lib.ptr(ib), _lib.ptr(gb),
                                               _lib.ptr(mptr), _lib.ptr(midx), kk,
                                               _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_dot_topk_f32")
        self._check(u.device, hu)
        return out_v, out_i

    def recommend(self, user_ids, filter_items: Optional[Dict[int, set]] = None):
        """Top-`top_k` item ids per user (`matrix_factorization.py:220-246`)."""
        self._check_top_k()
        self.eval()
        with torch.no_grad():
            return self.recommend_with_scores(user_ids, filter_items)[1]
