"""WideDeep drop-in (reference: `src/models/wide_deep.py`).

Same constructor, submodules and state_dict keys (`:19-155`).  Scoring runs on the HIP
library (hnm_widedeep_*): the one-hot wide input becomes two weight lookups, eval-mode
BatchNorm is folded into the next layer, layer 1 is decomposed into per-user and per-item
projections, and layers 2-3 run as fp32 MFMA chains fused with the top-K.

* `forward(user_ids, item_ids, user_features, item_features)` (`:157-230`)
* `predict_all_items(user_ids, user_features)` (`:232-285`)
* `recommend(user_ids, user_features, filter_items)` (`:405-435`)
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import _lib
from ..evaluation import RecommendationMetrics
from .base import RecModule, dense_topk, empty_topk, f32c, filter_csr


class WideDeep(RecModule):
    def __init__(
        self,
        num_users: int,
        num_items: int,
        num_user_features: int = 0,
        num_item_features: int = 0,
        embedding_dim: int = 64,
        deep_layers: List[int] = [512, 256, 128],
        dropout: float = 0.1,
        use_wide_user_item: bool = True,
        use_wide_features: bool = True,
        learning_rate: float = 0.001,
        weight_decay: float = 0.0001,
        top_k: int = 12,
    ):
        super().__init__()
        self.save_hyperparameters()
        self.num_users = num_users
        self.num_items = num_items
        self.num_user_features = num_user_features
        self.num_item_features = num_item_features
        self.embedding_dim = embedding_dim
        self.deep_layers = deep_layers
        self.dropout = dropout
        self.use_wide_user_item = use_wide_user_item
        self.use_wide_features = use_wide_features
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.top_k = top_k
        self._build_wide_component()
        self._build_deep_component()
        self.final_layer = nn.Linear(self._calculate_wide_dim() + deep_layers[-1], 1)
        self._init_weights()
        self.metrics = RecommendationMetrics(top_k=top_k)

    def _calculate_wide_dim(self) -> int:
        """`wide_deep.py:83-90`."""
        dim = 0
        if self.use_wide_user_item:
            dim += self.num_users + self.num_items
        if self.use_wide_features:
            dim += self.num_user_features + self.num_item_features
        return dim

    def _build_wide_component(self):
        """`wide_deep.py:92-103` (the wide embeddings are created but unused by forward)."""
        if self.use_wide_user_item:
            self.wide_user_embedding = nn.Embedding(self.num_users, 1)
            self.wide_item_embedding = nn.Embedding(self.num_items, 1)
        if self.use_wide_features and self.num_user_features > 0:
            self.wide_user_features = nn.Linear(self.num_user_features, self.num_user_features)
        if self.use_wide_features and self.num_item_features > 0:
            self.wide_item_features = nn.Linear(self.num_item_features, self.num_item_features)

    def _build_deep_component(self):
        """`wide_deep.py:105-134`: [Linear -> ReLU -> BatchNorm1d -> Dropout] per layer."""
        d = self.embedding_dim
        self.deep_user_embedding = nn.Embedding(self.num_users, d)
        self.deep_item_embedding = nn.Embedding(self.num_items, d)
        if self.num_user_features > 0:
            self.deep_user_features = nn.Linear(self.num_user_features, d)
        if self.num_item_features > 0:
            self.deep_item_features = nn.Linear(self.num_item_features, d)
        prev = 2 * d + (d if self.num_user_features > 0 else 0) + (d if self.num_item_features > 0 else 0)
        layers = []
        for hidden in self.deep_layers:
            layers += [nn.Linear(prev, hidden), nn.ReLU(), nn.BatchNorm1d(hidden),
                       nn.Dropout(self.dropout)]
            prev = hidden
        self.deep_network = nn.Sequential(*layers)

    def _init_weights(self):
        """`wide_deep.py:136-155`."""
        if self.use_wide_user_item:
            nn.init.xavier_uniform_(self.wide_user_embedding.weight)
            nn.init.xavier_uniform_(self.wide_item_embedding.weight)
        nn.init.xavier_uniform_(self.deep_user_embedding.weight)
        nn.init.xavier_uniform_(self.deep_item_embedding.weight)
        for layer in self.deep_network:
            if isinstance(layer, nn.Linear):
                nn.init.xavier_uniform_(layer.weight)
                nn.init.zeros_(layer.bias)
        nn.init.xavier_uniform_(self.final_layer.weight)
        nn.init.zeros_(self.final_layer.bias)

    # ------------------------------------------------------------------ HIP plumbing
    def _wide_zero(self, n, device):
        """use_wide_user_item=False: the one-hot wide terms are absent (wide_deep.py:179-188);
        the kernels read an all-zero wide vector instead (adding +0.0 changes no score)."""
        z = getattr(self, "_zeros", None)
        if z is None or z.numel() < n or z.device != device:
            z = torch.zeros(max(n, self.num_users, self.num_items), dtype=torch.float32,
                            device=device)
            self._zeros = z
        return z

    def _weights(self):
        lin = [m for m in self.deep_network if isinstance(m, nn.Linear)]
        bns = [m for m in self.deep_network if isinstance(m, nn.BatchNorm1d)]
        if len(lin) not in (2, 3):
            raise ValueError(f"the fused Wide&Deep kernel covers 2- or 3-layer deep towers; "
                             f"got deep_layers={self.deep_layers}")
        keep = []

        def t(x):
            if x is None:
                return None
            y = f32c(x)
            keep.append(y)
            return y.data_ptr()

        def bn(m):
            return [t(m.weight), t(m.bias), t(m.running_mean), t(m.running_var)]

        has3 = len(lin) == 3
        none4 = [None] * 4
        U, I = self.num_users, self.num_items
        fw = t(self.final_layer.weight.reshape(-1))  # [wide_dim + last]
        duf = getattr(self, "deep_user_features", None)
        wuf = getattr(self, "wide_user_features", None) if self.use_wide_features else None
        # final_layer input order (wide_deep.py:225): [user one-hot | item one-hot]
        # (use_wide_user_item), [user features | item features] (use_wide_features), deep
        feat0 = U + I if self.use_wide_user_item else 0
        if self.use_wide_user_item:
            wu, wi = fw, fw + 4 * U
        else:
            z = self._wide_zero(max(U, I), self.final_layer.weight.device)
            wu = wi = z.data_ptr()
        ptrs = [t(self.deep_user_embedding.weight), t(self.deep_item_embedding.weight),
                t(lin[0].weight), t(lin[0].bias), *bn(bns[0]),
                t(lin[1].weight), t(lin[1].bias), *bn(bns[1]),
                t(lin[2].weight) if has3 else None, t(lin[2].bias) if has3 else None,
                *(bn(bns[2]) if has3 else none4),
                wu, wi, (fw + 4 * feat0) if wuf is not None else None,
                fw + 4 * self._calculate_wide_dim(), t(self.final_layer.bias),
                t(duf.weight) if duf is not None else None, t(duf.bias) if duf is not None else None,
                t(wuf.weight) if wuf is not None else None, t(wuf.bias) if wuf is not None else None]
        _lib.require_gpu(*keep)
        d = self.embedding_dim
        w = _lib.WideDeepWeights(*ptrs, self.num_users, self.num_items, d,
                                 lin[0].in_features, lin[0].out_features, lin[1].out_features,
                                 lin[2].out_features if has3 else 0, self.num_user_features,
                                 float(bns[0].eps))
        return w, keep

    def _item_feature_weights(self, keep):
        """hnm_widedeep_item_features of a model with num_item_features > 0."""
        dif = self.deep_item_features
        wif = getattr(self, "wide_item_features", None) if self.use_wide_features else None
        fw = self.final_layer.weight.reshape(-1)
        off = (self.num_users + self.num_items if self.use_wide_user_item else 0) + \
            (self.num_user_features if self.use_wide_features else 0)
        vals = [f32c(dif.weight), f32c(dif.bias)]
        if wif is not None:
            vals += [f32c(wif.weight), f32c(wif.bias),
                     f32c(fw[off: off + self.num_item_features])]
        keep.extend(vals)
        ptrs = [v.data_ptr() for v in vals] + [None] * (5 - len(vals))
        return _lib.WideDeepItemFeatures(*ptrs, self.num_item_features)

    def _features(self, user_features, n, device):
        if self.num_item_features > 0:
            raise ValueError("predict_all_items/recommend cannot use item features: the "
                             "reference passes item_features=None there (wide_deep.py:275) and "
                             "its deep input then does not match the network")
        if self.num_user_features == 0:
            return None
        if user_features is None:
            raise ValueError("user_features are required when num_user_features > 0")
        f = f32c(user_features).to(device)
        if f.shape != (n, self.num_user_features):
            raise ValueError(f"user_features must be [{n}, {self.num_user_features}]")
        return f

    # ------------------------------------------------------------------ reference API
    def forward(self, user_ids, item_ids, user_features=None, item_features=None):
        """Pairwise scores (`wide_deep.py:157-230`), user and item side features included.
        As in the reference, a model built with features needs them: its deep network's
        input width counts them (`:118-123`)."""
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
        i, hi = self._ids(item_ids, self.num_items, "item_ids")
        f = fi = None
        if self.num_user_features > 0:
            if user_features is None:
                raise ValueError("user_features are required when num_user_features > 0")
            f = f32c(user_features).to(u.device)
            if f.shape != (u.numel(), self.num_user_features):
                raise ValueError(f"user_features must be [{u.numel()}, {self.num_user_features}]")
        itf = None
        if self.num_item_features > 0:
            if item_features is None:
                raise ValueError("item_features are required when num_item_features > 0")
            fi = f32c(item_features).to(u.device)
            if fi.shape != (u.numel(), self.num_item_features):
                raise ValueError(f"item_features must be [{u.numel()}, {self.num_item_features}]")
            itf = self._item_feature_weights(keep)
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_widedeep_pair_scores_ex_f32")(
            c, w, None if itf is None else C.byref(itf), _lib.ptr(u), _lib.ptr(i), _lib.ptr(f),
            _lib.ptr(fi), u.numel(), _lib.ptr(out)), "hnm_widedeep_pair_scores_ex_f32")
        self._check(u.device, hu, hi)
        return out.squeeze()

    def predict_all_items(self, user_ids, user_features=None):
        """Dense scores [B, num_items] (`wide_deep.py:232-285`)."""
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
        f = self._features(user_features, u.numel(), u.device)
        out = torch.empty(u.numel(), self.num_items, dtype=torch.float32, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_widedeep_scores_f32")(c, w, _lib.ptr(u), u.numel(), _lib.ptr(f),
                                                      _lib.ptr(out), out.stride(0)),
                   "hnm_widedeep_scores_f32")
        self._check(u.device, hu)
        return out

    def recommend_with_scores(self, user_ids, user_features=None,
                              filter_items: Optional[Dict[int, set]] = None,
                              k: Optional[int] = None):
        k = self.top_k if k is None else k
        w, keep = self._weights()
        u, hu = self._ids(user_ids, self.num_users)
        f = self._features(user_features, u.numel(), u.device)
        mptr, midx = filter_csr(u, filter_items, self.num_items, u.device)
        kk = min(k, self.num_items)
        if kk <= 0:
            return empty_topk(k, u)
        if kk > 64:
            return dense_topk(self.predict_all_items(u, user_features), kk, mptr, midx)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_widedeep_topk_f32")(c, w, _lib.ptr(u), u.numel(), _lib.ptr(f),
                                                    _lib.ptr(mptr), _lib.ptr(midx), kk,
                                                    _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_widedeep_topk_f32")
        self._check(u.device, hu)
        return out_v, out_i

    def _validation_topk(self, batch):
        """`predict_all_items(user_ids, user_features)` + torch.topk of the reference's
        validation_step (wide_deep.py:314-332), as the fused top-K."""
        return self.recommend_with_scores(batch["user_ids"], batch.get("user_features"),
                                          k=self.top_k)[1]

    def recommend(self, user_ids, user_features=None,
                  filter_items: Optional[Dict[int, set]] = None):
        """Top-`top_k` item ids per user (`wide_deep.py:405-435`)."""
        self._check_top_k()
        self.eval()
        with torch.no_grad():
            return self.recommend_with_scores(user_ids, user_features, filter_items)[1]
