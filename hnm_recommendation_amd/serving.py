"""Serving core: checkpoint ingestion and batched recommendation requests.

Mirrors the model-facing half of the reference's `scripts/serve.py` `ModelServer`
 without the HTTP layer, the pandas data module and the
article-metadata tables (out of scope: SURVEY §2):

* `create_model_from_checkpoint` -- `ModelServer._create_model_from_checkpoint`
  (`serve.py:216-258`): class chosen by a substring of the checkpoint's directory name,
  `hyper_parameters` with num_users / num_items overridden, `load_state_dict`,
  `.to(device).eval()`, LightGCN gets `set_graph`; any failure -> None (logged).
* `load_checkpoints` -- `ModelServer._load_models` (`serve.py:170-209`): every
  `**/*.ckpt` under a directory, model name = parent directory name.  Files are read with
  `torch.load(..., weights_only=True)` (tensors and plain containers only; the reference's
  full unpickling load is not reproduced).
* `Recommender.get_recommendations` / `get_batch_recommendations` -- `serve.py:305-413`.
  The reference scores one user at a time: dense `predict_all_items` [1, I], `-inf` on the
  purchase history (`:350-352`), `torch.topk(num_items)` (`:355`).  Here a batch of users is
  ONE fused call (`recommend_with_scores`: scoring + in-kernel history mask + top-k on the
  GPU); per-user errors (unknown user) become `{"user_id", "error"}` entries as in the
  reference loop (`:396-411`).
"""
from __future__ import annotations

import glob
import logging
import os
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Union

import torch

from .models import LightGCN, MatrixFactorization, NeuralCF, WideDeep
from .models.base import UserHistory

logger = logging.getLogger(__name__)

# serve.py:56: RecommendationRequest.num_items = Field(12, ge=1, le=100)
MAX_NUM_ITEMS = 100

# serve.py:238-248, tested in this order
_DISPATCH = (("matrix_factorization", MatrixFactorization), ("neural_cf", NeuralCF),
             ("wide_deep", WideDeep), ("lightgcn", LightGCN))


def load_checkpoint(path: str, device="cpu") -> Dict:
    """A Lightning `.ckpt` dict ({'state_dict', 'hyper_parameters', ...}); safe loader."""
    return torch.load(path, map_location=device, weights_only=True)


def create_model_from_checkpoint(model_name: str, checkpoint: Dict, num_users: int,
                                 num_items: int, device="cuda", graph=None):
    """`_create_model_from_checkpoint` (`serve.py:216-258`).  `graph` = (edge_index,
    edge_weight) for LightGCN (the data module's `get_graph()`, `:246`).  Returns the module
    in eval mode on `device`, or None when the name matches no model or anything fails."""
    try:
        state_dict = checkpoint["state_dict"]
        hparams = dict(checkpoint.get("hyper_parameters", {}))
        hparams["num_users"] = num_users
        hparams["num_items"] = num_items
        cls = next((c for key, c in _DISPATCH if key in model_name), None)
        if cls is None:
            return None
        model = cls(**hparams)
        if cls is LightGCN:
            if graph is None:
                raise ValueError("LightGCN checkpoint needs the interaction graph")
            edge_index, edge_weight = graph
            model.set_graph(edge_index, edge_weight)
        model.load_state_dict(state_dict)
        model.to(device)
        model.eval()
        return model
    except Exception as e:  # serve.py:255-257: log and skip the model
        logger.error("creating model from checkpoint failed: %s", e)
        return None


class Recommender:
    """The request-facing part of `ModelServer` (`serve.py:116-413`).

    models: {name: module}; model_metrics: {name: {'test_map': ...}} (what the checkpoint's
    'metrics' entry holds, `serve.py:203`); user_history: {user_idx: set(item_idx)} (the
    purchase history, `:166-168`); customer_index: optional {customer_id str: user_idx}
    (the encoder lookup, `:294-300`); article_ids: optional sequence item_idx -> article id.
    """

    def __init__(self, num_users: int, num_items: int, models: Optional[Dict] = None,
                 model_metrics: Optional[Dict[str, Dict[str, float]]] = None,
                 user_history: Optional[Dict[int, set]] = None,
                 customer_index: Optional[Dict[str, int]] = None,
                 article_ids: Optional[Sequence] = None, device="cuda"):
        self.num_users = num_users
        self.num_items = num_items
        self.device = torch.device(device)
        self.models: Dict[str, torch.nn.Module] = {}
        self.model_metrics: Dict[str, Dict[str, float]] = {}
        self.user_history = user_history or {}
        self._history_dev: Optional[UserHistory] = None
        self.customer_index = customer_index
        self.article_ids = article_ids
        for name, m in (models or {}).items():
            self.add_model(name, m, (model_metrics or {}).get(name))

    def add_model(self, name: str, model, metrics: Optional[Dict[str, float]] = None):
        self.models[name] = model.to(self.device).eval()
        if isinstance(model, NeuralCF) and model._fused():
            model.cache_item_tables()  # a server's weights are fixed: keep the item projection
        self.model_metrics[name] = dict(metrics or {})

    def load_checkpoints(self, checkpoint_dir: str, graph=None) -> List[str]:
        """`_load_models` (`serve.py:170-209`): every `**/*.ckpt`, name = parent dir."""
        loaded = []
        for path in sorted(glob.glob(os.path.join(checkpoint_dir, "**", "*.ckpt"),
                                     recursive=True)):
            name = os.path.basename(os.path.dirname(path))
            try:
                ckpt = load_checkpoint(path)
            except Exception as e:
                logger.error("loading %s failed: %s", path, e)
                continue
            model = create_model_from_checkpoint(name, ckpt, self.num_users, self.num_items,
                                                 self.device, graph)
            if model is not None:
                self.models[name] = model
                self.model_metrics[name] = dict(ckpt.get("metrics", {}) or {})
                loaded.append(name)
        return loaded

    def set_user_history(self, user_history: Dict[int, set]):
        """Replace the purchase history (the device copy is rebuilt on the next request)."""
        self.user_history = user_history or {}
        self._history_dev = None

    def _device_history(self) -> Optional[UserHistory]:
        """The purchase history as a device-resident CSR (built once, on first use): each
        filtered batch gathers its rows on the GPU instead of building a mask on the host."""
        if not self.user_history:
            return None
        if self._history_dev is None:
            self._history_dev = UserHistory(self.user_history, self.num_users, self.num_items,
                                            self.device)
        return self._history_dev

    # ------------------------------------------------------------------ lookups
    def get_user_idx(self, user_id: Union[int, str]) -> Optional[int]:
        """`serve.py:282-303`: ints are indices (< num_users); strings go through the
        customer-id index."""
        if isinstance(user_id, bool):
            user_id = int(user_id)
        if isinstance(user_id, int):
            return user_id if user_id < self.num_users else None
        if self.customer_index is not None:
            return self.customer_index.get(user_id)
        return None

    def _get_best_model(self) -> str:
        """`serve.py:415-430`: highest 'test_map'; without any, the reference falls back
        to its popularity baseline (out of scope here) -- we take the first model."""
        best, best_score = None, 0
        for name, m in self.model_metrics.items():
            if "test_map" in m and m["test_map"] > best_score:
                best, best_score = name, m["test_map"]
        if best is None:
            if not self.models:
                raise ValueError("no model loaded")
            best = next(iter(self.models))
        return best

    def _resolve_model(self, model_name: str):
        if model_name == "best":
            model_name = self._get_best_model()
        if model_name not in self.models:
            raise ValueError(f"model {model_name} is not available")
        return model_name, self.models[model_name]

    def _item_info(self, item_idx: int, score: Optional[float]) -> Dict:
        """`ItemInfo` (`serve.py:80-88`) without the article metadata table."""
        aid = str(item_idx)
        if self.article_ids is not None and 0 <= item_idx < len(self.article_ids):
            aid = str(self.article_ids[item_idx])
        return {"article_id": aid, "product_name": None, "product_type_name": None,
                "product_group_name": None, "colour_group_name": None,
                "department_name": None, "score": score}

    # ------------------------------------------------------------------ requests
    def _score_batch(self, model, idx: List[int], num_items: int, filter_purchased: bool):
        # serve.py:56 RecommendationRequest: num_items = Field(12, ge=1, le=100)
        hi = min(MAX_NUM_ITEMS, self.num_items)
        if isinstance(num_items, bool) or not isinstance(num_items, int) or not 1 <= num_items <= hi:
            raise ValueError(f"num_items must be an integer in [1, {hi}]")
        # host ids: range-checked on the host by the model (no device-side check / sync),
        # then one fused scoring + history-mask + top-k call; the history mask is gathered
        # on the GPU from the device-resident history (serve.py:350-352)
        users = torch.tensor(idx, dtype=torch.int64)
        hist = self._device_history() if filter_purchased else None
        with torch.no_grad():
            vals, items = model.recommend_with_scores(users, filter_items=hist, k=num_items)
        return vals.cpu().tolist(), items.cpu().tolist()

    def _result(self, user_id, model_name, vals, items, include_scores):
        recs = [self._item_info(int(i), float(v) if include_scores else None)
                for v, i in zip(vals, items)]
        return {"user_id": user_id, "recommendations": recs, "model_name": model_name,
                "generated_at": datetime.now().isoformat()}

    def get_recommendations(self, user_id: Union[int, str], model_name: str = "best",
                            num_items: int = 12, filter_purchased: bool = True,
                            include_scores: bool = False) -> Dict:
        """`serve.py:305-371` (ValueError for an unknown user or model)."""
        uidx = self.get_user_idx(user_id)
        if uidx is None:
            raise ValueError(f"user {user_id} not found")
        name, model = self._resolve_model(model_name)
        vals, items = self._score_batch(model, [uidx], num_items, filter_purchased)
        return self._result(user_id, name, vals[0], items[0], include_scores)

    def get_batch_recommendations(self, user_ids: List[Union[int, str]],
                                  model_name: str = "best", num_items: int = 12,
                                  filter_purchased: bool = True,
                                  include_scores: bool = False) -> List[Dict]:
        """`serve.py:373-413`, batched: one fused scoring + mask + top-k call for all
        known users; unknown users get {'user_id', 'error'} in their slot."""
        name, model = self._resolve_model(model_name)
        idx, slots, results = [], [], []
        for j, uid in enumerate(user_ids):
            u = self.get_user_idx(uid)
            if u is None:
                results.append({"user_id": uid, "error": f"user {uid} not found"})
            elif u < 0:  # the reference's embedding lookup raises; its loop records it
                results.append({"user_id": uid, "error": "index out of range in self"})
            else:
                results.append(None)
                idx.append(u)
                slots.append(j)
        if idx:
            vals, items = self._score_batch(model, idx, num_items, filter_purchased)
            for r, j in enumerate(slots):
                results[j] = self._result(user_ids[j], name, vals[r], items[r], include_scores)
        return results
