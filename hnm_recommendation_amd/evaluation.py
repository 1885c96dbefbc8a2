"""`RecommendationMetrics` -- the class every reference model imports
(`neural_cf.py:6`, `lightgcn.py:10`, `wide_deep.py:6`, `matrix_factorization.py:7`) but
the published snapshot does not define.  Keys follow its callers
(`benchmark_models.py:203-206`, `train.py:257-260`): map_at_k, recall_at_k,
precision_at_k, ndcg_at_k.  Per-user formulas are those of `src/evaluation/metrics.py`
(MAP `:49-62`, Recall `:95-100`, Precision `:133-137`, NDCG `:176-186`).

This is a consumer of the top-K output, host-side bookkeeping on
K=12 indices per user, not part of the scoring hot path.
"""
from __future__ import annotations

import numpy as np
import torch


def _rows(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    out = []
    for r in x:
        r = np.asarray(r).reshape(-1)
        out.append([int(v) for v in r if v >= 0])
    return out


class RecommendationMetrics:
    def __init__(self, top_k: int = 12):
        self.top_k = top_k
        self.reset()

    def reset(self):
        self._ap = self._rec = self._prec = self._ndcg = 0.0
        self._n_ap = self._n_rec = self._n_prec = self._n_ndcg = 0

    def update(self, top_k_items, ground_truth):
        k = self.top_k
        for pred, true in zip(_rows(top_k_items), _rows(ground_truth)):
            pred = pred[:k]
            tset = set(true)
            hits_flags = [p in tset for p in pred]
            # MAP@K (metrics.py:49-62): 0 for users with no ground truth, still counted
            if tset:
                nh, s = 0.0, 0.0
                for i, h in enumerate(hits_flags):
                    if h:
                        nh += 1.0
                        s += nh / (i + 1.0)
                self._ap += s / min(len(tset), k)
            self._n_ap += 1
            hits = sum(hits_flags)
            if tset:  # Recall@K (metrics.py:95-100)
                self._rec += hits / len(tset)
                self._n_rec += 1
            self._prec += hits / len(pred) if pred else 0.0  # Precision@K (:133-137)
            self._n_prec += 1
            if tset:  # NDCG@K (:176-186)
                dcg = sum(1.0 / np.log2(i + 2) for i, h in enumerate(hits_flags) if h)
                idcg = sum(1.0 / np.log2(i + 2) for i in range(min(len(tset), k)))
                self._ndcg += dcg / idcg if idcg > 0 else 0.0
                self._n_ndcg += 1

    def compute(self):
        def avg(s, n):
            return torch.tensor(s / n if n else 0.0)
        return {"map_at_k": avg(self._ap, self._n_ap), "recall_at_k": avg(self._rec, self._n_rec),
                "precision_at_k": avg(self._prec, self._n_prec),
                "ndcg_at_k": avg(self._ndcg, self._n_ndcg)}
