"""LightGCN drop-in (reference: `src/models/lightgcn.py`).

* `set_graph(edge_index, edge_weight)` (`:81-134`): records the edges; the normalized CSR
  (hnm_csr_build_norm) and the SpMM plan are built on the module's GPU on first use, so
  the reference's serve order -- set_graph, then load_state_dict, then .to(device)
  (`serve.py:243-252`) -- works unchanged.
* `forward()` (`:136-164`): L x hnm_spmm_csr_f32 with the alpha-weighted layer sum fused
  into the SpMM epilogue.  The reference re-propagates on every call; here the result is
  cached and invalidated whenever the embedding weight (torch version counter / storage)
  or the graph changes -- same outputs, without L SpMMs per recommend().
* `predict_all_items` (`:188-204`) -> hnm_dot_scores_f32;  `recommend` (`:332-358`) ->
  hnm_dot_topk_f32 (fused score GEMM + filter + top-K, user gather fused).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from .. import _lib
from ..evaluation import RecommendationMetrics
from .base import RecModule, dense_topk, empty_topk, f32c, filter_csr


class NormalizedGraph:
    """D^-1/2 (A + I) D^-1/2 as device CSR (rowptr int64, col int32, val fp32) + SpMM plan."""

    def __init__(self, edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor],
                 num_nodes: int, device: torch.device):
        _lib.require_gpu(torch.empty(0, device=device))
        ei = edge_index.to(device=device, dtype=torch.int64).contiguous()
        if ei.dim() != 2 or ei.shape[0] != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(ei.shape)}")
        E = ei.shape[1]
        ew = None
        if edge_weight is not None:
            ew = edge_weight.to(device=device, dtype=torch.float32).contiguous()
            if ew.numel() != E:
                raise ValueError("edge_weight must have one entry per edge")
        self.num_nodes = num_nodes
        self.nnz = E + num_nodes
        self.device = device
        self.rowptr = torch.empty(num_nodes + 1, dtype=torch.int64, device=device)
        self.col = torch.empty(self.nnz, dtype=torch.int32, device=device)
        self.val = torch.empty(self.nnz, dtype=torch.float32, device=device)
        c = _lib.ctx(device)
        _lib.check(_lib.fn("hnm_csr_build_norm")(c, _lib.ptr(ei), _lib.ptr(ew), E, num_nodes,
                                                 _lib.ptr(self.rowptr), _lib.ptr(self.col),
                                                 _lib.ptr(self.val)), "hnm_csr_build_norm")
        _lib.sync_check(device)
        plan = C.c_void_p()
        _lib.check(_lib.fn("hnm_spmm_plan_create")(c, num_nodes, _lib.ptr(self.rowptr),
                                                   C.byref(plan)), "hnm_spmm_plan_create")
        self.plan = plan
        self.prepared = set()
        self._restricted: Dict[tuple, C.c_void_p] = {}
        # bind the plan to this CSR's col / val (a walk plan sorts a copy of every row once)
        self.prepare(0)

    def prepare(self, d: int, plan=None):
        """One-time plan work for embedding width d (hnm_spmm_plan_prepare: the walk schedules;
        d = 0 binds the plan to col / val only), so no SpMM call does host work or syncs."""
        key = (d, None if plan is None else plan.value)
        if key in self.prepared:
            return
        c = _lib.ctx(self.device)
        _lib.check(_lib.fn("hnm_spmm_plan_prepare")(c, self.plan if plan is None else plan,
                                                    _lib.ptr(self.col), _lib.ptr(self.val), int(d)),
                   "hnm_spmm_plan_prepare")
        self.prepared.add(key)

    def restricted(self, ranges, d: int = 0):
        """A plan that computes only the rows of `ranges` ((begin, end) pairs, ascending), each
        summed exactly as by the whole-graph plan (hnm_spmm_plan_restrict): one rank's share of
        the item-sharded propagation.  Built once per ranges (host work), prepared for d."""
        key = tuple((int(a), int(b)) for a, b in ranges)
        p = self._restricted.get(key)
        if p is None:
            flat = (C.c_int64 * (2 * len(key)))(*[x for r in key for x in r])
            p = C.c_void_p()
            _lib.check(_lib.fn("hnm_spmm_plan_restrict")(_lib.ctx(self.device), self.plan, flat,
                                                         len(key), C.byref(p)),
                       "hnm_spmm_plan_restrict")
            self._restricted[key] = p
        if d:
            self.prepare(d, p)
        return p

    def spmm(self, X: torch.Tensor, Y: Optional[torch.Tensor], alpha: float,
             acc: Optional[torch.Tensor], acc_in: bool = True, beta: float = 0.0,
             rows: Optional[Tuple[int, int]] = None, acc_row0: int = 0, plan=None):
        """Y = A X on rows [r0, r1) (default all);  acc = fma(alpha, Y, acc or beta * X) on
        rows >= acc_row0, stored from acc_row0 on (either output optional).  plan: a
        `restricted` plan (only its rows are computed) instead of the whole-graph one."""
        r0, r1 = (0, self.num_nodes) if rows is None else rows
        c = _lib.ctx(X.device)
        _lib.check(_lib.fn("hnm_spmm_csr_range_f32")(
            c, self.plan if plan is None else plan, self.num_nodes, _lib.ptr(self.rowptr),
            _lib.ptr(self.col), _lib.ptr(self.val), _lib.ptr(X), X.shape[1], _lib.ptr(Y), alpha,
            _lib.ptr(acc) if acc_in else None, _lib.ptr(acc), beta, r0, r1, acc_row0),
            "hnm_spmm_csr_range_f32")

    def rows_combine(self, rows: torch.Tensor, layers, alphas) -> torch.Tensor:
        """Final embeddings of `rows` from the layer inputs E_0..E_{L-1} (last layer for
        these rows only): hnm_spmm_rows_combine_f32."""
        L = len(layers)
        d = layers[0].shape[1]
        out = torch.empty(rows.numel(), d, dtype=torch.float32, device=rows.device)
        ptrs = (C.c_void_p * L)(*[t.data_ptr() for t in layers])
        al = (C.c_float * (L + 1))(*[float(a) for a in alphas])
        c = _lib.ctx(rows.device)
        _lib.check(_lib.fn("hnm_spmm_rows_combine_f32")(
            c, self.plan, self.num_nodes, _lib.ptr(self.rowptr), _lib.ptr(self.col), _lib.ptr(self.val),
            _lib.ptr(rows), rows.numel(), d, ptrs, al, L, _lib.ptr(out)),
            "hnm_spmm_rows_combine_f32")
        return out

    def __del__(self):
        plan = getattr(self, "plan", None)
        if plan and _lib._lib is not None:
            try:
                torch.cuda.synchronize(self.device)
                for p in getattr(self, "_restricted", {}).values():
                    _lib.fn("hnm_spmm_plan_destroy")(p)
                _lib.fn("hnm_spmm_plan_destroy")(plan)
            except Exception:
                pass


class _GraphSpec:
    """What set_graph received; the device CSR is built lazily per device."""

    def __init__(self, edge_index, edge_weight):
        self.edge_index = edge_index
        self.edge_weight = edge_weight
        self.built: Dict[torch.device, NormalizedGraph] = {}


class LightGCN(RecModule):
    def __init__(
        self,
        num_users: int,
        num_items: int,
        embedding_dim: int = 64,
        num_layers: int = 3,
        learning_rate: float = 0.001,
        weight_decay: float = 1e-4,
        top_k: int = 12,
        alpha: Optional[float] = None,
    ):
        super().__init__()
        self.save_hyperparameters()
        self.num_users = num_users
        self.num_items = num_items
        self.num_nodes = num_users + num_items
        self.embedding_dim = embedding_dim
        self.num_layers = num_layers
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.top_k = top_k
        if alpha is None:  # lightgcn.py:59-67
            self.alpha = [1.0 / (num_layers + 1)] * (num_layers + 1)
        else:
            self.alpha = [alpha ** i for i in range(num_layers + 1)]
            s = sum(self.alpha)
            self.alpha = [a / s for a in self.alpha]
        self.embeddings = nn.Embedding(self.num_nodes, embedding_dim)
        nn.init.xavier_uniform_(self.embeddings.weight)
        self.graph = None
        self.edge_index = None
        self.edge_weight = None
        self.metrics = RecommendationMetrics(top_k=top_k)
        self._cache_key = None
        self._cache = None

    # ------------------------------------------------------------------ graph
    def set_graph(self, edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor] = None):
        """Record the interaction graph (`lightgcn.py:81-112`)."""
        if edge_index.dim() != 2 or edge_index.shape[0] != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        self.edge_index = edge_index
        self.edge_weight = edge_weight
        self.graph = _GraphSpec(edge_index, edge_weight)
        self._cache_key = None
        self._cache = None

    def _device_graph(self) -> NormalizedGraph:
        if self.graph is None:
            raise RuntimeError("Graph not set. Call set_graph() first.")
        dev = self.device
        g = self.graph.built.get(dev)
        if g is None:
            g = NormalizedGraph(self.graph.edge_index, self.graph.edge_weight, self.num_nodes, dev)
            self.graph.built[dev] = g
        if self.embedding_dim in (4, 8, 16, 32, 64, 128, 256):
            g.prepare(self.embedding_dim)
        return g

    # ------------------------------------------------------------------ propagation
    def forward(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(final user embeddings [U, d], final item embeddings [I, d]) (`lightgcn.py:136-164`)."""
        g = self._device_graph()
        w = self.embeddings.weight
        key = (w.data_ptr(), w._version, id(g), w.device)
        if self._cache_key != key:
            self._cache = self.propagate(g)
            self._cache_key = key
        F = self._cache
        return F[: self.num_users], F[self.num_users:]

    def propagate(self, g: Optional[NormalizedGraph] = None) -> torch.Tensor:
        """E_{l+1} = A E_l, F = sum_l alpha_l E_l on the HIP SpMM (no cache); the alpha_0 E_0
        term is folded into layer 1's epilogue."""
        g = self._device_graph() if g is None else g
        E0 = f32c(self.embeddings.weight)
        _lib.require_gpu(E0)
        acc = torch.empty_like(E0)
        if self.num_layers == 0:
            return acc.copy_(E0).mul_(float(self.alpha[0]))
        cur = E0
        for layer in range(self.num_layers):
            last = layer == self.num_layers - 1
            nxt = None if last else torch.empty_like(E0)
            g.spmm(cur, nxt, float(self.alpha[layer + 1]), acc, acc_in=layer > 0,
                   beta=float(self.alpha[0]))
            cur = nxt
        return acc

    def propagate_for(self, user_ids: torch.Tensor,
                      g: Optional[NormalizedGraph] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """What one `recommend(user_ids)` reads of `forward()` (`lightgcn.py:197-199`): the
        final rows of the listed users [B, d] and every item [I, d], recomputed (no cache).

        Layers 1..L-1 run over the whole graph (every node feeds the last layer); the last
        layer runs over the item rows only, and the users' final rows come from
        hnm_spmm_rows_combine_f32.  The layer combine is kept for item rows only.  Outputs
        are identical to forward()'s rows (same operations in the same order), without the
        last layer's 1.37M user rows and the users' combine traffic."""
        g = self._device_graph() if g is None else g
        U, N, L = self.num_users, self.num_nodes, self.num_layers
        u, hu = self._ids(user_ids, U)
        E0 = f32c(self.embeddings.weight)
        _lib.require_gpu(E0)
        if L == 0:
            F = E0 * float(self.alpha[0])
            return F[u], F[U:]
        acc = torch.empty(N - U, E0.shape[1], dtype=torch.float32, device=E0.device)
        layers = [E0]
        for layer in range(L):
            last = layer == L - 1
            nxt = None if last else torch.empty_like(E0)
            g.spmm(layers[-1], nxt, float(self.alpha[layer + 1]), acc, acc_in=layer > 0,
                   beta=float(self.alpha[0]), rows=(U, N) if last else None, acc_row0=U)
            if not last:
                layers.append(nxt)
        return g.rows_combine(u, layers, self.alpha), acc

    def propagate_for_shard(self, user_ids: torch.Tensor, lo: int, hi: int, exchange,
                            g: Optional[NormalizedGraph] = None
                            ) -> Tuple[torch.Tensor, torch.Tensor]:
        """propagate_for with the item rows sharded over the ranks of a node:
        (final rows of the listed users [B, d], final rows of THIS rank's items [lo, hi)
        [hi - lo, d]).  Every rank computes all user rows of layers 1..L-1 (they gather the
        whole item table) and only its own item rows (a restricted plan: hnm_spmm_plan_restrict),
        `exchange(Y)` (sharding.ItemRowExchange: one all_gather of the [I, d] item rows) fills
        the other shards' item rows after each of those layers, and the last layer runs on the
        rank's items alone.  Rows are summed exactly as by the whole-graph plan, so the outputs
        are bitwise those of propagate_for / forward()."""
        from ..sharding import item_sharded_layers
        g = self._device_graph() if g is None else g
        U, L, d = self.num_users, self.num_layers, self.embedding_dim
        if not 0 <= lo <= hi <= self.num_items:
            raise ValueError(f"item shard [{lo}, {hi}) outside [0, {self.num_items})")
        if lo == 0 and hi == self.num_items:
            return self.propagate_for(user_ids, g)
        u, hu = self._ids(user_ids, U)
        E0 = f32c(self.embeddings.weight)
        _lib.require_gpu(E0)
        if L == 0:
            return E0[u] * float(self.alpha[0]), E0[U + lo:U + hi] * float(self.alpha[0])
        plan = g.restricted(((0, U), (U + lo, U + hi)), d)

        def layer(X, Y, alpha, acc, acc_in, beta, last):
            g.spmm(X, Y, alpha, acc, acc_in=acc_in, beta=beta,
                   rows=(U + lo, U + hi) if last else None, acc_row0=U + lo, plan=plan)
        layers, acc = item_sharded_layers(E0, U, L, self.alpha, lo, hi, layer, exchange)
        return g.rows_combine(u, layers, self.alpha), acc

    # ------------------------------------------------------------------ scoring
    def predict(self, user_ids: torch.Tensor, item_ids: torch.Tensor) -> torch.Tensor:
        """Pairwise dot of propagated embeddings (`lightgcn.py:166-186`)."""
        fu, fi = self.forward()
        u, hu = self._ids(user_ids, self.num_users)
        i, hi = self._ids(item_ids, self.num_items, "item_ids")
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_pair_dot_f32")(c, _lib.ptr(fu), self.num_users, d, _lib.ptr(fi),
                                               self.num_items, d, d, _lib.ptr(u), _lib.ptr(i),
                                               u.numel(), None, None, None, _lib.ptr(out)),
                   "hnm_pair_dot_f32")
        self._check(u.device, hu, hi)
        return out

    def predict_all_items(self, user_ids: torch.Tensor) -> torch.Tensor:
        """Dense scores F_U[ids] @ F_I^T, [B, num_items] (`lightgcn.py:188-204`)."""
        fu, fi = self.forward()
        u, hu = self._ids(user_ids, self.num_users)
        out = torch.empty(u.numel(), self.num_items, dtype=torch.float32, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_dot_scores_f32")(c, _lib.ptr(fu), self.num_users, d, _lib.ptr(u),
                                                 u.numel(), _lib.ptr(fi), self.num_items, d, d,
                                                 None, None, None, _lib.ptr(out), out.stride(0)),
                   "hnm_dot_scores_f32")
        self._check(u.device, hu)
        return out

    def recommend_with_scores(self, user_ids: torch.Tensor,
                              filter_items: Optional[Dict[int, set]] = None,
                              k: Optional[int] = None):
        """(scores [B, k], items [B, k]) sorted by score desc, item asc."""
        k = self.top_k if k is None else k
        fu, fi = self.forward()
        u, hu = self._ids(user_ids, self.num_users)
        n_items = fi.shape[0]
        mptr, midx = filter_csr(u, filter_items, self.num_items, u.device)
        kk = min(k, n_items)
        if kk <= 0:
            return empty_topk(k, u)
        if kk > 64:
            scores = self.predict_all_items(u)
            return dense_topk(scores, kk, mptr, midx)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        d = self.embedding_dim
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_dot_topk_f32")(c, _lib.ptr(fu), self.num_users, d, _lib.ptr(u),
                                               u.numel(), _lib.ptr(fi), n_items, fi.stride(0), d,
                                               None, None, None, _lib.ptr(mptr), _lib.ptr(midx),
                                               kk, _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_dot_topk_f32")
        self._check(u.device, hu)
        return out_v, out_i

    def recommend(self, user_ids: torch.Tensor,
                  filter_items: Optional[Dict[int, set]] = None) -> torch.Tensor:
        """Top-`top_k` item ids per user (`lightgcn.py:332-358`)."""
        self._check_top_k()
        self.eval()
        with torch.no_grad():
            return self.recommend_with_scores(user_ids, filter_items)[1]
