"""Item-row sharding across the GPUs of a node (north_star).

The reference has no distributed code; this is the MI355X design:

* rank g owns items [floor(g I / G), floor((g+1) I / G)) -- its slice of the item tables
  and of the per-item precompute;
* every rank brings its own batch of B users; one `all_gather` of the user ids (int64,
  B*8 bytes per rank) gives every rank the G*B users of the step;
* each rank runs the fused score + top-K kernel over its item shard for all G*B users
  (per-GPU work is the single-GPU work: weak scaling).  With the certified pre-filter the
  local scorer runs in two phases: `begin_lists` gives every user's k best certified sample
  lower bounds over the rank's items (distinct items), one `all_gather` of those G*B*k floats
  and the k-th best of their union give every rank a lower bound of the GLOBAL k-th (a scorer
  with a single-bound `begin` gets the `all_reduce(MAX)` of those), and `finish` keeps only items that can be in the global top-k (candidates per user stay
  ~constant as G grows instead of G x; rows may come back short, padded with -inf / -1);
* one `all_to_all` returns to every rank the G candidate lists (k score bits + global
  item ids, packed as int32 pairs) of ITS users (B*k*8 bytes per rank pair: latency-bound
  on xGMI, so one collective, not a ring of per-layer exchanges);
* the owner merges G*k candidates per user with the HIP merge kernel.  The order
  (score desc, item asc) is total, so the result is exactly the single-GPU top-k.

Collectives go through `torch.distributed` (backend "nccl" = RCCL over xGMI on ROCm; gloo
for the CPU tests).  The local scorer and the merge are injected so the host logic above
is tested with gloo on CPU (tests/test_sharding_gloo.py) while the product wires the HIP
kernels (`ncf_shard_topk`, `dot_shard_topk`, `hip_merge`).
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from . import _lib

LocalTopK = Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]
Merge = Callable[[torch.Tensor, torch.Tensor, int], Tuple[torch.Tensor, torch.Tensor]]


def shard_range(num_items: int, rank: int, world: int) -> Tuple[int, int]:
    return num_items * rank // world, num_items * (rank + 1) // world


class ItemShardedRecommender:
    def __init__(self, local_topk: LocalTopK, merge: Merge, k: int, item_offset: int,
                 rank: int = 0, world: int = 1, group=None, exchange: Optional[bool] = None):
        """exchange: run the collective path (all_gather, bound exchange, all_to_all,
        merge) -- the default whenever world > 1; True forces it at world == 1 as well
        (a 1-rank process group: the RCCL calls of the multi-GPU path on one GPU)."""
        self.local_topk = local_topk
        self.merge = merge
        self.k = k
        self.item_offset = item_offset
        self.rank = rank
        self.world = world
        self.group = group
        self.exchange = world > 1 if exchange is None else bool(exchange)
        if self.exchange and not dist.is_initialized():
            raise RuntimeError("the item-shard exchange needs an initialized process group")

    def recommend(self, user_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k (scores, global item ids) for this rank's users [B] (same B on all ranks)."""
        G, k = self.world, self.k
        B = user_ids.numel()
        if not self.exchange:
            v, i = self.local_topk(user_ids)
            if self.item_offset == 0:  # ids are already global (no elementwise pass)
                return v, i
            return v, torch.where(i >= 0, i + self.item_offset, i)
        dev = user_ids.device
        # gloo (CPU tests, single-GPU rehearsal) moves host tensors; RCCL moves device tensors
        host = dist.get_backend(self.group) == "gloo"
        stage = (lambda t: t.cpu()) if host else (lambda t: t)
        ids = stage(user_ids.contiguous())
        all_ids = torch.empty(G * B, dtype=ids.dtype, device=ids.device)
        dist.all_gather_into_tensor(all_ids, ids, group=self.group)
        all_ids = all_ids.to(dev)
        if hasattr(self.local_topk, "begin_lists"):
            # every shard's k best sample lower bounds per user, all_gathered: the k-th best of
            # their union is a lower bound of the user's GLOBAL k-th best (G*B*k*4 bytes)
            try:
                lists = stage(self.local_topk.begin_lists(all_ids).contiguous())
                rows, kk = lists.shape
                allv = torch.empty((G * rows, kk), dtype=lists.dtype, device=lists.device)
                dist.all_gather_into_tensor(allv, lists, group=self.group)
                lb = _kth_of_lists(allv.to(dev).view(G, rows, kk), k)
            except BaseException:
                abort = getattr(self.local_topk, "abort", None)
                if abort is not None:
                    abort()
                raise
            v, i = self.local_topk.finish(all_ids, lb)
        elif hasattr(self.local_topk, "begin"):
            # two-phase local scorer: global lower bounds of each user's k-th best score
            try:
                lb = stage(self.local_topk.begin(all_ids).contiguous())
                dist.all_reduce(lb, op=dist.ReduceOp.MAX, group=self.group)
            except BaseException:
                abort = getattr(self.local_topk, "abort", None)
                if abort is not None:
                    abort()  # close the open two-phase call so the ctx stays usable
                raise
            v, i = self.local_topk.finish(all_ids, lb.to(dev))  # [G*B, k], shard-local ids
        else:
            v, i = self.local_topk(all_ids)  # [G*B, k], shard-local ids
        # ONE exchange: (score bits, global item id) packed as int32 pairs -- item ids are
        # < 2^31 -- so values and ids travel in a single all_to_all (B*k*8 bytes per pair)
        pm = getattr(self.merge, "packed", None)   # (pack, merge) HIP kernels on device
        if pm is not None and v.is_cuda:
            packed = stage(pm[0](v, i, self.item_offset).reshape(-1))
        else:
            i = torch.where(i >= 0, i + self.item_offset, i)
            packed = torch.stack([v.contiguous().view(torch.int32), i.to(torch.int32)], dim=-1)
            packed = stage(packed.reshape(-1))
        recv = torch.empty_like(packed)
        dist.all_to_all_single(recv, packed, group=self.group)
        recv = recv.to(dev).view(G, B, k, 2)
        if pm is not None and recv.is_cuda:
            return pm[1](recv, k)
        rv = recv.view(torch.float32)[..., 0].contiguous()
        ri = recv[..., 1].to(torch.int64)
        return self.merge(rv, ri, k)


# ------------------------------------------------------------------ HIP wiring
def _kth_of_lists(allv: torch.Tensor, k: int) -> torch.Tensor:
    """[G, B, kc] bound lists (each row descending) -> [B] the k-th best of each row's union.
    On the GPU one thread per row merges the G lists (hnm_topk_lists_kth_f32); host tensors
    (the CPU tests' scorers) and G > 16 use torch.topk over the concatenation."""
    G, B, kc = allv.shape
    if not allv.is_cuda or G > 16:
        return torch.topk(allv.permute(1, 0, 2).reshape(B, G * kc), k, dim=1).values[:, k - 1].contiguous()
    allv = allv.contiguous()
    out = torch.empty(B, dtype=torch.float32, device=allv.device)
    _lib.check(_lib.fn("hnm_topk_lists_kth_f32")(_lib.ctx(allv.device), _lib.ptr(allv), B, G, kc,
                                                 k, _lib.ptr(out)), "hnm_topk_lists_kth_f32")
    return out


def _pad(v, i, k):
    """Keep k candidate columns on every rank (equal all_to_all splits) for tiny shards."""
    if v.shape[1] == k:
        return v, i
    pv = torch.full((v.shape[0], k), float("-inf"), dtype=v.dtype, device=v.device)
    pi = torch.full((v.shape[0], k), -1, dtype=i.dtype, device=i.device)
    pv[:, : v.shape[1]] = v
    pi[:, : v.shape[1]] = i
    return pv, pi


def hip_merge(cand_v: torch.Tensor, cand_i: torch.Tensor, k: int):
    """[G, B, kc] candidates -> [B, k] via hnm_topk_merge_f32."""
    G, B, kc = cand_v.shape
    out_v = torch.empty(B, k, dtype=torch.float32, device=cand_v.device)
    out_i = torch.empty(B, k, dtype=torch.int64, device=cand_v.device)
    c = _lib.ctx(cand_v.device)
    _lib.check(_lib.fn("hnm_topk_merge_f32")(c, _lib.ptr(cand_v), _lib.ptr(cand_i), B, G, B * kc,
                                             kc, kc, k, _lib.ptr(out_v), _lib.ptr(out_i)),
               "hnm_topk_merge_f32")
    return out_v, out_i


def _pack_pairs(v: torch.Tensor, i: torch.Tensor, offset: int) -> torch.Tensor:
    """[R, k] scores + shard-local ids -> [R, k, 2] int32 (score bits, global id; -1 stays)."""
    v, i = v.contiguous(), i.to(torch.int64).contiguous()
    out = torch.empty(v.shape + (2,), dtype=torch.int32, device=v.device)
    _lib.check(_lib.fn("hnm_pack_candidates_i32")(_lib.ctx(v.device), _lib.ptr(v), _lib.ptr(i),
                                                  v.numel(), offset, _lib.ptr(out)),
               "hnm_pack_candidates_i32")
    return out


def _merge_pairs(recv: torch.Tensor, k: int):
    """[G, B, kc, 2] received pairs, each list in top-K order -> [B, k] (scores, global ids)."""
    G, B, kc, _ = recv.shape
    if G > 16:
        rv = recv.view(torch.float32)[..., 0].contiguous()
        return hip_merge(rv, recv[..., 1].to(torch.int64), k)
    recv = recv.contiguous()
    out_v = torch.empty(B, k, dtype=torch.float32, device=recv.device)
    out_i = torch.empty(B, k, dtype=torch.int64, device=recv.device)
    _lib.check(_lib.fn("hnm_topk_merge_sorted_pairs_i32")(
        _lib.ctx(recv.device), _lib.ptr(recv), B, G, kc, k, _lib.ptr(out_v), _lib.ptr(out_i)),
        "hnm_topk_merge_sorted_pairs_i32")
    return out_v, out_i


hip_merge.packed = (_pack_pairs, _merge_pairs)


def _mask(history, u, lo, hi):
    """The batch's -inf mask restricted to the shard's items (UserHistory on the device)."""
    if history is None:
        return None, None
    return history.mask_for(u, (lo, hi))


class ncf_shard_topk:
    """Fused NCF score + top-K over item rows [lo, hi) of `model` (a NeuralCF on a GPU).

    Called directly: one hnm_ncf_topk_f32.  `begin` / `finish`: the two phases of
    hnm_ncf_topk_begin_f32 / _finish_f32 around a cross-shard bound exchange.  `history`
    (a UserHistory): mask each user's history items, gathered on the device per call.
    A model whose tower the fused kernels do not take (any other `mlp_dims`) gets an
    `ncf_deep_shard_topk` instead."""

    def __new__(cls, model, lo: int, hi: int, k: int, history=None):
        if cls is ncf_shard_topk and not model._fused():
            return ncf_deep_shard_topk(model, lo, hi, k, history)
        return super().__new__(cls)

    def __init__(self, model, lo: int, hi: int, k: int, history=None):
        self.model, self.lo, self.hi, self.k = model, lo, hi, k
        self.history = history
        self._open = None

    def _args(self, user_ids):
        w, keep = self.model._weights()
        w = _lib.NcfWeights.from_buffer_copy(w)  # the module may reuse its struct: shift a copy
        mf, h0 = self.model.mf_dim, self.model.mlp_dims[0] // 2
        w.gmf_item = w.gmf_item + self.lo * mf * 4
        w.mlp_item = w.mlp_item + self.lo * h0 * 4
        if w.item_proj:  # the model's cached item projection: this shard's rows
            w.item_proj = w.item_proj + self.lo * (128 if (w.h1 > 64 or w.mf > 64) else 64) * 4
        w.num_items = self.hi - self.lo
        u = user_ids.to(torch.int64).contiguous()
        return w, keep, u, min(self.k, self.hi - self.lo)

    def _out(self, u, kk):
        return (torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device),
                torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device))

    def __call__(self, user_ids: torch.Tensor):
        w, keep, u, kk = self._args(user_ids)
        mp, mi = _mask(self.history, u, self.lo, self.hi)
        out_v, out_i = self._out(u, kk)
        _lib.check(_lib.fn("hnm_ncf_topk_f32")(_lib.ctx(u.device), w, _lib.ptr(u), u.numel(),
                                               _lib.ptr(mp), _lib.ptr(mi), kk, _lib.ptr(out_v),
                                               _lib.ptr(out_i)), "hnm_ncf_topk_f32")
        return _pad(out_v, out_i, self.k)

    def begin(self, user_ids: torch.Tensor) -> torch.Tensor:
        w, keep, u, kk = self._args(user_ids)
        mp, mi = _mask(self.history, u, self.lo, self.hi)
        lb = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        _lib.check(_lib.fn("hnm_ncf_topk_begin_f32")(_lib.ctx(u.device), w, _lib.ptr(u), u.numel(),
                                                     _lib.ptr(mp), _lib.ptr(mi), kk, _lib.ptr(lb)),
                   "hnm_ncf_topk_begin_f32")
        self._open = (w, keep, u, kk, mp, mi)  # finish must pass the same ids / tables / mask
        return lb

    def begin_lists(self, user_ids: torch.Tensor) -> torch.Tensor:
        """begin with each row's k best certified sample lower bounds [B, k] (distinct items,
        real units, descending, -inf padded) instead of one bound: the k-th best of the union
        over the item shards bounds the GLOBAL k-th (hnm_ncf_topk_begin_lists_f32)."""
        w, keep, u, kk = self._args(user_ids)
        mp, mi = _mask(self.history, u, self.lo, self.hi)
        out = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        _lib.check(_lib.fn("hnm_ncf_topk_begin_lists_f32")(
            _lib.ctx(u.device), w, _lib.ptr(u), u.numel(), _lib.ptr(mp), _lib.ptr(mi), kk,
            _lib.ptr(out)), "hnm_ncf_topk_begin_lists_f32")
        self._open = (w, keep, u, kk, mp, mi)
        return _pad_lists(out, self.k)

    def abort(self):
        if self._open is not None:
            _lib.abort_pending(self._open[2].device)
            self._open = None

    def finish(self, user_ids: torch.Tensor, lb: torch.Tensor):
        w, keep, u, kk, mp, mi = self._open
        self._open = None
        lb = lb.to(torch.float32).contiguous()
        out_v, out_i = self._out(u, kk)
        _lib.check(_lib.fn("hnm_ncf_topk_finish_f32")(_lib.ctx(u.device), w, _lib.ptr(u), u.numel(),
                                                      _lib.ptr(mp), _lib.ptr(mi), kk, _lib.ptr(lb),
                                                      1, _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_ncf_topk_finish_f32")
        return _pad(out_v, out_i, self.k)


class ncf_deep_shard_topk:
    """NeuralCF towers other than the fused two-layer one over item rows [lo, hi):
    hnm_ncf_deep_topk_f32 on the shard's item tables (fp32-MFMA tile kernel with fused
    per-partition top-k lists, scores bitwise the unsharded ones).  Single-phase: the exchange
    merges every shard's k best (no bound exchange), so k <= 64."""

    def __init__(self, model, lo: int, hi: int, k: int, history=None):
        if k > 64:
            raise ValueError("ncf_deep_shard_topk: k <= 64 (the fused deep top-k)")
        self.model, self.lo, self.hi, self.k = model, lo, hi, k
        self.history = history

    def __call__(self, user_ids: torch.Tensor):
        w, keep = self.model._deep_weights()
        w = _lib.NcfDeepWeights.from_buffer_copy(w)
        w.gmf_item = w.gmf_item + self.lo * self.model.mf_dim * 4
        w.mlp_item = w.mlp_item + self.lo * (self.model.mlp_dims[0] // 2) * 4
        w.num_items = self.hi - self.lo
        u = user_ids.to(torch.int64).contiguous()
        kk = min(self.k, self.hi - self.lo)
        mp, mi = _mask(self.history, u, self.lo, self.hi)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        _lib.check(_lib.fn("hnm_ncf_deep_topk_f32")(
            _lib.ctx(u.device), C.byref(w), _lib.ptr(u), u.numel(), _lib.ptr(mp), _lib.ptr(mi),
            kk, _lib.ptr(out_v), _lib.ptr(out_i)), "hnm_ncf_deep_topk_f32")
        return _pad(out_v, out_i, self.k)


def _pad_lists(out: torch.Tensor, k: int) -> torch.Tensor:
    """Bound lists of a shard of fewer than k items, -inf padded to k (equal all_gather shapes)."""
    if out.shape[1] == k:
        return out
    lists = torch.full((out.shape[0], k), float("-inf"), dtype=torch.float32, device=out.device)
    lists[:, :out.shape[1]] = out
    return lists


class dot_shard_topk:
    """Fused dot score + top-K (LightGCN; MF with its user / item / global biases) over item
    rows [lo, hi).

    Called directly: one hnm_dot_topk_f32.  `begin` / `finish`: the two phases of
    hnm_dot_topk_begin_f32 / _finish_f32 around a cross-shard bound exchange.  `history`
    (a UserHistory): mask each user's history items (user_ids must then be the history's
    user ids: `rows` maps the table rows scored to them when they differ, e.g. LightGCN's
    per-call user rows)."""

    def __init__(self, user_tab: torch.Tensor, item_tab: torch.Tensor, lo: int, hi: int, k: int,
                 history=None, user_bias=None, item_bias=None, const_bias=None,
                 shard_table: bool = False):
        """shard_table: item_tab holds the shard's rows [lo, hi) only (an item-sharded
        LightGCN propagation's output) instead of the whole catalogue."""
        if shard_table and item_tab.shape[0] != hi - lo:
            raise ValueError(f"shard table of {item_tab.shape[0]} rows for items [{lo}, {hi})")
        self.user_tab, self.shard, self.k = user_tab, (item_tab if shard_table else item_tab[lo:hi]), k
        self.lo, self.hi, self.n = lo, hi, hi - lo
        self.history = history
        # MatrixFactorization's score terms (matrix_factorization.py:108-131): [U], [I] (the
        # shard's slice is used), [1]; None = absent
        self.ub = None if user_bias is None else user_bias.reshape(-1).contiguous()
        self.ib = None if item_bias is None else item_bias.reshape(-1)[lo:hi].contiguous()
        self.cb = None if const_bias is None else const_bias.reshape(-1).contiguous()
        self.mask_users = None   # ids the history is keyed by, when the table rows differ
        self._open = None

    def _common(self, u, mask=(None, None)):
        ut, sh = self.user_tab, self.shard
        return (_lib.ptr(ut), ut.shape[0], ut.stride(0), _lib.ptr(u), u.numel(), _lib.ptr(sh),
                self.n, sh.stride(0), ut.shape[1], _lib.ptr(self.ub), _lib.ptr(self.ib),
                _lib.ptr(self.cb), _lib.ptr(mask[0]), _lib.ptr(mask[1]))

    def _mask(self, u):
        return _mask(self.history, u if self.mask_users is None else self.mask_users,
                     self.lo, self.hi)

    def _out(self, u, kk):
        return (torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device),
                torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device))

    def __call__(self, user_ids: torch.Tensor):
        u = user_ids.to(torch.int64).contiguous()
        kk = min(self.k, self.n)
        out_v, out_i = self._out(u, kk)
        _lib.check(_lib.fn("hnm_dot_topk_f32")(_lib.ctx(u.device), *self._common(u, self._mask(u)),
                                               kk, _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_dot_topk_f32")
        return _pad(out_v, out_i, self.k)

    def begin(self, user_ids: torch.Tensor) -> torch.Tensor:
        u = user_ids.to(torch.int64).contiguous()
        kk = min(self.k, self.n)
        mask = self._mask(u)
        lb = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        _lib.check(_lib.fn("hnm_dot_topk_begin_f32")(_lib.ctx(u.device), *self._common(u, mask), kk,
                                                     _lib.ptr(lb)), "hnm_dot_topk_begin_f32")
        self._open = (u, kk, mask)  # finish must pass the same ids and mask
        return lb

    def begin_lists(self, user_ids: torch.Tensor) -> torch.Tensor:
        """begin with each row's k best certified sample lower bounds [B, k]
        (hnm_dot_topk_begin_lists_f32; see ncf_shard_topk.begin_lists)."""
        u = user_ids.to(torch.int64).contiguous()
        kk = min(self.k, self.n)
        mask = self._mask(u)
        out = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        _lib.check(_lib.fn("hnm_dot_topk_begin_lists_f32")(
            _lib.ctx(u.device), *self._common(u, mask), kk, _lib.ptr(out)),
            "hnm_dot_topk_begin_lists_f32")
        self._open = (u, kk, mask)
        return _pad_lists(out, self.k)

    def abort(self):
        if self._open is not None:
            _lib.abort_pending(self._open[0].device)
            self._open = None

    def finish(self, user_ids: torch.Tensor, lb: torch.Tensor):
        u, kk, mask = self._open
        self._open = None
        lb = lb.to(torch.float32).contiguous()
        out_v, out_i = self._out(u, kk)
        _lib.check(_lib.fn("hnm_dot_topk_finish_f32")(_lib.ctx(u.device), *self._common(u, mask), kk,
                                                      _lib.ptr(lb), 1, _lib.ptr(out_v),
                                                      _lib.ptr(out_i)), "hnm_dot_topk_finish_f32")
        return _pad(out_v, out_i, self.k)


def widedeep_shard_topk(model, lo: int, hi: int, k: int, history=None) -> LocalTopK:
    """Fused Wide&Deep score + top-K over item rows [lo, hi) of `model` (a WideDeep on a GPU);
    `history` (a UserHistory) masks each user's history items."""
    def run(user_ids: torch.Tensor):
        w, keep = model._weights()
        w = _lib.WideDeepWeights.from_buffer_copy(w)
        d = model.embedding_dim
        w.deep_item = w.deep_item + lo * d * 4
        w.wide_item = w.wide_item + lo * 4
        w.num_items = hi - lo
        u = user_ids.to(torch.int64).contiguous()
        mp, mi = _mask(history, u, lo, hi)
        kk = min(k, hi - lo)
        out_v = torch.empty(u.numel(), kk, dtype=torch.float32, device=u.device)
        out_i = torch.empty(u.numel(), kk, dtype=torch.int64, device=u.device)
        c = _lib.ctx(u.device)
        _lib.check(_lib.fn("hnm_widedeep_topk_f32")(c, w, _lib.ptr(u), u.numel(), None,
                                                    _lib.ptr(mp), _lib.ptr(mi), kk,
                                                    _lib.ptr(out_v), _lib.ptr(out_i)),
                   "hnm_widedeep_topk_f32")
        return _pad(out_v, out_i, k)
    return run


def item_sharded_layers(E0: torch.Tensor, num_users: int, num_layers: int, alphas, lo: int,
                        hi: int, layer, exchange):
    """The layer loop of the item-sharded LightGCN propagation (`lightgcn.py:136-164`, one rank
    of a node): every rank computes ALL user rows of layers 1..L-1 (each gathers the whole item
    table) but only ITS item rows [U+lo, U+hi); after each of those layers `exchange(Y)` fills
    the other shards' item rows of Y (an all_gather of [I, d]: 54 MB at the H&M shape, d = 128,
    against the 702 MB user half it would take to shard the users too), and the last layer runs
    on the rank's item rows alone.  The combine sum_l alpha_l E_l is kept for those rows.

    layer(X, Y, alpha, acc, acc_in, beta, last) computes rows [0, U) and [U+lo, U+hi) of
    Y = A_hat X (only [U+lo, U+hi) when last; Y None then) with the fused combine into acc
    (rows U+lo.. stored from 0; acc_in False: beta * X).  Returns (E_0 .. E_{L-1}, acc [hi-lo, d]).
    The product passes a restricted SpMM plan (LightGCN.propagate_for_shard); the CPU tests
    pass the oracle's row-restricted SpMM and a gloo exchange."""
    acc = torch.empty(hi - lo, E0.shape[1], dtype=E0.dtype, device=E0.device)
    layers = [E0]
    for li in range(num_layers):
        last = li == num_layers - 1
        nxt = None if last else torch.empty_like(E0)
        layer(layers[-1], nxt, float(alphas[li + 1]), acc, li > 0, float(alphas[0]), last)
        if not last:
            exchange(nxt)
            layers.append(nxt)
    return layers, acc


class ItemRowExchange:
    """Fills the other shards' item rows of a propagation layer Y [U + I, d]: rank r computed
    rows U + shard_range(I, r, G); one all_gather_into_tensor of every shard's rows (padded to
    the largest shard, m rows: G * m * d * 4 bytes received per rank), then one copy per other
    shard into place.  RCCL moves device tensors; gloo (CPU tests, one-GPU rehearsal) is staged
    through host memory."""

    def __init__(self, num_users: int, num_items: int, rank: int, world: int, group=None):
        self.U, self.I, self.rank, self.world, self.group = num_users, num_items, rank, world, group
        self.ranges = [shard_range(num_items, r, world) for r in range(world)]
        self.m = max(b - a for a, b in self.ranges)
        self.calls = 0

    def bytes_per_call(self, d: int, itemsize: int = 4) -> int:
        return self.world * self.m * d * itemsize

    def __call__(self, Y: torch.Tensor):
        G, m, U = self.world, self.m, self.U
        lo, hi = self.ranges[self.rank]
        d = Y.shape[1]
        host = dist.get_backend(self.group) == "gloo"
        own = Y[U + lo:U + hi]
        if hi - lo == m and not host:
            send = own                     # contiguous rows: no staging copy
        else:
            send = torch.empty(m, d, dtype=Y.dtype, device="cpu" if host else Y.device)
            send[:hi - lo].copy_(own)
            if hi - lo < m:
                send[hi - lo:].zero_()
        recv = torch.empty(G * m, d, dtype=Y.dtype, device=send.device)
        dist.all_gather_into_tensor(recv, send, group=self.group)
        for r, (a, b) in enumerate(self.ranges):
            if r != self.rank and b > a:
                Y[U + a:U + b].copy_(recv[r * m:r * m + (b - a)])
        self.calls += 1


class lightgcn_shard_topk:
    """LightGCN recommend() over item rows [lo, hi) with the propagation recomputed per
    call, as the reference does (`lightgcn.py:197` -> `forward()`), restricted to what the
    call reads, then the dot top-K over the shard.  exchange None: `LightGCN.propagate_for(all
    users of the step)` (layers 1..L-1 whole graph, the last layer on item rows + these users),
    replicated per rank; an `ItemRowExchange`: `LightGCN.propagate_for_shard` -- the item rows
    of every layer sharded over the ranks, one all_gather of [I, d] after each of layers
    1..L-1, the last layer on this shard's items only (outputs bitwise the same)."""

    def __init__(self, model, lo: int, hi: int, k: int, history=None, exchange=None):
        self.model, self.lo, self.hi, self.k = model, lo, hi, k
        self.history = history
        self.exchange = exchange
        self._dot = None
        self._rows = None

    def _scorer(self, user_ids):
        if self.exchange is None:
            fb, fi = self.model.propagate_for(user_ids)
            shard = False
        else:
            fb, fi = self.model.propagate_for_shard(user_ids, self.lo, self.hi, self.exchange)
            shard = True
        n, dev = user_ids.numel(), user_ids.device
        if self._rows is None or self._rows.numel() < n or self._rows.device != dev:
            # kept across calls (one launch less a call); completed before any stream reads it
            self._rows = torch.arange(n, dtype=torch.int64, device=dev)
            if dev.type == "cuda":
                torch.cuda.current_stream(dev).synchronize()
        rows = self._rows[:n]
        dot = dot_shard_topk(fb, fi, self.lo, self.hi, self.k, self.history, shard_table=shard)
        dot.mask_users = user_ids.to(torch.int64).contiguous()   # history keyed by user id
        return dot, rows

    def __call__(self, user_ids: torch.Tensor):
        dot, rows = self._scorer(user_ids)
        return dot(rows)

    def begin(self, user_ids: torch.Tensor) -> torch.Tensor:
        dot, rows = self._scorer(user_ids)
        self._dot = (dot, rows)
        return dot.begin(rows)

    def begin_lists(self, user_ids: torch.Tensor) -> torch.Tensor:
        dot, rows = self._scorer(user_ids)
        self._dot = (dot, rows)
        return dot.begin_lists(rows)

    def abort(self):
        if self._dot is not None:
            self._dot[0].abort()
            self._dot = None

    def finish(self, user_ids: torch.Tensor, lb: torch.Tensor):
        dot, rows = self._dot
        self._dot = None
        return dot.finish(rows, lb)
