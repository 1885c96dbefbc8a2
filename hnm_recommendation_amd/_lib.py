"""ctypes binding of libhnm_mi355x.so (the C ABI in include/hnm.h).

This is the ONLY route to compute: there is no CPU or eager-PyTorch fallback.  If the
library is missing, or a tensor is not on an AMD GPU, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref

import torch

PKG = os.path.dirname(os.path.abspath(__file__))
# HNM_LIB_PATH: load another build of the same library (A/B timing of kernel variants built
# from tools/; the in-tree build is the product and the default)
LIB_PATH = os.environ.get("HNM_LIB_PATH") or os.path.join(PKG, "libhnm_mi355x.so")

HNM_OK, HNM_EINVAL, HNM_EOOB, HNM_EHIP, HNM_ENOMEM, HNM_EUNSUPPORTED, HNM_ECOLL = 0, -1, -2, -3, -4, -5, -6

_p = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int32
_f32 = C.c_float


class NcfWeights(C.Structure):
    """hnm_ncf_weights (include/hnm.h)."""
    _fields_ = [("gmf_user", _p), ("gmf_item", _p), ("mlp_user", _p), ("mlp_item", _p),
                ("w1", _p), ("b1", _p), ("w2", _p), ("b2", _p), ("wp", _p), ("bp", _p),
                ("num_users", _i64), ("num_items", _i64), ("mf", _i32), ("h0", _i32),
                ("h1", _i32), ("h2", _i32), ("item_proj", _p)]


class NcfDeepWeights(C.Structure):
    """hnm_ncf_deep_weights (include/hnm.h)."""
    _fields_ = [("gmf_user", _p), ("gmf_item", _p), ("mlp_user", _p), ("mlp_item", _p),
                ("w", _p * 8), ("b", _p * 8), ("wp", _p), ("bp", _p),
                ("num_users", _i64), ("num_items", _i64), ("mf", _i32), ("nl", _i32),
                ("dims", _i32 * 9)]


class WideDeepWeights(C.Structure):
    """hnm_widedeep_weights (include/hnm.h)."""
    _fields_ = [(n, _p) for n in (
        "deep_user", "deep_item", "w1", "b1", "bn1_w", "bn1_b", "bn1_mean", "bn1_var",
        "w2", "b2", "bn2_w", "bn2_b", "bn2_mean", "bn2_var",
        "w3", "b3", "bn3_w", "bn3_b", "bn3_mean", "bn3_var",
        "wide_user", "wide_item", "wide_feat", "final_deep", "final_b",
        "duf_w", "duf_b", "wuf_w", "wuf_b")] + [
        ("num_users", _i64), ("num_items", _i64),
        ("d", _i32), ("l1_in", _i32), ("l1", _i32), ("l2", _i32), ("l3", _i32),
        ("num_user_features", _i32), ("eps", _f32)]


class WideDeepItemFeatures(C.Structure):
    """hnm_widedeep_item_features (include/hnm.h)."""
    _fields_ = [("dif_w", _p), ("dif_b", _p), ("wif_w", _p), ("wif_b", _p), ("wide_feat", _p),
                ("num_item_features", _i32)]


_SIGS = {
    "hnm_abi_version": (C.c_int, []),
    "hnm_last_error": (C.c_char_p, []),
    "hnm_ctx_create": (_i32, [C.c_int, C.POINTER(_p)]),
    "hnm_ctx_destroy": (_i32, [_p]),
    "hnm_ctx_set_stream": (_i32, [_p, _p]),
    "hnm_ctx_reserve": (_i32, [_p, C.c_size_t]),
    "hnm_ctx_check": (_i32, [_p]),
    "hnm_ctx_num_cus": (_i32, [_p, C.POINTER(C.c_int)]),
    "hnm_ctx_abort_pending": (_i32, [_p]),
    "hnm_ctx_enable_timing": (_i32, [_p, C.c_int]),
    "hnm_ctx_timing": (_i32, [_p, C.POINTER(C.c_double), C.POINTER(_i64)]),
    "hnm_ctx_set_option": (_i32, [_p, C.c_int, _i64]),
    "hnm_ctx_prefilter_stats": (_i32, [_p, C.POINTER(_i64), C.c_int]),
    "hnm_ctx_prefilter_stats_ex": (_i32, [_p, C.POINTER(_i64), C.c_int, C.c_int]),
    "hnm_gather_rows_f32": (_i32, [_p, _p, _i64, _i64, C.c_int, _p, _i64, _p, _i64]),
    "hnm_linear_rows_f32": (_i32, [_p, _p, _i64, _p, _i64, _i64, C.c_int, _p, _i64, _p,
                                   C.c_int, _p, _i64, C.c_int]),
    "hnm_dot_topk_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int, _p, _p,
                                _p, _p, _p, C.c_int, _p, _p]),
    "hnm_dot_topk_begin_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int, _p,
                                      _p, _p, _p, _p, C.c_int, _p]),
    "hnm_pack_candidates_i32": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "hnm_topk_merge_sorted_pairs_i32": (_i32, [_p, _p, _i64, _i64, C.c_int, C.c_int, _p, _p]),
    "hnm_topk_lists_kth_f32": (_i32, [_p, _p, _i64, _i64, C.c_int, C.c_int, _p]),
    "hnm_dot_topk_begin_lists_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int,
                                            _p, _p, _p, _p, _p, C.c_int, _p]),
    "hnm_dot_topk_finish_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int, _p,
                                       _p, _p, _p, _p, C.c_int, _p, C.c_int, _p, _p]),
    "hnm_dot_prefilter_debug_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int,
                                           _p, _p, _p, _p, _i64, _p]),
    "hnm_dot_scores_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64, C.c_int, _p,
                                  _p, _p, _p, _i64]),
    "hnm_pair_dot_f32": (_i32, [_p, _p, _i64, _i64, _p, _i64, _i64, C.c_int, _p, _p, _i64, _p,
                                _p, _p, _p]),
    "hnm_ncf_topk_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _p, C.c_int, _p, _p]),
    "hnm_ncf_topk_begin_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _p, C.c_int, _p]),
    "hnm_ncf_topk_begin_lists_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _p, C.c_int,
                                            _p]),
    "hnm_ncf_topk_finish_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _p, C.c_int, _p,
                                       C.c_int, _p, _p]),
    "hnm_ncf_scores_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _i64]),
    "hnm_ncf_item_proj_f32": (_i32, [_p, C.POINTER(NcfWeights), _p]),
    "hnm_ncf_deep_scores_f32": (_i32, [_p, C.POINTER(NcfDeepWeights), _p, _i64, _p, _p, _i64]),
    "hnm_ncf_deep_topk_f32": (_i32, [_p, C.POINTER(NcfDeepWeights), _p, _i64, _p, _p, C.c_int,
                                     _p, _p]),
    "hnm_ncf_deep_prefilter_debug_f32": (_i32, [_p, C.POINTER(NcfDeepWeights), _p, _i64, _p,
                                                _i64, _p]),
    "hnm_ncf_pair_scores_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _p, _i64, _p]),
    "hnm_ncf_prefilter_debug_f32": (_i32, [_p, C.POINTER(NcfWeights), _p, _i64, _p, _i64, _p]),
    "hnm_topk_merge_f32": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64, C.c_int, C.c_int, _p, _p]),
    "hnm_rccl_unique_id": (_i32, [_p, _i64]),
    "hnm_ctx_rccl_init": (_i32, [_p, C.c_int, C.c_int, _p, _i64]),
    "hnm_ctx_set_rccl_comm": (_i32, [_p, _p]),
    "hnm_ctx_rccl_abort": (_i32, [_p]),
    "hnm_topk_allgather_merge_f32": (_i32, [_p, _p, _p, _i64, C.c_int, _p, _p]),
    "hnm_topk_rows_f32": (_i32, [_p, _p, _i64, _i64, _i64, _p, _p, C.c_int, _p, _p]),
    "hnm_csr_build_norm": (_i32, [_p, _p, _p, _i64, _i64, _p, _p, _p]),
    "hnm_spmm_plan_create": (_i32, [_p, _i64, _p, C.POINTER(_p)]),
    "hnm_spmm_plan_prepare": (_i32, [_p, _p, _p, _p, C.c_int]),
    "hnm_spmm_plan_destroy": (_i32, [_p]),
    "hnm_spmm_plan_restrict": (_i32, [_p, _p, C.POINTER(_i64), C.c_int, C.POINTER(_p)]),
    "hnm_spmm_csr_f32": (_i32, [_p, _p, _i64, _p, _p, _p, _p, C.c_int, _p, _f32, _p, _p]),
    "hnm_spmm_csr_range_f32": (_i32, [_p, _p, _i64, _p, _p, _p, _p, C.c_int, _p, _f32, _p, _p,
                                      _f32, _i64, _i64, _i64]),
    "hnm_spmm_rows_combine_f32": (_i32, [_p, _p, _i64, _p, _p, _p, _p, _i64, C.c_int,
                                         C.POINTER(_p), C.POINTER(_f32), C.c_int, _p]),
    "hnm_axpby_f32": (_i32, [_p, _i64, _f32, _p, _f32, _p, _p]),
    "hnm_widedeep_topk_f32": (_i32, [_p, C.POINTER(WideDeepWeights), _p, _i64, _p, _p, _p,
                                     C.c_int, _p, _p]),
    "hnm_widedeep_scores_f32": (_i32, [_p, C.POINTER(WideDeepWeights), _p, _i64, _p, _p, _i64]),
    "hnm_widedeep_pair_scores_f32": (_i32, [_p, C.POINTER(WideDeepWeights), _p, _p, _p, _i64,
                                            _p]),
    "hnm_widedeep_pair_scores_ex_f32": (_i32, [_p, C.POINTER(WideDeepWeights),
                                               C.POINTER(WideDeepItemFeatures), _p, _p, _p, _p,
                                               _i64, _p]),
    "hnm_widedeep_prefilter_debug_f32": (_i32, [_p, C.POINTER(WideDeepWeights), _p, _i64, _p, _p,
                                                _i64, _p]),
    "hnm_widedeep_refine_debug_f32": (_i32, [_p, C.POINTER(WideDeepWeights), _p, _i64, _p, _p,
                                                _i64, _p]),
    "hnm_mask_gather_csr": (_i32, [_p, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _p, _p]),
    "hnm_rank_metrics_f64": (_i32, [_p, _p, _i64, _i64, _p, C.c_int, _p, _p, _i64, _p, _p, _p,
                                    _p, _p]),
}

_lib = None
_lock = threading.RLock()
_tls = threading.local()        # .ctxs: {device index: _Ctx} of the calling thread
_live = weakref.WeakSet()       # every live _Ctx (all threads), for device-wide options/stats


def declared_symbols():
    return sorted(_SIGS)


def load(path: str = LIB_PATH):
    """Load libhnm_mi355x.so (raises if it was not built -- no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"{path} is missing: the MI355X HIP library was not built "
                "(run `python -m hnm_recommendation_amd.build`). There is no CPU fallback.")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        if lib.hnm_abi_version() != 1:
            raise RuntimeError("libhnm_mi355x ABI version mismatch")
        _lib = lib
        return lib


def fn(name):
    lib = load()
    f = getattr(lib, name, None)
    if f is None:
        raise RuntimeError(f"{name} is not exported by {LIB_PATH}")
    return f


def check(status: int, what: str = ""):
    if status == HNM_OK:
        return
    msg = load().hnm_last_error().decode(errors="replace")
    if status == HNM_EOOB:
        raise IndexError(msg)
    if status in (HNM_EINVAL, HNM_EUNSUPPORTED):
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what}: {msg} (status {status})")


def require_gpu(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise RuntimeError(
                "hnm_recommendation_amd runs on an AMD Instinct GPU (MI355X) through its HIP "
                "library; move the module and its inputs to a GPU device (model.to('cuda')). "
                "There is no CPU path.")


def _dev_index(device) -> int:
    dev = torch.device(device)
    return dev.index if dev.index is not None else torch.cuda.current_device()


_opts: dict = {}  # device -> {option: value}, applied to every ctx of that device


class _Ctx:
    """One hnm_ctx, owned by the thread-local slot of the thread that created it: when the
    thread exits its slot is cleared and the ctx (workspace, side stream, events) destroyed,
    so a server whose worker threads come and go does not accumulate contexts, and a new
    thread never inherits a dead thread's ctx (or its open two-phase call)."""
    __slots__ = ("handle", "device", "__weakref__")

    def __init__(self, device: int):
        h = _p()
        check(fn("hnm_ctx_create")(device, C.byref(h)), "hnm_ctx_create")
        self.handle, self.device = h, device

    def __del__(self):
        h, self.handle = self.handle, None
        lib = _lib
        if h and lib is not None:
            try:
                lib.hnm_ctx_destroy(h)  # synchronizes the device before freeing
            except Exception:
                pass


def _thread_ctx(idx: int) -> "_Ctx":
    slots = getattr(_tls, "ctxs", None)
    if slots is None:
        slots = _tls.ctxs = {}
    c = slots.get(idx)
    if c is None:
        c = _Ctx(idx)
        with _lock:
            for opt, val in _opts.get(idx, {}).items():
                check(fn("hnm_ctx_set_option")(c.handle, int(opt), int(val)), "hnm_ctx_set_option")
            _live.add(c)
        slots[idx] = c
    return c


def _device_ctxs(idx: int):
    with _lock:
        return [c for c in list(_live) if c.device == idx and c.handle]


def live_contexts(device=None) -> int:
    """Number of live hnm_ctx objects (all threads), optionally on one device."""
    if device is None:
        with _lock:
            return sum(1 for c in list(_live) if c.handle)
    return len(_device_ctxs(_dev_index(device)))


def ctx(device: torch.device):
    """The calling thread's hnm_ctx on `device`, bound to torch's current stream.

    One ctx per (device, thread): a ctx owns a workspace and the state of an open two-phase
    call, so concurrent callers (a threaded server) never share them; it lives as long as
    its thread.  Switching streams is ordered inside the library (hnm_ctx_set_stream queues
    the new stream behind the old one)."""
    idx = _dev_index(device)
    c = _thread_ctx(idx)
    stream = torch.cuda.current_stream(idx).cuda_stream
    check(fn("hnm_ctx_set_stream")(c.handle, _p(stream)), "hnm_ctx_set_stream")
    return c.handle


def abort_pending(device):
    """Close an open two-phase top-K call on this thread's ctx (after a failed exchange)."""
    check(fn("hnm_ctx_abort_pending")(ctx(device)), "hnm_ctx_abort_pending")


def sync_check(device):
    """Synchronize this thread's ctx stream and raise IndexError if one of this thread's
    calls saw an out-of-range id (per thread: each caller checks its own calls)."""
    check(fn("hnm_ctx_check")(ctx(device)), "hnm_ctx_check")


TIME_SCORE, TIME_SPMM = 1, 2


def enable_timing(device, on=True):
    """on: False/0 off, True/1 scoring kernels, 2 SpMM layers, 3 both."""
    check(fn("hnm_ctx_enable_timing")(ctx(device), int(on)), "hnm_ctx_enable_timing")


def kernel_timing(device):
    """(summed dominant-kernel ms, launches) of this thread's calls since enable_timing;
    syncs the stream (per thread, like enable_timing)."""
    t = C.c_double()
    n = _i64()
    check(fn("hnm_ctx_timing")(ctx(device), C.byref(t), C.byref(n)), "hnm_ctx_timing")
    return t.value, n.value


HNM_OPT_PREFILTER = 1
HNM_OPT_STATS = 3
HNM_OPT_STRIDED = 4
HNM_OPT_DEEP_MFMA = 5
HNM_OPT_LINEAR_MFMA = 6


def set_option(device, option, value):
    """Set a ctx option for every thread's ctx on `device` (current and future)."""
    idx = _dev_index(device)
    ctx(device)  # validates through the library first
    with _lock:
        _opts.setdefault(idx, {})[int(option)] = int(value)
    for c in _device_ctxs(idx):
        check(fn("hnm_ctx_set_option")(c.handle, int(option), int(value)), "hnm_ctx_set_option")


def set_prefilter(device, on=True):
    """Certified f16 pre-filter for top-K (default on); off = exact fp32 scan."""
    set_option(device, HNM_OPT_PREFILTER, int(bool(on)))


def prefilter_stats(device, reset=False, extended=False):
    """(rows scored, candidates re-scored in fp32, rows that took the exact fallback) summed
    over every thread's ctx on `device`; counted only while HNM_OPT_STATS is on
    (set_option(dev, HNM_OPT_STATS, 1)).  extended: a 4th count, rows whose bound also used
    the gated per-user strided sample (NeuralCF); extended="gate" adds the last NCF call's
    gate inputs (its proxies' predicted candidates without / with the strided sample).  Each read syncs the device; calls other
    threads issue meanwhile may be counted before or after a reset (exact when they are idle)."""
    ctx(device)
    n = (6 if extended == "gate" else 4) if extended else 3
    tot = [0] * n
    for c in _device_ctxs(_dev_index(device)):
        out = (_i64 * n)()
        check(fn("hnm_ctx_prefilter_stats_ex")(c.handle, out, n, int(reset)),
              "hnm_ctx_prefilter_stats_ex")
        for j in range(n):
            tot[j] += int(out[j])
    return tuple(tot)


def ptr(t):
    return None if t is None else _p(t.data_ptr())
