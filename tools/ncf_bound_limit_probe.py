"""How many candidates a row the certified NCF scan would keep with a PERFECT sample: the
threshold at the row's exact K-th best score itself, so only the bound's width admits extra
items (items with approx + e >= exact K-th).  Against the measured candidates a row (champion
sample, optionally the strided sample) this says whether a weight set is sample-limited (a
better sample would help) or bound-limited (only a tighter bound would).
    python tools/ncf_bound_limit_probe.py [weights ...]     (bench.py's weight sets)"""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402
from test_gpu_prefilter import prefilter_debug  # noqa: E402

K, NU = 12, 64
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
for wt in sys.argv[1:] or ["init", "personal", "norms", "student_t"]:
    wl, info, _ = build_workload("ncf", 0, 1, dev, 4096, False, wt)
    m = info["_module"]
    users = torch.from_numpy(syn.user_batch(syn.HM_USERS, NU, seed=100)).to(dev)
    approx, bound = prefilter_debug(m, users)
    bp = float(m.prediction_layer.bias.detach())
    exact = m.predict_all_items(users)
    kth = exact.topk(K, dim=1).values[:, K - 1:K]
    oracle = ((approx + bp + bound) >= kth).sum(1).float()
    # the measured candidates of the real step on a 4,096-row batch containing these users
    batch = torch.from_numpy(syn.user_batch(syn.HM_USERS, 4096, seed=100)).to(dev)
    _lib.prefilter_stats(dev, reset=True)
    _lib.set_option(dev, _lib.HNM_OPT_STATS, 1)
    wl["step"](batch)
    _lib.set_option(dev, _lib.HNM_OPT_STATS, 0)
    rows, cands, fb = _lib.prefilter_stats(dev, reset=True)
    rel = (bound / exact.std(1, keepdim=True)).mean().item()
    print(f"{wt:10s}: perfect-sample candidates/row mean {oracle.mean().item():7.1f} "
          f"median {oracle.median().item():7.1f} max {oracle.max().item():7.0f} | measured "
          f"{cands / max(rows - fb, 1):7.1f} (fallback {fb}) | bound / score std {rel:.4f}",
          flush=True)
    del wl, info, m, approx, bound, exact
    torch.cuda.empty_cache()
