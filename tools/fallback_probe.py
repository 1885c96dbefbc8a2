"""Timing of the exact fp32 NCF scan (ncf32_kernel: HNM_OPT_PREFILTER=0, every row) and of the
certified path at the full H&M catalogue for bench.py's weight sets: whether the exact scan's
cost depends on the weights (its top-K list inserts are data-dependent)."""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
for wt in sys.argv[1:] or ["init", "norms"]:
    wl, info, _ = build_workload("ncf", 0, 1, dev, 4096, False, wt)
    step = wl["step"]
    b = torch.from_numpy(syn.user_batch(syn.HM_USERS, 4096, seed=101)).to(dev)
    for pf in (False, True):
        _lib.set_prefilter(dev, pf)
        step(b)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step(b)
        torch.cuda.synchronize()
        print(f"{wt:10s} prefilter={pf}: {(time.perf_counter() - t0) / 3 * 1e3:8.3f} ms", flush=True)
    _lib.set_prefilter(dev, True)
    del wl, info, step
    torch.cuda.empty_cache()
