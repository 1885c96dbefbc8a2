"""Per-batch pre-filter statistics of the certified NCF step on bench.py's weight sets (rows,
candidates re-scored per row, exact-fallback rows, rows with the strided sample) and the
step time of each batch: which batches of a weight set leave the certified path, and why.
    python tools/robust_probe.py [--strided] [weights ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
args = sys.argv[1:]
if "--strided" in args:
    args.remove("--strided")
    _lib.set_option(dev, _lib.HNM_OPT_STRIDED, 1)
for wt in args or ["init", "personal", "norms", "student_t"]:
    wl, info, _ = build_workload("ncf", 0, 1, dev, 4096, False, wt)
    step = wl["step"]
    batches = [torch.from_numpy(syn.user_batch(syn.HM_USERS, 4096, seed=100 + j)).to(dev)
               for j in range(4)]
    for b in batches:
        step(b)
    torch.cuda.synchronize()
    for j, b in enumerate(batches):
        _lib.prefilter_stats(dev, reset=True)
        _lib.set_option(dev, _lib.HNM_OPT_STATS, 1)
        step(b)
        _lib.set_option(dev, _lib.HNM_OPT_STATS, 0)
        rows, cands, fb, smp, g0, g1 = _lib.prefilter_stats(dev, reset=True, extended="gate")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            step(b)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        # the same timing with the counters on (atomics): a stats-dependent path would show here
        _lib.set_option(dev, _lib.HNM_OPT_STATS, 1)
        t0 = time.perf_counter()
        for _ in range(5):
            step(b)
        torch.cuda.synchronize()
        ms_on = (time.perf_counter() - t0) / 5 * 1e3
        _lib.set_option(dev, _lib.HNM_OPT_STATS, 0)
        rows2, cands2, fb2, smp2, _, _ = _lib.prefilter_stats(dev, reset=True, extended="gate")
        print(f"{wt:10s} batch {j}: {ms:7.3f} ms (counters on {ms_on:7.3f})  candidates/row "
              f"{cands / max(rows - fb, 1):7.1f}  fallback {fb:5d}  strided {smp}  "
              f"| 5 more: fallback {fb2} strided {smp2} | gate proxies {g0 / 8:.0f} -> {g1 / 8:.0f}",
              flush=True)
    del wl, info, step
    torch.cuda.empty_cache()
