"""A/B of a ctx option on the same box and process: the bench step of a workload timed with the
option at each value, interleaved (7 rounds of `--steps` steps each), medians reported.
    python tools/ab_option.py <workload> <option id> [weights] [steps]
(e.g. 4 = HNM_OPT_STRIDED: the NCF gated strided sample vs the champion sample alone.)"""
import os
import statistics
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

wl_name, opt = sys.argv[1], int(sys.argv[2])
weights = sys.argv[3] if len(sys.argv) > 3 else "init"
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
wl, info, _ = build_workload(wl_name, 0, 1, dev, 4096, False, weights)
step = wl["step"]
batches = [torch.from_numpy(syn.user_batch(syn.HM_USERS, 4096, seed=100 + j)).to(dev) for j in range(4)]
res = {0: [], 1: []}
for rnd in range(7):
    for v in (1, 0) if rnd % 2 else (0, 1):
        _lib.set_option(dev, opt, v)
        for j in range(3):
            step(batches[j % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(steps):
            step(batches[j % 4])
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / steps * 1e3)
_lib.set_option(dev, opt, 1)
for v in (0, 1):
    print(f"{wl_name} {weights} option {opt}={v}: median {statistics.median(res[v]):.4f} ms/step "
          f"(runs {', '.join(f'{x:.4f}' for x in res[v])})", flush=True)
