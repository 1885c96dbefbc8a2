"""Per-rank work of the item-sharded step at world W on ONE GPU (no collectives): each rank
scores all W*4096 users against its I/W items (bench.py --gpus W, weak scaling).  Times the
local two-phase scorer (begin + finish with the rank's own bounds) per W, the part of the
sharded step that grows with W beside the exchange.
    python tools/rank_shape_probe.py [ncf|mf] [W list, e.g. 1,8] [modes, e.g. max,lists,ideal]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hnm_recommendation_amd import MatrixFactorization, NeuralCF, _lib  # noqa: E402
from hnm_recommendation_amd import sharding as S  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

K, B = 12, 4096
U, I = syn.HM_USERS, syn.HM_ITEMS
w = sys.argv[1] if len(sys.argv) > 1 else "ncf"
WS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
# bound exchange(s), comma-separated, timed interleaved in one process (box clock drift
# cancels): "lists" (ncf default: every shard's k best sample bounds all_gathered, the k-th of
# their union -- what ItemShardedRecommender does), "max" (all_reduce of the shards' single
# bounds; the dot scorer's protocol), "ideal" (the single-GPU bound: an exchange's best case)
MODES = (sys.argv[3] if len(sys.argv) > 3 else ("lists" if w == "ncf" else "max")).split(",")
dev = torch.device("cuda", 0)
if w == "ncf":
    sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0)
    m = NeuralCF(U, I)
else:
    sd = syn.mf_state_dict(U, I, 64, seed=0)
    m = MatrixFactorization(U, I, sparse=False)
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
m = m.to(dev).eval()
base = None
for W in WS:
    lo, hi = S.shard_range(I, 0, W)
    if w == "ncf":
        sc = S.ncf_shard_topk(m, lo, hi, K)
    else:
        sc = S.dot_shard_topk(m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(),
                              lo, hi, K, user_bias=m.user_bias.weight.detach(),
                              item_bias=m.item_bias.weight.detach(), const_bias=m.global_bias.detach())
    users = [torch.from_numpy(syn.user_batch(U, W * B, seed=s)).to(dev) for s in range(3)]
    # the exchange's all_reduce(MAX) of every shard's bounds, computed once per batch outside
    # the timing (the other shards' begin phases are the other ranks' work)
    others = []
    for r in range(1, W):
        olo, ohi = S.shard_range(I, r, W)
        others.append(S.ncf_shard_topk(m, olo, ohi, K) if w == "ncf" else S.dot_shard_topk(
            m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(), olo, ohi, K,
            user_bias=m.user_bias.weight.detach(), item_bias=m.item_bias.weight.detach(),
            const_bias=m.global_bias.detach()))
    full = None
    if "ideal" in MODES:
        full = S.ncf_shard_topk(m, 0, I, K) if w == "ncf" else S.dot_shard_topk(
            m.user_embeddings.weight.detach(), m.item_embeddings.weight.detach(), 0, I, K,
            user_bias=m.user_bias.weight.detach(), item_bias=m.item_bias.weight.detach(),
            const_bias=m.global_bias.detach())
    bounds = {}
    for mode in MODES:
        bounds[mode] = []
        for u in users:
            if mode == "lists":
                allv = [sc.begin_lists(u)]
                sc.abort()
                for o in others:
                    allv.append(o.begin_lists(u))
                    o.abort()
                bounds[mode].append(torch.topk(torch.cat(allv, dim=1), K, dim=1).values[:, K - 1].contiguous())
                continue
            lb = sc.begin(u)
            sc.abort()
            for o in others:
                lb = torch.maximum(lb, o.begin(u))
                o.abort()
            if mode == "ideal":
                lb = torch.maximum(lb, full.begin(u))
                full.abort()
            bounds[mode].append(lb)

    def step(mode, s):
        u = users[s % 3]
        if mode == "lists":
            sc.begin_lists(u)
            return sc.finish(u, bounds[mode][s % 3])
        lb = sc.begin(u)
        return sc.finish(u, torch.maximum(lb, bounds[mode][s % 3]))

    for mode in MODES:
        for s in range(3):
            step(mode, s)
    torch.cuda.synchronize()
    n, reps = 10, 7
    times = {mode: [] for mode in MODES}
    for _ in range(reps):
        for mode in MODES:
            t0 = time.perf_counter()
            for s in range(n):
                step(mode, s)
            torch.cuda.synchronize()
            times[mode].append((time.perf_counter() - t0) / n * 1e3)
    for mode in MODES:
        ms = float(np.median(times[mode]))
        base = base if base is not None else ms
        print(f"{w} W={W} [{mode}]: {W * B} users x {hi - lo} items: {ms:.3f} ms per rank step "
              f"(local, median of {reps}); whole job {W * B / ms * 1e3 / 1e6:.3f} M users/s before "
              f"the exchange = {base / ms:.3f} of W x the W=1 rate", flush=True)
