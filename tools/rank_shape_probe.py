"""Per-rank work of the item-sharded step at world W on ONE GPU (no collectives): each rank
scores all W*4096 users against its I/W items (bench.py --gpus W, weak scaling).  Times the
local two-phase scorer (begin + finish with the rank's own bounds) per W, the part of the
sharded step that grows with W beside the exchange.
    python tools/rank_shape_probe.py [ncf|mf|lightgcn|lightgcn128] [W list, e.g. 1,8] [modes]

lightgcn / lightgcn128 (configs[2] / configs[4]): the rank-0 step of the per-call propagation +
certified top-K with the propagation's item rows sharded ("sharded": restricted SpMM plans; the
two all_gathers of the [I, d] item rows STUBBED -- the other shards' rows are copied in from a
whole-graph run, the bytes the all_gather would move are printed) or replicated ("replicated":
every rank propagates the whole graph, the round-5 design), with the all_gathered bound lists."""
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


def lightgcn_probe(d):
    from hnm_recommendation_amd import LightGCN
    modes = (sys.argv[3] if len(sys.argv) > 3 else "sharded,replicated").split(",")
    edges = syn.bipartite_edge_index(U, I, syn.HM_INTERACTIONS, seed=2)
    m = LightGCN(U, I, embedding_dim=d, num_layers=3)
    m.set_graph(torch.from_numpy(edges))
    del edges
    sd = syn.lightgcn_state_dict(U, I, d, seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev).eval()
    g = m._device_graph()
    ref = [m.embeddings.weight.detach()]
    for _ in range(2):
        y = torch.empty_like(ref[0])
        g.spmm(ref[-1], y, 0.0, None)
        ref.append(y)
    F = m.propagate(g)
    base = None
    for W in WS:
        lo, hi = S.shard_range(I, 0, W)
        calls = [0]

        def stub(Y, lo=lo, hi=hi):
            want = ref[calls[0] % 2 + 1]
            Y[U:U + lo] = want[U:U + lo]
            Y[U + hi:] = want[U + hi:]
            calls[0] += 1
        ex_bytes = S.ItemRowExchange(U, I, 0, W).bytes_per_call(d) if W > 1 else 0
        users = [torch.from_numpy(syn.user_batch(U, W * B, seed=s)).to(dev) for s in range(3)]
        bounds = []
        for u in users:   # every shard's k best sample bounds, merged (the bound exchange)
            allv = []
            for r in range(W):
                sc = S.dot_shard_topk(F[:U], F[U:], *S.shard_range(I, r, W), K)
                allv.append(sc.begin_lists(u))
                sc.abort()
            bounds.append(torch.topk(torch.cat(allv, dim=1), K, dim=1).values[:, K - 1].contiguous())
        scs = {"sharded": S.lightgcn_shard_topk(m, lo, hi, K, exchange=stub if W > 1 else None),
               "replicated": S.lightgcn_shard_topk(m, lo, hi, K)}
        outs = {}

        def step(mode, s):
            sc = scs[mode]
            sc.begin_lists(users[s % 3])
            return sc.finish(users[s % 3], bounds[s % 3])
        for mode in modes:
            outs[mode] = [step(mode, s) for s in range(3)]
        if len(modes) > 1:
            a, b = outs[modes[0]], outs[modes[1]]
            same = all(torch.equal(x[1], y[1]) and torch.equal(x[0].view(torch.int32), y[0].view(torch.int32))
                       for x, y in zip(a, b))
            print(f"lightgcn d={d} W={W}: {modes[0]} == {modes[1]} bitwise: {same}", flush=True)
        torch.cuda.synchronize()
        n, reps = 10, 7
        times = {mode: [] for mode in modes}
        for _ in range(reps):
            for mode in modes:
                t0 = time.perf_counter()
                for s in range(n):
                    step(mode, s)
                torch.cuda.synchronize()
                times[mode].append((time.perf_counter() - t0) / n * 1e3)
        for mode in modes:
            ms = float(np.median(times[mode]))
            base = base if base is not None else ms
            print(f"lightgcn d={d} W={W} [{mode}]: {W * B} users x {hi - lo} items: {ms:.3f} ms per "
                  f"rank step (local, median of {reps}; all_gathers stubbed: 2 x {ex_bytes / 1e6:.1f} MB "
                  f"received per rank per step); whole job {W * B / ms * 1e3 / 1e6:.3f} M users/s "
                  f"before the exchanges = {base / ms:.3f} of W x the W=1 rate", flush=True)


if w.startswith("lightgcn"):
    lightgcn_probe(128 if w == "lightgcn128" else 64)
    sys.exit(0)
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
