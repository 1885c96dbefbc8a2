"""SpMM layer split into its two halves on the full synthetic H&M graph (run on the GPU box).

    python tools/spmm_halves.py [--d 64] [--reps 10] [--dump out.npz]

The bipartite graph's user rows gather ITEM rows (a 105,542-row table: 27 MB at d = 64,
Infinity-Cache resident) and its item rows gather USER rows (1,371,980 rows: 351 MB, past
the Infinity Cache); MI355X_MICROARCH.md's gather ceilings differ for the two (8.6 TB/s for a
38 MB table, 7.4-7.9 TB/s for 151 MB, ~7.2 TB/s at 358 MB by tools/gather_probe.hip).  This
times hnm_spmm_csr_range_f32 over [0, U) (users), [U, N) (items, incl. the heavy segmented
rows on the side stream) and [0, N) (a whole layer) with torch events on the ctx stream, and
prints each half's gathered bytes (entries x d x 4) and rate.  The library is the in-tree
build unless HNM_LIB_PATH names a variant.  --dump saves sampled rows of a 3-layer forward()
for cross-variant comparison.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hnm_recommendation_amd import LightGCN, _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    U, I, d = syn.HM_USERS, syn.HM_ITEMS, a.d
    N = U + I
    m = LightGCN(U, I, embedding_dim=d, num_layers=3)
    m.set_graph(torch.from_numpy(syn.bipartite_edge_index(U, I, syn.HM_INTERACTIONS, seed=2)))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in syn.lightgcn_state_dict(U, I, d, seed=0).items()})
    m = m.to("cuda:0").eval()
    g = m._device_graph()
    X = m.embeddings.weight.detach()
    Y = torch.empty_like(X)
    acc = torch.empty_like(X)
    rp = g.rowptr.cpu()
    nnz_u, nnz_i = int(rp[U]), int(rp[N] - rp[U])
    halves = {"users": (0, U, nnz_u), "items": (U, N, nnz_i), "layer": (0, N, nnz_u + nnz_i)}
    out = {"lib": os.environ.get("HNM_LIB_PATH", "in-tree"), "d": d}
    for name, (r0, r1, nnz) in halves.items():
        for _ in range(2):
            g.spmm(X, Y, 0.25, acc, rows=(r0, r1))
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.spmm(X, Y, 0.25, acc, rows=(r0, r1))
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        gathered = nnz * d * 4.0
        out[name] = {"ms": round(ms, 4), "entries": nnz, "gathered_GB": round(gathered / 1e9, 3),
                     "gather_TBps": round(gathered / (ms * 1e-3) / 1e12, 3)}
        print(name, out[name], flush=True)
    _lib.sync_check("cuda:0")
    if a.dump:
        fu, fi = m.forward()
        rng = np.random.default_rng(0)
        ur = rng.choice(U, 2000, replace=False)
        ir = rng.choice(I, 2000, replace=False)
        np.savez(a.dump, ur=ur, ir=ir, fu=fu[torch.from_numpy(ur).cuda()].cpu().numpy(),
                 fi=fi[torch.from_numpy(ir).cuda()].cpu().numpy())
    import json
    print(json.dumps(out))


if __name__ == "__main__":
    main()
