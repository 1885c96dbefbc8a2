"""Throughput of the NCF recommend() step with independent batches in flight on 1, 2 or 3
HIP streams (run on the GPU box).

    python tools/stream_overlap.py [--steps 40] [--streams 1 2 3]

Each worker thread owns a torch stream and therefore its own hnm_ctx (one ctx per thread);
batches are dealt round-robin to the workers, every batch is a full `ncf_shard_topk` call
(per-call projections, bound statistics, champion sample, certified scan, re-scoring) --
nothing is shared or skipped.  The question: how much of a step's low-occupancy phases
(small prep kernels, champion sample, re-scoring) a second batch's work can fill.
Results are checked bitwise against the single-stream answers.
"""
import argparse
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hnm_recommendation_amd import NeuralCF  # noqa: E402
from hnm_recommendation_amd import sharding as S  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3])
    a = ap.parse_args()
    U, I, B = syn.HM_USERS, syn.HM_ITEMS, 4096
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    m = NeuralCF(U, I)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in syn.ncf_state_dict(U, I, seed=0).items()})
    m = m.to(dev).eval()
    sc = S.ncf_shard_topk(m, 0, I, 12)
    batches = [torch.from_numpy(syn.user_batch(U, B, seed=100 + j)).to(dev) for j in range(8)]
    ref = [sc(b) for b in batches]
    torch.cuda.synchronize()
    for ns in a.streams:
        streams = [torch.cuda.Stream() for _ in range(ns)]
        outs = [None] * a.steps
        start = threading.Barrier(ns + 1)

        def work(w):
            torch.cuda.set_device(0)
            with torch.cuda.stream(streams[w]):
                sc(batches[w % len(batches)])          # warm this thread's ctx
                torch.cuda.current_stream().synchronize()
                start.wait()
                for j in range(w, a.steps, ns):
                    outs[j] = sc(batches[j % len(batches)])
                torch.cuda.current_stream().synchronize()

        ts = [threading.Thread(target=work, args=(w,)) for w in range(ns)]
        for t in ts:
            t.start()
        start.wait()
        t0 = time.perf_counter()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        for j in range(a.steps):
            r = ref[j % len(batches)]
            assert torch.equal(outs[j][1], r[1]) and torch.equal(outs[j][0].view(torch.int32),
                                                                   r[0].view(torch.int32))
        print(f"streams {ns}: {B * a.steps / el:,.0f} users/s, {el / a.steps * 1e3:.4f} ms/batch "
              f"(bitwise equal to single-stream)", flush=True)


if __name__ == "__main__":
    main()
