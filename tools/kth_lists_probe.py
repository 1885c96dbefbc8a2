"""Time the item-shard exchange's k-th best of G bound lists: the HIP merge vs torch.topk.
    python tools/kth_lists_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hnm_recommendation_amd import sharding as S
v = torch.sort(torch.randn(8, 32768, 12, device="cuda"), dim=2, descending=True).values
for name, f in (("hip merge", lambda: S._kth_of_lists(v, 12)),
                ("torch.topk", lambda: torch.topk(v.permute(1, 0, 2).reshape(32768, 96), 12, dim=1).values[:, 11].contiguous())):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50): f()
    torch.cuda.synchronize()
    print(name, round((time.perf_counter() - t) / 50 * 1e6, 1), "us per call, [8, 32768, 12]")
