"""Deep NeuralCF tower throughput: recommend (top-12) of a B-user batch over the full H&M
catalogue, the fp32-MFMA fused top-k (default) vs the per-pair LDS kernel + dense row top-k
(HNM_OPT_DEEP_MFMA = 0).  Prints one line per (tower, route) with ms / step, users/s and the
scan kernel's achieved fp32 rate (useful MACs: the MLP layers after the first, GMF and the
prediction layer).
    python tools/deep_probe.py [B] [steps]"""
import os
import sys
import time

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from hnm_recommendation_amd import NeuralCF, _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
DEV = torch.device("cuda", 0)
torch.cuda.set_device(0)
U, I = syn.HM_USERS, syn.HM_ITEMS
for mf, dims in [(64, (128, 64, 32, 16)), (32, (64, 32, 16, 8)), (64, (128, 64, 64, 32))]:
    sd = syn.ncf_state_dict(U, I, mf, dims, seed=3, bias_scale=0.05)
    m = NeuralCF(U, I, mf_dim=mf, mlp_dims=list(dims))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to(DEV).eval()
    users = torch.from_numpy(syn.user_batch(U, B, seed=1)).to(DEV)
    macs = mf + sum(dims[l] * dims[l + 1] for l in range(1, len(dims) - 1)) + dims[-1]
    for route, opt in (("mfma", 1), ("per-pair", 0)):
        _lib.set_option(DEV, _lib.HNM_OPT_DEEP_MFMA, opt)
        steps = STEPS if opt else 1
        with torch.no_grad():
            m.recommend_with_scores(users)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                m.recommend_with_scores(users)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        tf = 2.0 * macs * B * I / (ms * 1e-3) / 1e12
        print(f"mf {mf} mlp {list(dims)} {route:8s}: {ms:8.2f} ms/step  "
              f"{B / ms * 1e3:10.0f} users/s  {tf:6.1f} TF/s useful fp32", flush=True)
    _lib.set_option(DEV, _lib.HNM_OPT_DEEP_MFMA, 1)
    del m
    torch.cuda.empty_cache()
