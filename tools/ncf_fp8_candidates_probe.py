"""VERDICT r5 #3, step two: how many candidates a row an e4m3 (fp8) first pass of the certified
NCF scan would leave.  The scan's bound e(u, i) = 6u (c0 + A_u + B_i + C_u D_i) is linear in the
unit roundoff u of its operands (f16: 2^-11); an e4m3 layer 2 (u = 2^-4) multiplies the layer-2
terms by 2^7.  Counted here with a PERFECT sample (threshold = the row's exact K-th, the best any
sample can give) and the whole bound scaled by f (f = 128 over-counts slightly: the GMF term
C_u D_i would stay f16), for the bench's weight sets.
    python tools/ncf_fp8_candidates_probe.py [weights ...]"""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402
from test_gpu_prefilter import prefilter_debug  # noqa: E402

K, NU = 12, 64
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
for wt in sys.argv[1:] or ["init", "personal"]:
    wl, info, _ = build_workload("ncf", 0, 1, dev, 4096, False, wt)
    m = info["_module"]
    users = torch.from_numpy(syn.user_batch(syn.HM_USERS, NU, seed=100)).to(dev)
    approx, bound = prefilter_debug(m, users)
    bp = float(m.prediction_layer.bias.detach())
    exact = m.predict_all_items(users)
    kth = exact.topk(K, dim=1).values[:, K - 1:K]
    I = exact.shape[1]
    for f in (1, 16, 128):
        c = ((approx + bp + f * bound) >= kth).sum(1).float()
        print(f"{wt:9s} bound x {f:3d} ({'f16' if f == 1 else 'e4m3 layer 2' if f == 128 else 'e5m2-like'}): "
              f"perfect-sample candidates/row mean {c.mean().item():9.1f} median {c.median().item():9.1f} "
              f"max {c.max().item():9.0f} = {c.mean().item() / I:.4f} of the catalogue", flush=True)
    del wl, info, m, approx, bound, exact
    torch.cuda.empty_cache()
