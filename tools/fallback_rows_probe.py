"""One certified NCF call whose exact fallback handles few rows, two ways: (a) bench.py's
"norms" weights, batch seed 101 (19 rows overflow their candidate segments), (b) 19 users with
one item row at 1e6 (every row's bound unusable).  Run under rocprofv3 to compare the two
fallback launches (ncf32_kernel with a device-side row list)."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from bench import build_workload  # noqa: E402
from hnm_recommendation_amd import NeuralCF, _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
wl, info, _ = build_workload("ncf", 0, 1, dev, 4096, False, "norms")
b = torch.from_numpy(syn.user_batch(syn.HM_USERS, 4096, seed=101)).to(dev)
for _ in range(2):
    wl["step"](b)
torch.cuda.synchronize()
del wl, info
U, I = 50000, syn.HM_ITEMS
sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=1, bias_scale=0.05)
sd = syn.stress_state_dict(sd, "big", syn.NCF_EMB_KEYS, "mlp_item_embedding.weight", 1)
m = NeuralCF(U, I)
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
m = m.to(dev).eval()
u = torch.from_numpy(syn.user_batch(U, 19, seed=9)).to(dev)
for _ in range(2):
    m.recommend_with_scores(u)
torch.cuda.synchronize()
print("done")
