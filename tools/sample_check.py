"""Diagnostic: 12th best of (approx - bound) over the tile sample vs the strided-item sample,
from the certified scan's debug output (hnm_ncf_prefilter_debug_f32), full bench shape."""
import numpy as np
import torch

from hnm_recommendation_amd import NeuralCF, _lib
from hnm_recommendation_amd import synthetic as syn

U, I, B, K = syn.HM_USERS, syn.HM_ITEMS, 64, 12
sd = syn.ncf_state_dict(U, I, 64, (128, 64, 32), seed=0)
m = NeuralCF(U, I)
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
m = m.to("cuda").eval()
users = torch.from_numpy(syn.user_batch(U, B, seed=1)).cuda()
w, keep = m._weights()
approx = torch.empty(B, I, device="cuda")
bound = torch.empty(B, I, device="cuda")
_lib.check(_lib.fn("hnm_ncf_prefilter_debug_f32")(_lib.ctx(users.device), w, _lib.ptr(users), B,
                                                  _lib.ptr(approx), I, _lib.ptr(bound)), "debug")
_lib.sync_check(users.device)
v = (approx - bound).cpu().numpy()
st = max(8, I // 12288)
items = np.arange(0, I, st)
tiles = np.concatenate([np.arange(t * 32, min(t * 32 + 32, I)) for t in range(0, (I + 31) // 32, st)])
for name, idx in (("items", items), ("tiles", tiles), ("all", np.arange(I))):
    k = np.sort(v[:, idx], axis=1)[:, -K]
    print(f"{name:6s} n={idx.size:6d}  mean K-th {k.mean():.6g}  std {k.std():.3g}")
ex = m.predict_all_items(users).cpu().numpy()
for name, idx in (("items", items), ("tiles", tiles)):
    k = np.sort(v[:, idx], axis=1)[:, -K]
    print(name, "exact-score rank of the sample K-th (mean):",
          float(np.mean([(ex[r] >= np.sort(ex[r, idx])[-K]).sum() for r in range(B)])))

# data-driven sample: top-N items by the mean (approx - bound) of a few of the batch's users
proxy_users = 16
proxy = v[:proxy_users].mean(axis=0)
order = np.argsort(-proxy)
rest = slice(proxy_users, B)
for N in (512, 1024, 2048, 4096, 8192, 13193):
    idx = order[:N]
    k = np.sort(v[rest][:, idx], axis=1)[:, -K]
    rank = np.mean([(ex[r] >= np.sort(ex[r, idx])[-K]).sum() for r in range(proxy_users, B)])
    cand = np.mean([(v[r] + 2 * (approx[r].cpu().numpy() - v[r] - approx[r].cpu().numpy()) * 0 >= 0).sum() for r in range(1)])
    print(f"proxy top-{N:5d}: mean K-th {k.mean():.6g}; exact rank of the sample K-th {rank:.1f}")
