"""W&D re-scoring cascade: how many scan survivors would a best-first refine leave? (GPU box)

    python tools/wd_best_first_probe.py [n_users]

For n users of the bench's configs[3] model (full H&M shape, 512-256-128 tower) this reads the
certified scan's approx/bound (hnm_widedeep_prefilter_debug_f32), the three-pass refined
approx/bound (hnm_widedeep_refine_debug_f32) and the exact scores over the whole catalogue and
counts, per row:
  survivors  items with scan ub >= Lu (Lu = the K-th best scan lower bound): what the cascade
             refines today (wdc_collect_kernel)
  best-first the M survivors with the best scan ub refined first; their K-th best refined lower
             bound L2' (a certified lower bound of the exact K-th); then only the remaining
             survivors with scan ub >= max(L2', Lu) -- refined count M + that
  exact      items the final exact pass re-scores (refined ub >= K-th best refined lb)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from hnm_recommendation_amd import WideDeep, _lib  # noqa: E402
from hnm_recommendation_amd import synthetic as syn  # noqa: E402


def debug(fn, m, users):
    w, keep = m._weights()
    B, I = users.numel(), m.num_items
    a = torch.empty(B, I, device=users.device)
    e = torch.empty(B, I, device=users.device)
    _lib.check(_lib.fn(fn)(_lib.ctx(users.device), w, _lib.ptr(users), B, None, _lib.ptr(a), I,
                           _lib.ptr(e)), fn)
    _lib.sync_check(users.device)
    return a.cpu().numpy().astype(np.float64), e.cpu().numpy().astype(np.float64)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    K = 12
    dev = torch.device("cuda", 0)
    U, I = syn.HM_USERS, syn.HM_ITEMS
    sd = syn.widedeep_state_dict(U, I, 64, (512, 256, 128), seed=0)
    m = WideDeep(U, I)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev).eval()
    del sd
    users = torch.from_numpy(syn.user_batch(U, n, seed=11)).to(dev)
    sa, se = debug("hnm_widedeep_prefilter_debug_f32", m, users)
    ra, re = debug("hnm_widedeep_refine_debug_f32", m, users)
    ex = m.predict_all_items(users).cpu().numpy().astype(np.float64)
    rows = []
    for b in range(n):
        slb, sub = sa[b] - se[b], sa[b] + se[b]
        rlb, rub = ra[b] - re[b], ra[b] + re[b]
        Lu = np.sort(slb)[-K]
        surv = np.nonzero(sub >= Lu)[0]
        kth = np.sort(ex[b])[-K]
        assert (rlb <= ex[b] + 1e-6 * np.abs(ex[b]).max()).all()
        row = {"survivors": len(surv)}
        L2all = np.sort(rlb[surv])[-K]
        row["exact"] = int((rub[surv] >= max(L2all, Lu)).sum())
        for M in (32, 64, 128, 256):
            order = surv[np.lexsort((surv, -sub[surv]))]
            top = order[:M]
            L2p = np.sort(rlb[top])[-K] if len(top) >= K else -np.inf
            rest = order[M:]
            nb = int((sub[rest] >= max(L2p, Lu)).sum())
            row[f"M{M}"] = len(top) + nb
            assert L2p <= kth + 1e-6 * abs(kth)
        row["gap_scan_e"] = float(np.median(se[b][surv]))
        row["gap_ref_e"] = float(np.median(re[b][surv]))
        row["kth_minus_Lu"] = float(kth - Lu)
        rows.append(row)
    keys = list(rows[0])
    print("per-row means over", n, "users (W&D configs[3], init weights):")
    for k in keys:
        print(f"  {k:14s} {np.mean([r[k] for r in rows]):12.4g}   "
              f"min {np.min([r[k] for r in rows]):10.4g}  max {np.max([r[k] for r in rows]):10.4g}")


if __name__ == "__main__":
    main()
