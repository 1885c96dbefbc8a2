"""GPU: BASELINE configs[2] pinned at FULL graph size -- LightGCN d=64, 3 layers, on the
synthetic H&M adjacency (1,371,980 users + 105,542 items, 31.8M interactions stored
symmetric: 65,054,170 CSR entries with self-loops).

The reference goldens (tests/golden/lightgcn_*.npz) pin `oracle/torch_cpu.lightgcn_forward`
(the reference's `torch.sparse.mm` propagation restated, test_torch_cpu_baseline.py); here
that CPU propagation runs on the full graph and is compared with the HIP SpMM path on
sampled rows:

* 48 random users and the 4 highest-degree users (short rows: the column-ordered short walk,
  spmm_swalk_kernel), and 16 item rows of more than 2,048 entries (the user-ordered walk,
  split into pieces summed by spmm_walk_finish_kernel) -- including the 4 most popular items
  and the 4 shortest of those rows -- within 1e-4 of the row scale;
* the top-12 of every sampled user against the CPU's dense F_U[u] @ F_I^T scores
  (identical sets up to near-ties at the 12th, scores within 1e-4);
* `propagate_for` (what recommend() and the bench step run) bit-identical to forward().
(Reference: lightgcn.py:136-164, 188-204.)
"""
import os

import numpy as np
import pytest
import torch

from parity import assert_topk_equivalent
from hnm_recommendation_amd import LightGCN
from hnm_recommendation_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
K = 12
HEAVY = 2048


def test_lightgcn_d64_full_graph_vs_cpu_reference():
    U, I, E, d = syn.HM_USERS, syn.HM_ITEMS, syn.HM_INTERACTIONS, 64
    ei = torch.from_numpy(syn.bipartite_edge_index(U, I, E, seed=2))
    sd = syn.lightgcn_state_dict(U, I, d, seed=0)
    m = LightGCN(U, I, embedding_dim=d, num_layers=3)
    m.set_graph(ei)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(DEV).eval()
    g = m._device_graph()
    assert g.nnz == 2 * E + U + I
    deg = (g.rowptr[1:] - g.rowptr[:-1]).cpu().numpy()          # entries incl. self-loop
    rng = np.random.default_rng(17)
    users = np.concatenate([rng.choice(U, 48, replace=False), np.argsort(deg[:U])[-4:]])
    items_deg = deg[U:]
    heavy = np.nonzero(items_deg > HEAVY)[0]
    assert heavy.size >= 16, heavy.size
    by_deg = heavy[np.argsort(items_deg[heavy])]
    items = np.unique(np.concatenate([by_deg[:4], by_deg[-4:],
                                      rng.choice(heavy, 8, replace=False)]))
    ut = torch.from_numpy(users).to(DEV)
    fu, fi = m.forward()
    fb, fi_b = m.propagate_for(ut)
    assert torch.equal(fi_b, fi) and torch.equal(fb, fu[ut])
    got_u = fu[ut].cpu().numpy()
    got_i = fi[torch.from_numpy(items).to(DEV)].cpu().numpy()
    v, idx = m.recommend_with_scores(ut)
    v, idx = v.cpu().numpy(), idx.cpu().numpy()
    del fu, fi, fb, fi_b, m, g
    torch.cuda.empty_cache()

    from oracle import torch_cpu as T
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    graph = T.lightgcn_graph(ei, U + I)
    del ei
    cu, ci = T.lightgcn_forward(torch.from_numpy(sd["embeddings.weight"]), graph, U)
    del graph
    ref_u = cu[torch.from_numpy(users)].numpy()
    ref_i = ci[torch.from_numpy(items)].numpy()
    for got, ref, what in ((got_u, ref_u, "user rows"), (got_i, ref_i, "heavy item rows")):
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4 * float(np.abs(ref).max()),
                                   err_msg=what)
    dense = (torch.from_numpy(ref_u) @ ci.t()).numpy()
    assert_topk_equivalent(idx, dense, K, what="lightgcn d=64 full graph top-12 vs CPU reference")
    np.testing.assert_allclose(v, np.take_along_axis(dense, idx, 1), rtol=1e-4,
                               atol=1e-4 * float(np.abs(dense).max()))
