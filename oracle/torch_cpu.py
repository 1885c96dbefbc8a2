"""CPU BASELINE: the reference's PyTorch-CPU path restated with torch ops -- TEST / BENCH
INFRASTRUCTURE ONLY (imported by `bench.py`'s `cpu_baseline` leg and by `tests/`; the
product path never calls it).

`oracle/hnm_oracle.py` is the numpy checker; this module is the *timed* CPU baseline the
north_star asks for ("the reference's PyTorch-CPU path timed on the same box's host
cores").  The reference cannot travel to the GPU box, so its hot path is restated here in
the same torch operators, chunk sizes and data flow, citing the lines each step follows:
embedding gathers, `expand` + `cat` over 1000-item chunks, `nn.Linear` layers, ReLU, the
prediction layer, `torch.topk` (NeuralCF); the layer-wise sparse propagation + `matmul`
(LightGCN); `matmul` + bias broadcast (MatrixFactorization); the one-hot wide input +
deep tower over 500-item chunks (Wide&Deep).  Eval mode: dropout is the identity and
BatchNorm uses its running statistics.  `tests/test_torch_cpu_baseline.py` checks every
function here against the reference-produced golden fixtures.

The one substitution: the reference's `torch_sparse.SparseTensor @ X` (`lightgcn.py:152`;
torch_sparse is not installed anywhere in this image) becomes `torch.sparse.mm` on a CSR
tensor with the same (duplicate-summing) semantics.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def as_torch(sd: Dict[str, np.ndarray]) -> Dict[str, Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}


def _topk(scores: Tensor, k: int, user_ids: Tensor, filter_items=None) -> Tensor:
    """`recommend` tail (`neural_cf.py:314-324`): -inf mask loop, then torch.topk."""
    if filter_items is not None:
        for i, u in enumerate(user_ids.tolist()):
            if u in filter_items:
                scores[i, list(filter_items[u])] = float("-inf")
    return torch.topk(scores, k, dim=1)


# --------------------------------------------------------------------------- NeuralCF
def ncf_predict_all_items(sd: Dict[str, Tensor], user_ids: Tensor) -> Tensor:
    """`NeuralCF.predict_all_items` (`neural_cf.py:143-208`)."""
    B = user_ids.shape[0]
    gmf_user = F.embedding(user_ids, sd["gmf_user_embedding.weight"])        # :155
    mlp_user = F.embedding(user_ids, sd["mlp_user_embedding.weight"])        # :156
    num_items = sd["gmf_item_embedding.weight"].shape[0]
    all_items = torch.arange(num_items)
    gmf_items = F.embedding(all_items, sd["gmf_item_embedding.weight"])      # :160
    mlp_items = F.embedding(all_items, sd["mlp_item_embedding.weight"])      # :161
    layers = sorted({int(k.split(".")[1]) for k in sd if k.startswith("mlp_layers.")})
    scores = []
    for s in range(0, num_items, 1000):                                       # :167-168
        e = min(s + 1000, num_items)
        n = e - s
        gu = gmf_user.unsqueeze(1).expand(B, n, -1)                          # :173
        mu = mlp_user.unsqueeze(1).expand(B, n, -1)                          # :176
        gi = gmf_items[s:e].unsqueeze(0).expand(B, -1, -1)                   # :181
        mi = mlp_items[s:e].unsqueeze(0).expand(B, -1, -1)                   # :184
        gmf_out = gu * gi                                                    # :189
        x = torch.cat([mu, mi], dim=2).view(-1, 2 * mu.shape[-1])            # :192-194
        for li in layers:                                                    # :195 mlp_layers
            x = F.relu(F.linear(x, sd[f"mlp_layers.{li}.weight"], sd[f"mlp_layers.{li}.bias"]))
        mlp_out = x.view(B, n, -1)
        cat = torch.cat([gmf_out, mlp_out], dim=2)                           # :199
        s_ = F.linear(cat.view(-1, cat.shape[-1]), sd["prediction_layer.weight"],
                      sd["prediction_layer.bias"]).view(B, -1)               # :200-201
        scores.append(s_)
    return torch.cat(scores, dim=1)                                          # :206


def ncf_recommend(sd, user_ids, k=12, filter_items=None):
    """`NeuralCF.recommend` (`neural_cf.py:300-326`) -> (values, indices)."""
    with torch.no_grad():
        return _topk(ncf_predict_all_items(sd, user_ids), k, user_ids, filter_items)


# --------------------------------------------------------------------------- LightGCN
def lightgcn_graph(edge_index: Tensor, num_nodes: int, edge_weight: Optional[Tensor] = None):
    """`LightGCN.set_graph` + `_add_self_loops` (`lightgcn.py:81-134`) as a CSR tensor:
    self-loops appended, deg = scatter-add of the weights over rows, D^-1/2 (A+I) D^-1/2
    with inf -> 0; duplicate edges are summed by the CSR conversion, as torch_sparse's
    SpMM sums them."""
    E = edge_index.shape[1]
    w = torch.ones(E) if edge_weight is None else edge_weight.float()
    loop = torch.arange(num_nodes)
    row = torch.cat([edge_index[0], loop])
    col = torch.cat([edge_index[1], loop])
    w = torch.cat([w, torch.ones(num_nodes)])
    deg = torch.zeros(num_nodes).index_add_(0, row, w)                       # :103
    dinv = deg.pow(-0.5)
    dinv[torch.isinf(dinv)] = 0                                              # :105
    val = dinv[row] * w * dinv[col]                                          # :106
    coo = torch.sparse_coo_tensor(torch.stack([row, col]), val, (num_nodes, num_nodes))
    return coo.coalesce().to_sparse_csr()


def lightgcn_alphas(num_layers, alpha=None):
    """`lightgcn.py:59-67`."""
    if alpha is None:
        return [1.0 / (num_layers + 1)] * (num_layers + 1)
    a = [alpha ** i for i in range(num_layers + 1)]
    return [x / sum(a) for x in a]


def lightgcn_forward(weight: Tensor, graph, num_users: int, num_layers=3, alpha=None):
    """`LightGCN.forward` (`lightgcn.py:136-164`)."""
    with torch.no_grad():
        x = weight
        embs = [x]
        for _ in range(num_layers):                                          # :151-153
            x = torch.sparse.mm(graph, x)
            embs.append(x)
        final = torch.zeros_like(embs[0])
        for a, e in zip(lightgcn_alphas(num_layers, alpha), embs):           # :156-158
            final += a * e
        return final[:num_users], final[num_users:]


def lightgcn_recommend(final_users: Tensor, final_items: Tensor, user_ids, k=12,
                       filter_items=None):
    """`LightGCN.predict_all_items` + `recommend` (`lightgcn.py:188-204`, `:332-358`)
    given the propagated tables (the reference re-propagates inside every call)."""
    with torch.no_grad():
        scores = torch.matmul(final_users[user_ids], final_items.t())       # :199-202
        return _topk(scores, k, user_ids, filter_items)


# --------------------------------------------------------------------------- MF
def mf_recommend(sd, user_ids, k=12, filter_items=None):
    """`MatrixFactorization.predict_all_items` + `recommend`
    (`matrix_factorization.py:108-131`, `:220-246`)."""
    with torch.no_grad():
        u = F.embedding(user_ids, sd["user_embeddings.weight"])
        ub = F.embedding(user_ids, sd["user_bias.weight"])
        s = torch.matmul(u, sd["item_embeddings.weight"].t())
        s = s + ub + sd["item_bias.weight"].t() + sd["global_bias"]
        return _topk(s, k, user_ids, filter_items)


# --------------------------------------------------------------------------- Wide&Deep
def widedeep_forward(sd, user_ids, item_ids, num_users, num_items, user_features=None):
    """`WideDeep.forward` (`wide_deep.py:157-230`) with its one-hot wide input
    (`:180-188`), use_wide_user_item / use_wide_features on, eval mode."""
    B = user_ids.shape[0]
    wide_user = torch.zeros(B, num_users)
    wide_user.scatter_(1, user_ids.unsqueeze(1), 1)
    wide_item = torch.zeros(B, num_items)
    wide_item.scatter_(1, item_ids.unsqueeze(1), 1)
    wide = [wide_user, wide_item]
    deep = [F.embedding(user_ids, sd["deep_user_embedding.weight"]),
            F.embedding(item_ids, sd["deep_item_embedding.weight"])]
    if user_features is not None and "wide_user_features.weight" in sd:
        wide.append(F.linear(user_features, sd["wide_user_features.weight"],
                             sd["wide_user_features.bias"]))
        deep.append(F.linear(user_features, sd["deep_user_features.weight"],
                             sd["deep_user_features.bias"]))
    x = torch.cat(deep, dim=1)
    lin = sorted({int(k.split(".")[1]) for k in sd
                  if k.startswith("deep_network.") and k.endswith(".weight")
                  and sd[k].dim() == 2})
    for li in lin:                                                           # :125-134
        x = F.relu(F.linear(x, sd[f"deep_network.{li}.weight"], sd[f"deep_network.{li}.bias"]))
        p = f"deep_network.{li + 2}."
        x = F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"],
                         sd[p + "bias"], training=False, eps=1e-5)
    combined = torch.cat([torch.cat(wide, dim=1), x], dim=1)                 # :225
    return F.linear(combined, sd["final_layer.weight"], sd["final_layer.bias"]).squeeze()


def widedeep_predict_all_items(sd, user_ids, user_features=None):
    """`WideDeep.predict_all_items` (`wide_deep.py:232-285`): 500-item chunks of expanded
    (user, item) pairs through `forward`."""
    num_users = sd["deep_user_embedding.weight"].shape[0]
    num_items = sd["deep_item_embedding.weight"].shape[0]
    B = user_ids.shape[0]
    out = []
    for s in range(0, num_items, 500):                                       # :250-251
        e = min(s + 500, num_items)
        items = torch.arange(s, e)
        eu = user_ids.unsqueeze(1).expand(B, e - s).contiguous().view(-1)    # :256-258
        ei = items.unsqueeze(0).expand(B, -1).contiguous().view(-1)          # :261-263
        ef = None
        if user_features is not None:
            ef = user_features.unsqueeze(1).expand(B, e - s, -1).contiguous().view(
                -1, user_features.shape[-1])
        out.append(widedeep_forward(sd, eu, ei, num_users, num_items, ef).view(B, -1))
    return torch.cat(out, dim=1)


def widedeep_recommend(sd, user_ids, k=12, filter_items=None, user_features=None):
    """`WideDeep.recommend` (`wide_deep.py:405-435`)."""
    with torch.no_grad():
        return _topk(widedeep_predict_all_items(sd, user_ids, user_features), k, user_ids,
                     filter_items)
