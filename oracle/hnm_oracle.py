"""CPU ORACLE for the top-N scoring hot path -- TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
this module, and only as the checker / the timed CPU baseline. The product path
(`hnm_recommendation_amd`) never calls it; it fails loudly without its HIP library.

This is a numpy (fp32) restatement, op for op, of the reference implementation of
hyunlord/hnm_recommendation @ 2025-07-25 (`src/models/*.py`).  Every function cites the
reference lines it follows.  Parity of this restatement is PINNED against the golden
fixtures in `tests/golden/*.npz`, which were produced by running the reference itself
(`tests/golden/make_golden.py`, torch CPU, with the SURVEY §8(c) stubs); see
`tests/test_oracle_golden.py`.

The third-party arithmetic boundary `torch_sparse` (not in the reference's
requirements.txt, no pinned version, absent here) is restated from its documented
semantics: `torch_sparse.sum(value, row, dim=0, dim_size=N)` as the scatter-add degree
`lightgcn.py:103` intends, and `SparseTensor @ X` as a duplicate-summing SpMM.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------- top-K
def topk(scores: np.ndarray, k: int):
    """`torch.topk(scores, k, dim=1)` (`neural_cf.py:324`, `lightgcn.py:356`,
    `wide_deep.py:433`, `serve.py:355`).  torch leaves the tie order unspecified; the
    oracle fixes it to (score desc, index asc), the order the HIP path guarantees."""
    scores = np.asarray(scores)
    n = scores.shape[1]
    idx = np.argsort(-scores, axis=1, kind="stable")[:, :k]
    # argsort of -x is ascending on -x with stable index order -> score desc, idx asc
    vals = np.take_along_axis(scores, idx, axis=1)
    assert idx.shape[1] == min(k, n)
    return vals, idx.astype(np.int64)


def apply_filter(scores: np.ndarray, user_ids, filter_items):
    """The `-inf` mask loop of every `recommend` (`neural_cf.py:316-321`,
    `lightgcn.py:349-353`, `wide_deep.py:425-430`) and of `serve.py:350-352`."""
    if filter_items is None:
        return scores
    scores = scores.copy()
    for i, u in enumerate(np.asarray(user_ids).tolist()):
        if u in filter_items:
            items = list(filter_items[u])
            if items:
                scores[i, items] = -np.inf
    return scores


def recommend(scores, user_ids, k, filter_items=None):
    """`*.recommend` = predict_all_items -> filter -> topk (`neural_cf.py:300-326`)."""
    return topk(apply_filter(scores, user_ids, filter_items), k)[1]


# --------------------------------------------------------------------------- layers
def linear(x, w, b):
    """nn.Linear: x @ W^T + b (fp32)."""
    y = x @ w.T.astype(F32)
    if b is not None:
        y = y + b
    return y.astype(F32)


def relu(x):
    return np.maximum(x, F32(0))


# --------------------------------------------------------------------------- NeuralCF
def ncf_mlp_layer_keys(sd):
    keys = sorted({int(k.split(".")[1]) for k in sd if k.startswith("mlp_layers.")})
    return keys


def ncf_forward(sd, user_ids, item_ids):
    """`NeuralCF.forward` (`neural_cf.py:112-141`): GMF u*i, MLP on cat(u,i), Linear."""
    gu = sd["gmf_user_embedding.weight"][user_ids]
    gi = sd["gmf_item_embedding.weight"][item_ids]
    gmf = gu * gi
    x = np.concatenate([sd["mlp_user_embedding.weight"][user_ids],
                        sd["mlp_item_embedding.weight"][item_ids]], axis=1)
    for li in ncf_mlp_layer_keys(sd):
        x = relu(linear(x, sd[f"mlp_layers.{li}.weight"], sd[f"mlp_layers.{li}.bias"]))
    cat = np.concatenate([gmf, x], axis=1)
    return linear(cat, sd["prediction_layer.weight"], sd["prediction_layer.bias"])[:, 0]


def ncf_predict_all_items(sd, user_ids, item_batch_size=1000):
    """`NeuralCF.predict_all_items` (`neural_cf.py:143-208`), including the 1000-item
    chunking (`:167-203`): expand user/item rows, GMF mul (`:189`), cat + MLP
    (`:192-196`), cat + prediction layer (`:199-201`), cat chunks (`:206`)."""
    user_ids = np.asarray(user_ids)
    B = user_ids.shape[0]
    gmf_user = sd["gmf_user_embedding.weight"][user_ids]
    mlp_user = sd["mlp_user_embedding.weight"][user_ids]
    gmf_items = sd["gmf_item_embedding.weight"]
    mlp_items = sd["mlp_item_embedding.weight"]
    I = gmf_items.shape[0]
    layers = [(sd[f"mlp_layers.{li}.weight"], sd[f"mlp_layers.{li}.bias"])
              for li in ncf_mlp_layer_keys(sd)]
    wp, bp = sd["prediction_layer.weight"], sd["prediction_layer.bias"]
    out = []
    for s in range(0, I, item_batch_size):
        e = min(s + item_batch_size, I)
        n = e - s
        gmf = gmf_user[:, None, :] * gmf_items[None, s:e, :]                     # [B,n,mf]
        x = np.concatenate([np.broadcast_to(mlp_user[:, None, :], (B, n, mlp_user.shape[1])),
                            np.broadcast_to(mlp_items[None, s:e, :], (B, n, mlp_items.shape[1]))],
                           axis=2).reshape(B * n, -1)
        for w, b in layers:
            x = relu(linear(x, w, b))
        cat = np.concatenate([gmf.reshape(B * n, -1), x], axis=1)
        out.append(linear(cat, wp, bp).reshape(B, n))
    return np.concatenate(out, axis=1)


# --------------------------------------------------------------------------- LightGCN
def lightgcn_alphas(num_layers, alpha=None):
    """Layer-combination weights (`lightgcn.py:59-67`)."""
    if alpha is None:
        return [1.0 / (num_layers + 1)] * (num_layers + 1)
    a = [alpha ** i for i in range(num_layers + 1)]
    s = sum(a)
    return [x / s for x in a]


def lightgcn_set_graph(edge_index, edge_weight, num_nodes):
    """`LightGCN.set_graph` + `_add_self_loops` (`lightgcn.py:81-134`):
    append (n, n, 1) for every node, deg = scatter-add of weights over row,
    deg^-1/2 with inf -> 0, value = dinv[row] * w * dinv[col].  Returns COO (row, col, val)
    in the reference's edge order (duplicates kept, summed by the SpMM)."""
    edge_index = np.asarray(edge_index, np.int64)
    E = edge_index.shape[1]
    w = np.ones(E, F32) if edge_weight is None else np.asarray(edge_weight, F32)
    loop = np.arange(num_nodes, dtype=np.int64)
    row = np.concatenate([edge_index[0], loop])
    col = np.concatenate([edge_index[1], loop])
    w = np.concatenate([w, np.ones(num_nodes, F32)])
    deg = np.zeros(num_nodes, F32)
    np.add.at(deg, row, w)
    with np.errstate(divide="ignore"):
        dinv = deg ** F32(-0.5)
    dinv[np.isinf(dinv)] = 0
    val = (dinv[row] * w * dinv[col]).astype(F32)
    return row, col, val


def spmm(row, col, val, x, num_nodes):
    """`SparseTensor @ X` (`lightgcn.py:152`): Y[r] += val * X[c] over all entries."""
    y = np.zeros((num_nodes, x.shape[1]), F32)
    np.add.at(y, row, x[col] * val[:, None])
    return y


def lightgcn_forward(emb, graph, num_users, num_layers=3, alpha=None):
    """`LightGCN.forward` (`lightgcn.py:136-164`): E_{l+1} = A E_l, F = sum_l a_l E_l,
    split into users [:U] and items [U:]."""
    row, col, val = graph
    N = emb.shape[0]
    alphas = lightgcn_alphas(num_layers, alpha)
    e = np.asarray(emb, F32)
    embs = [e]
    for _ in range(num_layers):
        e = spmm(row, col, val, e, N)
        embs.append(e)
    final = np.zeros_like(embs[0])
    for a, x in zip(alphas, embs):
        final += F32(a) * x
    return final[:num_users], final[num_users:]


def lightgcn_predict_all_items(final_users, final_items, user_ids):
    """`LightGCN.predict_all_items` (`lightgcn.py:188-204`): F_U[ids] @ F_I^T."""
    return (final_users[np.asarray(user_ids)] @ final_items.T).astype(F32)


# --------------------------------------------------------------------------- MF
def mf_predict_all_items(sd, user_ids):
    """`MatrixFactorization.predict_all_items` (`matrix_factorization.py:108-131`)."""
    u = sd["user_embeddings.weight"][user_ids]
    s = u @ sd["item_embeddings.weight"].T
    s = s + sd["user_bias.weight"][user_ids] + sd["item_bias.weight"].T + sd["global_bias"]
    return s.astype(F32)


# --------------------------------------------------------------------------- Wide&Deep
def widedeep_layers(sd):
    lin = sorted({int(k.split(".")[1]) for k in sd
                  if k.startswith("deep_network.") and k.endswith(".weight")
                  and sd[k].ndim == 2})
    return lin


def batchnorm_eval(x, sd, prefix, eps=1e-5):
    """nn.BatchNorm1d in eval mode (`wide_deep.py:130`): running statistics."""
    m = sd[prefix + "running_mean"]
    v = sd[prefix + "running_var"]
    g = sd[prefix + "weight"]
    b = sd[prefix + "bias"]
    return ((x - m) / np.sqrt(v + F32(eps)) * g + b).astype(F32)


def widedeep_forward(sd, user_ids, item_ids, user_features=None, num_users=None,
                     num_items=None, item_features=None):
    """`WideDeep.forward` (`wide_deep.py:157-230`), use_wide_features on.  The one-hot wide
    input (`:180-188`, present when use_wide_user_item: the state dict then holds
    `wide_user_embedding`) times `final_layer.weight` is restated as the two weights it
    selects: w[u] + w[U + i]; the feature crosses follow in the concat order (`:190-195`);
    the deep tower is Linear -> ReLU -> BatchNorm(eval) -> Dropout(identity) per layer
    (`:125-134`) over [e_u; e_i; user-feature proj; item-feature proj] (`:207-219`)."""
    user_ids = np.asarray(user_ids)
    item_ids = np.asarray(item_ids)
    U = num_users if num_users is not None else sd["deep_user_embedding.weight"].shape[0]
    I = num_items if num_items is not None else sd["deep_item_embedding.weight"].shape[0]
    wf = sd["final_layer.weight"][0]
    deep_in = [sd["deep_user_embedding.weight"][user_ids], sd["deep_item_embedding.weight"][item_ids]]
    wide_terms = np.zeros(len(user_ids), F32)
    off = 0
    if "wide_user_embedding.weight" in sd:  # use_wide_user_item
        wide_terms = wf[user_ids] + wf[U + item_ids]
        off = U + I
    has_uf = "wide_user_features.weight" in sd
    nuf = sd["wide_user_features.weight"].shape[0] if has_uf else 0
    if has_uf and user_features is not None:
        wuf = linear(user_features, sd["wide_user_features.weight"], sd["wide_user_features.bias"])
        wide_terms = wide_terms + wuf @ wf[off:off + nuf]
    off += nuf
    has_if = "wide_item_features.weight" in sd
    nif = sd["wide_item_features.weight"].shape[0] if has_if else 0
    if has_if and item_features is not None:
        wif = linear(item_features, sd["wide_item_features.weight"], sd["wide_item_features.bias"])
        wide_terms = wide_terms + wif @ wf[off:off + nif]
    off += nif
    if "deep_user_features.weight" in sd and user_features is not None:
        deep_in.append(linear(user_features, sd["deep_user_features.weight"],
                              sd["deep_user_features.bias"]))
    if "deep_item_features.weight" in sd and item_features is not None:
        deep_in.append(linear(item_features, sd["deep_item_features.weight"],
                              sd["deep_item_features.bias"]))
    x = np.concatenate(deep_in, axis=1)
    for li in widedeep_layers(sd):
        x = relu(linear(x, sd[f"deep_network.{li}.weight"], sd[f"deep_network.{li}.bias"]))
        x = batchnorm_eval(x, sd, f"deep_network.{li + 2}.")
    deep = x @ wf[off:]
    return (wide_terms + deep + sd["final_layer.bias"][0]).astype(F32)


def widedeep_predict_all_items(sd, user_ids, user_features=None, item_batch_size=500):
    """`WideDeep.predict_all_items` (`wide_deep.py:232-285`): 500-item chunks, each
    expanding (user, item) pairs and calling forward (`:254-276`)."""
    user_ids = np.asarray(user_ids)
    B = user_ids.shape[0]
    I = sd["deep_item_embedding.weight"].shape[0]
    out = []
    for s in range(0, I, item_batch_size):
        e = min(s + item_batch_size, I)
        items = np.arange(s, e)
        eu = np.repeat(user_ids, e - s)
        ei = np.tile(items, B)
        ef = None if user_features is None else np.repeat(user_features, e - s, axis=0)
        out.append(widedeep_forward(sd, eu, ei, ef).reshape(B, e - s))
    return np.concatenate(out, axis=1)


# --------------------------------------------------------------------------- metrics
def inv_log2_table(k):
    """[1.0 / np.log2(i + 2) for i < k] -- the per-position NDCG discount exactly as the
    reference forms each term (`metrics.py:180`, `:243`), one scalar np.log2 at a time."""
    return np.asarray([1.0 / np.log2(i + 2) for i in range(k)], np.float64)


def user_metrics(pred_items, true_items, k):
    """One user's (AP@k, Recall@k, Precision@k, NDCG@k) with the float64 arithmetic and
    loop order of `evaluate_recommendations` (`metrics.py:218-247`).  `true_items` is
    the already de-duplicated truth collection (a set there, `:212`); `pred_items` the
    first k predictions (`:223`).  Zero denominators -> 0.0 (the reference's guards;
    its AP division by min(0, k) would raise -- callers check that case)."""
    pred = list(pred_items)[:k]
    ap, nh = 0.0, 0.0
    for i, it in enumerate(pred):
        if it in true_items:
            nh += 1.0
            ap += nh / (i + 1.0)
    lim = min(len(true_items), k)
    hits = sum(1 for it in pred if it in true_items)
    dcg = 0.0
    for i, it in enumerate(pred):
        if it in true_items:
            dcg += 1.0 / np.log2(i + 2)
    idcg = sum(1.0 / np.log2(i + 2) for i in range(lim))
    return (ap / lim if lim else 0.0,
            hits / len(true_items) if len(true_items) else 0.0,
            hits / len(pred) if pred else 0.0,
            dcg / idcg if idcg > 0 else 0.0)


def evaluate_recommendations(predictions, ground_truth, k=12):
    """`evaluate_recommendations` (`metrics.py:193-255`): mean over the ground-truth users;
    users without predictions contribute zeros (`:214-220`)."""
    rows = []
    for u in ground_truth:
        t = set(ground_truth[u])
        if u not in predictions:
            rows.append((0.0, 0.0, 0.0, 0.0))
            continue
        if not t:
            raise ZeroDivisionError("float division by zero")  # `:229` with an empty set
        rows.append(user_metrics(predictions[u], t, k))
    a = np.asarray(rows, np.float64).reshape(-1, 4)
    return {f"map@{k}": np.mean(a[:, 0]), f"recall@{k}": np.mean(a[:, 1]),
            f"precision@{k}": np.mean(a[:, 2]), f"ndcg@{k}": np.mean(a[:, 3])}, a


def metric_classes(scores, target, mask, k=12):
    """The torchmetrics classes MeanAveragePrecision / RecallAtK / PrecisionAtK / NDCGAtK
    (`metrics.py:10-190`) over one `update(preds, target, mask)`: 2-D preds are scores, so
    each row's top-min(k, n_items) is taken first (`:33-35`; tie order (score desc, index
    asc) here); truth = `target[i][mask[i]]` with duplicates counted in len() (tensor
    semantics, `:41-44`).  MAP and Precision average over every row, Recall and NDCG over
    rows with non-empty truth (`:97`, `:170`).  Returns (dict of means, per-row [B, 4])."""
    scores = np.asarray(scores)
    kk = min(k, scores.shape[1])
    _, top = topk(scores, kk)
    B = scores.shape[0]
    per = np.zeros((B, 4))
    has = np.zeros(B, bool)
    for b in range(B):
        t = np.asarray(target[b])
        if mask is not None:
            t = t[np.asarray(mask[b], bool)]
        tset = set(t.tolist())
        n = len(t)
        has[b] = n > 0
        pred = top[b].tolist()
        hits = [p in tset for p in pred]
        ap, nh, dcg = 0.0, 0.0, 0.0
        for i, h in enumerate(hits):
            if h:
                nh += 1.0
                ap += nh / (i + 1.0)
                dcg += 1.0 / np.log2(i + 2)
        idcg = sum(1.0 / np.log2(i + 2) for i in range(min(n, k)))
        per[b] = (ap / min(n, k) if n else 0.0, nh / n if n else 0.0,
                  nh / len(pred) if pred else 0.0, dcg / idcg if idcg > 0 else 0.0)
    mean = lambda col, sel: float(per[sel, col].mean()) if sel.any() else 0.0  # noqa: E731
    allr = np.ones(B, bool)
    return {"map": mean(0, allr), "recall": mean(1, has), "precision": mean(2, allr),
            "ndcg": mean(3, has)}, per
