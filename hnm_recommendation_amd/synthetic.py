"""Synthetic H&M-shape inputs: weights, interaction graph, user batches.

There is no network and no Kaggle data, so every workload is generated here from
documented numpy PCG64 recipes:

* seed 0 -> weights, following the reference init distributions
  (xavier_uniform for embeddings / Linear: `lightgcn.py:71`, `neural_cf.py:98-110`,
  `wide_deep.py:138-155`; normal(0, 0.01) for the NCF GMF tables `neural_cf.py:95-96`
  and the MF tables `matrix_factorization.py:75-76`).
* seed 1 -> user-id batches (distinct ids, uniform over [0, U)).
* seed 2 -> the bipartite interaction graph: users uniform, items Zipf p ~ rank^-0.9,
  stored symmetric with the `+num_users` item offset of `tests/test_models.py:177-185`.

`bias_scale > 0` / `randomize_bn=True` replace the reference's zero biases and identity
BatchNorm statistics with random values so that parity tests exercise every term.
Arrays are returned as float32 / int64 numpy arrays keyed exactly like the reference
state_dicts.
"""
from __future__ import annotations

import numpy as np

# Kaggle H&M sizes (CLAUDE.md:12-14 of the reference, exact counts from SURVEY.md §8).
HM_USERS = 1_371_980
HM_ITEMS = 105_542
HM_INTERACTIONS = 31_788_324


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def xavier(rng, shape):
    """torch.nn.init.xavier_uniform_ on a 2-D tensor: U(-b, b), b = sqrt(6/(rows+cols))."""
    b = np.sqrt(6.0 / (shape[0] + shape[1]))
    return rng.uniform(-b, b, size=shape).astype(np.float32)


def normal(rng, shape, std):
    return (rng.standard_normal(size=shape) * std).astype(np.float32)


def _bias(rng, n, scale):
    if scale == 0.0:
        return np.zeros(n, np.float32)
    return rng.uniform(-scale, scale, size=n).astype(np.float32)


def ncf_state_dict(num_users, num_items, mf_dim=64, mlp_dims=(128, 64, 32), seed=0,
                   bias_scale=0.0, emb_scale=1.0):
    """NeuralCF weights (`neural_cf.py:56-67`, init `:92-110`)."""
    rng = _rng(seed)
    h = mlp_dims[0] // 2
    sd = {
        "gmf_user_embedding.weight": normal(rng, (num_users, mf_dim), 0.01 * emb_scale),
        "gmf_item_embedding.weight": normal(rng, (num_items, mf_dim), 0.01 * emb_scale),
        "mlp_user_embedding.weight": xavier(rng, (num_users, h)) * np.float32(emb_scale),
        "mlp_item_embedding.weight": xavier(rng, (num_items, h)) * np.float32(emb_scale),
    }
    for i in range(len(mlp_dims) - 1):
        sd[f"mlp_layers.{3 * i}.weight"] = xavier(rng, (mlp_dims[i + 1], mlp_dims[i]))
        sd[f"mlp_layers.{3 * i}.bias"] = _bias(rng, mlp_dims[i + 1], bias_scale)
    sd["prediction_layer.weight"] = xavier(rng, (1, mf_dim + mlp_dims[-1]))
    sd["prediction_layer.bias"] = _bias(rng, 1, bias_scale)
    return sd


def lightgcn_state_dict(num_users, num_items, embedding_dim=64, seed=0, emb_scale=1.0):
    """LightGCN joint (U+I) x d table (`lightgcn.py:70-71`)."""
    rng = _rng(seed)
    w = xavier(rng, (num_users + num_items, embedding_dim))
    if emb_scale != 1.0:
        w *= np.float32(emb_scale)
    return {"embeddings.weight": w}


def mf_state_dict(num_users, num_items, embedding_dim=64, seed=0, bias_scale=0.0):
    """MatrixFactorization (`matrix_factorization.py:48-78`)."""
    rng = _rng(seed)
    return {
        "user_embeddings.weight": normal(rng, (num_users, embedding_dim), 0.01),
        "item_embeddings.weight": normal(rng, (num_items, embedding_dim), 0.01),
        "user_bias.weight": _bias(rng, num_users, bias_scale).reshape(num_users, 1),
        "item_bias.weight": _bias(rng, num_items, bias_scale).reshape(num_items, 1),
        "global_bias": _bias(rng, 1, bias_scale),
    }


def widedeep_state_dict(num_users, num_items, embedding_dim=64, deep_layers=(512, 256, 128),
                        num_user_features=0, num_item_features=0, seed=0, bias_scale=0.0,
                        randomize_bn=False, emb_scale=1.0):
    """Wide&Deep weights (`wide_deep.py:92-155`), key order of the reference module."""
    rng = _rng(seed)
    d = embedding_dim
    sd = {
        "wide_user_embedding.weight": xavier(rng, (num_users, 1)),
        "wide_item_embedding.weight": xavier(rng, (num_items, 1)),
    }
    if num_user_features > 0:
        sd["wide_user_features.weight"] = xavier(rng, (num_user_features, num_user_features))
        sd["wide_user_features.bias"] = _bias(rng, num_user_features, bias_scale)
    if num_item_features > 0:
        sd["wide_item_features.weight"] = xavier(rng, (num_item_features, num_item_features))
        sd["wide_item_features.bias"] = _bias(rng, num_item_features, bias_scale)
    sd["deep_user_embedding.weight"] = xavier(rng, (num_users, d)) * np.float32(emb_scale)
    sd["deep_item_embedding.weight"] = xavier(rng, (num_items, d)) * np.float32(emb_scale)
    if num_user_features > 0:
        sd["deep_user_features.weight"] = xavier(rng, (d, num_user_features))
        sd["deep_user_features.bias"] = _bias(rng, d, bias_scale)
    if num_item_features > 0:
        sd["deep_item_features.weight"] = xavier(rng, (d, num_item_features))
        sd["deep_item_features.bias"] = _bias(rng, d, bias_scale)
    prev = 2 * d + (d if num_user_features > 0 else 0) + (d if num_item_features > 0 else 0)
    for li, hdim in enumerate(deep_layers):
        sd[f"deep_network.{4 * li}.weight"] = xavier(rng, (hdim, prev))
        sd[f"deep_network.{4 * li}.bias"] = _bias(rng, hdim, bias_scale)
        if randomize_bn:
            sd[f"deep_network.{4 * li + 2}.weight"] = rng.uniform(0.5, 1.5, hdim).astype(np.float32)
            sd[f"deep_network.{4 * li + 2}.bias"] = rng.uniform(-0.2, 0.2, hdim).astype(np.float32)
            sd[f"deep_network.{4 * li + 2}.running_mean"] = rng.uniform(-0.1, 0.1, hdim).astype(np.float32)
            sd[f"deep_network.{4 * li + 2}.running_var"] = rng.uniform(0.5, 2.0, hdim).astype(np.float32)
        else:
            sd[f"deep_network.{4 * li + 2}.weight"] = np.ones(hdim, np.float32)
            sd[f"deep_network.{4 * li + 2}.bias"] = np.zeros(hdim, np.float32)
            sd[f"deep_network.{4 * li + 2}.running_mean"] = np.zeros(hdim, np.float32)
            sd[f"deep_network.{4 * li + 2}.running_var"] = np.ones(hdim, np.float32)
        sd[f"deep_network.{4 * li + 2}.num_batches_tracked"] = np.zeros((), np.int64)
        prev = hdim
    wide_dim = num_users + num_items + num_user_features + num_item_features
    sd["final_layer.weight"] = xavier(rng, (1, wide_dim + deep_layers[-1]))
    sd["final_layer.bias"] = _bias(rng, 1, bias_scale)
    return sd


def _t3(rng, shape, spread):
    """Student-t(3) scaled to `spread` (t3's std is sqrt(3))."""
    return (rng.standard_t(3, size=shape) * (spread / np.sqrt(3.0))).astype(np.float32)


def _row_norms(rng, a, lo=50.0, hi=200.0):
    n = np.linalg.norm(a, axis=1, keepdims=True)
    n[n == 0] = 1.0
    return (a / n * rng.uniform(lo, hi, (a.shape[0], 1))).astype(np.float32)


def stress_state_dict(sd, kind, emb_keys, item_key, seed=0):
    """Weights unlike the init -- what trained models look like (the certified pre-filters'
    stress cases, tests/test_gpu_bound_stress.py, and bench.py --weights):

    norms      every embedding row of `emb_keys` rescaled to a norm uniform in [50, 200];
    student_t  every float weight (embeddings, Linear weights AND biases; BatchNorm statistics
               and affine kept) Student-t(nu = 3) at the original spread (heavy tailed);
    bn         (W&D) BatchNorm running_var down to 1e-4, |gamma| up to 10;
    big / huge one item row of `item_key` at 1e6 / 1e13.
    Returns a new dict (the input is not modified)."""
    rng = _rng(1000 + seed)
    sd = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in sd.items()}
    if kind == "norms":
        for k in emb_keys:
            sd[k] = _row_norms(rng, sd[k])
    elif kind == "student_t":
        for k, v in sd.items():
            if not isinstance(v, np.ndarray) or v.dtype != np.float32 or "running" in k:
                continue
            if k.startswith("deep_network") and v.ndim == 1 and int(k.split(".")[1]) % 4 == 2:
                continue  # BatchNorm affine: kept (the "bn" kind stresses it)
            spread = float(v.std()) if v.std() > 0 else 0.05
            sd[k] = _t3(rng, v.shape, spread)
    elif kind == "big":
        sd[item_key][77] = np.float32(1e6) * np.sign(sd[item_key][77] + 1e-30)
    elif kind == "huge":
        sd[item_key][77] = np.float32(1e13) * np.sign(sd[item_key][77] + 1e-30)
    elif kind == "bn":
        for k in list(sd):
            if k.endswith("running_var"):
                n = sd[k].size
                sd[k] = (10.0 ** rng.uniform(-4, 0, n)).astype(np.float32)
                g = k.replace("running_var", "weight")
                sd[g] = (rng.choice([-1.0, 1.0], n) * rng.uniform(0.1, 10.0, n)).astype(np.float32)
                sd[k.replace("running_var", "bias")] = rng.uniform(-1, 1, n).astype(np.float32)
                sd[k.replace("running_var", "running_mean")] = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    else:
        raise ValueError(kind)
    return sd


NCF_EMB_KEYS = ("gmf_user_embedding.weight", "gmf_item_embedding.weight",
                "mlp_user_embedding.weight", "mlp_item_embedding.weight")
MF_EMB_KEYS = ("user_embeddings.weight", "item_embeddings.weight")


def user_batch(num_users, batch, seed=1, distinct=True):
    """B user ids drawn uniformly from [0, U) (distinct when B <= U)."""
    rng = _rng(seed)
    if distinct and batch <= num_users:
        ids = rng.choice(num_users, size=batch, replace=False)
    else:
        ids = rng.integers(0, num_users, size=batch)
    return ids.astype(np.int64)


def interactions(num_users, num_items, num_edges, seed=2, zipf=0.9):
    """E (user, item) interactions: users uniform, items Zipf(rank^-zipf), duplicates kept."""
    rng = _rng(seed)
    users = rng.integers(0, num_users, size=num_edges, dtype=np.int64)
    p = np.arange(1, num_items + 1, dtype=np.float64) ** (-zipf)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    ranks = np.searchsorted(cdf, rng.random(num_edges), side="right")
    ranks = np.minimum(ranks, num_items - 1)
    # rank -> item id through a fixed random permutation so popular items are scattered
    perm = rng.permutation(num_items)
    items = perm[ranks].astype(np.int64)
    return users, items


def bipartite_edge_index(num_users, num_items, num_edges, seed=2, zipf=0.9):
    """Symmetric edge_index [2, 2E] with items offset by +U (`tests/test_models.py:177-185`)."""
    u, i = interactions(num_users, num_items, num_edges, seed=seed, zipf=zipf)
    i = i + num_users
    return np.stack([np.concatenate([u, i]), np.concatenate([i, u])])


def filter_dict(user_ids, num_items, per_user=23, seed=3):
    """A `filter_items` dict {user_id: set(items)} like the reference `recommend` takes."""
    rng = _rng(seed)
    out = {}
    for u in np.unique(np.asarray(user_ids)):
        n = int(rng.integers(0, 2 * per_user + 1))
        out[int(u)] = set(int(x) for x in rng.choice(num_items, size=min(n, num_items), replace=False))
    return out
