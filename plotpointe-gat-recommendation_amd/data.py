"""Host-side data plumbing that feeds the GAT hot path.

Mirrors the reference trainer's data utilities (same names, argument meaning and
outputs) so a caller of ``scripts/train_gat_pyg.py`` / ``scripts/train_gat_custom.py``
finds them here:

* ``build_splits``      -- scripts/train_gat_pyg.py:114-128 (identical custom :148-162)
* ``to_indexed``        -- scripts/train_gat_pyg.py:131-136
* ``index_maps``        -- scripts/train_gat_custom.py:178-181
* ``build_edge_index``  -- scripts/train_gat_pyg.py:139-147 (custom :166-175)
* ``sample_bpr_epoch``  -- scripts/train_gat_pyg.py:179-190
* ``node_maps_from_interactions`` -- graphs/build_ui_edges.py:50-57,97-104

The reference builds ``edge_index`` with a Python double loop.  Here it is the
same column order produced by vectorised numpy (the order matters: it fixes the
CSR in-segment order and therefore the fp32 summation order on the device).

Synthetic stand-ins for the absent Amazon-Electronics artefacts
(``.MISSING_LARGE_BLOBS``) follow SURVEY.md section 8(d) configs 1/2/3/5.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np

try:  # pandas is only needed for the DataFrame-shaped mirror functions
    import pandas as pd
except Exception:  # pragma: no cover
    pd = None


# ----------------------------------------------------------------------------
# Mirrors of the reference data utilities
# ----------------------------------------------------------------------------

def build_splits(interactions):
    """Per-user chronological leave-2-out split (scripts/train_gat_pyg.py:114-128).

    Users are visited in ``groupby("user_id")`` order (sorted raw ids); within a
    user the items are in timestamp order.  >=3 items: train=items[:-2],
    val=items[-2], test=items[-1]; 2 items: train=items[:-1], test=items[-1];
    1 item: dropped.  Vectorised: one stable sort instead of a per-group loop.
    Timestamps equal *within* one user are ordered by row position here; the
    reference's default (non-stable) quicksort leaves that order unspecified.
    """
    df = interactions[["user_id", "asin", "ts"]]
    order = np.lexsort((np.arange(len(df)), df["ts"].to_numpy(), ))
    df = df.iloc[order]
    # groupby(sort=True) order of users, ts order inside each user (stable)
    df = df.iloc[np.argsort(df["user_id"].to_numpy(), kind="stable")]
    users = df["user_id"].to_numpy()
    items = df["asin"].to_numpy()
    if len(users) == 0:
        return {}, {}, {}
    starts = np.flatnonzero(np.r_[True, users[1:] != users[:-1]])
    ends = np.r_[starts[1:], len(users)]
    train_pos, val_pos, test_pos = {}, {}, {}
    for s, e in zip(starts.tolist(), ends.tolist()):
        u = users[s]
        n = e - s
        if n >= 3:
            train_pos[u] = items[s:e - 2]
            val_pos[u] = items[e - 2]
            test_pos[u] = items[e - 1]
        elif n >= 2:
            train_pos[u] = items[s:e - 1]
            test_pos[u] = items[e - 1]
    return train_pos, val_pos, test_pos


def to_indexed(interactions, user_to_idx: Dict[str, int], item_to_idx: Dict[str, int]):
    """scripts/train_gat_pyg.py:131-136."""
    df = interactions[["user_id", "asin", "ts"]].copy()
    df["u"] = df["user_id"].map(user_to_idx)
    df["i"] = df["asin"].map(item_to_idx)
    df = df.dropna(subset=["u", "i"]).astype({"u": int, "i": int})
    return df


def index_maps(maps: dict):
    """scripts/train_gat_custom.py:178-181."""
    u2i = {k: int(v) for k, v in maps["user_to_idx"].items()}
    i2i = {k: int(v) for k, v in maps["item_to_idx"].items()}
    return u2i, i2i


def node_maps_from_interactions(interactions) -> dict:
    """First-appearance node ids, the ``node_maps.json`` schema of graphs/build_ui_edges.py:50-57,97-104."""
    unique_users = interactions["user_id"].unique()
    unique_items = interactions["asin"].unique()
    user_to_idx = {str(uid): idx for idx, uid in enumerate(unique_users)}
    item_to_idx = {str(iid): idx for idx, iid in enumerate(unique_items)}
    return {
        "user_to_idx": user_to_idx,
        "item_to_idx": item_to_idx,
        "idx_to_user": {idx: uid for uid, idx in user_to_idx.items()},
        "idx_to_item": {idx: iid for iid, idx in item_to_idx.items()},
        "n_users": len(user_to_idx),
        "n_items": len(item_to_idx),
    }


def build_ui_edges(interactions):
    """graphs/build_ui_edges.py:50-85 without the GCS I/O: first-appearance node ids
    (``node_maps_from_interactions``) and the user x item COO matrix of rating weights
    (r - 1) / 4 (1.0 where there is no rating column), float32, one entry per interaction in
    row order.  Returns (scipy.sparse.coo_matrix, node_maps)."""
    from scipy.sparse import coo_matrix
    maps = node_maps_from_interactions(interactions)
    u2i = {k: v for k, v in maps["user_to_idx"].items()}
    i2i = {k: v for k, v in maps["item_to_idx"].items()}
    users = interactions["user_id"].astype(str).map(u2i).to_numpy()
    items = interactions["asin"].astype(str).map(i2i).to_numpy()
    if "rating" in interactions.columns:
        values = (interactions["rating"].to_numpy() - 1.0) / 4.0
    else:
        values = np.ones(len(interactions), dtype=np.float32)
    ui = coo_matrix((values.astype(np.float32), (users, items)), shape=(maps["n_users"], maps["n_items"]),
                    dtype=np.float32)
    return ui, maps


def save_ui_edges(path, ui) -> None:
    """Write ``ui_edges.npz`` exactly as graphs/build_ui_edges.py:84-85 (scipy.sparse.save_npz
    of the COO matrix)."""
    from scipy.sparse import save_npz
    save_npz(str(path), ui)


def load_ui_edges(path):
    """Read a ``ui_edges.npz`` (scipy.sparse npz, no pickles): -> (users int64, items int64,
    weights float32, (n_users, n_items)) in stored entry order."""
    from scipy.sparse import load_npz
    m = load_npz(str(path)).tocoo()
    return (m.row.astype(np.int64), m.col.astype(np.int64), m.data.astype(np.float32), tuple(int(v) for v in m.shape))


def edge_index_from_ui_edges(users: np.ndarray, items: np.ndarray, n_users: int) -> np.ndarray:
    """The homogeneous message edge_index of a U-I COO (u -> n_users + i, n_users + i -> u per
    entry, the column order of train_gat_pyg.py:141-146 for entries in user order)."""
    return edge_index_numpy(n_users, users, items)


def map_splits_to_index(train_pos_raw, val_pos_raw, test_pos_raw, user_to_idx, item_to_idx):
    """Raw-id -> index mapping exactly as scripts/train_gat_pyg.py:272-288."""
    train_pos_idx: Dict[int, np.ndarray] = {}
    val_pos_idx: Dict[int, int] = {}
    test_pos_idx: Dict[int, int] = {}
    for u_raw, items in train_pos_raw.items():
        u = user_to_idx.get(str(u_raw), user_to_idx.get(u_raw, None))
        if u is None:
            continue
        idx_items = []
        for it in items:
            it_idx = item_to_idx.get(str(it), item_to_idx.get(it, None))
            if it_idx is not None:
                idx_items.append(it_idx)
        if idx_items:
            train_pos_idx[int(u)] = np.array(idx_items, dtype=np.int64)
    for d_raw, d_idx in ((val_pos_raw, val_pos_idx), (test_pos_raw, test_pos_idx)):
        for u_raw, it in d_raw.items():
            u = user_to_idx.get(str(u_raw), user_to_idx.get(u_raw, None))
            it_idx = item_to_idx.get(str(it), item_to_idx.get(it, None))
            if u is not None and it_idx is not None:
                d_idx[int(u)] = int(it_idx)
    return train_pos_idx, val_pos_idx, test_pos_idx


def edge_index_numpy(n_users: int, user_of: np.ndarray, item_of: np.ndarray) -> np.ndarray:
    """Interleaved U-I message columns for already-ordered (user, item) pairs.

    Column 2t = (u -> n_users+i), column 2t+1 = (n_users+i -> u), the order of
    scripts/train_gat_pyg.py:141-146.  Returns int64 [2, 2T].
    """
    u = np.asarray(user_of, dtype=np.int64)
    it = np.asarray(item_of, dtype=np.int64) + int(n_users)
    ei = np.empty((2, 2 * len(u)), dtype=np.int64)
    ei[0, 0::2] = u
    ei[1, 0::2] = it
    ei[0, 1::2] = it
    ei[1, 1::2] = u
    return ei


def build_edge_index(n_users: int, n_items: int, train_pos_idx: Dict[int, np.ndarray]):
    """scripts/train_gat_pyg.py:139-147 -> ``torch.LongTensor[2, E]`` in reference column order."""
    import torch
    if train_pos_idx:
        keys = list(train_pos_idx.keys())
        lens = np.fromiter((len(train_pos_idx[k]) for k in keys), dtype=np.int64, count=len(keys))
        users = np.repeat(np.asarray(keys, dtype=np.int64), lens)
        items = np.concatenate([np.asarray(train_pos_idx[k], dtype=np.int64) for k in keys])
    else:
        users = np.zeros(0, np.int64)
        items = np.zeros(0, np.int64)
    return torch.from_numpy(edge_index_numpy(n_users, users, items))


def sample_bpr_epoch(train_pos_idx: Dict[int, np.ndarray], n_items: int, samples: int):
    """scripts/train_gat_pyg.py:179-190 -- same Python ``random`` draw sequence,
    so a seeded run yields the reference's exact triples."""
    users = list(train_pos_idx.keys())
    pos_sets = {u: set(int(x) for x in v) for u, v in train_pos_idx.items()}
    out_u, out_i, out_j = [], [], []
    while len(out_u) < samples:
        u = random.choice(users)
        i = int(random.choice(train_pos_idx[u]))
        s = pos_sets[u]
        while True:
            j = random.randrange(n_items)
            if j not in s:
                break
        out_u.append(u); out_i.append(i); out_j.append(j)
    return np.array(out_u), np.array(out_i), np.array(out_j)


def sample_bpr_numpy(user_ptr: np.ndarray, user_items: np.ndarray, n_items: int, samples: int,
                     seed: int = 42):
    """Vectorised uniform BPR sampler over a CSR user->train-items table (same
    distribution as ``sample_bpr_epoch``, different stream). Used by the bench to
    keep sampling out of the timed region; parity runs use ``sample_bpr_epoch``."""
    rng = np.random.default_rng(seed)
    n_users = len(user_ptr) - 1
    deg = np.diff(user_ptr)
    users = np.flatnonzero(deg > 0)
    u = users[rng.integers(0, len(users), samples)]
    i = user_items[user_ptr[u] + (rng.random(samples) * deg[u]).astype(np.int64)]
    j = rng.integers(0, n_items, samples)
    # reject negatives that are positives (vectorised rounds, tiny residue)
    for _ in range(32):
        lo, hi = user_ptr[u], user_ptr[u + 1]
        bad = np.zeros(samples, dtype=bool)
        # per-row membership: rows are short (mean ~7), loop over max degree
        maxd = int(deg[u].max()) if samples else 0
        for d in range(maxd):
            idx = lo + d
            ok = idx < hi
            bad |= ok & (user_items[np.minimum(idx, len(user_items) - 1)] == j)
        if not bad.any():
            break
        j[bad] = rng.integers(0, n_items, int(bad.sum()))
    return u.astype(np.int64), i.astype(np.int64), j.astype(np.int64)


# ----------------------------------------------------------------------------
# Synthetic stand-ins
# ----------------------------------------------------------------------------

def synthetic_interactions_small(n_users: int = 1500, n_item_pool: int = 1200, seed: int = 0):
    """Config 1 "10k-edge" plumbing set: user degree 5+Geom(0.5)-1 capped at 40,
    item popularity ~ rank^-0.8, globally distinct timestamps, rows shuffled so
    first-appearance ids differ from sorted raw ids. Returns a DataFrame with the
    reference's ``interactions.parquet`` columns (user_id, asin, ts, rating)."""
    rng = np.random.default_rng(seed)
    deg = np.minimum(5 + rng.geometric(0.5, n_users) - 1, 40)
    pop = np.arange(1, n_item_pool + 1, dtype=np.float64) ** -0.8
    pop /= pop.sum()
    us, its = [], []
    for u in range(n_users):
        items = rng.choice(n_item_pool, size=int(deg[u]), replace=False, p=pop)
        us.append(np.full(len(items), u))
        its.append(items)
    us = np.concatenate(us)
    its = np.concatenate(its)
    ts = 1_000_000_000 + rng.permutation(len(us)).astype(np.int64) * 60
    perm = rng.permutation(len(us))
    us, its, ts = us[perm], its[perm], ts[perm]
    rating = rng.integers(1, 6, len(us)).astype(np.float32)
    return pd.DataFrame({
        "user_id": np.char.add("U", np.char.zfill(us.astype(str), 6)),
        "asin": np.char.add("B", np.char.zfill(its.astype(str), 9)),
        "ts": ts,
        "rating": rating,
    })


@dataclass
class UIGraph:
    """Integer-indexed U-I training graph in the reference's layout."""
    n_users: int
    n_items: int
    user_ptr: np.ndarray      # [n_users+1] CSR of train items per user (ts order)
    user_items: np.ndarray    # [T] item index
    val_item: np.ndarray      # [n_users] (-1 if none)
    test_item: np.ndarray     # [n_users]
    n_interactions: int

    @property
    def n_nodes(self) -> int:
        return self.n_users + self.n_items

    def edge_index_numpy(self) -> np.ndarray:
        users = np.repeat(np.arange(self.n_users, dtype=np.int64), np.diff(self.user_ptr))
        return edge_index_numpy(self.n_users, users, self.user_items)

    def train_pos_idx(self) -> Dict[int, np.ndarray]:
        return {u: self.user_items[self.user_ptr[u]:self.user_ptr[u + 1]]
                for u in range(self.n_users) if self.user_ptr[u + 1] > self.user_ptr[u]}


def _fix_sum(deg: np.ndarray, total: int, lo: int, rng) -> np.ndarray:
    deg = deg.astype(np.int64)
    diff = total - int(deg.sum())
    while diff != 0:
        idx = rng.integers(0, len(deg), abs(diff))
        if diff > 0:
            np.add.at(deg, idx, 1)
        else:
            np.add.at(deg, idx, -1)
            deg = np.maximum(deg, lo)
        diff = total - int(deg.sum())
    return deg


def synthetic_ui_graph(n_users: int = 192_403, n_items: int = 63_001,
                       n_interactions: int = 1_689_116, seed: int = 42,
                       user_min: int = 5, item_min: int = 5,
                       user_extra_mean: Optional[float] = None,
                       item_sigma: float = 1.64) -> UIGraph:
    """Config 2 statistics-matched stand-in for the Amazon-Electronics 5-core U-I
    graph: user degree >=5 (mean 8.78, over-dispersed negative
    binomial), item degree >=5 (mean 26.8, log-normal heavy tail, std ~81),
    no duplicate (user,item) pairs, globally distinct timestamps, per-user
    leave-2-out exactly as ``build_splits``."""
    rng = np.random.default_rng(seed)
    if user_extra_mean is None:
        user_extra_mean = n_interactions / n_users - user_min
    # users: 5 + NB(r=0.2, mean=extra)  -> std ~ 8.7 at cfg2
    r = 0.2
    p = r / (r + max(user_extra_mean, 1e-6))
    udeg = user_min + rng.negative_binomial(r, p, n_users)
    udeg = np.minimum(udeg, max(user_min, n_items // 2))
    udeg = _fix_sum(udeg, n_interactions, user_min, rng)
    # items: 5 + lognormal
    item_extra_mean = n_interactions / n_items - item_min
    mu = np.log(max(item_extra_mean, 1e-6)) - item_sigma ** 2 / 2
    ideg = item_min + np.floor(rng.lognormal(mu, item_sigma, n_items)).astype(np.int64)
    ideg = np.minimum(ideg, n_users // 2)
    ideg = _fix_sum(ideg, n_interactions, item_min, rng)
    # configuration model pairing, then break duplicate (user,item) pairs by swaps
    u_slots = np.repeat(np.arange(n_users, dtype=np.int64), udeg)
    i_slots = rng.permutation(np.repeat(np.arange(n_items, dtype=np.int64), ideg))
    for _ in range(200):
        key = u_slots * n_items + i_slots
        order = np.argsort(key, kind="stable")
        sk = key[order]
        dup = order[1:][sk[1:] == sk[:-1]]
        if len(dup) == 0:
            break
        other = rng.integers(0, len(i_slots), len(dup))
        tmp = i_slots[dup].copy()
        i_slots[dup] = i_slots[other]
        i_slots[other] = tmp
    else:  # pragma: no cover - drop the residue
        key = u_slots * n_items + i_slots
        _, first = np.unique(key, return_index=True)
        keep = np.zeros(len(key), bool); keep[first] = True
        u_slots, i_slots = u_slots[keep], i_slots[keep]
    n_int = len(u_slots)
    ts = rng.permutation(n_int).astype(np.int64)
    # per-user ts order
    order = np.lexsort((ts, u_slots))
    u_sorted = u_slots[order]
    i_sorted = i_slots[order]
    counts = np.bincount(u_sorted, minlength=n_users)
    ptr = np.zeros(n_users + 1, np.int64)
    np.cumsum(counts, out=ptr[1:])
    val_item = np.full(n_users, -1, np.int64)
    test_item = np.full(n_users, -1, np.int64)
    keep = np.ones(n_int, bool)
    has3 = counts >= 3
    has2 = counts == 2
    last = ptr[1:] - 1
    test_item[counts >= 2] = i_sorted[last[counts >= 2]]
    val_item[has3] = i_sorted[last[has3] - 1]
    keep[last[counts >= 2]] = False
    keep[last[has3] - 1] = False
    drop1 = counts == 1
    keep[last[drop1]] = False
    u_tr = u_sorted[keep]
    i_tr = i_sorted[keep]
    tcounts = np.bincount(u_tr, minlength=n_users)
    tptr = np.zeros(n_users + 1, np.int64)
    np.cumsum(tcounts, out=tptr[1:])
    return UIGraph(n_users, n_items, tptr, i_tr, val_item, test_item, n_int)


def synthetic_scaling_graph(scale: float = 1.0, seed: int = 42, n_users: int = 10_000_000,
                            n_items: int = 5_000_000, n_interactions: int = 100_000_000,
                            zipf_a: float = 0.8) -> UIGraph:
    """Config 5 of SURVEY.md 8(d) (the roofline / scaling run): 10M users x 5M items x 100M
    interactions, symmetrised to E = 200M message edges, every size multiplied by
    ``scale`` (scale 1/8 = one GPU's share of the 8-GPU run).  User degree 1 + Poisson(mean
    - 1), item popularity Zipf (p(i) ~ (i + 1)^-zipf_a over the item ids), items drawn by
    inverse CDF.  Repeated (user, item) pairs are kept (harmless for message passing; the
    graph only has to carry config 5's size and skew).  No held-out split: every
    interaction is a training edge."""
    nu = max(int(round(n_users * scale)), 1)
    ni = max(int(round(n_items * scale)), 1)
    nt = max(int(round(n_interactions * scale)), 1)
    rng = np.random.default_rng(seed)
    mean = nt / nu
    udeg = 1 + rng.poisson(max(mean - 1.0, 0.0), nu)
    udeg = _fix_sum(udeg, nt, 1, rng)
    w = np.arange(1, ni + 1, dtype=np.float64) ** (-zipf_a)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    items = np.searchsorted(cdf, rng.random(nt), side="right").astype(np.int64)
    np.minimum(items, ni - 1, out=items)
    ptr = np.zeros(nu + 1, np.int64)
    np.cumsum(udeg, out=ptr[1:])
    none = np.full(nu, -1, np.int64)
    return UIGraph(nu, ni, ptr, items, none, none, nt)


def synthetic_ii_edges(g: UIGraph, k: int = 20, seed: int = 42, min_sim: float = 0.3):
    """Config 3 I-I kNN stand-in: per item up to k neighbours drawn proportional to
    popularity, similarity U(0.3,1) kept if >= min_sim (graphs/build_ii_knn.py:91-111
    row=item, col=neighbour). Returns (rows, cols, sims) in item index space."""
    rng = np.random.default_rng(seed + 1)
    pop = np.bincount(g.user_items, minlength=g.n_items).astype(np.float64) + 1.0
    pop /= pop.sum()
    rows = np.repeat(np.arange(g.n_items, dtype=np.int64), k)
    cols = rng.choice(g.n_items, size=len(rows), p=pop)
    sims = rng.uniform(0.3, 1.0, len(rows)).astype(np.float32)
    keep = (cols != rows) & (sims >= min_sim)
    return rows[keep], cols[keep], sims[keep]


def ii_edge_columns(n_users: int, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    """I-I kNN edges appended to the homogeneous edge_index (SURVEY.md A10,
    "extension": no reference trainer consumes them). Message flows neighbour ->
    item, i.e. src = n_users+col, dst = n_users+row."""
    ei = np.empty((2, len(rows)), np.int64)
    ei[0] = n_users + np.asarray(cols, np.int64)
    ei[1] = n_users + np.asarray(rows, np.int64)
    return ei


def synthetic_item_features(n_items: int, dim: int = 128, seed: int = 42, normalize: bool = True):
    """``fused_interacted.npy`` stand-in: N(0,1) rows, L2-normalised like
    embeddings/fuse_modal.py:239-241."""
    rng = np.random.default_rng(seed + 7)
    x = rng.standard_normal((n_items, dim), dtype=np.float32)
    if normalize:
        x /= (np.linalg.norm(x, axis=1, keepdims=True) + 1e-8)
    return x
