"""Synthetic Amazon-shaped interaction graphs (own generator, seed-deterministic).

The Amazon datasets the reference trains on are a Google-Drive download
(reference `data/README.md:3`) and are not available offline, so every config
runs on graphs with the same shape statistics:

* every user has ``5 + Geometric`` interactions (5-core on the user side),
  with the mean matching the dataset's interactions per user;
* item popularity follows Zipf(0.8) over a random permutation of item ids;
* (user, item) pairs are unique;
* ``x_label`` follows the reference's preprocessing split rule
  (`preprocessing/1splitting.ipynb`, cell "new_label"): a user with fewer
  than 10 interactions keeps the last two as valid (1) / test (2); otherwise
  80 / 10 / 10 in interaction order.

Output is a pandas DataFrame with the reference's `.inter` columns
(`userID`, `itemID`, `x_label`, reference `src/configs/dataset/*.yaml`), or a
TSV file in the layout `RecDataset` reads (`src/utils/dataset.py:50-55`).
"""
from __future__ import annotations

import os

import numpy as np

# Amazon dataset shapes quoted by the reference (`evaluation/README.md:8-9`) and
# by the SMORE paper for clothing (SURVEY.md section 8 sizes table).
SHAPES = {
    "baby": (19445, 7050, 160792),
    "sports": (35598, 18357, 296337),
    "clothing": (39387, 23033, 278677),
    "elec": (192403, 63001, 1689188),
}


def _draw_unique_items(rng, deg, weights, n_items):
    """Return (users, items) with ``deg[u]`` distinct items per user drawn ~ weights."""
    n_users = deg.shape[0]
    cdf = np.cumsum(weights, dtype=np.float64)
    cdf /= cdf[-1]
    need = deg.astype(np.int64).copy()
    have_u = []
    have_i = []
    got = np.zeros(n_users, dtype=np.int64)
    keys_seen = np.empty(0, dtype=np.int64)
    for _ in range(64):
        short = need - got
        active = np.nonzero(short > 0)[0]
        if active.size == 0:
            break
        # oversample so that most users finish in one round
        cnt = np.ceil(short[active] * 1.25 + 2).astype(np.int64)
        users = np.repeat(active, cnt)
        items = np.searchsorted(cdf, rng.random(users.size), side="right")
        items = np.minimum(items, n_items - 1)
        keys = users.astype(np.int64) * n_items + items
        # first occurrence order is preserved (interaction order matters for the split)
        _, first = np.unique(keys, return_index=True)
        first.sort()
        keys = keys[first]
        keys = keys[~np.isin(keys, keys_seen)]
        users = keys // n_items
        # cap each user at its remaining need, keeping draw order
        order = np.argsort(users, kind="stable")
        users_s = users[order]
        starts = np.searchsorted(users_s, users_s, side="left")
        rank = np.arange(users_s.size) - starts
        keep_sorted = rank < short[users_s]
        keep = np.zeros(users.size, dtype=bool)
        keep[order[keep_sorted]] = True
        keys = keys[keep]
        users = keys // n_items
        np.add.at(got, users, 1)
        keys_seen = np.concatenate([keys_seen, keys])
        have_u.append(users)
        have_i.append(keys % n_items)
    u = np.concatenate(have_u)
    i = np.concatenate(have_i)
    # group by user, keeping per-user draw order (stable)
    order = np.argsort(u, kind="stable")
    return u[order], i[order]


def split_labels(user_sorted: np.ndarray) -> np.ndarray:
    """x_label per interaction for interactions grouped by user in order."""
    n = user_sorted.size
    starts = np.r_[0, np.nonzero(np.diff(user_sorted))[0] + 1]
    counts = np.diff(np.r_[starts, n])
    pos = np.arange(n) - np.repeat(starts, counts)
    cnt = np.repeat(counts, counts)
    label = np.zeros(n, dtype=np.int64)
    small = cnt < 10
    label[small & (pos == cnt - 2)] = 1
    label[small & (pos == cnt - 1)] = 2
    n_train = np.floor(cnt * 0.8).astype(np.int64)
    n_valid = np.floor(cnt * 0.1).astype(np.int64)
    big = ~small
    label[big & (pos >= n_train) & (pos < n_train + n_valid)] = 1
    label[big & (pos >= n_train + n_valid)] = 2
    return label


def amazon_like(n_users: int, n_items: int, n_inter: int, seed: int = 0, zipf: float = 0.8):
    """Generate an Amazon-shaped interaction table.

    Returns a pandas DataFrame with columns userID, itemID, x_label.
    """
    import pandas as pd

    rng = np.random.default_rng(seed)
    avg = max(n_inter / n_users, 5.0 + 1e-3)
    p = 1.0 / max(avg - 4.0, 1.0 + 1e-9)
    deg = 5 + rng.geometric(p, size=n_users) - 1
    deg = np.minimum(deg, max(5, n_items // 2))
    perm = rng.permutation(n_items)
    w = np.empty(n_items, dtype=np.float64)
    w[perm] = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), zipf)
    u, i = _draw_unique_items(rng, deg, w, n_items)
    lab = split_labels(u)
    # make sure the largest item id exists so that n_items = max(itemID) + 1
    # (reference `src/utils/dataset.py:47`)
    df = pd.DataFrame({"userID": u.astype(np.int64), "itemID": i.astype(np.int64),
                       "x_label": lab})
    if df["itemID"].max() != n_items - 1:
        df.loc[df.index[df["x_label"] == 0][0], "itemID"] = n_items - 1
        df = df.drop_duplicates(["userID", "itemID"]).reset_index(drop=True)
    return df


def shaped(name: str, seed: int = 0, scale: float = 1.0):
    nu, ni, ne = SHAPES[name]
    return amazon_like(max(8, int(nu * scale)), max(8, int(ni * scale)), max(40, int(ne * scale)), seed)


def write_inter(df, data_root: str, dataset: str, file_name: str | None = None) -> str:
    """Write `df` as `<data_root>/<dataset>/<dataset>.inter` (TSV, reference layout)."""
    d = os.path.join(data_root, dataset)
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, file_name or f"{dataset}.inter")
    df[["userID", "itemID", "x_label"]].to_csv(path, sep="\t", index=False)
    return path


def features(n_items: int, dim: int, seed: int, l2_normalise: bool = False) -> np.ndarray:
    """Synthetic item feature table: N(0,1) f32, optionally L2-normalised rows."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n_items, dim), dtype=np.float32)
    if l2_normalise:
        x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x


# C4: 10M users x 1M items, ~10 interactions per user (1e8), Zipf(0.8)
# items.  The global graph is a fixed sequence of user chunks, each generated from
# its own seed, so a rank owning chunks [c0, c1) builds exactly its share of the
# same graph whatever the world size.
C4 = dict(n_users=10_000_000, n_items=1_000_000, avg=10.0, chunk_users=1_250_000)


def zipf_cdf(n_items: int, seed: int, zipf: float = 0.8) -> np.ndarray:
    """Cumulative Zipf(zipf) popularity over a seeded random permutation of item ids."""
    rng = np.random.default_rng([seed, 0x5EED])
    perm = rng.permutation(n_items)
    w = np.empty(n_items, dtype=np.float64)
    w[perm] = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), zipf)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return cdf


def chunk_graph(chunk: int, chunk_users: int, n_items: int, avg: float, cdf: np.ndarray, seed: int = 0):
    """Interactions of users [chunk*chunk_users, (chunk+1)*chunk_users) as
    (user - chunk*chunk_users, item, x_label) arrays, grouped by user.  Degrees are
    5 + Geometric (mean `avg`); duplicate draws of a user are dropped (so the mean
    lands slightly below `avg`); labels follow the reference split rule."""
    rng = np.random.default_rng([seed, chunk])
    p = 1.0 / max(avg - 4.0, 1.0 + 1e-9)
    deg = 5 + rng.geometric(p, size=chunk_users) - 1
    u = np.repeat(np.arange(chunk_users, dtype=np.int64), deg)
    i = np.minimum(np.searchsorted(cdf, rng.random(u.size), side="right"), n_items - 1).astype(np.int64)
    key = np.unique(u * n_items + i)  # sorted by (user, item), duplicates dropped
    u, i = key // n_items, key % n_items
    return u, i, split_labels(u)
