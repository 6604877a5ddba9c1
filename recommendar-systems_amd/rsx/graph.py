"""Host-side graph builders: normalised adjacencies in CSR form (once per model / epoch).

Value semantics follow the reference exactly (pinned bit-for-bit by
tests/test_graph_golden.py against the reference's own tensors):

* LightGCN / LayerGCN eval graph (src/models/lightgcn.py:65-103,
  src/models/layergcn.py:91-117): binary symmetric A = [[0, R], [R^T, 0]],
  d_v = deg_v + 1e-7 in float64, value = d_r^-1/2 * d_c^-1/2 in float64, cast to f32.
* LayerGCN edge-dropout graph (src/models/layergcn.py:51-89): degrees of the
  kept edges + 1e-7 in float32, value = r^-1/2 * c^-1/2 in float32.
* SMORE UI graph (src/models/smore.py:176-207): float32 row sums, ^-1/2 with
  inf -> 0 (no epsilon), value = d_r * 1 * d_c in float32.

The reference builds these with a Python dok loop (2-4 s at Amazon scale, hours at
10^8 edges); here they are vectorised numpy, O(E log E).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _sym_edges(u: np.ndarray, i: np.ndarray, n_users: int):
    """Unique (row, col) pairs of the symmetric bipartite graph, users first."""
    key = np.unique(u.astype(np.int64) * (1 << 32) + i.astype(np.int64))
    uu = (key >> 32).astype(np.int64)
    ii = (key & 0xFFFFFFFF).astype(np.int64)
    rows = np.concatenate([uu, ii + n_users])
    cols = np.concatenate([ii + n_users, uu])
    return rows, cols


def to_csr(rows: np.ndarray, cols: np.ndarray, vals: np.ndarray, n_rows: int, n_cols: int):
    """(rowptr int64, col int32, val f32) with columns sorted inside each row."""
    order = np.lexsort((cols, rows))
    r = rows[order]
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum(np.bincount(r, minlength=n_rows)[:n_rows])
    return rowptr, cols[order].astype(np.int32), vals[order].astype(np.float32)


def lightgcn_norm_adj(train_u: np.ndarray, train_i: np.ndarray, n_users: int, n_items: int):
    """D^-1/2 A D^-1/2 with the reference's float64 normalisation; returns CSR triple."""
    n = n_users + n_items
    rows, cols = _sym_edges(train_u, train_i, n_users)
    deg = np.bincount(rows, minlength=n).astype(np.float64) + 1e-7
    dinv = np.power(deg, -0.5)
    vals = (dinv[rows] * dinv[cols]).astype(np.float32)
    return to_csr(rows, cols, vals, n, n)


def layergcn_edge_values(e_u: np.ndarray, e_i: np.ndarray, n_users: int, n_items: int) -> np.ndarray:
    """float32 1/sqrt(deg+1e-7) products of the kept user-item edges (layergcn.py:72-81)."""
    ru = np.bincount(e_u, minlength=n_users).astype(np.float32)
    ci = np.bincount(e_i, minlength=n_items).astype(np.float32)
    r = np.float32(1e-7) + ru
    c = np.float32(1e-7) + ci
    r_inv = (np.float32(1.0) / np.sqrt(r)).astype(np.float32)
    c_inv = (np.float32(1.0) / np.sqrt(c)).astype(np.float32)
    return (r_inv[e_u] * c_inv[e_i]).astype(np.float32)


def layergcn_masked_adj(e_u: np.ndarray, e_i: np.ndarray, n_users: int, n_items: int):
    """Symmetric adjacency of the kept edges with float32 renormalisation; CSR triple."""
    vals = layergcn_edge_values(e_u, e_i, n_users, n_items)
    rows = np.concatenate([e_u, e_i + n_users]).astype(np.int64)
    cols = np.concatenate([e_i + n_users, e_u]).astype(np.int64)
    v = np.concatenate([vals, vals])
    n = n_users + n_items
    # duplicates cannot occur (multinomial / random.sample draw without replacement)
    return to_csr(rows, cols, v, n, n)


def smore_norm_adj(train_u: np.ndarray, train_i: np.ndarray, n_users: int, n_items: int):
    """SMORE's float32 sym-normalised UI adjacency (no epsilon, inf -> 0); CSR triple."""
    n = n_users + n_items
    rows, cols = _sym_edges(train_u, train_i, n_users)
    deg = np.bincount(rows, minlength=n).astype(np.float32)
    with np.errstate(divide="ignore"):
        dinv = np.power(deg, np.float32(-0.5)).astype(np.float32)
    dinv[np.isinf(dinv)] = 0.0
    vals = (dinv[rows] * np.float32(1.0) * dinv[cols]).astype(np.float32)
    return to_csr(rows, cols, vals, n, n)


def csr_block(rowptr, col, val, r0: int, r1: int, c0: int, c1: int):
    """Sub-block rows [r0, r1) x cols [c0, c1) of a CSR matrix, columns rebased to c0."""
    n_cols = max(c1, int(col.max()) + 1 if col.size else c1)
    sub = sp.csr_matrix((val, col.astype(np.int64), rowptr), shape=(rowptr.size - 1, n_cols))[r0:r1, c0:c1].tocsr()
    sub.sort_indices()
    return sub.indptr.astype(np.int64), sub.indices.astype(np.int32), sub.data.astype(np.float32)


def history_csr(train_u: np.ndarray, train_i: np.ndarray, n_users: int):
    """Per-user sorted training items (mask for full-sort, history for the sampler)."""
    key = np.unique(train_u.astype(np.int64) * (1 << 32) + train_i.astype(np.int64))
    u = (key >> 32).astype(np.int64)
    i = (key & 0xFFFFFFFF).astype(np.int32)
    rowptr = np.zeros(n_users + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum(np.bincount(u, minlength=n_users)[:n_users])
    return rowptr, i
