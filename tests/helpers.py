"""Shared test helpers: fixture decoding, comparisons and the multi-process rendezvous."""
from __future__ import annotations

import atexit
import os
import shutil
import tempfile

import numpy as np
import torch


def store_path() -> str:
    """A fresh rendezvous file for `init_pg` (one per spawned job).

    Spawned tests rendezvous through a torch FileStore, not a TCP port: a port picked by
    binding port 0 and closing the socket can be taken again before rank 0 listens on it
    (GPUTEST_r05: EADDRINUSE), and a rank retrying connect to a not-yet-listening
    ephemeral port can connect to itself. A file cannot race that way."""
    d = tempfile.mkdtemp(prefix="rsx_pg_")
    atexit.register(shutil.rmtree, d, True)
    return os.path.join(d, "store")


def init_pg(backend: str, rank: int, world: int, store: str, **kw):
    """torch.distributed.init_process_group over the FileStore at `store`; RANK and
    WORLD_SIZE are exported too, as a torchrun launch would (rsx reads WORLD_SIZE)."""
    import torch.distributed as dist

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    for k in ("MASTER_ADDR", "MASTER_PORT"):
        os.environ.pop(k, None)
    dist.init_process_group(backend, init_method="file://" + store, rank=rank, world_size=world, **kw)


def coo_from(z, prefix, n):
    idx = torch.from_numpy(z[prefix + "_idx"].astype(np.int64))
    val = torch.from_numpy(z[prefix + "_val"])
    return torch.sparse_coo_tensor(idx, val, (n, n)).coalesce()


def coo_sorted(idx: np.ndarray, val: np.ndarray):
    """(row, col, val) sorted by (row, col)."""
    order = np.lexsort((idx[1], idx[0]))
    return idx[0][order], idx[1][order], val[order]


def csr_to_sorted(rowptr, col, val):
    rows = np.repeat(np.arange(rowptr.size - 1), np.diff(rowptr))
    return rows.astype(np.int64), col.astype(np.int64), val


def params(z, prefix, model):
    if model == "LightGCN":
        return z[prefix + "embedding_dict.user_emb"], z[prefix + "embedding_dict.item_emb"]
    if model == "LayerGCN":
        return z[prefix + "user_embeddings"], z[prefix + "item_embeddings"]
    return z[prefix + "user_embedding.weight"], z[prefix + "item_id_embedding.weight"]


def metric_dict(z, tag):
    return {str(k): float(v) for k, v in zip(z[tag + "_metric_keys"], z[tag + "_metric_vals"])}


def eval_lists(z, tag):
    lens = z[tag + "_eval_len"]
    items = z[tag + "_eval_items"]
    out = []
    o = 0
    for n in lens:
        out.append(items[o:o + n])
        o += n
    return out


def train_mask_pairs(z, users: np.ndarray):
    """(batch_row, item) of the users' training items (EvalDataLoader mask, dataloader.py:370-391)."""
    tu, ti = z["train_u"], z["train_i"]
    pos = {int(u): k for k, u in enumerate(users)}
    sel = np.isin(tu, users)
    rows = np.array([pos[int(u)] for u in tu[sel]], dtype=np.int64)
    return rows, ti[sel].astype(np.int64)


def topk_equal_modulo_ties(idx_a, idx_b, scores, rtol=1e-5):
    """Rows match exactly, or differ only among items whose scores tie within rtol."""
    bad = 0
    for r in range(idx_a.shape[0]):
        if np.array_equal(idx_a[r], idx_b[r]):
            continue
        sa = scores[r, idx_a[r]]
        sb = scores[r, idx_b[r]]
        scale = max(1e-6, float(np.abs(scores[r]).max()))
        if not np.allclose(sa, sb, rtol=0, atol=rtol * scale):
            bad += 1
    return bad


def canonical_topk_fast(scores: np.ndarray, k: int):
    """oracle.canonical_topk (score desc, index asc) for wide rows: the k-th largest value
    per row by partition, then an exact (score, index) sort of the items at or above it."""
    n_rows, n = scores.shape
    kth = -np.partition(-scores, k - 1, axis=1)[:, k - 1]
    idx = np.empty((n_rows, k), dtype=np.int64)
    val = np.empty((n_rows, k), dtype=scores.dtype)
    for r in range(n_rows):
        cand = np.nonzero(scores[r] >= kth[r])[0]
        sv = scores[r, cand]
        order = np.lexsort((cand, -sv))[:k]
        idx[r] = cand[order]
        val[r] = sv[order]
    return val, idx
