"""CPU restatement of the reference's hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, as the checker (and the timed CPU
baseline, `cpu_baseline.kind = "port"`), never as the thing measured or shipped.

It restates, op for op, the torch CPU calls of the reference
(EXLYSHA/Recommendar-Systems @ 2025-10-03, an MMRec fork) on the path named by
BASELINE.json's north_star; each function cites the reference file:line it
follows.  The restatement is pinned by the golden fixtures in tests/golden/,
captured from the reference itself in the build container by
tools/capture_golden.py (tests/test_oracle_golden.py).

Third-party arithmetic: PyTorch CPU kernels (sparse addmm, sgemm, topk, Adam),
torch 2.10.0 here; the reference pins torch 1.11.0 (requirements.txt:5).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------
# adjacency construction
# ---------------------------------------------------------------------------
def lightgcn_norm_adj_dok(train_u, train_i, n_users, n_items):
    """Literal restatement of LightGCN.get_norm_adj_mat (src/models/lightgcn.py:65-103):
    dict of (row, col) -> 1 over both halves, dok matrix, (A>0).sum(1)+1e-7, ^-0.5 in
    float64, D*A*D, coo, float32 values.  Small graphs only (Python loop)."""
    n = n_users + n_items
    A = sp.dok_matrix((n, n), dtype=np.float32)
    data = dict(zip(zip(train_u, train_i + n_users), [1] * len(train_u)))
    data.update(dict(zip(zip(train_i + n_users, train_u), [1] * len(train_u))))
    for (r, c), v in data.items():
        A[r, c] = v
    deg = np.array((A > 0).sum(axis=1).flatten())[0] + 1e-7
    D = sp.diags(np.power(deg, -0.5))
    L = sp.coo_matrix(D * A * D)
    idx = torch.from_numpy(np.vstack([L.row, L.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(L.data.astype(np.float32)), (n, n))


def lightgcn_norm_adj_vec(train_u, train_i, n_users, n_items):
    """Vectorised restatement with identical float64 -> float32 values (for large graphs)."""
    n = n_users + n_items
    key = np.unique(train_u.astype(np.int64) * (1 << 32) + train_i.astype(np.int64))
    u = key >> 32
    i = key & 0xFFFFFFFF
    rows = np.concatenate([u, i + n_users])
    cols = np.concatenate([i + n_users, u])
    deg = np.bincount(rows, minlength=n).astype(np.float64) + 1e-7
    dinv = np.power(deg, -0.5)
    vals = (dinv[rows] * dinv[cols]).astype(np.float32)
    idx = torch.from_numpy(np.vstack([rows, cols]))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(vals), (n, n)).coalesce()


def layergcn_normalize(indices: torch.Tensor, n_users: int, n_items: int) -> torch.Tensor:
    """LayerGCN._normalize_adj_m (src/models/layergcn.py:72-81), float32."""
    adj = torch.sparse_coo_tensor(indices, torch.ones_like(indices[0]), (n_users, n_items))
    row_sum = 1e-7 + torch.sparse.sum(adj, -1).to_dense()
    col_sum = 1e-7 + torch.sparse.sum(adj.t(), -1).to_dense()
    r = torch.pow(row_sum, -0.5)[indices[0]]
    c = torch.pow(col_sum, -0.5)[indices[1]]
    return r * c


def layergcn_masked_adj(edge_indices: torch.Tensor, keep_idx: torch.Tensor, n_users: int, n_items: int):
    """LayerGCN.pre_epoch_processing body after sampling keep_idx (layergcn.py:63-70)."""
    keep = edge_indices[:, keep_idx].clone()
    vals = layergcn_normalize(keep, n_users, n_items)
    allv = torch.cat((vals, vals))
    keep[1] += n_users
    alli = torch.cat((keep, torch.flip(keep, [0])), 1)
    n = n_users + n_items
    return torch.sparse_coo_tensor(alli, allv, (n, n))


def smore_norm_adj(train_u, train_i, n_users, n_items):
    """SMORE.get_adj_mat (src/models/smore.py:176-207): float32, no epsilon, inf -> 0."""
    n = n_users + n_items
    R = sp.coo_matrix((np.ones(len(train_u), dtype=np.float32), (train_u, train_i)), shape=(n_users, n_items))
    adj = sp.dok_matrix((n, n), dtype=np.float32).tolil()
    R = R.tolil()
    adj[:n_users, n_users:] = R
    adj[n_users:, :n_users] = R.T
    adj = adj.todok()
    rowsum = np.array(adj.sum(1))
    with np.errstate(divide="ignore"):
        d_inv = np.power(rowsum, -0.5).flatten()
    d_inv[np.isinf(d_inv)] = 0.0
    Dm = sp.diags(d_inv)
    norm = Dm.dot(adj).dot(Dm).tocoo().tolil()
    Rn = norm[:n_users, n_users:]
    norm = norm.tocsr()

    def to_t(m):
        m = m.tocoo().astype(np.float32)
        idx = torch.from_numpy(np.vstack((m.row, m.col)).astype(np.int64))
        return torch.sparse_coo_tensor(idx, torch.from_numpy(m.data), m.shape)

    return to_t(norm), to_t(Rn)


def knn_normalized_graph(feat: torch.Tensor, k: int) -> torch.Tensor:
    """build_sim + build_knn_normalized_graph(is_sparse=True, 'sym')
    (src/utils/utils.py:134-181, called at src/models/smore.py:59-60,69-70)."""
    ctx = feat.div(torch.norm(feat, p=2, dim=-1, keepdim=True))
    sim = torch.mm(ctx, ctx.transpose(1, 0))
    knn_val, knn_ind = torch.topk(sim, k, dim=-1)
    n = sim.shape[0]
    row = torch.arange(n).repeat_interleave(k)
    col = knn_ind.reshape(-1)
    v = knn_val.flatten()
    deg = torch.zeros(n, dtype=v.dtype).index_add_(0, row, v)
    dis = deg.pow_(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    w = dis[row] * v * dis[col]
    return torch.sparse_coo_tensor(torch.stack([row, col]), w, (n, n))


def max_pool_fusion(image_adj: torch.Tensor, text_adj: torch.Tensor) -> torch.Tensor:
    """SMORE.max_pool_fusion (src/models/smore.py:153-174): elementwise max over the edge union."""
    ia, ta = image_adj.coalesce(), text_adj.coalesce()
    ci = torch.cat((ia.indices(), ta.indices()), dim=1)
    ci, inv = torch.unique(ci, dim=1, return_inverse=True)
    vi = torch.full((ci.size(1),), float("-inf"))
    vt = torch.full((ci.size(1),), float("-inf"))
    vi[inv[: ia.indices().size(1)]] = ia.values()
    vt[inv[ia.indices().size(1):]] = ta.values()
    v, _ = torch.max(torch.stack((vi, vt)), dim=0)
    return torch.sparse_coo_tensor(ci, v, ia.size()).coalesce()


# ---------------------------------------------------------------------------
# propagation
# ---------------------------------------------------------------------------
def lightgcn_forward(A: torch.Tensor, E0: torch.Tensor, K: int) -> torch.Tensor:
    """LightGCN.forward (src/models/lightgcn.py:117-130): mean of E^0..E^K."""
    layers = [E0]
    x = E0
    for _ in range(K):
        x = torch.sparse.mm(A, x)
        layers.append(x)
    return torch.mean(torch.stack(layers, dim=1), dim=1)


def layergcn_forward(A: torch.Tensor, E0: torch.Tensor, K: int) -> torch.Tensor:
    """LayerGCN.forward (src/models/layergcn.py:127-140): cosine-reweighted layers, sum of 1..K."""
    x = E0
    out = []
    for _ in range(K):
        x = torch.sparse.mm(A, x)
        w = F.cosine_similarity(x, E0, dim=-1)
        x = torch.einsum("a,ab->ab", w, x)
        out.append(x)
    return torch.sum(torch.stack(out, dim=0), dim=0)


# ---------------------------------------------------------------------------
# losses (autograd gives the gradients)
# ---------------------------------------------------------------------------
def lightgcn_loss(user_emb, item_emb, A, K, trip, reg):
    """LightGCN.calculate_loss (src/models/lightgcn.py:132-156) with BPRLoss/EmbLoss
    (src/common/loss.py:33-51)."""
    n_users = user_emb.shape[0]
    allf = lightgcn_forward(A, torch.cat([user_emb, item_emb], 0), K)
    uf, itf = allf[:n_users], allf[n_users:]
    u, p, n = trip[0], trip[1], trip[2]
    ps = torch.mul(uf[u], itf[p]).sum(dim=1)
    ns = torch.mul(uf[u], itf[n]).sum(dim=1)
    mf = -torch.log(1e-10 + torch.sigmoid(ps - ns)).mean()
    e = [user_emb[u], item_emb[p], item_emb[n]]
    r = torch.zeros(1)
    for x in e:
        r += torch.norm(x, p=2)
    r /= e[-1].shape[0]
    return mf + reg * r


def layergcn_loss(user_emb, item_emb, A, K, trip, reg):
    """LayerGCN.calculate_loss (src/models/layergcn.py:142-177) with L2Loss (loss.py:58-61)."""
    n_users = user_emb.shape[0]
    allf = layergcn_forward(A, torch.cat([user_emb, item_emb], 0), K)
    uf, itf = allf[:n_users], allf[n_users:]
    u, p, n = trip[0], trip[1], trip[2]
    ps = torch.mul(uf[u], itf[p]).sum(dim=1)
    ns = torch.mul(uf[u], itf[n]).sum(dim=1)
    mf = torch.sum(-F.logsigmoid(ps - ns))
    r = torch.zeros(1)
    for x in (user_emb[u], item_emb[p], item_emb[n]):
        r += torch.sum(x ** 2) * 0.5
    return mf + reg * r


# ---------------------------------------------------------------------------
# evaluation
# ---------------------------------------------------------------------------
def fullsort_reference(U: torch.Tensor, I: torch.Tensor, users: torch.Tensor, mask_u: torch.Tensor,
                       mask_i: torch.Tensor, k: int):
    """full_sort_predict + mask + topk (src/models/lightgcn.py:158-166, trainer.py:521-526).
    mask_u are batch-row indices, mask_i item ids.  Returns (scores, vals, idx)."""
    scores = torch.matmul(U[users], I.transpose(0, 1))
    raw = scores.clone()
    scores[mask_u, mask_i] = -1e10
    vals, idx = torch.topk(scores, k, dim=-1)
    return raw, vals, idx


def canonical_topk(scores: np.ndarray, k: int):
    """Top-k by (score desc, index asc) — the build's canonical tie-break."""
    order = np.lexsort((np.broadcast_to(np.arange(scores.shape[1]), scores.shape), -scores), axis=1)
    idx = order[:, :k]
    return np.take_along_axis(scores, idx, 1), idx


def metrics_reference(topk_idx: np.ndarray, eval_items: list, metrics=("recall", "ndcg", "precision", "map"),
                      topk=(5, 10, 20, 50)):
    """TopKEvaluator.evaluate + metrics.* (src/utils/topk_evaluator.py:58-102,
    src/utils/metrics.py:12-118): Python hit matrix, cumulative metrics, round(.,4)."""
    pos_len = np.asarray([len(x) for x in eval_items])
    hit = np.asarray([[True if i in m else False for i in n] for m, n in zip(eval_items, topk_idx)])

    def recall(h, pl):
        return (np.cumsum(h, axis=1) / pl.reshape(-1, 1)).mean(axis=0)

    def ndcg(h, pl):
        len_rank = np.full_like(pl, h.shape[1])
        il = np.where(pl > len_rank, len_rank, pl)
        ir = np.zeros_like(h, dtype=np.float64)
        ir[:, :] = np.arange(1, h.shape[1] + 1)
        idcg = np.cumsum(1.0 / np.log2(ir + 1), axis=1)
        for row, x in enumerate(il):
            idcg[row, x:] = idcg[row, x - 1]
        rk = np.zeros_like(h, dtype=np.float64)
        rk[:, :] = np.arange(1, h.shape[1] + 1)
        dcg = np.cumsum(np.where(h, 1.0 / np.log2(rk + 1), 0), axis=1)
        return (dcg / idcg).mean(axis=0)

    def precision(h, pl):
        return (h.cumsum(axis=1) / np.arange(1, h.shape[1] + 1)).mean(axis=0)

    def map_(h, pl):
        pre = h.cumsum(axis=1) / np.arange(1, h.shape[1] + 1)
        sp_ = np.cumsum(pre * h.astype(np.float64), axis=1)
        len_rank = np.full_like(pl, h.shape[1])
        al = np.where(pl > len_rank, len_rank, pl)
        res = np.zeros_like(h, dtype=np.float64)
        for row, x in enumerate(al):
            rg = np.arange(1, h.shape[1] + 1)
            rg[x:] = rg[x - 1]
            res[row] = sp_[row] / rg
        return res.mean(axis=0)

    fns = {"recall": recall, "ndcg": ndcg, "precision": precision, "map": map_}
    out = {}
    for m in metrics:
        v = fns[m](hit, pos_len)
        for k in topk:
            out[f"{m}@{k}"] = round(v[k - 1], 4)
    return out


# ---------------------------------------------------------------------------
# a whole LightGCN step on CPU (the cpu_baseline leg of bench.py)
# ---------------------------------------------------------------------------
class LightGCNCPU:
    """Reference-identical CPU LightGCN training step: forward with torch.sparse.mm,
    autograd backward, torch.optim.Adam (src/models/lightgcn.py, src/common/trainer.py:186-238)."""

    def __init__(self, A: torch.Tensor, user_emb: np.ndarray, item_emb: np.ndarray, K: int, reg: float,
                 lr: float = 1e-3):
        self.A = A
        self.K = K
        self.reg = reg
        self.u = torch.nn.Parameter(torch.from_numpy(user_emb.copy()))
        self.i = torch.nn.Parameter(torch.from_numpy(item_emb.copy()))
        self.opt = torch.optim.Adam([self.u, self.i], lr=lr)

    def step(self, trip: torch.Tensor) -> float:
        self.opt.zero_grad()
        loss = lightgcn_loss(self.u, self.i, self.A, self.K, trip, self.reg)
        v = loss.item()
        loss.backward()
        self.opt.step()
        return v


# ---------------------------------------------------------------------------
# training-batch feeder (cpu_baseline leg: the reference's Python sampler)
# ---------------------------------------------------------------------------
class ReferenceSampler:
    """TrainDataLoader._get_neg_sample / _sample_neg_ids / _random restated
    (src/utils/dataloader.py:226-275,307-309): sequential slices of the shuffled
    training interactions, one negative per row drawn with random.sample from the
    training-item list and redrawn while it is in the user's history."""

    def __init__(self, train_u, train_i, seed=999):
        import random

        self.rand = random.Random(seed)
        self.u = np.asarray(train_u)
        self.i = np.asarray(train_i)
        self.hist = {}
        for a, b in zip(self.u.tolist(), self.i.tolist()):
            self.hist.setdefault(a, set()).add(b)
        self.all_items = sorted(set(self.i.tolist()))
        self.rng = np.random.default_rng(seed)
        self.order = self.rng.permutation(self.u.size)
        self.pr = 0

    def next(self, batch):
        if self.pr >= self.u.size:
            self.order = self.rng.permutation(self.u.size)
            self.pr = 0
        sel = self.order[self.pr:self.pr + batch]
        self.pr += batch
        us = self.u[sel]
        neg = []
        for a in us.tolist():
            x = self.rand.sample(self.all_items, 1)[0]
            while x in self.hist[a]:
                x = self.rand.sample(self.all_items, 1)[0]
            neg.append(x)
        return torch.from_numpy(np.vstack([us, self.i[sel], np.asarray(neg)]).astype(np.int64))
