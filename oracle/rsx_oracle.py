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


# ---------------------------------------------------------------------------
# SMORE on CPU (parity oracle for the SMORE path + the C3/C5 cpu_baseline leg)
# ---------------------------------------------------------------------------
class SMORECPU(torch.nn.Module):
    """SMORE (src/models/smore.py:24-411) restated in torch on the CPU: parameters in
    the reference's creation order (:38-138), graphs from the restatements above
    (:45-75, 176-207), forward (:256-349), bpr_loss / InfoNCE / calculate_loss
    (:352-411).  inject_mode 'residual', spectral_weight_norm True (the YAML
    defaults); the diagnostics (.item() statistics) are omitted, they change no state."""

    def __init__(self, train_u, train_i, n_users, n_items, v_feat, t_feat, d=64, n_ui_layers=4, n_layers=1,
                 reg_weight=1e-5, image_k=20, text_k=15, dropout=0.0, cl_loss=0.01, cl_temp=0.2, batch_size=2048,
                 init: dict | None = None):
        super().__init__()
        nn = torch.nn
        self.n_users, self.n_items, self.d = n_users, n_items, d
        self.n_ui_layers, self.n_layers = n_ui_layers, n_layers
        self.reg_weight, self.cl_loss, self.cl_temp, self.batch_size = reg_weight, cl_loss, cl_temp, batch_size
        self.inject_scale = 0.7
        self.dropout = nn.Dropout(p=dropout)
        self.user_embedding = nn.Embedding(n_users, d)
        self.item_id_embedding = nn.Embedding(n_items, d)
        nn.init.xavier_uniform_(self.user_embedding.weight)
        nn.init.xavier_uniform_(self.item_id_embedding.weight)
        self.norm_adj, self.R = smore_norm_adj(np.asarray(train_u), np.asarray(train_i), n_users, n_items)
        v = torch.as_tensor(np.asarray(v_feat, dtype=np.float32))
        t = torch.as_tensor(np.asarray(t_feat, dtype=np.float32))
        self.image_embedding = nn.Embedding.from_pretrained(v.clone(), freeze=False)
        self.image_original_adj = knn_normalized_graph(v, image_k)
        self.text_embedding = nn.Embedding.from_pretrained(t.clone(), freeze=False)
        self.text_original_adj = knn_normalized_graph(t, text_k)
        self.fusion_adj = max_pool_fusion(self.image_original_adj, self.text_original_adj)
        self.image_trs = nn.Linear(v.shape[1], d)
        self.text_trs = nn.Linear(t.shape[1], d)
        self.query_v = nn.Sequential(nn.Linear(d, d), nn.Tanh(), nn.Linear(d, d, bias=False))
        self.query_t = nn.Sequential(nn.Linear(d, d), nn.Tanh(), nn.Linear(d, d, bias=False))
        self.gate_v = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.gate_t = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.gate_f = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.gate_image_prefer = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.gate_text_prefer = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.gate_fusion_prefer = nn.Sequential(nn.Linear(d, d), nn.Sigmoid())
        self.image_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.text_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.fusion_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.mg_interval, self.mg_alpha, self.mg_beta = 3, 0.5, 0.2
        self.global_step = 0
        if init is not None:
            with torch.no_grad():
                for n, p in self.named_parameters():
                    p.copy_(torch.as_tensor(init[n]))

    def spectrum_convolution(self, img, txt):
        """smore.py:209-252 (band-energy diagnostics omitted)."""
        fi = torch.fft.rfft(img, dim=1, norm="ortho")
        ft = torch.fft.rfft(txt, dim=1, norm="ortho")

        def unit(w):
            wc = torch.view_as_complex(w)
            return wc / (torch.abs(wc) + 1e-8)

        n = img.shape[1]
        cv = torch.fft.irfft(fi * unit(self.image_complex_weight), n=n, dim=1, norm="ortho")
        ct = torch.fft.irfft(ft * unit(self.text_complex_weight), n=n, dim=1, norm="ortho")
        cf = torch.fft.irfft(ft * fi * unit(self.fusion_complex_weight), n=n, dim=1, norm="ortho")
        return cv, ct, cf

    def forward(self, train=False):
        """smore.py:256-349 (sparse=True, inject_mode='residual')."""
        cv, ct, cf = self.spectrum_convolution(self.image_trs(self.image_embedding.weight),
                                               self.text_trs(self.text_embedding.weight))
        item_id = self.item_id_embedding.weight
        img_i = item_id + self.inject_scale * self.gate_v(cv)
        txt_i = item_id + self.inject_scale * self.gate_t(ct)
        fus_i = item_id + self.inject_scale * self.gate_f(cf)
        ego = torch.cat([self.user_embedding.weight, item_id], dim=0)
        layers = [ego]
        for _ in range(self.n_ui_layers):
            ego = torch.sparse.mm(self.norm_adj, ego)
            layers.append(ego)
        content = torch.stack(layers, dim=1).mean(dim=1)
        for _ in range(self.n_layers):
            img_i = torch.sparse.mm(self.image_original_adj, img_i)
        image_embeds = torch.cat([torch.sparse.mm(self.R, img_i), img_i], dim=0)
        for _ in range(self.n_layers):
            txt_i = torch.sparse.mm(self.text_original_adj, txt_i)
        text_embeds = torch.cat([torch.sparse.mm(self.R, txt_i), txt_i], dim=0)
        for _ in range(self.n_layers):
            fus_i = torch.sparse.mm(self.fusion_adj, fus_i)
        fusion_embeds = torch.cat([torch.sparse.mm(self.R, fus_i), fus_i], dim=0)
        agg_img = torch.softmax(self.query_v(fusion_embeds), dim=-1) * image_embeds
        agg_txt = torch.softmax(self.query_t(fusion_embeds), dim=-1) * text_embeds
        ip = self.dropout(self.gate_image_prefer(content))
        tp = self.dropout(self.gate_text_prefer(content))
        fp = self.dropout(self.gate_fusion_prefer(content))
        side = torch.mean(torch.stack([ip * agg_img, tp * agg_txt, fp * fusion_embeds]), dim=0)
        all_e = content + side
        u, i = torch.split(all_e, [self.n_users, self.n_items], dim=0)
        if train:
            return u, i, side, content
        return u, i

    @staticmethod
    def info_nce(v1, v2, temp):
        """smore.py:366-373."""
        v1, v2 = F.normalize(v1, dim=1), F.normalize(v2, dim=1)
        pos = torch.exp((v1 * v2).sum(dim=-1) / temp)
        ttl = torch.exp(torch.matmul(v1, v2.transpose(0, 1)) / temp).sum(dim=1)
        return torch.mean(-torch.log(pos / ttl))

    def calculate_loss(self, inter):
        """smore.py:352-364 (bpr_loss) + 375-391."""
        users, pos, neg = inter[0], inter[1], inter[2]
        ua, ia, side, content = self.forward(train=True)
        self.global_step += 1
        u, p, n = ua[users], ia[pos], ia[neg]
        ps, ns = (u * p).sum(dim=1), (u * n).sum(dim=1)
        reg = (0.5 * (u ** 2).sum() + 0.5 * (p ** 2).sum() + 0.5 * (n ** 2).sum()) / self.batch_size
        mf = -torch.mean(F.logsigmoid(ps - ns))
        su, si = torch.split(side, [self.n_users, self.n_items], dim=0)
        cu, ci = torch.split(content, [self.n_users, self.n_items], dim=0)
        cl = self.info_nce(si[pos], ci[pos], self.cl_temp) + self.info_nce(su[users], cu[users], self.cl_temp)
        return mf + self.reg_weight * reg + 0.0 + self.cl_loss * cl


def smore_train_batch(model: SMORECPU, opt, inter, lr, target_rel=1e-3, max_scale=20.0):
    """One batch of Trainer._train_epoch on a model with mg_enable (src/common/trainer.py:
    186-201, 244-336): loss, backward, Adam step, then the model-level mirror gradient
    when global_step % mg_interval == 0.  Returns the batch loss (a float)."""
    opt.zero_grad(set_to_none=True)
    loss = model.calculate_loss(inter)
    value = loss.item()
    loss.backward()
    opt.step()
    if model.global_step % model.mg_interval == 0:
        opt.zero_grad(set_to_none=True)
        model.calculate_loss(inter).backward()
        params, grads = [], []
        for p in model.parameters():
            if p.requires_grad and p.grad is not None:
                params.append(p)
                grads.append(p.grad.detach().clone())
        with torch.no_grad():
            g_all = torch.cat([g.view(-1) for g in grads])
            grad_rms = float(g_all.norm() / (g_all.numel() ** 0.5))
            p_all = torch.cat([p.detach().view(-1) for p in params])
            param_rms = float(p_all.norm() / (p_all.numel() ** 0.5) + 1e-12)
            alpha = max(model.mg_alpha, target_rel * param_rms / (lr * grad_rms + 1e-12))
            alpha = min(alpha, model.mg_alpha * max_scale)
            for p, g in zip(params, grads):
                p.add_(-alpha * lr * g)
        opt.zero_grad(set_to_none=True)
        model.calculate_loss(inter).backward()
        with torch.no_grad():
            for p in model.parameters():
                if p.requires_grad and p.grad is not None:
                    p.grad.mul_(-model.mg_beta)
            for p, g in zip(params, grads):
                p.add_(+alpha * lr * g)
        opt.step()
        opt.zero_grad(set_to_none=True)
    return value


class LayerGCNCPU:
    """Reference-identical CPU LayerGCN training (src/models/layergcn.py:31-177):
    per-epoch edge dropout (`pre_epoch_processing`, :51-70: torch.multinomial on the
    normalised edge values, alternating with random.sample), the cosine-gated
    propagation on the masked graph, BPR-sum + L2 loss, autograd, torch.optim.Adam."""

    def __init__(self, train_u, train_i, n_users, n_items, user_emb, item_emb, K, reg, dropout, lr=1e-3, seed=999):
        import random

        self.rand = random.Random(seed)
        self.n_users, self.n_items, self.K, self.reg, self.dropout = n_users, n_items, K, reg, dropout
        self.norm_adj = lightgcn_norm_adj_vec(np.asarray(train_u), np.asarray(train_i), n_users, n_items)
        self.edge_indices = torch.from_numpy(np.vstack([np.asarray(train_u), np.asarray(train_i)]).astype(np.int64))
        self.edge_values = layergcn_normalize(self.edge_indices, n_users, n_items)
        self.pruning_random = False
        self.masked_adj = self.norm_adj
        self.u = torch.nn.Parameter(torch.from_numpy(np.array(user_emb, dtype=np.float32)))
        self.i = torch.nn.Parameter(torch.from_numpy(np.array(item_emb, dtype=np.float32)))
        self.opt = torch.optim.Adam([self.u, self.i], lr=lr)

    def pre_epoch(self):
        if self.dropout <= 0.0:
            self.masked_adj = self.norm_adj
            return
        n = self.edge_values.size(0)
        keep_len = int(n * (1.0 - self.dropout))
        if self.pruning_random:
            keep = torch.tensor(self.rand.sample(range(n), keep_len))
        else:
            keep = torch.multinomial(self.edge_values, keep_len)
        self.pruning_random = not self.pruning_random
        self.masked_adj = layergcn_masked_adj(self.edge_indices, keep, self.n_users, self.n_items)

    def step(self, trip: torch.Tensor) -> float:
        self.opt.zero_grad()
        loss = layergcn_loss(self.u, self.i, self.masked_adj, self.K, trip, self.reg)
        v = loss.item()
        loss.backward()
        self.opt.step()
        return v


# ---------------------------------------------------------------------------
# full-sort scores as the kernels compute them (oracle/fs_oracle.c, C fmaf chain)
# ---------------------------------------------------------------------------
def fmaf_scores(U: np.ndarray, users: np.ndarray, I: np.ndarray) -> np.ndarray:
    """[len(users), n_items] f32: the fmaf chain over d in order of U[users[b]] . I[i]
    -- the exact score the rsx full-sort ranks by (csrc/fullsort.hip exact_dot), computed
    on the CPU by oracle/fs_oracle.c (src/common/trainer.py:509-528 ranks U I^T)."""
    import ctypes as C
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libfsoracle.so")
    if not os.path.exists(path):
        import subprocess

        os.makedirs(os.path.dirname(path), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fPIC", "-shared", "-o", path,
                        os.path.join(os.path.dirname(path), "..", "fs_oracle.c"), "-lm"], check=True)
    lib = C.CDLL(path)
    U = np.ascontiguousarray(U, dtype=np.float32)
    I = np.ascontiguousarray(I, dtype=np.float32)
    users = np.ascontiguousarray(users, dtype=np.int64)
    out = np.empty((users.size, I.shape[0]), dtype=np.float32)
    P = C.c_void_p
    lib.rsx_oracle_fmaf_scores.argtypes = [P, P, C.c_int64, P, C.c_int64, C.c_int32, P]
    lib.rsx_oracle_fmaf_scores(U.ctypes.data, users.ctypes.data, users.size, I.ctypes.data, I.shape[0],
                               U.shape[1], out.ctypes.data)
    return out
