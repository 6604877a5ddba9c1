"""SMORE on the rsx HIP path — drop-in for the reference's models/smore.py (WSDM'25).

Same class name, constructor, YAML keys, module names and creation order (so
`init_seed` gives the reference's initial weights), forward and loss
(reference src/models/smore.py:24-449):

* UI backbone: n_ui_layers propagations of the float32 sym-normalised graph,
  mean over layers — the HIP propagation (rsx_lightgcn_forward machinery) with
  autograd whose backward is the same operator (the graph is symmetric);
* item-item views (image / text kNN graphs and their max-pooled fusion, built
  once like the reference and cached next to the data) and the item -> user
  aggregation R — HIP SpMM with autograd (backward = SpMM with the transposed
  CSR, the kNN graphs are not symmetric);
* projection + spectral denoise / fusion (smore.py:209-252,256-272) — the fused
  HIP pass rsx_smore_spectral (forward and backward, see csrc/smore.hip);
* BPR part of the loss — the fused HIP BPR kernel (variant SMORE);
* gates + inject, the item views' propagation into [R x; x], the preference
  block (query MLPs, softmax over d, dropout'd preference gates, mean, content +
  side) and both InfoNCE terms — fused HIP kernels with autograd (rsx.smore_fuse,
  csrc/smore_fuse.hip).

The kernels are instantiated for embedding_size 64 and 128 (the SMORE.yaml default
and C5's CLIP width) with both modalities present and feature widths that are
multiples of 32; any other shape raises RuntimeError (RSX_ERR_UNSUPPORTED) at
construction: there is no torch fallback on this path.

Diagnostics that the reference gathers with per-step `.item()` calls
(spectrum band energies, gate statistics, CL values) are computed lazily, only
when `log_mm_diagnostics` runs, so training issues no per-step host syncs.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from . import graph, ops
from .lightgcn import _BprLoss
from . import smore_fuse as SF
from .nn import RsxLinear
from .recommender import GeneralRecommender


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, A, AT):
        ctx.AT = AT
        return A.spmm(x.contiguous())

    @staticmethod
    def backward(ctx, g):
        return ctx.AT.spmm(g.contiguous()), None, None


def _prop_mean(A, x, K):
    import ctypes as C

    x = x.contiguous()
    out = torch.empty_like(x)
    s, h0, h1 = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    d = x.shape[1]
    rc = L.lib().rsx_lightgcn_forward(C.byref(A.struct), d, K, ops._p(x), ops._p(s), ops._p(h0), ops._p(h1),
                                      ops._p(out), ops._p(A.slab(d)), ops._stream())
    L.check(rc, "rsx_lightgcn_forward")
    return out


class _PropMean(torch.autograd.Function):
    """mean_{k=0..K} A^k x for a symmetric A (backward: the same operator)."""

    @staticmethod
    def forward(ctx, x, A, K):
        ctx.A, ctx.K = A, K
        return _prop_mean(A, x, K)

    @staticmethod
    def backward(ctx, g):
        return _prop_mean(ctx.A, g, ctx.K), None, None


class _Joined(torch.autograd.Function):
    """torch.cat([U, I]) without the copy when U and I are adjacent row blocks of one
    buffer (SMORE keeps its user and item-id tables so: rsx.smore.SMORE.__init__): the
    output aliases their storage (a new tensor, not an autograd view of either input);
    backward: the two row blocks of the gradient, as cat's."""

    @staticmethod
    def forward(ctx, u, i):
        ctx.nu = u.shape[0]
        out = torch.empty(0, dtype=u.dtype, device=u.device)
        out.set_(u.untyped_storage(), u.storage_offset(), (u.shape[0] + i.shape[0], u.shape[1]), (u.shape[1], 1))
        return out

    @staticmethod
    def backward(ctx, g):
        return g[: ctx.nu], g[ctx.nu:]


def _ego(u: torch.Tensor, i: torch.Tensor) -> torch.Tensor:
    """[U; I] (the reference's torch.cat([user_embeds, item_embeds]), smore.py:278)."""
    adjacent = (u.device == i.device and u.dtype == i.dtype and u.is_contiguous() and i.is_contiguous()
                and u.dim() == 2 and i.dim() == 2 and u.shape[1] == i.shape[1]
                and u.untyped_storage().data_ptr() == i.untyped_storage().data_ptr()
                and i.storage_offset() == u.storage_offset() + u.numel())
    return _Joined.apply(u, i) if adjacent else torch.cat([u, i], dim=0)


class _RowTags:
    """Batch-row tags for the tagged propagation: row r is in the batch when
    row_tag[r] == *tag_dev; `mark` bumps the device tag and tags the batch's rows
    (one launch, rsx_tag_rows_next; no host sync: graph-capture safe).  tag_dev is
    {tag, ticket}: the products read word 0."""

    def __init__(self, n: int, device):
        self.row_tag = torch.zeros(n, dtype=torch.int32, device=device)
        self.tag_dev = torch.zeros(2, dtype=torch.int32, device=device)

    def mark(self, rows: torch.Tensor):
        rows = rows.to(torch.int64).contiguous()
        L.check(L.lib().rsx_tag_rows_next(ops._p(self.row_tag), ops._p(rows), rows.numel(), ops._p(self.tag_dev),
                                          ops._stream()), "rsx_tag_rows_next")


class _PropMeanRows(torch.autograd.Function):
    """mean_{k=0..K} A^k x for a symmetric A, needed at the tagged rows only (K <= 4;
    the batch rows of the SMORE training loss): E^1..E^{K-1} stored (no running sum),
    the last layer and the mean on the tagged rows only, in the running sum's order
    (((E0 + E1) + E2) + E3) + A E3 (other rows of the output are left unwritten).  The
    backward is Horner on the incoming gradient G, which is zero off the tagged rows
    (`rows`: the forward's rows, re-tagged in the backward, so several forwards may run
    before their backwards, as in a sum of batch losses):
    H = G + A H from H = G, the first layer gathering only the tagged rows of G, every
    layer reading G on the tagged rows only, the last scaled by 1/(K+1) (the dense
    path's arithmetic: the same mean operator applied to G)."""

    @staticmethod
    def forward(ctx, x, A, K, tags, rows=None):
        x = x.contiguous()
        n, d = x.shape
        out = torch.empty_like(x)
        hs = torch.empty(max(K - 1, 1), n, d, dtype=torch.float32, device=x.device)
        cur = x
        for k in range(1, K):
            A.spmm_epi(cur, ops.epi(L.RSX_EPI_STORE, y=hs[k - 1]), d)
            cur = hs[k - 1]
        stored = dict(zip(("s_in", "r_add", "aux", "e0"), [x] + [hs[i] for i in range(K - 1)]))
        e = ops.epi(L.RSX_EPI_FINAL, beta=1.0 / (K + 1), f=out, row_tag=tags.row_tag, tag_dev=tags.tag_dev, **stored)
        e.tag_flags = L.RSX_TAG_ROWS
        A.spmm_epi(cur, e, d)
        ctx.A, ctx.K, ctx.tags, ctx.rows = A, K, tags, rows
        return out

    @staticmethod
    def backward(ctx, g):
        A, K, tags = ctx.A, ctx.K, ctx.tags
        if ctx.rows is not None:
            # re-tag this forward's rows: a later forward (another calculate_loss before this
            # backward) may have moved the tag on, and G is zero off exactly these rows
            tags.mark(ctx.rows)
        g = g.contiguous()
        d = g.shape[1]
        bufs = torch.empty(2, *g.shape, dtype=torch.float32, device=g.device)
        h = g
        for k in range(1, K + 1):
            y = bufs[k & 1]
            e = ops.epi(L.RSX_EPI_ADD, beta=1.0 / (K + 1) if k == K else 1.0, y=y, s_in=g, row_tag=tags.row_tag,
                        tag_dev=tags.tag_dev)
            e.tag_flags = L.RSX_TAG_SPARSE_S | (L.RSX_TAG_SPARSE_X if k == 1 else 0)
            A.spmm_epi(h, e, d)
            h = y
        return h, None, None, None, None


def knn_graph(feat: np.ndarray, k: int):
    """build_sim + build_knn_normalized_graph(sparse, 'sym') (src/utils/utils.py:134-181) on the CPU,
    float32 as the reference: cosine similarities, top-k per row, deg = sum of kept values,
    w = d_r^-1/2 * s * d_c^-1/2.  Returns (rows, cols, vals)."""
    x = torch.from_numpy(feat)
    xn = x.div(torch.norm(x, p=2, dim=-1, keepdim=True))
    n = xn.shape[0]
    rows, cols, vals = [], [], []
    step = max(1, (1 << 26) // max(n, 1))
    for s in range(0, n, step):
        sim = torch.mm(xn[s:s + step], xn.t())
        v, i = torch.topk(sim, k, dim=-1)
        rows.append(torch.arange(s, s + sim.shape[0]).repeat_interleave(k))
        cols.append(i.reshape(-1))
        vals.append(v.reshape(-1))
    r, c, v = torch.cat(rows), torch.cat(cols), torch.cat(vals)
    deg = torch.zeros(n, dtype=v.dtype).index_add_(0, r, v)
    dis = deg.pow_(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    w = dis[r] * v * dis[c]
    return r.numpy().astype(np.int64), c.numpy().astype(np.int64), w.numpy().astype(np.float32)


def knn_graph_device(feat: torch.Tensor, k: int):
    """build_sim + build_knn_normalized_graph(sparse, 'sym') on the device through the
    hand-written builder rsx_knn_graph (csrc/knn.hip: row normalisation, the cosine
    similarities on f32 MFMA with the per-row top-k kept in registers — the n x n
    matrix is never formed — and the sym-norm in the reference's order: deg = the
    row's kept values added in rank order, 1/sqrt(deg), (d_r * v) * d_c).  The
    similarities are f32 MFMA sums, so values can differ from the CPU build in the
    last bits and neighbours at exact near-ties can swap (tests/test_gpu_smore.py
    pins that).  Returns host (rows, cols, vals) like knn_graph."""
    import ctypes as C

    x = feat.detach().to(torch.float32).contiguous()
    n, f = x.shape
    if k > 32 or k > n:
        raise ValueError(f"rsx_knn_graph: k = {k} (supported: k <= 32 and k <= n = {n})")
    lib = L.lib()
    v = torch.empty(n, k, dtype=torch.float32, device=x.device)
    i = torch.empty(n, k, dtype=torch.int64, device=x.device)
    w = torch.empty(n, k, dtype=torch.float32, device=x.device)
    ws = torch.empty(max(int(lib.rsx_knn_ws_bytes(n, f)), 4), dtype=torch.uint8, device=x.device)
    L.check(lib.rsx_knn_graph(ops._p(x), n, f, k, ops._p(v), ops._p(i), ops._p(w), ops._p(ws), ws.numel(),
                              ops._stream()), "rsx_knn_graph")
    r = np.repeat(np.arange(n, dtype=np.int64), k)
    return r, i.reshape(-1).cpu().numpy().astype(np.int64), w.reshape(-1).cpu().numpy().astype(np.float32)


def load_reference_knn(path: str, n: int):
    """The reference's own kNN cache (smore.py:46-47,56-62: `torch.save` of the
    sparse [n, n] graph as `{image,text}_adj_{k}_{sparse}.pt` in the dataset
    directory), read with the loader that executes nothing from the file
    (`weights_only=True`).  Returns (rows, cols, vals) in coalesced order, or None
    when the file is absent, refused by the safe loader or not an [n, n] graph."""
    if not os.path.exists(path):
        return None
    try:
        t = torch.load(path, map_location="cpu", weights_only=True)
    except Exception:  # noqa: BLE001 - a file the safe loader refuses is rebuilt, not trusted
        return None
    if not isinstance(t, torch.Tensor) or t.dim() != 2 or tuple(t.shape) != (n, n):
        return None
    if t.layout == torch.sparse_coo:
        t = t.coalesce()
        idx, val = t.indices(), t.values()
    elif t.layout == torch.strided:  # is_sparse False: build_knn_normalized_graph's dense matrix
        idx = t.nonzero().t()
        val = t[idx[0], idx[1]]
    else:
        return None
    return (idx[0].numpy().astype(np.int64), idx[1].numpy().astype(np.int64),
            val.to(torch.float32).numpy().astype(np.float32))


def max_pool_union(a, b, n):
    """Elementwise max over the union of two edge sets (smore.py:153-174)."""
    ka = a[0] * n + a[1]
    kb = b[0] * n + b[1]
    keys = np.concatenate([ka, kb])
    vals = np.concatenate([a[2], b[2]])
    # coalesce duplicates inside each graph first (values are unique per (r,c) already)
    order = np.argsort(keys, kind="stable")
    keys, vals = keys[order], vals[order]
    uk, start = np.unique(keys, return_index=True)
    mx = np.maximum.reduceat(vals, start)
    return (uk // n).astype(np.int64), (uk % n).astype(np.int64), mx.astype(np.float32)


class _DevGraph:
    """A sparse operator with its transpose on the device (forward / backward SpMM)."""

    def __init__(self, rows, cols, vals, n_rows, n_cols, device, chunk):
        self.A = ops.DeviceCSR(*graph.to_csr(rows, cols, vals, n_rows, n_cols), n_cols, device, chunk)
        self.AT = ops.DeviceCSR(*graph.to_csr(cols, rows, vals, n_cols, n_rows), n_rows, device, chunk)

    def __call__(self, x):
        return _SpMM.apply(x, self.A, self.AT)


def spectrum_torch(img, txt, wv, wt, wf, normalize=True):
    """Reference spectrum_convolution (smore.py:209-237) with torch.fft: the fp32
    statement the tests check the HIP pass against (not called by the model)."""
    d = img.shape[1]
    fi = torch.fft.rfft(img, dim=1, norm="ortho")
    ft = torch.fft.rfft(txt, dim=1, norm="ortho")
    cw = [torch.view_as_complex(w) for w in (wv, wt, wf)]
    if normalize:
        cw = [w / (torch.abs(w) + 1e-8) for w in cw]
    cv = torch.fft.irfft(fi * cw[0], n=d, dim=1, norm="ortho")
    ct = torch.fft.irfft(ft * cw[1], n=d, dim=1, norm="ortho")
    cf = torch.fft.irfft(ft * fi * cw[2], n=d, dim=1, norm="ortho")
    return cv, ct, cf


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _require_supported(d, v_feat, t_feat):
    """The shapes the SMORE kernels are instantiated for; anything else is refused
    (RSX_ERR_UNSUPPORTED) rather than run on torch ops."""
    from .smore_spectral import spectral_supported

    if v_feat is None or t_feat is None:
        raise RuntimeError("RSX_ERR_UNSUPPORTED: rsx SMORE needs both the image and the text features")
    dv, dt = int(v_feat.shape[1]), int(t_feat.shape[1])
    if not (SF.supported(d) and spectral_supported(d, dv, dt)):
        raise RuntimeError(f"RSX_ERR_UNSUPPORTED: rsx SMORE kernels are built for embedding_size 64 / 128 and "
                           f"feature widths that are multiples of 32 (got d={d}, image {dv}, text {dt})")


class SMORE(GeneralRecommender):
    # a training batch has no host syncs and global_step advances once per
    # calculate_loss: the Trainer may capture it in a HIP graph (rsx.trainer._GraphStep)
    supports_graph_step = True
    # no per-epoch buffer rebuilds (pre_epoch_processing is a no-op): the captured
    # steps stay valid across epochs
    graph_step_persistent = True

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        ops.require_device(self.device)
        self.sparse = True
        self.cl_loss = config["cl_loss"]
        self.n_ui_layers = config["n_ui_layers"]
        self.embedding_dim = config["embedding_size"]
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        self.image_knn_k = config["image_knn_k"]
        self.text_knn_k = config["text_knn_k"]
        self.dropout_rate = config["dropout_rate"]
        self.dropout = nn.Dropout(p=self.dropout_rate)
        chunk = int(config["rsx_chunk"] or 32)
        d = self.embedding_dim
        self.interaction_matrix = dataset.inter_matrix(form="coo").astype(np.float32)
        # parameters in the reference's creation order (identical init under init_seed)
        self.user_embedding = nn.Embedding(self.n_users, d)
        self.item_id_embedding = nn.Embedding(self.n_items, d)
        nn.init.xavier_uniform_(self.user_embedding.weight)
        nn.init.xavier_uniform_(self.item_id_embedding.weight)
        nu, ni = self.n_users, self.n_items
        if torch.device(self.device).type == "cuda":
            # the two tables as adjacent row blocks of one device buffer (drawn on the CPU as
            # the reference does, then copied): the UI backbone's ego table [U; I] is that
            # buffer itself (_ego), no per-forward concatenation copy
            joint = torch.empty(nu + ni, d, dtype=torch.float32, device=self.device)
            joint[:nu].copy_(self.user_embedding.weight.detach())
            joint[nu:].copy_(self.item_id_embedding.weight.detach())
            self.user_embedding.weight = nn.Parameter(joint[:nu])
            self.item_id_embedding.weight = nn.Parameter(joint[nu:])
        im = self.interaction_matrix
        if os.environ.get("RSX_GRAPH_BUILDER", "device") == "host":
            rp, col, val = graph.smore_norm_adj(im.row.astype(np.int64), im.col.astype(np.int64), nu, ni)
            self.norm_adj_csr = ops.DeviceCSR(rp, col, val, nu + ni, self.device, chunk)
        else:  # rsx_adj_build (csrc/graph.hip), bit-equal to graph.smore_norm_adj
            drp, dcol, dval = ops.adj_build(im.row.astype(np.int64), im.col.astype(np.int64), nu, ni,
                                            ops.ADJ_SMORE, self.device)
            self.norm_adj_csr = ops.DeviceCSR.from_device(drp, dcol, dval, nu + ni, chunk)
            rp, col, val = self.norm_adj_csr.rowptr_host, dcol.cpu().numpy(), dval.cpu().numpy()
        # the item views' graphs (kNN graphs and R) in 64-wide work items: a kNN row (k <= ~40
        # in the fusion union) or a user's R row is one item; R^T's popular items split in
        # half as many chunks (C5 5.89 -> 5.77 ms/step, C3 3.05 -> 2.94 against 32)
        kchunk = int(config["rsx_knn_chunk"] or 64)
        # R = the user rows' item block (users first: rows [0, nu), item columns rebased)
        e = int(rp[nu])
        rows = np.repeat(np.arange(nu), np.diff(rp[: nu + 1]))
        self.R = _DevGraph(rows, col[:e].astype(np.int64) - nu, val[:e], nu, ni, self.device, kchunk)
        root = os.path.abspath((config["data_path"] or "") + (config["dataset"] or ""))
        self.knn_mode = config["rsx_knn"] or config["rsx_sampler"] or "device"
        if self.knn_mode not in ("device", "host"):
            raise ValueError(f"rsx_knn must be 'device' or 'host', got {self.knn_mode!r}")
        img_g = txt_g = None
        if self.v_feat is not None:
            self.image_embedding = nn.Embedding.from_pretrained(self.v_feat.clone(), freeze=False)
            img_g = self._cached_knn(root, "image", self.v_feat, self.image_knn_k)
        if self.t_feat is not None:
            self.text_embedding = nn.Embedding.from_pretrained(self.t_feat.clone(), freeze=False)
            txt_g = self._cached_knn(root, "text", self.t_feat, self.text_knn_k)
        self.image_graph = _DevGraph(*img_g, ni, ni, self.device, kchunk)
        self.text_graph = _DevGraph(*txt_g, ni, ni, self.device, kchunk)
        self.fusion_graph = _DevGraph(*max_pool_union(img_g, txt_g, ni), ni, ni, self.device, kchunk)
        if self.v_feat is not None:
            self.image_trs = nn.Linear(self.v_feat.shape[1], d)
        if self.t_feat is not None:
            self.text_trs = nn.Linear(self.t_feat.shape[1], d)
        self.softmax = nn.Softmax(dim=-1)
        self.query_v = nn.Sequential(RsxLinear(d, d), nn.Tanh(), RsxLinear(d, d, bias=False))
        self.query_t = nn.Sequential(RsxLinear(d, d), nn.Tanh(), RsxLinear(d, d, bias=False))
        self.gate_v = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.gate_t = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.gate_f = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.gate_image_prefer = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.gate_text_prefer = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.gate_fusion_prefer = nn.Sequential(RsxLinear(d, d), nn.Sigmoid())
        self.image_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.text_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.fusion_complex_weight = nn.Parameter(torch.randn(1, d // 2 + 1, 2, dtype=torch.float32))
        self.mg_enable = bool(config.get("mg_enable", True))
        self.mg_interval = int(config.get("mg_interval", 3))
        self.mg_alpha = float(config.get("mg_alpha", 0.5))
        self.mg_beta = float(config.get("mg_beta", 0.2))
        self.mg_verbose = bool(config.get("mg_verbose", True))
        self.global_step = 0
        self.inject_mode = config.get("inject_mode", "residual")
        self.inject_scale = float(config.get("inject_scale", 0.7))
        self.spectral_weight_norm = bool(config.get("spectral_weight_norm", True))
        self.cl_temp = float(config.get("cl_temp", 0.2))
        self.diag_spectrum = bool(config.get("diag_spectrum", True))
        self.diag_gate = bool(config.get("diag_gate", True))
        self.diag_grad = bool(config.get("diag_grad", True))
        _require_supported(d, self.v_feat, self.t_feat)
        # training loss on the batch rows only (rsx_smore_batch_rows: False = full tables)
        self.batch_rows = bool(config.get("rsx_smore_batch_rows", True))
        self._bidx = {}
        self._rows_off = {}
        self._tags = None
        self._vtags = None  # the views' backward batch-row tags (rsx.smore_fuse._ViewProp3)
        self.batch_views = bool(config.get("rsx_smore_batch_views", True))
        # the item side (projections, spectral part, gates) as one launch (rsx_smore_item_fwd)
        # instead of the three-launch chain (same values, bit for bit).  Off by default: it
        # measured slower (C5 235 vs 209 us, C3 111 vs 77: tools/gpu/micro_item.py)
        self.item_fused = bool(config.get("rsx_smore_item_fused", False))
        # dropout masks of the fused preference block: a hash of (seed, call, row,
        # feature); the seed word lives on the device and advances once per training
        # forward (graph-capture safe).  Derived from the config seed, not torch's RNG,
        # so the parameter initialisation stream matches the reference.
        self._drop_seed = torch.tensor([int(config["seed"] or 999) * 1000003 + 17], dtype=torch.int64,
                                       device=self.device)
        self._last = {}
        self.to(self.device)
        from .lightgcn import _world

        world, rank = _world()
        flag = config["rsx_sharded"]  # None: shard whenever the process group has > 1 rank
        self.sharded = bool(flag) if flag is not None else world > 1
        # multi-rank scheme: "dp" (default; every table replicated, each rank its own batch, one
        # batch-row gradient exchange per backward: rsx.smore_dist.RowGradExchange) or
        # "usershard" (users row-sharded, the item partials all-reduced per UI layer: SmoreShard)
        self.scheme = str(config.get("rsx_smore_scheme") or "dp") if self.sharded else None
        if self.scheme not in (None, "dp", "usershard"):
            raise ValueError(f"rsx_smore_scheme must be 'dp' or 'usershard', got {self.scheme!r}")
        self._exch = None
        if self.scheme == "usershard":
            self._init_sharded(config, rp, col, val, (rows, col[:e].astype(np.int64) - nu, val[:e]), world, rank)
        elif self.scheme == "dp":
            self._init_dp(config, world)

    def _epoch_slices(self, config, sel, world):
        """(steps per epoch, this rank's largest slice) for a rank holding the `sel`
        interactions: every rank cuts its epoch into the same number of balanced slices
        (each interaction visited once); a rank with fewer interactions than steps is
        refused on every rank alike."""
        import torch.distributed as dist

        e_r = int(sel.sum())
        B = int(config["train_batch_size"])
        # the global count in int64 (an f32 sum is exact only to 2^24 interactions)
        group = dist.is_available() and dist.is_initialized()
        cdev = self.device if group and dist.get_backend() == "nccl" else torch.device("cpu")
        stats = torch.tensor([e_r, -e_r], dtype=torch.int64, device=cdev)
        tot = stats[:1].clone()
        if group:
            dist.all_reduce(tot)
        steps = max(1, -(-int(tot.item()) // (world * B)))
        if group:
            dist.all_reduce(stats, op=dist.ReduceOp.MAX)  # [max E_r, -min E_r]
        if -int(stats[1].item()) < steps:
            raise RuntimeError(f"sharded SMORE: a rank holds {-int(stats[1].item())} training interactions, fewer than "
                               f"the {steps} steps per epoch (world {world}, batch {B}); use fewer ranks")
        return steps, -(-e_r // steps)

    def _init_dp(self, config, world):
        """Data-parallel SMORE: every table replicated on every rank (the
        reference's initial weights, drawn identically under init_seed); rank r trains on
        its own batches of the interactions of its user block [a_r, b_r) (global ids, so
        the single-process loss path runs unchanged); the objective is the sum over ranks
        of the reference loss of each rank's batch.  The preference block's backward
        exchanges the batch-row table gradients and its weights' gradients once
        (RowGradExchange); everything after it is identical on every rank."""
        import torch.distributed as dist

        from .smore_dist import Comm, RowGradExchange, ranges

        nu, ni = self.n_users, self.n_items
        self.comm = Comm(None, self.device)
        W, r = self.comm.world, self.comm.rank
        a, b = ranges(nu, W)[r]
        self.user_range = (a, b)
        im = self.interaction_matrix
        rows, cols = im.row.astype(np.int64), im.col.astype(np.int64)
        sel = (rows >= a) & (rows < b)
        self.steps_per_epoch, self.local_batch = self._epoch_slices(config, sel, world)
        self._sampler = ops.DeviceSampler(rows[sel], cols[sel], nu, self.device, seed=int(config["seed"] or 0) + r)
        # negatives from the whole training-item list, as the reference's sampler draws them
        self._sampler.all_items = torch.from_numpy(np.unique(cols).astype(np.int32)).to(self.device)
        self._epoch_buf = None
        self._epoch_of_buf = None
        self._gate_buf = torch.zeros(1, dtype=torch.float32, device=self.device)
        lb = torch.tensor([self.local_batch], dtype=torch.int64,
                          device=self.device if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu")
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(lb, op=dist.ReduceOp.MAX)
        self._exch = RowGradExchange(self.comm, nu + ni, self.embedding_dim, 3 * int(lb.item()), self.device)
        # the step's collectives are captured with it only over RCCL (a gloo group's are host calls)
        self.supports_graph_step = self.comm.native

    def _init_sharded(self, config, rp, col, val, r_coo, world, rank):
        """Users sharded over the process group, the item side replicated (rsx.smore_dist):
        this rank keeps its rows of the user table (drawn in full first, so every rank
        holds the reference's initial weights), its rows of the UI graph and of R, and
        samples its own users' interactions on the device."""
        from .smore_dist import Comm, HipSmoreBackend, SmoreShard

        nu, ni = self.n_users, self.n_items
        self.comm = Comm(None, self.device)
        graphs = {"norm_adj": (np.asarray(rp), np.asarray(col), np.asarray(val)),
                  "R": graph.to_csr(r_coo[0], r_coo[1], r_coo[2], nu, ni),
                  "image": self.image_graph, "text": self.text_graph, "fusion": self.fusion_graph}
        # the item side sharded by item rows too (projection, spectral fusion, the gates'
        # inject term; the raw feature tables row-sharded): residual inject mode only (its
        # inject term is row-local and additive); rsx_smore_item_shard: False replicates it
        flag = config.get("rsx_smore_item_shard", True)
        item_shard = bool(flag if flag is not None else True) and self.inject_mode != "mul"
        self._shard = SmoreShard(graphs, nu, ni, self.n_ui_layers, self.n_layers,
                                 HipSmoreBackend(self.device, int(config["rsx_chunk"] or 32)), self.comm,
                                 item_shard=item_shard)
        a, b = self._shard.own_u
        self.user_range = (a, b)
        w = self.user_embedding.weight.detach()[a:b].clone()
        self.user_embedding = nn.Embedding(b - a, self.embedding_dim, _weight=w, device=self.device)
        if self._shard.item_shard:  # this rank's rows of the raw feature tables
            ia, ib = self._shard.own_i
            self.image_embedding = nn.Embedding.from_pretrained(
                self.image_embedding.weight.detach()[ia:ib].clone(), freeze=False)
            self.text_embedding = nn.Embedding.from_pretrained(
                self.text_embedding.weight.detach()[ia:ib].clone(), freeze=False)
        # the step's collectives are captured with it only over RCCL (a gloo group's are host calls)
        self.supports_graph_step = self.comm.native
        # this rank's interactions, visited once per epoch in the common step count
        im = self.interaction_matrix
        rows, cols = im.row.astype(np.int64), im.col.astype(np.int64)
        sel = (rows >= a) & (rows < b)
        self.steps_per_epoch, self.local_batch = self._epoch_slices(config, sel, world)
        self._sampler = ops.DeviceSampler(rows[sel] - a, cols[sel], b - a, self.device,
                                          seed=int(config["seed"] or 0) + rank)
        self._epoch_buf = None
        self._epoch_of_buf = None
        self._gate_buf = torch.zeros(1, dtype=torch.float32, device=self.device)

    def _side_stream(self):
        """The UI backbone's stream (one per model), or None (RSX_SMORE_STREAMS=0).  None as
        well for a multi-rank model over an rsx communicator: its captured step, with the
        UI backbone's branch and the exchange's comm-stream branch beside the main stream,
        replayed at 9.2 ms a C5 step (latency-injected, W = 4) where the same step without
        the side branch takes 6.1 and eagerly issued 6.2 (profiles/r06/c5_dp/diag)."""
        if os.environ.get("RSX_SMORE_STREAMS", "1") == "0":
            return None
        if self.sharded and getattr(getattr(self, "comm", None), "native", False):
            return None
        st = getattr(self, "_ui_stream", None)
        if st is None:
            st = self._ui_stream = torch.cuda.Stream(device=self.device)
        return st

    def local_batches(self, epoch: int):
        """This rank's training batches of `epoch` (device-sampled [3, B_j] triplets; users
        as local row ids under "usershard", global ids under "dp"; items global):
        steps_per_epoch balanced slices of its epoch on every rank (sizes differ by at
        most one), each interaction visited once."""
        S = self.steps_per_epoch
        if self._epoch_of_buf != epoch:
            self._epoch_buf = self._sampler.sample_epoch_slices(epoch, S, out=self._epoch_buf)
            self._epoch_of_buf = epoch
        for j in range(S):
            yield ops.DeviceSampler.slice_view(self._epoch_buf, self._sampler.n_inter, S, j)

    def gate_loss(self, loss):
        """The NaN gate's input on a sharded model: the loss summed over the ranks, so a NaN
        batch on any rank stops every rank's updates (the replicas stay equal)."""
        if not self.sharded:
            return loss
        self._gate_buf.copy_(loss.detach().reshape(1))
        return self.comm.allreduce_(self._gate_buf)

    def mg_alpha_global(self, params, grads, base, lr, rel_step, max_scale, lr_dev=None):
        """The mirror gradient's alpha over the global parameter vector (sharded model).
        "dp": every rank holds the whole vector and the same summed gradient, so the
        single-process reduction already is the global one (no exchange)."""
        if self.scheme == "dp":
            return SF.mg_alpha(params, grads, base, lr, rel_step, max_scale, lr_dev)
        return self._shard.mg_alpha(self, params, grads, base, lr, rel_step, max_scale, lr_dev)

    def full_sort_topk_local(self, eval_users, k: int, eval_data):
        """(positions in eval_users of this rank's users, their top-k item ids)."""
        if self.scheme == "dp":  # the replicated tables: this rank ranks its user block's share
            a, b = self.user_range
            pos = torch.nonzero((eval_users >= a) & (eval_users < b)).flatten()
            users = eval_users.index_select(0, pos).contiguous()
            _, topk = self.full_sort_topk([users], k, eval_data)
            return pos, topk
        return self._shard.full_sort_topk_local(self, self._drop_seed, eval_users, k, eval_data.mask_rowptr,
                                                eval_data.mask_col)

    # ---------------------------------------------------------------- graphs
    def _cached_knn(self, root, name, feat, k):
        """kNN item graph (reference smore.py:45-75): the reference's own
        {name}_adj_{k}_{sparse}.pt cache when the dataset directory holds one, else
        built on the device (knn_graph_device) or, with rsx_knn: host (the default when
        rsx_sampler is host), by the CPU restatement of the reference's build."""
        # a cache the reference wrote for this dataset is the graph its runs trained on: use it
        ref = load_reference_knn(os.path.join(root, f"{name}_adj_{k}_{self.sparse}.pt"), feat.shape[0])
        if ref is not None:
            return ref
        device_build = self.knn_mode == "device"
        path = os.path.join(root, f"rsx_{name}_knn_{k}{'_dev' if device_build else ''}.npz")
        f = feat.detach().cpu().numpy()
        sig = np.array([f.shape[0], f.shape[1], float(np.float64(f[:4].sum())), float(np.float64(f[-4:].sum()))])
        if os.path.exists(path):
            try:
                z = np.load(path)
                if np.array_equal(z["sig"], sig):
                    return z["r"], z["c"], z["v"]
            except (OSError, ValueError, KeyError, EOFError):  # another rank still writing it: rebuild
                pass
        r, c, v = knn_graph_device(feat.detach().to(self.device), k) if device_build else knn_graph(f, k)
        from .lightgcn import _world

        if _world()[1] == 0:  # one writer per job (every rank builds the same graph)
            try:
                os.makedirs(root, exist_ok=True)
                tmp = f"{path}.{os.getpid()}.tmp.npz"
                np.savez(tmp, r=r, c=c, v=v, sig=sig)
                os.replace(tmp, path)
            except OSError:
                pass
        return r, c, v

    # --------------------------------------------------------------- forward
    def spectrum_convolution(self, image_embeds, text_embeds):
        """Reference API (smore.py:209-237) on already projected tables: the fused HIP
        pass with an identity projection (x I + 0 is exact in f32)."""
        from .smore_spectral import spectral

        d = self.embedding_dim
        eye = torch.eye(d, device=image_embeds.device, dtype=torch.float32)
        zero = torch.zeros(d, device=image_embeds.device, dtype=torch.float32)
        cv, ct, cf, _, _ = spectral(image_embeds, eye, zero, text_embeds, eye, zero, self.image_complex_weight,
                                    self.text_complex_weight, self.fusion_complex_weight, self.spectral_weight_norm)
        self._last["spec_in"] = (image_embeds.detach(), text_embeds.detach())
        return cv, ct, cf

    def _projected_spectrum(self):
        from .smore_spectral import spectral_fused

        return spectral_fused(self)

    def forward(self, adj=None, train=False):
        """Reference signature: (users, items) or, with train=True, (users, items, side, content)."""
        all_embeds, side, content = self._forward_all(train)
        users, items = torch.split(all_embeds, [self.n_users, self.n_items], dim=0)
        if train:
            return users, items, side, content
        return users, items

    def _forward_all(self, train=False):
        return self._forward_all_fused(train)

    def _sparse_rows(self, rows) -> bool:
        """The batch-row path with tag-aware consumers of the preference block's table
        gradients (the UI backbone's _PropMeanRows, the views' _ViewProp3)."""
        return rows is not None and 1 <= self.n_ui_layers <= 4 and self.batch_views

    def _views_fused(self, train=False, rows=None, bw_rows=None):
        """Everything before the preference block: (content, image, text, fusion tables,
        dropout seed).  With `rows` (the batch rows) content is exact on those rows only.

        The UI backbone (content) does not depend on the item side (projection, spectral
        fusion, gates) before the views meet it in the preference block, so it runs on a
        side stream concurrently with it; its backward then runs on that stream too
        (autograd keeps each op's backward on its forward's stream), overlapping the
        item side's backward.  Both are latency-bound chains of mid-size launches, and
        in a captured step the two streams become parallel branches of the HIP graph.
        RSX_SMORE_STREAMS=0 keeps everything on one stream.  `bw_rows`: the rows the
        backward's incoming gradients are defined on, when they are not `rows` (data-parallel
        SMORE: the union of the ranks' batch rows, filled in by the exchange)."""
        bw = bw_rows if bw_rows is not None else rows
        # the leaves enter the graph through views made on THIS stream, so every leaf has one
        # consumer on one stream: its AccumulateGrad runs on the stream of the node that
        # produces its gradient (a leaf read on both streams had its accumulator bound to
        # the side stream while the gates' backward fed it from this one: torch's
        # AccumulateGrad stream-mismatch warning, and a cross-stream sync per backward)
        item_id = self.item_id_embedding.weight.view_as(self.item_id_embedding.weight)
        user_w = self.user_embedding.weight.view_as(self.user_embedding.weight)
        main = torch.cuda.current_stream()
        side = self._side_stream()
        if side is not None:
            side.wait_stream(main)
            if rows is not None:
                rows.record_stream(side)  # made on this stream, read on the side stream (also in the backward)
        with torch.cuda.stream(side) if side is not None else _nullctx():
            ego = _ego(user_w, item_id)
            if rows is not None and 1 <= self.n_ui_layers <= 4:
                if self._tags is None:
                    self._tags = _RowTags(self.n_users + self.n_items, self.device)
                self._tags.mark(rows)
                content = _PropMeanRows.apply(ego, self.norm_adj_csr, self.n_ui_layers, self._tags, bw)
            else:
                content = _PropMean.apply(ego, self.norm_adj_csr, self.n_ui_layers)
        if self.item_fused and type(self)._projected_spectrum is SMORE._projected_spectrum:
            from .smore_spectral import item_side_fused

            (img_i, txt_i, fus_i), (cv, ct, cf) = item_side_fused(self, item_id)
        else:
            cv, ct, cf = self._projected_spectrum()
            img_i, txt_i, fus_i = SF.gates(cv, ct, cf, item_id, self.gate_v, self.gate_t, self.gate_f,
                                           self.inject_scale, self.inject_mode == "mul")
        if side is not None:
            main.wait_stream(side)
            content.record_stream(main)  # allocated on the side stream, read on this one
        nu, L_ = self.n_users, self.n_layers
        if self.batch_views:  # the three views' products batched into shared launches
            # the batch rows' tags (marked above for the UI backbone; the side stream has joined)
            tags = self._tags if self._sparse_rows(rows) else None
            gtags = None
            if tags is not None:  # the backward's own tags (the UI backbone re-tags on the side stream)
                if self._vtags is None:
                    self._vtags = _RowTags(self.n_users + self.n_items, self.device)
                gtags = self._vtags
            image_embeds, text_embeds, fusion_embeds = SF.view_prop3(
                (img_i, txt_i, fus_i), (self.image_graph, self.text_graph, self.fusion_graph), self.R, L_, nu,
                tags=tags, gtags=gtags, rows=bw if gtags is not None else None)
        else:
            image_embeds = SF.view_prop(img_i, self.image_graph, self.R, L_, nu)
            text_embeds = SF.view_prop(txt_i, self.text_graph, self.R, L_, nu)
            fusion_embeds = SF.view_prop(fus_i, self.fusion_graph, self.R, L_, nu)
        if self.training and self.dropout.p > 0:
            # advanced before use (not after): the backward of this forward, which runs
            # before the next forward, reads the same value, so no copy is kept
            self._drop_seed.add_(1)
        seed = self._drop_seed
        if train:
            self._last["conv"] = (cv.detach(), ct.detach(), cf.detach())
        return content, image_embeds, text_embeds, fusion_embeds, seed

    def _forward_all_fused(self, train=False):
        content, image_embeds, text_embeds, fusion_embeds, seed = self._views_fused(train)
        all_embeds, side = SF.preference(self, content, image_embeds, text_embeds, fusion_embeds, seed)
        return all_embeds, side, content

    # ------------------------------------------------------------------ loss
    @staticmethod
    def InfoNCE(view1, view2, temperature):
        """Reference API (smore.py:395-401): mean -log(exp(<v1,v2>/t) / sum_j exp(<v1,v2_j>/t))
        of the L2-normalised rows, on the fused HIP kernels (rsx_smore_infonce_*)."""
        ar = torch.arange(view1.shape[0], dtype=torch.int64, device=view1.device)
        cl, _ = SF.infonce2(view1.contiguous(), view2.contiguous(), ar, ar, 0, temperature)
        return cl

    def _batch_index(self, B: int):
        """(ar, trip): arange(B) and the compact triplets (b, b, B + b) of the batch rows
        [users; B + positives; 2B + negatives] (cached per batch size)."""
        c = self._bidx.get(B)
        if c is None:
            ar = torch.arange(B, dtype=torch.int64, device=self.device)
            c = self._bidx[B] = (ar, torch.stack([ar, ar, ar + B]).contiguous())
            self._rows_off[B] = torch.cat([torch.zeros(B, dtype=torch.int64, device=self.device),
                                           torch.full((2 * B,), self.n_users, dtype=torch.int64, device=self.device)])
        return c

    def _calculate_loss_rows(self, interaction):
        """The training loss with the preference block on the batch rows only: the BPR
        and InfoNCE terms read all / side / content at the batch's users, positives
        and negatives alone, and the block is row-local (smore.py:320-341), so its
        other rows are never computed.  Same loss and gradients as the full-table
        form (duplicate rows are computed once per occurrence, their gradients added)."""
        nu, B = self.n_users, interaction.shape[1]
        ar, trip = self._batch_index(B)
        rows = interaction[:3].reshape(-1) + self._rows_off[B]  # [users; nu + positives; nu + negatives]
        exch = self._exch  # data-parallel SMORE: the batch-row gradient exchange
        content, image_embeds, text_embeds, fusion_embeds, seed = self._views_fused(
            train=True, rows=rows, bw_rows=exch.union if exch is not None else None)
        all_c, side_c, content_c = SF.preference_rows(self, content, image_embeds, text_embeds, fusion_embeds,
                                                      rows, seed, sparse_grads=self._sparse_rows(rows), exch=exch)
        self.global_step += 1
        total, parts = SF.smore_loss_rows(all_c, side_c, content_c, trip, ar, B, self.reg_weight, self.batch_size,
                                          self.cl_loss, self.cl_temp)
        self._last["cl"] = (parts[0], parts[1])
        return total

    def calculate_loss(self, interaction):
        if self.scheme == "usershard":  # this rank's batch (users as local row ids): rsx.smore_dist
            if self.training and self.dropout.p > 0:
                self._drop_seed.add_(1)
            self.global_step += 1
            return self._shard.loss(self, interaction, self._drop_seed)
        if self.batch_rows:  # (data-parallel: this rank's batch, global ids, the same path)
            return self._calculate_loss_rows(interaction)
        if self.scheme == "dp":
            raise RuntimeError("data-parallel SMORE trains on the batch rows (rsx_smore_batch_rows: True)")
        users, pos, neg = interaction[0], interaction[1], interaction[2]
        all_embeds, side, content = self._forward_all(train=True)
        self.global_step += 1
        nu = self.n_users
        bpr = _BprLoss.apply(all_embeds, None, None, interaction[:3].contiguous(), L.RSX_BPR_SMORE,
                             float(self.reg_weight), float(self.batch_size), nu, self.n_items)
        cl_items, cl_users = SF.infonce2(side, content, users, pos, nu, self.cl_temp)
        self._last["cl"] = (cl_items.detach(), cl_users.detach())
        return bpr + self.cl_loss * (cl_items + cl_users)

    def full_sort_predict(self, interaction):
        if self.scheme == "usershard":
            raise NotImplementedError("the sharded SMORE evaluates through full_sort_topk_local")
        with torch.no_grad():
            u, i = self.forward(self.norm_adj_csr)
        return ops.score_dense(u.contiguous(), interaction[0].contiguous(), i.contiguous())

    def full_sort_topk(self, interaction, k, eval_data):
        if self.scheme == "usershard":
            raise NotImplementedError("the sharded SMORE evaluates through full_sort_topk_local")
        with torch.no_grad():
            if getattr(self, "_eval_cache", None) is None:
                u, i = self.forward(self.norm_adj_csr)
                self._eval_cache = (u.contiguous(), i.contiguous())
            u, i = self._eval_cache
        return ops.fullsort_topk(u, interaction[0].contiguous(), i, eval_data.mask_rowptr, eval_data.mask_col, k)

    def train(self, mode: bool = True):
        self._eval_cache = None
        return super().train(mode)

    # ----------------------------------------------------------- diagnostics
    def diagnostics_enabled(self) -> bool:
        return bool(self.mg_verbose or self.diag_grad or self.diag_spectrum or self.diag_gate)

    @torch.no_grad()
    def log_mm_diagnostics(self, optimizer=None):
        if not self.diagnostics_enabled():
            return
        parts = []
        if self.diag_spectrum and "spec_in" in self._last:
            def band(x):
                f = torch.fft.rfft(x, dim=1, norm="ortho")
                m2 = (f.real ** 2 + f.imag ** 2).mean(dim=0)
                n = m2.numel()
                lo, mid, hi = m2[:max(1, n // 3)].sum(), m2[max(1, n // 3):max(2, 2 * n // 3)].sum(), m2[max(2, 2 * n // 3):].sum()
                t = lo + mid + hi + 1e-12
                return (lo / t).item(), (mid / t).item(), (hi / t).item()
            a, b = self._last["spec_in"]
            i3, t3 = band(a), band(b)
            parts.append(f"[spec] image(lo/mid/hi)={i3[0]:.2f}/{i3[1]:.2f}/{i3[2]:.2f} "
                         f"text={t3[0]:.2f}/{t3[1]:.2f}/{t3[2]:.2f}")
        if "cl" in self._last:
            ci, cu = self._last["cl"]
            parts.append(f"[cl] cl_items={ci.item():.4f}, cl_users={cu.item():.4f}")
        if optimizer is not None and len(optimizer.param_groups) > 0:
            lr = optimizer.param_groups[0].get("lr", float("nan"))
            parts.append(f"[mg] step={self.global_step} τ={self.mg_interval} α={self.mg_alpha} β={self.mg_beta} lr={lr}")
        print(" | ".join(parts))
