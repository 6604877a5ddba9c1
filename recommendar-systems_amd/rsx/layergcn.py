"""LayerGCN on the rsx HIP path — drop-in for the reference's models/layergcn.py.

Forward (reference src/models/layergcn.py:127-140): Z^k = A E^{k-1},
c^k = cos(Z^k, E^0) (F.cosine_similarity, eps 1e-8), E^k = c^k Z^k,
out = sum_{k=1..K} E^k — one SpMM per layer with the cosine scaling and the
running sum fused into its epilogue (RSX_EPI_LAYERGCN), which also saves Z^k
and c^k for the backward.  Training uses the per-epoch edge-dropout graph
(`pre_epoch_processing`, layergcn.py:51-70: alternating torch.multinomial over
the degree-normalised edge values and random.sample, float32 renormalisation —
on the device by default (DeviceEdgeDropout), or host-side with the reference's own
RNG calls, so that the kept edges are the reference's (rsx_edge_dropout: host, the
default when rsx_sampler is host)); evaluation uses the full normalised graph.

Backward: dE^K = G; for k = K..1 the LAYERGCN_BWD epilogue turns dE^k into
dZ^k and accumulates the cosine's dependence on E^0; dE^{k-1} = A dZ^k + G is
the next SpMM with the same epilogue; the last SpMM's epilogue applies Adam to
E^0 with g = A dZ^1 + (cosine terms) + reg.  Loss: sum-BPR + reg * L2
(layergcn.py:142-177), fused kernel RSX_BPR_LAYERGCN.
"""
from __future__ import annotations

import ctypes as C
import os

import random

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import graph, ops
from .engine import lightgcn_adj
from .recommender import GeneralRecommender


class LayerGCNEngine:
    def __init__(self, train_u, train_i, n_users, n_items, dim, n_layers, reg, lr, device, user_emb, item_emb,
                 chunk=32, weight_decay=0.0, batch=2048):
        self.device = ops.require_device(device)
        self.n_users, self.n_items, self.d, self.K = int(n_users), int(n_items), int(dim), int(n_layers)
        if self.K < 1:
            raise RuntimeError("LayerGCN needs n_layers >= 1")
        self.reg, self.lr, self.wd, self.chunk = float(reg), float(lr), float(weight_decay), int(chunk)
        n = self.n_users + self.n_items
        self.norm_adj = lightgcn_adj(train_u, train_i, self.n_users, self.n_items, self.device, chunk)
        self.train_adj = self.norm_adj
        dev = self.device
        self.p = torch.from_numpy(np.concatenate([user_emb, item_emb]).astype(np.float32)).to(dev)
        z = lambda: torch.zeros(n, dim, dtype=torch.float32, device=dev)  # noqa: E731
        self.m, self.v = z(), z()
        self.out, self.g, self.r, self.acc = z(), z(), z(), z()
        self.h = [z(), z()]
        self.zs = [z() for _ in range(self.K)]
        self.cs = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(self.K)]
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self.step_count = 0
        self._eval_out = z()
        self._eval_valid = False

    def set_train_graph(self, rowptr, col, val):
        n = self.n_users + self.n_items
        self.train_adj = ops.DeviceCSR(rowptr, col, val, n, self.device, self.chunk)

    def use_eval_graph_for_training(self):
        self.train_adj = self.norm_adj

    def invalidate(self):
        self._eval_valid = False

    def _forward(self, A, out, zero_grads=False, save=True):
        d, K = self.d, self.K
        x = self.p
        for k in range(1, K + 1):
            y = self.h[(k - 1) & 1]
            kw = dict(e0=self.p, y=y, s_out=out, s_in=(out if k > 1 else None))
            if save:
                kw.update(aux=self.zs[k - 1], aux_w=self.cs[k - 1])
            if k == K and zero_grads:
                kw.update(zero0=self.g, zero1=self.r)
            A.spmm_epi(x, ops.epi(L.RSX_EPI_LAYERGCN, **kw), d)
            x = y
        return out

    def forward(self):
        """Evaluation forward on the full normalised graph (layergcn.py:179-188)."""
        if not self._eval_valid:
            self._forward(self.norm_adj, self._eval_out, save=False)
            self._eval_valid = True
        return self._eval_out

    def _c_step(self, triplets: torch.Tensor):
        """The batch as one rsx_layergcn_step call (the same kernels and order as the
        Python-issued sequence below; host cost one ctypes call)."""
        st = getattr(self, "_cst", None)
        if st is None:
            st = self._cst = L.LayerGcnStep()
            st.n_users, st.n_items, st.d, st.n_layers, st.reg = self.n_users, self.n_items, self.d, self.K, self.reg
            for name in ("p", "m", "v", "out", "g", "r", "acc"):
                setattr(st, name, getattr(self, name).data_ptr())
            st.h0, st.h1 = self.h[0].data_ptr(), self.h[1].data_ptr()
            self._zs_arr = (C.c_void_p * self.K)(*[z.data_ptr() for z in self.zs])
            self._cs_arr = (C.c_void_p * self.K)(*[c.data_ptr() for c in self.cs])
            st.zs, st.cs = C.cast(self._zs_arr, C.c_void_p), C.cast(self._cs_arr, C.c_void_p)
            st.loss_acc = self.loss_acc.data_ptr()
            st.loss_out = None
        A = self.train_adj
        if getattr(self, "_cst_adj", None) is not A:  # a new epoch graph
            st.adj = C.pointer(A.struct)
            slab = A.slab(self.d)
            st.slab = slab.data_ptr() if slab is not None else None
            self._cst_adj = A
        trip = triplets[:3].contiguous()
        B = trip.shape[1]
        ws = ops._ws(self.device, L.lib().rsx_bpr_ws_bytes(B))
        st.ws, st.ws_bytes = ws.data_ptr(), ws.numel()
        st.triplets, st.batch = trip.data_ptr(), B
        st.adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd)
        self._keep = trip
        L.check(L.lib().rsx_layergcn_step(C.byref(st), ops._stream()), "rsx_layergcn_step")
        self._eval_valid = False

    def step(self, triplets: torch.Tensor):
        d, K, n = self.d, self.K, self.n_users + self.n_items
        A = self.train_adj
        self.step_count += 1
        if os.environ.get("RSX_LAYERGCN_CSTEP", "1") != "0":
            self._c_step(triplets)
            return
        self._forward(A, self.out, zero_grads=True, save=True)
        ops.bpr(L.RSX_BPR_LAYERGCN, self.out, self.p, self.n_users, self.n_items, triplets[:3].contiguous(),
                self.reg, g_final=self.g, g_ego=self.r, loss_acc=self.loss_acc)
        # dE^K = G -> dZ^K (rowwise), ego-cosine terms into acc
        hz = self.h[0]
        ops.rowwise(n, d, ops.epi(L.RSX_EPI_LAYERGCN_BWD, r_add=self.g, aux=self.zs[K - 1],
                                  aux_w=self.cs[K - 1], e0=self.p, y=hz, s_out=self.acc))
        adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd)
        for k in range(K - 1, 0, -1):
            y = self.h[(K - k) & 1]
            A.spmm_epi(hz, ops.epi(L.RSX_EPI_LAYERGCN_BWD, r_add=self.g, aux=self.zs[k - 1], aux_w=self.cs[k - 1],
                                   e0=self.p, y=y, s_in=self.acc, s_out=self.acc), d)
            hz = y
        # dE^0 = A dZ^1 + cosine terms + reg -> Adam
        A.spmm_epi(hz, ops.epi(L.RSX_EPI_ADAM, s_in=self.acc, r_add=self.r, p=self.p, m=self.m, v=self.v,
                               adam=adam), d)
        self._eval_valid = False


class DeviceEdgeDropout:
    """The per-epoch edge dropout of the training graph on the device (reference
    layergcn.py:51-81).  Kept edges: `torch.multinomial(edge_values, keep_len)` on
    the device (without replacement: the exponential race, the same distribution as
    the reference's CPU draw) or a uniform `randperm` subset (the reference's
    `random.sample` epochs), alternating as in the reference.  Values: float32
    1/sqrt(1e-7 + kept degree) products, the reference's _normalize_adj_m, computed
    with correctly rounded f32 ops (bit-equal to graph.layergcn_edge_values on the
    same kept set, tests/test_gpu_kernels.py).  CSR: the symmetric template of all
    edges, sorted by (row, col) once, compacted by the keep mask (cumsum + scatter;
    the kept count is known, so nothing waits on the device); only rowptr goes to
    the host, for the SpMM work schedule.

    Per epoch ~0.1 ms of device work where the host path (CPU multinomial + numpy
    CSR) takes ~150-370 ms at Amazon-baby: the epoch is ~12 ms of GPU steps."""

    def __init__(self, e_u: np.ndarray, e_i: np.ndarray, n_users: int, n_items: int, edge_values: np.ndarray,
                 device, chunk: int = 32):
        self.device = torch.device(device)
        self.n_users, self.n_items, self.chunk = int(n_users), int(n_items), int(chunk)
        e_u = np.asarray(e_u, dtype=np.int64)
        e_i = np.asarray(e_i, dtype=np.int64)
        E = e_u.size
        self.n_edges = E
        self.u = torch.from_numpy(e_u).to(self.device)
        self.i = torch.from_numpy(e_i).to(self.device)
        self.w = torch.from_numpy(np.asarray(edge_values, dtype=np.float32)).to(self.device)
        n = self.n_users + self.n_items
        rows = np.concatenate([e_u, e_i + n_users])
        cols = np.concatenate([e_i + n_users, e_u])
        eid = np.concatenate([np.arange(E), np.arange(E)])
        order = np.lexsort((cols, rows))
        rowptr = np.zeros(n + 1, dtype=np.int64)
        rowptr[1:] = np.cumsum(np.bincount(rows, minlength=n)[:n])
        self.t_rowptr = torch.from_numpy(rowptr).to(self.device)
        self.t_col = torch.from_numpy(cols[order].astype(np.int32)).to(self.device)
        self.t_eid = torch.from_numpy(eid[order].astype(np.int64)).to(self.device)
        self._tmpl = None

    def keep_mask(self, keep_len: int, pruning_random: bool) -> torch.Tensor:
        if pruning_random:
            keep = torch.randperm(self.n_edges, device=self.device)[:keep_len]
        else:
            keep = torch.multinomial(self.w, keep_len)
        return torch.zeros(self.n_edges, dtype=torch.bool, device=self.device).index_fill_(0, keep, True)

    def build(self, mask: torch.Tensor, keep_len: int):
        """(rowptr, col, val) device tensors of the symmetric masked adjacency: kept
        degrees, f32 values and the template's compaction in one rsx_edge_dropout_build
        (csrc/graph.hip); RSX_GRAPH_BUILDER=host keeps the torch-op statement below."""
        if os.environ.get("RSX_GRAPH_BUILDER", "device") != "host":
            if not hasattr(self, "_t_col32"):
                self._t_col32 = self.t_col.contiguous()
            rp, col, val = ops.edge_dropout_build(self.u, self.i, mask, self.n_users, self.n_items, self.t_rowptr,
                                                  self._t_col32, self.t_eid)
            return rp, col[: 2 * keep_len], val[: 2 * keep_len]
        mf = mask.to(torch.float32)
        ru = torch.zeros(self.n_users, dtype=torch.float32, device=self.device).index_add_(0, self.u, mf)
        ci = torch.zeros(self.n_items, dtype=torch.float32, device=self.device).index_add_(0, self.i, mf)
        r_inv = 1.0 / torch.sqrt(1e-7 + ru)
        c_inv = 1.0 / torch.sqrt(1e-7 + ci)
        vals = r_inv[self.u] * c_inv[self.i]
        ek = mask[self.t_eid]
        ck = torch.cumsum(ek, 0)
        nnz = 2 * keep_len
        rowptr = torch.cat([ck.new_zeros(1), ck])[self.t_rowptr]
        dst = torch.where(ek, ck - 1, torch.full_like(ck, nnz))
        col = torch.empty(nnz + 1, dtype=torch.int32, device=self.device).scatter_(0, dst, self.t_col)
        val = torch.empty(nnz + 1, dtype=torch.float32, device=self.device).scatter_(0, dst, vals[self.t_eid])
        return rowptr, col[:nnz], val[:nnz]

    def epoch_graph(self, dropout: float, pruning_random: bool) -> "ops.DeviceCSR":
        """The epoch's masked graph.  Its work schedule is rewritten on the device over
        the layout of the full training graph's (every masked row is a subset of the
        template row: rsx_csr_schedule_rebind), so the rebuild has no host round trip;
        RSX_EPOCH_SCHEDULE=host schedules it on the host from a copy of rowptr."""
        keep_len = int(self.n_edges * (1.0 - dropout))
        rowptr, col, val = self.build(self.keep_mask(keep_len, pruning_random), keep_len)
        if os.environ.get("RSX_EPOCH_SCHEDULE", "device") == "host":
            return ops.DeviceCSR.from_device(rowptr, col, val, self.n_users + self.n_items, self.chunk)
        if self._tmpl is None:  # the full symmetric template's schedule (host, once)
            self._tmpl = ops.DeviceCSR(self.t_rowptr.cpu().numpy(), self.t_col.to(torch.int32).contiguous(),
                                       torch.zeros(self.t_col.numel(), dtype=torch.float32, device=self.device),
                                       self.n_users + self.n_items, self.device, self.chunk)
        return ops.DeviceCSR.rebind(self._tmpl, rowptr, col, val)


def reference_edge_dropout(edge_indices: torch.Tensor, edge_values: torch.Tensor, dropout: float,
                           pruning_random: bool):
    """Kept edge ids for one epoch with the reference's RNG calls (layergcn.py:55-62)."""
    keep_len = int(edge_values.size(0) * (1.0 - dropout))
    if pruning_random:
        return torch.tensor(random.sample(range(edge_values.size(0)), keep_len))
    return torch.multinomial(edge_values, keep_len)


class LayerGCN(GeneralRecommender):
    supports_fused_step = True

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.cpu = torch.device(self.device).type == "cpu"  # the CPU configuration (BASELINE C1, rsx.cpu_engine)
        if not self.cpu:
            ops.require_device(self.device)
        self.interaction_matrix = dataset.inter_matrix(form="coo").astype(np.float32)
        self.latent_dim = config["embedding_size"]
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        self.dropout = config["dropout"]
        self.n_nodes = self.n_users + self.n_items
        u0 = nn.init.xavier_uniform_(torch.empty(self.n_users, self.latent_dim))
        i0 = nn.init.xavier_uniform_(torch.empty(self.n_items, self.latent_dim))
        im = self.interaction_matrix
        if self.cpu:
            from .cpu_engine import CpuGCNEngine

            self.engine = CpuGCNEngine("layergcn", im.row, im.col, self.n_users, self.n_items, self.latent_dim,
                                       self.n_layers, self.reg_weight, config["learning_rate"] or 1e-3, u0.numpy(),
                                       i0.numpy(), weight_decay=float(config["weight_decay"] or 0.0))
        else:
            self.engine = LayerGCNEngine(im.row.astype(np.int64), im.col.astype(np.int64), self.n_users,
                                         self.n_items, self.latent_dim, self.n_layers, self.reg_weight,
                                         config["learning_rate"] or 1e-3, self.device, u0.numpy(), i0.numpy(),
                                         chunk=int(config["rsx_chunk"] or 32),
                                         weight_decay=float(config["weight_decay"] or 0.0))
        nu = self.n_users
        self.user_embeddings = nn.Parameter(self.engine.p[:nu])
        self.item_embeddings = nn.Parameter(self.engine.p[nu:])
        # edge info for the per-epoch dropout (layergcn.py:83-89), CPU tensors as in the reference
        self.edge_indices = torch.from_numpy(np.vstack([im.row, im.col]).astype(np.int64))
        self.edge_values = torch.from_numpy(graph.layergcn_edge_values(im.row.astype(np.int64),
                                                                       im.col.astype(np.int64), nu, self.n_items))
        self.pruning_random = False
        mode = config["rsx_edge_dropout"] or config["rsx_sampler"] or "device"
        if mode not in ("device", "host"):
            raise ValueError(f"rsx_edge_dropout must be 'device' or 'host', got {mode!r}")
        if self.cpu:  # the reference's own per-epoch draw and host graph (layergcn.py:51-89)
            mode = "host"
        self.edge_dropout_mode = mode
        self._dev_dropout = None

    def train(self, mode: bool = True):
        self.engine.invalidate()
        return super().train(mode)

    def pre_epoch_processing(self):
        if self.dropout <= 0.0:
            self.engine.use_eval_graph_for_training()
            return
        if self.edge_dropout_mode == "device":
            if self._dev_dropout is None:
                ei = self.edge_indices.numpy()
                self._dev_dropout = DeviceEdgeDropout(ei[0], ei[1], self.n_users, self.n_items,
                                                      self.edge_values.numpy(), self.device, self.engine.chunk)
            self.engine.train_adj = self._dev_dropout.epoch_graph(self.dropout, self.pruning_random)
            self.pruning_random = True ^ self.pruning_random
            return
        keep = reference_edge_dropout(self.edge_indices, self.edge_values, self.dropout, self.pruning_random)
        self.pruning_random = True ^ self.pruning_random
        kept = self.edge_indices[:, keep].numpy()
        self.engine.set_train_graph(*graph.layergcn_masked_adj(kept[0], kept[1], self.n_users, self.n_items))

    def calculate_loss(self, interaction):
        raise NotImplementedError("LayerGCN on rsx trains through fused_step (rsx.trainer.Trainer)")

    def _final(self):
        with torch.no_grad():
            return self.engine.forward()

    def forward(self):
        f = self._final()
        return f[: self.n_users], f[self.n_users:]

    def full_sort_predict(self, interaction):
        f = self._final()
        if self.cpu:  # reference layergcn.py:179-188 on the CPU tables
            return torch.matmul(f[: self.n_users][interaction[0]], f[self.n_users:].t())
        return ops.score_dense(f[: self.n_users], interaction[0].contiguous(), f[self.n_users:])

    def fused_step(self, interaction, lr: float):
        self.engine.lr = float(lr)
        self.engine.step(interaction)

    def full_sort_topk(self, interaction, k: int, eval_data):
        f = self._final()
        if self.cpu:
            return torch.ops.rsx.fullsort_topk(f[: self.n_users].contiguous(), interaction[0].contiguous(),
                                               f[self.n_users:].contiguous(), eval_data.mask_rowptr,
                                               eval_data.mask_col, k)
        return ops.fullsort_topk(f[: self.n_users], interaction[0].contiguous(), f[self.n_users:],
                                 eval_data.mask_rowptr, eval_data.mask_col, k)

    @property
    def device_loss_acc(self):
        return self.engine.loss_acc
