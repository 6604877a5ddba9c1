"""Device-resident training engines: all state in HBM, one C-ABI call per batch.

`LightGCNEngine` holds the LightGCN parameters (users then items, one [N, d]
buffer so that the reference's `torch.cat([user_emb, item_emb])`
(src/models/lightgcn.py:105-115) is free), Adam moments, layer scratch and the
CSR adjacency, and runs a whole batch — optional device sampling, K-layer
propagation, BPR loss, Horner backward, Adam — through `rsx_lightgcn_step`.
The loss is accumulated on the device (f64) so a training epoch needs no
per-batch host sync (the reference calls loss.item() per batch,
src/common/trainer.py:196-200).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib as L
from . import graph, ops


def lightgcn_adj(train_u, train_i, n_users: int, n_items: int, device, chunk: int = 32) -> "ops.DeviceCSR":
    """The normalised adjacency (reference lightgcn.py:65-103) built on the device
    (rsx_adj_build, csrc/graph.hip; bit-equal to graph.lightgcn_norm_adj, which
    RSX_GRAPH_BUILDER=host selects)."""
    n = n_users + n_items
    if os.environ.get("RSX_GRAPH_BUILDER", "device") == "host":
        rp, col, val = graph.lightgcn_norm_adj(train_u, train_i, n_users, n_items)
        return ops.DeviceCSR(rp, col, val, n, device, chunk)
    rp, col, val = ops.adj_build(train_u, train_i, n_users, n_items, ops.ADJ_LIGHTGCN, device)
    return ops.DeviceCSR.from_device(rp, col, val, n, chunk)


class LightGCNEngine:
    def __init__(self, train_u: np.ndarray, train_i: np.ndarray, n_users: int, n_items: int, dim: int,
                 n_layers: int, reg: float, lr: float, device, user_emb: np.ndarray | None = None,
                 item_emb: np.ndarray | None = None, seed: int = 0, chunk: int = 32, batch: int = 2048,
                 weight_decay: float = 0.0, adj=None):
        self.device = ops.require_device(device)
        self.n_users, self.n_items, self.d, self.K = int(n_users), int(n_items), int(dim), int(n_layers)
        self.reg, self.lr, self.wd = float(reg), float(lr), float(weight_decay)
        n = self.n_users + self.n_items
        if adj is None:
            adj = lightgcn_adj(train_u, train_i, self.n_users, self.n_items, self.device, chunk)
        self.adj = adj
        if user_emb is None:
            # xavier_uniform_ as reference lightgcn.py:56-63 (CPU RNG, caller seeds)
            user_emb = torch.nn.init.xavier_uniform_(torch.empty(self.n_users, dim)).numpy()
            item_emb = torch.nn.init.xavier_uniform_(torch.empty(self.n_items, dim)).numpy()
        p = np.concatenate([user_emb, item_emb]).astype(np.float32)
        dev = self.device
        self.p = torch.from_numpy(p).to(dev)
        z = lambda: torch.zeros(n, dim, dtype=torch.float32, device=dev)  # noqa: E731
        self.m, self.v = z(), z()
        self.s, self.h0, self.h1 = z(), z(), z()
        self.final, self.g, self.r = z(), z(), z()
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self.step_count = 0
        self.batch = int(batch)
        self.ws = torch.empty(L.lib().rsx_bpr_ws_bytes(max(self.batch, 1)), dtype=torch.uint8, device=dev)
        self.sampler = ops.DeviceSampler(np.asarray(train_u), np.asarray(train_i), self.n_users, dev, seed=seed)
        self.n_inter = self.sampler.n_inter
        self.trip = torch.zeros(3, self.batch, dtype=torch.int64, device=dev)
        self.epoch_trip = torch.zeros(3 * self.n_inter, dtype=torch.int64, device=dev)
        self._epoch_sampled = None
        # batch-row tags (rsx_lgcn_step.row_tag): last forward layer on the batch rows,
        # sparse G in the first backward layer; RSX_BATCH_TAGS=0 selects the dense path
        self.row_tag = torch.zeros(n, dtype=torch.int32, device=dev)
        self.use_tags = self.K >= 2 and os.environ.get("RSX_BATCH_TAGS", "1") != "0"
        # one-launch BPR with the regulariser gradient as per-row counts (tagged step only)
        self.reg_cnt = torch.zeros(3 * n + 4, dtype=torch.int32, device=dev)
        self.use_reg_cnt = os.environ.get("RSX_BPR_FUSED", "1") != "0"
        # NaN halt flag of the step (every path: tagged, dense, K >= 4): {halted, tag of the NaN step}
        self.halt = torch.zeros(2, dtype=torch.int32, device=dev)
        self._st = L.LgcnStep()
        self._sa = L.SamplerArgs()
        self._fill_static()
        self._fwd_valid = False

    # -- views matching the reference's parameter names ------------------------
    @property
    def user_emb(self):
        return self.p[: self.n_users]

    @property
    def item_emb(self):
        return self.p[self.n_users:]

    def _fill_static(self):
        st = self._st
        st.adj = C.pointer(self.adj.struct)
        st.n_users, st.n_items, st.d, st.n_layers, st.reg = self.n_users, self.n_items, self.d, self.K, self.reg
        for name in ("p", "m", "v", "s", "h0", "h1", "g", "r"):
            setattr(st, name, getattr(self, name).data_ptr())
        st.final_emb = self.final.data_ptr()
        slab = self.adj.slab(self.d)
        st.slab = slab.data_ptr() if slab is not None else 0
        st.loss_out = self.loss_out.data_ptr()
        st.loss_acc = self.loss_acc.data_ptr()
        st.ws, st.ws_bytes = self.ws.data_ptr(), self.ws.numel()
        st.row_tag = self.row_tag.data_ptr() if self.use_tags else None
        st.reg_cnt = self.reg_cnt.data_ptr() if (self.use_tags and self.use_reg_cnt) else None
        st.halt = self.halt.data_ptr()

    def set_lr(self, lr: float):
        self.lr = float(lr)

    def step(self, triplets: torch.Tensor | None = None, epoch: int = 0, start: int = 0) -> None:
        """One batch.  With `triplets` (int64 [3, B] on the device) the batch is given
        (parity mode); otherwise it is sampled on the device for (epoch, start)."""
        st = self._st
        self.step_count += 1
        st.adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd)
        st.tag = self.step_count  # fresh per step, > 0
        if triplets is not None:
            t = triplets[:3].contiguous()
            if t.shape[1] > self.batch:
                raise RuntimeError("batch larger than the engine's batch size")
            self._keep = t
            st.triplets = t.data_ptr()
            st.batch = t.shape[1]
            st.sample = None
        else:
            # one sampling launch per epoch (batch-major buffer), then slices
            if self._epoch_sampled != epoch:
                self.sampler.sample_epoch(epoch, self.batch, out=self.epoch_trip)
                self._epoch_sampled = epoch
            if start % self.batch:
                raise RuntimeError("start must be a multiple of the batch size")
            t = ops.DeviceSampler.batch_view(self.epoch_trip, self.n_inter, self.batch, start // self.batch)
            st.triplets = t.data_ptr()
            st.batch = t.shape[1]
            st.sample = None
        L.check(L.lib().rsx_lightgcn_step(C.byref(st), ops._stream()), "rsx_lightgcn_step")
        self._fwd_valid = False

    def forward(self) -> torch.Tensor:
        """final = mean_k A^k E^0 (reference lightgcn.py:117-130); cached until the next step."""
        if not self._fwd_valid:
            slab = self.adj.slab(self.d)
            rc = L.lib().rsx_lightgcn_forward(C.byref(self.adj.struct), self.d, self.K, ops._p(self.p),
                                             ops._p(self.s), ops._p(self.h0), ops._p(self.h1), ops._p(self.final),
                                             ops._p(slab), ops._stream())
            L.check(rc, "rsx_lightgcn_forward")
            self._fwd_valid = True
        return self.final

    def invalidate(self):
        self._fwd_valid = False
