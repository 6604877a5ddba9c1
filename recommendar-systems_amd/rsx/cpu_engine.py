"""The reference's CPU configuration through the rsx operator boundary.

BASELINE config C1 is "LayerGCN K=2 d=64 on Amazon-baby, CPU PyTorch reference path
(plumbing, no GPU)": the reference trains it on the CPU with torch's sparse ops
(src/models/layergcn.py:127-177, src/common/trainer.py:186-238).  When the config's
device is the CPU (no GPU, or `use_gpu: False`) the drop-in LayerGCN and LightGCN
classes train on this engine instead of the HIP one: the same step — propagation,
the fused BPR loss, its backward, Adam — as torch.ops.rsx calls on CPU tensors, which
the dispatcher sends to the C++ CPU kernels of librsx (csrc/cpu_ops.cpp).  It is the
CPU configuration, not a fallback: a model whose device is a GPU never builds it (the
HIP engine raises when the library or the GPU is missing), and a CPU tensor never
reaches a GPU kernel.

Graphs are host CSR tensors (rowptr int64, col int32, val f32); the parameters are one
[users; items] table, so the models' nn.Parameters are views of it as on the GPU.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib as L
from . import graph
from . import torch_ops  # noqa: F401  registers torch.ops.rsx (CPU and CUDA kernels)

KINDS = {"lightgcn": L.RSX_BPR_LIGHTGCN, "layergcn": L.RSX_BPR_LAYERGCN}


def _csr_tensors(rowptr, col, val):
    return (torch.from_numpy(np.ascontiguousarray(rowptr, dtype=np.int64)),
            torch.from_numpy(np.ascontiguousarray(col, dtype=np.int32)),
            torch.from_numpy(np.ascontiguousarray(val, dtype=np.float32)))


class CpuGCNEngine:
    """LightGCN (mean of K propagated layers) or LayerGCN (cosine-gated layers, ego
    excluded) on the CPU kernels; the step is the reference's calculate_loss + backward +
    torch.optim.Adam step (lightgcn.py:132-156 / layergcn.py:142-177, trainer.py:238)."""

    def __init__(self, kind: str, train_u, train_i, n_users: int, n_items: int, dim: int, n_layers: int, reg: float,
                 lr: float, user_emb: np.ndarray, item_emb: np.ndarray, weight_decay: float = 0.0):
        if kind not in KINDS:
            raise ValueError(f"CpuGCNEngine: kind {kind!r} not in {sorted(KINDS)}")
        self.kind, self.variant = kind, KINDS[kind]
        self.n_users, self.n_items, self.d, self.K = int(n_users), int(n_items), int(dim), int(n_layers)
        if self.K < (0 if kind == "lightgcn" else 1):
            raise RuntimeError(f"{kind}: n_layers {self.K} out of range")
        self.reg, self.lr, self.wd = float(reg), float(lr), float(weight_decay)
        self.device = torch.device("cpu")
        self.norm_adj = _csr_tensors(*graph.lightgcn_norm_adj(np.asarray(train_u, np.int64),
                                                              np.asarray(train_i, np.int64), self.n_users,
                                                              self.n_items))
        self.train_adj = self.norm_adj
        self.p = torch.from_numpy(np.ascontiguousarray(np.concatenate([user_emb, item_emb]), dtype=np.float32))
        self.m, self.v = torch.zeros_like(self.p), torch.zeros_like(self.p)
        self.step_t = torch.zeros((), dtype=torch.int64)
        self.loss_acc = torch.zeros(1, dtype=torch.float64)
        self.step_count = 0
        self._eval = None
        self.kind_id = 0 if kind == "lightgcn" else 1
        self.use_ops = os.environ.get("RSX_CPU_STEP", "fused") == "ops"
        self._ws = None
        self._loss = torch.zeros(1, dtype=torch.float32)

    # -- graphs ------------------------------------------------------------------
    def set_train_graph(self, rowptr, col, val):
        self.train_adj = _csr_tensors(rowptr, col, val)

    def use_eval_graph_for_training(self):
        self.train_adj = self.norm_adj

    def invalidate(self):
        self._eval = None

    def set_lr(self, lr: float):
        self.lr = float(lr)

    def _prop(self, adj, x):
        if self.kind == "lightgcn":
            return torch.ops.rsx.propagate_mean(*adj, x, self.K)
        return torch.ops.rsx.propagate_layergcn(*adj, x, self.K)

    # -- training / evaluation -----------------------------------------------------
    def loss(self, x: torch.Tensor, triplets: torch.Tensor, adj=None) -> torch.Tensor:
        """The reference calculate_loss of one batch on the table x (autograd through the ops)."""
        f = self._prop(self.train_adj if adj is None else adj, x)
        return torch.ops.rsx.bpr_loss(f, x, triplets[:3].contiguous(), self.n_users, self.reg, self.variant, 0.0)

    def step(self, triplets: torch.Tensor):
        """One batch: `rsx_cpu_gcn_step` (the whole step in one C-ABI call, csrc/cpu_ops.cpp);
        with `use_ops` the torch.ops.rsx sequence (propagate + bpr_loss + autograd + adam_),
        the same formulas (tests/test_cpu_e2e.py checks the two against each other)."""
        self.step_count += 1
        if self.use_ops or self.K < 1:
            x = self.p.detach().requires_grad_(True)
            loss = self.loss(x, triplets)
            (g,) = torch.autograd.grad(loss, [x])
            self.step_t += 1
            torch.ops.rsx.adam_(self.p, g, self.m, self.v, self.step_t, self.lr, 0.9, 0.999, 1e-8, self.wd)
            self.loss_acc += loss.detach().double()
            self._eval = None
            return
        trip = triplets[:3].to(torch.int64).contiguous()
        B = int(trip.shape[1])
        n = self.n_users + self.n_items
        lib = L.lib()
        need = int(lib.rsx_cpu_gcn_step_ws_floats(self.kind_id, n, self.d, self.K, B))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.float32)
        rp, col, val = self.train_adj
        self.step_t += 1
        L.check(lib.rsx_cpu_gcn_step(self.kind_id, rp.data_ptr(), col.data_ptr(), val.data_ptr(), self.n_users,
                                     self.n_items, self.d, self.K, trip.data_ptr(), B, self.reg, self.p.data_ptr(),
                                     self.m.data_ptr(), self.v.data_ptr(), int(self.step_t), self.lr, 0.9, 0.999,
                                     1e-8, self.wd, self._ws.data_ptr(), self._ws.numel(), self._loss.data_ptr()),
                "rsx_cpu_gcn_step")
        self.loss_acc += self._loss.double()
        self._eval = None

    def forward(self) -> torch.Tensor:
        """The evaluation tables on the full normalised graph (full_sort_predict's forward)."""
        if self._eval is None:
            with torch.no_grad():
                self._eval = self._prop(self.norm_adj, self.p)
        return self._eval
