"""LightGCN on the rsx HIP path — drop-in for the reference's models/lightgcn.py.

Same class name, constructor `(config, dataset)`, YAML keys (embedding_size,
n_layers, reg_weight), parameter names (embedding_dict.user_emb / item_emb),
initialisation (xavier_uniform_ on the CPU RNG, users then items) and loss
(reference src/models/lightgcn.py:22-166).

The two parameters are views of one device buffer [users; items] owned by a
LightGCNEngine, so `torch.cat([user_emb, item_emb])` is free and both paths
below update the same storage:

* autograd path (`calculate_loss`): custom autograd Functions whose forward and
  backward are the HIP propagation (the backward of mean_k A^k E is the same
  operator, A symmetric) and the fused BPR kernel — the reference Trainer with a
  torch optimizer works unchanged;
* fused path (`fused_step`): one `rsx_lightgcn_step` call per batch, Adam in
  the last backward SpMM's epilogue (used by rsx.trainer.Trainer).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .engine import LightGCNEngine
from .recommender import GeneralRecommender


def propagate_mean(engine, x: torch.Tensor) -> torch.Tensor:
    """mean_{k=0..K} A^k x with the engine's adjacency (fresh output tensor)."""
    x = x.contiguous()
    out = torch.empty_like(x)
    s, h0, h1 = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    slab = engine.adj.slab(engine.d)
    rc = L.lib().rsx_lightgcn_forward(C.byref(engine.adj.struct), engine.d, engine.K, ops._p(x), ops._p(s),
                                      ops._p(h0), ops._p(h1), ops._p(out), ops._p(slab), ops._stream())
    L.check(rc, "rsx_lightgcn_forward")
    return out


class _Propagate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, user_emb, item_emb, engine):
        ctx.engine = engine
        return propagate_mean(engine, torch.cat([user_emb, item_emb], 0))

    @staticmethod
    def backward(ctx, g):
        eng = ctx.engine
        gx = propagate_mean(eng, g)  # A symmetric: d/dE0 of mean_k A^k E0 applied to g
        return gx[: eng.n_users], gx[eng.n_users:], None


class _BprLoss(torch.autograd.Function):
    """Fused BPR (+ regulariser) loss; gradients are produced by the forward kernel."""

    @staticmethod
    def forward(ctx, final, user_emb, item_emb, triplets, variant, reg, batch_cfg, n_users, n_items):
        ego = torch.cat([user_emb, item_emb], 0) if variant != L.RSX_BPR_SMORE else None
        loss, gf, ge = ops.bpr(variant, final.contiguous(), ego, n_users, n_items, triplets, reg, batch_cfg)
        ctx.save_for_backward(gf, ge if ge is not None else torch.zeros(0, device=final.device))
        ctx.n_users = n_users
        ctx.has_ego = ge is not None
        return loss[0]

    @staticmethod
    def backward(ctx, go):
        gf, ge = ctx.saved_tensors
        nu = ctx.n_users
        gu = gi = None
        if ctx.has_ego:
            gu, gi = go * ge[:nu], go * ge[nu:]
        return go * gf, gu, gi, None, None, None, None, None, None


class LightGCN(GeneralRecommender):
    supports_fused_step = True

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        ops.require_device(self.device)
        self.interaction_matrix = dataset.inter_matrix(form="coo").astype(np.float32)
        self.latent_dim = config["embedding_size"]
        self.n_layers = config["n_layers"]
        self.reg_weight = config["reg_weight"]
        # reference _init_model (lightgcn.py:56-63): xavier_uniform_, users then items, CPU RNG
        u0 = nn.init.xavier_uniform_(torch.empty(self.n_users, self.latent_dim))
        i0 = nn.init.xavier_uniform_(torch.empty(self.n_items, self.latent_dim))
        im = self.interaction_matrix
        wd = config["weight_decay"] or 0.0
        self.engine = LightGCNEngine(im.row.astype(np.int64), im.col.astype(np.int64), self.n_users, self.n_items,
                                     self.latent_dim, self.n_layers, self.reg_weight,
                                     lr=config["learning_rate"] or 1e-3, device=self.device, user_emb=u0.numpy(),
                                     item_emb=i0.numpy(), seed=int(config["seed"] or 0),
                                     batch=int(config["train_batch_size"]), chunk=int(config["rsx_chunk"] or 32),
                                     weight_decay=float(wd))
        nu = self.n_users
        self.embedding_dict = nn.ParameterDict({
            "user_emb": nn.Parameter(self.engine.p[:nu]),
            "item_emb": nn.Parameter(self.engine.p[nu:]),
        })

    # -- reference API -----------------------------------------------------------
    def train(self, mode: bool = True):
        self.engine.invalidate()
        return super().train(mode)

    def get_ego_embeddings(self):
        return torch.cat([self.embedding_dict["user_emb"], self.embedding_dict["item_emb"]], 0)

    def forward(self):
        final = _Propagate.apply(self.embedding_dict["user_emb"], self.embedding_dict["item_emb"], self.engine)
        return final[: self.n_users], final[self.n_users:]

    def calculate_loss(self, interaction):
        self.engine.invalidate()
        final = _Propagate.apply(self.embedding_dict["user_emb"], self.embedding_dict["item_emb"], self.engine)
        return _BprLoss.apply(final, self.embedding_dict["user_emb"], self.embedding_dict["item_emb"],
                              interaction[:3].contiguous(), L.RSX_BPR_LIGHTGCN, float(self.reg_weight),
                              float(interaction.shape[1]), self.n_users, self.n_items)

    def _final(self):
        with torch.no_grad():
            return self.engine.forward()

    def full_sort_predict(self, interaction):
        f = self._final()
        return ops.score_dense(f[: self.n_users], interaction[0].contiguous(), f[self.n_users:])

    # -- rsx fast paths ----------------------------------------------------------
    def fused_step(self, interaction, lr: float):
        self.engine.set_lr(lr)
        self.engine.step(triplets=interaction)

    def full_sort_topk(self, interaction, k: int, eval_data):
        f = self._final()
        return ops.fullsort_topk(f[: self.n_users], interaction[0].contiguous(), f[self.n_users:],
                                 eval_data.mask_rowptr, eval_data.mask_col, k)

    @property
    def device_loss_acc(self):
        return self.engine.loss_acc
