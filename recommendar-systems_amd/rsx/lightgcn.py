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

Sharded (torch.distributed initialised with world > 1, e.g. `torchrun
--nproc-per-node 8 main.py -m LightGCN -d sports`, or config `rsx_sharded: True`):
rank r owns the contiguous user block [r N/W, (r+1) N/W) and a
rsx.dist.ShardedLightGCNEngine (items replicated).  The initial
tables are the reference's (every rank draws the full xavier tables from the
same seed and keeps its users), the parameters are the local user block and the
item replica.  Training is data-parallel over the user shards: every rank samples
its own users' interactions on the device (`fused_step_index`); every rank runs
the same number of steps per epoch, ceil(E / (W B)), over its epoch cut into that
many balanced slices (sizes ceil / floor of E_r / steps ~ B), so it visits each of
its interactions exactly once, and the step minimises the sum of the ranks'
reference losses.
Evaluation ranks each rank's own evaluation users against all items
(`full_sort_topk_local`); rsx.trainer all-gathers the metric sums.

Config `rsx_dist: dp` selects the data-parallel engine instead (rsx.dp: the whole graph
and the tables on every rank, the global batch of every rank's triplets per step, two
small all-gathers a step), the evaluation users split over the ranks.
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


def _world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


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
        self.cpu = torch.device(self.device).type == "cpu"  # the CPU configuration (rsx.cpu_engine)
        if not self.cpu:
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
        world, rank = _world()
        if self.cpu:  # torch.ops.rsx's CPU kernels; one process (the reference's CPU run)
            from .cpu_engine import CpuGCNEngine

            self.sharded = self.dp = False
            self.engine = CpuGCNEngine("lightgcn", im.row, im.col, self.n_users, self.n_items, self.latent_dim,
                                       self.n_layers, self.reg_weight, config["learning_rate"] or 1e-3, u0.numpy(),
                                       i0.numpy(), weight_decay=float(wd))
            nu = self.n_users
            self.embedding_dict = nn.ParameterDict({
                "user_emb": nn.Parameter(self.engine.p[:nu]),
                "item_emb": nn.Parameter(self.engine.p[nu:]),
            })
            return
        self.sharded = world > 1 or bool(config["rsx_sharded"])
        self.dp = self.sharded and str(config["rsx_dist"] or "rowshard").lower() == "dp"
        if self.dp:
            self._init_dp(config, im, u0, i0, world, rank, float(wd))
            return
        if self.sharded:
            self._init_sharded(config, im, u0, i0, world, rank, float(wd))
            return
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

    def _init_sharded(self, config, im, u0, i0, world, rank, wd):
        import torch.distributed as dist

        from .dist import ShardedLightGCNEngine

        nu = self.n_users
        a, b = rank * nu // world, (rank + 1) * nu // world
        self.user_range = (a, b)
        rows, cols = im.row.astype(np.int64), im.col.astype(np.int64)
        sel = (rows >= a) & (rows < b)
        B = int(config["train_batch_size"])
        # every rank visits each of its interactions once per epoch in the same number of
        # steps: steps = ceil(E / (W B)) over the global count E, and rank r's epoch is cut
        # into `steps` balanced slices of its E_r interactions (sizes ceil / floor of
        # E_r / steps, ~B; rsx_sample_epoch_slices).  A rank with fewer interactions than
        # steps would have empty slices: refused on every rank alike (no rank may leave
        # the collectives early).
        e_r = int(sel.sum())
        dev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
        stats = torch.tensor([e_r, -e_r], dtype=torch.int64, device=dev)
        tot = stats[:1].clone()
        dist.all_reduce(tot)
        steps = max(1, -(-int(tot.item()) // (world * B)))
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)  # [max E_r, -min E_r]
        if -int(stats[1].item()) < steps:
            raise RuntimeError(f"sharded LightGCN: a rank holds {-int(stats[1].item())} training interactions, fewer "
                               f"than the {steps} steps per epoch (world {world}, batch {B}); use fewer ranks")
        b_r = -(-e_r // steps)
        cap = -(-int(stats[0].item()) // steps)  # the largest slice of any rank
        self.engine = ShardedLightGCNEngine(rows[sel] - a, cols[sel], b - a, self.n_items, self.latent_dim,
                                            self.n_layers, self.reg_weight, lr=config["learning_rate"] or 1e-3,
                                            device=self.device, user_emb=u0.numpy()[a:b], item_emb=i0.numpy(),
                                            seed=int(config["seed"] or 0) + rank, batch=b_r,
                                            chunk=int(config["rsx_chunk"] or 32), weight_decay=wd,
                                            union_cap=cap)
        self.steps_per_epoch = steps
        nl = b - a
        self.embedding_dict = nn.ParameterDict({
            "user_emb": nn.Parameter(self.engine.p[:nl]),
            "item_emb": nn.Parameter(self.engine.p[nl:]),
        })

    def _init_dp(self, config, im, u0, i0, world, rank, wd):
        """Data-parallel (config rsx_dist: dp, rsx.dp): the whole graph and the tables on
        every rank, each rank trains its slice of every global batch (the reference
        objective at batch W * train_batch_size); the replicas stay bit-identical."""
        from .dp import DataParallelLightGCNEngine

        self.engine = DataParallelLightGCNEngine(
            im.row.astype(np.int64), im.col.astype(np.int64), self.n_users, self.n_items, self.latent_dim,
            self.n_layers, self.reg_weight, lr=config["learning_rate"] or 1e-3, device=self.device,
            user_emb=u0.numpy(), item_emb=i0.numpy(), seed=int(config["seed"] or 0),
            batch=int(config["train_batch_size"]), chunk=int(config["rsx_chunk"] or 32), weight_decay=wd)
        self.steps_per_epoch = self.engine.steps_per_epoch()
        nu = self.n_users
        self.user_range = (rank * nu // world, (rank + 1) * nu // world)  # this rank's evaluation users
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
        if self.cpu:
            final = self.engine._prop(self.engine.norm_adj, self.get_ego_embeddings())
            return final[: self.n_users], final[self.n_users:]
        final = _Propagate.apply(self.embedding_dict["user_emb"], self.embedding_dict["item_emb"], self.engine)
        return final[: self.n_users], final[self.n_users:]

    def calculate_loss(self, interaction):
        if self.cpu:  # the same ops on CPU tensors (autograd reaches both parameters)
            return self.engine.loss(self.get_ego_embeddings(), interaction, self.engine.norm_adj)
        if self.sharded:
            raise NotImplementedError("the sharded LightGCN trains through fused_step_index (rsx.trainer's fused path)")
        self.engine.invalidate()
        final = _Propagate.apply(self.embedding_dict["user_emb"], self.embedding_dict["item_emb"], self.engine)
        return _BprLoss.apply(final, self.embedding_dict["user_emb"], self.embedding_dict["item_emb"],
                              interaction[:3].contiguous(), L.RSX_BPR_LIGHTGCN, float(self.reg_weight),
                              float(interaction.shape[1]), self.n_users, self.n_items)

    def _final(self):
        with torch.no_grad():
            return self.engine.forward()

    def full_sort_predict(self, interaction):
        if self.sharded:
            raise NotImplementedError("the sharded LightGCN evaluates through full_sort_topk_local")
        f = self._final()
        if self.cpu:  # reference lightgcn.py:158-166 on the CPU tables
            return torch.matmul(f[: self.n_users][interaction[0]], f[self.n_users:].t())
        return ops.score_dense(f[: self.n_users], interaction[0].contiguous(), f[self.n_users:])

    # -- rsx fast paths ----------------------------------------------------------
    def fused_step(self, interaction, lr: float):
        if self.sharded:
            raise NotImplementedError("the sharded LightGCN samples on the device: fused_step_index")
        self.engine.set_lr(lr)
        self.engine.step(triplets=interaction)

    def fused_step_index(self, epoch: int, i: int, lr: float):
        """Sharded training: this rank's batch i (of steps_per_epoch, the same count on every
        rank) of `epoch` from its device sampler."""
        self.engine.lr = float(lr)
        if self.dp:
            self.engine.step_index(epoch, i)
            return
        self.engine.step_slice(epoch, i, self.steps_per_epoch)

    def full_sort_topk_local(self, eval_users: torch.Tensor, k: int, eval_data):
        """(row positions in eval_users, top-k item ids) for this rank's evaluation users
        (global ids in [user_range)), ranked against every item with the training mask."""
        a, b = self.user_range
        pos = torch.nonzero((eval_users >= a) & (eval_users < b)).flatten()
        f = self._final()
        if self.dp:  # replicated tables: this rank's slice of the users, global ids
            nu = self.n_users
            users = eval_users.index_select(0, pos).contiguous()
            _, topk = ops.fullsort_topk(f[:nu], users, f[nu:], eval_data.mask_rowptr, eval_data.mask_col, k)
            return pos, topk
        local = (eval_users.index_select(0, pos) - a).contiguous()
        nl = b - a
        _, topk = ops.fullsort_topk(f[:nl], local, f[nl:], eval_data.mask_rowptr[a:], eval_data.mask_col, k)
        return pos, topk

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

    @property
    def device_halt(self):
        """(halt flag [2] int32 on the device, engine step count) of the single or
        data-parallel engine's step: {1, tag of the step} once a (global) batch loss was NaN
        (the parameters stay those of the last finite step; the tag is the engine's step
        count, so the Trainer reports the batch index), or None where the step has no flag
        (row-sharded engine)."""
        e = self.engine
        if getattr(self, "cpu", False) or (self.sharded and not getattr(self, "dp", False)):
            return None
        return e.halt, e.step_count
