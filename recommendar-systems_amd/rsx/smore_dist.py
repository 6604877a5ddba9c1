"""SMORE sharded over the ranks of a process group ("the same
scheme ... shard the projection by item rows and all-gather the projected NI x d").

Partition: users and items are split into contiguous per-rank ranges; a rank owns
its users' and items' rows of every table — the user and item-id embeddings and
the raw image / text feature tables (Embedding.from_pretrained(freeze=False): the
largest parameters, 7050 x 4096 at Amazon-baby).  The small weights (projections,
gates, query MLPs, spectral filters) are replicated and their gradients summed.

Forward (reference src/models/smore.py:256-349), per rank:
  * projection + spectral fusion and the modality gates on its own item rows
    (row-local, smore.py:256-272);
  * the UI backbone, n_ui_layers times: all-gather the [users; items] table, multiply
    by this rank's rows of the normalised adjacency (smore.py:276-287);
  * each item view: all-gather the item rows, multiply by this rank's rows of the
    kNN graph, n_layers times; then this rank's users through R (smore.py:289-317);
  * the preference block on its own rows (smore.py:320-341).
Loss: the all_embeds / side / content tables are all-gathered and every rank
evaluates the reference loss on the whole batch (BPR + regulariser + both InfoNCE
terms, smore.py:352-411), scaled by 1/W: the gathers' backward (an all-reduce of the
full gradient, then this rank's slice) sums the W copies into exactly the
single-process gradient of the owned rows; `sync_grads` sums the replicated
weights' gradients.  One step therefore equals the single-process step (the
gloo tests compare them), up to f32 summation order.

The gather is an autograd Function over torch.distributed (all_gather forward,
all_reduce + slice backward: works over gloo and RCCL; device tensors over gloo
travel through host copies).  Compute goes through a backend: `HipSmoreBackend`
(the rsx kernels: fused spectral pass, gates, preference, InfoNCE, SpMM, BPR) or
a torch restatement (tests on the CPU).  Dropout masks (p > 0) are drawn per local
row, so they differ from a single-process run's (same distribution).

Evaluation: each rank ranks its own users against the gathered item table
(`full_sort_topk_local`); rsx.evaluator.sharded_metric_dict all-gathers the sums.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import _lib as L
from . import graph, ops

# parameters split by rows: (name, "u" users | "i" items)
SHARDED = {"user_embedding.weight": "u", "item_id_embedding.weight": "i", "image_embedding.weight": "i",
           "text_embedding.weight": "i"}


def ranges(n: int, world: int):
    return [(r * n // world, (r + 1) * n // world) for r in range(world)]


def _host_if_gloo(t, group):
    return t.cpu() if (t.is_cuda and dist.get_backend(group) != "nccl") else t


class _Gather(torch.autograd.Function):
    """x = this rank's rows [a_r, b_r) -> the full [n, ...] table (all ranks' rows in
    rank order); backward: the full gradient all-reduced, this rank's slice."""

    @staticmethod
    def forward(ctx, x, rng, group):
        r = dist.get_rank(group)
        mx = max(b - a for a, b in rng)
        buf = x.new_zeros((mx,) + tuple(x.shape[1:]))
        buf[: x.shape[0]] = x
        hb = _host_if_gloo(buf, group)
        parts = [torch.empty_like(hb) for _ in rng]
        dist.all_gather(parts, hb.contiguous(), group=group)
        full = torch.cat([p[: b - a] for p, (a, b) in zip(parts, rng)]).to(x.device)
        ctx.rng, ctx.r, ctx.group = rng, r, group
        return full

    @staticmethod
    def backward(ctx, g):
        h = _host_if_gloo(g.contiguous(), ctx.group).clone()
        dist.all_reduce(h, group=ctx.group)
        a, b = ctx.rng[ctx.r]
        return h[a:b].to(g.device), None, None


def gather(x, rng, group=None):
    return _Gather.apply(x, rng, group)


def csr_rows(rowptr, col, val, r0: int, r1: int):
    """Rows [r0, r1) of a host CSR (columns unchanged)."""
    a, b = int(rowptr[r0]), int(rowptr[r1])
    return rowptr[r0:r1 + 1] - a, col[a:b], val[a:b]


def stack_csr(*blocks):
    """Row-concatenation of host CSR blocks with the same columns."""
    rps, cols, vals, off = [np.zeros(1, np.int64)], [], [], 0
    for rp, c, v in blocks:
        rps.append(rp[1:] + off)
        off += int(rp[-1])
        cols.append(c)
        vals.append(v)
    return np.concatenate(rps), np.concatenate(cols), np.concatenate(vals)


# ---------------------------------------------------------------------------
# backends
# ---------------------------------------------------------------------------
class HipSmoreBackend:
    """The rsx kernels (the single-process rsx.smore.SMORE's path)."""

    def __init__(self, device, chunk=32):
        self.device = ops.require_device(device)
        self.chunk = chunk

    def operator(self, rowptr, col, val, n_cols):
        """(A, A^T) device CSRs of a local row block (the backward multiplies by A^T)."""
        n_rows = rowptr.size - 1
        A = ops.DeviceCSR(rowptr, col, val, n_cols, self.device, self.chunk)
        rows = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(rowptr))
        AT = ops.DeviceCSR(*graph.to_csr(col.astype(np.int64), rows, val, n_cols, n_rows), n_rows, self.device,
                           self.chunk)
        return A, AT

    def spmm(self, op, x):
        from .smore import _SpMM

        return _SpMM.apply(x, op[0], op[1])

    def spectral(self, m, V, T):
        from .smore_spectral import spectral

        return spectral(V, m.image_trs.weight, m.image_trs.bias, T, m.text_trs.weight, m.text_trs.bias,
                        m.image_complex_weight, m.text_complex_weight, m.fusion_complex_weight, True)[:3]

    def gates(self, m, cv, ct, cf, item):
        from . import smore_fuse as SF

        return SF.gates(cv, ct, cf, item, m.gate_v, m.gate_t, m.gate_f, m.inject_scale, False)

    def preference(self, m, C, IE, TE, FE):
        from . import smore_fuse as SF

        return SF.preference(m, C, IE, TE, FE, m._seed)

    def loss(self, m, all_e, side, content, inter):
        from . import smore_fuse as SF
        from .lightgcn import _BprLoss

        nu = m.n_users
        bpr = _BprLoss.apply(all_e, None, None, inter[:3].contiguous(), L.RSX_BPR_SMORE, float(m.reg_weight),
                             float(m.batch_size), nu, m.n_items)
        ci, cu = SF.infonce2(side, content, inter[0].contiguous(), inter[1].contiguous(), nu, m.cl_temp)
        return bpr + m.cl_loss * (ci + cu)

    def mean_layers(self, layers):
        return torch.stack(layers, dim=1).mean(dim=1)


# ---------------------------------------------------------------------------
# the sharded model
# ---------------------------------------------------------------------------
class ShardedSMORE(nn.Module):
    """SMORE over the process group; parameters named as the reference's, the
    row-sharded ones holding this rank's rows (see the module docstring)."""

    def __init__(self, params: dict, graphs: dict, n_users: int, n_items: int, cfg: dict, backend, group=None):
        super().__init__()
        self.group = group
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.be = backend
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.urng, self.irng = ranges(self.n_users, self.world), ranges(self.n_items, self.world)
        (ua, ub), (ia, ib) = self.urng[self.rank], self.irng[self.rank]
        self.own_u, self.own_i = (ua, ub), (ia, ib)
        self.reg_weight = float(cfg.get("reg_weight", 1e-5))
        self.cl_loss = float(cfg.get("cl_loss", 0.01))
        self.cl_temp = float(cfg.get("cl_temp", 0.2))
        self.batch_size = float(cfg.get("batch_size", 2048))
        self.n_ui_layers = int(cfg.get("n_ui_layers", 4))
        self.n_layers = int(cfg.get("n_layers", 1))
        self.inject_scale = float(cfg.get("inject_scale", 0.7))
        d = params["user_embedding.weight"].shape[1]
        dev = getattr(backend, "device", torch.device("cpu"))
        mods = {}
        for name, full in params.items():  # nn containers in the reference's layout
            full = torch.as_tensor(full, dtype=torch.float32)
            part = SHARDED.get(name)
            if part == "u":
                full = full[ua:ub]
            elif part == "i":
                full = full[ia:ib]
            mods[name] = nn.Parameter(full.clone().to(dev))
        self.user_embedding = nn.Module()
        self.item_id_embedding = nn.Module()
        self.image_embedding = nn.Module()
        self.text_embedding = nn.Module()
        lin = lambda i, o, b=True: nn.Linear(i, o, bias=b, device=dev)  # noqa: E731
        dv, dt = params["image_trs.weight"].shape[1], params["text_trs.weight"].shape[1]
        self.image_trs, self.text_trs = lin(dv, d), lin(dt, d)
        self.query_v = nn.Sequential(lin(d, d), nn.Tanh(), lin(d, d, False))
        self.query_t = nn.Sequential(lin(d, d), nn.Tanh(), lin(d, d, False))
        for g in ("gate_v", "gate_t", "gate_f", "gate_image_prefer", "gate_text_prefer", "gate_fusion_prefer"):
            setattr(self, g, nn.Sequential(lin(d, d), nn.Sigmoid()))
        self.dropout = nn.Dropout(p=float(cfg.get("dropout_rate", 0.0)))
        for name, p in mods.items():  # the given values replace the fresh modules' parameters
            obj = self
            *path, leaf = name.split(".")
            for k in path:
                obj = obj[int(k)] if k.isdigit() else getattr(obj, k)
            obj._parameters.pop(leaf, None)
            obj.register_parameter(leaf, p)
        self._seed = torch.tensor([int(cfg.get("seed", 999)) * 1000003 + 17 + self.rank], dtype=torch.int64,
                                  device=dev)
        # this rank's rows of every operator: UI adjacency (own users, then own items; all
        # N columns), each kNN graph (own items; item columns), R (own users; item columns)
        nu, ni = self.n_users, self.n_items
        rp, col, val = graphs["norm_adj"]
        ui = stack_csr(csr_rows(rp, col, val, ua, ub), csr_rows(rp, col, val, nu + ia, nu + ib))
        self.A_ui = backend.operator(*ui, nu + ni)
        self.G = {}
        for v in ("image", "text", "fusion"):
            grp, gcol, gval = graphs[v]
            self.G[v] = backend.operator(*csr_rows(grp, gcol, gval, ia, ib), ni)
        rrp, rcol, rval = graphs["R"]
        self.R = backend.operator(*csr_rows(rrp, rcol, rval, ua, ub), ni)

    # -- gathers ----------------------------------------------------------------
    def _users(self, x):
        return gather(x, self.urng, self.group)

    def _items(self, x):
        return gather(x, self.irng, self.group)

    def _table(self, x):
        """[own users; own items] -> the full [users; items] table."""
        nu_own = self.own_u[1] - self.own_u[0]
        return torch.cat([self._users(x[:nu_own]), self._items(x[nu_own:])])

    # -- forward ----------------------------------------------------------------
    def forward_local(self):
        """(all_embeds, side, content) of this rank's rows [own users; own items]."""
        be = self.be
        cv, ct, cf = be.spectral(self, self.image_embedding.weight, self.text_embedding.weight)
        item = self.item_id_embedding.weight
        img, txt, fus = be.gates(self, cv, ct, cf, item)
        x = torch.cat([self.user_embedding.weight, item])
        layers = [x]
        for _ in range(self.n_ui_layers):
            x = be.spmm(self.A_ui, self._table(x))
            layers.append(x)
        content = be.mean_layers(layers)
        views = []
        for v, xi in (("image", img), ("text", txt), ("fusion", fus)):
            for _ in range(self.n_layers):
                xi = be.spmm(self.G[v], self._items(xi))
            views.append(torch.cat([be.spmm(self.R, self._items(xi)), xi]))
        all_e, side = be.preference(self, content, *views)
        return all_e, side, content

    def calculate_loss(self, interaction):
        """1/W of the reference loss of the whole batch (every rank holds the same batch)."""
        all_e, side, content = self.forward_local()
        return self.be.loss(self, self._table(all_e), self._table(side), self._table(content),
                            interaction) / self.world

    def replicated_parameters(self):
        return [p for n, p in self.named_parameters() if n not in SHARDED]

    @torch.no_grad()
    def sync_grads(self):
        """Sum the replicated weights' gradients over the ranks (each rank's covers its rows)."""
        for p in self.replicated_parameters():
            if p.grad is None:
                continue
            h = _host_if_gloo(p.grad, self.group).clone()
            dist.all_reduce(h, group=self.group)
            p.grad.copy_(h.to(p.grad.device))

    # -- training with the model-level mirror gradient ----------------------------
    @torch.no_grad()
    def mg_alpha(self, params, grads, base, lr, rel_step, max_scale):
        """alpha_eff of the reference's mirror gradient (src/common/trainer.py:290-307)
        over the GLOBAL parameter vector: sums of squares of the row-sharded tensors
        all-reduced, the replicated ones counted once, then the reference's arithmetic
        (rms values rounded to f32 as its float() of f32 tensors, the rest in f64)."""
        dev = params[0].device
        sh = torch.zeros(3, dtype=torch.float64, device=dev)  # sum g^2, sum p^2, numel (sharded)
        rep = torch.zeros(3, dtype=torch.float64, device=dev)
        names = {id(p): n for n, p in self.named_parameters()}
        for p, g in zip(params, grads):
            acc = sh if names.get(id(p)) in SHARDED else rep
            acc[0] += g.double().pow(2).sum()
            acc[1] += p.detach().double().pow(2).sum()
            acc[2] += p.numel()
        h = _host_if_gloo(sh, self.group).clone()
        dist.all_reduce(h, group=self.group)
        tot = h.to(dev) + rep
        n = float(tot[2].item())
        grad_rms = float(torch.tensor(float(tot[0].sqrt()), dtype=torch.float32) / (n ** 0.5))
        param_rms = float(torch.tensor(float(tot[1].sqrt()), dtype=torch.float32) / (n ** 0.5) + 1e-12)
        alpha = max(base, rel_step * param_rms / (lr * grad_rms + 1e-12))
        return min(alpha, base * max_scale)

    def train_batch(self, inter, opt, lr, step_id, mg_interval=3, mg_alpha=0.5, mg_beta=0.2, rel_step=1e-3,
                    max_scale=20.0):
        """One batch of the reference Trainer on a mirror-gradient model (src/common/
        trainer.py:186-201, 244-336) over the process group: loss, backward, gradient
        sync, Adam; then, when step_id % mg_interval == 0, the mirror gradient: g(theta)
        again, theta' = theta - alpha lr g, g(theta') scaled by -beta, theta restored,
        Adam.  `opt` holds this rank's parameters (Adam is per element, so the sharded
        rows' update is the single-process update of those rows).  Returns 1/W of the
        batch loss (a float)."""
        opt.zero_grad(set_to_none=True)
        loss = self.calculate_loss(inter)
        value = float(loss.detach())
        loss.backward()
        self.sync_grads()
        opt.step()
        if mg_interval > 0 and step_id % mg_interval == 0:
            opt.zero_grad(set_to_none=True)
            self.calculate_loss(inter).backward()
            self.sync_grads()
            params = [p for p in self.parameters() if p.requires_grad and p.grad is not None]
            grads = [p.grad.detach().clone() for p in params]
            alpha = self.mg_alpha(params, grads, mg_alpha, lr, rel_step, max_scale)
            with torch.no_grad():
                for p, g in zip(params, grads):
                    p.add_(-alpha * lr * g)
            opt.zero_grad(set_to_none=True)
            self.calculate_loss(inter).backward()
            self.sync_grads()
            with torch.no_grad():
                for p in self.parameters():
                    if p.requires_grad and p.grad is not None:
                        p.grad.mul_(-mg_beta)
                for p, g in zip(params, grads):
                    p.add_(+alpha * lr * g)
            opt.step()
            opt.zero_grad(set_to_none=True)
        return value

    @torch.no_grad()
    def full_sort_topk_local(self, k: int, mask_rowptr, mask_col):
        """Top-k item ids of this rank's users (global user ids ua..ub-1, in order)."""
        all_e, _, _ = self.forward_local()
        nu_own = self.own_u[1] - self.own_u[0]
        items = self._items(all_e[nu_own:].contiguous())
        users = torch.arange(nu_own, device=all_e.device)
        return ops.fullsort_topk(all_e[:nu_own].contiguous(), users, items.contiguous(),
                                 mask_rowptr[self.own_u[0]:], mask_col, k)[1]


def graphs_from_rsx(model):
    """Host CSRs of a single-process rsx.smore.SMORE's operators (for ShardedSMORE)."""
    def host(A):
        return A.rowptr_host, A.col.cpu().numpy(), A.val.cpu().numpy()

    return {"norm_adj": host(model.norm_adj_csr), "image": host(model.image_graph.A),
            "text": host(model.text_graph.A), "fusion": host(model.fusion_graph.A), "R": host(model.R.A)}
