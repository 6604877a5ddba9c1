"""Data-parallel LightGCN over several GPUs (one process per GPU; torch.distributed,
backend "nccl" = RCCL over xGMI on ROCm).

The reference trains one batch on one device (src/common/trainer.py:186-238,
src/utils/configurator.py:114-118).  Here every rank holds the whole graph and a
bit-identical replica of the embedding table and Adam moments; a step trains the
GLOBAL batch of every rank's triplets (rank r draws its own B): the reference
LightGCN objective at batch W*B (src/models/lightgcn.py:132-156: mean BPR over the
global batch, reg * (|U|_F + |P|_F + |N|_F) / (W B) with norms over the global batch).

Only the triplets are exchanged.  The propagation is replicated (on these graphs its
cost is per step, not per triplet), so once every rank knows every rank's triplets (one
all-gather of 48 KB per rank at B = 2048, hidden behind the forward) each rank evaluates
the whole global batch itself: the last layer on the union of the batch rows, the loss and
dL/dfinal of every triplet (accumulated per row in 64-bit fixed point: the sum cannot
depend on the order of the atomics), the backward and Adam (csrc/dp.hip).  Every rank runs
the same kernels on the same inputs, so the replicas stay bit-identical with no parameter
or gradient exchange.  (Round 4 all-gathered every rank's dL/dfinal rows instead: 1.6 MB
per rank on the critical path between the loss and the backward.)

The scaling this buys is the global batch's: a step costs about what one GPU's step of
batch B costs (the union's last layer and the global batch's loss grow with W), and
processes W B triplets.  Row sharding (rsx.dist.ShardedLightGCNEngine) splits the
propagation itself, and stays the choice when the graph is too large to propagate on
every rank in time (C4's strong-scaling leg).

Epochs: the epoch's interactions (one device-sampled stream, the same seed on every
rank) cut into S * W balanced slices, S = ceil(E / (W B)); step j of rank r trains
slice j W + r, so the global batch of step j is slices [j W, (j+1) W) and every
interaction is visited once per epoch.

`backend="torch"` runs a CPU restatement of the same sequence (gloo tests): the
triplet all-gather, then the global batch's loss and gradient on every rank.
"""
from __future__ import annotations

import ctypes as C
import gc
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from . import ops


def _comm_init(group, device, views, sim=None):
    """An rsx communicator over `group`: RCCL ("nccl": unique-id handshake) or, on any
    other backend (gloo: tests, several ranks on one GPU), the host hook that runs each
    collective on host copies of the registered device buffers `views` ({ptr: flat});
    with `sim` (rsx.dist.sim_comm_params, a one-rank group) the latency-injected stand-in."""
    lib = L.lib()
    comm = C.c_void_p()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if sim is not None:
        if world != 1:
            raise RuntimeError("RSX_COMM_SIM models a multi-rank job on ONE rank (world 1)")
        with torch.cuda.device(device):
            L.check(lib.rsx_comm_init_sim(C.byref(comm), sim["world"], sim["busbw_gbs"], sim["latency_us"],
                                          sim["blocks"], sim["scratch_mb"]), "rsx_comm_init_sim")
        return comm, None
    if dist.get_backend(group) == "nccl":
        nb = int(lib.rsx_comm_unique_id_bytes())
        buf = (C.c_uint8 * nb)()
        if rank == 0:
            L.check(lib.rsx_comm_get_unique_id(buf), "rsx_comm_get_unique_id")
        uid = torch.tensor(bytearray(bytes(buf)), dtype=torch.uint8, device=device)
        dist.broadcast(uid, src=dist.get_global_rank(group, 0) if group else 0, group=group)
        C.memmove(buf, bytes(uid.cpu().numpy().tobytes()), nb)
        with torch.cuda.device(device):
            L.check(lib.rsx_comm_init(C.byref(comm), buf, rank, world), "rsx_comm_init")
        return comm, None

    def host_collective(op, ptr, count, dtype, _ctx):
        try:
            v = views[ptr]
            if op != L.RSX_COLL_ALLGATHER:
                raise ValueError(op)
            mine = v[rank * count:(rank + 1) * count].cpu()
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine, group=group)
            v[: world * count].copy_(torch.cat(parts))
            return 0
        except Exception:  # noqa: BLE001
            return 1

    cb = L.HOST_COLLECTIVE_FN(host_collective)
    L.check(lib.rsx_comm_init_host(C.byref(comm), rank, world, cb, None), "rsx_comm_init_host")
    return comm, cb


class DataParallelLightGCNEngine:
    """LightGCN with the graph and tables replicated on every rank, the global batch split."""

    def __init__(self, train_u: np.ndarray, train_i: np.ndarray, n_users: int, n_items: int, dim: int,
                 n_layers: int, reg: float, lr: float, device, user_emb: np.ndarray, item_emb: np.ndarray,
                 seed: int = 0, batch: int = 2048, chunk: int = 32, weight_decay: float = 0.0, group=None,
                 backend: str = "hip"):
        if not 2 <= n_layers <= 4:
            raise RuntimeError("the data-parallel LightGCN step is the stored-layer step: n_layers 2..4")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = backend
        self.n_users, self.n_items, self.d, self.K = int(n_users), int(n_items), int(dim), int(n_layers)
        self.reg, self.lr, self.wd = float(reg), float(lr), float(weight_decay)
        self.batch = self.cap = int(batch)
        nu, ni, d = self.n_users, self.n_items, self.d
        n = nu + ni
        tu = np.asarray(train_u, dtype=np.int64)
        ti = np.asarray(train_i, dtype=np.int64)
        # every rank starts from rank 0's tables (replicas bit-identical from step 0)
        p0 = torch.from_numpy(np.ascontiguousarray(np.concatenate([user_emb, item_emb]), dtype=np.float32))
        self.loss_acc_host = 0.0
        self.step_count = 0
        if backend == "torch":
            self._init_torch(tu, ti, p0)
            return
        self.device = ops.require_device(device)
        dev = self.device
        p0 = self._bcast(p0.to(dev))
        from .engine import lightgcn_adj

        self.adj = lightgcn_adj(tu, ti, nu, ni, dev, chunk)
        self.p = p0
        z = lambda: torch.zeros(n, d, dtype=torch.float32, device=dev)  # noqa: E731
        self.m, self.v, self.h0, self.h1, self.final, self.g = z(), z(), z(), z(), z(), z()
        self.s = z() if self.K == 4 else None
        self.row_tag = torch.zeros(n, dtype=torch.int32, device=dev)
        self.reg_cnt = torch.zeros(3 * n + 4, dtype=torch.int32, device=dev)
        self.halt = torch.zeros(2, dtype=torch.int32, device=dev)
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self._step_dev = torch.zeros(1, dtype=torch.int64, device=dev)  # Adam's step; its low word = the tag
        lib = L.lib()
        # latency injection (RSX_COMM_SIM=W on a one-rank group, csrc/dp.hip): rank 0 of a
        # modelled W-rank job, its slots and workspace sized for W ranks
        from .dist import sim_comm_params

        self.sim = sim_comm_params() if self.world == 1 else None
        W, cap = (self.sim["world"] if self.sim else self.world), self.cap
        self.model_world = W
        self.slots = torch.zeros(W * (3 * cap + 1), dtype=torch.int64, device=dev)
        # the step's workspace: fixed-point G' accumulators, the occurrence sort, loss partials
        self.work = torch.zeros(int(lib.rsx_dp_work_bytes(n, d, cap, W)), dtype=torch.uint8, device=dev)
        self.sampler = ops.DeviceSampler(tu, ti, nu, dev, seed=seed)
        self.n_inter = self.sampler.n_inter
        self._epoch_buf = None
        self._epoch_key = None
        self._views = {self.slots.data_ptr(): self.slots}
        self._comm, self._host_cb = _comm_init(group, dev, self._views, self.sim)
        if self.sim:
            self._fill_peer_slots()
        st = self._st = L.DpStep()
        st.adj = C.pointer(self.adj.struct)
        st.n_users, st.n_items, st.d, st.n_layers, st.reg = nu, ni, d, self.K, self.reg
        for name in ("p", "m", "v", "h0", "h1", "g"):
            setattr(st, name, getattr(self, name).data_ptr())
        st.s = self.s.data_ptr() if self.s is not None else None
        st.final_emb = self.final.data_ptr()
        slab = self.adj.slab(d)
        st.slab = slab.data_ptr() if slab is not None else None
        st.loss_out, st.loss_acc = self.loss_out.data_ptr(), self.loss_acc.data_ptr()
        st.comm = self._comm.value
        st.row_tag = self.row_tag.data_ptr()
        st.tag_dev = self._step_dev.data_ptr()
        st.inc_step = 1  # dp_pack increments the counter (no separate add launch a step)
        st.reg_cnt, st.halt = self.reg_cnt.data_ptr(), self.halt.data_ptr()
        st.cap = cap
        st.slots = self.slots.data_ptr()
        st.work, st.work_bytes = self.work.data_ptr(), self.work.numel()
        # issued eagerly by default: the step is one C-ABI call of ~14 launches, and a replayed
        # graph measured slower (one real RCCL rank 0.201 vs 0.178 ms a step; latency-injected
        # W = 2 / 8: 0.206 / 0.234 vs 0.202 / 0.232, profiles/r05/dp/eager_vs_graph/): its
        # RCCL node, its per-step triplet copy into the captured buffer and the cross-queue
        # start of its forward branch.  RSX_DP_GRAPH=1 captures it.
        self.use_graph = dist.get_backend(group) == "nccl" and os.environ.get("RSX_DP_GRAPH", "0") == "1"
        self._graphs = {}
        self._warm = set()
        self._fwd_valid = False

    # ------------------------------------------------------------------ helpers
    def _bcast(self, t):
        if dist.get_backend(self.group) == "nccl":
            dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group else 0, group=self.group)
            return t
        h = t.cpu()
        dist.broadcast(h, src=0, group=self.group)
        return h.to(t.device)

    def _fill_peer_slots(self):
        """Latency injection: the modelled job's other ranks' slots, once — ranks 1..W-1
        train slices 1..W-1 of epoch 0 cut into batch-sized balanced slices (a batch each,
        as in the job), so the step indexes, merges and back-propagates a global batch of
        the job's size and union (a timing mode: those ranks' own steps are not run)."""
        W, cap, L_ = self.model_world, self.cap, 3 * self.cap + 1
        n = max(W, -(-self.n_inter // cap))
        buf = self.sampler.sample_epoch_slices(0, n)
        for r in range(1, W):
            t = ops.DeviceSampler.slice_view(buf, self.n_inter, n, r)
            b = int(t.shape[1])
            slot = self.slots[r * L_:(r + 1) * L_]
            slot[0] = b
            slot[1:].view(3, cap)[:, :b].copy_(t[:3])
        torch.cuda.synchronize(self.device)

    def steps_per_epoch(self) -> int:
        return -(-self.n_inter // (self.world * self.batch))

    # ------------------------------------------------------------------- steps
    def step_index(self, epoch: int, j: int):
        """Step j of `epoch`: this rank trains slice j W + rank of the epoch cut into S W
        balanced slices (S = steps_per_epoch(); every rank the same stream)."""
        S = self.steps_per_epoch()
        key = (epoch, S)
        if self._epoch_key != key:
            self._epoch_buf = self.sampler.sample_epoch_slices(epoch, S * self.world, out=self._epoch_buf)
            self._epoch_key = key
        self.step(ops.DeviceSampler.slice_view(self._epoch_buf, self.n_inter, S * self.world,
                                               j * self.world + self.rank))

    def step(self, triplets: torch.Tensor):
        """One global batch: this rank's triplets [3, B] (B <= the engine's batch)."""
        self.step_count += 1
        if self.backend == "torch":
            return self._torch_step(triplets)
        B = int(triplets.shape[1])
        if not 1 <= B <= self.cap:
            raise RuntimeError(f"batch {B} outside [1, {self.cap}]")
        lib, st = L.lib(), self._st
        st.adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd, step_dev=self._step_dev)
        cap = self._graphs.get(B)
        if cap is not None and cap[1] == self.lr:
            cap[2].copy_(triplets)
            cap[0].replay()
            self._fwd_valid = False
            return
        if self.use_graph and B in self._warm:
            buf = cap[2] if cap is not None else torch.zeros(3, B, dtype=torch.int64, device=self.device)
            buf.copy_(triplets)
            st.triplets, st.batch = buf.data_ptr(), B
            g = torch.cuda.CUDAGraph()
            gc_on = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g):
                    L.check(lib.rsx_dp_lightgcn_step(C.byref(st), ops._stream()), "rsx_dp_lightgcn_step")
            except Exception:  # noqa: BLE001  capture refused: eager from now on
                self.use_graph = False
                torch.cuda.synchronize()
            else:
                self._graphs[B] = (g, self.lr, buf)
                g.replay()
                self._fwd_valid = False
                return
            finally:
                if gc_on:
                    gc.enable()
        t = triplets[:3].contiguous()
        self._keep = t
        st.triplets, st.batch = t.data_ptr(), B
        L.check(lib.rsx_dp_lightgcn_step(C.byref(st), ops._stream()), "rsx_dp_lightgcn_step")
        self._warm.add(B)
        self._fwd_valid = False

    def forward(self) -> torch.Tensor:
        """final = mean_k A^k E^0 on this rank's replica (evaluation)."""
        if self.backend == "torch":
            return self._torch_forward()
        if not self._fwd_valid:
            s = self.s if self.s is not None else torch.empty_like(self.p)
            slab = self.adj.slab(self.d)
            L.check(L.lib().rsx_lightgcn_forward(C.byref(self.adj.struct), self.d, self.K, ops._p(self.p),
                                                 ops._p(s), ops._p(self.h0), ops._p(self.h1), ops._p(self.final),
                                                 ops._p(slab), ops._stream()), "rsx_lightgcn_forward")
            self._fwd_valid = True
        return self.final

    def invalidate(self):
        self._fwd_valid = False

    def close(self):
        if getattr(self, "_comm", None) is not None and self.backend != "torch":
            self._graphs = {}
            torch.cuda.synchronize(self.device)
            L.lib().rsx_comm_destroy(self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------- CPU restatement (gloo tests)
    def _init_torch(self, tu, ti, p0):
        """The step of csrc/dp.hip in torch on the CPU: same decomposition, same exchanges
        (gloo all-gathers), same merge order."""
        from . import graph

        nu, ni = self.n_users, self.n_items
        rp, col, val = graph.lightgcn_norm_adj(tu, ti, nu, ni)
        rows = np.repeat(np.arange(nu + ni), np.diff(rp))
        self.A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])),
                                         torch.from_numpy(val), (nu + ni, nu + ni)).coalesce()
        dist.broadcast(p0, src=0, group=self.group)
        self.p = p0.clone()
        self.m, self.v = torch.zeros_like(self.p), torch.zeros_like(self.p)
        self.loss_out = torch.zeros(1)

    def _torch_layers(self):
        xs = [self.p]
        for _ in range(self.K):
            xs.append(torch.sparse.mm(self.A, xs[-1]))
        return xs

    def _torch_forward(self):
        xs = self._torch_layers()
        acc = xs[0]
        for x in xs[1:]:
            acc = acc + x
        return acc / (self.K + 1)

    def _torch_step(self, trip):
        W, nu, K = self.world, self.n_users, self.K
        trip = trip[:3].long()
        # (1) every rank's triplets: the step's only exchange
        counts = [torch.zeros(1, dtype=torch.int64) for _ in range(W)]
        dist.all_gather(counts, torch.tensor([trip.shape[1]]), group=self.group)
        cap = int(max(c.item() for c in counts))
        pad = torch.zeros(3, cap, dtype=torch.int64)
        pad[:, : trip.shape[1]] = trip
        trips = [torch.zeros_like(pad) for _ in range(W)]
        dist.all_gather(trips, pad, group=self.group)
        glob = torch.cat([t[:, : int(c.item())] for t, c in zip(trips, counts)], 1)
        Bg = float(glob.shape[1])
        # (2) forward; (3) the GLOBAL batch's loss and G' = dL/dfinal / (K+1), on every rank
        final = self._torch_forward()
        f = final.clone().requires_grad_(True)
        u, pi, ni_ = glob[0], glob[1] + nu, glob[2] + nu
        sg = torch.sigmoid((f[u] * f[pi]).sum(1) - (f[u] * f[ni_]).sum(1))
        (-torch.log(1e-10 + sg)).sum().div(Bg).backward()
        G = f.grad / (K + 1)
        e = self.p
        tl = float((-torch.log(1e-10 + sg.detach())).double().sum())
        nrm = torch.tensor([float((e[x].double() ** 2).sum()) for x in (u, pi, ni_)], dtype=torch.float64).sqrt()
        loss = tl / Bg + self.reg * float(nrm.sum()) / Bg
        self.loss_out[0] = float(loss)
        self.loss_acc_host += float(loss)
        k = [float(self.reg / (Bg * x)) if x > 0 else 0.0 for x in nrm.tolist()]
        cnt = torch.zeros(self.p.shape[0], 3)
        for kind, ids in enumerate((u, pi, ni_)):
            cnt[:, kind].index_add_(0, ids, torch.ones(ids.numel()))
        R = (cnt[:, 0:1] * k[0] + cnt[:, 1:2] * k[1] + cnt[:, 2:3] * k[2]) * self.p
        # (5) backward: H = G' + A H from H = G', g = H^K + R; Adam
        H = G
        for _ in range(K):
            H = G + torch.sparse.mm(self.A, H)
        g = H + R
        step = self.step_count
        self.m.mul_(0.9).add_(g, alpha=0.1)
        self.v.mul_(0.999).addcmul_(g, g, value=0.001)
        bc1, bc2 = 1 - 0.9 ** step, 1 - 0.999 ** step
        self.p.sub_((self.lr / bc1) * self.m / (self.v.sqrt() / (bc2 ** 0.5) + 1e-8))
