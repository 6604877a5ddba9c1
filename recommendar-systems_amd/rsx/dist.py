"""Row-sharded LightGCN over several GPUs (one process per GPU; torch.distributed,
backend "nccl" = RCCL over xGMI on ROCm).

The reference is single-process, single-device ("Parallelism
strategies: none"); this is the build's scaling axis for graph size.

Partitioning.  A = [[0, R], [R^T, 0]] is bipartite, so with users split into
contiguous per-rank blocks U_g and the item rows replicated:
    users^k = R_g items^{k-1}           (local: items^{k-1} is replicated)
    items^k = sum_g R_g^T users_g^{k-1} (each rank computes its partial, then
                                         one all-reduce of the [n_items, d] block)
Per propagation layer the item-row SpMM runs first and its all-reduce is
issued asynchronously; the user-row SpMM of the same layer (which only needs
the previous, already reduced items) runs on the compute stream meanwhile, and
so does the NEXT layer's item partial (it needs only this layer's users), whose
exchange is queued behind this one: the comm stream runs the exchanges back to
back.  The backward is the same layer sums on G = dL/dfinal with the same
exchange (G's per-rank item rows are reduced first, queued together with layer
1's partial); the item-side gradient and the last layer's partial are reduced
together, so a K-layer step issues 2K+1 all-reduces of n_items*d floats.  Adam runs on every rank: user rows locally, item rows identically on
each replica (the reduced inputs are bit-identical on all ranks).

Normalisation uses GLOBAL item degrees (one all-reduce of a degree vector at
construction), so every value equals the single-GPU graph's bit for bit
(float64 product, cast to f32, reference src/models/lightgcn.py:93-99).

Objective.  Each rank draws B triplets from its own users' interactions; the
step minimises the sum of the per-rank reference losses (mean BPR over each
rank's batch + its EmbLoss term), i.e. data-parallel batches of B per GPU.

The compute primitives come from a backend: `HipBackend` (the product: HIP
kernels through the C ABI) — tests substitute a CPU restatement to check the
partitioning and the collectives with the gloo backend on CPU.

Native step.  With the HIP backend over RCCL ("nccl" process group) the whole
step is one C-ABI call, `rsx_sharded_lightgcn_step` (csrc/dist.hip): the same
sequence as `_propagate` / `step` below, issued from C++ on the compute stream
with the exchanges on the rsx communicator's own stream (an RCCL communicator
created by the unique-id handshake over this process group).  Issued from
Python, the ~20 launches + 7 collectives of a step cost more host time than the
device needs for them (0.46 ms/step vs 0.16 ms at N=1, bench --sharded); the
Python sequence remains the statement the gloo tests check and the fallback
when `native=False`.  For K = 2, 3 the native step is the stored-layer form
(csrc/dist.hip:sharded_stored_layers): no layer-sum passes, the last user layer
on the batch rows only, the backward as Horner on G/(K+1) with rank 0 adding the
summed G'_I into its item partials and every rank its own regulariser rows into
the last one — 2K SpMM launches + one item Adam per step instead of 2K SpMMs +
2K row-block sums.  Over RCCL it is captured once as a HIP graph and replayed
(`_native_step`).  With a non-RCCL group
(gloo, tests) the native step's exchanges go through a host hook
(`rsx_comm_init_host`) so several ranks can share one GPU.
"""
from __future__ import annotations

import ctypes as C
import gc
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from . import graph, ops


class HipBackend:
    """Product backend: rsx HIP kernels on the current torch stream."""

    def __init__(self, device):
        self.device = ops.require_device(device)

    def tensor(self, a):
        return torch.as_tensor(a).to(self.device)

    def zeros(self, rows, d):
        return torch.zeros(rows, d, dtype=torch.float32, device=self.device)

    def csr(self, rowptr, col, val, n_cols, chunk=32):
        return ops.DeviceCSR(rowptr, col, val, n_cols, self.device, chunk)

    def spmm(self, A, x, d, kind, alpha=1.0, beta=1.0, adam=None, **t):
        A.spmm_epi(x, ops.epi(kind, alpha, beta, adam=adam, **t), d)

    def rowwise(self, n, d, kind, alpha=1.0, beta=1.0, adam=None, **t):
        ops.rowwise(n, d, ops.epi(kind, alpha, beta, adam=adam, **t))

    def adam(self, lr, step, weight_decay=0.0):
        return ops.adam_struct(lr, step, weight_decay=weight_decay)

    def bpr(self, fin, ego, nu, ni, trip, reg, g, r, loss_acc):
        loss, _, _ = ops.bpr(L.RSX_BPR_LIGHTGCN, fin, ego, nu, ni, trip, reg, g_final=g, g_ego=r,
                             loss_acc=loss_acc)
        return loss

    def sampler(self, train_u, train_i, n_users, seed):
        return ops.DeviceSampler(train_u, train_i, n_users, self.device, seed=seed)


class ShardedLightGCNEngine:
    """LightGCN with users row-sharded over the process group, items replicated."""

    def __init__(self, train_u: np.ndarray, train_i: np.ndarray, n_users: int, n_items: int, dim: int,
                 n_layers: int, reg: float, lr: float, device, user_emb: np.ndarray, item_emb: np.ndarray,
                 seed: int = 0, batch: int = 2048, chunk: int = 32, weight_decay: float = 0.0, group=None,
                 backend=None, native: bool | None = None):
        if n_layers < 1:
            raise RuntimeError("sharded LightGCN needs n_layers >= 1")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.be = backend or HipBackend(device)
        self.n_users, self.n_items, self.d, self.K = int(n_users), int(n_items), int(dim), int(n_layers)
        self.reg, self.lr, self.wd = float(reg), float(lr), float(weight_decay)
        self.batch = int(batch)
        nu, ni, d = self.n_users, self.n_items, self.d
        tu = np.asarray(train_u, dtype=np.int64)
        ti = np.asarray(train_i, dtype=np.int64)
        key = np.unique(tu * (1 << 32) + ti)
        uu, ii = key >> 32, key & 0xFFFFFFFF
        # global item degrees (sum of every rank's interactions)
        deg_i = torch.from_numpy(np.bincount(ii, minlength=ni).astype(np.int64))
        deg_i = self._allreduce_host(deg_i)
        deg_u = np.bincount(uu, minlength=nu).astype(np.float64)
        du = np.power(deg_u + 1e-7, -0.5)
        di = np.power(deg_i.numpy().astype(np.float64) + 1e-7, -0.5)
        v_u = (du[uu] * di[ii]).astype(np.float32)   # user rows: d_u * d_i
        v_i = (di[ii] * du[uu]).astype(np.float32)   # item rows: d_i * d_u (same value)
        n = nu + ni
        self.A_U = self.be.csr(*graph.to_csr(uu, ii + nu, v_u, nu, n), n, chunk)
        self.A_I = self.be.csr(*graph.to_csr(ii, uu, v_i, ni, n), n, chunk)
        self.nnz = int(2 * key.size)
        # replicated items: every rank starts from rank 0's item table
        it = torch.from_numpy(np.ascontiguousarray(item_emb, dtype=np.float32))
        it = self._broadcast_host(it)
        p = torch.cat([torch.from_numpy(np.ascontiguousarray(user_emb, dtype=np.float32)), it])
        self.p = self.be.tensor(p)
        if hasattr(self.be, "zeros"):
            z = lambda rows=n: self.be.zeros(rows, d)  # noqa: E731
        else:
            z = lambda rows=n: self.be.tensor(torch.zeros(rows, d, dtype=torch.float32))  # noqa: E731
        self.m, self.v, self.s, self.h0, self.h1 = z(), z(), z(), z(), z()
        self.final, self.g, self.r = z(), z(), z()
        self.t = z(ni)
        self.loss_acc = self.be.tensor(torch.zeros(1, dtype=torch.float64))
        self.step_count = 0
        self.sampler = self.be.sampler(tu, ti, nu, seed)
        self.n_inter = self.sampler.n_inter
        self._epoch_buf = None
        self._epoch_sampled = None
        self._fwd_valid = False
        # batch-row tags (rsx_sharded_lgcn_step.row_tag): the stored-layer step for K = 2, 3
        self.row_tag = None
        if isinstance(self.be, HipBackend) and self.K in (2, 3):
            self.row_tag = torch.zeros(n, dtype=torch.int32, device=self.be.device)
        if native is None:
            native = isinstance(self.be, HipBackend) and dist.get_backend(self.group) == "nccl"
        self.native = bool(native)
        self._comm = None
        if self.native:
            if not isinstance(self.be, HipBackend):
                raise RuntimeError("the native sharded step needs the HIP backend")
            self._init_native()
        elif self.row_tag is not None and self.K in (2, 3):
            self.row_tag = None  # the Python-issued sequence keeps the running sums

    # ------------------------------------------------------------ native step
    def _init_native(self):
        """Communicator for csrc/dist.hip: RCCL over this process group ("nccl": unique-id
        handshake), or — any other backend, tests — the host hook driving this group's
        all_reduce on host copies of the exchanged rows."""
        lib = L.lib()
        comm = C.c_void_p()
        if dist.get_backend(self.group) == "nccl":
            nb = int(lib.rsx_comm_unique_id_bytes())
            buf = (C.c_uint8 * nb)()
            if self.rank == 0:
                L.check(lib.rsx_comm_get_unique_id(buf), "rsx_comm_get_unique_id")
            uid = self._broadcast_host(torch.tensor(bytearray(bytes(buf)), dtype=torch.uint8))
            C.memmove(buf, bytes(uid.numpy().tobytes()), nb)
            with torch.cuda.device(self.be.device):
                L.check(lib.rsx_comm_init(C.byref(comm), buf, self.rank, self.world), "rsx_comm_init")
        else:
            nu = self.n_users
            views = [self.t] + [getattr(self, k)[nu:] for k in ("h0", "h1", "final", "g", "r")]
            self._views = {(v.data_ptr(), v.numel()): v for v in views}

            def host_allreduce(ptr, n, _ctx):
                try:
                    v = self._views[(ptr, n)]
                    x = v.cpu()
                    dist.all_reduce(x, group=self.group)
                    v.copy_(x)
                    return 0
                except Exception:  # noqa: BLE001
                    return 1

            self._host_cb = L.HOST_ALLREDUCE_FN(host_allreduce)  # kept alive with the engine
            L.check(lib.rsx_comm_init_host(C.byref(comm), self.rank, self.world, self._host_cb, None),
                    "rsx_comm_init_host")
        self._comm = comm
        st = self._st = L.ShardedStep()
        st.adj_u = C.pointer(self.A_U.struct)
        st.adj_i = C.pointer(self.A_I.struct)
        st.n_users, st.n_items, st.d, st.n_layers, st.reg = self.n_users, self.n_items, self.d, self.K, self.reg
        for name in ("p", "m", "v", "s", "h0", "h1", "g", "r", "t"):
            setattr(st, name, getattr(self, name).data_ptr())
        st.final_emb = self.final.data_ptr()
        su, si = self.A_U.slab(self.d), self.A_I.slab(self.d)
        st.slab_u = su.data_ptr() if su is not None else 0
        st.slab_i = si.data_ptr() if si is not None else 0
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=self.be.device)
        st.loss_out = self.loss_out.data_ptr()
        st.loss_acc = self.loss_acc.data_ptr()
        self.ws = torch.empty(lib.rsx_bpr_ws_bytes(max(self.batch, 1)), dtype=torch.uint8, device=self.be.device)
        st.ws, st.ws_bytes = self.ws.data_ptr(), self.ws.numel()
        st.comm = comm.value
        st.row_tag = self.row_tag.data_ptr() if self.row_tag is not None else None
        # the one-launch BPR (regulariser as per-row occurrence counts, applied and
        # cleared by the user Adam layer and the last item partial), as the single engine
        self.reg_cnt = None
        if self.row_tag is not None and os.environ.get("RSX_BPR_FUSED", "1") != "0":
            self.reg_cnt = torch.zeros(3 * (self.n_users + self.n_items) + 4, dtype=torch.int32,
                                       device=self.be.device)
        st.reg_cnt = self.reg_cnt.data_ptr() if self.reg_cnt is not None else None
        # Adam's step count and (its low word) the batch-row tag live on the device, so
        # the step's launches and collectives are the same every batch: over RCCL the
        # step is captured once as a HIP graph and replayed (host cost per batch: one
        # triplet copy + one graph launch instead of ~20 launches and 7 collectives)
        self._step_dev = torch.zeros(1, dtype=torch.int64, device=self.be.device)
        st.tag_dev = self._step_dev.data_ptr()
        self._trip_buf = torch.zeros(3, self.batch, dtype=torch.int64, device=self.be.device)
        self._graph = None
        self._graph_lr = None
        self._graph_warm = False
        self.use_graph = (dist.get_backend(self.group) == "nccl" and self.row_tag is not None
                          and os.environ.get("RSX_SHARDED_GRAPH", "1") != "0")

    def _native_step(self, trip):
        """One batch through csrc/dist.hip.  Full batches over RCCL: the first runs
        eagerly (RCCL sets up its connections on first use), the second is captured
        into a HIP graph, every later one replays it after copying its triplets into
        the captured buffer.  Partial batches, a changed lr and host-hook
        communicators run eagerly."""
        lib, st = L.lib(), self._st
        B = int(trip.shape[1])
        st.adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd, step_dev=self._step_dev)
        graph = self.use_graph and B == self.batch
        if graph and self._graph is not None and self._graph_lr == self.lr:
            self._trip_buf.copy_(trip)
            self._graph.replay()
            return
        if graph and self._graph_warm:
            self._trip_buf.copy_(trip)
            st.triplets, st.batch = self._trip_buf.data_ptr(), B
            g = torch.cuda.CUDAGraph()
            gc_on = gc.isenabled()
            gc.disable()  # no finalizers inside the capture (see rsx/trainer.py:_capture)
            try:
                with torch.cuda.graph(g):
                    self._step_dev.add_(1)
                    L.check(lib.rsx_sharded_lightgcn_step(C.byref(st), ops._stream()), "rsx_sharded_lightgcn_step")
            except Exception:  # noqa: BLE001  capture refused: this engine stays eager
                self.use_graph = False
                torch.cuda.synchronize()
            else:
                self._graph, self._graph_lr = g, self.lr
            finally:
                if gc_on:
                    gc.enable()
            if self._graph is g:
                g.replay()
                return
        t = trip.contiguous()
        self._keep = t
        nb = lib.rsx_bpr_ws_bytes(B)
        if nb > self.ws.numel():  # a given batch larger than the engine's
            # a captured graph holds the old workspace pointer: drop it (and re-warm)
            # before that memory returns to the caching allocator
            if self._graph is not None:
                torch.cuda.synchronize(self.be.device)
                self._graph = None
            self._graph_warm = False
            self.ws = torch.empty(nb, dtype=torch.uint8, device=self.be.device)
            st.ws, st.ws_bytes = self.ws.data_ptr(), self.ws.numel()
        st.triplets, st.batch = t.data_ptr(), B
        self._step_dev.add_(1)
        L.check(lib.rsx_sharded_lightgcn_step(C.byref(st), ops._stream()), "rsx_sharded_lightgcn_step")
        if graph:
            self._graph_warm = True

    def close(self):
        """Release the rsx communicator (before destroy_process_group)."""
        if self._comm is not None:
            self._graph = None  # the captured collectives belong to the communicator
            torch.cuda.synchronize(self.be.device)
            L.lib().rsx_comm_destroy(self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------ comms
    def _allreduce_host(self, t):
        if dist.get_backend(self.group) == "nccl":
            x = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(x, group=self.group)
            return x.cpu()
        dist.all_reduce(t, group=self.group)
        return t

    def _broadcast_host(self, t):
        if dist.get_backend(self.group) == "nccl":
            x = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(x, src=dist.get_global_rank(self.group, 0) if self.group else 0, group=self.group)
            return x.cpu()
        dist.broadcast(t, src=0, group=self.group)
        return t

    def _ar(self, x):
        return dist.all_reduce(x, group=self.group, async_op=True)

    # --------------------------------------------------------------- forward
    def _propagate(self, zero_grads: bool):
        """Forward layers with every item all-reduce issued as soon as its partial
        exists: layer k+1's item partial needs only users^k (local), so it is
        computed and its exchange queued before waiting for layer k's; the comm
        stream then runs the K exchanges back to back while the compute stream
        does the user-row SpMMs.  Per-element arithmetic = one layer at a time."""
        be, nu, ni, d, K = self.be, self.n_users, self.n_items, self.d, self.K
        p, s, f = self.p, self.s, self.final
        bufs = (self.h0, self.h1)
        beta = 1.0 / (K + 1)
        ys = [p] + [bufs[(k - 1) & 1] for k in range(1, K + 1)]  # ys[k]: users^k | items^k
        works = {}

        def item_partial(k):  # items^k partial = R_g^T users^{k-1}; exchange queued
            be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_STORE, y=ys[k][nu:])
            works[k] = self._ar(ys[k][nu:])

        item_partial(1)
        for k in range(1, K + 1):
            s_in = p if k == 1 else s
            if k < K:
                be.spmm(self.A_U, ys[k - 1], d, L.RSX_EPI_LAYERSUM, y=ys[k][:nu], s_in=s_in[:nu], s_out=s[:nu])
                item_partial(k + 1)
            else:
                zero = dict(zero0=self.g[:nu], zero1=self.r[:nu]) if zero_grads else {}
                be.spmm(self.A_U, ys[k - 1], d, L.RSX_EPI_FINAL, beta=beta, f=f[:nu], s_in=s_in[:nu], **zero)
            works.pop(k).wait()
            if k < K:
                be.rowwise(ni, d, L.RSX_EPI_ADD, y=s[nu:], s_in=s_in[nu:], r_add=ys[k][nu:])
            else:
                zi = dict(zero0=self.g[nu:], zero1=self.r[nu:]) if zero_grads else {}
                be.rowwise(ni, d, L.RSX_EPI_ADD, beta=beta, y=f[nu:], s_in=s_in[nu:], r_add=ys[k][nu:], **zi)

    def forward(self):
        if not self._fwd_valid:
            if self.native:
                L.check(L.lib().rsx_sharded_lightgcn_forward(C.byref(self._st), ops._stream()),
                        "rsx_sharded_lightgcn_forward")
            else:
                self._propagate(zero_grads=False)
            self._fwd_valid = True
        return self.final

    def invalidate(self):
        self._fwd_valid = False

    # ------------------------------------------------------------------ step
    def step(self, triplets=None, epoch: int = 0, start: int = 0):
        be, nu, ni, d, K = self.be, self.n_users, self.n_items, self.d, self.K
        self.step_count += 1
        if triplets is None:
            if self._epoch_sampled != epoch:
                self._epoch_buf = self.sampler.sample_epoch(epoch, self.batch, out=self._epoch_buf)
                self._epoch_sampled = epoch
            triplets = ops.DeviceSampler.batch_view(self._epoch_buf, self.n_inter, self.batch,
                                                    start // self.batch)
        if self.native:
            self._native_step(triplets[:3])
            self._fwd_valid = False
            return
        self._propagate(zero_grads=True)
        self.loss_out = be.bpr(self.final, self.p, nu, ni, triplets, self.reg, self.g, self.r, self.loss_acc)
        adam = be.adam(self.lr, self.step_count, self.wd)
        beta = 1.0 / (K + 1)
        g, s, r, t = self.g, self.s, self.r, self.t
        bufs = (self.h0, self.h1)
        # backward = the same layer sums on G = dL/dfinal (A symmetric); G's item rows
        # are per-rank partials: their exchange and layer 1's item partial (which
        # needs only G's local user rows) are queued together, and so on per layer
        ys = [g] + [bufs[(k - 1) & 1] for k in range(1, K + 1)]
        works = {0: self._ar(g[nu:])}

        def item_partial(k):
            if k < K:
                be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_STORE, y=ys[k][nu:])
                works[k] = self._ar(ys[k][nu:])
            else:  # t = H_I^K/(K+1) + R_I: this rank's share of the item gradient beyond s_I/(K+1)
                be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_ADD, alpha=beta, y=t, r_add=r[nu:])
                works[k] = self._ar(t)

        item_partial(1)
        works.pop(0).wait()
        for k in range(1, K + 1):
            s_in = g if k == 1 else s
            if k < K:
                be.spmm(self.A_U, ys[k - 1], d, L.RSX_EPI_LAYERSUM, y=ys[k][:nu], s_in=s_in[:nu], s_out=s[:nu])
                item_partial(k + 1)
                works.pop(k).wait()
                be.rowwise(ni, d, L.RSX_EPI_ADD, y=s[nu:], s_in=s_in[nu:], r_add=ys[k][nu:])
            else:
                be.spmm(self.A_U, ys[k - 1], d, L.RSX_EPI_ADAM, beta=beta, adam=adam, s_in=s_in[:nu], r_add=r[:nu],
                        p=self.p[:nu], m=self.m[:nu], v=self.v[:nu])
                works.pop(k).wait()
                be.rowwise(ni, d, L.RSX_EPI_ADAM, beta=beta, adam=adam, s_in=s_in[nu:], r_add=t,
                           p=self.p[nu:], m=self.m[nu:], v=self.v[nu:])
        self._fwd_valid = False
