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

Sparse exchange (`sparse=True`; by default for K = 2, 3 once the item block
n_items * d * 4 reaches 16 MiB, RSX_SPARSE_MIN_BYTES).  The loss reads the
final rows of the batch items only, and G = dL/dfinal is nonzero on them only:
every rank all-gathers the (pos, neg) ids of every rank's batch (the union U,
world * 2 * batch ids), and the last layer's item rows and G's item rows are
summed as compact [|U|, d] blocks instead of [n_items, d].  The item gradient is
reduce-scattered over n_items_pad = world * ceil(n_items / world) rows, each
rank runs Adam on its own slice of item rows (its moments only there), and the
updated slices are all-gathered into every replica.  Per K = 3 step that is 4
dense all-reduces + 1 reduce-scatter + 1 all-gather of n_items * d floats (the
volume of 5 all-reduces, against 7) + 2 compact all-reduces.  The Python
sequence below states the same schedule with torch collectives (over gloo,
reduce-scatter and all-gather are emulated with all-reduce / all_gather).
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


# xGMI link model (MI355X_MICROARCH.md): 7 links per GPU, ~76.5 GB/s per
# direction each; a W-rank ring on a fully connected node drives min(W-1, 7) of them at
# an efficiency of 0.8 (RCCL's ring / LL128 protocols on large messages)
XGMI_LINK_GBS, XGMI_LINKS, RING_EFF, RCCL_LATENCY_US, RCCL_BLOCKS = 76.5, 7, 0.8, 30.0, 32


def model_busbw_gbs(world: int) -> float:
    return min(world - 1, XGMI_LINKS) * XGMI_LINK_GBS * RING_EFF


SIM_OPT_IN = "RSX_COMM_SIM_OPT_IN"  # set to 1 by bench.py and the tests only


def sim_comm_params():
    """RSX_COMM_SIM = "W[:busbw_gbs[:latency_us[:blocks]]]": run the one-rank engine over a
    latency-injected communicator modelling a W-rank job (rsx_comm_init_sim); None if unset.

    The modelled job trains rank 0's share on stand-in peer data (the DP step's other
    slots hold frozen triplets), so it is a measurement mode, never a training run: it
    needs the second variable RSX_COMM_SIM_OPT_IN=1, which only bench.py and the tests
    set.  RSX_COMM_SIM alone (say, left over in a shell) is ignored with a warning."""
    v = os.environ.get("RSX_COMM_SIM")
    if not v:
        return None
    if os.environ.get(SIM_OPT_IN) != "1":
        import warnings

        warnings.warn(f"RSX_COMM_SIM={v} ignored: latency injection is a benchmark mode that trains on "
                      f"stand-in peer data; set {SIM_OPT_IN}=1 as well to run it", RuntimeWarning, stacklevel=2)
        return None
    f = v.split(":")
    w = int(f[0])
    if w < 2:
        raise ValueError(f"RSX_COMM_SIM={v}: the modelled world must be >= 2")
    return {"world": w, "busbw_gbs": float(f[1]) if len(f) > 1 and f[1] else model_busbw_gbs(w),
            "latency_us": float(f[2]) if len(f) > 2 and f[2] else RCCL_LATENCY_US,
            "blocks": int(f[3]) if len(f) > 3 and f[3] else RCCL_BLOCKS, "scratch_mb": 512}


def head_pieces_knob(default: int) -> int:
    """RSX_SHARDED_HEAD: row pieces of the step's first item partial (1 = one launch)."""
    v = os.environ.get("RSX_SHARDED_HEAD")
    if v is None or v == "":
        return default
    if not v.isdigit() or not 1 <= int(v) <= 64:
        raise ValueError(f"RSX_SHARDED_HEAD={v!r}: an integer in [1, 64] expected")
    return int(v)


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
                 backend=None, native: bool | None = None, sparse: bool | None = None, union_cap: int | None = None):
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
        self._deg_i_global = deg_i.numpy().astype(np.int64)  # the same on every rank
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
        if sparse is None:
            # bandwidth regime only: the sparse schedule trades 7 dense all-reduces for 4 + a
            # reduce-scatter + an all-gather + 3 small collectives, which pays once the item
            # block is large (C4: 1 GB) and costs latency when it is small (C2: 4.7 MB)
            sparse = self.K in (2, 3) and ni * d * 4 >= int(os.environ.get("RSX_SPARSE_MIN_BYTES", 16 << 20))
        self.sparse = bool(sparse)
        if self.sparse and self.K not in (2, 3):
            raise RuntimeError("the sparse exchange schedule is implemented for n_layers 2 and 3")
        # item rows padded to a multiple of the world size (reduce-scatter / all-gather slices)
        self.n_items_pad = -(-ni // self.world) * self.world
        self.q = self.n_items_pad // self.world  # item rows per owner
        pad = self.n_items_pad - ni
        p = torch.cat([torch.from_numpy(np.ascontiguousarray(user_emb, dtype=np.float32)), it,
                       torch.zeros(pad, d, dtype=torch.float32)])
        self._p_full = self.be.tensor(p)
        self._p = self._p_full[: nu + ni]
        self.defer_ag = False  # the native sparse step's deferred parameter all-gather (_init_native)
        self._ag_dirty = False
        if hasattr(self.be, "zeros"):
            z = lambda rows=n: self.be.zeros(rows, d)  # noqa: E731
        else:
            z = lambda rows=n: self.be.tensor(torch.zeros(rows, d, dtype=torch.float32))  # noqa: E731
        self.m, self.v, self.s, self.h0, self.h1 = z(), z(), z(), z(), z()
        self.final, self.g, self.r = z(), z(), z()
        self.t = z(self.n_items_pad)  # pad rows stay zero
        # the union exchange's per-rank slice: equal on every rank (ranks may step with
        # different batch sizes; the largest bounds the slice)
        self.union_cap = int(union_cap or self.batch)
        if self.sparse:
            mk = (lambda a: self.be.tensor(a)) if not hasattr(self.be, "zeros") else \
                (lambda a: a.to(self.be.device))  # noqa: E731
            self.union = mk(torch.zeros(self.world * 2 * self.union_cap, dtype=torch.int64))
            self.item_tag = mk(torch.zeros(ni, dtype=torch.int32))
            self.cbuf0 = z(self.world * 2 * self.union_cap)
            self.cbuf1 = z(self.world * 2 * self.union_cap)
            self.nbr = None  # the sparse last-layer exchange's buffers (native step, _init_native)
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
        self.sim = None  # the latency-injection model (RSX_COMM_SIM), if the communicator is one
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
        # the fused-round schedule (RSX_SHARDED_FUSED=1; dense, K = 2, 3, batch-row tags):
        # two layers' item partials per collective, 4 collectives per K = 3 step instead of
        # 7 (csrc/dist.hip:sharded_fused_rounds).  Off by default: it saves three collective
        # latencies but serialises the compute the per-layer schedule hides behind its
        # exchanges (one rank: 0.236 vs 0.219 ms/step)
        self.xch = None
        if (not self.sparse and self.row_tag is not None and self.K in (2, 3)
                and os.environ.get("RSX_SHARDED_FUSED", "0") == "1"):
            self.xch = torch.zeros(2 * self.n_items, self.d, dtype=torch.float32, device=self.be.device)
        # the step's heads in row pieces (rsx_sharded_lgcn_step.n_head): the first forward
        # and backward item partials' rows all-reduced piece by piece.  Off by default: in
        # the graph-replayed C4 step at a modelled 8-rank job (latency injection) 4 pieces
        # took 28.5 ms/step against 25.2 without (the replay spreads the extra launches and
        # collectives over the hardware queues, and a piece can queue behind an exchange);
        # RSX_SHARDED_HEAD=n turns them on.
        self.head = []
        n_head = head_pieces_knob(1)
        if n_head > 1 and self.row_tag is not None and self.xch is None and self.A_I.rowptr_host is not None:
            # cut by the GLOBAL item degrees (every rank the same pieces: the collectives match)
            rp = np.concatenate([[0], np.cumsum(self._deg_i_global)])
            cuts = np.searchsorted(rp, np.arange(1, n_head) * rp[-1] / n_head, side="left")
            row0 = np.unique(np.concatenate([[0], np.clip(cuts, 1, self.n_items - 1), [self.n_items]]))
            row0 = row0.astype(np.int64)
            if row0.size - 1 > 1:
                self.head = [ops.DeviceCSR.row_slice(self.A_I, int(a), int(b)) for a, b in zip(row0[:-1], row0[1:])]
                self.head_row0 = row0
        # the last stored forward layer's item rows summed on the rows the loss reads only
        # (rsx_sharded_lgcn_step.nbr_items; RSX_SHARDED_NBR=0 keeps its dense all-reduce)
        self.nbr = None
        if (self.sparse and self.row_tag is not None and self.A_U.rowptr_host is not None
                and os.environ.get("RSX_SHARDED_NBR", "1") != "0"):
            self._alloc_nbr(self.union_cap)
        comm = C.c_void_p()
        sim = sim_comm_params()
        if sim is not None:
            if self.world != 1:
                raise RuntimeError("RSX_COMM_SIM models a multi-rank job on ONE rank (world 1)")
            self.sim = sim
            with torch.cuda.device(self.be.device):
                L.check(lib.rsx_comm_init_sim(C.byref(comm), sim["world"], sim["busbw_gbs"], sim["latency_us"],
                                              sim["blocks"], sim["scratch_mb"]), "rsx_comm_init_sim")
        elif dist.get_backend(self.group) == "nccl":
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
            views = [self.t, self._p_full[nu:]] + [getattr(self, k)[nu:] for k in ("h0", "h1", "final", "g", "r")]
            if self.sparse:
                views += [self.union, self.cbuf0, self.cbuf1]
            if self.xch is not None:
                views.append(self.xch)
            if self.nbr is not None:
                views += [self.nbr["ids"], self.nbr["buf"]]
            if self.head:  # the head pieces' item rows of E^1
                views += [self.h0[nu + int(a): nu + int(b)] for a, b in zip(self.head_row0[:-1], self.head_row0[1:])]
            # one view per start pointer: the largest (the first head piece starts where the
            # whole item block of h0 does; collectives use the first `count` floats)
            self._views = {}
            for v in views:
                f = v.view(-1)
                if f.numel() > self._views.get(v.data_ptr(), f[:0]).numel():
                    self._views[v.data_ptr()] = f

            def host_collective(op, ptr, count, dtype, _ctx):
                try:
                    v = self._views[ptr]
                    self._host_coll(op, v, count)
                    return 0
                except Exception:  # noqa: BLE001
                    return 1

            self._host_cb = L.HOST_COLLECTIVE_FN(host_collective)  # kept alive with the engine
            L.check(lib.rsx_comm_init_host(C.byref(comm), self.rank, self.world, self._host_cb, None),
                    "rsx_comm_init_host")
        self._comm = comm
        st = self._st = L.ShardedStep()
        st.adj_u = C.pointer(self.A_U.struct)
        st.adj_i = C.pointer(self.A_I.struct)
        st.n_users, st.n_items, st.d, st.n_layers, st.reg = self.n_users, self.n_items, self.d, self.K, self.reg
        for name in ("m", "v", "s", "h0", "h1", "g", "r", "t"):
            setattr(st, name, getattr(self, name).data_ptr())
        st.p = self._p.data_ptr()
        # the parameter all-gather deferred to the next step (include/rsx.h defer_ag; the
        # sparse schedule only; RSX_SHARDED_DEFER_AG=0 keeps it at the end of the step)
        self.defer_ag = bool(self.sparse and self.row_tag is not None
                             and os.environ.get("RSX_SHARDED_DEFER_AG", "1") != "0")
        st.defer_ag = int(self.defer_ag)
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
        st.n_items_pad = self.n_items_pad
        st.union_cap = self.union_cap
        if self.sparse and self.row_tag is not None:
            st.union_items, st.item_tag = self.union.data_ptr(), self.item_tag.data_ptr()
            st.cbuf0, st.cbuf1 = self.cbuf0.data_ptr(), self.cbuf1.data_ptr()
        st.xch = self.xch.data_ptr() if self.xch is not None else None
        # the sparse exchange's row-list error bits (include/rsx.h rsx_sharded_lgcn_step.err)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.be.device)
        st.err = self.err.data_ptr()
        self._set_nbr_struct()
        if self.head:
            self._head_structs = (L.Csr * len(self.head))(*[h.struct for h in self.head])
            self._head_row0 = (C.c_int64 * self.head_row0.size)(*[int(x) for x in self.head_row0])
            slabs = [h.slab(self.d) for h in self.head]
            self._head_slab_keep = slabs
            self._head_slab = (C.c_void_p * len(slabs))(*[s.data_ptr() if s is not None else None for s in slabs])
            st.n_head = len(self.head)
            st.head_i = C.cast(self._head_structs, C.POINTER(L.Csr))
            st.head_row0 = C.cast(self._head_row0, C.c_void_p)
            st.head_slab = C.cast(self._head_slab, C.c_void_p)
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
        # one captured graph per batch size (balanced epoch slices come in two sizes)
        self._graphs = {}  # B -> (graph, lr, triplet buffer)
        self._graph_warm = set()
        self.use_graph = (dist.get_backend(self.group) == "nccl" and self.row_tag is not None
                          and os.environ.get("RSX_SHARDED_GRAPH", "1") != "0")

    def _native_step(self, trip):
        """One batch through csrc/dist.hip.  Over RCCL, per batch size: the first batch runs
        eagerly (RCCL sets up its connections on first use, workspaces settle), the second
        is captured into a HIP graph, every later one replays it after copying its
        triplets into the captured buffer.  A changed lr re-captures; host-hook
        communicators run eagerly."""
        lib, st = L.lib(), self._st
        B = int(trip.shape[1])
        st.adam = ops.adam_struct(self.lr, self.step_count, weight_decay=self.wd, step_dev=self._step_dev)
        graph = self.use_graph and B <= self.union_cap
        cap = self._graphs.get(B) if graph else None
        if cap is not None and cap[1] == self.lr:
            cap[2].copy_(trip)
            cap[0].replay()
            return
        if graph and B in self._graph_warm:
            buf = cap[2] if cap is not None else torch.zeros(3, B, dtype=torch.int64, device=self.be.device)
            buf.copy_(trip)
            st.triplets, st.batch = buf.data_ptr(), B
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
                self._graphs[B] = (g, self.lr, buf)
                g.replay()
                return
            finally:
                if gc_on:
                    gc.enable()
        t = trip.contiguous()
        self._keep = t
        nb = lib.rsx_bpr_ws_bytes(B)
        grow_union = self.sparse and B > self.union_cap
        if nb > self.ws.numel() or grow_union:  # a given batch larger than the engine's
            # captured graphs hold the old workspace pointers: drop them (and re-warm)
            # before that memory returns to the caching allocator
            if self._graphs:
                torch.cuda.synchronize(self.be.device)
                self._graphs.clear()
            self._graph_warm.clear()
            if nb > self.ws.numel():
                self.ws = torch.empty(nb, dtype=torch.uint8, device=self.be.device)
                st.ws, st.ws_bytes = self.ws.data_ptr(), self.ws.numel()
            if grow_union:  # every rank must step with the same batch size (collective counts)
                self._grow_union(B)
        st.triplets, st.batch = t.data_ptr(), B
        self._step_dev.add_(1)
        L.check(lib.rsx_sharded_lightgcn_step(C.byref(st), ops._stream()), "rsx_sharded_lightgcn_step")
        if graph:
            self._graph_warm.add(B)

    def _alloc_nbr(self, B):
        cap = self._nbr_cap(B)
        sim = sim_comm_params()
        if sim is not None and self.world == 1:
            # one rank modelling a W-rank job: its list padded to the job's W slices (item 0),
            # so the injected compact all-reduce moves the modelled job's bytes
            cap *= sim["world"]
        dev = self.be.device
        self.nbr = {"cap": cap, "ids": torch.zeros(self.world * cap, dtype=torch.int64, device=dev),
                    "count": torch.zeros(1, dtype=torch.int32, device=dev),
                    "buf": torch.zeros(self.world * cap, self.d, dtype=torch.float32, device=dev)}

    def _set_nbr_struct(self):
        st = getattr(self, "_st", None)
        if st is None:
            return
        if self.nbr is None:
            st.nbr_items = st.nbr_count = st.cbufN = None
            st.nbr_cap = 0
        else:
            st.nbr_items, st.nbr_count = self.nbr["ids"].data_ptr(), self.nbr["count"].data_ptr()
            st.cbufN, st.nbr_cap = self.nbr["buf"].data_ptr(), self.nbr["cap"]

    def _grow_union(self, B):
        """Union-exchange buffers for batches of up to B pairs per rank."""
        self.union_cap = int(B)
        dev = self.union.device
        self.union = torch.zeros(self.world * 2 * B, dtype=torch.int64, device=dev)
        self.cbuf0 = torch.zeros(self.world * 2 * B, self.d, dtype=torch.float32, device=dev)
        self.cbuf1 = torch.zeros_like(self.cbuf0)
        if getattr(self, "nbr", None) is not None:
            self._alloc_nbr(B)
            self._set_nbr_struct()
        if getattr(self, "_views", None) is not None:
            for v in (self.union, self.cbuf0, self.cbuf1) + ((self.nbr["ids"], self.nbr["buf"]) if self.nbr else ()):
                self._views[v.data_ptr()] = v.view(-1)
        if getattr(self, "_st", None) is not None:
            st = self._st
            st.union_cap = self.union_cap
            st.union_items = self.union.data_ptr()
            st.cbuf0, st.cbuf1 = self.cbuf0.data_ptr(), self.cbuf1.data_ptr()

    def close(self):
        """Release the rsx communicator (before destroy_process_group)."""
        if self._comm is not None:
            self.flush()
            self._graphs = {}  # the captured collectives belong to the communicator
            torch.cuda.synchronize(self.be.device)
            L.lib().rsx_comm_destroy(self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------ comms
    def _allreduce_host(self, t, op=dist.ReduceOp.SUM):
        if dist.get_backend(self.group) == "nccl":
            x = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(x, op=op, group=self.group)
            return x.cpu()
        dist.all_reduce(t, op=op, group=self.group)
        return t

    def _nbr_cap(self, B):
        """rsx_sharded_lgcn_step.nbr_cap for batches of up to B triplets per rank: 2 B union
        items + the largest neighbour count any B of this rank's users can have (the sum of
        the B largest user degrees), the maximum over the ranks (the slices line up)."""
        deg = np.diff(self.A_U.rowptr_host)
        top = int(np.sort(deg)[::-1][:B].sum()) if deg.size else 0
        cap = torch.tensor([2 * int(B) + top], dtype=torch.int64)
        return int(self._allreduce_host(cap, op=dist.ReduceOp.MAX).item())

    def _broadcast_host(self, t):
        if dist.get_backend(self.group) == "nccl":
            x = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(x, src=dist.get_global_rank(self.group, 0) if self.group else 0, group=self.group)
            return x.cpu()
        dist.broadcast(t, src=0, group=self.group)
        return t

    def _ar(self, x):
        return dist.all_reduce(x, group=self.group, async_op=True)

    def _host_coll(self, op, v, count):
        """One in-place collective on the flat tensor v (the host hook's statement of
        RSX_COLL_*): the exchange goes through host copies over this group."""
        w, r = self.world, self.rank
        if op == L.RSX_COLL_ALLREDUCE:
            x = v[:count].cpu()
            dist.all_reduce(x, group=self.group)
            v[:count].copy_(x)
        elif op == L.RSX_COLL_ALLGATHER:
            mine = v[r * count:(r + 1) * count].cpu()
            parts = [torch.empty_like(mine) for _ in range(w)]
            dist.all_gather(parts, mine, group=self.group)
            v[: w * count].copy_(torch.cat(parts))
        elif op == L.RSX_COLL_REDUCESCATTER:
            x = v[: w * count].cpu()
            dist.all_reduce(x, group=self.group)  # gloo has no reduce-scatter: keep this rank's slice
            v[r * count:(r + 1) * count].copy_(x[r * count:(r + 1) * count])
        else:
            raise ValueError(op)

    def _coll(self, op, v, count):
        """The same collectives issued from Python on device (or CPU) tensors."""
        if dist.get_backend(self.group) == "nccl":
            w, r = self.world, self.rank
            if op == L.RSX_COLL_ALLREDUCE:
                dist.all_reduce(v[:count], group=self.group)
            elif op == L.RSX_COLL_ALLGATHER:
                dist.all_gather_into_tensor(v[: w * count], v[r * count:(r + 1) * count].clone(), group=self.group)
            else:
                out = torch.empty(count, dtype=v.dtype, device=v.device)
                dist.reduce_scatter_tensor(out, v[: w * count], group=self.group)
                v[r * count:(r + 1) * count].copy_(out)
            return
        if v.is_cuda:
            self._host_coll(op, v, count)
            return
        w, r = self.world, self.rank
        if op == L.RSX_COLL_ALLREDUCE:
            dist.all_reduce(v[:count], group=self.group)
        elif op == L.RSX_COLL_ALLGATHER:
            parts = [torch.empty(count, dtype=v.dtype) for _ in range(w)]
            dist.all_gather(parts, v[r * count:(r + 1) * count].clone(), group=self.group)
            v[: w * count].copy_(torch.cat(parts))
        else:
            x = v[: w * count].clone()
            dist.all_reduce(x, group=self.group)
            v[r * count:(r + 1) * count].copy_(x[r * count:(r + 1) * count])

    # --------------------------------------------------------------- forward
    def _propagate(self, zero_grads: bool, union=None):
        """Forward layers with every item all-reduce issued as soon as its partial
        exists: layer k+1's item partial needs only users^k (local), so it is
        computed and its exchange queued before waiting for layer k's; the comm
        stream then runs the K exchanges back to back while the compute stream
        does the user-row SpMMs.  Per-element arithmetic = one layer at a time.
        `union` (sparse schedule): the last layer's item rows are summed on those
        rows only (the final item rows elsewhere are left unsummed: nothing reads them)."""
        be, nu, ni, d, K = self.be, self.n_users, self.n_items, self.d, self.K
        p, s, f = self._p, self.s, self.final
        bufs = (self.h0, self.h1)
        beta = 1.0 / (K + 1)
        ys = [p] + [bufs[(k - 1) & 1] for k in range(1, K + 1)]  # ys[k]: users^k | items^k
        works = {}

        def item_partial(k):  # items^k partial = R_g^T users^{k-1}; exchange queued
            be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_STORE, y=ys[k][nu:])
            if not (union is not None and k == K):
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
            if k < K or union is None:
                works.pop(k).wait()
            if k < K:
                be.rowwise(ni, d, L.RSX_EPI_ADD, y=s[nu:], s_in=s_in[nu:], r_add=ys[k][nu:])
            elif union is None:
                zi = dict(zero0=self.g[nu:], zero1=self.r[nu:]) if zero_grads else {}
                be.rowwise(ni, d, L.RSX_EPI_ADD, beta=beta, y=f[nu:], s_in=s_in[nu:], r_add=ys[k][nu:], **zi)
            else:
                cb = ys[k][nu:].index_select(0, union)
                self._coll(L.RSX_COLL_ALLREDUCE, cb.view(-1), cb.numel())
                f[nu:].index_copy_(0, union, ((s_in[nu:].index_select(0, union) + cb) * beta))
                if zero_grads:
                    self.g[nu:].zero_()
                    self.r[nu:].zero_()

    @property
    def p(self):
        """The [users; items] parameter table, read as it is: no collective (a rank-0-only
        checkpoint must not block).  With the deferred all-gather (defer_ag) the item rows
        owned by other ranks are one step old until every rank has called flush(), which
        the Trainer does at the end of each epoch and forward() does before evaluation."""
        return self._p

    def flush(self):
        """Complete a deferred parameter all-gather (defer_ag: the sparse native step issues
        it at the start of the next step), so every replica's item rows are current.  It is
        a collective when one is pending: every rank must call it at the same point (the
        Trainer does, at the end of each epoch and before evaluation)."""
        if self._ag_dirty and self._comm is not None:
            L.check(L.lib().rsx_sharded_lightgcn_flush(C.byref(self._st), ops._stream()),
                    "rsx_sharded_lightgcn_flush")
        self._ag_dirty = False
        self.check_err()

    def check_err(self):
        """Raise if a step's sparse row lists met an out-of-range id or overflowed (bits of
        rsx_sharded_lgcn_step.err; reading it synchronises the stream).

        The bits depend on each rank's own batches and neighbour lists, so the word is
        OR-ed over the group first (a MAX all-reduce of each bit) and every rank raises
        together: a rank raising alone would leave its peers blocked in the next
        collective.  A collective: every rank calls it at the same point (flush())."""
        err = getattr(self, "err", None)
        if err is None or not self.native:
            return
        if self.world > 1:
            bits = (err.to(torch.int64) >> torch.arange(2, device=err.device)) & 1
            if dist.get_backend(self.group) != "nccl":
                bits = bits.cpu()
            dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=self.group)
            e = int((bits.cpu() << torch.arange(2)).sum())
        else:
            e = int(err.item())
        if e:
            raise RuntimeError(f"sharded LightGCN step: row-list error bits {e:#x} on some rank "
                               "(1: an item id outside [0, n_items); 2: neighbour list over nbr_cap)")

    def forward(self):
        self.flush()
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
    def step_slice(self, epoch: int, j: int, n_slices: int):
        """Batch j of `epoch` cut into n_slices balanced slices of this rank's interactions
        (rsx_sample_epoch_slices): every rank runs the same n_slices steps per epoch and
        visits each of its interactions exactly once; a slice holds >= 1 triplet."""
        if self._epoch_sampled != (epoch, n_slices):
            self._epoch_buf = self.sampler.sample_epoch_slices(epoch, n_slices, out=self._epoch_buf)
            self._epoch_sampled = (epoch, n_slices)
        self.step(triplets=ops.DeviceSampler.slice_view(self._epoch_buf, self.n_inter, n_slices, j))

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
            self._ag_dirty = self.defer_ag
            return
        union = None
        if self.sparse:  # every rank's (pos, neg) ids, padded to the fixed slice with item 0
            B = int(triplets.shape[1])
            if B > self.union_cap:  # every rank must step with the same batch size
                self._grow_union(B)
            cap = self.union_cap
            mine = self.union[self.rank * 2 * cap:(self.rank + 1) * 2 * cap]
            mine.zero_()
            mine[: 2 * B].copy_(triplets[1:3].reshape(-1))
            self._coll(L.RSX_COLL_ALLGATHER, self.union, 2 * cap)
            union = self.union
        self._propagate(zero_grads=True, union=union)
        self.loss_out = be.bpr(self.final, self._p, nu, ni, triplets, self.reg, self.g, self.r, self.loss_acc)
        adam = be.adam(self.lr, self.step_count, self.wd)
        beta = 1.0 / (K + 1)
        g, s, r, t = self.g, self.s, self.r, self.t
        bufs = (self.h0, self.h1)
        # backward = the same layer sums on G = dL/dfinal (A symmetric); G's item rows
        # are per-rank partials: their exchange and layer 1's item partial (which
        # needs only G's local user rows) are queued together, and so on per layer
        ys = [g] + [bufs[(k - 1) & 1] for k in range(1, K + 1)]
        if union is not None:  # G's item rows are nonzero on the batch items only
            cb = g[nu:].index_select(0, union)
            self._coll(L.RSX_COLL_ALLREDUCE, cb.view(-1), cb.numel())
            g[nu:].index_copy_(0, union, cb)
            works = {}
        else:
            works = {0: self._ar(g[nu:])}

        def item_partial(k):
            if k < K:
                be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_STORE, y=ys[k][nu:])
                works[k] = self._ar(ys[k][nu:])
            else:  # t = H_I^K/(K+1) + R_I: this rank's share of the item gradient beyond s_I/(K+1)
                be.spmm(self.A_I, ys[k - 1], d, L.RSX_EPI_ADD, alpha=beta, y=t[:ni], r_add=r[nu:])
                if union is None:
                    works[k] = self._ar(t[:ni])

        item_partial(1)
        if 0 in works:
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
                        p=self._p[:nu], m=self.m[:nu], v=self.v[:nu])
                if union is None:
                    works.pop(k).wait()
                    be.rowwise(ni, d, L.RSX_EPI_ADAM, beta=beta, adam=adam, s_in=s_in[nu:], r_add=t[:ni],
                               p=self._p[nu:], m=self.m[nu:], v=self.v[nu:])
                else:  # reduce-scatter the item gradient; Adam on this rank's item rows; all-gather them
                    q = self.q
                    self._coll(L.RSX_COLL_REDUCESCATTER, t.view(-1), q * d)
                    r0 = self.rank * q
                    r1 = min(ni, r0 + q)
                    if r1 > r0:
                        sl = slice(nu + r0, nu + r1)
                        be.rowwise(r1 - r0, d, L.RSX_EPI_ADAM, beta=beta, adam=adam, s_in=s_in[sl],
                                   r_add=t[r0:r1], p=self._p[sl], m=self.m[sl], v=self.v[sl])
                    self._coll(L.RSX_COLL_ALLGATHER, self._p_full[nu:].view(-1), q * d)
        self._fwd_valid = False
