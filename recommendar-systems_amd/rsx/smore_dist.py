"""SMORE over the ranks of a process group: users sharded, the item side replicated
("replicate the item-side tables and kNN graphs", 141 MB at
Amazon-clothing).  Reference model: src/models/smore.py:24-411; the multi-GPU
scheme replaces the reference's one-device pinning (src/utils/configurator.py:114-118).

Partition.  Rank r owns the contiguous user block [a_r, b_r): its rows of the user
embedding (the only row-sharded parameter), of the normalised UI adjacency and of R.
Everything item-side is replicated and bit-identical on every rank: the item-id
embedding, the raw image / text feature tables (trainable, the largest
parameters), the projections, spectral filters, gates and preference weights, and
the kNN item graphs.

Step (per rank, on its own batch of its own users' interactions; the objective is
the sum over ranks of the reference loss of each rank's batch, i.e. data-parallel
batches of B per GPU):
  * projection + spectral fusion and the modality gates on every item (replicated);
  * the UI backbone, n_ui_layers times: users^k = A_U items^{k-1} (local rows),
    items^k = sum_g A_I,g users_g^{k-1} — ONE all-reduce of the item partial
    [n_items, d] per layer;
  * the three item views through their kNN graphs (replicated), their user rows
    through the rank's rows of R;
  * the preference block and the loss (BPR + both InfoNCE terms) on the batch rows
    only ([users; positives; negatives], rsx.smore._calculate_loss_rows' form).
Backward: the UI backbone's gradient is the same operator on (G_U, sum_g G_I,g) —
one all-reduce of G's item rows, then one per layer; the three views' item-row
gradients (their own rows plus R^T of the user rows) are summed over the ranks in
ONE all-reduce before the replicated kNN / gate / spectral / projection backward,
which then runs identically everywhere; the preference weights' gradients (the only
replicated weights fed by rank-local rows) are summed in one all-reduce.  Every
replicated parameter therefore receives the complete, identical gradient and the
replicas stay bit-identical under the per-element Adam; no table is ever gathered.

Exchange per forward + backward pass at C5 (n_items 23,033, d 128: X = 11.8 MB):
4 (UI forward) + 1 + 4 (UI backward) + 3 (views, one call) all-reduces of X + a
0.5 MB weight all-reduce = 12 X per pass, ~2.9 passes per step with the mirror
gradient (DESIGN.md §6 models the time).

Collectives go through `Comm`: over "nccl" an rsx communicator (csrc/dist.hip,
RCCL, stream-ordered, captured with the step's HIP graph), otherwise (gloo, tests)
torch.distributed on host copies.  Compute goes through a backend: `HipSmoreBackend`
(the rsx kernels) or, in the CPU tests, a torch restatement.

Evaluation: every rank ranks its own users against the (replicated) item rows;
rsx.evaluator.sharded_metric_dict all-gathers the metric sums.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import _lib as L
from . import graph, ops

# the SMORE item side as one launch (rsx_smore_item_fwd) instead of the projection +
# spectral + gates chain: same values bit for bit, measured slower, so opt-in
ITEM_FUSED = os.environ.get("RSX_SMORE_ITEM_FUSED", "0") == "1"

# the row-sharded parameter (its rows [a_r, b_r) live on rank r); everything else is replicated
SHARDED = {"user_embedding.weight": "u"}
# with the item side sharded (SmoreShard item_shard): the raw feature tables' rows
ITEM_SHARDED = {"image_embedding.weight": "i", "text_embedding.weight": "i"}
# the preference block's Linear layers: replicated weights fed by rank-local rows
PREF = ("query_v.0", "query_v.2", "query_t.0", "query_t.2", "gate_image_prefer.0", "gate_text_prefer.0",
        "gate_fusion_prefer.0")


def ranges(n: int, world: int):
    return [(r * n // world, (r + 1) * n // world) for r in range(world)]


class Comm:
    """In-place f32 sum all-reduce over the process group.  "nccl": an rsx
    communicator (RCCL through csrc/dist.hip: rsx_comm_allreduce_f32 on the caller's
    stream, capturable in a HIP graph); other backends: torch.distributed on host
    copies (gloo; several ranks may share one GPU)."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.sim = None
        from .dist import sim_comm_params

        sim = sim_comm_params()
        one = not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1
        if sim is not None and one:
            # latency injection (RSX_COMM_SIM=W): this one process is rank 0 of a modelled
            # W-rank job — SmoreShard partitions users and item rows W ways, and every
            # collective is the one-rank identity plus a comm-stream stand-in holding the
            # modelled time, CUs and HBM bytes of that collective (csrc/dist.hip)
            self.world, self.rank, self.native, self.sim = int(sim["world"]), 0, True, sim
            h = C.c_void_p()
            with torch.cuda.device(device):
                L.check(L.lib().rsx_comm_init_sim(C.byref(h), sim["world"], sim["busbw_gbs"], sim["latency_us"],
                                                  sim["blocks"], sim["scratch_mb"]), "rsx_comm_init_sim")
            self.handle = h
            return
        if not (dist.is_available() and dist.is_initialized()):  # rsx_sharded without a group: one rank
            self.world, self.rank, self.native, self.handle = 1, 0, False, None
            return
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.native = dist.get_backend(group) == "nccl"
        self.handle = None
        if self.native and self.world > 1:
            lib = L.lib()
            nb = int(lib.rsx_comm_unique_id_bytes())
            buf = (C.c_uint8 * nb)()
            if self.rank == 0:
                L.check(lib.rsx_comm_get_unique_id(buf), "rsx_comm_get_unique_id")
            uid = torch.tensor(bytearray(bytes(buf)), dtype=torch.uint8, device=device)
            dist.broadcast(uid, src=dist.get_global_rank(group, 0) if group else 0, group=group)
            C.memmove(buf, bytes(uid.cpu().numpy().tobytes()), nb)
            h = C.c_void_p()
            with torch.cuda.device(device):
                L.check(lib.rsx_comm_init(C.byref(h), buf, self.rank, self.world), "rsx_comm_init")
            self.handle = h

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError("Comm.allreduce_: contiguous float32 tensors")
        if self.handle is not None:
            L.check(L.lib().rsx_comm_allreduce_f32(self.handle, t.data_ptr(), t.numel(), ops._stream()),
                    "rsx_comm_allreduce_f32")
            return t
        h = t.cpu() if t.is_cuda else t
        dist.all_reduce(h, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def allreduce_start_(self, t: torch.Tensor):
        """allreduce_ without the wait (RCCL: on the communicator's stream; the caller's
        stream runs on until wait()); host collectives are synchronous."""
        if self.world == 1:
            return t
        if self.handle is not None:
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("Comm.allreduce_start_: contiguous float32 tensors")
            L.check(L.lib().rsx_comm_allreduce_f32_start(self.handle, t.data_ptr(), t.numel(), ops._stream()),
                    "rsx_comm_allreduce_f32_start")
            return t
        return self.allreduce_(t)

    def wait(self):
        if self.handle is not None:
            L.check(L.lib().rsx_comm_wait(self.handle, ops._stream()), "rsx_comm_wait")

    def allgather_(self, t: torch.Tensor, count: int) -> torch.Tensor:
        """t[r count:(r+1) count] := rank r's slice, every r (t: world * count floats)."""
        if self.world == 1:
            return t
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < self.world * count:
            raise RuntimeError("Comm.allgather_: a contiguous float32 tensor of world * count elements")
        if self.handle is not None:
            # (the stand-in is given the whole world * count buffer: its byte count is the buffer's)
            n = int(count) * (self.world if self.sim else 1)
            L.check(L.lib().rsx_comm_allgather_f32(self.handle, t.data_ptr(), n, ops._stream()),
                    "rsx_comm_allgather_f32")
            return t
        flat = t.view(-1)
        mine = flat[self.rank * count:(self.rank + 1) * count].cpu()
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine, group=self.group)
        flat[: self.world * count].copy_(torch.cat(parts).to(t.device))
        return t

    def close(self):
        if self.handle is not None:
            torch.cuda.synchronize()
            L.lib().rsx_comm_destroy(self.handle)
            self.handle = None


class _AllReduceGrad(torch.autograd.Function):
    """Identity forward; backward: the gradients of all inputs summed over the ranks in
    one all-reduce (replicated tensors fed by rank-local work)."""

    @staticmethod
    def forward(ctx, comm, *ts):
        ctx.comm = comm
        ctx.shapes = [t.shape for t in ts]
        return tuple(t.view_as(t) for t in ts)

    @staticmethod
    def backward(ctx, *gs):
        ref = next(g for g in gs if g is not None)
        flat = torch.cat([(g if g is not None else torch.zeros(s, dtype=ref.dtype, device=ref.device)).reshape(-1)
                          for g, s in zip(gs, ctx.shapes)])
        ctx.comm.allreduce_(flat)
        out, o = [], 0
        for s in ctx.shapes:
            n = int(np.prod(s)) if len(s) else 1
            out.append(flat[o:o + n].view(s))
            o += n
        return (None, *out)


def allreduce_grad(comm, *ts):
    return _AllReduceGrad.apply(comm, *ts)


class RowGradExchange:
    """Data-parallel SMORE's one exchange per backward (rsx.smore scheme "dp"): every table
    replicated, each rank its own batch, the objective the sum over ranks of the reference
    loss of each rank's batch (src/models/smore.py:366-411).  Every path from a rank's
    loss to the parameters runs through the preference block on its batch rows
    (smore.py:320-341), so that block's backward is the exchange point:

    * its four [N, d] table gradients (content, image, text, fusion), defined on this
      rank's batch rows, are packed one entry per occurrence (a flag on each row's first
      occurrence), all-gathered, and every rank rebuilds the same tables on the union of
      the ranks' rows: the rows zeroed, then each rank's rows added in rank order
      (csrc/rowx.hip: no float atomics, so all ranks hold the same bits);
    * its seven weights' and biases' gradients (rank-local rows) are summed in one
      all-reduce, which leaves the same bits on every rank.

    The rest of the backward (UI backbone, the views, the item side) then runs on
    identical inputs everywhere: identical parameter gradients, replicas that stay
    bit-identical under the per-element Adam, and no other collective in the step.
    `union` receives the union row list (the tag-aware backward consumers re-tag it).
    Off the GPU (gloo tests) the same steps run as torch ops."""

    T = 4

    def __init__(self, comm: Comm, n_rows: int, d: int, n_max: int, device):
        self.comm, self.d, self.n_max = comm, int(d), int(n_max)
        self.device = torch.device(device)
        self.hip = self.device.type == "cuda"
        W = comm.world
        self.E = 4 + self.T * self.d
        self.packed = torch.zeros(W, self.n_max, self.E, dtype=torch.float32, device=self.device)
        self.union = torch.zeros(W * self.n_max, dtype=torch.int64, device=self.device)
        self.lead = torch.zeros(int(n_rows), dtype=torch.int64, device=self.device)
        self.tag = torch.zeros(1, dtype=torch.int32, device=self.device)

    def exchange(self, rows: torch.Tensor, tables, wgrads):
        """tables: the T [N, d] gradients (valid on `rows`; rebuilt in place on the union
        rows); wgrads: weight / bias gradients (None entries kept), returned summed."""
        self.start(rows, tables)
        return self.finish(tables, wgrads)

    def start(self, rows: torch.Tensor, tables):
        """Pack this rank's rows and all-gather the packs.  (The all-gather is joined before
        the caller's next launch: started asynchronously beside the preference weights'
        gradient products, the captured C5 step replayed at 9.3-10.4 ms instead of 6.0-6.4
        under latency injection, profiles/r06/c5_dp/overlap_dropped/ -- the same pathology as
        a side-stream branch next to the comm branch, §6.5 of DESIGN.md.)"""
        n = int(rows.numel())
        if n > self.n_max or n < 1:
            raise RuntimeError(f"RowGradExchange: {n} batch rows (capacity {self.n_max})")
        W, r = self.comm.world, self.comm.rank
        if self.hip:
            lib = L.lib()
            tp = (C.c_void_p * self.T)(*[t.data_ptr() for t in tables])
            L.check(lib.rsx_rowx_pack(ops._p(rows), n, self.n_max, tp, self.T, self.d, ops._p(self.lead),
                                      ops._p(self.tag), ops._p(self.packed[r]), ops._stream()), "rsx_rowx_pack")
        else:
            self._pack_torch(rows, tables, self.packed[r])
        if self.comm.sim is not None:
            # latency injection: the modelled peers' packs are this rank's (so the combine does
            # the work of W real packs; the collective itself is the modelled stand-in)
            for q in range(W):
                if q != r:
                    self.packed[q].copy_(self.packed[r])
        self.comm.allgather_(self.packed.view(-1), self.n_max * self.E)

    def finish(self, tables, wgrads):
        """Rebuild the tables on the union rows, sum the weights' gradients (one
        all-reduce); returns the summed weight gradients."""
        W = self.comm.world
        if self.hip:
            tp = (C.c_void_p * self.T)(*[t.data_ptr() for t in tables])
            L.check(L.lib().rsx_rowx_combine(ops._p(self.packed), W, self.n_max, tp, self.T, self.d,
                                             ops._p(self.union), ops._stream()), "rsx_rowx_combine")
        else:
            self._combine_torch(tables)
        live = [g for g in wgrads if g is not None]
        if live and W > 1:
            flat = torch.cat([g.reshape(-1) for g in live])
            self.comm.allreduce_(flat)
            out, o = [], 0
            for g in wgrads:
                if g is None:
                    out.append(None)
                    continue
                out.append(flat[o:o + g.numel()].view_as(g))
                o += g.numel()
            wgrads = out
        return wgrads

    # the CPU statement of csrc/rowx.hip (gloo tests)
    def _pack_torch(self, rows, tables, out):
        n, d = rows.numel(), self.d
        first = torch.zeros(n, dtype=torch.bool)
        seen = set()
        for j, x in enumerate(rows.tolist()):
            if x not in seen:
                seen.add(x)
                first[j] = True
        out.zero_()
        head = torch.full((self.n_max,), int(rows[0]), dtype=torch.int64)  # padding names a real row
        head[:n] = rows.cpu()
        out[:, :2] = _i64_words(head).to(out.device)
        out[:n, 2] = first.float().to(out.device)
        for t, tab in enumerate(tables):
            out[:n, 4 + t * d:4 + (t + 1) * d] = tab[rows]

    def _combine_torch(self, tables):
        d, W = self.d, self.comm.world
        ents = self.packed.view(W * self.n_max, self.E)
        rows = _words_i64(ents[:, :2])
        self.union.copy_(rows)
        for tab in tables:
            tab[rows] = 0.0
        for q in range(W):
            e = self.packed[q]
            sel = e[:, 2] != 0
            rq = _words_i64(e[sel, :2])
            for t, tab in enumerate(tables):
                tab[rq] += e[sel, 4 + t * d:4 + (t + 1) * d]


def _i64_words(x: torch.Tensor) -> torch.Tensor:
    """int64 [n] -> its two 32-bit words as float32 [n, 2] (a bit copy, as the kernel's)."""
    return x.contiguous().view(torch.int32).view(-1, 2).view(torch.float32)


def _words_i64(w: torch.Tensor) -> torch.Tensor:
    return w.contiguous().view(torch.int32).view(torch.int64).view(-1)


class _GatherRows(torch.autograd.Function):
    """Every rank's rows of k row-sharded tables (rank r: rows [r q, r q + n_r) of each,
    n_r <= q) gathered into [k, n, d] on every rank in ONE all-gather of [k, q, d] slices
    (padded); backward: the replicated gradient's own rows (no exchange: the gradient of
    a replicated consumer is the same on every rank)."""

    @staticmethod
    def forward(ctx, comm, q, n, *own):
        k = len(own)
        n_r, d = own[0].shape
        W, r = comm.world, comm.rank
        buf = torch.zeros(W, k, q, d, dtype=torch.float32, device=own[0].device)
        for j, x in enumerate(own):
            buf[r, j, :n_r].copy_(x)
        comm.allgather_(buf, k * q * d)
        out = buf.permute(1, 0, 2, 3).reshape(k, W * q, d)[:, :n].contiguous()
        ctx.rq = (r * q, r * q + n_r)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.rq
        return (None, None, None, *[g[j, a:b] for j in range(g.shape[0])])


def gather_rows(comm, q, n, *own):
    return _GatherRows.apply(comm, q, n, *own)


def item_ranges(n_items: int, world: int):
    """Rank r's item rows [r q, min((r+1) q, n_items)), q = ceil(n_items / world): equal
    slices (the last may be shorter), so one all-gather of q-row slices lines them up."""
    q = -(-n_items // world)
    return q, [(min(r * q, n_items), min((r + 1) * q, n_items)) for r in range(world)]


# the item side's weights: each rank's gradient covers its own item rows only
ITEM_W = ("image_trs.weight", "image_trs.bias", "text_trs.weight", "text_trs.bias", "image_complex_weight",
          "text_complex_weight", "fusion_complex_weight", "gate_v.0.weight", "gate_v.0.bias", "gate_t.0.weight",
          "gate_t.0.bias", "gate_f.0.weight", "gate_f.0.bias")


class _UIProp(torch.autograd.Function):
    """content = mean_{k=0..K} A^k E0 of the users-sharded UI graph, rows [own users;
    all items] (the item rows identical on every rank).  A is symmetric, so the
    backward is the same operator applied to (G_U, sum over ranks of G_I)."""

    @staticmethod
    def forward(ctx, x, core):
        ctx.core = core
        return core.ui_mean(x.contiguous())

    @staticmethod
    def backward(ctx, g):
        core = ctx.core
        g = g.contiguous().clone()
        core.comm.allreduce_(g[core.nu_own:])
        return core.ui_mean(g), None


# ---------------------------------------------------------------------------
# backends
# ---------------------------------------------------------------------------
class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class HipSmoreBackend:
    """The rsx kernels (the single-process rsx.smore.SMORE's path)."""

    def __init__(self, device, chunk=32):
        self.device = ops.require_device(device)
        self.chunk = chunk
        self._side = None

    def side_stream(self):
        """The UI backbone's stream (RSX_SMORE_STREAMS=0: none)."""
        import os

        if os.environ.get("RSX_SMORE_STREAMS", "1") == "0":
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def operator(self, rowptr, col, val, n_cols, transpose=False):
        """A device CSR of a local row block (and, with transpose, the pair (A, A^T) for a
        product whose backward multiplies by A^T)."""
        A = ops.DeviceCSR(rowptr, col, val, n_cols, self.device, self.chunk)
        if not transpose:
            return A
        n_rows = rowptr.size - 1
        rows = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(rowptr))
        AT = ops.DeviceCSR(*graph.to_csr(col.astype(np.int64), rows, val, n_cols, n_rows), n_rows, self.device,
                           self.chunk)
        return _Pair(A, AT)

    def ui_mean(self, core, x):
        """mean over layers with the running sums in the SpMM epilogues (users) and one
        all-reduce of every item partial (its running sum a row-wise ADD after it)."""
        nu, K, d = core.nu_own, core.K, x.shape[1]
        ni = x.shape[0] - nu
        out = torch.empty_like(x)
        s = torch.empty_like(x)
        bufs = torch.empty(2, *x.shape, dtype=torch.float32, device=x.device)
        cur = x
        beta = 1.0 / (K + 1)
        for k in range(1, K + 1):
            y = bufs[k & 1]
            s_in = x if k == 1 else s
            # item partial = A_I users^{k-1}, summed over the ranks; the exchange runs on the
            # communicator's stream while this layer's user rows (they read the previous
            # layer's items only) are computed
            core.A_I.spmm_epi(cur[:nu], ops.epi(L.RSX_EPI_STORE, y=y[nu:]), d)
            core.comm.allreduce_start_(y[nu:])
            if k < K:
                core.A_U.spmm_epi(cur[nu:], ops.epi(L.RSX_EPI_LAYERSUM, y=y[:nu], s_in=s_in[:nu], s_out=s[:nu]), d)
                core.comm.wait()
                ops.rowwise(ni, d, ops.epi(L.RSX_EPI_ADD, y=s[nu:], s_in=s_in[nu:], r_add=y[nu:]))
            else:
                core.A_U.spmm_epi(cur[nu:], ops.epi(L.RSX_EPI_FINAL, beta=beta, f=out[:nu], s_in=s_in[:nu]), d)
                core.comm.wait()
                ops.rowwise(ni, d, ops.epi(L.RSX_EPI_ADD, beta=beta, y=out[nu:], s_in=s_in[nu:], r_add=y[nu:]))
            cur = y
        if K == 0:
            out.copy_(x)
        return out

    def spectral(self, m):
        from .smore_spectral import spectral

        return spectral(m.image_embedding.weight, m.image_trs.weight, m.image_trs.bias, m.text_embedding.weight,
                        m.text_trs.weight, m.text_trs.bias, m.image_complex_weight, m.text_complex_weight,
                        m.fusion_complex_weight, getattr(m, "spectral_weight_norm", True))[:3]

    def gates(self, m, cv, ct, cf, item):
        from . import smore_fuse as SF

        return SF.gates(cv, ct, cf, item, m.gate_v, m.gate_t, m.gate_f, m.inject_scale, False)

    def item_side(self, m, item):
        """spectral + gates as the one-launch item side (rsx_smore_item_fwd)."""
        from .smore_spectral import item_side

        return item_side(m.image_embedding.weight, m.image_trs.weight, m.image_trs.bias, m.text_embedding.weight,
                         m.text_trs.weight, m.text_trs.bias, m.image_complex_weight, m.text_complex_weight,
                         m.fusion_complex_weight, item, m.gate_v, m.gate_t, m.gate_f, m.inject_scale, False,
                         getattr(m, "spectral_weight_norm", True))[:3]

    def item_side_sharded(self, core, m, item):
        """Projection -> spectral -> the gates' inject term on this rank's item rows only
        (the fused kernels on n_own rows), gathered once; + the replicated item-id table."""
        from . import smore_fuse as SF
        from .smore_spectral import _ItemSide, spectral

        w = dict(zip(ITEM_W, allreduce_grad(core.comm, *[m.get_parameter(n) for n in ITEM_W])))
        # the gates' item operand is zero: the kernels write the inject term alone
        zero = core.zero_rows(m.image_embedding.weight.shape[0], item.shape[1], item.device)
        norm = bool(getattr(m, "spectral_weight_norm", True))
        if ITEM_FUSED:
            dv, dt, df = _ItemSide.apply(m.image_embedding.weight, w["image_trs.weight"], w["image_trs.bias"],
                                         m.text_embedding.weight, w["text_trs.weight"], w["text_trs.bias"],
                                         w["image_complex_weight"], w["text_complex_weight"],
                                         w["fusion_complex_weight"], zero, w["gate_v.0.weight"], w["gate_v.0.bias"],
                                         w["gate_t.0.weight"], w["gate_t.0.bias"], w["gate_f.0.weight"],
                                         w["gate_f.0.bias"], norm, float(m.inject_scale), False)[:3]
        else:
            cv, ct, cf, _, _ = spectral(m.image_embedding.weight, w["image_trs.weight"], w["image_trs.bias"],
                                        m.text_embedding.weight, w["text_trs.weight"], w["text_trs.bias"],
                                        w["image_complex_weight"], w["text_complex_weight"],
                                        w["fusion_complex_weight"], norm)
            dv, dt, df = SF._Gates.apply(cv, ct, cf, zero, w["gate_v.0.weight"], w["gate_v.0.bias"],
                                         w["gate_t.0.weight"], w["gate_t.0.bias"], w["gate_f.0.weight"],
                                         w["gate_f.0.bias"], float(m.inject_scale), False)
        D = gather_rows(core.comm, core.iq, core.n_items, dv, dt, df)
        return (D + item.unsqueeze(0)).unbind(0)

    def views(self, core, xs):
        from . import smore_fuse as SF

        return SF.view_prop3(xs, core.G, core.R, core.L, core.nu_own, comm=core.comm)

    def pref_rows(self, m, content, views, rows, seed, weights):
        from . import smore_fuse as SF

        return SF.preference_rows(m, content, *views, rows, seed, weights=weights)

    def pref_full(self, m, content, views, seed):
        from . import smore_fuse as SF

        return SF.preference(m, content, *views, seed)

    def loss_rows(self, m, all_c, side_c, content_c, trip, ar, B):
        from . import smore_fuse as SF

        total, parts = SF.smore_loss_rows(all_c, side_c, content_c, trip, ar, B, m.reg_weight, m.batch_size,
                                          m.cl_loss, m.cl_temp)
        return total


class _Pair:
    """(A, A^T) device CSRs: the forward product and its transpose for the backward."""

    def __init__(self, A, AT):
        self.A, self.AT = A, AT


# ---------------------------------------------------------------------------
# the sharded computation
# ---------------------------------------------------------------------------
class SmoreShard:
    """The users-sharded SMORE step and evaluation over a parameter holder `m` that has
    the reference's module layout (rsx.smore.SMORE in sharded mode, or a test container):
    m.user_embedding.weight holds this rank's user rows, the rest the full tables."""

    def __init__(self, graphs: dict, n_users: int, n_items: int, n_ui_layers: int, n_layers: int, backend,
                 comm: Comm, item_shard: bool = False):
        self.be, self.comm = backend, comm
        self.world, self.rank = comm.world, comm.rank
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.urng = ranges(self.n_users, self.world)
        a, b = self.urng[self.rank]
        self.own_u = (a, b)
        self.nu_own = b - a
        self.K, self.L = int(n_ui_layers), int(n_layers)
        nu, ni = self.n_users, self.n_items
        rp, col, val = graphs["norm_adj"]
        # A_U: own user rows, item columns rebased to 0..ni; A_I: item rows, own-user columns rebased to 0..nu_own
        up, uc, uv = csr_rows(rp, col, val, a, b)
        self.A_U = backend.operator(up, uc.astype(np.int64) - nu, uv, ni)
        ip, ic, iv = csr_rows(rp, col, val, nu, nu + ni)
        rows = np.repeat(np.arange(ni, dtype=np.int64), np.diff(ip))
        keep = (ic >= a) & (ic < b)
        self.A_I = backend.operator(*graph.to_csr(rows[keep], ic[keep].astype(np.int64) - a, iv[keep], ni,
                                                  self.nu_own), self.nu_own)
        # the kNN item graphs (replicated): prebuilt (A, A^T) pairs or host CSRs
        self.G = tuple(graphs[v] if hasattr(graphs[v], "AT") else backend.operator(*graphs[v], ni, transpose=True)
                       for v in ("image", "text", "fusion"))
        rrp, rcol, rval = graphs["R"]
        self.R = backend.operator(*csr_rows(rrp, rcol, rval, a, b), ni, transpose=True)
        self._rows_cache = {}
        # the item side (projection, spectral fusion, the gates' inject term) on this rank's
        # item rows only, the raw feature tables row-sharded with it (rank r: rows
        # [r q, (r+1) q)); the three inject tables gathered once per forward
        self.iq, irng = item_ranges(ni, self.world)
        self.own_i = irng[self.rank]
        self.item_shard = bool(item_shard) and self.world > 1 and all(b_ > a_ for a_, b_ in irng)
        self._zero = None

    # -- pieces -----------------------------------------------------------------
    def ui_mean(self, x):
        return self.be.ui_mean(self, x)

    def zero_rows(self, n, d, device):
        """A zero [n_own_items, d] table (the gates' item operand: the inject term alone)."""
        z = self._zero
        if z is None or z.shape != (n, d) or z.device != torch.device(device):
            self._zero = z = torch.zeros(n, d, dtype=torch.float32, device=device)
        return z

    def _item_side(self, m, item=None):
        item = m.item_id_embedding.weight if item is None else item
        if self.item_shard:
            return self.be.item_side_sharded(self, m, item)
        if ITEM_FUSED and hasattr(self.be, "item_side"):
            return self.be.item_side(m, item)
        cv, ct, cf = self.be.spectral(m)
        return self.be.gates(m, cv, ct, cf, item)

    def _content_views(self, m):
        """The UI backbone (with its per-layer all-reduces) on a side stream of the HIP
        backend, concurrent with the replicated item side, so its exchanges hide behind
        the projection / spectral / gate kernels (and likewise in the backward, which
        autograd runs on the same streams)."""
        # (not with an rsx communicator: a collective forked from a side stream that joined a
        # graph capture makes HIP's capture end segfault -- tools/gpu/diag_smore_sim.py,
        # pattern `side`, DESIGN §6 -- so the native-comm step keeps the UI backbone and its
        # all-reduces on the capturing stream, where the fork is the DP / row-sharded steps')
        side = self.be.side_stream() if hasattr(self.be, "side_stream") and not self.comm.native else None
        main = torch.cuda.current_stream() if side is not None else None
        # every leaf enters through a view made here, on one stream (rsx.smore._views_fused)
        uw = m.user_embedding.weight.view_as(m.user_embedding.weight)
        iw = m.item_id_embedding.weight.view_as(m.item_id_embedding.weight)
        if side is not None:
            side.wait_stream(main)
        with torch.cuda.stream(side) if side is not None else _Null():
            ego = torch.cat([uw, iw])
            content = _UIProp.apply(ego, self)
        img, txt, fus = self._item_side(m, iw)
        if side is not None:
            main.wait_stream(side)
            content.record_stream(main)
        return content, self.be.views(self, (img, txt, fus))

    def pref_weights(self, m):
        """The preference block's weights and biases, their gradients summed over the ranks."""
        lin = [m.get_submodule(n) for n in PREF]
        ws = [x.weight for x in lin] + [x.bias for x in lin if x.bias is not None]
        out = allreduce_grad(self.comm, *ws)
        w, b = list(out[:7]), iter(out[7:])
        return w + [next(b) if x.bias is not None else None for x in lin]

    def _rows(self, B, device):
        c = self._rows_cache.get(B)
        if c is None:
            ar = torch.arange(B, dtype=torch.int64, device=device)
            off = torch.cat([torch.zeros(B, dtype=torch.int64, device=device),
                             torch.full((2 * B,), self.nu_own, dtype=torch.int64, device=device)])
            c = self._rows_cache[B] = (ar, torch.stack([ar, ar, ar + B]).contiguous(), off)
        return c

    # -- training ---------------------------------------------------------------
    def loss(self, m, inter, seed):
        """The reference loss of this rank's batch `inter` [3, B] (users as local row ids
        0..nu_own-1, items global): BPR + reg + cl * (InfoNCE(items) + InfoNCE(users)) on
        the batch rows, with the collectives above in its backward."""
        B = int(inter.shape[1])
        ar, trip, off = self._rows(B, inter.device)
        rows = inter[:3].reshape(-1) + off
        content, views = self._content_views(m)
        all_c, side_c, content_c = self.be.pref_rows(m, content, views, rows, seed, self.pref_weights(m))
        return self.be.loss_rows(m, all_c, side_c, content_c, trip, ar, B)

    # -- evaluation ---------------------------------------------------------------
    @torch.no_grad()
    def tables(self, m, seed):
        """all_embeds rows [own users; all items] (evaluation forward, no dropout)."""
        content, views = self._content_views(m)
        all_e, _ = self.be.pref_full(m, content, views, seed)
        return all_e

    @torch.no_grad()
    def full_sort_topk_local(self, m, seed, eval_users, k, mask_rowptr, mask_col):
        """(positions in eval_users of this rank's users, their top-k item ids)."""
        a, b = self.own_u
        pos = torch.nonzero((eval_users >= a) & (eval_users < b)).flatten()
        local = (eval_users.index_select(0, pos) - a).contiguous()
        f = self.tables(m, seed)
        nl = self.nu_own
        _, topk = ops.fullsort_topk(f[:nl].contiguous(), local, f[nl:].contiguous(), mask_rowptr[a:], mask_col, k)
        return pos, topk

    # -- mirror gradient -----------------------------------------------------------
    @torch.no_grad()
    def mg_alpha(self, m, params, grads, base, lr, rel_step, max_scale, lr_dev=None):
        """alpha_eff of the reference's mirror gradient (src/common/trainer.py:290-307) over
        the GLOBAL parameter vector, as a 0-d f64 device tensor (no host sync): sums of
        squares of the row-sharded user table summed over the ranks (one all-reduce),
        the replicated parameters counted once."""
        sharded = {id(m.user_embedding.weight)}
        if self.item_shard:  # the raw feature tables: this rank's item rows
            sharded |= {id(m.image_embedding.weight), id(m.text_embedding.weight)}
        sh_g = [g for p, g in zip(params, grads) if id(p) in sharded]
        sh_p = [p.detach() for p in params if id(p) in sharded]
        rp_g = [g for p, g in zip(params, grads) if id(p) not in sharded]
        rp_p = [p.detach() for p in params if id(p) not in sharded]
        dev = params[0].device

        def sq(ts):
            if not ts:
                return torch.zeros((), dtype=torch.float64, device=dev)
            return torch.stack([n.double() for n in torch._foreach_norm(ts)]).pow(2).sum()

        part = torch.stack([sq(sh_g), sq(sh_p), torch.full((), float(sum(p.numel() for p in sh_p)),
                                                           dtype=torch.float64, device=dev)]).float()
        self.comm.allreduce_(part)
        tot = part.double() + torch.stack([sq(rp_g), sq(rp_p), torch.full((), float(sum(p.numel() for p in rp_p)),
                                                                             dtype=torch.float64, device=dev)])
        n = tot[2]
        grad_rms = (tot[0].sqrt().float() / n.sqrt().float()).double()
        param_rms = (tot[1].sqrt().float() / n.sqrt().float() + 1e-12).double()
        lr_t = lr_dev[0] if lr_dev is not None else torch.full((), float(lr), dtype=torch.float64, device=dev)
        alpha = rel_step * param_rms / (lr_t * grad_rms + 1e-12)
        alpha = torch.where(alpha > base, alpha, torch.full_like(alpha, base))
        return torch.clamp(alpha, max=base * max_scale)


def csr_rows(rowptr, col, val, r0: int, r1: int):
    """Rows [r0, r1) of a host CSR (columns unchanged)."""
    a, b = int(rowptr[r0]), int(rowptr[r1])
    return rowptr[r0:r1 + 1] - a, col[a:b], val[a:b]


def graphs_from_rsx(model):
    """Host CSRs of a single-process rsx.smore.SMORE's operators."""
    def host(A):
        return A.rowptr_host, A.col.cpu().numpy(), A.val.cpu().numpy()

    return {"norm_adj": host(model.norm_adj_csr), "image": host(model.image_graph.A),
            "text": host(model.text_graph.A), "fusion": host(model.fusion_graph.A), "R": host(model.R.A)}


def param_container(params: dict, cfg: dict, user_range, device="cpu", item_range=None):
    """An nn.Module with the reference's SMORE parameter layout holding `params` (full
    tables; the user table cut to `user_range`, with `item_range` the raw feature tables
    cut to those item rows) — the parameter holder of the CPU tests and of tools that
    drive SmoreShard without rsx.smore.SMORE."""
    m = nn.Module()
    a, b = user_range
    d = params["user_embedding.weight"].shape[1]
    lin = lambda i, o, bias=True: nn.Linear(i, o, bias=bias, device=device)  # noqa: E731
    dv, dt = params["image_trs.weight"].shape[1], params["text_trs.weight"].shape[1]
    for name in ("user_embedding", "item_id_embedding", "image_embedding", "text_embedding"):
        setattr(m, name, nn.Module())
    m.image_trs, m.text_trs = lin(dv, d), lin(dt, d)
    m.query_v = nn.Sequential(lin(d, d), nn.Tanh(), lin(d, d, False))
    m.query_t = nn.Sequential(lin(d, d), nn.Tanh(), lin(d, d, False))
    for g in ("gate_v", "gate_t", "gate_f", "gate_image_prefer", "gate_text_prefer", "gate_fusion_prefer"):
        setattr(m, g, nn.Sequential(lin(d, d), nn.Sigmoid()))
    m.dropout = nn.Dropout(p=float(cfg.get("dropout_rate", 0.0)))
    for name, full in params.items():
        full = torch.as_tensor(full, dtype=torch.float32)
        if SHARDED.get(name) == "u":
            full = full[a:b]
        elif item_range is not None and ITEM_SHARDED.get(name) == "i":
            full = full[item_range[0]:item_range[1]]
        obj = m
        *path, leaf = name.split(".")
        for k in path:
            obj = obj[int(k)] if k.isdigit() else getattr(obj, k)
        obj._parameters.pop(leaf, None)
        obj.register_parameter(leaf, nn.Parameter(full.clone().to(device)))
    m.reg_weight = float(cfg.get("reg_weight", 1e-5))
    m.cl_loss = float(cfg.get("cl_loss", 0.01))
    m.cl_temp = float(cfg.get("cl_temp", 0.2))
    m.batch_size = float(cfg.get("batch_size", 2048))
    m.inject_scale = float(cfg.get("inject_scale", 0.7))
    m.spectral_weight_norm = True
    return m
