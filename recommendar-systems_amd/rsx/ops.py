"""Torch-tensor wrappers over the librsx C ABI (device memory and streams come from torch).

Every op checks that its tensors live on the GPU and raises otherwise: there is
no CPU fallback on the product path.  Each wrapper cites the reference call
site it replaces (paths relative to the reference root).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _pi(t):
    return 0 if t is None else t.data_ptr()


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("rsx ops run on the GPU (HIP kernels); got a CPU tensor")
        if t is not None and not t.is_contiguous():
            raise RuntimeError("rsx ops need contiguous tensors")


def require_device(device) -> torch.device:
    device = torch.device(device)
    if device.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("rsx: the HIP path needs a ROCm GPU (config use_gpu/device); no CPU fallback")
    L.lib()
    return device


# ---------------------------------------------------------------------------
# CSR adjacency + schedule
# ---------------------------------------------------------------------------
class DeviceCSR:
    """Row-major CSR on the device plus the nnz-balanced work schedule.

    Built once per graph from host arrays (rowptr int64, col int32, val f32).
    Replaces the torch COO adjacency of reference src/models/lightgcn.py:65-103.
    """

    def __init__(self, rowptr: np.ndarray, col, val, n_cols: int, device, chunk: int = 32):
        """rowptr: host int64 [n_rows+1]; col / val: host arrays, or int32 / float32
        tensors already on `device` (then used in place, see from_device)."""
        lib = L.lib()
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        on_dev = torch.is_tensor(col)
        if not on_dev:
            col = np.ascontiguousarray(col, dtype=np.int32)
            val = np.ascontiguousarray(val, dtype=np.float32)
        n_rows = rowptr.size - 1
        nw, nl, ns = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(lib.rsx_csr_schedule_host(rowptr.ctypes.data_as(C.c_void_p), n_rows, chunk, None, None,
                                          C.byref(nw), C.byref(nl), C.byref(ns)), "rsx_csr_schedule_host")
        work = np.zeros((max(nw.value, 1), 4), dtype=np.int32)
        longr = np.zeros((max(nl.value, 1), 4), dtype=np.int32)
        L.check(lib.rsx_csr_schedule_host(rowptr.ctypes.data_as(C.c_void_p), n_rows, chunk,
                                          work.ctypes.data_as(C.c_void_p), longr.ctypes.data_as(C.c_void_p),
                                          C.byref(nw), C.byref(nl), C.byref(ns)), "rsx_csr_schedule_host")
        self.device = torch.device(device)
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.nnz = int(col.numel()) if on_dev else int(col.size)
        if self.nnz != int(rowptr[-1]):
            raise RuntimeError(f"DeviceCSR: rowptr ends at {int(rowptr[-1])}, {self.nnz} nonzeros given")
        self.chunk = chunk
        self.n_work, self.n_long, self.n_slots = nw.value, nl.value, ns.value
        self.rowptr_host = rowptr
        self.rowptr = torch.from_numpy(rowptr).to(self.device)
        if on_dev:
            if col.dtype != torch.int32 or val.dtype != torch.float32 or col.device != self.device \
                    or val.device != self.device or not (col.is_contiguous() and val.is_contiguous()):
                raise RuntimeError("DeviceCSR: device col/val must be contiguous int32/float32 on the CSR's device")
            self.col, self.val = col, val
        else:
            self.col = torch.from_numpy(col).to(self.device)
            self.val = torch.from_numpy(val).to(self.device)
        self.work = torch.from_numpy(work).to(self.device)
        self.long_rows = torch.from_numpy(longr).to(self.device)
        self.struct = L.Csr(self.n_rows, self.n_cols, self.nnz, self.rowptr.data_ptr(), self.col.data_ptr(),
                            self.val.data_ptr(), chunk, 0, self.n_work, self.work.data_ptr(), self.n_long,
                            self.long_rows.data_ptr(), self.n_slots)
        self._slabs = {}

    @classmethod
    def from_device(cls, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n_cols: int,
                    chunk: int = 32):
        """A CSR built on the device: only rowptr comes to the host (one copy, for
        the work schedule, rsx_csr_schedule_host); col / val stay where they are."""
        return cls(rowptr.cpu().numpy(), col, val, n_cols, col.device, chunk)

    @classmethod
    def rebind(cls, tmpl: "DeviceCSR", rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor) -> "DeviceCSR":
        """A device-built CSR whose every row has at most the template's nonzeros (an
        edge-dropout graph of it) on the template's work layout: the schedule is
        rewritten on the device (rsx_csr_schedule_rebind), nothing comes to the host,
        and the template's long-row table and partial-sum slabs are shared (a graph
        and its template must not run in the same launch)."""
        self = cls.__new__(cls)
        self.device = tmpl.device
        self.n_rows, self.n_cols, self.chunk = tmpl.n_rows, tmpl.n_cols, tmpl.chunk
        self.nnz = int(col.numel())
        self.n_work, self.n_long, self.n_slots = tmpl.n_work, tmpl.n_long, tmpl.n_slots
        self.rowptr_host = None
        self.rowptr = rowptr.contiguous()
        if col.dtype != torch.int32 or val.dtype != torch.float32 or not (col.is_contiguous() and val.is_contiguous()):
            raise RuntimeError("DeviceCSR.rebind: contiguous int32 col / float32 val expected")
        self.col, self.val = col, val
        self.work = torch.empty_like(tmpl.work)
        L.check(L.lib().rsx_csr_schedule_rebind(C.byref(tmpl.struct), _p(self.rowptr), _p(self.work), _stream()),
                "rsx_csr_schedule_rebind")
        self.long_rows = tmpl.long_rows
        self.struct = L.Csr(self.n_rows, self.n_cols, self.nnz, self.rowptr.data_ptr(), self.col.data_ptr(),
                            self.val.data_ptr(), self.chunk, 0, self.n_work, self.work.data_ptr(), self.n_long,
                            self.long_rows.data_ptr(), self.n_slots)
        self._slabs = tmpl._slabs
        self._tmpl = tmpl
        return self

    @classmethod
    def row_slice(cls, parent: "DeviceCSR", r0: int, r1: int) -> "DeviceCSR":
        """Rows [r0, r1) of a host-scheduled CSR as a CSR of its own: its own work
        schedule (row ids local to the slice, nonzero offsets into the parent's col / val,
        which are shared) and its own slabs.  A product over it writes rows y[0 : r1-r0]
        bit-identically to the parent's rows r0..r1 (same chunks, same fixup order)."""
        if parent.rowptr_host is None or not 0 <= r0 < r1 <= parent.n_rows:
            raise RuntimeError("DeviceCSR.row_slice: a host-scheduled CSR and 0 <= r0 < r1 <= n_rows")
        lib = L.lib()
        rp = np.ascontiguousarray(parent.rowptr_host[r0:r1 + 1])
        nw, nl, ns = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(lib.rsx_csr_schedule_host(rp.ctypes.data_as(C.c_void_p), r1 - r0, parent.chunk, None, None,
                                          C.byref(nw), C.byref(nl), C.byref(ns)), "rsx_csr_schedule_host")
        work = np.zeros((max(nw.value, 1), 4), dtype=np.int32)
        longr = np.zeros((max(nl.value, 1), 4), dtype=np.int32)
        L.check(lib.rsx_csr_schedule_host(rp.ctypes.data_as(C.c_void_p), r1 - r0, parent.chunk,
                                          work.ctypes.data_as(C.c_void_p), longr.ctypes.data_as(C.c_void_p),
                                          C.byref(nw), C.byref(nl), C.byref(ns)), "rsx_csr_schedule_host")
        self = cls.__new__(cls)
        self.device = parent.device
        self.n_rows, self.n_cols, self.chunk = r1 - r0, parent.n_cols, parent.chunk
        self.nnz = int(rp[-1] - rp[0])
        self.n_work, self.n_long, self.n_slots = nw.value, nl.value, ns.value
        self.rowptr_host = rp
        self.rowptr = parent.rowptr[r0:r1 + 1]
        self.col, self.val = parent.col, parent.val
        self.work = torch.from_numpy(work).to(self.device)
        self.long_rows = torch.from_numpy(longr).to(self.device)
        self.struct = L.Csr(self.n_rows, self.n_cols, self.nnz, self.rowptr.data_ptr(), self.col.data_ptr(),
                            self.val.data_ptr(), self.chunk, 0, self.n_work, self.work.data_ptr(), self.n_long,
                            self.long_rows.data_ptr(), self.n_slots)
        self._slabs = {}
        self._parent = parent
        return self

    @classmethod
    def from_scipy(cls, m, device, chunk: int = 32):
        m = m.tocsr()
        m.sort_indices()
        return cls(m.indptr.astype(np.int64), m.indices.astype(np.int32), m.data.astype(np.float32), m.shape[1],
                   device, chunk)

    def slab(self, d: int, k: int = 0):
        """The partial-sum slab for width d (k > 0: another one, for a second product
        over this graph in the same launch)."""
        if self.n_slots == 0:
            return None
        key = d if k == 0 else (d, k)
        s = self._slabs.get(key)
        if s is None:
            # partial-sum slots, then one int32 arrival counter per long row (zero; the
            # kernel re-arms them), see rsx_spmm in include/rsx.h
            s = torch.zeros(self.n_slots * d + self.n_long, dtype=torch.float32, device=self.device)
            self._slabs[key] = s
        return s

    def spmm_epi(self, x: torch.Tensor, epi: "L.Epilogue", d: int):
        _gpu(x)
        _check_x(self, x, d)
        rc = L.lib().rsx_spmm(C.byref(self.struct), _p(x), d, C.byref(epi), _p(self.slab(d)), _stream())
        L.check(rc, "rsx_spmm")

    def spmm(self, x: torch.Tensor, alpha: float = 1.0, out: torch.Tensor | None = None) -> torch.Tensor:
        """y = alpha * A @ x (torch.sparse.mm(A, x), reference lightgcn.py:122)."""
        if x.shape[0] != self.n_cols:
            raise RuntimeError(f"spmm: x has {x.shape[0]} rows, A has {self.n_cols} columns")
        d = x.shape[1]
        y = out if out is not None else torch.empty(self.n_rows, d, dtype=torch.float32, device=x.device)
        self.spmm_epi(x, epi(L.RSX_EPI_STORE, alpha=alpha, y=y), d)
        return y


def _check_x(A, x, d: int):
    """The kernel gathers rows 0..n_cols-1 of x with d contiguous floats each: check that
    before the launch (an out-of-range gather would fault the GPU)."""
    if x.dim() != 2 or x.shape[1] != d or x.shape[0] < A.n_cols or not x.is_contiguous() \
            or x.dtype != torch.float32:
        raise RuntimeError(f"spmm: x {tuple(x.shape)} {x.dtype} does not cover the {A.n_cols} x {d} operand")


def spmm_batch(csrs, xs, epis, d: int):
    """Y_p = A_p X_p with epilogue epis[p] for up to 4 products in one launch (rsx_spmm_batch)."""
    n = len(csrs)
    for a, x in zip(csrs, xs):
        _gpu(x)
        _check_x(a, x, d)
    arr_a = (C.c_void_p * n)(*[C.addressof(a.struct) for a in csrs])
    arr_x = (C.c_void_p * n)(*[x.data_ptr() for x in xs])
    arr_e = (L.Epilogue * n)(*epis)
    seen = {}
    slabs = []
    for a in csrs:  # a graph used twice in one launch: a slab per product
        k = seen.get(id(a), 0)
        seen[id(a)] = k + 1
        slabs.append(_pi(a.slab(d, k)))
    arr_s = (C.c_void_p * n)(*slabs)
    L.check(L.lib().rsx_spmm_batch(n, arr_a, arr_x, d, arr_e, arr_s, _stream()), "rsx_spmm_batch")


def epi(kind: int, alpha: float = 1.0, beta: float = 1.0, adam: "L.Adam | None" = None, **ptrs) -> "L.Epilogue":
    e = L.Epilogue()
    e.kind = kind
    e.alpha = alpha
    e.beta = beta
    for k, t in ptrs.items():
        setattr(e, k, _pi(t))
    if adam is not None:
        e.adam = adam
    return e


def adam_struct(lr: float, step: int, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step_dev=None):
    a = L.Adam()
    a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = lr, beta1, beta2, eps, weight_decay
    a.step_dev = _pi(step_dev)
    a.step = int(step)
    return a


def rowwise(n_rows: int, d: int, e: "L.Epilogue"):
    L.check(L.lib().rsx_rowwise(n_rows, d, C.byref(e), _stream()), "rsx_rowwise")


def adam_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
          betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, step_dev=None):
    """In-place Adam on one parameter tensor (torch.optim.Adam, reference trainer.py:133,238).
    `step_dev`: a 0-d int64 device tensor holding the (already incremented) step,
    read by the kernel instead of `step`."""
    _gpu(p, g, m, v)
    if step_dev is not None and (step_dev.dtype != torch.int64 or not step_dev.is_cuda):
        raise ValueError("step_dev must be an int64 tensor on the GPU")
    d = p.shape[-1] if p.dim() > 1 else p.numel()
    n = p.numel() // d
    if d not in (32, 64, 128, 256):
        # flatten into 64-wide rows plus a tail handled as another view
        flat = [t.view(-1) for t in (p, g, m, v)]
        tot = flat[0].numel()
        main = (tot // 64) * 64
        if main:
            adam_(*(f[:main].view(-1, 64) for f in flat), step=step, lr=lr, betas=betas, eps=eps,
                  weight_decay=weight_decay, step_dev=step_dev)
        if tot - main:
            tail = [torch.zeros(32, dtype=torch.float32, device=p.device) for _ in range(4)]
            for tt, f in zip(tail, flat):
                tt[: tot - main].copy_(f[main:])
            adam_(*(t.view(1, 32) for t in tail), step=step, lr=lr, betas=betas, eps=eps,
                  weight_decay=weight_decay, step_dev=step_dev)
            for tt, f, upd in zip(tail, flat, (True, False, True, True)):
                if upd:
                    f[main:].copy_(tt[: tot - main])
        return
    e = epi(L.RSX_EPI_ADAM, s_in=g, p=p, m=m, v=v,
            adam=adam_struct(lr, step, betas[0], betas[1], eps, weight_decay, step_dev=step_dev))
    rowwise(n, d, e)


# ---------------------------------------------------------------------------
# BPR
# ---------------------------------------------------------------------------
_WS = {}


def _ws(device, nbytes: int) -> torch.Tensor:
    key = (str(device),)
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _WS[key] = t
    return t


def bpr(variant: int, final: torch.Tensor, ego: torch.Tensor | None, n_users: int, n_items: int,
        triplets: torch.Tensor, reg: float, batch_cfg: float | None = None,
        g_final: torch.Tensor | None = None, g_ego: torch.Tensor | None = None,
        loss_acc: torch.Tensor | None = None, compact_rows: bool = False):
    """Fused BPR loss forward+backward; returns (loss[1], g_final, g_ego).

    LightGCN: reference lightgcn.py:132-156; LayerGCN: layergcn.py:142-177; SMORE: smore.py:366-378.
    RSX_BPR_SMORE_ROWS is internal to rsx.smore_fuse's compact-rows loss (compact_rows=True,
    triplets (b, b, B + b) it builds itself); the kernel also NaN-poisons any other layout.
    """
    if (variant == L.RSX_BPR_SMORE_ROWS) != compact_rows:
        raise RuntimeError("bpr: RSX_BPR_SMORE_ROWS is the compact-rows loss's internal variant "
                           "(rsx.smore_fuse.smore_loss_rows)")
    _gpu(final, ego, triplets)
    if triplets.dtype != torch.int64 or triplets.dim() != 2 or triplets.shape[0] < 3:
        raise RuntimeError("bpr: triplets must be int64 [3, B]")
    trip = triplets[:3].contiguous()
    B = trip.shape[1]
    d = final.shape[1]
    lib = L.lib()
    if g_final is None:  # (RSX_BPR_SMORE_ROWS writes every row: no fill)
        g_final = torch.empty_like(final) if variant == L.RSX_BPR_SMORE_ROWS else torch.zeros_like(final)
    if g_ego is None and ego is not None and variant not in (L.RSX_BPR_SMORE, L.RSX_BPR_SMORE_ROWS):
        g_ego = torch.zeros_like(ego)
    loss = torch.empty(1, dtype=torch.float32, device=final.device)
    nb = lib.rsx_bpr_ws_bytes(B)
    ws = _ws(final.device, nb)
    rc = lib.rsx_bpr(variant, _p(final), _p(ego), n_users, n_items, d, _p(trip), B, reg,
                     float(batch_cfg if batch_cfg is not None else B), _p(g_final), _p(g_ego), _p(loss),
                     _p(loss_acc), _p(ws), ws.numel(), _stream())
    L.check(rc, "rsx_bpr")
    return loss, g_final, g_ego


# ---------------------------------------------------------------------------
# full sort
# ---------------------------------------------------------------------------
def fullsort_topk(user_emb: torch.Tensor, users: torch.Tensor | None, item_emb: torch.Tensor,
                  mask_rowptr: torch.Tensor | None, mask_col: torch.Tensor | None, k: int):
    """Fused scores + train-item mask (-1e10) + top-k, order (score desc, index asc).

    Replaces reference trainer.py:521-526 (full_sort_predict, mask, torch.topk).
    """
    _gpu(user_emb, users, item_emb, mask_rowptr, mask_col)
    nb = users.numel() if users is not None else user_emb.shape[0]
    ni, d = item_emb.shape
    lib = L.lib()
    val = torch.empty(nb, k, dtype=torch.float32, device=item_emb.device)
    idx = torch.empty(nb, k, dtype=torch.int64, device=item_emb.device)
    if nb == 0:
        return val, idx
    wsb = lib.rsx_fullsort_ws_bytes(nb, ni, k)
    ws = _ws(item_emb.device, wsb)
    rc = lib.rsx_fullsort_topk(_p(user_emb), _p(users), nb, _p(item_emb), ni, d, _p(mask_rowptr), _p(mask_col), k,
                               _p(val), _p(idx), _p(ws), ws.numel(), _stream())
    L.check(rc, "rsx_fullsort_topk")
    return val, idx


_CUTS = {}


def topk_metrics(topk_idx: torch.Tensor, eval_rowptr: torch.Tensor, eval_col: torch.Tensor, cutoffs,
                 gain: torch.Tensor, exact: bool = True) -> torch.Tensor:
    """Per-cutoff sums over users of recall, precision, ndcg, map and hit count
    (rsx_topk_metrics; reference topk_evaluator.py:58-102 + metrics.py:12-118).
    Returns a float64 device tensor [5, len(cutoffs)].  exact: summed in user
    order (numpy's mean(axis=0) order, bit for bit); else in a fixed parallel order
    (rsx_topk_metrics_fast, within evaluator.sum_order_bound of it)."""
    _gpu(topk_idx, eval_rowptr, eval_col, gain)
    if topk_idx.dtype != torch.int64 or topk_idx.dim() != 2:
        raise RuntimeError("topk_metrics: topk_idx must be int64 [n_users, k]")
    topk_idx = topk_idx.contiguous()
    n, k = topk_idx.shape
    dev = topk_idx.device
    key = (tuple(int(c) for c in cutoffs), str(dev))
    cut = _CUTS.get(key)
    if cut is None:  # a host->device copy once, not per evaluation (a pageable copy waits for the stream)
        cut = _CUTS[key] = torch.tensor(list(key[0]), dtype=torch.int32, device=dev)
    out = torch.empty(5, cut.numel(), dtype=torch.float64, device=dev)
    lib = L.lib()
    ws = _ws(dev, lib.rsx_topk_metrics_ws_bytes(n, cut.numel()))
    fn = lib.rsx_topk_metrics if exact else lib.rsx_topk_metrics_fast
    L.check(fn(_p(topk_idx), n, k, _p(eval_rowptr), _p(eval_col), _p(cut), cut.numel(), _p(gain),
               _p(out), _p(ws), ws.numel(), _stream()), "rsx_topk_metrics")
    return out


def linear_bwd_supported(out_dim: int, in_dim: int) -> bool:
    return out_dim in (32, 64, 128) and in_dim % 4 == 0


def linear_bwd(g: torch.Tensor, x: torch.Tensor, W: torch.Tensor, bias: bool = True):
    """(dW = g^T x, dx = g W, db = colsum g | None) of a Linear over many rows in one
    pass (rsx_linear_bwd; deterministic)."""
    g, x, W = g.contiguous(), x.contiguous(), W.contiguous()
    n, o = g.shape
    i = x.shape[1]
    lib = L.lib()
    dw = torch.empty(o, i, dtype=torch.float32, device=g.device)
    dx = torch.empty(n, i, dtype=torch.float32, device=g.device)
    db = torch.empty(o, dtype=torch.float32, device=g.device) if bias else None
    ws = _ws(g.device, lib.rsx_linear_bwd_ws_bytes(n, o, i))
    L.check(lib.rsx_linear_bwd(_p(g), _p(x), _p(W), n, o, i, _p(dw), _p(dx), _p(db), _p(ws), ws.numel(), _stream()),
            "rsx_linear_bwd")
    return dw, dx, db


def linear_bwd_pair(p0, p1):
    """linear_bwd of two Linears over the same rows and output width, p = (g, x, W, bias),
    in one launch pair (rsx_linear_bwd_pair); None when the two need different kernel
    tilings (call linear_bwd twice then)."""
    (g0, x0, W0, b0), (g1, x1, W1, b1) = p0, p1
    g0, x0, W0, g1, x1, W1 = (t.contiguous() for t in (g0, x0, W0, g1, x1, W1))
    n, o = g0.shape
    i0, i1 = x0.shape[1], x1.shape[1]
    if g1.shape != (n, o) or x1.shape[0] != n:
        return None
    lib = L.lib()
    dev = g0.device
    out = []
    for i, b in ((i0, b0), (i1, b1)):
        out.append((torch.empty(o, i, dtype=torch.float32, device=dev), torch.empty(n, i, dtype=torch.float32, device=dev),
                    torch.empty(o, dtype=torch.float32, device=dev) if b else None))
    ws = _ws(dev, lib.rsx_linear_bwd_pair_ws_bytes(n, o, i0, i1))
    (dw0, dx0, db0), (dw1, dx1, db1) = out
    rc = lib.rsx_linear_bwd_pair(_p(g0), _p(x0), _p(W0), i0, _p(dw0), _p(dx0), _p(db0), _p(g1), _p(x1), _p(W1), i1,
                                 _p(dw1), _p(dx1), _p(db1), n, o, _p(ws), ws.numel(), _stream())
    if rc == L.RSX_ERR_UNSUPPORTED:
        return None
    L.check(rc, "rsx_linear_bwd_pair")
    return out


def linear_wgrad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW = g^T x for nn.Linear over many rows (rsx_linear_wgrad): split-K over row
    blocks with an ordered partial sum, where a library GEMM would see a 64x64
    output and a 26k-long reduction."""
    _gpu(g, x)
    g, x = g.contiguous(), x.contiguous()
    n, o = g.shape
    i = x.shape[1]
    dw = torch.empty(o, i, dtype=torch.float32, device=g.device)
    lib = L.lib()
    ws = _ws(g.device, lib.rsx_linear_wgrad_ws_bytes(n, o, i))
    L.check(lib.rsx_linear_wgrad(_p(g), _p(x), n, o, i, _p(dw), _p(ws), ws.numel(), _stream()), "rsx_linear_wgrad")
    return dw


def score_dense(user_emb: torch.Tensor, users: torch.Tensor | None, item_emb: torch.Tensor) -> torch.Tensor:
    """scores = user_emb[users] @ item_emb.T (reference lightgcn.py:164)."""
    _gpu(user_emb, users, item_emb)
    nb = users.numel() if users is not None else user_emb.shape[0]
    ni, d = item_emb.shape
    out = torch.empty(nb, ni, dtype=torch.float32, device=item_emb.device)
    L.check(L.lib().rsx_score_dense(_p(user_emb), _p(users), nb, _p(item_emb), ni, d, _p(out), _stream()),
            "rsx_score_dense")
    return out


def gather_rows(src: torch.Tensor, idx: torch.Tensor, offset: int = 0) -> torch.Tensor:
    _gpu(src, idx)
    d = src.shape[1]
    out = torch.empty(idx.numel(), d, dtype=torch.float32, device=src.device)
    L.check(L.lib().rsx_gather_rows(_p(src), _p(idx), idx.numel(), offset, d, _p(out), _stream()),
            "rsx_gather_rows")
    return out


# ---------------------------------------------------------------------------
# sampler
# ---------------------------------------------------------------------------
class DeviceSampler:
    """Per-epoch shuffle + rejection negative sampling on the device (throughput mode).

    Replaces reference TrainDataLoader._get_neg_sample / _sample_neg_ids / _random
    (src/utils/dataloader.py:226-275,307-309) and RecDataset.shuffle (dataset.py:98-101).
    """

    def __init__(self, train_u: np.ndarray, train_i: np.ndarray, n_users: int, device, seed: int = 0):
        order = np.lexsort((train_i, train_u))
        u_sorted = train_u[order]
        i_sorted = train_i[order]
        rowptr = np.zeros(n_users + 1, dtype=np.int64)
        rowptr[1:] = np.cumsum(np.bincount(u_sorted, minlength=n_users)[:n_users])
        self.device = torch.device(device)
        self.n_inter = int(train_u.size)
        self.inter_u = torch.from_numpy(train_u.astype(np.int32)).to(self.device)
        self.inter_i = torch.from_numpy(train_i.astype(np.int32)).to(self.device)
        self.hist_rowptr = torch.from_numpy(rowptr).to(self.device)
        self.hist_col = torch.from_numpy(i_sorted.astype(np.int32)).to(self.device)
        self.all_items = torch.from_numpy(np.unique(train_i).astype(np.int32)).to(self.device)
        self.seed = int(seed) & ((1 << 64) - 1)

    def args(self, epoch: int, start: int) -> "L.SamplerArgs":
        return L.SamplerArgs(self.inter_u.data_ptr(), self.inter_i.data_ptr(), self.n_inter,
                             self.hist_rowptr.data_ptr(), self.hist_col.data_ptr(), self.all_items.data_ptr(),
                             self.all_items.numel(), self.seed, epoch, start)

    def sample_epoch(self, epoch: int, batch: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """All triplets of one epoch, batch-major (batch j = out[3*batch*j : ...] as [3, Bj])."""
        if out is None:
            out = torch.empty(3 * self.n_inter, dtype=torch.int64, device=self.device)
        L.check(L.lib().rsx_sample_epoch(self.inter_u.data_ptr(), self.inter_i.data_ptr(), self.n_inter,
                                         self.hist_rowptr.data_ptr(), self.hist_col.data_ptr(),
                                         self.all_items.data_ptr(), self.all_items.numel(), self.seed, epoch,
                                         batch, _pi(out), _stream()), "rsx_sample_epoch")
        return out

    @staticmethod
    def batch_view(epoch_buf: torch.Tensor, n_inter: int, batch: int, j: int) -> torch.Tensor:
        b = min(batch, n_inter - j * batch)
        return epoch_buf[3 * batch * j: 3 * batch * j + 3 * b].view(3, b)

    def sample_epoch_slices(self, epoch: int, n_slices: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """The epoch cut into n_slices balanced slices (rsx_sample_epoch_slices): slice j =
        positions [j E // S, (j+1) E // S), read with `slice_view`."""
        if not 1 <= n_slices <= self.n_inter:
            raise ValueError(f"{n_slices} slices of an epoch of {self.n_inter} interactions")
        if out is None:
            out = torch.empty(3 * self.n_inter, dtype=torch.int64, device=self.device)
        L.check(L.lib().rsx_sample_epoch_slices(self.inter_u.data_ptr(), self.inter_i.data_ptr(), self.n_inter,
                                                self.hist_rowptr.data_ptr(), self.hist_col.data_ptr(),
                                                self.all_items.data_ptr(), self.all_items.numel(), self.seed, epoch,
                                                n_slices, _pi(out), _stream()), "rsx_sample_epoch_slices")
        return out

    @staticmethod
    def slice_bounds(n_inter: int, n_slices: int, j: int):
        return j * n_inter // n_slices, (j + 1) * n_inter // n_slices

    @staticmethod
    def slice_view(epoch_buf: torch.Tensor, n_inter: int, n_slices: int, j: int) -> torch.Tensor:
        a, e = DeviceSampler.slice_bounds(n_inter, n_slices, j)
        return epoch_buf[3 * a: 3 * e].view(3, e - a)

    def sample(self, epoch: int, start: int, batch: int, out: torch.Tensor | None = None) -> torch.Tensor:
        count = min(batch, self.n_inter - start)
        if out is None:
            out = torch.empty(3, count, dtype=torch.int64, device=self.device)
        L.check(L.lib().rsx_sample_triplets(self.inter_u.data_ptr(), self.inter_i.data_ptr(), self.n_inter,
                                            self.hist_rowptr.data_ptr(), self.hist_col.data_ptr(),
                                            self.all_items.data_ptr(), self.all_items.numel(), self.seed,
                                            epoch, start, batch, _pi(out), _stream()), "rsx_sample_triplets")
        return out


# ---------------------------------------------------------------------------
# graph builders on the device (csrc/graph.hip)
# ---------------------------------------------------------------------------
ADJ_LIGHTGCN, ADJ_SMORE = 0, 1


def dinv_table(max_deg: int, mode: int) -> np.ndarray:
    """The per-node factor of every degree 0..max_deg with the reference's own host
    arithmetic: mode ADJ_LIGHTGCN (deg + 1e-7)^-1/2 in float64 numpy
    (lightgcn.py:93-96), ADJ_SMORE numpy's float32 power with inf -> 0
    (smore.py:194-198), widened to float64 for the kernel."""
    deg = np.arange(max_deg + 1)
    if mode == ADJ_LIGHTGCN:
        return np.power(deg.astype(np.float64) + 1e-7, -0.5)
    with np.errstate(divide="ignore"):
        d = np.power(deg.astype(np.float32), np.float32(-0.5)).astype(np.float32)
    d[np.isinf(d)] = 0.0
    return d.astype(np.float64)


def adj_build(u, i, n_users: int, n_items: int, mode: int, device):
    """(rowptr int64 [n+1], col int32 [nnz], val f32 [nnz]) device tensors of the
    normalised symmetric adjacency (rsx_adj_build): mode ADJ_LIGHTGCN = reference
    lightgcn.py:65-103, ADJ_SMORE = smore.py:176-207; equal to rsx.graph's host
    builders bit for bit (the per-degree factors are the host pow's, a table up to a
    degree bound: the largest raw interaction count of any user or item).  u, i: host
    arrays or device int64 tensors."""
    dev = torch.device(device)
    u = torch.as_tensor(u, dtype=torch.int64).to(dev).contiguous()
    i = torch.as_tensor(i, dtype=torch.int64).to(dev).contiguous()
    E = u.numel()
    n = n_users + n_items
    lib = L.lib()
    bound = 0
    if E:
        bound = int(torch.stack([torch.bincount(u).max(), torch.bincount(i).max()]).max().item())
    table = torch.from_numpy(dinv_table(bound, mode)).to(dev)
    rowptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
    col = torch.empty(max(2 * E, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(2 * E, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(int(lib.rsx_adj_build_ws_bytes(E, n_users, n_items)), dtype=torch.uint8, device=dev)
    L.check(lib.rsx_adj_build(_p(u), _p(i), E, n_users, n_items, mode, _p(table), table.numel(), _p(rowptr),
                              _p(col), _p(val), _p(ws), ws.numel(), _stream()), "rsx_adj_build")
    nnz = int(rowptr[-1].item())
    return rowptr, col[:nnz], val[:nnz]


def edge_dropout_build(e_u, e_i, keep, n_users: int, n_items: int, t_rowptr, t_col, t_eid):
    """(rowptr, col, val) of LayerGCN's masked graph (rsx_edge_dropout_build)."""
    _gpu(e_u, e_i, keep, t_rowptr, t_col, t_eid)
    E = e_u.numel()
    n = n_users + n_items
    dev = e_u.device
    lib = L.lib()
    keep8 = keep.to(torch.uint8).contiguous()
    rowptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
    col = torch.empty(max(2 * E, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(2 * E, 1), dtype=torch.float32, device=dev)
    ws = _ws(dev, int(lib.rsx_edge_dropout_ws_bytes(E, n_users, n_items)))
    L.check(lib.rsx_edge_dropout_build(_p(e_u), _p(e_i), _p(keep8), E, n_users, n_items, _p(t_rowptr), _p(t_col),
                                       _p(t_eid), _p(rowptr), _p(col), _p(val), _p(ws), ws.numel(), _stream()),
            "rsx_edge_dropout_build")
    return rowptr, col, val
