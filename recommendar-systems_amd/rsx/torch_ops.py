"""`torch.ops.rsx.*`: the hot path as PyTorch custom operators with autograd
(SURVEY.md 8(b)2), so that unmodified reference code can call the HIP kernels
through the dispatcher instead of importing the rsx model classes:

    torch.ops.rsx.spmm_csr(rowptr, col, val, x, n_cols)          torch.sparse.mm(A, x)
    torch.ops.rsx.propagate_mean(rowptr, col, val, x, n_layers)   LightGCN.forward's layer mean
    torch.ops.rsx.propagate_layergcn(rowptr, col, val, x, n_layers)  LayerGCN.forward
    torch.ops.rsx.bpr_loss(final, ego, triplets, n_users, reg, variant, batch_cfg)
    torch.ops.rsx.fullsort_topk(user_emb, users, item_emb, mask_rowptr, mask_col, k)
    torch.ops.rsx.adam_(p, g, m, v, step, lr, beta1, beta2, eps, weight_decay)
    torch.ops.rsx.smore_spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf, normalize)

(reference call sites: src/models/lightgcn.py:117-166, src/models/layergcn.py:127-188,
src/models/smore.py:209-272, src/common/loss.py:33-61, src/common/trainer.py:238,509-528).

Graphs are plain CSR tensors (rowptr int64 [N+1], col int32 [nnz], val f32 [nnz]);
on the GPU the nnz-balanced work schedule (and, for spmm_csr's backward, the
transposed CSR) is built once per graph and cached, keyed by the tensors (held,
so their storage cannot be reused while cached).  The adjacency is a constant of
the reference models (no gradient to `val`).  Each op has two kernels, chosen by the
dispatcher from the tensors' device: CUDA (ROCm) tensors run the HIP kernels, CPU
tensors the C++ CPU kernels of the same library (csrc/cpu_ops.cpp, include/rsx.h
"CPU kernels": the reference's CPU configuration, BASELINE C1).  Neither is a fallback
for the other: a GPU tensor never reaches a CPU kernel (the HIP library failing to load
raises).  smore_spectral is GPU-only (CPU tensors raise NotImplementedError).
Backward passes that need forward intermediates recompute the forward (a few
SpMMs), so the ops hold no hidden state between forward and backward.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
from torch import Tensor

from . import _lib as L
from . import graph, ops

import os
from collections import OrderedDict

# graph cache, least recently used first.  Bounded two ways, because a caller such as
# the reference's LayerGCN builds a fresh masked_adj every epoch (src/models/layergcn.py:
# 51-70) and would otherwise pin one graph per epoch: at most _PER_SHAPE graphs of one
# (n_rows, n_cols, transpose) shape (a model's train and eval graph), and at most
# _CACHE_BYTES of graph memory (held tensors + work schedule + transposed copies) in all.
_CACHE: "OrderedDict" = OrderedDict()
_CACHE_MAX = 32
_PER_SHAPE = 2
_CACHE_BYTES = int(os.environ.get("RSX_TORCH_OPS_CACHE_BYTES", 4 << 30))


def _key(*ts):
    return tuple((t.data_ptr(), t.numel(), t._version) for t in ts)


def _graph_bytes(A, transpose):
    """Device bytes a cache entry keeps alive: the CSR arrays (held, or transposed
    copies) and the work schedule (16 B per work item, 16 B per split row)."""
    b = 8 * (A.n_rows + 1) + 8 * A.nnz + 16 * (A.n_work + A.n_long)
    return b * (2 if transpose else 1)


def _evict(shape):
    same = [k for k in _CACHE if k[1:] == shape]
    while len(same) >= _PER_SHAPE:
        _CACHE.pop(same.pop(0))
    while _CACHE and (len(_CACHE) >= _CACHE_MAX or sum(v[4] for v in _CACHE.values()) > _CACHE_BYTES):
        _CACHE.popitem(last=False)


def _csr(rowptr: Tensor, col: Tensor, val: Tensor, n_cols: int, transpose: bool = False):
    """The cached DeviceCSR of (rowptr, col, val) (or of its transpose)."""
    shape = (_n_rows(rowptr), int(n_cols), bool(transpose))
    key = (_key(rowptr, col, val),) + shape
    hit = _CACHE.get(key)
    if hit is not None:
        _CACHE.move_to_end(key)
        return hit[0]
    if col.dtype != torch.int32 or val.dtype != torch.float32 or rowptr.dtype != torch.int64:
        raise RuntimeError("rsx CSR: rowptr int64, col int32, val float32")
    if transpose:
        rp = rowptr.cpu().numpy()
        rows = np.repeat(np.arange(rp.size - 1, dtype=np.int64), np.diff(rp))
        trp, tcol, tval = graph.to_csr(col.cpu().numpy().astype(np.int64), rows, val.cpu().numpy(), int(n_cols),
                                       rp.size - 1)
        A = ops.DeviceCSR(trp, tcol, tval, rp.size - 1, val.device)
    else:
        A = ops.DeviceCSR.from_device(rowptr, col.contiguous(), val.contiguous(), int(n_cols))
    _evict(shape)
    # the tensors are held: their storage cannot be reused while the entry lives
    _CACHE[key] = (A, rowptr, col, val, _graph_bytes(A, transpose))
    return A


def _n_rows(rowptr):
    return rowptr.shape[0] - 1


def _cp(t):
    """Host pointer of a contiguous CPU tensor (None for None)."""
    return None if t is None else t.data_ptr()


def _cpu_csr(rowptr, col, val):
    if col.dtype != torch.int32 or val.dtype != torch.float32 or rowptr.dtype != torch.int64:
        raise RuntimeError("rsx CSR: rowptr int64, col int32, val float32")
    return rowptr.contiguous(), col.contiguous(), val.contiguous()


def _cpu_spmm(rowptr, col, val, x):
    rowptr, col, val = _cpu_csr(rowptr, col, val)
    x = x.contiguous()
    if x.dtype != torch.float32 or x.dim() != 2:
        raise RuntimeError("rsx::spmm_csr: x must be float32 [n_cols, d]")
    y = x.new_empty(_n_rows(rowptr), x.shape[1])
    L.check(L.lib().rsx_cpu_spmm(_cp(rowptr), _cp(col), _cp(val), _n_rows(rowptr), _cp(x), x.shape[1], _cp(y)),
            "rsx_cpu_spmm")
    return y


def _cpu_transpose(rowptr, col, val, n_cols):
    """(rowptr, col, val) of A^T on the host (graph.to_csr: rows sorted, columns in order)."""
    rp = rowptr.numpy()
    rows = np.repeat(np.arange(rp.size - 1, dtype=np.int64), np.diff(rp))
    trp, tcol, tval = graph.to_csr(col.numpy().astype(np.int64), rows, val.numpy(), int(n_cols), rp.size - 1)
    return torch.from_numpy(trp), torch.from_numpy(tcol.astype(np.int32)), torch.from_numpy(tval.astype(np.float32))


# ---------------------------------------------------------------------------
# SpMM
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::spmm_csr", mutates_args=(), device_types="cuda")
def spmm_csr(rowptr: Tensor, col: Tensor, val: Tensor, x: Tensor, n_cols: int) -> Tensor:
    """y = A x for A = (rowptr, col, val) [N, n_cols] (torch.sparse.mm(A, x))."""
    return _csr(rowptr, col, val, n_cols).spmm(x.contiguous())


@spmm_csr.register_fake
def _(rowptr, col, val, x, n_cols):
    return x.new_empty(rowptr.shape[0] - 1, x.shape[1])


def _spmm_setup(ctx, inputs, output):
    rowptr, col, val, _, n_cols = inputs
    ctx.save_for_backward(rowptr, col, val)
    ctx.n_cols = n_cols


def _spmm_bwd(ctx, g):
    rowptr, col, val = ctx.saved_tensors
    if not g.is_cuda:  # the CPU kernel on the host transpose
        return None, None, None, _cpu_spmm(*_cpu_transpose(rowptr, col, val, ctx.n_cols), g), None
    AT = _csr(rowptr, col, val, ctx.n_cols, transpose=True)
    return None, None, None, AT.spmm(g.contiguous()), None


spmm_csr.register_autograd(_spmm_bwd, setup_context=_spmm_setup)


@spmm_csr.register_kernel("cpu")
def _(rowptr, col, val, x, n_cols):
    return _cpu_spmm(rowptr, col, val, x)


# ---------------------------------------------------------------------------
# LightGCN propagation: mean_{k=0..K} A^k x (A symmetric)
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::propagate_mean", mutates_args=(), device_types="cuda")
def propagate_mean(rowptr: Tensor, col: Tensor, val: Tensor, x: Tensor, n_layers: int) -> Tensor:
    """LightGCN.forward's layer mean (reference lightgcn.py:117-130) for a symmetric A."""
    from .smore import _prop_mean

    return _prop_mean(_csr(rowptr, col, val, _n_rows(rowptr)), x.contiguous(), int(n_layers))


@propagate_mean.register_fake
def _(rowptr, col, val, x, n_layers):
    return torch.empty_like(x)


def _pm_setup(ctx, inputs, output):
    rowptr, col, val, _, K = inputs
    ctx.save_for_backward(rowptr, col, val)
    ctx.K = K


def _pm_bwd(ctx, g):
    rowptr, col, val = ctx.saved_tensors
    return None, None, None, torch.ops.rsx.propagate_mean(rowptr, col, val, g.contiguous(), ctx.K), None


propagate_mean.register_autograd(_pm_bwd, setup_context=_pm_setup)


@propagate_mean.register_kernel("cpu")
def _(rowptr, col, val, x, n_layers):
    rowptr, col, val = _cpu_csr(rowptr, col, val)
    x = x.contiguous()
    out = torch.empty_like(x)
    L.check(L.lib().rsx_cpu_propagate_mean(_cp(rowptr), _cp(col), _cp(val), _n_rows(rowptr), _cp(x), x.shape[1],
                                           int(n_layers), _cp(out)), "rsx_cpu_propagate_mean")
    return out


# ---------------------------------------------------------------------------
# LayerGCN propagation: E^k = cos(A E^{k-1}, E^0) * A E^{k-1}; out = sum_{k=1..K} E^k
# ---------------------------------------------------------------------------
def _lgcn_forward(A, x, K, save):
    n, d = x.shape
    out = torch.empty_like(x)
    h = [torch.empty_like(x), torch.empty_like(x)]
    zs = [torch.empty_like(x) for _ in range(K)] if save else None
    cs = [torch.empty(n, dtype=torch.float32, device=x.device) for _ in range(K)] if save else None
    cur = x
    for k in range(1, K + 1):
        y = h[(k - 1) & 1]
        kw = dict(e0=x, y=y, s_out=out, s_in=(out if k > 1 else None))
        if save:
            kw.update(aux=zs[k - 1], aux_w=cs[k - 1])
        A.spmm_epi(cur, ops.epi(L.RSX_EPI_LAYERGCN, **kw), d)
        cur = y
    return out, zs, cs


@torch.library.custom_op("rsx::propagate_layergcn", mutates_args=(), device_types="cuda")
def propagate_layergcn(rowptr: Tensor, col: Tensor, val: Tensor, x: Tensor, n_layers: int) -> Tensor:
    """LayerGCN.forward (reference layergcn.py:127-140): ego excluded from the sum."""
    if n_layers < 1:
        raise RuntimeError("propagate_layergcn: n_layers >= 1")
    return _lgcn_forward(_csr(rowptr, col, val, _n_rows(rowptr)), x.contiguous(), int(n_layers), False)[0]


@propagate_layergcn.register_fake
def _(rowptr, col, val, x, n_layers):
    return torch.empty_like(x)


def _lg_setup(ctx, inputs, output):
    rowptr, col, val, x, K = inputs
    ctx.save_for_backward(rowptr, col, val, x)
    ctx.K = K


def _lg_bwd_cpu(rowptr, col, val, x, K, G):
    rowptr, col, val = _cpu_csr(rowptr, col, val)
    n, d = x.shape
    zs = x.new_empty(K, n, d)
    cs = x.new_empty(K, n)
    out = torch.empty_like(x)
    lib = L.lib()
    L.check(lib.rsx_cpu_layergcn_forward(_cp(rowptr), _cp(col), _cp(val), n, _cp(x), d, K, _cp(out), _cp(zs),
                                         _cp(cs)), "rsx_cpu_layergcn_forward")
    dx = torch.empty_like(x)
    L.check(lib.rsx_cpu_layergcn_backward(_cp(rowptr), _cp(col), _cp(val), n, _cp(x), d, K, _cp(G), _cp(zs), _cp(cs),
                                          _cp(dx)), "rsx_cpu_layergcn_backward")
    return dx


def _lg_bwd(ctx, G):
    rowptr, col, val, x = ctx.saved_tensors
    K = ctx.K
    x = x.contiguous()
    if not x.is_cuda:
        return None, None, None, _lg_bwd_cpu(rowptr, col, val, x, K, G.contiguous()), None
    A = _csr(rowptr, col, val, _n_rows(rowptr))
    _, zs, cs = _lgcn_forward(A, x, K, True)  # recompute the pre-scale rows and cosine weights
    n, d = x.shape
    G = G.contiguous()
    acc = torch.empty_like(x)
    hz = torch.empty_like(x)
    # layer K: dE^K = G -> dZ^K, the ego-cosine terms into acc (the engine's backward, rsx/layergcn.py)
    ops.rowwise(n, d, ops.epi(L.RSX_EPI_LAYERGCN_BWD, r_add=G, aux=zs[K - 1], aux_w=cs[K - 1], e0=x, y=hz,
                              s_out=acc))
    for k in range(K - 1, 0, -1):
        y = torch.empty_like(x)
        A.spmm_epi(hz, ops.epi(L.RSX_EPI_LAYERGCN_BWD, r_add=G, aux=zs[k - 1], aux_w=cs[k - 1], e0=x, y=y,
                               s_in=acc, s_out=acc), d)
        hz = y
    dx = torch.empty_like(x)
    A.spmm_epi(hz, ops.epi(L.RSX_EPI_ADD, y=dx, s_in=acc), d)  # dE^0 = A dZ^1 + cosine terms
    return None, None, None, dx, None


propagate_layergcn.register_autograd(_lg_bwd, setup_context=_lg_setup)


@propagate_layergcn.register_kernel("cpu")
def _(rowptr, col, val, x, n_layers):
    if n_layers < 1:
        raise RuntimeError("propagate_layergcn: n_layers >= 1")
    rowptr, col, val = _cpu_csr(rowptr, col, val)
    x = x.contiguous()
    out = torch.empty_like(x)
    L.check(L.lib().rsx_cpu_layergcn_forward(_cp(rowptr), _cp(col), _cp(val), x.shape[0], _cp(x), x.shape[1],
                                             int(n_layers), _cp(out), None, None), "rsx_cpu_layergcn_forward")
    return out


# ---------------------------------------------------------------------------
# BPR (+ regulariser)
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::bpr_loss", mutates_args=(), device_types="cuda")
def bpr_loss(final: Tensor, ego: Optional[Tensor], triplets: Tensor, n_users: int, reg: float, variant: int,
             batch_cfg: float) -> Tensor:
    """The fused BPR loss (variant 0 LightGCN, 1 LayerGCN, 2 SMORE; include/rsx.h);
    batch_cfg <= 0: the batch size."""
    ni = final.shape[0] - n_users
    loss, _, _ = ops.bpr(int(variant), final.contiguous(), None if ego is None else ego.contiguous(), int(n_users),
                         ni, triplets, float(reg), float(batch_cfg) if batch_cfg > 0 else None)
    return loss[0].clone()


@bpr_loss.register_fake
def _(final, ego, triplets, n_users, reg, variant, batch_cfg):
    return final.new_empty(())


def _bpr_setup(ctx, inputs, output):
    final, ego, triplets, n_users, reg, variant, batch_cfg = inputs
    ctx.save_for_backward(final, ego if ego is not None else final.new_empty(0), triplets)
    ctx.cfg = (n_users, reg, variant, batch_cfg, ego is not None)


def _cpu_bpr(final, ego, triplets, n_users, reg, variant, batch_cfg, grads):
    final = final.contiguous()
    ego = ego.contiguous() if ego is not None else None
    trip = triplets[:3].contiguous()
    if trip.dtype != torch.int64:
        raise RuntimeError("rsx::bpr_loss: triplets must be int64 [3, B]")
    B = trip.shape[1]
    ni = final.shape[0] - n_users
    gf = torch.zeros_like(final) if grads else None
    ge = torch.zeros_like(ego) if (grads and ego is not None and variant != L.RSX_BPR_SMORE) else None
    loss = final.new_empty(1)
    L.check(L.lib().rsx_cpu_bpr(int(variant), _cp(final), _cp(ego), int(n_users), ni, final.shape[1], _cp(trip), B,
                                float(reg), float(batch_cfg) if batch_cfg > 0 else float(B), _cp(gf), _cp(ge),
                                _cp(loss)), "rsx_cpu_bpr")
    return loss, gf, ge


@bpr_loss.register_kernel("cpu")
def _(final, ego, triplets, n_users, reg, variant, batch_cfg):
    return _cpu_bpr(final, ego, triplets, n_users, reg, variant, batch_cfg, False)[0][0].clone()


def _bpr_bwd(ctx, go):
    final, ego, triplets = ctx.saved_tensors
    n_users, reg, variant, batch_cfg, has_ego = ctx.cfg
    if not final.is_cuda:
        _, gf, ge = _cpu_bpr(final, ego if has_ego else None, triplets, n_users, reg, variant, batch_cfg, True)
        return go * gf, (go * ge if ge is not None else None), None, None, None, None, None
    ni = final.shape[0] - n_users
    _, gf, ge = ops.bpr(int(variant), final.contiguous(), ego.contiguous() if has_ego else None, int(n_users), ni,
                        triplets, float(reg), float(batch_cfg) if batch_cfg > 0 else None)
    return go * gf, (go * ge if (has_ego and ge is not None) else None), None, None, None, None, None


bpr_loss.register_autograd(_bpr_bwd, setup_context=_bpr_setup)


# ---------------------------------------------------------------------------
# full-sort top-k (no gradient)
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::fullsort_topk", mutates_args=(), device_types="cuda")
def fullsort_topk(user_emb: Tensor, users: Tensor, item_emb: Tensor, mask_rowptr: Tensor, mask_col: Tensor,
                  k: int) -> tuple[Tensor, Tensor]:
    """(scores, item ids) [B, k]: user_emb[users] . item_emb^T, training items masked to
    -1e10, top-k in (score desc, index asc) order (reference trainer.py:509-528)."""
    return ops.fullsort_topk(user_emb.contiguous(), users.contiguous(), item_emb.contiguous(),
                             mask_rowptr.contiguous(), mask_col.contiguous(), int(k))


@fullsort_topk.register_kernel("cpu")
def _(user_emb, users, item_emb, mask_rowptr, mask_col, k):
    ue, it = user_emb.contiguous(), item_emb.contiguous()
    users = users.contiguous()
    nb = users.numel()
    val = ue.new_empty(nb, int(k))
    idx = torch.empty(nb, int(k), dtype=torch.int64)
    if nb:
        L.check(L.lib().rsx_cpu_fullsort_topk(_cp(ue), _cp(users), nb, _cp(it), it.shape[0], it.shape[1],
                                              _cp(mask_rowptr.contiguous()), _cp(mask_col.contiguous()), int(k),
                                              _cp(val), _cp(idx)), "rsx_cpu_fullsort_topk")
    return val, idx


@fullsort_topk.register_fake
def _(user_emb, users, item_emb, mask_rowptr, mask_col, k):
    nb = users.shape[0]
    return user_emb.new_empty(nb, k), users.new_empty(nb, k, dtype=torch.int64)


# ---------------------------------------------------------------------------
# Adam (in place)
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::adam_", mutates_args=("p", "m", "v"), device_types="cuda")
def adam_(p: Tensor, g: Tensor, m: Tensor, v: Tensor, step: Tensor, lr: float, beta1: float, beta2: float,
          eps: float, weight_decay: float) -> None:
    """torch.optim.Adam's single-tensor update of p, m, v; `step`: the (already
    incremented) int64 step count, a 0-d GPU tensor."""
    from .smore_fuse import adam_multi

    adam_multi([p], [g.contiguous()], [m], [v], [step], lr, betas=(beta1, beta2), eps=eps, weight_decay=weight_decay)


@adam_.register_kernel("cpu")
def _(p, g, m, v, step, lr, beta1, beta2, eps, weight_decay):
    for t in (p, m, v):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError("rsx::adam_: p, m, v must be contiguous float32")
    g = g.contiguous()
    L.check(L.lib().rsx_cpu_adam(_cp(p), _cp(g), _cp(m), _cp(v), p.numel(), int(step), float(lr), float(beta1),
                                 float(beta2), float(eps), float(weight_decay)), "rsx_cpu_adam")


# ---------------------------------------------------------------------------
# SMORE projection + spectral fusion
# ---------------------------------------------------------------------------
@torch.library.custom_op("rsx::smore_spectral", mutates_args=(), device_types="cuda")
def smore_spectral(V: Tensor, Wv: Tensor, bv: Tensor, T: Tensor, Wt: Tensor, bt: Tensor, wv: Tensor, wt: Tensor,
                   wf: Tensor, normalize: bool) -> tuple[Tensor, Tensor, Tensor]:
    """(conv_v, conv_t, conv_f) of SMORE's projection + spectrum_convolution
    (reference smore.py:209-259) through the fused HIP pass."""
    from .smore_spectral import spectral

    with torch.no_grad():
        cv, ct, cf, _, _ = spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf, normalize)
    return cv, ct, cf


@smore_spectral.register_fake
def _(V, Wv, bv, T, Wt, bt, wv, wt, wf, normalize):
    n, d = V.shape[0], Wv.shape[0]
    return V.new_empty(n, d), V.new_empty(n, d), V.new_empty(n, d)


def _sp_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs[:9])
    ctx.normalize = inputs[9]


def _sp_bwd(ctx, gv, gt, gf):
    from .smore_spectral import spectral

    args = [x.detach().requires_grad_(True) for x in ctx.saved_tensors]
    with torch.enable_grad():
        outs = spectral(*args, ctx.normalize)[:3]  # recompute, then the fused backward
        ups = [(o, g) for o, g in zip(outs, (gv, gt, gf)) if g is not None]
        grads = torch.autograd.grad([o for o, _ in ups], args, [g for _, g in ups], allow_unused=True)
    return (*grads, None)


smore_spectral.register_autograd(_sp_bwd, setup_context=_sp_setup)

OPS = ["spmm_csr", "propagate_mean", "propagate_layergcn", "bpr_loss", "fullsort_topk", "adam_", "smore_spectral"]
