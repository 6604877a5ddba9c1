"""SMORE's per-row blocks on the fused HIP kernels (csrc/smore_fuse.hip), with autograd.

Each torch.autograd.Function below replaces a chain of ~10-40 torch kernels of the
reference forward (src/models/smore.py) and its autograd backward by one forward
launch and one backward launch (+ one batched weight-gradient launch pair):

* `gates`       — gate_v/t/f + inject (smore.py:262-272)
* `preference`  — query MLPs, softmax over d, view products, dropout'd preference
                  gates, mean of the three views, content + side (smore.py:320-341)
* `view_prop`   — an item view through n_layers item-item SpMMs, then the item ->
                  user aggregation R, written as one [n_users + n_items, d] table (the
                  reference's torch.cat([R x, x]), smore.py:299-317)
* `infonce2`    — InfoNCE(side[pos], content[pos]) and InfoNCE(side[u], content[u])
                  (smore.py:380-387, 398-404) from the full side/content tables and the
                  batch indices (no gathered copies, no index_put backward)

The weight gradients of every Linear (dW = dZ^T X, db = colsum dZ) come from
rsx_smore_wgrad in one launch pair per block.  Arithmetic is f32 throughout (MFMA
f32 products are exact, sums in f32); results equal the torch ops within float
rounding, which tests/test_gpu_smore_fuse.py checks against torch autograd.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib as L
from . import ops

_p = ops._p


# RSX_PREF_SAVED=0: the batch-row preference backward and the gates' backward recompute the
# forward's activations (the round-5 form; A/B and tests) instead of reading the ones their
# forwards saved
_SAVED = os.environ.get("RSX_PREF_SAVED", "1") != "0"
# RSX_PREF_PLAN=0: the backward's per-row sums scan the row ids (pref_segsum_lds) instead of
# reading the occurrence plan the forward built (pref_segsum_plan; same sums, same order)
_PLAN = os.environ.get("RSX_PREF_PLAN", "1") != "0"
_LEAD = {}


def _lead_scratch(n_rows: int, device) -> torch.Tensor:
    """The occurrence plan's u64 [1 + table rows] key scratch (zeroed once, then tagged per
    call by the kernels; one per device and table size, used in stream order)."""
    key = (torch.device(device).index, int(n_rows))
    t = _LEAD.get(key)
    if t is None:
        t = _LEAD[key] = torch.zeros(1 + int(n_rows), dtype=torch.int64, device=device)
    return t


def _arr(ts):
    return (C.c_void_p * len(ts))(*[(t.data_ptr() if t is not None else None) for t in ts])


def supported(d: int) -> bool:
    return d in (64, 128)


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _wgrad(pairs, d, device):
    """[(dz, x, has_bias)] -> [(dW, db | None)] through rsx_smore_wgrad (<= 8 pairs)."""
    lib = L.lib()
    n = pairs[0][0].shape[0]
    dws = [torch.empty(d, d, dtype=torch.float32, device=device) for _ in pairs]
    dbs = [torch.empty(d, dtype=torch.float32, device=device) if hb else None for _, _, hb in pairs]
    ws = torch.empty(max(int(lib.rsx_smore_wgrad_ws_bytes(n, d, len(pairs))), 4), dtype=torch.uint8,
                     device=device)
    L.check(lib.rsx_smore_wgrad(len(pairs), _arr([p[0] for p in pairs]), _arr([p[1] for p in pairs]), _arr(dws),
                                _arr(dbs), n, d, _p(ws), ws.numel(), ops._stream()), "rsx_smore_wgrad")
    return list(zip(dws, dbs))


# ---------------------------------------------------------------------------
# modality gates
# ---------------------------------------------------------------------------
class _Gates(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cv, ct, cf, item, Wv, bv, Wt, bt, Wf, bf, scale, mul):
        conv = [_c(x) for x in (cv, ct, cf)]
        W = [_c(x) for x in (Wv, Wt, Wf)]
        b = [_c(x) for x in (bv, bt, bf)]
        item = _c(item)
        n, d = item.shape
        outs = [torch.empty_like(item) for _ in range(3)]
        # residual mode: the sigmoid rows for the backward (one product a row there, not two)
        saved = (torch.empty(3, n, d, dtype=torch.float32, device=item.device)
                 if _SAVED and not mul and any(ctx.needs_input_grad) else None)
        L.check(L.lib().rsx_smore_gates_saved(0, _arr(conv), _p(item), _arr(W), _arr(b), n, d, float(scale),
                                              int(mul), _arr(outs), None, None, None, None, _p(saved),
                                              ops._stream()), "rsx_smore_gates_saved")
        ctx.save_for_backward(*conv, item, *W, *b, saved if saved is not None else torch.empty(0))
        ctx.has_saved = saved is not None
        ctx.cfg = (float(scale), int(mul))
        return tuple(outs)

    @staticmethod
    def backward(ctx, gv, gt, gf):
        cv, ct, cf, item, Wv, Wt, Wf, bv, bt, bf, saved = ctx.saved_tensors
        gc, gi, wg = _gates_backward((cv, ct, cf), item, (Wv, Wt, Wf), (bv, bt, bf), ctx.cfg, (gv, gt, gf),
                                     saved if ctx.has_saved else None)
        return (*gc, gi, *wg, None, None)


def _gates_backward(conv, item, W, b, cfg, gouts, saved=None):
    """(d conv[3], d item, (d Wv, d bv, d Wt, d bt, d Wf, d bf)) of the gates: one launch
    for the row gradients, one rsx_smore_wgrad pair for the weights.  `saved`: the
    forward's [3, n, d] sigmoid rows (rsx_smore_gates_saved), or None (recomputed)."""
    scale, mul = cfg
    n, d = item.shape
    gi = torch.empty_like(item)
    gc = [torch.empty_like(item) for _ in range(3)]
    dz = [torch.empty_like(item) for _ in range(3)]
    gouts = [None if g is None else _c(g) for g in gouts]
    L.check(L.lib().rsx_smore_gates_saved(1, _arr(list(conv)), _p(item), _arr(list(W)), _arr(list(b)), n, d, scale,
                                          mul, None, _arr(gouts), _p(gi), _arr(gc), _arr(dz), _p(saved),
                                          ops._stream()), "rsx_smore_gates_saved")
    (gWv, gbv), (gWt, gbt), (gWf, gbf) = _wgrad([(dz[0], conv[0], True), (dz[1], conv[1], True),
                                                 (dz[2], conv[2], True)], d, item.device)
    return gc, gi, (gWv, gbv, gWt, gbt, gWf, gbf)


def gates(cv, ct, cf, item, gate_v, gate_t, gate_f, scale: float, mul: bool):
    """(img_i, txt_i, fus_i) = item + scale * sigmoid(gate_x(conv_x)) (or item * sigmoid(..));
    gate_x are the reference's nn.Sequential(Linear, Sigmoid) modules."""
    lv, lt, lf = gate_v[0], gate_t[0], gate_f[0]
    return _Gates.apply(cv, ct, cf, item, lv.weight, lv.bias, lt.weight, lt.bias, lf.weight, lf.bias, scale, mul)


# ---------------------------------------------------------------------------
# preference block
# ---------------------------------------------------------------------------
class _Pref(torch.autograd.Function):
    @staticmethod
    def forward(ctx, C_, IE, TE, FE, p_drop, seed, *wb):
        W = [_c(x) for x in wb[:7]]
        b = [None if x is None else _c(x) for x in wb[7:]]
        C_, IE, TE, FE = _c(C_), _c(IE), _c(TE), _c(FE)
        n, d = C_.shape
        all_ = torch.empty_like(C_)
        side = torch.empty_like(C_)
        L.check(L.lib().rsx_smore_pref(0, _arr(W), _arr(b), _p(C_), _p(IE), _p(TE), _p(FE), n, d, float(p_drop),
                                       _p(seed), _p(all_), _p(side), None, None, None, None, None, None, None,
                                       None, None, ops._stream()), "rsx_smore_pref")
        ctx.save_for_backward(C_, IE, TE, FE, seed, *W, *[x if x is not None else torch.empty(0) for x in b])
        ctx.has_b = [x is not None for x in b]
        ctx.p_drop = float(p_drop)
        return all_, side

    @staticmethod
    def backward(ctx, g_all, g_side):
        sv = ctx.saved_tensors
        C_, IE, TE, FE, seed = sv[:5]
        W = list(sv[5:12])
        b = [x if h else None for x, h in zip(sv[12:19], ctx.has_b)]
        n, d = C_.shape
        if g_all is None:
            g_all = torch.zeros_like(C_)
        g_all = _c(g_all)
        g_side = None if g_side is None else _c(g_side)
        gC, gIE, gTE, gFE = (torch.empty_like(C_) for _ in range(4))
        hv, ht = torch.empty_like(C_), torch.empty_like(C_)
        dz = [torch.empty_like(C_) for _ in range(7)]
        L.check(L.lib().rsx_smore_pref(1, _arr(W), _arr(b), _p(C_), _p(IE), _p(TE), _p(FE), n, d, ctx.p_drop,
                                       _p(seed), None, None, _p(g_all), _p(g_side), _p(gC), _p(gIE), _p(gTE),
                                       _p(gFE), _p(hv), _p(ht), _arr(dz), ops._stream()), "rsx_smore_pref")
        # Linear inputs: query_v.0 <- F, query_v.2 <- hv, query_t.0 <- F, query_t.2 <- ht, prefer gates <- content
        xs = [FE, hv, FE, ht, C_, C_, C_]
        grads = _wgrad([(dz[i], xs[i], ctx.has_b[i]) for i in range(7)], d, C_.device)
        gW = [g[0] for g in grads]
        gb = [g[1] for g in grads]
        return (gC, gIE, gTE, gFE, None, None, *gW, *gb)


def preference(model, content, image_embeds, text_embeds, fusion_embeds, seed):
    """(all_embeds, side) of the reference's preference block; `seed`: a 1-element
    int64 device tensor (this call's dropout seed; unused when dropout is off)."""
    m = model
    lin = [m.query_v[0], m.query_v[2], m.query_t[0], m.query_t[2], m.gate_image_prefer[0], m.gate_text_prefer[0],
           m.gate_fusion_prefer[0]]
    p = float(m.dropout.p) if m.training else 0.0
    return _Pref.apply(content, image_embeds, text_embeds, fusion_embeds, p, seed, *[x.weight for x in lin],
                       *[x.bias for x in lin])


class _PrefRows(torch.autograd.Function):
    """The preference block on the batch rows `rows` (int64 [n], may repeat): from the
    full content / view tables to compact (all, side, content) rows; the backward writes
    the row gradients per occurrence and sums them per table row in a fixed order into
    full zero tables (rsx_smore_pref_rows with occ: deterministic, no float atomics)."""

    @staticmethod
    def forward(ctx, C_, IE, TE, FE, rows, p_drop, seed, sparse, exch, *wb):
        ctx.exch = exch
        W = [_c(x) for x in wb[:7]]
        b = [None if x is None else _c(x) for x in wb[7:]]
        C_, IE, TE, FE, rows = _c(C_), _c(IE), _c(TE), _c(FE), _c(rows)
        ctx.sparse = bool(sparse)
        n, d = rows.numel(), C_.shape[1]
        out = torch.empty(5, n, d, dtype=torch.float32, device=C_.device)
        all_, side, c_rows, f_rows, x2 = out.unbind(0)  # x2: the split forward's scratch
        # the forward's activations for the backward (7 products instead of 20 there)
        grad = any(ctx.needs_input_grad)
        saved = torch.empty(int(L.lib().rsx_smore_pref_rows_saved_floats(n, d)), dtype=torch.float32,
                            device=C_.device) if _SAVED and grad else None
        # the occurrence plan of the backward's per-row sums, built by this forward
        plan = torch.empty(int(L.lib().rsx_smore_pref_plan_words(n)), dtype=torch.int32,
                           device=C_.device) if _PLAN and grad and n > 0 else None
        lead = _lead_scratch(C_.shape[0], C_.device) if plan is not None else None
        L.check(L.lib().rsx_smore_pref_rows_saved(0, _arr(W), _arr(b), _p(C_), _p(IE), _p(TE), _p(FE), _p(rows), n,
                                                  d, float(p_drop), _p(seed), _p(all_), _p(side), _p(c_rows),
                                                  _p(f_rows), None, None, None, None, None, None, None, _p(x2), None,
                                                  None, None, _p(saved), _p(plan), _p(lead), ops._stream()),
                "rsx_smore_pref_rows_saved")
        ctx.has_saved = saved is not None
        ctx.plan = plan
        ctx.save_for_backward(C_, IE, TE, FE, rows, seed, c_rows, f_rows,
                              saved if saved is not None else torch.empty(0), *W,
                              *[x if x is not None else torch.empty(0) for x in b])
        ctx.has_b = [x is not None for x in b]
        ctx.p_drop = float(p_drop)
        return all_, side, c_rows

    @staticmethod
    def backward(ctx, g_all, g_side, g_crows):
        sv = ctx.saved_tensors
        C_, IE, TE, FE, rows, seed, c_rows, f_rows, saved = sv[:9]
        W = list(sv[9:16])
        b = [x if h else None for x, h in zip(sv[16:23], ctx.has_b)]
        n, d = rows.numel(), C_.shape[1]
        if g_all is None:
            g_all = torch.zeros_like(c_rows)
        g_all = _c(g_all)
        g_side = None if g_side is None else _c(g_side)
        g_crows = None if g_crows is None else _c(g_crows)
        # sparse: every consumer of these tables reads them on the batch rows only (the
        # tagged UI backbone, _PropMeanRows; the views' tagged R^T product, _ViewProp3), so
        # the rows the kernel does not write are never read and need no zero fill
        alloc = torch.empty if ctx.sparse else torch.zeros
        gfull = alloc(4, *C_.shape, dtype=torch.float32, device=C_.device)
        gC, gIE, gTE, gFE = gfull.unbind(0)
        # hv, ht (the tanh rows: saved by the forward, else recomputed here), dz[7] and the
        # per-occurrence row gradients (deterministic sums, no atomics)
        occ_n = int(L.lib().rsx_smore_pref_rows_occ_floats(n, d))
        nh = 0 if ctx.has_saved else 2
        scratch = torch.empty((7 + nh) * n * d + occ_n, dtype=torch.float32, device=C_.device)
        fields = scratch[: (7 + nh) * n * d].view(7 + nh, n, d).unbind(0)
        if ctx.has_saved:
            dz = list(fields)
            hv, ht = saved.view(-1, n, d)[1], saved.view(-1, n, d)[4]  # slots h_img, h_txt
        else:
            hv, ht, *dz = fields
        occ = scratch[(7 + nh) * n * d:]
        L.check(L.lib().rsx_smore_pref_rows_saved(1, _arr(W), _arr(b), _p(C_), _p(IE), _p(TE), _p(FE), _p(rows), n,
                                                  d, ctx.p_drop, _p(seed), None, None, None, None, _p(g_all),
                                                  _p(g_side), _p(g_crows), _p(gC), _p(gIE), _p(gTE), _p(gFE),
                                                  None if ctx.has_saved else _p(hv), None if ctx.has_saved else _p(ht),
                                                  _arr(dz), _p(occ), _p(saved) if ctx.has_saved else None,
                                                  _p(ctx.plan), None, ops._stream()), "rsx_smore_pref_rows_saved")
        tables = (gC, gIE, gTE, gFE)
        if ctx.exch is not None:  # data-parallel SMORE: the exchange (RowGradExchange)
            ctx.exch.start(rows, tables)
        xs = [f_rows, hv, f_rows, ht, c_rows, c_rows, c_rows]
        grads = _wgrad([(dz[i], xs[i], ctx.has_b[i]) for i in range(7)], d, C_.device)
        gW = [g[0] for g in grads]
        gb = [g[1] for g in grads]
        if ctx.exch is not None:
            gwb = ctx.exch.finish(tables, gW + gb)
            gW, gb = gwb[:7], gwb[7:]
        return (gC, gIE, gTE, gFE, None, None, None, None, None, *gW, *gb)


def preference_rows(model, content, image_embeds, text_embeds, fusion_embeds, rows, seed, weights=None,
                    sparse_grads=False, exch=None):
    """(all, side, content) rows of the reference's preference block at table rows
    `rows` only (the training loss reads no other row; the block is row-local).
    `weights`: the 7 weights then the 7 biases (None where absent) to use instead of
    the model's own tensors (the sharded model passes them through a gradient sum).
    `sparse_grads`: the four table gradients are defined on the batch rows only (their
    consumers read nothing else: see _PrefRows.backward).  `exch`: data-parallel SMORE's
    RowGradExchange, run on the block's gradients in its backward."""
    m = model
    if weights is None:
        lin = [m.query_v[0], m.query_v[2], m.query_t[0], m.query_t[2], m.gate_image_prefer[0],
               m.gate_text_prefer[0], m.gate_fusion_prefer[0]]
        weights = [x.weight for x in lin] + [x.bias for x in lin]
    p = float(m.dropout.p) if m.training else 0.0
    return _PrefRows.apply(content, image_embeds, text_embeds, fusion_embeds, rows, p, seed, bool(sparse_grads),
                           exch, *weights)


# ---------------------------------------------------------------------------
# item view -> [users; items] table
# ---------------------------------------------------------------------------
class _ViewProp(torch.autograd.Function):
    """out = [R G^L x ; G^L x] for one item-item graph G (L = n_layers) and the
    user-item block R (smore.py:299-317: the loop, then torch.cat([R x, x]))."""

    @staticmethod
    def forward(ctx, x, G, R, n_layers, n_users):
        x = _c(x)
        ni, d = x.shape
        out = torch.empty(n_users + ni, d, dtype=torch.float32, device=x.device)
        cur = x
        for k in range(n_layers):
            dst = out[n_users:] if k == n_layers - 1 else torch.empty_like(x)
            G.A.spmm(cur, out=dst)
            cur = dst
        if n_layers == 0:
            out[n_users:].copy_(x)
        R.A.spmm(out[n_users:], out=out[:n_users])
        ctx.G, ctx.R, ctx.L, ctx.nu = G, R, n_layers, n_users
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        nu = ctx.nu
        d = g.shape[1]
        gi = torch.empty_like(g[nu:])
        # d items = g_items + R^T g_users, in one launch (ADD epilogue)
        ctx.R.AT.spmm_epi(g[:nu], ops.epi(L.RSX_EPI_ADD, y=gi, r_add=g[nu:]), d)
        for _ in range(ctx.L):
            gi = ctx.G.AT.spmm(gi)
        return gi, None, None, None, None


def view_prop(x, G, R, n_layers, n_users):
    return _ViewProp.apply(x, G, R, int(n_layers), int(n_users))


class _ViewProp3(torch.autograd.Function):
    """The three item views (image, text, fusion) through _ViewProp's chain together:
    each layer's three item-graph products, the three R products, and in the backward
    the three R^T and item-graph transposes, each set as ONE rsx_spmm_batch launch."""

    @staticmethod
    def forward(ctx, x0, x1, x2, Gs, R, n_layers, n_users, comm, tags, gtags, rows):
        xs = [_c(x) for x in (x0, x1, x2)]
        ni, d = xs[0].shape
        outs = [torch.empty(n_users + ni, d, dtype=torch.float32, device=xs[0].device) for _ in range(3)]
        cur = xs
        for k in range(n_layers):
            dst = [o[n_users:] if k == n_layers - 1 else torch.empty_like(x) for o, x in zip(outs, xs)]
            ops.spmm_batch([G.A for G in Gs], cur, [ops.epi(L.RSX_EPI_STORE, y=y) for y in dst], d)
            cur = dst
        if n_layers == 0:
            for o, x in zip(outs, xs):
                o[n_users:].copy_(x)
        epis = [ops.epi(L.RSX_EPI_STORE, y=o[:n_users]) for o in outs]
        if tags is not None:  # user rows on the tagged (batch) users only; the rest are left unwritten
            for e in epis:
                e.row_tag, e.tag_dev = tags.row_tag.data_ptr(), tags.tag_dev.data_ptr()
                e.tag_flags = L.RSX_TAG_ROWS
        ops.spmm_batch([R.A] * 3, [o[n_users:] for o in outs], epis, d)
        ctx.Gs, ctx.R, ctx.L, ctx.nu, ctx.comm = Gs, R, n_layers, n_users, comm
        ctx.gtags, ctx.rows = gtags, rows
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        nu = ctx.nu
        ref = next(g for g in grads if g is not None)
        gs = [_c(g) if g is not None else torch.zeros_like(ref) for g in grads]
        d = ref.shape[1]
        gbuf = torch.empty(3, ref.shape[0] - nu, d, dtype=torch.float32, device=ref.device)
        gi = list(gbuf.unbind(0))
        # d items = g_items + R^T g_users (ADD epilogue), the three views in one launch.
        # (A scatter from the batch users instead, by float atomics, measured slower: 92 us
        # against 104 at C5, and at baby d = 64 three times the gather.)
        epis = [ops.epi(L.RSX_EPI_ADD, y=y, r_add=g[nu:]) for y, g in zip(gi, gs)]
        t = ctx.gtags
        if t is not None:
            # the incoming gradients are defined on the batch rows only (_PrefRows, sparse):
            # the users' rows are gathered (x_tag) and the items' rows added (row_tag on the
            # item block) on the tagged rows only -- re-tagged here, on this stream, as
            # _PropMeanRows does with its own tags on the side stream
            t.mark(ctx.rows)
            for e in epis:
                e.row_tag, e.x_tag, e.tag_dev = t.row_tag[nu:].data_ptr(), t.row_tag.data_ptr(), t.tag_dev.data_ptr()
                e.tag_flags = L.RSX_TAG_SPARSE_X | L.RSX_TAG_SPARSE_R
        ops.spmm_batch([ctx.R.AT] * 3, [g[:nu] for g in gs], epis, d)
        if ctx.comm is not None:  # users sharded (rsx.smore_dist): the item rows' gradient summed over the ranks
            ctx.comm.allreduce_(gbuf)
        for _ in range(ctx.L):
            nxt = [torch.empty_like(x) for x in gi]
            ops.spmm_batch([G.AT for G in ctx.Gs], gi, [ops.epi(L.RSX_EPI_STORE, y=y) for y in nxt], d)
            gi = nxt
        return gi[0], gi[1], gi[2], None, None, None, None, None, None, None, None


def view_prop3(xs, Gs, R, n_layers, n_users, comm=None, tags=None, gtags=None, rows=None):
    """(image, text, fusion) [R G^L x; G^L x] tables of the three views (one launch per
    layer for all three graphs, one for the three R products).  With `comm` (R = this
    rank's user rows) the item rows' gradients are summed over the ranks in one
    all-reduce before the item-graph backward.  With `tags` (the batch-row tags of the
    training loss, rsx.smore._RowTags over [users; items], already marked) the user rows
    are computed on the tagged users only: the preference block reads no other user row
    of a view.  With `gtags` (a _RowTags of its own) and `rows` the backward takes the
    incoming gradients as defined on `rows` only (preference_rows(sparse_grads=True))
    and reads nothing else of them."""
    return _ViewProp3.apply(xs[0], xs[1], xs[2], tuple(Gs), R, int(n_layers), int(n_users), comm, tags, gtags, rows)


# ---------------------------------------------------------------------------
# InfoNCE x 2
# ---------------------------------------------------------------------------
class _InfoNCE2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, side, content, users, pos, n_users, tau):
        side, content = _c(side), _c(content)
        users, pos = _c(users), _c(pos)
        B = users.numel()
        d = side.shape[1]
        lib = L.lib()
        ws = torch.empty(max(int(lib.rsx_smore_infonce_ws_bytes(B, d)), 4), dtype=torch.uint8, device=side.device)
        loss = torch.empty(2, dtype=torch.float32, device=side.device)
        L.check(lib.rsx_smore_infonce_fwd(_p(side), _p(content), _p(users), _p(pos), int(n_users), B, d, float(tau),
                                          _p(loss), _p(ws), ws.numel(), ops._stream()), "rsx_smore_infonce_fwd")
        ctx.save_for_backward(side, content, users, pos, ws)
        ctx.cfg = (int(n_users), float(tau), side.shape)
        return loss[0], loss[1]

    @staticmethod
    def backward(ctx, g_items, g_users):
        side, content, users, pos, ws = ctx.saved_tensors
        nu, tau, shape = ctx.cfg
        dev = side.device
        gl = torch.stack([g_items if g_items is not None else torch.zeros((), device=dev),
                          g_users if g_users is not None else torch.zeros((), device=dev)]).float().contiguous()
        gs = torch.zeros(shape, dtype=torch.float32, device=dev)
        gc = torch.zeros(shape, dtype=torch.float32, device=dev)
        L.check(L.lib().rsx_smore_infonce_bwd(_p(side), _p(content), _p(users), _p(pos), nu, users.numel(),
                                              shape[1], tau, _p(gl), _p(gs), _p(gc), _p(ws), ws.numel(),
                                              ops._stream()), "rsx_smore_infonce_bwd")
        return gs, gc, None, None, None, None


def infonce2(side, content, users, pos, n_users, tau):
    """(cl_items, cl_users) = (InfoNCE(side_i[pos], content_i[pos]), InfoNCE(side_u[u], content_u[u]))."""
    return _InfoNCE2.apply(side, content, users, pos, n_users, tau)


class _SmoreLossRows(torch.autograd.Function):
    """The SMORE training loss on compact batch rows ([users; positives; negatives]):
    BPR (RSX_BPR_SMORE, gradients computed with the loss) + cl * (InfoNCE(items) +
    InfoNCE(users)), the total formed by the InfoNCE mean kernel in the reference's
    f32 order; backward: the BPR gradient times the upstream gradient, the InfoNCE
    backward with the upstream gradient x cl read on the device (no loss-combination
    kernels either way)."""

    @staticmethod
    def forward(ctx, all_c, side_c, content_c, trip, ar, B, reg, batch_cfg, cl, tau):
        side_c, content_c = _c(side_c), _c(content_c)
        d = side_c.shape[1]
        # compact rows (b, b, B + b): the gradient rows are stored, no zero fill
        bl, gf, _ = ops.bpr(L.RSX_BPR_SMORE_ROWS, all_c.contiguous(), None, B, 2 * B, trip, reg, batch_cfg,
                            compact_rows=True)
        lib = L.lib()
        ws = torch.empty(max(int(lib.rsx_smore_infonce_ws_bytes(B, d)), 4), dtype=torch.uint8, device=side_c.device)
        out = torch.empty(3, dtype=torch.float32, device=side_c.device)  # cl_items, cl_users, total
        L.check(lib.rsx_smore_infonce_fwd_total(_p(side_c), _p(content_c), _p(ar), _p(ar), int(B), int(B), d,
                                                float(tau), _p(out), _p(bl), float(cl), _p(out[2:]), _p(ws),
                                                ws.numel(), ops._stream()), "rsx_smore_infonce_fwd_total")
        ctx.save_for_backward(side_c, content_c, ar, ws, gf)
        ctx.cfg = (int(B), float(tau), float(cl))
        parts = out[:2]
        ctx.mark_non_differentiable(parts)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the parts (a fill launch)
        return out[2], parts

    @staticmethod
    def backward(ctx, g_total, g_parts):
        side_c, content_c, ar, ws, gf = ctx.saved_tensors
        B, tau, cl = ctx.cfg
        # one launch: the InfoNCE rows stored (each batch row once), the negatives' rows
        # zeroed and the BPR rows' gradient times g_total -- no fill or multiply launches
        if side_c.shape[0] != 3 * B or gf.shape != side_c.shape:
            raise RuntimeError(f"smore_loss_rows: {tuple(side_c.shape)} side rows, {tuple(gf.shape)} BPR rows for a "
                               f"batch of {B} (3 B rows each expected)")
        g_all = torch.empty_like(gf)
        gsc = torch.empty(2, *side_c.shape, dtype=torch.float32, device=side_c.device)
        gt = g_total.contiguous()
        L.check(L.lib().rsx_smore_loss_rows_bwd(_p(side_c), _p(content_c), _p(ar), B, side_c.shape[1], tau, _p(gt), cl,
                                                _p(gf), _p(g_all), _p(gsc[0]), _p(gsc[1]), _p(ws), ws.numel(),
                                                ops._stream()), "rsx_smore_loss_rows_bwd")
        return g_all, gsc[0], gsc[1], None, None, None, None, None, None, None


def smore_loss_rows(all_c, side_c, content_c, trip, ar, B, reg, batch_cfg, cl, tau):
    """(total loss, [cl_items, cl_users]) of SMORE's training loss on compact batch rows."""
    return _SmoreLossRows.apply(all_c, side_c, content_c, trip, ar, int(B), float(reg), float(batch_cfg), float(cl),
                                float(tau))


# ---------------------------------------------------------------------------
# multi-tensor Adam
# ---------------------------------------------------------------------------
def adam_multi(params, grads, exp_avgs, exp_avg_sqs, steps, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
               grad_scale=1.0, lr_dev=None, halt=None, restore=None):
    """torch.optim.Adam's update over many tensors in one launch (per 32 tensors); the
    gradients are taken as g * grad_scale (f32 product) when grad_scale != 1; with
    lr_dev (a 1-element f64 device tensor) the learning rate is read from it; with
    halt (nan_gate's int32 flag) nothing is updated once it is set.  restore = (xs,
    alpha, mult): the mirror gradient's restore p += float(alpha * mult [* lr]) * x
    (axpy_multi's arithmetic) folded into the same launch (rsx_adam_multi_mg)."""
    n = len(params)
    if n == 0:
        return
    xs = list(restore[0]) if restore is not None else []
    for t in (*params, *grads, *exp_avgs, *exp_avg_sqs, *xs):
        if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
            raise RuntimeError("adam_multi: contiguous f32 GPU tensors only")
    sizes = (C.c_int64 * n)(*[p.numel() for p in params])
    if restore is not None:
        if len(xs) != n or any(x.numel() != p.numel() for x, p in zip(xs, params)):
            raise RuntimeError("adam_multi: one restore tensor per parameter, of its size")
        L.check(L.lib().rsx_adam_multi_mg(n, _arr(params), _arr(grads), _arr(exp_avgs), _arr(exp_avg_sqs),
                                          _arr(steps), sizes, float(lr), float(betas[0]), float(betas[1]), float(eps),
                                          float(weight_decay), float(grad_scale), _p(lr_dev), _p(halt), _arr(xs),
                                          _p(restore[1]), float(restore[2]), ops._stream()),
                "rsx_adam_multi_mg")
        return
    L.check(L.lib().rsx_adam_multi_scaled(n, _arr(params), _arr(grads), _arr(exp_avgs), _arr(exp_avg_sqs),
                                          _arr(steps), sizes, float(lr), float(betas[0]), float(betas[1]), float(eps),
                                          float(weight_decay), float(grad_scale), _p(lr_dev), _p(halt),
                                          ops._stream()),
            "rsx_adam_multi_scaled")


# ---------------------------------------------------------------------------
# model-level mirror gradient
# ---------------------------------------------------------------------------
def mg_alpha(params, grads, base, lr, rel_step, max_scale, lr_dev=None):
    """alpha_eff of the reference's mirror gradient (trainer.py:290-307) as a 0-d f64
    device tensor, from one pass over the (param, grad) pairs (two launches)."""
    n = len(params)
    sizes = (C.c_int64 * n)(*[p.numel() for p in params])
    lib = L.lib()
    dev = params[0].device
    ws = torch.empty(max(int(lib.rsx_mg_alpha_ws_bytes(n, sizes)), 16), dtype=torch.uint8, device=dev)
    alpha = torch.empty((), dtype=torch.float64, device=dev)
    L.check(lib.rsx_mg_alpha(n, _arr([p.detach() for p in params]), _arr(grads), sizes, float(base), float(lr),
                             float(rel_step), float(max_scale), _p(alpha), _p(ws), ws.numel(), _p(lr_dev),
                             ops._stream()),
            "rsx_mg_alpha")
    return alpha


def nan_gate(loss, halt, counter):
    """The batch loss's NaN check on the device (rsx_nan_gate; reference
    src/common/trainer.py:192-203): counter += 1, and on the first NaN loss
    halt = {1, counter}; the optimizer launches given `halt` then update nothing."""
    loss = loss.detach().reshape(1)
    if loss.dtype != torch.float32 or not loss.is_cuda:
        raise RuntimeError("nan_gate: a float32 GPU loss")
    L.check(L.lib().rsx_nan_gate(_p(loss), _p(halt), _p(counter), ops._stream()), "rsx_nan_gate")


def axpy_multi(ys, xs, alpha, mult, lr_dev=None, halt=None):
    """y += float(alpha * mult) * x for every pair (alpha: 0-d f64 device tensor; with
    lr_dev, a 1-element f64 device tensor, the scale is float(alpha * (mult * lr)));
    with halt (nan_gate's flag) nothing is updated once it is set."""
    n = len(ys)
    if n == 0:
        return
    sizes = (C.c_int64 * n)(*[y.numel() for y in ys])
    L.check(L.lib().rsx_axpy_multi(n, _arr([y.detach() for y in ys]), _arr(xs), sizes, _p(alpha), float(mult),
                                   _p(lr_dev), _p(halt), ops._stream()), "rsx_axpy_multi")
