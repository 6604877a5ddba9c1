"""SMORE's modality projection + spectral denoise / cross-modal fusion as the fused
HIP pass `rsx_smore_spectral_fwd` (reference src/models/smore.py:256-259 image_trs /
text_trs and :209-237 spectrum_convolution), with autograd.

Forward: two launches (fp32 MFMA): img = V Wv^T + bv, txt = T Wt^T + bt, then
their rfft's (saved for the backward), the three filtered spectra and the three
irfft's -- or, with the modality gates (smore.py:262-272), ONE launch (`item_side`,
rsx_smore_item_fwd).  Backward: two launches for the spectral part (d img, d txt, d w), then the
projection gradients of each modality in one pass over its rows (rsx_linear_bwd,
csrc/linear.hip): d Wv = d img^T V split-K, d V = d img Wv, d bv = colsum d img.
The unit normalisation of the complex weights (:221-229) and its backward are two
small launches (rsx_smore_unit_weights / _bwd, which also sums the spectral
backward's per-block weight partials) instead of ~40 torch complex-op kernels.
"""
from __future__ import annotations

import torch

import os

from . import _lib as L
from . import ops

# RSX_LBWD_PAIR=0: the two projection backwards as two launches (A/B)
_PAIR = os.environ.get("RSX_LBWD_PAIR", "1") != "0"


def spectral_supported(d: int, dv: int, dt: int) -> bool:
    """The shapes rsx_smore_spectral_fwd/bwd and rsx_linear_bwd are built for."""
    return d in (64, 128) and ops.linear_bwd_supported(d, dv) and ops.linear_bwd_supported(d, dt)


def unit_weight(w: torch.Tensor, normalize: bool) -> torch.Tensor:
    """[1, d/2+1, 2] parameter -> [(d/2+1), 2] (optionally unit-magnitude) weights."""
    cw = torch.view_as_complex(w)
    if normalize:
        cw = cw / (torch.abs(cw) + 1e-8)
    return torch.view_as_real(cw).reshape(-1, 2)


class _Spectral(torch.autograd.Function):
    @staticmethod
    def forward(ctx, V, Wv, bv, T, Wt, bt, rv, rt, rf, normalize):
        n, dv = V.shape
        dt = T.shape[1]
        d = Wv.shape[0]
        args = [x.contiguous() for x in (V, Wv, bv, T, Wt, bt, rv, rt, rf)]
        V, Wv, bv, T, Wt, bt, rv, rt, rf = args
        unit = _unit_weights(rv, rt, rf, d, normalize)
        wv, wt, wf = unit[0], unit[1], unit[2]
        img = torch.empty(n, d, device=V.device, dtype=torch.float32)
        txt = torch.empty_like(img)
        cv, ct, cf = torch.empty_like(img), torch.empty_like(img), torch.empty_like(img)
        lib = L.lib()
        spec = torch.empty(max(int(lib.rsx_smore_spectral_spec_floats(n, d)), 1), device=V.device,
                           dtype=torch.float32)
        p = ops._p
        ws = ops._ws(V.device, int(lib.rsx_smore_spectral_fwd_ws_bytes(n, d, dv, dt)))
        L.check(lib.rsx_smore_spectral_fwd(p(V), dv, p(Wv), p(bv), p(T), dt, p(Wt), p(bt), p(wv), p(wt), p(wf),
                                           n, d, p(img), p(txt), p(cv), p(ct), p(cf), p(spec), p(ws), ws.numel(),
                                           ops._stream()), "rsx_smore_spectral_fwd")
        ctx.save_for_backward(V, Wv, T, Wt, unit, rv, rt, rf, spec)
        ctx.nd = (n, d, int(bool(normalize)))
        # img / txt are diagnostics outputs that usually get no gradient: no zero-filled
        # stand-ins for them (nor for an unused conv) in the backward
        ctx.set_materialize_grads(False)
        return cv, ct, cf, img, txt

    @staticmethod
    def backward(ctx, g_cv, g_ct, g_cf, g_img_out, g_txt_out):
        return (*_spectral_backward(ctx.saved_tensors, ctx.nd, ctx.needs_input_grad, (g_cv, g_ct, g_cf), g_img_out,
                                    g_txt_out), None)


def _unit_weights(rv, rt, rf, d, normalize):
    unit = torch.empty(3, d // 2 + 1, 2, device=rv.device, dtype=torch.float32)
    L.check(L.lib().rsx_smore_unit_weights(ops._p(rv), ops._p(rt), ops._p(rf), d, int(bool(normalize)), ops._p(unit),
                                           ops._stream()), "rsx_smore_unit_weights")
    return unit


def _spectral_backward(saved, nd, need, g_conv, g_img_out=None, g_txt_out=None):
    """Gradients of (V, Wv, bv, T, Wt, bt, rv, rt, rf) from those of (conv_v, conv_t, conv_f,
    img, txt): the spectral backward launch, the unit-weight backward, then d W, d X, d b
    of each projection in one pass over its rows (rsx_linear_bwd)."""
    V, Wv, T, Wt, unit, rv, rt, rf, spec = saved
    wv, wt, wf = unit[0], unit[1], unit[2]
    n, d, normalize = nd
    p = ops._p
    lib = L.lib()
    gi = torch.empty(n, d, device=V.device, dtype=torch.float32)
    gt = torch.empty_like(gi)
    part = torch.empty(max(int(lib.rsx_smore_spectral_bwd_partials(n, d)), 1), device=V.device, dtype=torch.float32)
    gs = [None if g is None else g.contiguous() for g in g_conv]
    ws = ops._ws(V.device, int(lib.rsx_smore_spectral_bwd_ws_bytes(n, d)))
    L.check(lib.rsx_smore_spectral_bwd(p(spec), p(wv), p(wt), p(wf), *(None if g is None else p(g) for g in gs),
                                       n, d, p(gi), p(gt), p(part), p(ws), ws.numel(), ops._stream()),
            "rsx_smore_spectral_bwd")
    if g_img_out is not None:
        gi = gi + g_img_out
    if g_txt_out is not None:
        gt = gt + g_txt_out
    nb = d // 2 + 1
    grv, grt, grf = torch.empty_like(rv), torch.empty_like(rt), torch.empty_like(rf)
    L.check(lib.rsx_smore_unit_weights_bwd(p(part), part.numel() // (6 * nb), p(rv), p(rt), p(rf), d, normalize,
                                           p(grv), p(grt), p(grf), ops._stream()), "rsx_smore_unit_weights_bwd")
    # both projections' d W, d X, d b in one launch pair (rsx_linear_bwd_pair)
    if all(need[:6]) and _PAIR:
        res = ops.linear_bwd_pair((gi, V, Wv, True), (gt, T, Wt, True))
        if res is not None:
            (dWv, dV, dbv), (dWt, dT, dbt) = res
            return (dV, dWv, dbv, dT, dWt, dbt, grv, grt, grf)
    grads = []
    for g, X, Wx, k in ((gi, V, Wv, 0), (gt, T, Wt, 3)):
        if not (need[k] or need[k + 1] or need[k + 2]):
            grads += [None, None, None]
            continue
        # d W, d X and d b in one pass over the rows (rsx_linear_bwd)
        dW, dX, db = ops.linear_bwd(g, X, Wx, bias=need[k + 2])
        grads += [dX if need[k] else None, dW if need[k + 1] else None, db if need[k + 2] else None]
    return (*grads, grv, grt, grf)


_TILE_CNT = {}


def _tile_counters(device, n: int) -> torch.Tensor:
    """The fused pass's per-tile arrival counters: zero once, re-armed by the kernel (one
    buffer per device and stream: calls on one stream are ordered)."""
    key = (str(device), torch.cuda.current_stream().cuda_stream, int(n))
    t = _TILE_CNT.get(key)
    if t is None:
        t = torch.zeros(max(int(L.lib().rsx_smore_item_tiles(n)), 1), dtype=torch.int32, device=device)
        _TILE_CNT[key] = t
    return t


class _ItemSide(torch.autograd.Function):
    """smore.py:256-272 in one forward launch (rsx_smore_item_fwd): projections, spectral
    part, modality gates.  Backward: the gates' launch (+ their weight gradients), then the
    spectral part's (as _Spectral)."""

    @staticmethod
    def forward(ctx, V, Wv, bv, T, Wt, bt, rv, rt, rf, item, gWv, gbv, gWt, gbt, gWf, gbf, normalize, scale, mul):
        from .smore_fuse import _arr, _c

        n, dv = V.shape
        dt = T.shape[1]
        d = Wv.shape[0]
        V, Wv, bv, T, Wt, bt, rv, rt, rf, item = (_c(x) for x in (V, Wv, bv, T, Wt, bt, rv, rt, rf, item))
        gW = [_c(x) for x in (gWv, gWt, gWf)]
        gb = [_c(x) for x in (gbv, gbt, gbf)]
        unit = _unit_weights(rv, rt, rf, d, normalize)
        img = torch.empty(n, d, device=V.device, dtype=torch.float32)
        txt, cv, ct, cf = (torch.empty_like(img) for _ in range(4))
        outs = [torch.empty_like(img) for _ in range(3)]
        lib = L.lib()
        spec = torch.empty(max(int(lib.rsx_smore_spectral_spec_floats(n, d)), 1), device=V.device,
                           dtype=torch.float32)
        p = ops._p
        ws = ops._ws(V.device, int(lib.rsx_smore_spectral_fwd_ws_bytes(n, d, dv, dt)))
        L.check(lib.rsx_smore_item_fwd(p(V), dv, p(Wv), p(bv), p(T), dt, p(Wt), p(bt), p(unit[0]), p(unit[1]),
                                       p(unit[2]), n, d, p(img), p(txt), p(cv), p(ct), p(cf), p(spec), p(ws),
                                       ws.numel(), p(_tile_counters(V.device, n)), p(item), _arr(gW), _arr(gb),
                                       float(scale), int(mul), _arr(outs), ops._stream()), "rsx_smore_item_fwd")
        ctx.save_for_backward(V, Wv, T, Wt, unit, rv, rt, rf, spec, cv, ct, cf, item, *gW, *gb)
        ctx.nd = (n, d, int(bool(normalize)))
        ctx.cfg = (float(scale), int(mul))
        ctx.mark_non_differentiable(cv, ct, cf, img, txt)
        ctx.set_materialize_grads(False)
        return (*outs, cv, ct, cf, img, txt)

    @staticmethod
    def backward(ctx, gv, gt, gf, *_unused):
        from .smore_fuse import _gates_backward

        saved = ctx.saved_tensors
        cv, ct, cf, item = saved[9:13]
        gW, gb = saved[13:16], saved[16:19]
        need = ctx.needs_input_grad
        gc, g_item, gate_grads = _gates_backward((cv, ct, cf), item, gW, gb, ctx.cfg, (gv, gt, gf))
        spec_grads = _spectral_backward(saved[:9], ctx.nd, need, gc)
        return (*spec_grads, g_item if need[9] else None, *gate_grads, None, None, None)


def item_side(V, Wv, bv, T, Wt, bt, wv, wt, wf, item, gate_v, gate_t, gate_f, scale: float, mul: bool,
              normalize=True):
    """(img_i, txt_i, fus_i, conv_v, conv_t, conv_f, img, txt) through the one-launch item
    side; gate_x are the reference's nn.Sequential(Linear, Sigmoid) modules."""
    lv, lt, lf = gate_v[0], gate_t[0], gate_f[0]
    return _ItemSide.apply(V, Wv, bv, T, Wt, bt, wv, wt, wf, item, lv.weight, lv.bias, lt.weight, lt.bias, lf.weight,
                           lf.bias, bool(normalize), float(scale), bool(mul))


def spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf, normalize=True):
    """(conv_v, conv_t, conv_f, img, txt) through the fused HIP pass."""
    return _Spectral.apply(V, Wv, bv, T, Wt, bt, wv, wt, wf, bool(normalize))


def spectral_available() -> bool:
    return hasattr(L.lib(), "rsx_smore_spectral_fwd")


def spectral_fused(model):
    """The model's projected spectrum (conv_v, conv_t, conv_f) via the fused pass."""
    cv, ct, cf, img, txt = spectral(model.image_embedding.weight, model.image_trs.weight, model.image_trs.bias,
                                    model.text_embedding.weight, model.text_trs.weight, model.text_trs.bias,
                                    model.image_complex_weight, model.text_complex_weight,
                                    model.fusion_complex_weight, model.spectral_weight_norm)
    model._last["spec_in"] = (img.detach(), txt.detach())
    return cv, ct, cf


def item_side_fused(model, item):
    """The model's (img_i, txt_i, fus_i) and (conv_v, conv_t, conv_f) via the one-launch
    item side (item: the item_id embedding table, as the caller's view of it)."""
    img_i, txt_i, fus_i, cv, ct, cf, img, txt = item_side(
        model.image_embedding.weight, model.image_trs.weight, model.image_trs.bias, model.text_embedding.weight,
        model.text_trs.weight, model.text_trs.bias, model.image_complex_weight, model.text_complex_weight,
        model.fusion_complex_weight, item, model.gate_v, model.gate_t, model.gate_f, model.inject_scale,
        model.inject_mode == "mul", model.spectral_weight_norm)
    model._last["spec_in"] = (img.detach(), txt.detach())
    return (img_i, txt_i, fus_i), (cv, ct, cf)
