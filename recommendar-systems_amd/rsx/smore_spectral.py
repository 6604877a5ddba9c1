"""SMORE's modality projection + spectral denoise / cross-modal fusion as the fused
HIP pass `rsx_smore_spectral_fwd` (reference src/models/smore.py:256-259 image_trs /
text_trs and :209-237 spectrum_convolution), with autograd.

Forward: two launches (fp32 MFMA): img = V Wv^T + bv, txt = T Wt^T + bt, then
their rfft's (saved for the backward), the three filtered spectra and the three
irfft's.  Backward: one launch for the spectral part (d img, d txt, d w), then the
projection gradients of each modality in one pass over its rows (rsx_linear_bwd,
csrc/linear.hip): d Wv = d img^T V split-K, d V = d img Wv, d bv = colsum d img.
The unit normalisation of the complex weights (:221-229) and its backward are two
small launches (rsx_smore_unit_weights / _bwd, which also sums the spectral
backward's per-block weight partials) instead of ~40 torch complex-op kernels.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import ops


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
        unit = torch.empty(3, d // 2 + 1, 2, device=V.device, dtype=torch.float32)
        L.check(L.lib().rsx_smore_unit_weights(ops._p(rv), ops._p(rt), ops._p(rf), d, int(bool(normalize)),
                                               ops._p(unit), ops._stream()), "rsx_smore_unit_weights")
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
        V, Wv, T, Wt, unit, rv, rt, rf, spec = ctx.saved_tensors
        wv, wt, wf = unit[0], unit[1], unit[2]
        n, d, normalize = ctx.nd
        p = ops._p
        lib = L.lib()
        gi = torch.empty(n, d, device=V.device, dtype=torch.float32)
        gt = torch.empty_like(gi)
        part = torch.empty(max(int(lib.rsx_smore_spectral_bwd_partials(n, d)), 1), device=V.device,
                           dtype=torch.float32)
        gs = [None if g is None else g.contiguous() for g in (g_cv, g_ct, g_cf)]
        L.check(lib.rsx_smore_spectral_bwd(p(spec), p(wv), p(wt), p(wf),
                                           *(None if g is None else p(g) for g in gs),
                                           n, d, p(gi), p(gt), p(part), ops._stream()), "rsx_smore_spectral_bwd")
        if g_img_out is not None:
            gi = gi + g_img_out
        if g_txt_out is not None:
            gt = gt + g_txt_out
        nb = d // 2 + 1
        grv, grt, grf = torch.empty_like(rv), torch.empty_like(rt), torch.empty_like(rf)
        L.check(lib.rsx_smore_unit_weights_bwd(p(part), part.numel() // (6 * nb), p(rv), p(rt), p(rf), d, normalize,
                                               p(grv), p(grt), p(grf), ops._stream()), "rsx_smore_unit_weights_bwd")
        need = ctx.needs_input_grad
        grads = []
        for g, X, Wx, k in ((gi, V, Wv, 0), (gt, T, Wt, 3)):
            if not (need[k] or need[k + 1] or need[k + 2]):
                grads += [None, None, None]
                continue
            # d W, d X and d b in one pass over the rows (rsx_linear_bwd)
            dW, dX, db = ops.linear_bwd(g, X, Wx, bias=need[k + 2])
            grads += [dX if need[k] else None, dW if need[k + 1] else None, db if need[k + 2] else None]
        return (*grads, grv, grt, grf, None)


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
