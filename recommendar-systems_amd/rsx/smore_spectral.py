"""SMORE's modality projection + spectral denoise / cross-modal fusion as the fused
HIP pass `rsx_smore_spectral_fwd` (reference src/models/smore.py:256-259 image_trs /
text_trs and :209-237 spectrum_convolution), with autograd.

Forward: two launches (fp32 MFMA): img = V Wv^T + bv, txt = T Wt^T + bt, then
their rfft's (saved for the backward), the three filtered spectra and the three
irfft's.  Backward: one launch for the spectral part (d img, d txt, d w), then the
projection gradients:
d Wv = d img^T V on the split-K kernel (rsx_linear_wgrad), d V = d img Wv as a
library GEMM, d bv = colsum.
The unit normalisation of the complex weights (:221-229) stays a torch op on the
(d/2+1)-sized parameters so autograd handles it exactly as the reference does.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import ops


def spectral_supported(d: int, dv: int, dt: int) -> bool:
    return d in (64, 128) and dv % 4 == 0 and dt % 4 == 0


def unit_weight(w: torch.Tensor, normalize: bool) -> torch.Tensor:
    """[1, d/2+1, 2] parameter -> [(d/2+1), 2] (optionally unit-magnitude) weights."""
    cw = torch.view_as_complex(w)
    if normalize:
        cw = cw / (torch.abs(cw) + 1e-8)
    return torch.view_as_real(cw).reshape(-1, 2)


def _wgrad(g, x):
    """d W = g^T x (a d x dv output over the n items): the split-K kernel when the
    widths allow it (rsx_linear_wgrad), else a library GEMM."""
    if g.shape[1] % 32 == 0 and x.shape[1] % 32 == 0:
        return ops.linear_wgrad(g, x)
    return g.t() @ x


class _Spectral(torch.autograd.Function):
    @staticmethod
    def forward(ctx, V, Wv, bv, T, Wt, bt, wv, wt, wf):
        n, dv = V.shape
        dt = T.shape[1]
        d = Wv.shape[0]
        args = [x.contiguous() for x in (V, Wv, bv, T, Wt, bt, wv, wt, wf)]
        V, Wv, bv, T, Wt, bt, wv, wt, wf = args
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
        ctx.save_for_backward(V, Wv, T, Wt, wv, wt, wf, spec)
        ctx.nd = (n, d)
        return cv, ct, cf, img, txt

    @staticmethod
    def backward(ctx, g_cv, g_ct, g_cf, g_img_out, g_txt_out):
        V, Wv, T, Wt, wv, wt, wf, spec = ctx.saved_tensors
        n, d = ctx.nd
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
        gw = part.view(-1, 3, d // 2 + 1, 2).sum(0)
        need = ctx.needs_input_grad
        gV = gi @ Wv if need[0] else None
        gWv = _wgrad(gi, V) if need[1] else None
        gbv = gi.sum(0) if need[2] else None
        gT = gt @ Wt if need[3] else None
        gWt = _wgrad(gt, T) if need[4] else None
        gbt = gt.sum(0) if need[5] else None
        return gV, gWv, gbv, gT, gWt, gbt, gw[0], gw[1], gw[2]


def spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf, normalize=True):
    """(conv_v, conv_t, conv_f, img, txt) through the fused HIP pass."""
    return _Spectral.apply(V, Wv, bv, T, Wt, bt, unit_weight(wv, normalize), unit_weight(wt, normalize),
                           unit_weight(wf, normalize))


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
