"""nn.Linear container for SMORE's gate / query / preference layers.

RsxLinear keeps nn.Linear's parameters, initialisation order and state-dict names
(reference src/models/smore.py:106-120), so `init_seed` reproduces the reference's
weights and checkpoints load unchanged.  The SMORE training and evaluation path
never calls these modules: the fused kernels (csrc/smore_fuse.hip, rsx.smore_fuse)
read their weight / bias tensors directly.  `forward` remains for API callers that
apply a layer themselves (a library GEMM; with its weight gradient on the split-K
kernel rsx_linear_wgrad when the widths allow).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import ops


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        need = ctx.needs_input_grad
        g2 = g.reshape(-1, g.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        gx = (g @ w) if need[0] else None
        gw = ops.linear_wgrad(g2, x2) if need[1] else None
        gb = g2.sum(0) if (ctx.has_b and need[2]) else None
        return gx, gw, gb


class RsxLinear(nn.Linear):
    """Drop-in nn.Linear (same parameters, init and names) with the rsx weight gradient
    when the widths are multiples of 32 and the input is on the GPU."""

    def forward(self, x):
        if (x.is_cuda and self.in_features % 32 == 0 and self.out_features % 32 == 0
                and torch.is_grad_enabled() and self.weight.requires_grad):
            return _LinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)
