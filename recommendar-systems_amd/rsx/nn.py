"""nn.Linear whose weight gradient runs on rsx_linear_wgrad.

SMORE applies several Linear(d, d) layers to every user+item row (26k rows at
Amazon-baby; reference src/models/smore.py:106-120).  Their AddmmBackward weight
gradient g^T x has a d x d output and a 26k-long reduction, which a library GEMM
runs on a couple of workgroups (~130 us each, ~3 ms per SMORE step under the
mirror gradient).  RsxLinear keeps nn.Linear's parameters, initialisation and
state-dict names, and routes only that product to the split-K kernel; the input
gradient and the bias gradient stay torch ops.
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
