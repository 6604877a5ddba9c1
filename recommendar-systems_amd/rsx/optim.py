"""Adam with the rsx row kernel (RSX_EPI_ADAM through rsx_rowwise).

Same update as torch.optim.Adam's single-tensor path, which is what the reference
runs on CPU (src/common/trainer.py:133,238): bias corrections in float64, the
first moment by lerp, the second by mul + addcmul, then addcdiv.  One launch per
parameter tensor: a 28.9M-element SMORE feature table is one pass over p, g, m, v
instead of torch's chain of foreach kernels.  Works with torch LR schedulers (it
is a torch.optim.Optimizer and reads group["lr"] at every step).
"""
from __future__ import annotations

import torch

from . import ops


class RsxAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("RsxAdam does not support sparse gradients")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                ops.adam_(p.data, g, st["exp_avg"], st["exp_avg_sq"], st["step"], group["lr"],
                          betas=group["betas"], eps=group["eps"], weight_decay=group["weight_decay"])
        return loss
