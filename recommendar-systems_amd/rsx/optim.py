"""Adam with the rsx row kernel (RSX_EPI_ADAM through rsx_rowwise).

Same update as torch.optim.Adam's single-tensor path, which is what the reference
runs on CPU (src/common/trainer.py:133,238): bias corrections in float64, the
first moment by lerp, the second by mul + addcmul, then addcdiv.  One launch for
all of a group's parameter tensors (rsx_adam_multi, up to 32 tensors per launch):
a 28.9M-element SMORE feature table and its 28 small Linear / spectral tensors
are one pass over p, g, m, v instead of torch's chain of foreach kernels.  Works with torch LR schedulers (it
is a torch.optim.Optimizer and reads group["lr"] at every step).

The step count lives on the device (`state["step"]`, a 0-d int64 tensor, bumped by
one foreach launch per group; the kernel reads it through `rsx_adam.step_dev`), so
a step holds no host-side counter and can be captured in a HIP graph and replayed
(rsx.trainer's graph step); only a change of `lr` needs a new capture.
"""
from __future__ import annotations

import torch

from .smore_fuse import adam_multi, axpy_multi


class RsxAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        # the next step() takes every gradient as g * grad_scale (then resets it to 1):
        # the mirror gradient's p.grad.mul_(-beta) folded into the update
        self.grad_scale = 1.0
        # optional 1-element f64 device tensor holding the learning rate (set by
        # rsx.trainer for graph-captured steps: a new lr then needs no new capture)
        self.lr_dev = None
        # optional int32 [2] device flag of rsx.smore_fuse.nan_gate (set by rsx.trainer):
        # once a batch loss was NaN no update changes any parameter or moment
        self.halt = None
        # the mirror gradient's restore for the next step() (then reset): (params, xs,
        # alpha, mult, lr_dev, halt) — p += float(alpha * mult [* lr]) * x folded into the
        # Adam launch when the step updates exactly `params` with the same lr_dev / halt
        # (rsx.trainer); otherwise rsx_axpy_multi applies it before the update
        self.restore = None

    def lr_on_device(self) -> bool:
        """Whether every update reads the learning rate from `lr_dev` (one group of
        contiguous parameters: the rsx_adam_multi path); otherwise a captured step has
        the host lr baked into its launches."""
        return (self.lr_dev is not None and len(self.param_groups) == 1
                and all(p.is_contiguous() for p in self.param_groups[0]["params"]))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        gs, self.grad_scale = float(self.grad_scale), 1.0
        restore, self.restore = self.restore, None
        rmap = None
        if restore is not None:
            rps, rxs, ralpha, rmult, rlr, rhalt = restore
            live_all = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
            fold = (len(self.param_groups) == 1 and len(rps) == len(live_all) and rlr is self.lr_dev
                    and rhalt is self.halt
                    and {id(p) for p in rps} == {id(p) for p in live_all}
                    and all(p.is_contiguous() for p in live_all))
            if fold:
                rmap = {id(p): x for p, x in zip(rps, rxs)}
            else:  # the restore as its own pass, then the plain update
                axpy_multi(rps, rxs, ralpha, rmult, rlr, rhalt)
        for group in self.param_groups:
            live = [p for p in group["params"] if p.grad is not None]
            for p in live:
                if p.grad.is_sparse:
                    raise RuntimeError("RsxAdam does not support sparse gradients")
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.int64, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif not (torch.is_tensor(st["step"]) and st["step"].dtype == torch.int64
                          and st["step"].device == p.device):
                    # a state dict saved by torch.optim.Adam (float step) or an older RsxAdam (int)
                    st["step"] = torch.tensor(int(st["step"]), dtype=torch.int64, device=p.device)
            if not live:
                continue
            steps = [self.state[p]["step"] for p in live]
            torch._foreach_add_(steps, 1)
            grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in live]
            if all(p.is_contiguous() for p in live):
                adam_multi([p.data for p in live], grads,
                           [self.state[p]["exp_avg"] for p in live], [self.state[p]["exp_avg_sq"] for p in live],
                           steps, group["lr"], betas=group["betas"], eps=group["eps"],
                           weight_decay=group["weight_decay"], grad_scale=gs,
                           lr_dev=self.lr_dev if len(self.param_groups) == 1 else None, halt=self.halt,
                           restore=None if rmap is None else ([rmap[id(p)] for p in live], ralpha, rmult))
                continue
            # a non-contiguous parameter: the same launch on contiguous copies, copied back
            ts = [[t.contiguous() for t in (p.data, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"])]
                  for p in live]
            adam_multi([t[0] for t in ts], grads, [t[1] for t in ts], [t[2] for t in ts], steps, group["lr"],
                       betas=group["betas"], eps=group["eps"], weight_decay=group["weight_decay"], grad_scale=gs,
                       halt=self.halt)
            for p, (pc, mc, vc) in zip(live, ts):
                for dst, src in ((p.data, pc), (self.state[p]["exp_avg"], mc), (self.state[p]["exp_avg_sq"], vc)):
                    if dst.data_ptr() != src.data_ptr():
                        dst.copy_(src)
        return loss
