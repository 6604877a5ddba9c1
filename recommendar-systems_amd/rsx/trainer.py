"""Trainer with the reference's behaviour and log format (src/common/trainer.py:47-548).

fit(): per epoch `pre_epoch_processing`, one pass over the training loader,
LambdaLR step (lr * gamma^(epoch/T) from `learning_rate_scheduler`), then every
`eval_step` epochs evaluation on valid and test, early stopping on
`valid_metric` with patience `stopping_step`; returns (best valid score, best
valid result, test result at the best valid epoch).

Training pass, two modes:
* fused (model.supports_fused_step and config rsx_fused_step, no classic mirror
  gradient): `model.fused_step(batch, lr)` per batch — forward, loss, backward
  and Adam on the device; the loss is summed on the device and read once per
  epoch (the reference syncs `loss.item()` every batch, trainer.py:196-200).  A
  NaN batch loss sets the step's device halt flag (LightGCN's tagged step): its
  own and every later Adam update of the epoch are skipped, so the parameters are
  those of the batch before it, as in the reference, which checks before backward
  and stops (trainer.py:201-203); the epoch-end read reports that batch index;
* autograd: calculate_loss / backward / torch optimizer exactly as the
  reference, including classic MG (`mg=True`) and the model-level mirror
  gradient (model.mg_enable, trainer.py:268-348).

evaluate(): per eval batch `model.full_sort_topk` (fused scores + mask + top-k)
when the model has it, else full_sort_predict + mask (-1e10) + torch.topk, then
TopKEvaluator (vectorised hit matrix, same metric values).
"""
from __future__ import annotations

import gc
import itertools
import os
from logging import getLogger
from time import time

import numpy as np
import torch
import torch.optim as optim
from torch.nn.utils.clip_grad import clip_grad_norm_

from .evaluator import TopKEvaluator
from .utils import dict2str, early_stopping


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _mg_alpha(params, grads, base, lr, rel_step, max_scale):
    """The mirror-gradient step scale (reference trainer.py:300-318) as a 0-d float64
    device tensor: max(base, rel * rms(p) / (lr * rms(g) + 1e-12)) capped at
    base * max_scale.  The RMS values are f32 tensor results, as in the reference
    (it converts them with float()); the rest is the same float64 arithmetic in the
    same order, so the value is the reference's bit for bit, with no host sync."""
    if not grads:
        dev = params[0].device if params else "cpu"
        return torch.tensor(base, dtype=torch.float64, device=dev)
    g_all = torch.cat([g.view(-1) for g in grads])
    p_all = torch.cat([p.detach().view(-1) for p in params])
    grad_rms = (g_all.norm() / (g_all.numel() ** 0.5)).double()
    param_rms = (p_all.norm() / (p_all.numel() ** 0.5) + 1e-12).double()
    alpha = rel_step * param_rms / (lr * grad_rms + 1e-12)
    # Python's max(base, x) keeps base when x is NaN; clamp would propagate it
    alpha = torch.where(alpha > base, alpha, torch.full_like(alpha, base))
    return torch.clamp(alpha, max=base * max_scale)


def _mg_print(step_id, mirror, alpha):
    print(f"[MG] step={step_id} mirror_loss={float(mirror.item()):.4f} α_eff={float(alpha):.3g}")


class _GraphStep:
    """One training batch (`Trainer._train_batch`: forward, loss, backward, Adam and
    the model-level mirror gradient) captured as a HIP graph and replayed.

    A SMORE batch is ~1000 small kernels; launched one by one from Python the host is
    slower than the GPU, so the step is host-bound.  Replaying a captured graph
    issues them in one submission.  What a replay must not depend on is host state,
    so the step keeps none on the host: the Adam step count is a device counter
    (rsx.optim.RsxAdam), the mirror-gradient scale a device scalar (_mg_alpha),
    losses stay device tensors, and the batch is copied into a static buffer.

    The control flow of a batch depends on the host counter `model.global_step`
    (mirror gradient when the step after the first calculate_loss is a multiple of
    mg_interval; diagnostics every mg_log_interval steps).  Each branch is its own
    graph ("kind", per batch shape), the host counter is advanced by what the
    capture advanced it by, and batches that log diagnostics run eagerly.  A kind is
    captured only after one eager batch of that kind and shape, so lazily allocated
    workspaces exist outside the graph's memory pool.  The learning rate is read
    on the device (Trainer._sync_lr), so the LambdaLR schedule keeps the graphs
    (without a device lr, a change of lr drops them).

    Contract for a model to opt in (`supports_graph_step = True`): calculate_loss
    increments `global_step` by one (if it has one), and no host syncs or
    data-dependent host branches in calculate_loss."""

    def __init__(self, trainer, loss_func):
        self.t = trainer
        self.loss_func = loss_func
        self.seen = set()
        self.graphs = {}
        self.lr = None
        self.replays = 0

    def _kind(self):
        """(mirror-gradient batch?) or None when the batch must run eagerly."""
        m = self.t.model
        g1 = int(getattr(m, "global_step", 0)) + 1  # the step id _mirror_gradient will see
        log_every = int(getattr(m, "mg_log_interval", 50))
        if log_every > 0 and g1 % log_every == 0 and hasattr(m, "log_mm_diagnostics"):
            if getattr(m, "diagnostics_enabled", lambda: True)():
                return None
        interval = int(getattr(m, "mg_interval", 0)) if getattr(m, "mg_enable", False) else 0
        return bool(interval > 0 and g1 % interval == 0)

    def step(self, inter):
        """The batch through a graph: (losses, loss), or None to run it eagerly."""
        if not (torch.is_tensor(inter) and inter.is_cuda):
            return None
        kind = self._kind()
        if kind is None:
            return None
        # one graph per (batch shape, kind): a sharded epoch's balanced slices come in two
        # sizes; the loader's last partial batch is a third
        kind = (tuple(inter.shape), kind)
        opt = self.t.optimizer
        lr = tuple(g["lr"] for g in opt.param_groups)
        if lr != self.lr and not getattr(opt, "lr_on_device", lambda: False)():
            self.graphs.clear()  # the lr is baked into the captured launches
        self.lr = lr
        if kind not in self.seen:
            self.seen.add(kind)
            return None
        m = self.t.model
        cap = self.graphs.get(kind)
        if cap is None:
            cap = self._capture(inter)
            self.graphs[kind] = cap
        else:
            cap["static"].copy_(inter)
            if hasattr(m, "global_step"):
                m.global_step += cap["dstep"]
        step_id = int(getattr(m, "global_step", 0)) - cap["dstep"] + 1
        cap["graph"].replay()
        self.replays += 1
        losses, loss = cap["out"]
        if cap["mg"] is not None and getattr(m, "mg_verbose", False):
            _mg_print(step_id, cap["mg"][1], cap["mg"][2])
        if isinstance(losses, tuple):
            return tuple(x.clone() for x in losses), loss.clone()
        loss = loss.clone()
        return loss, loss

    def _capture(self, inter):
        m = self.t.model
        static = inter.detach().clone()
        before = int(getattr(m, "global_step", 0))
        g = torch.cuda.CUDAGraph()
        if os.environ.get("RSX_GRAPH_DEBUG"):
            print(f"[graph] capture at global_step={before}", flush=True)
        # no cyclic GC inside the capture: a finalizer of some unrelated object (a
        # CUDA graph or stream-ordered buffer of an earlier run) that issues a HIP call
        # forbidden while a stream captures would abort the process
        # (torch.cuda.graph collects once on entry)
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g):
                losses, loss = self.t._train_batch(static, 0, self.loss_func)
                # detached: graph outputs that keep the captured autograd graph alive
                # would hold its AccumulateGrad nodes into the next capture
                out = (tuple(x.detach() for x in losses) if isinstance(losses, tuple) else losses.detach(),
                       loss.detach())
        finally:
            if gc_on:
                gc.enable()
        return dict(graph=g, static=static, out=out, mg=getattr(self.t, "_mg_last", None),
                    dstep=int(getattr(m, "global_step", 0)) - before)


class Trainer:
    def __init__(self, config, model, mg=False):
        self.config = config
        self.model = model
        self.logger = getLogger()
        self.learner = config["learner"]
        self.learning_rate = config["learning_rate"]
        self.epochs = config["epochs"]
        self.eval_step = min(config["eval_step"], self.epochs)
        self.stopping_step = config["stopping_step"]
        self.clip_grad_norm = config["clip_grad_norm"]
        self.valid_metric = config["valid_metric"].lower()
        self.valid_metric_bigger = config["valid_metric_bigger"]
        self.test_batch_size = config["eval_batch_size"]
        self.device = config["device"]
        wd = config["weight_decay"]
        self.weight_decay = (eval(wd) if isinstance(wd, str) else wd) if wd is not None else 0.0  # noqa: S307
        self.req_training = config["req_training"]
        self.start_epoch = 0
        self.cur_step = 0
        blank = {f"{m.lower()}@{k}": 0.0 for m, k in itertools.product(config["metrics"], config["topk"])}
        self.best_valid_score = -1
        self.best_valid_result = blank
        self.best_test_upon_valid = blank
        self.train_loss_dict = {}
        self.mg = mg
        self.alpha1, self.alpha2, self.beta = config["alpha1"], config["alpha2"], config["beta"]
        self.fused = bool(getattr(model, "supports_fused_step", False)) and bool(
            config.get("rsx_fused_step", True)) and not mg and not getattr(model, "mg_enable", False)
        sched = config["learning_rate_scheduler"] or [1.0, 50]
        self._lr_fac = lambda epoch: sched[0] ** (epoch / sched[1])
        self.optimizer = None if self.fused else self._build_optimizer()
        self.lr_scheduler = (optim.lr_scheduler.LambdaLR(self.optimizer, lr_lambda=self._lr_fac)
                             if self.optimizer is not None else None)
        self._epoch_for_lr = 0
        self.evaluator = TopKEvaluator(config)
        self.mg_target_rel_step = float(config.get("mg_target_rel_step", 1e-3))
        self.mg_alpha_max_scale = float(config.get("mg_alpha_max_scale", 20.0))
        self._graph = None

    # ------------------------------------------------------------------ setup
    def _build_optimizer(self):
        params = self.model.parameters()
        name = (self.learner or "adam").lower()
        if name == "adam":
            params = list(params)
            if bool(self.config.get("rsx_adam", True)) and params and all(p.is_cuda for p in params):
                from .optim import RsxAdam

                return RsxAdam(params, lr=self.learning_rate, weight_decay=self.weight_decay)
            return optim.Adam(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "sgd":
            return optim.SGD(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "adagrad":
            return optim.Adagrad(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        if name == "rmsprop":
            return optim.RMSprop(params, lr=self.learning_rate, weight_decay=self.weight_decay)
        self.logger.warning("Received unrecognized optimizer, set default Adam optimizer")
        return optim.Adam(params, lr=self.learning_rate)

    def current_lr(self):
        if self.optimizer is not None:
            return self.optimizer.param_groups[0]["lr"]
        return self.learning_rate * self._lr_fac(self._epoch_for_lr)

    # ------------------------------------------------------------------ train
    def _train_epoch(self, train_data, epoch_idx, loss_func=None):
        if not self.req_training:
            return 0.0, []
        self.model.train()
        if self.fused:
            return self._train_epoch_fused(train_data, epoch_idx)
        return self._train_epoch_autograd(train_data, epoch_idx, loss_func)

    def _train_epoch_fused(self, train_data, epoch_idx):
        acc = self.model.device_loss_acc
        acc.zero_()
        lr = self.current_lr()
        n = 0
        # the step's device NaN gate (single engine, data-parallel engine): cleared per epoch,
        # so a halt of an earlier fit() does not carry into this one
        halt = getattr(self.model, "device_halt", None)
        if halt is not None:
            halt[0].zero_()
        if getattr(self.model, "sharded", False):
            # user-sharded / data-parallel model (torchrun): every rank runs the same number
            # of steps on its own device-sampled batches; the epoch loss is the sum over ranks
            import torch.distributed as dist

            for i in range(self.model.steps_per_epoch):
                self.model.fused_step_index(epoch_idx, i, lr)
                n += 1
            # the row-sharded engine's deferred parameter all-gather is a collective: every
            # rank completes it here, at the same point, so that a later read of the
            # parameters (a rank-0 checkpoint, state_dict) needs no exchange
            flush = getattr(getattr(self.model, "engine", None), "flush", None)
            if flush is not None:
                flush()
            if getattr(self.model, "dp", False):  # data-parallel: every rank holds the global batches' loss
                total = float(acc.item())
            else:
                tot = acc.clone() if dist.get_backend() == "nccl" else acc.cpu()
                dist.all_reduce(tot)
                total = float(tot.item())
        else:
            for batch in train_data:
                self.model.fused_step(batch, lr)
                n += 1
            total = float(acc.item())  # one host sync per epoch
        if halt is not None:
            flag, s0 = halt  # (device flag, engine step count before this epoch)
            h = flag.cpu().tolist()
            if h[0]:  # the step's NaN gate: the batch, and the parameters of the batch before it
                b = h[1] - s0 - 1
                self.logger.info(f"Loss is nan at epoch: {epoch_idx}, batch index: {b}. Exiting.")
                return torch.tensor(float("nan")), torch.tensor(0.0)
        if np.isnan(total):
            self.logger.info(f"Loss is nan at epoch: {epoch_idx}. Exiting.")
            return torch.tensor(float("nan")), torch.tensor(0.0)
        return total, n

    def _check_nan(self, loss):
        return bool(torch.isnan(loss))

    def _nan_gate_on(self) -> bool:
        """The device NaN gate (rsx_nan_gate + the halt flag of RsxAdam / axpy_multi)
        replaces the reference's per-batch host check when every update goes through
        the rsx optimizer kernels."""
        from .optim import RsxAdam

        return isinstance(self.optimizer, RsxAdam) and torch.cuda.is_available() and \
            bool(self.config.get("rsx_nan_gate", True))

    def _arm_nan_gate(self):
        if getattr(self, "_halt", None) is None:
            dev = next(iter(self.model.parameters())).device
            self._halt = torch.zeros(2, dtype=torch.int32, device=dev)
            self._nan_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self._halt.zero_()
        self._nan_ctr.zero_()
        self.optimizer.halt = self._halt

    def _train_epoch_autograd(self, train_data, epoch_idx, loss_func=None):
        """Reference _train_epoch (trainer.py:170-260).  Per-batch losses stay on the
        device and are summed once at the end of the epoch (the reference calls
        .item() per batch, a host sync each).  A NaN batch loss (reference :192-203:
        checked before backward, training stops) is caught on the device by the NaN
        gate: from that batch on no optimizer or mirror-gradient launch changes a
        parameter, and the epoch-end read reports the batch index.  Without the rsx
        optimizer the loss is checked on the host after every batch, as the reference."""
        loss_func = loss_func or self.model.calculate_loss
        parts = []
        loss_batches = []
        gate = self._gate = self._nan_gate_on()
        if gate:
            self._arm_nan_gate()
        self.reset_graph_step()
        sharded = bool(getattr(self.model, "sharded", False)) and hasattr(self.model, "local_batches")
        if sharded:  # users sharded over the ranks: this rank's own device-sampled batches
            train_data = self.model.local_batches(epoch_idx)
        for batch_idx, interaction in enumerate(train_data):
            losses, loss = self.train_step(interaction, batch_idx, loss_func)
            parts.append(torch.stack(list(losses)) if isinstance(losses, tuple) else loss)
            loss_batches.append(loss)
            # sharded: the host check reads the loss summed over the ranks, so a NaN on any
            # rank stops every rank at the same batch (none is left waiting in a collective)
            chk = self.model.gate_loss(loss).clone() if (sharded and not gate) else loss
            if not gate and self._check_nan(chk):
                self.logger.info(f"Loss is nan at epoch: {epoch_idx}, batch index: {batch_idx}. Exiting.")
                return loss_batches[-1], torch.tensor(0.0)
        if gate:
            h = self._halt.cpu().tolist()  # one read per epoch
            if h[0]:
                b = h[1] - 1
                self.logger.info(f"Loss is nan at epoch: {epoch_idx}, batch index: {b}. Exiting.")
                return loss_batches[b], torch.tensor(0.0)
        if not parts:
            return 0.0, loss_batches
        host = torch.stack(parts).double()
        import torch.distributed as dist

        if sharded and dist.is_available() and dist.is_initialized():  # the job's epoch loss: every rank's batches
            host = host.float().contiguous()
            if dist.get_backend() == "nccl":
                dist.all_reduce(host)
            else:
                h = host.cpu()
                dist.all_reduce(h)
                host = h
            host = host.double()
        host = host.cpu().numpy()  # one sync per epoch
        if np.isnan(host).any():
            self.logger.info(f"Loss is nan at epoch: {epoch_idx}. Exiting.")
            return torch.tensor(float("nan")), torch.tensor(0.0)
        total_loss = tuple(float(x) for x in host.sum(0)) if host.ndim == 2 else float(host.sum())
        return total_loss, loss_batches

    def graph_step_enabled(self, loss_func=None) -> bool:
        from .optim import RsxAdam

        m = self.model
        return (bool(self.config.get("rsx_graph_step", True)) and bool(getattr(m, "supports_graph_step", False))
                and not self.fused and not self.mg and isinstance(self.optimizer, RsxAdam)
                and (loss_func is None or loss_func == m.calculate_loss) and torch.cuda.is_available())

    def reset_graph_step(self):
        """Drop the captured steps at an epoch start (pre_epoch_processing may have
        rebuilt buffers the graphs point at), unless the model declares its buffers
        stable across epochs (`graph_step_persistent`); the learning rate lives on the
        device (_sync_lr), so the LambdaLR schedule needs no new capture."""
        if getattr(self.model, "graph_step_persistent", False) and getattr(self, "_lr_dev", None) is not None \
                and getattr(self.optimizer, "lr_on_device", lambda: False)():
            return
        self._graph = None

    def _sync_lr(self):
        """The learning rate as a device f64 scalar that the captured Adam, alpha and
        axpy launches read (refreshed outside any capture, when the schedule moves it)."""
        lr = float(self.optimizer.param_groups[0]["lr"])
        if getattr(self, "_lr_dev", None) is None:
            self._lr_dev = torch.tensor([lr], dtype=torch.float64, device=self.device)
            self._lr_host = lr
            self.optimizer.lr_dev = self._lr_dev
        elif lr != self._lr_host:
            self._lr_dev.fill_(lr)
            self._lr_host = lr

    def train_step(self, interaction, batch_idx, loss_func=None):
        """One batch: replayed from a captured graph when possible (see _GraphStep),
        else `_train_batch`.  Returns (losses, loss), detached."""
        loss_func = loss_func or self.model.calculate_loss
        if self.graph_step_enabled(loss_func):
            self._sync_lr()
            if self._graph is None:
                self._graph = _GraphStep(self, loss_func)
            out = self._graph.step(interaction)
            if out is not None:
                return out
        losses, loss = self._train_batch(interaction, batch_idx, loss_func)
        # detached: a caller holding an eager batch's autograd graph keeps its
        # AccumulateGrad nodes (bound to the eager stream) alive into the next
        # capture, whose backward would then wait on a stream outside the graph
        if isinstance(losses, tuple):
            return tuple(x.detach() for x in losses), loss.detach()
        loss = loss.detach()
        return loss, loss

    def _train_batch(self, interaction, batch_idx, loss_func):
        """One training batch exactly as the reference's loop body: loss, backward,
        optimizer step, and the trainer-level (alpha1/alpha2) or model-level mirror
        gradient.  Returns (losses as returned by calculate_loss, summed loss)."""
        self._zero_grad()
        second = interaction.clone() if hasattr(interaction, "clone") else interaction
        losses = loss_func(interaction)
        loss = sum(losses) if isinstance(losses, tuple) else losses
        if getattr(self, "_gate", False):
            from .smore_fuse import nan_gate

            gl = self.model.gate_loss(loss) if hasattr(self.model, "gate_loss") else loss
            nan_gate(gl, self._halt, self._nan_ctr)
        if not getattr(self.model, "mg_enable", False):
            if self.mg and batch_idx % self.beta == 0:
                (self.alpha1 * loss).backward()
                self.optimizer.step()
                self.optimizer.zero_grad()
                l2 = loss_func(second)
                loss = sum(l2) if isinstance(l2, tuple) else l2
                (-1 * self.alpha2 * loss).backward()
            else:
                loss.backward()
            if self.clip_grad_norm:
                clip_grad_norm_(self.model.parameters(), **self.clip_grad_norm)
            self.optimizer.step()
            return losses, loss
        self._backward(loss)
        if self.clip_grad_norm:
            clip_grad_norm_(self.model.parameters(), **self.clip_grad_norm)
        self.optimizer.step()
        self._mirror_gradient(loss_func, second)
        return losses, loss

    def _backward(self, loss):
        """loss.backward() with a cached ones seed for a scalar loss on the device: autograd's
        own seed is a fill launch per backward (three a mirror-gradient step), and the
        captured step replays every launch."""
        if not (torch.is_tensor(loss) and loss.is_cuda and loss.dim() == 0):
            loss.backward()
            return
        key = (loss.device, loss.dtype)
        seeds = self.__dict__.setdefault("_seeds", {})
        one = seeds.get(key)
        if one is None:
            if _capturing():  # a fill launched inside the capture would be replayed every step
                loss.backward()
                return
            one = seeds[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
        loss.backward(one)

    def _zero_grad(self):
        try:
            self.optimizer.zero_grad(set_to_none=True)
        except TypeError:
            self.optimizer.zero_grad()
            self._grads_zeroed_in_place = True

    def _mg_fused(self) -> bool:
        """Mirror-gradient bookkeeping on the fused kernels (rsx_mg_alpha / rsx_axpy_multi):
        f32 CUDA parameters and an optimizer whose zero_grad drops the tensors."""
        from .optim import RsxAdam

        if getattr(self, "_grads_zeroed_in_place", False) or not isinstance(self.optimizer, RsxAdam):
            return False
        ps = [p for p in self.model.parameters() if p.requires_grad]
        return bool(ps) and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in ps)

    def _mirror_gradient(self, loss_func, inter):
        """Model-level mirror gradient (reference trainer.py:268-348)."""
        m = self.model
        interval = int(getattr(m, "mg_interval", 0))
        log_every = int(getattr(m, "mg_log_interval", 50))
        step_id = int(getattr(m, "global_step", 0))
        if log_every > 0 and step_id and step_id % log_every == 0 and hasattr(m, "log_mm_diagnostics"):
            try:
                m.log_mm_diagnostics(self.optimizer)
            except Exception as err:  # noqa: BLE001
                self.logger.warning(f"log_mm_diagnostics failed at step {step_id}: {err}")
        if interval <= 0 or step_id % interval != 0:
            self._mg_last = None
            return
        lr = self.optimizer.param_groups[0].get("lr", 1.0)
        self._zero_grad()
        cur = loss_func(inter)
        self._backward(sum(cur) if isinstance(cur, tuple) else cur)
        fused = self._mg_fused()
        params, grads = [], []
        for p in m.parameters():
            if p.requires_grad and p.grad is not None:
                params.append(p)
                # the fused path keeps the gradient tensors themselves: _zero_grad sets
                # .grad to None (it never zeroes them in place), so they stay g(theta)
                grads.append(p.grad.detach() if fused else p.grad.detach().clone())
        base = float(getattr(m, "mg_alpha", 0.5))
        sharded_m = bool(getattr(m, "sharded", False)) and hasattr(m, "mg_alpha_global")
        with torch.no_grad():
            if fused and params:
                from .smore_fuse import axpy_multi, mg_alpha

                lr_dev = getattr(self, "_lr_dev", None)  # graph-step runs: lr read on the device
                if sharded_m:  # over the global vector
                    alpha = m.mg_alpha_global(params, grads, base, lr, self.mg_target_rel_step,
                                              self.mg_alpha_max_scale, lr_dev)
                else:
                    alpha = mg_alpha(params, grads, base, lr, self.mg_target_rel_step, self.mg_alpha_max_scale,
                                     lr_dev)
                m._alpha_eff = alpha
                halt = self._halt if getattr(self, "_gate", False) else None
                axpy_multi(params, grads, alpha, -1.0 if lr_dev is not None else -lr, lr_dev, halt)  # theta - alpha lr g
            else:
                if sharded_m:  # every rank the same alpha (the replicated parameters stay equal)
                    alpha = m.mg_alpha_global(params, grads, base, lr, self.mg_target_rel_step,
                                              self.mg_alpha_max_scale)
                else:
                    alpha = _mg_alpha(params, grads, base, lr, self.mg_target_rel_step, self.mg_alpha_max_scale)
                m._alpha_eff = alpha
                if params:
                    down = (alpha * -lr).float()  # -alpha * lr, rounded to f32 as the scalar of a f32 op
                    torch._foreach_add_(params, torch._foreach_mul(grads, down))
        self._zero_grad()
        mir = loss_func(inter)
        mirror = sum(mir) if isinstance(mir, tuple) else mir
        self._backward(mirror)
        with torch.no_grad():
            beta = float(getattr(m, "mg_beta", 0.2))
            live = [p.grad for p in m.parameters() if p.requires_grad and p.grad is not None]
            if fused:  # folded into the Adam launch below (g * -beta, the same f32 product)
                self.optimizer.grad_scale = -beta
            elif live:
                torch._foreach_mul_(live, -beta)
            if params:
                if fused:  # restore theta, folded into the Adam launch below (rsx_adam_multi_mg)
                    self.optimizer.restore = (params, grads, alpha, 1.0 if lr_dev is not None else lr, lr_dev, halt)
                else:
                    torch._foreach_add_(params, torch._foreach_mul(grads, (alpha * lr).float()))
        self.optimizer.step()
        self._zero_grad()
        self._mg_last = (step_id, mirror.detach(), alpha)
        if getattr(m, "mg_verbose", False) and not _capturing():
            _mg_print(step_id, mirror, alpha)

    # ------------------------------------------------------------------- fit
    def _valid_epoch(self, valid_data):
        res = self.evaluate(valid_data)
        score = res[self.valid_metric] if self.valid_metric else res["NDCG@20"]
        return score, res

    def _generate_train_loss_output(self, epoch_idx, s_time, e_time, losses):
        out = "epoch %d training [time: %.2fs, " % (epoch_idx, e_time - s_time)
        if isinstance(losses, tuple):
            out = ", ".join("train_loss%d: %.4f" % (i + 1, x) for i, x in enumerate(losses))
        else:
            out += "train loss: %.4f" % losses
        return out + "]"

    def fit(self, train_data, valid_data=None, test_data=None, saved=False, verbose=True):
        for epoch_idx in range(self.start_epoch, self.epochs):
            t0 = time()
            self.model.cur_epoch = epoch_idx
            self.model.pre_epoch_processing()
            train_loss, _ = self._train_epoch(train_data, epoch_idx)
            if torch.is_tensor(train_loss):
                break
            if self.lr_scheduler is not None:
                self.lr_scheduler.step()
            self._epoch_for_lr += 1
            self.train_loss_dict[epoch_idx] = sum(train_loss) if isinstance(train_loss, tuple) else train_loss
            t1 = time()
            msg = self._generate_train_loss_output(epoch_idx, t0, t1, train_loss)
            post = self.model.post_epoch_processing()
            if verbose:
                self.logger.info(msg)
                if post is not None:
                    self.logger.info(post)
            if (epoch_idx + 1) % self.eval_step == 0:
                v0 = time()
                score, vres = self._valid_epoch(valid_data)
                self.best_valid_score, self.cur_step, stop, update = early_stopping(
                    score, self.best_valid_score, self.cur_step, max_step=self.stopping_step,
                    bigger=self.valid_metric_bigger)
                v1 = time()
                _, tres = self._valid_epoch(test_data)
                if verbose:
                    self.logger.info("epoch %d evaluating [time: %.2fs, valid_score: %f]" % (epoch_idx, v1 - v0, score))
                    self.logger.info("valid result: \n" + dict2str(vres))
                    self.logger.info("test result: \n" + dict2str(tres))
                if update:
                    if verbose:
                        self.logger.info("██ " + str(self.config["model"]) + "--Best validation results updated!!!")
                    self.best_valid_result = vres
                    self.best_test_upon_valid = tres
                if stop:
                    if verbose:
                        self.logger.info("+++++Finished training, best eval result in epoch %d" %
                                         (epoch_idx - self.cur_step * self.eval_step))
                    break
        return self.best_valid_score, self.best_valid_result, self.best_test_upon_valid

    # -------------------------------------------------------------- evaluate
    @torch.no_grad()
    def evaluate(self, eval_data, is_test=False, idx=0):
        self.model.eval()
        k = max(self.config["topk"])
        mats = []
        if getattr(self.model, "sharded", False):
            # each rank ranks its own evaluation users; the metric sums are all-gathered
            pos, topk = self.model.full_sort_topk_local(eval_data.eval_u, k, eval_data)
            return self.evaluator.evaluate_sharded(pos, topk, eval_data)
        fused = hasattr(self.model, "full_sort_topk") and hasattr(eval_data, "mask_rowptr")
        if fused:
            # one fused launch over every evaluation user: the score matrix is never
            # materialised, so the reference's eval_batch_size memory bound does not apply
            _, topk = self.model.full_sort_topk([eval_data.eval_u, None], k, eval_data)
            mats.append(topk)
        else:
            for batch in eval_data:
                scores = self.model.full_sort_predict(batch)
                m = batch[1]
                scores[m[0], m[1]] = -1e10
                _, topk = torch.topk(scores, k, dim=-1)
                mats.append(topk)
        return self.evaluator.evaluate(mats, eval_data, is_test=is_test, idx=idx)
