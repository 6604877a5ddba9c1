"""SMORE with users sharded over 2 / 4 ranks sharing the test box's GPU (rsx.smore in
sharded mode: rsx.smore_dist with the HIP backend; collectives over gloo — the
driver's multi-GPU runs use RCCL) against the single-process rsx SMORE on the
golden fixture (itself pinned to the reference's first step, tests/test_gpu_smore.py),
on the objective the sharded run optimises: the sum over ranks of the reference loss
of each rank's own batch.

* one batch: every rank's loss, every gradient (own user rows; the replicated item
  side equal on every rank) within 1e-4 of scale;
* the sharded evaluation (each rank ranks its own users; metric sums all-gathered)
  equal to the single-process evaluation of the same weights;
* one epoch through rsx.trainer.Trainer (device-sampled rank batches, the model-level
  mirror gradient, RsxAdam, the NaN gate) against the single-process Trainer fed the
  same rank batches: losses 1e-4 relative, parameters within 2e-4, replicas equal."""
import os
import socket
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def _models(root, rank, fx):
    """(config, train, valid, sharded model, single-process model), both from the
    reference's initial weights (init_seed before each)."""
    import test_gpu_smore as T

    z, c, train, valid, test = T._setup(Path(root) / f"r{rank}", _golden, fx)
    c["rsx_sampler"] = "device"  # the sharded model samples its own users on the device
    c["rsx_knn"] = "host"  # the kNN graphs of the fixture tests (tests/test_gpu_smore.py)
    sm = T._model(c, train)
    assert sm.sharded
    c["rsx_sharded"] = False
    ref = T._model(c, train)
    c["rsx_sharded"] = None
    assert not ref.sharded
    return z, c, train, valid, sm, ref


def _global_batch(sm, inter):
    """Every rank's batch with global user ids (all-gathered; rank order)."""
    B = torch.tensor([inter.shape[1]], dtype=torch.int64)
    sizes = [torch.zeros_like(B) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, B)
    mx = int(max(s.item() for s in sizes))
    g = inter.cpu().clone()
    g[0] += sm.user_range[0]
    pad = torch.zeros(3, mx, dtype=torch.int64)
    pad[:, : g.shape[1]] = g
    parts = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(parts, pad)
    return [p[:, : int(s.item())].to(inter.device) for p, s in zip(parts, sizes)]


def _worker(rank, world, port, root, out, fx):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.evaluator import TopKEvaluator

    z, c, train, valid, sm, ref = _models(root, rank, fx)
    sm.train()
    ref.train()
    inter = next(iter(sm.local_batches(0)))
    loss = sm.calculate_loss(inter)
    loss.backward()
    batches = _global_batch(sm, inter)
    rl = [ref.calculate_loss(b) for b in batches]
    sum(rl).backward()
    a, b = sm.user_range
    err = {}
    refp = dict(ref.named_parameters())
    assert set(refp) == set(n for n, _ in sm.named_parameters())
    for n, p in sm.named_parameters():
        g = refp[n].grad.detach()
        if n == "user_embedding.weight":
            g = g[a:b]
        scale = max(g.abs().max().item(), 1e-12)
        err[n] = (p.grad - g).abs().max().item() / scale
    grads = {n: p.grad.detach().cpu().numpy() for n, p in sm.named_parameters() if n != "user_embedding.weight"}
    # sharded evaluation of the initial weights vs the single-process evaluation
    sm.eval()
    ref.eval()
    k = max(c["topk"])
    ev = TopKEvaluator(c)
    pos, topk = sm.full_sort_topk_local(valid.eval_u, k, valid)
    got = ev.evaluate_sharded(pos, topk, valid)
    _, full = ref.full_sort_topk([valid.eval_u, None], k, valid)
    want = ev.evaluate_device(full, valid)
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=loss.item(), ref=rl[rank].item(),
             names=np.array(list(err)), errs=np.array(list(err.values())),
             keys=np.array(sorted(got)), got=np.array([got[x] for x in sorted(got)]),
             want=np.array([want[x] for x in sorted(got)]), **{"g." + n: v for n, v in grads.items()})
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out")
        os.makedirs(out)
        mp.spawn(fn, args=(world, _free_port(), d, out) + args, nprocs=world, join=True)
        return [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("fx,world", [("smore_small", 2), ("smore_d128_small", 2), ("smore_small", 4)])
def test_sharded_smore_hip_matches_single_process(cuda, fx, world):
    res = _spawn(_worker, world, fx)
    for x in res:
        assert abs(float(x["loss"]) - float(x["ref"])) <= 2e-5 * abs(float(x["ref"]))
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 1e-4}
        assert not bad, bad
        assert np.array_equal(x["got"], res[0]["got"])
        assert np.abs(x["got"] - x["want"]).max() <= 1e-4
        for n in x:  # replicated gradients are bit-identical on every rank
            if n.startswith("g."):
                assert np.array_equal(x[n], res[0][n]), n


def _trainer_worker(rank, world, port, root, out, fx):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.trainer import Trainer

    z, c, train, valid, sm, ref = _models(root, rank, fx)
    ts, tr = Trainer(c, sm), Trainer(c, ref)
    assert sm.mg_enable and not ts.fused and not sm.supports_graph_step  # gloo: eager steps
    # the rank batches of epoch 0, gathered: the single-process run trains step j on sum_g L(batch_g,j)
    steps = [_global_batch(sm, b.clone()) for b in sm.local_batches(0)]
    sm.pre_epoch_processing()
    loss_s, _ = ts._train_epoch(train, 0)

    def joint(batches):
        out = sum(ref.calculate_loss(b) for b in batches)
        ref.global_step -= len(batches) - 1  # one step per joint batch, as each rank's model counts
        return out

    ref.pre_epoch_processing()
    loss_r, _ = tr._train_epoch(steps, 0, loss_func=joint)
    a, b = sm.user_range
    refp = dict(ref.named_parameters())
    err = {}
    for n, p in sm.named_parameters():
        want = refp[n].detach()
        if n == "user_embedding.weight":
            want = want[a:b]
        err[n] = (p.detach() - want).abs().max().item()
    items = {n: p.detach().cpu().numpy() for n, p in sm.named_parameters() if n != "user_embedding.weight"}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=float(loss_s), ref=float(loss_r), steps=len(steps),
             gstep=sm.global_step, rstep=ref.global_step, names=np.array(list(err)), errs=np.array(list(err.values())),
             **{"p." + n: v for n, v in items.items()})
    dist.destroy_process_group()


def test_sharded_smore_trainer_epoch_matches_single_process(cuda):
    """gloo world 4 through rsx.trainer.Trainer: one epoch of the sharded SMORE (each rank
    its own device-sampled batches, the mirror gradient with the global alpha) equals the
    single-process Trainer on the joint objective of the same batches."""
    world = 4
    res = _spawn(_trainer_worker, world, "smore_small")
    for x in res:
        assert int(x["steps"]) >= 2 and int(x["gstep"]) == int(x["rstep"])
        assert abs(float(x["loss"]) - float(x["ref"])) <= 1e-4 * abs(float(x["ref"]))
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 2e-4}
        assert not bad, bad
        for n in x:
            if n.startswith("p."):
                assert np.array_equal(x[n], res[0][n]), n  # the replicas stay identical
