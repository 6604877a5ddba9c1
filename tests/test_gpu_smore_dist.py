"""SMORE with users sharded over 2 / 4 ranks sharing the test box's GPU (rsx.smore in
sharded mode: rsx.smore_dist with the HIP backend; collectives over gloo — the
driver's multi-GPU runs use RCCL) against the single-process rsx SMORE on the
golden fixture (itself pinned to the reference's first step, tests/test_gpu_smore.py),
on the objective the sharded run optimises: the sum over ranks of the reference loss
of each rank's own batch.

* one batch: every rank's loss, every gradient (own user rows; with the item side
  sharded, own rows of the raw feature tables; the replicated parameters equal on every
  rank) within 1e-4 of scale, against the single-process rsx SMORE AND directly against
  the oracle (oracle/rsx_oracle.py:SMORECPU, the reference's restatement) on the sum of
  the rank batches;
* the sharded evaluation (each rank ranks its own users; metric sums all-gathered)
  equal to the single-process evaluation of the same weights;
* one epoch through rsx.trainer.Trainer (device-sampled rank batches, the model-level
  mirror gradient, RsxAdam, the NaN gate) against the single-process Trainer fed the
  same rank batches: losses 1e-4 relative, parameters within 2e-4, replicas equal."""
import os
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import init_pg, store_path

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def _models(root, rank, fx, item_shard=True, scheme="usershard"):
    """(config, train, valid, sharded model, single-process model), both from the
    reference's initial weights (init_seed before each)."""
    import test_gpu_smore as T

    z, c, train, valid, test = T._setup(Path(root) / f"r{rank}", _golden, fx)
    c["rsx_sampler"] = "device"  # the sharded model samples its own users on the device
    c["rsx_knn"] = "host"  # the kNN graphs of the fixture tests (tests/test_gpu_smore.py)
    c["rsx_smore_item_shard"] = item_shard
    c["rsx_smore_scheme"] = scheme
    sm = T._model(c, train)
    assert sm.sharded and sm.scheme == scheme
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
    if sm.scheme == "usershard":  # local user row ids ("dp" batches carry global ids)
        g[0] += sm.user_range[0]
    pad = torch.zeros(3, mx, dtype=torch.int64)
    pad[:, : g.shape[1]] = g
    parts = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(parts, pad)
    return [p[:, : int(s.item())].to(inter.device) for p, s in zip(parts, sizes)]


def _own_rows(sm, n, t):
    """The rows of a (full-table) tensor `t` that rank's parameter `n` holds."""
    if sm.scheme == "dp":  # every table replicated
        return t
    if n == "user_embedding.weight":
        a, b = sm.user_range
        return t[a:b]
    if sm._shard.item_shard and n in ("image_embedding.weight", "text_embedding.weight"):
        a, b = sm._shard.own_i
        return t[a:b]
    return t


def _sharded_param(sm, n):
    if sm.scheme == "dp":
        return False
    return n == "user_embedding.weight" or (sm._shard.item_shard and n in ("image_embedding.weight",
                                                                            "text_embedding.weight"))


def _oracle_grads(z, c, batches):
    """The oracle's SMORE (the reference restated on the CPU) on the same fixture weights:
    the per-batch losses and the gradients of their sum."""
    import rsx_oracle as O

    init = {k[5:]: z[k] for k in z if k.startswith("init.")}
    m = O.SMORECPU(z["train_u"], z["train_i"], int(z["n_users"]), int(z["n_items"]), z["v_feat"], z["t_feat"],
                   d=int(c["embedding_size"]), image_k=int(c["image_knn_k"]), text_k=int(c["text_knn_k"]),
                   dropout=0.0, batch_size=int(c["train_batch_size"]), init=init)
    losses = [m.calculate_loss(b.cpu()) for b in batches]
    sum(losses).backward()
    return [x.item() for x in losses], {n: p.grad.detach() for n, p in m.named_parameters()}


def _worker(rank, world, store, root, out, fx, item_shard=True, scheme="usershard"):
    init_pg("gloo", rank, world, store)
    from rsx.evaluator import TopKEvaluator

    z, c, train, valid, sm, ref = _models(root, rank, fx, item_shard, scheme)
    if scheme == "usershard":
        assert sm._shard.item_shard == item_shard
    sm.train()
    ref.train()
    inter = next(iter(sm.local_batches(0)))
    loss = sm.calculate_loss(inter)
    loss.backward()
    batches = _global_batch(sm, inter)
    rl = [ref.calculate_loss(b) for b in batches]
    sum(rl).backward()
    ol, og = _oracle_grads(z, c, batches)
    err, oerr = {}, {}
    refp = dict(ref.named_parameters())
    assert set(refp) == set(n for n, _ in sm.named_parameters())
    for n, p in sm.named_parameters():
        g = _own_rows(sm, n, refp[n].grad.detach())
        scale = max(g.abs().max().item(), 1e-12)
        err[n] = (p.grad - g).abs().max().item() / scale
        go = _own_rows(sm, n, og[n]).to(p.device)
        oerr[n] = (p.grad - go).abs().max().item() / max(go.abs().max().item(), 1e-12)
    grads = {n: p.grad.detach().cpu().numpy() for n, p in sm.named_parameters() if not _sharded_param(sm, n)}
    # sharded evaluation of the initial weights vs the single-process evaluation
    sm.eval()
    ref.eval()
    k = max(c["topk"])
    ev = TopKEvaluator(c)
    pos, topk = sm.full_sort_topk_local(valid.eval_u, k, valid)
    got = ev.evaluate_sharded(pos, topk, valid)
    _, full = ref.full_sort_topk([valid.eval_u, None], k, valid)
    want = ev.evaluate_device(full, valid)
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=loss.item(), ref=rl[rank].item(), oracle=ol[rank],
             names=np.array(list(err)), errs=np.array(list(err.values())), oerrs=np.array(list(oerr.values())),
             keys=np.array(sorted(got)), got=np.array([got[x] for x in sorted(got)]),
             want=np.array([want[x] for x in sorted(got)]), **{"g." + n: v for n, v in grads.items()})
    dist.destroy_process_group()


def _spawn(fn, world, *args):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out")
        os.makedirs(out)
        mp.spawn(fn, args=(world, store_path(), d, out) + args, nprocs=world, join=True)
        return [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("fx,world,item_shard,scheme", [
    ("smore_small", 2, True, "usershard"), ("smore_d128_small", 2, True, "usershard"),
    ("smore_small", 4, True, "usershard"), ("smore_d128_small", 4, True, "usershard"),
    ("smore_small", 2, False, "usershard"),
    ("smore_small", 2, True, "dp"), ("smore_d128_small", 2, True, "dp"), ("smore_small", 4, True, "dp"),
    ("smore_d128_small", 4, True, "dp"), ("smore_small", 3, True, "dp")])
def test_sharded_smore_hip_matches_single_process(cuda, fx, world, item_shard, scheme):
    """usershard: users row-sharded, the item partials all-reduced per UI layer; dp: every
    table replicated, the batch-row gradients exchanged once (RowGradExchange)."""
    res = _spawn(_worker, world, fx, item_shard, scheme)
    for x in res:
        assert abs(float(x["loss"]) - float(x["ref"])) <= 2e-5 * abs(float(x["ref"]))
        assert abs(float(x["loss"]) - float(x["oracle"])) <= 2e-5 * abs(float(x["oracle"]))
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 1e-4}
        assert not bad, bad
        bad = {n: e for n, e in zip(x["names"], x["oerrs"]) if not e <= 1e-4}
        assert not bad, ("vs oracle", bad)
        assert np.array_equal(x["got"], res[0]["got"])
        assert np.abs(x["got"] - x["want"]).max() <= 1e-4
        for n in x:  # replicated gradients are bit-identical on every rank
            if n.startswith("g."):
                assert np.array_equal(x[n], res[0][n]), n


def _trainer_worker(rank, world, store, root, out, fx, scheme="usershard"):
    init_pg("gloo", rank, world, store)
    from rsx.trainer import Trainer

    z, c, train, valid, sm, ref = _models(root, rank, fx, scheme=scheme)
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
    refp = dict(ref.named_parameters())
    err = {}
    for n, p in sm.named_parameters():
        want = _own_rows(sm, n, refp[n].detach())
        err[n] = (p.detach() - want).abs().max().item()
    items = {n: p.detach().cpu().numpy() for n, p in sm.named_parameters() if not _sharded_param(sm, n)}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=float(loss_s), ref=float(loss_r), steps=len(steps),
             gstep=sm.global_step, rstep=ref.global_step, names=np.array(list(err)), errs=np.array(list(err.values())),
             **{"p." + n: v for n, v in items.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("scheme", ["usershard", "dp"])
def test_sharded_smore_trainer_epoch_matches_single_process(cuda, scheme):
    """gloo world 4 through rsx.trainer.Trainer: one epoch of the sharded SMORE (each rank
    its own device-sampled batches, the mirror gradient with the global alpha) equals the
    single-process Trainer on the joint objective of the same batches."""
    world = 4
    res = _spawn(_trainer_worker, world, "smore_small", scheme)
    for x in res:
        assert int(x["steps"]) >= 2 and int(x["gstep"]) == int(x["rstep"])
        assert abs(float(x["loss"]) - float(x["ref"])) <= 1e-4 * abs(float(x["ref"]))
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 2e-4}
        assert not bad, bad
        for n in x:
            if n.startswith("p."):
                assert np.array_equal(x[n], res[0][n]), n  # the replicas stay identical
