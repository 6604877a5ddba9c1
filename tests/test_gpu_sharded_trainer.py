"""The user-sharded LightGCN through the reference's training flow (rsx.lightgcn's
sharded mode + rsx.trainer's sharded epoch and evaluation): 2 ranks sharing the
test box's GPU, collectives over gloo (the driver's 8-GPU run uses RCCL).

Checks: every rank reports the same metric dict; that dict equals a single-process
evaluation (fused full-sort + the device metric tail) of the same final
embeddings gathered from the ranks — the sharded evaluation (per-rank top-k of the
rank's users, all-gathered metric sums) loses nothing; item replicas stay equal;
losses are finite and every rank ran the same number of steps."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import init_pg, store_path

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _setup(root, **extra):
    from rsx.config import Config
    from rsx.data import EvalDataLoader, RecDataset, TrainDataLoader

    cfg = dict(data_path=root + "/", train_batch_size=256, eval_batch_size=256, is_multimodal_model=False,
               n_layers=[3], reg_weight=[1e-2], rsx_dist_backend="gloo")
    cfg.update(extra)
    c = Config("LightGCN", "baby", cfg)
    for k in c["hyper_parameters"]:
        if isinstance(c[k], list):
            c[k] = c[k][0]
    ds = RecDataset(c)
    tr, va, te = ds.split()
    for x in (ds, tr, va, te):
        str(x)
    train = TrainDataLoader(c, tr, batch_size=256, shuffle=True)
    valid = EvalDataLoader(c, va, additional_dataset=tr, batch_size=256)
    return c, train, valid


def _worker(rank, world, store, root, out):
    init_pg("gloo", rank, world, store)
    from rsx.lightgcn import LightGCN
    from rsx.trainer import Trainer
    from rsx.utils import init_seed

    c, train, valid = _setup(root)
    init_seed(c["seed"])
    train.pretrain_setup()
    m = LightGCN(c, train)
    assert m.sharded
    t = Trainer(c, m)
    assert t.fused
    # every rank visits each of its interactions exactly once per epoch in the common
    # step count (no wrap-around re-training of a small shard's batches)
    E, Bm = m.engine.n_inter, m.engine.batch
    assert (m.steps_per_epoch - 1) * Bm < E <= m.steps_per_epoch * Bm
    seen = []
    step0 = m.engine.step

    def spy(triplets=None, epoch=0, start=0):
        seen.append(triplets[:2].cpu().numpy().copy())
        return step0(triplets=triplets, epoch=epoch, start=start)

    m.engine.step = spy
    losses = []
    inter = np.stack([m.engine.sampler.inter_u.cpu().numpy(), m.engine.sampler.inter_i.cpu().numpy()])
    for epoch in range(2):
        seen.clear()
        loss, n = t._train_epoch(train, epoch)
        assert not torch.is_tensor(loss) and n == m.steps_per_epoch
        losses.append(loss)
        t._epoch_for_lr += 1
        # the common step count, balanced slices (sizes within one), each interaction once
        sizes = [x.shape[1] for x in seen]
        assert len(seen) == m.steps_per_epoch and max(sizes) - min(sizes) <= 1 and max(sizes) <= Bm
        got = np.concatenate(seen, axis=1)
        assert sorted(map(tuple, got.T.tolist())) == sorted(map(tuple, inter.T.tolist()))
    vres = t.evaluate(valid)
    f = m._final().cpu()
    a, b = m.user_range
    np.savez(os.path.join(out, f"r{rank}.npz"), users=f[: b - a].numpy(), items=f[b - a:].numpy(),
             rng=np.array([a, b]), losses=np.array(losses), keys=np.array(sorted(vres)),
             vals=np.array([vres[k] for k in sorted(vres)]), steps=np.array([m.steps_per_epoch]))
    dist.barrier()
    dist.destroy_process_group()



def test_sharded_trainer_fit_and_evaluate(cuda):
    from rsx import ops
    from rsx.evaluator import TopKEvaluator

    world = 2
    with tempfile.TemporaryDirectory() as root:
        os.makedirs(os.path.join(root, "baby"))
        shutil.copy(os.path.join(GOLD, "gold_small.inter"), os.path.join(root, "baby", "baby.inter"))
        out = os.path.join(root, "out")
        os.makedirs(out)
        mp.spawn(_worker, args=(world, store_path(), root, out), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
        c, _, valid = _setup(root)
    for r in range(1, world):
        assert np.array_equal(res[0]["items"], res[r]["items"])
        assert np.array_equal(res[0]["vals"], res[r]["vals"]) and list(res[0]["keys"]) == list(res[r]["keys"])
        assert res[0]["steps"][0] == res[r]["steps"][0]
    assert all(np.isfinite(x["losses"]).all() for x in res)
    assert res[0]["rng"][0] == 0 and res[-1]["rng"][1] == sum(x["users"].shape[0] for x in res)
    # single-process evaluation of the gathered final embeddings
    U = torch.from_numpy(np.concatenate([x["users"] for x in res])).to(cuda)
    I = torch.from_numpy(res[0]["items"]).to(cuda)
    k = max(c["topk"])
    _, topk = ops.fullsort_topk(U, valid.eval_u, I, valid.mask_rowptr, valid.mask_col, k)
    want = TopKEvaluator(c).evaluate_device(topk, valid)
    got = dict(zip(res[0]["keys"], res[0]["vals"]))
    assert set(got) == set(want)
    for key in want:
        assert abs(got[key] - want[key]) <= 1e-4 + 1e-12, (key, got[key], want[key])
    # typically identical: the rank-ordered sums differ from user-ordered ones only at a rounding near-tie
    assert sum(got[key] != want[key] for key in want) <= 1
