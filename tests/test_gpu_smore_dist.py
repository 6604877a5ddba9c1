"""SMORE sharded over 2 ranks sharing the test box's GPU (rsx.smore_dist with the HIP
backend; collectives over gloo — the driver's multi-GPU runs use RCCL) against the
single-process rsx SMORE on the golden fixture (itself pinned to the reference's
first step, tests/test_gpu_smore.py): the loss, every parameter's gradient (sharded
rows gathered) within 1e-4 of scale, and the sharded full-sort evaluation (each rank
ranks its own users; metric sums all-gathered) equal to the single-process dict."""
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


def _worker(rank, world, port, root, out, fx):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import test_gpu_smore as T
    from rsx.evaluator import TopKEvaluator, sharded_metric_dict
    from rsx.smore_dist import HipSmoreBackend, ShardedSMORE, graphs_from_rsx

    z, c, train, valid, test = T._setup(Path(root) / f"r{rank}", _golden, fx)
    m = T._model(c, train)  # the single-process model: reference initial weights and graphs
    m.train()
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).cuda()
    params = {n: p.detach().clone() for n, p in m.named_parameters()}
    cfg = dict(reg_weight=c["reg_weight"], batch_size=c["train_batch_size"], n_ui_layers=c["n_ui_layers"],
               n_layers=c["n_layers"], cl_loss=c["cl_loss"], cl_temp=m.cl_temp, dropout_rate=0.0)
    sm = ShardedSMORE(params, graphs_from_rsx(m), m.n_users, m.n_items, cfg, HipSmoreBackend("cuda:0"))
    sm.train()
    loss = sm.calculate_loss(trip)
    loss.backward()
    sm.sync_grads()
    ref = m.calculate_loss(trip)
    ref.backward()
    (ua, ub), (ia, ib) = sm.own_u, sm.own_i
    from rsx.smore_dist import SHARDED

    err = {}
    ref_params = dict(m.named_parameters())
    assert set(ref_params) == set(n for n, _ in sm.named_parameters())
    for n, p in sm.named_parameters():
        g = ref_params[n].grad.detach()
        part = SHARDED.get(n)
        if part == "u":
            g = g[ua:ub]
        elif part == "i":
            g = g[ia:ib]
        scale = max(g.abs().max().item(), 1e-12)
        err[n] = (p.grad - g).abs().max().item() / scale
    # sharded evaluation vs the single-process fused evaluation
    sm.eval()
    m.eval()
    k = max(c["topk"])
    topk = sm.full_sort_topk_local(k, valid.mask_rowptr, valid.mask_col)
    eu = valid.eval_u
    pos = torch.nonzero((eu >= ua) & (eu < ub)).flatten()
    got = sharded_metric_dict(pos, topk.index_select(0, eu.index_select(0, pos) - ua), valid,
                              TopKEvaluator(c).metrics, TopKEvaluator(c).topk)
    _, full = m.full_sort_topk([eu, None], k, valid)
    want = TopKEvaluator(c).evaluate_device(full, valid)
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=loss.item() * world, ref=ref.item(),
             names=np.array(list(err)), errs=np.array(list(err.values())),
             keys=np.array(sorted(got)), got=np.array([got[x] for x in sorted(got)]),
             want=np.array([want[x] for x in sorted(got)]))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("fx", ["smore_small", "smore_d128_small"])
def test_sharded_smore_hip_matches_single_process(cuda, fx):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out")
        os.makedirs(out)
        mp.spawn(_worker, args=(world, _free_port(), d, out, fx), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
    for x in res:
        assert abs(float(x["loss"]) - float(x["ref"])) <= 2e-5 * abs(float(x["ref"]))
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 1e-4}
        assert not bad, bad
        assert np.array_equal(x["got"], res[0]["got"])
        assert np.abs(x["got"] - x["want"]).max() <= 1e-4


def _mg_worker(rank, world, port, root, out, fx):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rsx_oracle as O
    import test_gpu_smore as T
    from rsx.smore_dist import SHARDED, HipSmoreBackend, ShardedSMORE, graphs_from_rsx

    z, c, train, valid, test = T._setup(Path(root) / f"r{rank}", _golden, fx)
    m = T._model(c, train)
    m.train()
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).cuda()
    params = {n: p.detach().clone() for n, p in m.named_parameters()}
    cfg = dict(reg_weight=c["reg_weight"], batch_size=c["train_batch_size"], n_ui_layers=c["n_ui_layers"],
               n_layers=c["n_layers"], cl_loss=c["cl_loss"], cl_temp=m.cl_temp, dropout_rate=0.0)
    sm = ShardedSMORE(params, graphs_from_rsx(m), m.n_users, m.n_items, cfg, HipSmoreBackend("cuda:0"))
    sm.train()
    lr = c["learning_rate"]
    opt = torch.optim.Adam(sm.parameters(), lr=lr)
    losses = [sm.train_batch(trip, opt, lr, s + 1, mg_interval=1, mg_alpha=m.mg_alpha, mg_beta=m.mg_beta)
              for s in range(2)]
    m.mg_interval = 1
    ref_opt = torch.optim.Adam(m.parameters(), lr=lr)
    ref_losses = [O.smore_train_batch(m, ref_opt, trip, lr) for _ in range(2)]
    (ua, ub), (ia, ib) = sm.own_u, sm.own_i
    ref_params = dict(m.named_parameters())
    err = {}
    for n, p in sm.named_parameters():
        want = ref_params[n].detach()
        part = SHARDED.get(n)
        if part == "u":
            want = want[ua:ub]
        elif part == "i":
            want = want[ia:ib]
        err[n] = (p.detach() - want).abs().max().item()
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=np.array(losses) * world, ref=np.array(ref_losses),
             names=np.array(list(err)), errs=np.array(list(err.values())))
    dist.destroy_process_group()


def test_sharded_smore_hip_mirror_gradient(cuda):
    """Two batches with the mirror gradient firing on each (mg_interval 1) on 2 ranks
    with the HIP backend against the single-process rsx SMORE run through the
    oracle's Trainer batch (smore_train_batch): losses, and every parameter's rows
    within 1e-4 (Adam's first steps move each element by about lr)."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out")
        os.makedirs(out)
        mp.spawn(_mg_worker, args=(world, _free_port(), d, out, "smore_small"), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
    for x in res:
        np.testing.assert_allclose(x["loss"], x["ref"], rtol=2e-5)
        bad = {n: e for n, e in zip(x["names"], x["errs"]) if not e <= 1e-4}
        assert not bad, bad
