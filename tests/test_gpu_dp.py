"""Data-parallel LightGCN (rsx.dp, csrc/dp.hip) with the HIP backend.

* 2 and 3 ranks sharing the one GPU of the test box, the step's triplet all-gather through
  the host hook over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is the
  driver's): two steps must equal two reference steps (oracle loss + torch.optim.Adam)
  on the global batch, and every replica must stay bit-identical;
* 1 rank over a real RCCL communicator, eager and graph-captured: the step must equal the
  single-GPU fused step (rsx_lightgcn_step) on the same triplets.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import init_pg, store_path

import rsx_oracle as O
from test_dist_gloo import D, LR, NI, NU, REG, _local_graph

pytestmark = pytest.mark.gpu



def _trip(s, r, hot=False):
    t = _local_graph(10 * s + r)[2][:, : 20 - r].copy()  # unequal rank batches
    if hot:  # one positive item for every triplet and one user for half of them: runs of
        t[1, :] = 0  # equal rows that cross many chunks of the gradient pass
        t[0, ::2] = 0
    return t


def _worker(rank, world, store, out_dir, k, groups="0", hot=False):
    os.environ["RSX_DP_GROUPS"] = groups  # the loss passes' lane-group form (read at the first step)
    init_pg("gloo", rank, world, store)
    from rsx.dp import DataParallelLightGCNEngine

    tu, ti, _ = _local_graph(0)
    torch.manual_seed(7)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    if rank:
        U0, I0 = U0 * 0 + 1, I0 * 0 - 1  # replicas start from rank 0's tables
    eng = DataParallelLightGCNEngine(tu, ti, NU, NI, D, k, REG, LR, "cuda:0", U0, I0, batch=32)
    losses, ps = [], []
    for s in range(2):
        eng.step(torch.from_numpy(_trip(s, rank, hot)).cuda())
        losses.append(float(eng.loss_out.item()))
        ps.append(eng.p.cpu().numpy())
    # the union's G' rows and counts are cleared after the step
    assert torch.count_nonzero(eng.g).item() == 0
    assert torch.count_nonzero(eng.reg_cnt[:-4]).item() == 0
    # and the gradient pass's run state (csrc/dp.hip Work: the int64 accumulators and each
    # row's run start / cursor, carved first, 256-B aligned) is all zero again
    al = lambda x: (x + 255) & ~255  # noqa: E731
    n = NU + NI
    head = al(n * D * 8) + 2 * al(n * 4)
    assert torch.count_nonzero(eng.work[:head]).item() == 0
    # device-sampled epoch: every rank the same number of slices, all finite
    for j in range(eng.steps_per_epoch()):
        eng.step_index(0, j)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), p1=ps[0], p2=ps[1], losses=np.array(losses),
             after=eng.p.cpu().numpy(), f=eng.forward().cpu().numpy())
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,groups,hot", [(2, 3, "1", False), (3, 3, "2", False), (2, 2, "1", False),
                                               (2, 4, "2", False), (2, 3, "2", False), (3, 3, "3", False),
                                               (2, 4, "3", False), (2, 3, "1", True), (3, 3, "2", True),
                                               (2, 3, "3", True)])
def test_dp_hip_step_matches_global_batch(world, k, groups, hot):
    """hot: runs of equal rows across many chunks (the gradient pass's last-segment finish).
    groups: the loss passes' narrow (1: a triplet / 4 run places a lane group, the small
    batch form), wide (2: 4 triplets / 16 places, the large batch form) or middle (3: 2 / 8)
    lane groups."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, store_path(), d, k, groups, hot), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    tu, ti, _ = _local_graph(0)
    A = O.lightgcn_norm_adj_vec(tu, ti, NU, NI)
    torch.manual_seed(7)
    u = torch.nn.Parameter(torch.nn.init.xavier_uniform_(torch.empty(NU, D)))
    i = torch.nn.Parameter(torch.nn.init.xavier_uniform_(torch.empty(NI, D)))
    opt = torch.optim.Adam([u, i], lr=LR)
    ref_losses, ref_p = [], []
    for s in range(2):
        trip = torch.from_numpy(np.concatenate([_trip(s, r, hot) for r in range(world)], 1))
        opt.zero_grad()
        loss = O.lightgcn_loss(u, i, A, k, trip, REG)
        loss.backward()
        opt.step()
        ref_losses.append(loss.item())
        ref_p.append(np.concatenate([u.detach().numpy(), i.detach().numpy()]))
    for r in range(world):
        np.testing.assert_allclose(res[r]["losses"], ref_losses, rtol=1e-5)
        np.testing.assert_allclose(res[r]["p1"], ref_p[0], rtol=0, atol=2e-6)
        np.testing.assert_allclose(res[r]["p2"], ref_p[1], rtol=0, atol=3e-6)
        for key in ("p1", "p2", "after", "f"):  # replicas bit-identical, also after an epoch
            assert np.array_equal(res[0][key], res[r][key]), key
    assert np.isfinite(res[0]["after"]).all()


def _rccl_worker(rank, world, store, out_dir, k, graph="1", hot=False):
    os.environ["RSX_DP_GRAPH"] = graph  # read by the engine's constructor
    torch.cuda.set_device(0)
    init_pg("nccl", rank, world, store, device_id=torch.device("cuda", 0))
    from rsx.dp import DataParallelLightGCNEngine
    from rsx.engine import LightGCNEngine

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lightgcn_small.npz"))
    nu, ni = int(z["n_users"]), int(z["n_items"])
    U0, I0 = z["init.embedding_dict.user_emb"], z["init.embedding_dict.item_emb"]
    dp = DataParallelLightGCNEngine(z["train_u"], z["train_i"], nu, ni, 64, k, 1e-2, 1e-3, "cuda:0", U0, I0,
                                    batch=512)
    one = LightGCNEngine(z["train_u"], z["train_i"], nu, ni, 64, k, 1e-2, 1e-3, "cuda:0", U0, I0, batch=512)
    trips = torch.from_numpy(z["epoch0_triplets"].astype(np.int64)).cuda()
    if hot:  # one positive item for every triplet, one user for half of them: runs of equal
        trips = trips.clone()  # rows crossing many chunks of the solo step's run places
        trips[1, :] = 0
        trips[0, ::2] = trips[0, 0]
    la, lb = [], []
    for s in range(6):  # eager, eager (warm), captured, replayed ...; a partial batch at the end
        t = trips[:, s * 512:(s + 1) * 512] if s < 5 else trips[:, 5 * 512: 5 * 512 + 300]
        dp.step(t)
        one.step(triplets=t)
        la.append(float(dp.loss_out.item()))
        lb.append(float(one.loss_out.item()))
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rccl.npz"), la=np.array(la), lb=np.array(lb), pa=dp.p.cpu().numpy(),
             pb=one.p.cpu().numpy(), ma=dp.m.cpu().numpy(), mb=one.m.cpu().numpy(),
             graphs=np.array(sorted(dp._graphs)))
    dp.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("k,graph,hot", [(3, "1", False), (4, "1", False), (3, "0", False), (3, "0", True),
                                         (4, "1", True)])
def test_dp_one_rank_rccl_equals_single_gpu_step(k, graph, hot):
    """World 1 over RCCL, graph-captured (RSX_DP_GRAPH=1) or issued eagerly (the default):
    the same arithmetic as the single-GPU stored-layer step (only the BPR scatter's float
    atomics order differently run to run).  hot: the eager one-rank step is the solo path
    (the loss pass takes the run places, csrc/dp.hip) and meets runs of equal rows that
    cross chunk boundaries."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(1, store_path(), d, k, graph, hot), nprocs=1, join=True)
        z = dict(np.load(os.path.join(d, "rccl.npz")))
    np.testing.assert_allclose(z["la"], z["lb"], rtol=1e-6)
    np.testing.assert_allclose(z["pa"], z["pb"], rtol=0, atol=1e-6)
    # hot rows sum ~1,000 float atomics in the single-GPU step: its moments carry their order
    np.testing.assert_allclose(z["ma"], z["mb"], rtol=0, atol=1e-6 if hot else 1e-7)
    if graph == "1":
        assert 512 in z["graphs"].tolist()  # full batches replayed from a captured graph
    else:
        assert z["graphs"].size == 0


def _trainer_worker(rank, world, store, root, out):
    """LightGCN with config rsx_dist: dp through the reference's training flow (rsx.trainer
    fused epochs + sharded evaluation), two ranks on one GPU over gloo."""
    init_pg("gloo", rank, world, store)
    import test_gpu_sharded_trainer as TS
    from rsx.lightgcn import LightGCN
    from rsx.trainer import Trainer
    from rsx.utils import init_seed

    c, train, valid = TS._setup(root, rsx_dist="dp")
    init_seed(c["seed"])
    train.pretrain_setup()
    m = LightGCN(c, train)
    assert m.sharded and m.dp
    t = Trainer(c, m)
    assert t.fused
    seen = []
    step0 = m.engine.step

    def spy(triplets):
        seen.append(triplets[:2].cpu().numpy().copy())
        return step0(triplets)

    m.engine.step = spy
    losses = []
    for epoch in range(2):
        seen.clear()
        loss, n = t._train_epoch(train, epoch)
        assert not torch.is_tensor(loss) and n == m.steps_per_epoch
        losses.append(loss)
        t._epoch_for_lr += 1
        if epoch == 0:
            mine = np.concatenate(seen, axis=1)
    vres = t.evaluate(valid)
    f = m._final().cpu()
    np.savez(os.path.join(out, f"r{rank}.npz"), f=f.numpy(), p=m.engine.p.cpu().numpy(), losses=np.array(losses),
             keys=np.array(sorted(vres)), vals=np.array([vres[k] for k in sorted(vres)]), mine=mine,
             inter=np.stack([m.engine.sampler.inter_u.cpu().numpy(), m.engine.sampler.inter_i.cpu().numpy()]))
    dist.barrier()
    m.engine.close()
    dist.destroy_process_group()


def test_dp_trainer_fit_and_evaluate(cuda):
    """Every rank: the same losses, the same (bit-identical) tables and metric dict; the
    dict equals a single-process evaluation of those tables; one epoch's rank slices
    cover every training interaction exactly once."""
    import shutil

    from rsx import ops
    from rsx.evaluator import TopKEvaluator
    import test_gpu_sharded_trainer as TS

    world = 2
    with tempfile.TemporaryDirectory() as root:
        os.makedirs(os.path.join(root, "baby"))
        shutil.copy(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gold_small.inter"),
                    os.path.join(root, "baby", "baby.inter"))
        out = os.path.join(root, "out")
        os.makedirs(out)
        mp.spawn(_trainer_worker, args=(world, store_path(), root, out), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
        c, _, valid = TS._setup(root)
    for x in res[1:]:
        for key in ("f", "p", "losses", "vals"):
            assert np.array_equal(res[0][key], x[key]), key
    assert np.isfinite(res[0]["losses"]).all()
    got_pairs = sorted(map(tuple, np.concatenate([x["mine"] for x in res], axis=1).T.tolist()))
    assert got_pairs == sorted(map(tuple, res[0]["inter"].T.tolist()))
    f = torch.from_numpy(res[0]["f"]).to(cuda)
    nu = int(valid.mask_rowptr.numel() - 1)
    k = max(c["topk"])
    _, topk = ops.fullsort_topk(f[:nu], valid.eval_u, f[nu:], valid.mask_rowptr, valid.mask_col, k)
    want = TopKEvaluator(c).evaluate_device(topk, valid)
    got = dict(zip(res[0]["keys"], res[0]["vals"]))
    for key in want:
        assert abs(got[key] - want[key]) <= 1e-4 + 1e-12, (key, got[key], want[key])
