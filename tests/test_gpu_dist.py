"""Row-sharded LightGCN with the HIP backend: 2 ranks sharing the one GPU of the
test box, collectives over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run
is the driver's).  One step must equal the single-process global objective."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rsx_oracle as O
from test_dist_gloo import D, K, LR, NI, NU, REG, _local_graph

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy() if rank == 0 else np.zeros((NI, D), np.float32)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D), generator=torch.Generator().manual_seed(rank)).numpy()
    tu, ti, trip = _local_graph(rank)
    eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16)
    f0 = eng.forward().cpu().clone()
    eng.step(triplets=torch.from_numpy(trip).cuda())
    p1 = eng.p.cpu().numpy()
    # device-sampled steps run too (epoch buffer + slices)
    for s in range(0, eng.n_inter, 16):
        eng.step(epoch=0, start=s)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), p=p1, f0=f0.numpy(), U0=U0, I0=I0,
             after=eng.p.cpu().numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_hip_step_matches_global_objective():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    gu, gi, trips = [], [], []
    for r in range(world):
        tu, ti, trip = _local_graph(r)
        gu.append(tu + r * NU)
        gi.append(ti)
        t = trip.copy()
        t[0] += r * NU
        trips.append(torch.from_numpy(t))
    gu, gi = np.concatenate(gu), np.concatenate(gi)
    nu_all = world * NU
    A = O.lightgcn_norm_adj_vec(gu, gi, nu_all, NI)
    U0 = np.concatenate([res[r]["U0"] for r in range(world)])
    I0 = res[0]["I0"]
    fg = O.lightgcn_forward(A, torch.from_numpy(np.concatenate([U0, I0])), K).numpy()
    for r in range(world):
        np.testing.assert_allclose(res[r]["f0"][:NU], fg[r * NU:(r + 1) * NU], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(res[r]["f0"][NU:], fg[nu_all:], rtol=1e-5, atol=1e-7)
    u = torch.nn.Parameter(torch.from_numpy(U0.copy()))
    i = torch.nn.Parameter(torch.from_numpy(I0.copy()))
    opt = torch.optim.Adam([u, i], lr=LR)
    loss = sum(O.lightgcn_loss(u, i, A, K, t, REG) for t in trips)
    loss.backward()
    opt.step()
    for r in range(world):
        p = res[r]["p"]
        np.testing.assert_allclose(p[:NU], u.detach().numpy()[r * NU:(r + 1) * NU], rtol=0, atol=2e-6)
        np.testing.assert_allclose(p[NU:], i.detach().numpy(), rtol=0, atol=2e-6)
    assert np.array_equal(res[0]["p"][NU:], res[1]["p"][NU:])
    assert np.array_equal(res[0]["after"][NU:], res[1]["after"][NU:])
    assert np.isfinite(res[0]["after"]).all()
