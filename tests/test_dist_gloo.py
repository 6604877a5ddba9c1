"""Row-sharded LightGCN (rsx.dist) on 2, 4 and 8 CPU processes over gloo.

The HIP kernels cannot run here, so the engine's compute backend is replaced by
a CPU restatement of the same C-ABI epilogue semantics (include/rsx.h); what is
under test is the partitioning, the global-degree normalisation and the
collective schedule.  One sharded step must equal the single-process objective
sum_g L_ref(batch_g) on the union graph (reference LightGCN loss per rank
batch, src/models/lightgcn.py:132-156) followed by torch.optim.Adam.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rsx_oracle as O
from rsx import _lib as L

NU, NI, D, K, REG, LR = 60, 40, 32, 3, 1e-2, 1e-3


class CpuCSR:
    def __init__(self, rowptr, col, val, n_cols):
        n_rows = rowptr.size - 1
        rows = np.repeat(np.arange(n_rows), np.diff(rowptr))
        self.m = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])),
                                         torch.from_numpy(val), (n_rows, n_cols)).coalesce()
        self.n_rows = n_rows
        self.nnz = int(col.size)


class CpuSampler:
    def __init__(self, tu, ti):
        self.n_inter = tu.size


class CpuBackend:
    """CPU restatement of the rsx epilogues (include/rsx.h) for the gloo test."""

    def tensor(self, a):
        return torch.as_tensor(a).clone()

    def csr(self, rowptr, col, val, n_cols, chunk=32):
        return CpuCSR(rowptr, col, val, n_cols)

    def adam(self, lr, step, weight_decay=0.0):
        return {"lr": lr, "step": step}

    def sampler(self, tu, ti, nu, seed):
        return CpuSampler(tu, ti)

    def _epi(self, acc, kind, alpha, beta, adam, t):
        acc = acc * alpha
        s_in = t.get("s_in")
        if kind == L.RSX_EPI_STORE:
            t["y"].copy_(acc)
        elif kind == L.RSX_EPI_LAYERSUM:
            t["y"].copy_(acc)
            t["s_out"].copy_((s_in + acc) if s_in is not None else acc)
        elif kind == L.RSX_EPI_FINAL:
            t["f"].copy_(((s_in + acc) if s_in is not None else acc) * beta)
        elif kind == L.RSX_EPI_ADD:
            out = acc.clone()
            if s_in is not None:
                out = out + s_in
            if t.get("r_add") is not None:
                out = out + t["r_add"]
            t["y"].copy_(out * beta)
        elif kind == L.RSX_EPI_ADAM:
            g = ((s_in + acc) if s_in is not None else acc) * beta
            if t.get("r_add") is not None:
                g = g + t["r_add"]
            p, m, v = t["p"], t["m"], t["v"]
            step = adam["step"]
            m.copy_(m + 0.1 * (g - m))
            v.copy_(v * 0.999 + (0.001 * g) * g)
            bc1 = 1 - 0.9 ** step
            bc2 = 1 - 0.999 ** step
            denom = v.sqrt() / (bc2 ** 0.5) + 1e-8
            p.copy_(p - (adam["lr"] / bc1) * m / denom)
        else:
            raise NotImplementedError(kind)
        for z in ("zero0", "zero1"):
            if t.get(z) is not None:
                t[z].zero_()

    def spmm(self, A, x, d, kind, alpha=1.0, beta=1.0, adam=None, **t):
        self._epi(torch.sparse.mm(A.m, x), kind, alpha, beta, adam, t)

    def rowwise(self, n, d, kind, alpha=1.0, beta=1.0, adam=None, **t):
        self._epi(torch.zeros(n, d), kind, alpha, beta, adam, t)

    def bpr(self, fin, ego, nu, ni, trip, reg, g, r, loss_acc):
        f = fin.clone().requires_grad_(True)
        e = ego.clone().requires_grad_(True)
        u, p, n = trip[0], trip[1] + nu, trip[2] + nu
        ps = (f[u] * f[p]).sum(1)
        ns = (f[u] * f[n]).sum(1)
        mf = -torch.log(1e-10 + torch.sigmoid(ps - ns)).mean()
        rg = sum(torch.norm(x, p=2) for x in (e[u], e[p], e[n])) / trip.shape[1]
        loss = mf + reg * rg
        loss.backward()
        g.add_(f.grad)
        r.add_(e.grad)
        loss_acc.add_(loss.detach().double())
        return loss.detach()


def _local_graph(rank):
    rng = np.random.default_rng(100 + rank)
    tu = np.repeat(np.arange(NU), 4)
    ti = np.concatenate([rng.choice(NI, 4, replace=False) for _ in range(NU)])
    ti[:30] = 0  # a hub item shared by both ranks
    key = np.unique(tu * 1000 + ti)
    tu, ti = key // 1000, key % 1000
    trip_idx = rng.choice(tu.size, 24, replace=False)
    hist = set(zip(tu.tolist(), ti.tolist()))
    neg = []
    for u in tu[trip_idx]:
        x = int(rng.integers(NI))
        while (int(u), x) in hist:
            x = int(rng.integers(NI))
        neg.append(x)
    trip = np.vstack([tu[trip_idx], ti[trip_idx], np.array(neg)])
    return tu, ti, trip


def _worker(rank, world, port, out_dir, sparse=False, k=K):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy() if rank == 0 else np.zeros((NI, D), np.float32)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D), generator=torch.Generator().manual_seed(rank)).numpy()
    tu, ti, trip = _local_graph(rank)
    eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, k, REG, LR, "cpu", U0, I0, backend=CpuBackend(), batch=32,
                                sparse=sparse)
    assert eng.sparse == sparse
    f0 = eng.forward().clone()
    eng.step(triplets=torch.from_numpy(trip))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), p=eng.p.numpy(), f0=f0.numpy(), U0=U0,
             I0=eng.p.numpy()[NU:] * 0 + (I0 if rank == 0 else 0), loss=eng.loss_acc.numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,sparse,k", [(2, False, 3), (2, True, 3), (4, True, 3), (8, True, 3), (8, False, 3),
                                            (2, False, 4), (4, False, 4), (2, True, 2), (2, False, 1)])
def test_sharded_step_matches_global_objective(world, sparse, k):
    """sparse: the union-row exchange of the last layer / G's item rows and the
    reduce-scatter + owner Adam + all-gather of the item gradient (rsx/dist.py).
    k = 4: the reference's default depth (src/configs/model/LightGCN.yaml:3)."""
    K = k
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, sparse, k), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    # global graph: users of rank g offset by g*NU
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
    # forward before the step
    fg = O.lightgcn_forward(A, torch.from_numpy(np.concatenate([U0, I0])), K).numpy()
    for r in range(world):
        f0 = res[r]["f0"]
        np.testing.assert_allclose(f0[:NU], fg[r * NU:(r + 1) * NU], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(f0[NU:], fg[nu_all:], rtol=1e-5, atol=1e-7)
    # one step of sum_g L(batch_g) + Adam
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
    # item replicas stay identical
    for r in range(1, world):
        assert np.array_equal(res[0]["p"][NU:], res[r]["p"][NU:])
    assert abs(sum(float(x["loss"][0]) for x in res) - loss.item()) < 1e-5
