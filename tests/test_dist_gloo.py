"""Row-sharded LightGCN (rsx.dist) on 2, 4 and 8 CPU processes over gloo.

The HIP kernels cannot run here, so the engine's compute backend is replaced by
a CPU restatement of the same C-ABI epilogue semantics (include/rsx.h); what is
under test is the partitioning, the global-degree normalisation and the
collective schedule.  One sharded step must equal the single-process objective
sum_g L_ref(batch_g) on the union graph (reference LightGCN loss per rank
batch, src/models/lightgcn.py:132-156) followed by torch.optim.Adam.
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
        self.tu, self.ti = np.asarray(tu), np.asarray(ti)

    def sample_epoch_slices(self, epoch, n_slices, out=None):
        """The layout of rsx_sample_epoch_slices over a seeded permutation (negatives: the
        position's item + 1, unchecked: only the visiting order is under test here)."""
        from rsx.ops import DeviceSampler

        E = self.n_inter
        perm = np.random.default_rng(epoch).permutation(E)
        out = torch.empty(3 * E, dtype=torch.int64)
        for j in range(n_slices):
            a, e = DeviceSampler.slice_bounds(E, n_slices, j)
            sel = perm[a:e]
            out[3 * a:3 * e] = torch.from_numpy(np.concatenate([self.tu[sel], self.ti[sel], (self.ti[sel] + 1) % NI]))
        return out


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


def _worker(rank, world, store, out_dir, sparse=False, k=K):
    torch.set_num_threads(1)
    init_pg("gloo", rank, world, store)
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



@pytest.mark.parametrize("world,sparse,k", [(2, False, 3), (2, True, 3), (4, True, 3), (8, True, 3), (8, False, 3),
                                            (2, False, 4), (4, False, 4), (2, True, 2), (2, False, 1)])
def test_sharded_step_matches_global_objective(world, sparse, k):
    """sparse: the union-row exchange of the last layer / G's item rows and the
    reduce-scatter + owner Adam + all-gather of the item gradient (rsx/dist.py).
    k = 4: the reference's default depth (src/configs/model/LightGCN.yaml:3)."""
    K = k
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, store_path(), d, sparse, k), nprocs=world, join=True)
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


def _slices_worker(rank, world, store, out_dir):
    """Unequal shards with more steps per epoch than the small shard's batch (the case a
    fixed per-rank batch walked past the shard's end): every rank runs the common step
    count over balanced slices of its own interactions and visits each exactly once."""
    torch.set_num_threads(1)
    init_pg("gloo", rank, world, store)
    from rsx.dist import ShardedLightGCNEngine

    e_r = [11, 5, 7][rank]
    tu = np.arange(e_r) % 4
    ti = (np.arange(e_r) * 3) % NI
    key = np.unique(tu * 1000 + ti)
    tu, ti = key // 1000, key % 1000
    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    U0 = torch.nn.init.xavier_uniform_(torch.empty(4, D)).numpy()
    B = 2
    tot = torch.tensor([tu.size])
    dist.all_reduce(tot)
    steps = -(-int(tot.item()) // (world * B))
    eng = ShardedLightGCNEngine(tu, ti, 4, NI, D, 2, REG, LR, "cpu", U0, I0, backend=CpuBackend(),
                                batch=-(-tu.size // steps))
    seen = []
    real_step = eng.step

    def spy(triplets=None, **kw):
        seen.append(triplets.clone())
        return real_step(triplets=triplets, **kw)

    eng.step = spy
    for j in range(steps):
        eng.step_slice(0, j, steps)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), steps=steps, n=tu.size,
             users=torch.cat([t[0] for t in seen]).numpy(), items=torch.cat([t[1] for t in seen]).numpy(),
             sizes=np.array([t.shape[1] for t in seen]), tu=tu, ti=ti)
    dist.destroy_process_group()


def test_balanced_slices_visit_every_interaction_once():
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_slices_worker, args=(world, store_path(), d), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    steps = int(res[0]["steps"])
    for r in res:
        assert len(r["sizes"]) == steps  # the common step count on every rank
        assert r["sizes"].min() >= 1 and r["sizes"].max() - r["sizes"].min() <= 1
        got = sorted(zip(r["users"].tolist(), r["items"].tolist()))
        assert got == sorted(zip(r["tu"].tolist(), r["ti"].tolist()))  # each interaction exactly once
    assert any(int(r["n"]) < 2 * steps for r in res)  # a shard whose fixed-B walk would overrun


@pytest.mark.parametrize("E,S", [(5, 4), (3022, 7), (10, 10), (1, 1), (299_999, 147)])
def test_slice_bounds_partition(E, S):
    from rsx.ops import DeviceSampler

    b = [DeviceSampler.slice_bounds(E, S, j) for j in range(S)]
    assert b[0][0] == 0 and b[-1][1] == E
    assert all(b[j][1] == b[j + 1][0] for j in range(S - 1))
    sizes = [e - a for a, e in b]
    assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
    # the kernel's slice-of-position formula (csrc/step.hip sample_kernel)
    for t in list(range(min(E, 50))) + list(range(max(0, E - 50), E)):
        j = ((t + 1) * S - 1) // E
        assert b[j][0] <= t < b[j][1]


def _dp_worker(rank, world, store, out_dir, k):
    """rsx.dp's data-parallel step (its CPU restatement) on `world` gloo ranks: the
    graph and tables replicated, rank r's own triplets, one global batch per step."""
    torch.set_num_threads(1)
    init_pg("gloo", rank, world, store)
    from rsx.dp import DataParallelLightGCNEngine

    tu, ti, _ = _local_graph(0)  # one graph for every rank
    torch.manual_seed(7)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    if rank:  # replicas start from rank 0's tables whatever the others hold
        U0, I0 = U0 * 0 + 1, I0 * 0 - 1
    eng = DataParallelLightGCNEngine(tu, ti, NU, NI, D, k, REG, LR, "cpu", U0, I0, batch=32, backend="torch")
    losses = []
    for s in range(2):
        _, _, trip = _local_graph(10 * s + rank)  # rank-specific triplets (users < NU, items < NI)
        eng.step(torch.from_numpy(trip[:, : 20 - rank]))  # unequal rank batches
        losses.append(float(eng.loss_out[0]))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), p=eng.p.numpy(), losses=np.array(losses))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 3), (4, 3), (2, 2), (3, 4)])
def test_data_parallel_step_matches_global_batch(world, k):
    """Two data-parallel steps = two reference steps (loss + torch.optim.Adam) on the
    global batch (every rank's triplets concatenated, rank order) of the one graph;
    the replicas stay bit-identical."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dp_worker, args=(world, store_path(), d, k), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    tu, ti, _ = _local_graph(0)
    A = O.lightgcn_norm_adj_vec(tu, ti, NU, NI)
    torch.manual_seed(7)
    u = torch.nn.Parameter(torch.nn.init.xavier_uniform_(torch.empty(NU, D)))
    i = torch.nn.Parameter(torch.nn.init.xavier_uniform_(torch.empty(NI, D)))
    opt = torch.optim.Adam([u, i], lr=LR)
    ref_losses = []
    for s in range(2):
        trip = torch.from_numpy(np.concatenate([_local_graph(10 * s + r)[2][:, : 20 - r] for r in range(world)], 1))
        opt.zero_grad()
        loss = O.lightgcn_loss(u, i, A, k, trip, REG)
        loss.backward()
        opt.step()
        ref_losses.append(loss.item())
    for r in range(world):
        np.testing.assert_allclose(res[r]["losses"], ref_losses, rtol=1e-5)
        p = res[r]["p"]
        np.testing.assert_allclose(p[:NU], u.detach().numpy(), rtol=0, atol=2e-6)
        np.testing.assert_allclose(p[NU:], i.detach().numpy(), rtol=0, atol=2e-6)
        assert np.array_equal(res[0]["p"], p)  # replicas bit-identical


def _err_worker(rank, world, store, out_dir, bad_rank, bits):
    """ShardedLightGCNEngine.check_err on a rank group where only `bad_rank` holds error
    bits in its row-list word (its own batch met an out-of-range id, or its neighbour
    list overflowed)."""
    from types import SimpleNamespace

    init_pg("gloo", rank, world, store)
    from rsx.dist import ShardedLightGCNEngine

    me = SimpleNamespace(err=torch.tensor([bits if rank == bad_rank else 0], dtype=torch.int32), native=True,
                         world=world, group=None)
    try:
        ShardedLightGCNEngine.check_err(me)
        msg = ""
    except RuntimeError as e:
        msg = str(e)
    dist.barrier()  # no rank is left blocked: every rank reaches the next collective
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bad,bits", [(2, 1, 1), (3, 0, 2), (3, 2, 3), (2, 0, 0)])
def test_row_list_error_raises_on_every_rank(world, bad, bits):
    """the sticky row-list error word is per rank; check_err ORs it over the
    group so that all ranks raise together instead of one rank raising while its peers
    block in the epoch's loss all-reduce."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_err_worker, args=(world, store_path(), d, bad, bits), nprocs=world, join=True)
        msgs = [open(os.path.join(d, f"r{r}.txt")).read() for r in range(world)]
    if bits == 0:
        assert msgs == [""] * world
    else:
        assert all(f"bits {bits:#x}" in m for m in msgs), msgs
