"""Row-sharded LightGCN with the HIP backend: 2 ranks sharing the one GPU of the
test box, collectives over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run
is the driver's).  One step must equal the single-process global objective."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import init_pg, store_path

import rsx_oracle as O
from test_dist_gloo import D, K, LR, NI, NU, REG, _local_graph

pytestmark = pytest.mark.gpu


def _worker(rank, world, store, out_dir, native, sparse, k=K, fused=True, head=None):
    os.environ["RSX_SHARDED_FUSED"] = "1" if fused else "0"
    if head is not None:  # the step's first item partial in `head` row pieces (rsx_sharded_lgcn_step.n_head)
        os.environ["RSX_SHARDED_HEAD"] = str(head)
    init_pg("gloo", rank, world, store)
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy() if rank == 0 else np.zeros((NI, D), np.float32)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D), generator=torch.Generator().manual_seed(rank)).numpy()
    tu, ti, trip = _local_graph(rank)
    # native: csrc/dist.hip's one-call step, its exchanges through the host hook (gloo)
    eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, k, REG, LR, "cuda:0", U0, I0, batch=16, native=native,
                                sparse=sparse)
    assert eng.native == native and eng.sparse == sparse
    if native:  # the fused-round schedule: dense, K = 2, 3 (csrc/dist.hip:sharded_fused_rounds)
        assert (getattr(eng, "xch", None) is not None) == (fused and not sparse and k in (2, 3))
        if head is not None:
            assert len(eng.head) == head
    f0 = eng.forward().cpu().clone()
    eng.step(triplets=torch.from_numpy(trip).cuda())
    if rank == 0:  # a one-rank read of the parameters (a checkpoint) issues no collective
        _ = eng.p.cpu()
    eng.flush()  # every rank: the deferred all-gather of the owners' item rows
    p1 = eng.p.cpu().numpy()
    # device-sampled steps run too (epoch buffer + slices)
    for s in range(0, eng.n_inter, 16):
        eng.step(epoch=0, start=s)
    eng.flush()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), p=p1, f0=f0.numpy(), U0=U0, I0=I0,
             after=eng.p.cpu().numpy())
    dist.destroy_process_group()



@pytest.mark.parametrize("native,sparse,k,fused", [(False, False, 3, True), (True, False, 3, True),
                                                   (True, False, 3, False), (True, False, 2, True),
                                                   (False, True, 3, True), (True, True, 3, True),
                                                   (True, False, 4, True), (False, False, 4, True),
                                                   (True, True, 3, "head3"), (True, False, 3, "head3"),
                                                   (True, True, 2, "head3")])
def test_sharded_hip_step_matches_global_objective(native, sparse, k, fused):
    """sparse: the union-row exchange + reduce-scatter / owner Adam / all-gather schedule
    (csrc/dist.hip with the host hook's collectives when native).  Native dense K = 2, 3:
    the fused-round schedule (two layers' item partials per collective), fused=False the
    one-exchange-per-layer stored-layer step.  k = 4: the reference's default depth, the
    native step's dense (untagged) form.  "head3": the stored-layer step with its first
    item partial in 3 row pieces, each all-reduced as soon as it is computed."""
    world = 2
    K = k
    head = None
    if fused == "head3":
        fused, head = False, 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, store_path(), d, native, sparse, k, fused, head), nprocs=world, join=True)
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


def _native_worker(rank, world, store, out_dir, SPARSE=True):
    os.environ["RSX_SHARDED_FUSED"] = "0" if SPARSE else "1"  # dense: the fused-round schedule, graph-captured
    torch.cuda.set_device(0)
    init_pg("nccl", rank, world, store, device_id=torch.device("cuda", 0))
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
    tu, ti, trip = _local_graph(rank)
    res = {}
    for native in ("graph", True, False):
        eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16,
                                    native=bool(native), sparse=SPARSE)
        assert eng.native == bool(native)
        if native is True:
            eng.use_graph = False  # the eagerly issued native step
        f0 = eng.forward().cpu().clone()
        eng.step(triplets=torch.from_numpy(trip).cuda())
        losses = [float(eng.loss_acc.item())]
        for s in range(0, eng.n_inter, 16):
            eng.step(epoch=0, start=s)
        torch.cuda.synchronize()
        losses.append(float(eng.loss_acc.item()))
        if getattr(eng, "reg_cnt", None) is not None:  # the one-launch BPR's occurrence counts are all cleared
            assert torch.count_nonzero(eng.reg_cnt[:-4]).item() == 0
        eng.invalidate()
        f1 = eng.forward().cpu().clone()  # (forward flushes first: every rank calls it)
        if native == "graph":  # full batches after the first were replayed from one capture
            assert eng._graphs.get(16) is not None
        res[native] = (f0.numpy(), eng.p.cpu().numpy(), eng.m.cpu().numpy(), np.array(losses), f1.numpy())
        if native is True:  # the bare collective: one rank = identity, stream-ordered
            from rsx import _lib as L
            from rsx import ops
            import ctypes as C

            x = torch.arange(1000, dtype=torch.float32, device="cuda:0")
            L.check(L.lib().rsx_comm_allreduce_f32(eng._comm, C.c_void_p(x.data_ptr()), 1000, ops._stream()),
                    "allreduce")
            assert torch.equal(x.cpu(), torch.arange(1000, dtype=torch.float32))
        if native == "graph":
            # a batch larger than the engine's reallocates the workspace: the captured graph
            # (which holds the old pointer) is dropped, and the next full batches re-capture
            p_before = eng.p.clone()
            big = torch.from_numpy(np.concatenate([trip, trip], axis=1)).cuda()
            eng.step(triplets=big)
            assert not eng._graphs
            for s in range(0, 3 * 16, 16):
                eng.step(epoch=1, start=s)
            torch.cuda.synchronize()
            assert eng._graphs.get(16) is not None and torch.isfinite(eng.p).all()
            assert not torch.equal(p_before, eng.p)
        eng.close()
    np.savez(os.path.join(out_dir, "native.npz"), **{f"{k}_{i}": v for k in ("graph", True, False)
                                                     for i, v in enumerate(res[k])})
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [True, False])
def test_native_sharded_step_equals_python_sequence(sparse):
    """csrc/dist.hip's one-call step over an RCCL communicator (one rank here: the box
    has one GPU) equals the Python-issued sequence it restates: the forward bit for
    bit, training within 1e-5.  sparse: the sparse schedule's collectives (all-gather,
    reduce-scatter); dense: the fused-round schedule, graph-captured too."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_native_worker, args=(1, store_path(), d, sparse), nprocs=1, join=True)
        z = dict(np.load(os.path.join(d, "native.npz")))
    # forward before any step: same kernels, same order -> bit-identical; after the
    # steps the BPR gradient scatter's float atomics (duplicate rows in a batch, as the
    # reference's index_put_) may order differently run to run: 1e-6 absolute
    assert np.array_equal(z["True_0"], z["False_0"]) and np.array_equal(z["graph_0"], z["False_0"])
    # (the native step keeps the layers and runs Horner on G/(K+1); the Python sequence
    # keeps running sums: same objective, different rounding order)
    for i in range(1, 5):
        np.testing.assert_allclose(z[f"True_{i}"], z[f"False_{i}"], rtol=1e-5, atol=1e-5, err_msg=str(i))
        # the graph-replayed native step = the eagerly issued one (up to the BPR atomics' order)
        np.testing.assert_allclose(z[f"graph_{i}"], z[f"True_{i}"], rtol=1e-6, atol=1e-6, err_msg=str(i))
    assert np.isfinite(z["True_1"]).all()


def _sim_worker(rank, world, store, out_dir):
    """The one-rank sharded engine over the latency-injected communicator (RSX_COMM_SIM):
    every collective is the one-rank identity plus a comm-stream kernel holding the
    modelled time, so the trained tables equal the plain one-rank engine's and the step
    takes at least the modelled exchange time."""
    import time

    torch.cuda.set_device(0)
    init_pg("nccl", rank, world, store, device_id=torch.device("cuda", 0))
    from rsx import _lib as L
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
    tu, ti, trip = _local_graph(0)
    out = {}
    os.environ["RSX_COMM_SIM_OPT_IN"] = "1"  # the benchmark mode's second switch (rsx.dist.sim_comm_params)
    for sim in (None, "4:1.0:200"):  # 4 ranks at 1 GB/s bus bandwidth + 200 us per collective
        if sim:
            os.environ["RSX_COMM_SIM"] = sim
        else:
            os.environ.pop("RSX_COMM_SIM", None)
        eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16, sparse=True)
        assert (eng.sim is not None) == bool(sim)
        for s in range(0, 4 * 16, 16):  # eager, eager, captured, replayed
            eng.step(epoch=0, start=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(4 * 16, 8 * 16, 16):
            eng.step(epoch=0, start=s)
        torch.cuda.synchronize()
        out[f"ms_{bool(sim)}"] = (time.perf_counter() - t0) * 1e3 / 4
        eng.flush()
        out[f"p_{bool(sim)}"] = eng.p.cpu().numpy()
        if sim:
            X = NI * D * 4.0
            out["model_ar_ms"] = 1e3 * L.lib().rsx_comm_sim_seconds(eng._comm, L.RSX_COLL_ALLREDUCE, X)
        eng.close()
    os.environ.pop("RSX_COMM_SIM", None)
    np.savez(os.path.join(out_dir, "sim.npz"), **out)
    dist.destroy_process_group()


def test_latency_injected_comm_is_data_identity_and_takes_the_modelled_time():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_sim_worker, args=(1, store_path(), d), nprocs=1, join=True)
        z = dict(np.load(os.path.join(d, "sim.npz")))
    np.testing.assert_allclose(z["p_True"], z["p_False"], rtol=0, atol=1e-6)
    # model: 2 (W-1)/W X / busbw + latency for an all-reduce of the item block X
    X = NI * D * 4.0
    assert abs(float(z["model_ar_ms"]) - (1e3 * 2 * 0.75 * X / 1e9 + 0.2)) < 1e-6
    # a K = 3 sparse step issues 4 dense all-reduce-volume collectives + RS + AG + compact
    # ones: at least the 200 us latency of each of its >= 8 collectives on the comm stream
    assert float(z["ms_True"]) >= float(z["ms_False"]) + 8 * 0.2 * 0.9, (z["ms_True"], z["ms_False"])


def _hub_graph():
    """_local_graph's shape plus a hub user: user 0 holds 30 items (the others ~4), so a
    batch repeating user 0 lists 16 x 30 neighbour claims unless users are deduplicated."""
    rng = np.random.default_rng(5)
    tu = np.concatenate([np.repeat(np.arange(NU), 4), np.zeros(30, np.int64)])
    ti = np.concatenate([np.concatenate([rng.choice(NI, 4, replace=False) for _ in range(NU)]), np.arange(30)])
    key = np.unique(tu * 1000 + ti)
    return key // 1000, key % 1000


def _hub_batches(tu, ti, n=6, B=16):
    """n batches of B triplets (user, positive, sampled negative); batch 0 is user 0 sixteen
    times, the others mix user 0 with random users (duplicates included)."""
    rng = np.random.default_rng(11)
    hist = {}
    for u, i in zip(tu.tolist(), ti.tolist()):
        hist.setdefault(u, []).append(i)
    out = []
    for b in range(n):
        users = np.zeros(B, np.int64) if b == 0 else np.concatenate([[0, 0, 0], rng.integers(0, NU, B - 3)])
        pos = np.array([rng.choice(hist[int(u)]) for u in users], np.int64)
        neg = []
        for u in users:
            x = int(rng.integers(NI))
            while x in hist[int(u)]:
                x = int(rng.integers(NI))
            neg.append(x)
        out.append(np.stack([users, pos, np.array(neg, np.int64)]))
    return out


def _order_worker(rank, world, store, out_dir):
    """The sparse native step over the POISONED latency-injected communicator (every
    collective's buffer reads NaN / id -1 for its modelled time, then is restored): each
    combination of the owner-Adam placement and the deferred all-gather, graph-replayed
    and eager, with the comm stream at the greatest priority."""
    os.environ["RSX_COMM_SIM"] = "4:1.0:100"  # 4 modelled ranks, 1 GB/s, 100 us per collective
    os.environ["RSX_COMM_SIM_OPT_IN"] = "1"
    os.environ["RSX_COMM_SIM_POISON"] = "1"
    os.environ["RSX_COMM_PRIORITY"] = "1"
    os.environ.pop("RSX_COMM_SIM_SHARE", None)
    torch.cuda.set_device(0)
    init_pg("nccl", rank, world, store, device_id=torch.device("cuda", 0))
    from rsx.dist import ShardedLightGCNEngine

    torch.manual_seed(7)
    I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
    U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
    tu, ti = _hub_graph()
    batches = [torch.from_numpy(b).cuda() for b in _hub_batches(tu, ti)]
    out = {"U0": U0, "I0": I0}
    for comm_adam in (0, 1):
        for defer in (0, 1):
            for graph in (True, False):
                os.environ["RSX_SHARDED_COMM_ADAM"] = str(comm_adam)
                os.environ["RSX_SHARDED_DEFER_AG"] = str(defer)
                eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16, sparse=True)
                assert eng.sim is not None and eng.nbr is not None and eng.defer_ag == bool(defer)
                eng.use_graph = graph
                counts = []
                for t in batches:
                    eng.step(triplets=t)
                    counts.append(int(eng.nbr["count"].item()))
                eng.flush()  # raises on a row-list error bit
                torch.cuda.synchronize()
                key = f"a{comm_adam}_d{defer}_g{int(graph)}"
                out[f"p_{key}"] = eng.p.cpu().numpy()
                out[f"cnt_{key}"] = np.array(counts)
                out[f"err_{key}"] = int(eng.err.item())
                out[f"replays_{key}"] = int(16 in eng._graphs)
                eng.close()
    np.savez(os.path.join(out_dir, "order.npz"), **out)
    dist.destroy_process_group()


def test_sparse_step_stream_order_under_poisoned_collectives():
    """Pins the stream order of csrc/dist.hip's sparse step (round-4 faults):
    every collective runs on the comm stream (priority on) as a stand-in that poisons its
    buffer for the modelled time, so a reader or writer not fenced by the fork / join
    events sees NaN / an id of -1 (row lists: error bit, never a fault).  Graph-replayed
    = eager, both = the unsharded objective (one rank: the whole graph) after 6 Adam steps;
    the neighbour list holds each distinct batch user once (a repeated hub
    user overflowed nbr_cap)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_order_worker, args=(1, store_path(), d), nprocs=1, join=True)
        z = dict(np.load(os.path.join(d, "order.npz")))
    tu, ti = _hub_graph()
    A = O.lightgcn_norm_adj_vec(tu, ti, NU, NI)
    u = torch.nn.Parameter(torch.from_numpy(z["U0"].copy()))
    i = torch.nn.Parameter(torch.from_numpy(z["I0"].copy()))
    opt = torch.optim.Adam([u, i], lr=LR)
    batches = _hub_batches(tu, ti)
    for t in batches:
        opt.zero_grad()
        O.lightgcn_loss(u, i, A, K, torch.from_numpy(t), REG).backward()
        opt.step()
    ref = torch.cat([u, i]).detach().numpy()
    deg = np.bincount(tu, minlength=NU)
    want = [2 * 16 + int(deg[np.unique(t[0])].sum()) for t in batches]
    for comm_adam in (0, 1):
        for defer in (0, 1):
            key_g, key_e = f"a{comm_adam}_d{defer}_g1", f"a{comm_adam}_d{defer}_g0"
            assert z[f"replays_{key_g}"] == 1 and z[f"err_{key_g}"] == 0 and z[f"err_{key_e}"] == 0
            for key in (key_g, key_e):
                # the claim counter: every distinct batch user's degree once (2 B ids first)
                assert (z[f"cnt_{key}"] + 2 * 16).tolist() == want, key
                np.testing.assert_allclose(z[f"p_{key}"], ref, rtol=0, atol=2e-5, err_msg=key)
            # replayed = eager up to the BPR gradient atomics' order (repeated rows)
            np.testing.assert_allclose(z[f"p_{key_g}"], z[f"p_{key_e}"], rtol=0, atol=1e-5, err_msg=key_g)
