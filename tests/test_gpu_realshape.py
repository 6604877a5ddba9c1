"""The HIP path at the shapes the bench and the multi-GPU configs run, against the oracle.

The small fixtures (400 users x 200 items) only reach the full-sort kernel's
many-small-chunks plan and the SpMM's in-launch hub fixups.  These tests run the
production plans and check them on the CPU:

* full-sort at the C2 shape (35,598 users x 18,357 items, d=64: 2 chunks of 9,184
  items), the C5 shape (39,387 x 23,033, d=128: 2 chunks), a 16-chunk plan and a
  C4-like chunk (d=256, 2 chunks of 200,000 items).  Integer-valued embeddings make
  every score exact in f32, so the top-k indices must equal the oracle's canonical
  top-k (score desc, index asc) bit for bit, including runs of tied scores across
  the k boundary, scores rising with the item index (every tile inserts: the
  256-slot overflow compaction and the early-stop compactions run over and over)
  and users whose train items mask all but 10 items (-1e10 entries inside the
  top-50).  A trained sports table checks realistic scores modulo near-ties;
* SpMM with more than 1,024 hub rows (their fixups take their own launch) at d=64
  and d=256 against torch.sparse.mm;
* a LightGCN d=256 K=3 training run on a power-law graph with more than 1,024 hub
  rows (tagged and dense step) against oracle.LightGCNCPU, the reference-identical
  CPU restatement (src/models/lightgcn.py:117-156, src/common/trainer.py:186-238).
"""
import numpy as np
import pytest
import torch

import rsx_oracle as O
from helpers import canonical_topk_fast, topk_equal_modulo_ties
from rsx import _lib as L
from rsx import graph, ops, synth

pytestmark = pytest.mark.gpu


def _plan(nb, ni, d):
    import ctypes as C

    nc, per = C.c_int32(), C.c_int64()
    L.check(L.lib().rsx_fullsort_plan(nb, ni, d, C.byref(nc), C.byref(per)), "plan")
    return nc.value, per.value


def _cpu_scores(U, users, I, rp, mc, rows):
    """f32 scores of the checked rows with the train-item mask (-1e10, trainer.py:521-525)."""
    s = U[users[rows]] @ I.T
    for b, r in enumerate(rows):
        u = users[r]
        s[b, mc[rp[u]:rp[u + 1]]] = -1e10
    return s


def _history(nu, ni, rng, heavy):
    """Per-user train items (~Geometric, mean 6) plus `heavy` users masking all but 10 items."""
    deg = np.minimum(rng.geometric(1 / 6, size=nu), ni)
    tus = [np.repeat(np.arange(nu), deg)]
    tis = [rng.integers(0, ni, size=tus[0].size)]
    for u in heavy:
        others = np.setdiff1d(np.arange(ni), rng.choice(ni, size=10, replace=False))
        tus.append(np.full(others.size, u))
        tis.append(others)
    key = np.unique(np.concatenate(tus).astype(np.int64) * ni + np.concatenate(tis))
    return graph.history_csr(key // ni, key % ni, nu)


def _exact_tables(pattern, nb, ni, d, rng):
    """Integer-valued user/item tables: every score is an exactly representable f32."""
    if pattern == "ties":  # entries in {-1, 0, 1}: scores in [-d, d], long runs of equal scores
        U = rng.integers(-1, 2, size=(nb, d)).astype(np.float32)
        I = rng.integers(-1, 2, size=(ni, d)).astype(np.float32)
        return U, I
    # "ramp": users pick one of three item columns: score = i (rising with the index:
    # every tile inserts), ni-1-i (falling), i // 7 (rising in runs of 7 ties)
    U = np.zeros((nb, d), np.float32)
    U[np.arange(nb), np.arange(nb) % 3] = 1.0
    I = np.zeros((ni, d), np.float32)
    i = np.arange(ni, dtype=np.float32)
    I[:, 0], I[:, 1], I[:, 2] = i, ni - 1 - i, np.floor(i / 7)
    I[:, 3:] = rng.integers(-1, 2, size=(ni, d - 3))  # ignored by the one-hot users
    return U, I


def _run_fullsort(cuda, U, users, I, rp, mc, k=50):
    val, idx = ops.fullsort_topk(torch.from_numpy(U).to(cuda), torch.from_numpy(users).to(cuda),
                                 torch.from_numpy(I).to(cuda), torch.from_numpy(rp).to(cuda),
                                 torch.from_numpy(mc).to(cuda), k)
    return val.cpu().numpy(), idx.cpu().numpy()


# (n_users, n_items, d, expected item chunks): C2 sports and C5 clothing (2 chunks, the
# balanced split of the screened kernel: 4 lists a user), a 16-chunk plan (fs_select<16>
# over lists cut to top k), a C4-like 200k-item chunk at d=256
SHAPES = [(35598, 18357, 64, 2), (39387, 23033, 128, 2), (4096, 18357, 64, 16), (16384, 400000, 256, 2)]


@pytest.mark.parametrize("pattern", ["ties", "ramp"])
@pytest.mark.parametrize("nb,ni,d,chunks", SHAPES)
def test_fullsort_production_plans_exact(cuda, nb, ni, d, chunks, pattern):
    assert _plan(nb, ni, d)[0] == chunks
    rng = np.random.default_rng(nb + d)
    U, I = _exact_tables(pattern, nb, ni, d, rng)
    users = rng.permutation(nb).astype(np.int64)
    heavy = users[[0, 1, 2, 3, 4, 5]]
    rp, mc = _history(nb, ni, rng, heavy)
    val, idx = _run_fullsort(cuda, U, users, I, rp, mc)
    n_check = 1200 if ni < 100000 else 192
    rows = np.concatenate([np.arange(6), rng.choice(np.arange(6, nb), size=n_check, replace=False)])
    for r0 in range(0, rows.size, 64):
        rr = rows[r0:r0 + 64]
        cv, ci = canonical_topk_fast(_cpu_scores(U, users, I, rp, mc, rr), 50)
        assert np.array_equal(idx[rr], ci), f"rows {rr[np.any(idx[rr] != ci, axis=1)][:5]}"
        assert np.array_equal(val[rr], cv)
    # the heavy users' lists end in masked items at exactly -1e10, in index order
    assert np.all(val[:6, 10:] == np.float32(-1e10))


@pytest.mark.parametrize("k", [50, 64])
@pytest.mark.parametrize("nb,ni,d,chunks", SHAPES)
def test_fullsort_screen_exact_vs_cpu_fmaf(cuda, nb, ni, d, chunks, k):
    """Real-valued, heavy-tailed tables at every production plan, anchored on the CPU:
    the screened kernel's top-k must equal, index for index and bit for bit in value,
    the canonical top-k (score desc, index asc) of the scores oracle/fs_oracle.c computes
    with C's fmaf chain (the reference ranks U I^T with the train items at -1e10,
    src/common/trainer.py:509-528).  The tables stress the screen's invariants
    (csrc/fullsort.hip, "Screened full-sort"): row norms over six orders of magnitude
    (the margin eps |u||v_i| from 1e-3 to 1e3 of a typical score), exact duplicate item
    rows (score ties at the k boundary: the index order decides), a zero user (every
    score 0), negated users, and users whose train items mask all but 10 items (the top
    k holds -1e10 entries: masked items must reach the candidate rows as -1e10)."""
    assert _plan(nb, ni, d)[0] == chunks
    rng = np.random.default_rng(nb + d + k)
    U = (rng.standard_normal((nb, d)) * np.exp(rng.standard_normal((nb, 1)))).astype(np.float32)
    I = (rng.standard_normal((ni, d)) * np.exp(1.5 * rng.standard_normal((ni, 1)))).astype(np.float32)
    dup = rng.choice(ni, size=ni // 50, replace=False)
    I[dup] = I[rng.choice(ni, size=dup.size)]  # exact score ties
    U[3] = 0.0
    U[8:40] = -U[8:40]
    users = rng.permutation(nb).astype(np.int64)
    heavy = users[[1, 2]]
    rp, mc = _history(nb, ni, rng, heavy)
    val, idx = _run_fullsort(cuda, U, users, I, rp, mc, k)
    rows = np.concatenate([[0, 1, 2, int(np.nonzero(users == 3)[0][0])],
                           rng.choice(np.arange(3, nb), size=300 if d < 256 else 60, replace=False)])
    s = O.fmaf_scores(U, users[rows], I)
    for b, r in enumerate(rows):
        u = users[r]
        s[b, mc[rp[u]:rp[u + 1]]] = -1e10
    cv, ci = canonical_topk_fast(s, k)
    bad = np.nonzero(np.any(idx[rows] != ci, axis=1))[0]
    assert bad.size == 0, f"rows {rows[bad[:5]]}: {idx[rows[bad[0]]][:8]} vs {ci[bad[0]][:8]}"
    assert np.array_equal(val[rows].view(np.uint32), cv.view(np.uint32))
    assert np.sum(cv[1] == -1e10) > 0 and np.sum(cv[2] == -1e10) > 0  # the masked-heavy users' top k


def test_fullsort_sports_trained_tables(cuda):
    """Scores of a LightGCN table trained for 60 batches on the sports-shaped graph (the
    bench's evaluation: all 35,598 users, the train-item mask), modulo near-ties."""
    from rsx.engine import LightGCNEngine

    df = synth.shaped("sports", seed=0)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni = int(df.userID.max()) + 1, int(df.itemID.max()) + 1
    torch.manual_seed(999)
    eng = LightGCNEngine(tu, ti, nu, ni, 64, 3, 1e-2, 1e-2, cuda, seed=1, batch=2048)
    for j in range(60):
        eng.step(epoch=0, start=j * 2048)
    f = eng.forward().cpu().numpy()
    U, I = f[:nu], f[nu:]
    users = np.arange(nu, dtype=np.int64)
    assert _plan(nu, ni, 64) == (2, 9184)
    rp, mc = graph.history_csr(tu, ti, nu)
    val, idx = _run_fullsort(cuda, U, users, I, rp, mc)
    rows = np.random.default_rng(1).choice(nu, size=3000, replace=False)
    s = _cpu_scores(U, users, I, rp, mc, rows)
    cv, ci = canonical_topk_fast(s, 50)
    assert topk_equal_modulo_ties(idx[rows], ci, s, rtol=1e-5) == 0
    scale = np.abs(s).max(axis=1, keepdims=True)
    assert np.all(np.abs(val[rows] - cv) <= 1e-5 * scale)


def _hub_csr(n_rows, n_cols, n_hubs, seed):
    rng = np.random.default_rng(seed)
    deg = rng.geometric(0.15, size=n_rows)
    deg[::11] = 0
    hubs = rng.choice(n_rows, size=n_hubs, replace=False)
    deg[hubs] = rng.integers(33, 1500, size=n_hubs)
    deg = np.minimum(deg, n_cols)
    rows = np.repeat(np.arange(n_rows), deg)
    cols = np.concatenate([rng.choice(n_cols, size=k, replace=False) for k in deg])
    vals = rng.standard_normal(rows.size).astype(np.float32)
    return graph.to_csr(rows.astype(np.int64), cols.astype(np.int64), vals, n_rows, n_cols)


@pytest.mark.parametrize("d", [64, 256])
def test_spmm_out_of_launch_fixups_vs_torch(cuda, d):
    """> 1,024 hub rows: the partial sums' fixups run as their own launch (spmm.hip kInlineFixups)."""
    n_rows, n_cols = 30000, 20000
    rp, col, val = _hub_csr(n_rows, n_cols, 2500, seed=d)
    A = ops.DeviceCSR(rp, col, val, n_cols, cuda)
    assert A.n_long > 1024
    x = torch.randn(n_cols, d, generator=torch.Generator().manual_seed(d))
    rows = np.repeat(np.arange(n_rows), np.diff(rp))
    idx = torch.from_numpy(np.vstack([rows, col.astype(np.int64)]))
    ref = torch.sparse.mm(torch.sparse_coo_tensor(idx, torch.from_numpy(val), (n_rows, n_cols)), x).numpy()
    mag = torch.sparse.mm(torch.sparse_coo_tensor(idx, torch.from_numpy(np.abs(val)), (n_rows, n_cols)),
                          x.abs()).numpy()
    y = A.spmm(x.to(cuda)).cpu()
    deg = np.diff(rp)[:, None]
    err = np.abs(y.numpy() - ref)
    assert np.all(err <= 1e-5 * np.abs(ref) + 2e-7 * mag * np.sqrt(np.maximum(deg, 1)) + 1e-30)
    assert torch.equal(y, A.spmm(x.to(cuda)).cpu())  # deterministic


def _adam_first_step_bound(g, lr):
    """|p_gpu - p_cpu| bound after one Adam step: the first update is -lr g/(|g|+eps), so a
    gradient rounding difference delta moves it by at most lr |s(g+delta) - s(g)|,
    s(x) = x/(|x|+eps); delta = 2e-5 of the row's largest gradient (f32 sums in another
    order)."""
    delta = 2e-5 * np.abs(g).max(axis=1, keepdims=True) + 1e-30
    s = lambda x: x / (np.abs(x) + 1e-8)  # noqa: E731
    return lr * np.maximum(np.abs(s(g + delta) - s(g)), np.abs(s(g - delta) - s(g))) + 2e-7


@pytest.mark.parametrize("d,K,tags", [(256, 3, True), (256, 3, False), (64, 4, True), (64, 4, False),
                                      (256, 4, True), (64, 5, True)])
def test_lightgcn_hub_graph_vs_oracle(cuda, d, K, tags):
    """Three B=2048 LightGCN steps on a power-law graph with > 1,024 hub rows against
    the oracle's CPU training step, same triplets: every loss within rtol 1e-5; after
    the first step every parameter within Adam's rounding bound.  K = 4 is the
    reference's own default depth (src/configs/model/LightGCN.yaml:3, n_layers [4]):
    the step then takes the tag_rows + dense-forward + Horner path
    (csrc/step.hip rsx_lightgcn_step, K >= 4) instead of the stored-layer step."""
    from rsx.engine import LightGCNEngine

    df = synth.amazon_like(20000, 4000, 300000, seed=1)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni, lr, reg = int(df.userID.max()) + 1, 4000, 1e-3, 1e-2
    torch.manual_seed(999)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, d)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, d)).numpy()
    eng = LightGCNEngine(tu, ti, nu, ni, d, K, reg, lr, cuda, U0, I0, batch=2048)
    eng.use_tags = tags
    eng._fill_static()
    assert eng.adj.n_long > 1024
    cpu = O.LightGCNCPU(O.lightgcn_norm_adj_vec(tu, ti, nu, ni), U0, I0, K, reg, lr)
    samp = O.ReferenceSampler(tu, ti, seed=3)
    for step in range(3):
        trip = samp.next(2048)
        want = cpu.step(trip)
        eng.step(triplets=trip.to(cuda))
        got = eng.loss_out.item()
        assert abs(got - want) <= 1e-5 * abs(want), (step, got, want)
        if step == 0:
            g = np.concatenate([cpu.u.grad.numpy(), cpu.i.grad.numpy()])
            p_cpu = np.concatenate([cpu.u.detach().numpy(), cpu.i.detach().numpy()])
            p_gpu = eng.p.cpu().numpy()
            bound = _adam_first_step_bound(g, lr)
            assert np.all(np.abs(p_gpu - p_cpu) <= bound), np.abs(p_gpu - p_cpu).max()
    assert eng.halt.tolist() == [0, 0]


@pytest.mark.parametrize("K", [2, 4])
def test_layergcn_c_step_vs_oracle(cuda, K):
    """The LayerGCN batch as one C call (rsx_layergcn_step) against the oracle's CPU
    LayerGCN training step on a hub graph, same triplets, dropout 0 (the eval graph):
    losses rtol 1e-5 over three steps, step-1 parameters within Adam's rounding bound.
    K = 4 is LayerGCN.yaml's default n_layers (src/configs/model/LayerGCN.yaml:2)."""
    from rsx.layergcn import LayerGCNEngine

    df = synth.amazon_like(6000, 1500, 80000, seed=4)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni, d, lr, reg = int(df.userID.max()) + 1, 1500, 64, 1e-3, 1e-2
    torch.manual_seed(7)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, d)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, d)).numpy()
    eng = LayerGCNEngine(tu, ti, nu, ni, d, K, reg, lr, cuda, U0, I0)
    assert eng.norm_adj.n_long > 0
    cpu = O.LayerGCNCPU(tu, ti, nu, ni, U0, I0, K, reg, 0.0, lr=lr)
    cpu.pre_epoch()
    samp = O.ReferenceSampler(tu, ti, seed=5)
    prev = 0.0
    for step in range(3):
        trip = samp.next(2048)
        want = cpu.step(trip)
        eng.step(trip.to(cuda))
        now = eng.loss_acc.item()  # the step's loss is added to the f64 accumulator
        assert abs((now - prev) - want) <= 1e-5 * abs(want), (step, now - prev, want)
        prev = now
        if step == 0:
            g = np.concatenate([cpu.u.grad.numpy(), cpu.i.grad.numpy()])
            p_cpu = np.concatenate([cpu.u.detach().numpy(), cpu.i.detach().numpy()])
            assert np.all(np.abs(eng.p.cpu().numpy() - p_cpu) <= _adam_first_step_bound(g, lr))
