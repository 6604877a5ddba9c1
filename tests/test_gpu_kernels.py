"""HIP kernels (through the C ABI) against the CPU oracle and the reference's golden fixtures.

Tolerances: SpMM / propagation rtol 1e-5 (f32, different summation order: fma
chains vs torch's CPU addmm); BPR loss rtol 1e-5, gradients rtol 1e-4; Adam
parameters atol 1e-6 (one lr=1e-3 step); top-K indices exact except among
items whose scores tie within 1e-5 (fixture tie flags); integer work bit-exact.
"""
import numpy as np
import pytest
import torch

import rsx_oracle as O
from helpers import coo_from, eval_lists, metric_dict, params, topk_equal_modulo_ties, train_mask_pairs
from rsx import _lib as L
from rsx import graph, ops

pytestmark = pytest.mark.gpu


def _powerlaw_csr(n_rows, n_cols, seed, hub=600, empty_every=7):
    rng = np.random.default_rng(seed)
    deg = rng.geometric(0.15, size=n_rows)
    deg[::empty_every] = 0
    deg[3] = hub            # rows longer than one chunk -> fixup path
    deg[n_rows // 2] = 33   # just over one chunk
    deg = np.minimum(deg, n_cols)
    rows = np.repeat(np.arange(n_rows), deg)
    cols = np.concatenate([rng.choice(n_cols, size=k, replace=False) for k in deg]) if deg.sum() else np.zeros(0)
    vals = rng.standard_normal(rows.size).astype(np.float32)
    return graph.to_csr(rows.astype(np.int64), cols.astype(np.int64), vals, n_rows, n_cols)


@pytest.mark.parametrize("d", [32, 64, 128, 256])
def test_spmm_powerlaw_vs_torch(cuda, d):
    rp, col, val = _powerlaw_csr(900, 700, seed=d)
    A = ops.DeviceCSR(rp, col, val, 700, cuda)
    assert A.n_long >= 2
    x = torch.randn(700, d, generator=torch.Generator().manual_seed(d))
    rows = np.repeat(np.arange(900), np.diff(rp))
    At = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])), torch.from_numpy(val),
                                 (900, 700))
    ref = torch.sparse.mm(At, x)
    # f32 summation-order bound: |y - ref| <= 1e-5 |ref| + 2e-7 * (|A| |x|) * sqrt(deg)
    mag = torch.sparse.mm(torch.sparse_coo_tensor(At._indices(), At._values().abs(), At.shape), x.abs()).numpy()
    y = A.spmm(x.to(cuda)).cpu()
    err = np.abs(y.numpy() - ref.numpy())
    deg = np.diff(rp)[:, None]
    assert np.all(err <= 1e-5 * np.abs(ref.numpy()) + 2e-7 * mag * np.sqrt(np.maximum(deg, 1)) + 1e-30)
    # deterministic: same bits on a second launch
    y2 = A.spmm(x.to(cuda)).cpu()
    assert torch.equal(y, y2)


def test_spmm_empty_matrix(cuda):
    rp = np.zeros(17, dtype=np.int64)
    A = ops.DeviceCSR(rp, np.zeros(0, np.int32), np.zeros(0, np.float32), 5, cuda)
    y = A.spmm(torch.randn(5, 64, device=cuda))
    assert torch.count_nonzero(y).item() == 0


def _lgcn_csr(z, cuda):
    nu, ni = int(z["n_users"]), int(z["n_items"])
    rp, col, val = graph.lightgcn_norm_adj(z["train_u"], z["train_i"], nu, ni)
    return ops.DeviceCSR(rp, col, val, nu + ni, cuda), nu, ni


def test_lightgcn_forward_vs_fixture(cuda, golden):
    z = golden("lightgcn_small")
    A, nu, ni = _lgcn_csr(z, cuda)
    U0, I0 = params(z, "init.", "LightGCN")
    p = torch.from_numpy(np.concatenate([U0, I0])).to(cuda)
    s, h0, h1, f = (torch.empty_like(p) for _ in range(4))
    lib = L.lib()
    rc = lib.rsx_lightgcn_forward(A.struct, 64, 3, ops._p(p), ops._p(s), ops._p(h0), ops._p(h1), ops._p(f),
                                  ops._p(A.slab(64)), ops._stream())
    L.check(rc, "forward")
    f = f.cpu().numpy()
    np.testing.assert_allclose(f[:nu], z["fwd_user"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(f[nu:], z["fwd_item"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("variant", [L.RSX_BPR_LIGHTGCN, L.RSX_BPR_LAYERGCN, L.RSX_BPR_SMORE])
def test_bpr_vs_autograd(cuda, golden, variant):
    z = golden("lightgcn_small")
    nu, ni = int(z["n_users"]), int(z["n_items"])
    g = torch.Generator().manual_seed(variant)
    fin = torch.randn(nu + ni, 64, generator=g) * 0.1
    ego = torch.randn(nu + ni, 64, generator=g) * 0.1
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    reg = 1e-2
    fl = fin.clone().requires_grad_(True)
    el = ego.clone().requires_grad_(True)
    u, p_, n_ = trip[0], trip[1] + nu, trip[2] + nu
    ps = (fl[u] * fl[p_]).sum(1)
    ns = (fl[u] * fl[n_]).sum(1)
    if variant == L.RSX_BPR_LIGHTGCN:
        mf = -torch.log(1e-10 + torch.sigmoid(ps - ns)).mean()
        r = sum(torch.norm(x, p=2) for x in (el[u], el[p_], el[n_])) / trip.shape[1]
        loss = mf + reg * r
    elif variant == L.RSX_BPR_LAYERGCN:
        loss = torch.sum(-torch.nn.functional.logsigmoid(ps - ns)) + reg * sum(
            torch.sum(x ** 2) * 0.5 for x in (el[u], el[p_], el[n_]))
    else:
        reg_ = 0.5 * ((fl[u] ** 2).sum() + (fl[p_] ** 2).sum() + (fl[n_] ** 2).sum()) / 2048.0
        loss = -torch.mean(torch.nn.functional.logsigmoid(ps - ns)) + reg * reg_
    loss.backward()
    lo, gf, ge = ops.bpr(variant, fin.to(cuda), ego.to(cuda), nu, ni, trip.to(cuda), reg, batch_cfg=2048.0)
    assert abs(lo.item() - loss.item()) <= 1e-5 * abs(loss.item()) + 1e-7
    np.testing.assert_allclose(gf.cpu().numpy(), fl.grad.numpy(), rtol=1e-4, atol=1e-7)
    if variant != L.RSX_BPR_SMORE:
        np.testing.assert_allclose(ge.cpu().numpy(), el.grad.numpy(), rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("d", [64, 128])
def test_bpr_smore_rows_stores_what_smore_adds(cuda, d):
    """RSX_BPR_SMORE_ROWS on compact batch rows (triplets (b, b, B + b), n_users = B,
    n_items = 2B) writes every g_final row: the values RSX_BPR_SMORE adds into zeros,
    bit for bit, into a buffer that starts as garbage; the same loss; and the variant
    refuses any other row layout."""
    B = 300
    g = torch.Generator().manual_seed(11 + d)
    fin = (torch.randn(3 * B, d, generator=g) * 0.1).to(cuda)
    ar = torch.arange(B, device=cuda)
    trip = torch.stack([ar, ar, ar + B]).contiguous()
    l0, g0, _ = ops.bpr(L.RSX_BPR_SMORE, fin, None, B, 2 * B, trip, 1e-2, batch_cfg=2048.0)
    junk = torch.full((3 * B, d), float("nan"), device=cuda)
    l1, g1, _ = ops.bpr(L.RSX_BPR_SMORE_ROWS, fin, None, B, 2 * B, trip, 1e-2, batch_cfg=2048.0, g_final=junk,
                        compact_rows=True)
    assert torch.equal(l0, l1)
    assert torch.equal(g0 + 0.0, g1 + 0.0)  # (+0.0: a stored -0.0 equals the added +0.0)
    with pytest.raises(RuntimeError):
        ops.bpr(L.RSX_BPR_SMORE_ROWS, fin, None, B + 1, 2 * B - 1, trip, 1e-2, batch_cfg=2048.0, compact_rows=True)
    with pytest.raises(RuntimeError):  # internal variant: only the compact-rows loss may request it
        ops.bpr(L.RSX_BPR_SMORE_ROWS, fin, None, B, 2 * B, trip, 1e-2, batch_cfg=2048.0)
    # right sizes, wrong layout (a repeated row: stores would race): the device check NaN-poisons the loss
    bad = trip.clone()
    bad[1, 7] = 3
    l2, _, _ = ops.bpr(L.RSX_BPR_SMORE_ROWS, fin, None, B, 2 * B, bad, 1e-2, batch_cfg=2048.0, compact_rows=True)
    assert torch.isnan(l2).all()


def test_adam_vs_torch(cuda):
    g = torch.Generator().manual_seed(3)
    p = torch.randn(300, 64, generator=g)
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([ref], lr=1e-3)
    dp, dm, dv = p.clone().to(cuda), torch.zeros(300, 64, device=cuda), torch.zeros(300, 64, device=cuda)
    for step in range(1, 4):
        grad = torch.randn(300, 64, generator=g)
        grad[::5] = 0.0
        ref.grad = grad.clone()
        opt.step()
        ops.adam_(dp, grad.to(cuda), dm, dv, step=step, lr=1e-3)
    np.testing.assert_allclose(dp.cpu().numpy(), ref.detach().numpy(), rtol=0, atol=1e-6)


def test_lightgcn_fused_step_vs_fixture(cuda, golden):
    z = golden("lightgcn_small")
    A, nu, ni = _lgcn_csr(z, cuda)
    U0, I0 = params(z, "init.", "LightGCN")
    n = nu + ni
    p = torch.from_numpy(np.concatenate([U0, I0])).to(cuda)
    bufs = {k: torch.zeros(n, 64, device=cuda) for k in ("m", "v", "s", "h0", "h1", "f", "g", "r")}
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).to(cuda)
    loss = torch.zeros(1, device=cuda)
    lib = L.lib()
    ws = torch.empty(lib.rsx_bpr_ws_bytes(512), dtype=torch.uint8, device=cuda)
    st = L.LgcnStep()
    import ctypes as C

    st.adj = C.pointer(A.struct)
    st.n_users, st.n_items, st.d, st.n_layers, st.reg = nu, ni, 64, 3, 1e-2
    st.p, st.m, st.v = p.data_ptr(), bufs["m"].data_ptr(), bufs["v"].data_ptr()
    st.s, st.h0, st.h1 = bufs["s"].data_ptr(), bufs["h0"].data_ptr(), bufs["h1"].data_ptr()
    st.final_emb, st.g, st.r = bufs["f"].data_ptr(), bufs["g"].data_ptr(), bufs["r"].data_ptr()
    slab = A.slab(64)
    st.slab = slab.data_ptr() if slab is not None else 0
    st.triplets = trip.data_ptr()
    st.batch = 512
    st.adam = ops.adam_struct(1e-3, 1)
    st.loss_out = loss.data_ptr()
    st.ws, st.ws_bytes = ws.data_ptr(), ws.numel()
    L.check(lib.rsx_lightgcn_step(C.byref(st), ops._stream()), "step")
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    pu, pi = params(z, "step0_param.", "LightGCN")
    out = p.cpu().numpy()
    np.testing.assert_allclose(out[:nu], pu, rtol=0, atol=2e-6)
    np.testing.assert_allclose(out[nu:], pi, rtol=0, atol=2e-6)


@pytest.mark.parametrize("k", [5, 50])
def test_fullsort_topk_vs_fixture(cuda, golden, k):
    z = golden("lightgcn_small")
    nu, ni = int(z["n_users"]), int(z["n_items"])
    f = np.concatenate([z["fwd_user"], z["fwd_item"]])
    U = torch.from_numpy(f[:nu]).to(cuda)
    I = torch.from_numpy(f[nu:]).to(cuda)
    users = torch.from_numpy(z["init_valid_users"].astype(np.int64)).to(cuda)
    rp, mc = graph.history_csr(z["train_u"], z["train_i"], nu)
    val, idx = ops.fullsort_topk(U, users, I, torch.from_numpy(rp).to(cuda), torch.from_numpy(mc).to(cuda), k)
    scores = z["init_valid_scores"].copy()
    r, c = train_mask_pairs(z, z["init_valid_users"])
    scores[r, c] = -1e10
    cv, ci = O.canonical_topk(scores, k)
    idx = idx.cpu().numpy()
    assert topk_equal_modulo_ties(idx, ci, scores) == 0
    np.testing.assert_allclose(val.cpu().numpy(), cv, rtol=1e-5, atol=1e-6)
    if k == 50:
        ref = z["init_valid_topk_idx"].astype(np.int64)
        ties = z["init_valid_inner_tie"] | z["init_valid_boundary_tie"]
        assert np.all(np.all(idx == ref, axis=1) | ties)


@pytest.mark.parametrize("d", [32, 64, 128, 256])
def test_fullsort_random_sizes(cuda, d):
    """Ragged batch / item counts, all-masked-but-few users, exact vs a CPU canonical top-k."""
    g = torch.Generator().manual_seed(d)
    nb, ni, nu = 77, 1003, 120
    U = torch.randn(nu, d, generator=g)
    I = torch.randn(ni, d, generator=g)
    users = torch.randperm(nu, generator=g)[:nb]
    rng = np.random.default_rng(d)
    tu = np.repeat(np.arange(nu), 9)
    ti = rng.integers(0, ni, size=tu.size)
    # one user masks all but 20 items -> masked (-1e10) entries reach its top-50
    heavy = int(users[0])
    tu = np.concatenate([tu, np.full(ni - 20, heavy)])
    ti = np.concatenate([ti, np.arange(20, ni)])
    rp, mc = graph.history_csr(tu, ti, nu)
    val, idx = ops.fullsort_topk(U.to(cuda), users.to(cuda), I.to(cuda), torch.from_numpy(rp).to(cuda),
                                 torch.from_numpy(mc).to(cuda), 50)
    scores = (U[users].double() @ I.double().T).float().numpy()
    for b, u in enumerate(users.numpy()):
        scores[b, mc[rp[u]:rp[u + 1]]] = -1e10
    cv, ci = O.canonical_topk(scores, 50)
    assert topk_equal_modulo_ties(idx.cpu().numpy(), ci, scores, rtol=1e-5) == 0
    np.testing.assert_allclose(val.cpu().numpy(), cv, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("d", [32, 64, 128, 256])
@pytest.mark.parametrize("k", [1, 17, 50, 64])
def test_fullsort_screen_exact_vs_dense_scores(cuda, d, k):
    """The screened full-sort (k <= 64: bf16 bounds, exact f32 scores for candidates only)
    against the canonical top-k of score_dense's scores: both are the same fmaf chain over
    d, so the lists must match bit for bit -- an item the bounds wrongly dropped would
    show.  Heavy-tailed row norms (the margin eps |u||v_i| spans 1e-3..1e3 of a typical
    score), a zero user (every score ties at 0), negated users, masked runs, and a user
    count that needs the balanced split of the (user block, tile) work."""
    from helpers import canonical_topk_fast

    g = torch.Generator().manual_seed(d * 100 + k)
    nu, ni, nb = 36000, 6007, 35598  # 2 item chunks, more (block, chunk) waves than resident slots
    U = torch.randn(nu, d, generator=g) * torch.exp(torch.randn(nu, 1, generator=g))
    I = torch.randn(ni, d, generator=g) * torch.exp(2.0 * torch.randn(ni, 1, generator=g))
    U[7] = 0.0
    U[8:40] = -U[8:40]
    users = torch.randperm(nu, generator=g)[:nb]
    users[0] = 7
    rng = np.random.default_rng(d + k)
    tu = np.repeat(np.arange(nu), 5)
    ti = rng.integers(0, ni, size=tu.size)
    heavy = int(users[1])
    tu = np.concatenate([tu, np.full(ni - 30, heavy)])
    ti = np.concatenate([ti, np.arange(30, ni)])
    rp, mc = graph.history_csr(tu, ti, nu)
    Ud, Id, ud = U.to(cuda), I.to(cuda), users.to(cuda)
    val, idx = ops.fullsort_topk(Ud, ud, Id, torch.from_numpy(rp).to(cuda), torch.from_numpy(mc).to(cuda), k)
    rows = np.concatenate([np.arange(64), rng.choice(np.arange(64, nb), size=1200, replace=False)])
    scores = ops.score_dense(Ud, ud[torch.from_numpy(rows).to(cuda)].contiguous(), Id).cpu().numpy()
    for b, u in enumerate(users.numpy()[rows]):
        scores[b, mc[rp[u]:rp[u + 1]]] = -1e10
    cv, ci = canonical_topk_fast(scores, k)
    idx, val = idx.cpu().numpy()[rows], val.cpu().numpy()[rows]
    bad = np.nonzero(np.any(idx != ci, axis=1))[0]
    assert bad.size == 0, f"rows {bad[:5]}: {idx[bad[0]][:8]} vs {ci[bad[0]][:8]}"
    assert np.array_equal(val.view(np.uint32), cv.view(np.uint32))


def test_score_dense_and_gather(cuda):
    g = torch.Generator().manual_seed(1)
    U = torch.randn(50, 64, generator=g)
    I = torch.randn(333, 64, generator=g)
    users = torch.tensor([3, 0, 49, 7])
    out = ops.score_dense(U.to(cuda), users.to(cuda), I.to(cuda)).cpu()
    np.testing.assert_allclose(out.numpy(), (U[users] @ I.T).numpy(), rtol=1e-5, atol=1e-5)
    gr = ops.gather_rows(U.to(cuda), users.to(cuda)).cpu()
    assert torch.equal(gr, U[users])


def test_sampler_properties(cuda, golden):
    z = golden("lightgcn_small")
    nu = int(z["n_users"])
    tu, ti = z["train_u"], z["train_i"]
    s = ops.DeviceSampler(tu, ti, nu, cuda, seed=5)
    E = tu.size
    hist = {(int(a), int(b)) for a, b in zip(tu, ti)}
    all_items = set(int(x) for x in np.unique(ti))
    seen = []
    for start in range(0, E, 512):
        t = s.sample(epoch=0, start=start, batch=512).cpu().numpy()
        assert t.shape[0] == 3 and t.shape[1] == min(512, E - start)
        for u, p, n in t.T:
            assert (int(u), int(p)) in hist
            assert (int(u), int(n)) not in hist
            assert int(n) in all_items
        seen.append(t[:2])
    pairs = np.concatenate(seen, axis=1)
    keys = pairs[0] * 100000 + pairs[1]
    assert np.array_equal(np.sort(keys), np.sort(tu.astype(np.int64) * 100000 + ti))  # a permutation
    t0 = s.sample(epoch=0, start=0, batch=512).cpu().numpy()
    t1 = s.sample(epoch=1, start=0, batch=512).cpu().numpy()
    assert not np.array_equal(t0, t1)
    assert np.array_equal(t0, s.sample(epoch=0, start=0, batch=512).cpu().numpy())


def test_sample_epoch_matches_per_batch(cuda, golden):
    z = golden("lightgcn_small")
    s = ops.DeviceSampler(z["train_u"], z["train_i"], int(z["n_users"]), cuda, seed=9)
    buf = s.sample_epoch(epoch=3, batch=512)
    for j, start in enumerate(range(0, s.n_inter, 512)):
        a = ops.DeviceSampler.batch_view(buf, s.n_inter, 512, j).cpu()
        b = s.sample(epoch=3, start=start, batch=512).cpu()
        assert torch.equal(a, b)


@pytest.mark.parametrize("n_slices", [1, 3, 7, 64, 1000, 5000])
def test_sample_epoch_slices_recut_the_same_stream(cuda, golden, n_slices):
    """rsx_sample_epoch_slices: slice j = epoch positions [j E // S, (j+1) E // S) of the
    same stream rsx_sample_epoch writes (the sharded trainers' balanced epochs, every
    interaction once, sizes within one of each other)."""
    z = golden("lightgcn_small")
    s = ops.DeviceSampler(z["train_u"], z["train_i"], int(z["n_users"]), cuda, seed=9)
    E = s.n_inter
    if n_slices > E:
        with pytest.raises(ValueError):
            s.sample_epoch_slices(epoch=3, n_slices=n_slices)
        return
    plain = s.sample_epoch(epoch=3, batch=E).view(3, E).cpu()
    buf = s.sample_epoch_slices(epoch=3, n_slices=n_slices)
    sizes = []
    for j in range(n_slices):
        a, e = ops.DeviceSampler.slice_bounds(E, n_slices, j)
        v = ops.DeviceSampler.slice_view(buf, E, n_slices, j).cpu()
        assert torch.equal(v, plain[:, a:e])
        sizes.append(e - a)
    assert sum(sizes) == E and max(sizes) - min(sizes) <= 1 and min(sizes) >= 1


class _EvalStub:
    """The two EvalDataLoader members the device metric path reads."""

    def __init__(self, items, dev):
        import torch

        self.lens = np.array([len(x) for x in items], dtype=np.int64)
        rp = np.concatenate([[0], np.cumsum(self.lens)]).astype(np.int64)
        col = np.concatenate([np.sort(np.asarray(x, np.int64)) for x in items]).astype(np.int32)
        self.csr = (torch.from_numpy(rp).to(dev), torch.from_numpy(col).to(dev))

    def eval_csr(self):
        return self.csr

    def get_eval_len_list(self):
        return self.lens


@pytest.mark.parametrize("fx", ["lightgcn_small", "layergcn_small", "layergcn_drop_small", "smore_small"])
def test_topk_metrics_device_equals_reference_dicts(cuda, golden, fx):
    """rsx_topk_metrics + the evaluator's rounding == the reference's metric dicts (bit-exact)."""
    import torch

    from rsx.config import Config
    from rsx.evaluator import TopKEvaluator

    z = golden(fx)
    ev = TopKEvaluator(Config("LightGCN", "baby", {"use_gpu": False}))
    tags = [k[: -len("_metric_keys")] for k in z if k.endswith("_metric_keys")]
    for tag in tags:
        split = "test" if tag.endswith("test") else "valid"
        stub = _EvalStub(eval_lists(z, split), cuda)
        topk = torch.from_numpy(z[tag + "_topk_idx"].astype(np.int64)).to(cuda)
        assert ev.evaluate_device(topk, stub) == metric_dict(z, tag), tag


@pytest.mark.parametrize("k", [50, 64, 100])
def test_topk_metrics_device_bitwise_vs_numpy(cuda, k):
    """Large random case: the per-cutoff means before rounding equal the numpy restatement
    (reference metrics.py formulas, mean over users in numpy's order) bit for bit.  k = 64
    is the lockstep search's 64-bit hit-mask edge, k = 100 its serial fallback."""
    import torch

    from rsx import evaluator as E
    from rsx import ops

    rng = np.random.default_rng(5)
    n, ni = 6000, 3000
    items = [rng.choice(ni, size=int(rng.integers(1, 40)), replace=False) for _ in range(n)]
    rows = []
    for x in items:  # each ranked list: up to 10 true items, then distinct non-items, shuffled within the top 20
        first = x[: int(rng.integers(0, min(10, x.size) + 1))]
        rest = rng.permutation(np.setdiff1d(np.arange(ni), x))[: k - first.size]
        r = np.concatenate([first, rest])
        rng.shuffle(r[:20])
        rows.append(r)
    topk = np.stack(rows)
    pos = np.array([len(x) for x in items])
    hit = E.hit_matrix(topk, items)
    cuts = [1, 5, 10, 20, k]
    stub = _EvalStub(items, cuda)
    gain = torch.from_numpy(1.0 / np.log2(np.arange(1, k + 1, dtype=np.float64) + 1)).to(cuda)
    sums = ops.topk_metrics(torch.from_numpy(topk.astype(np.int64)).to(cuda), *stub.eval_csr(), cuts, gain).cpu().numpy()
    for row, fn in enumerate((E.recall, E.precision, E.ndcg, E.average_precision)):
        want = fn(hit, pos)
        for j, c in enumerate(cuts):
            assert sums[row, j] / n == want[c - 1], (fn.__name__, c)
    want2 = E.recall2(hit, pos)
    for j, c in enumerate(cuts):
        assert sums[4, j] / pos.sum() == want2[c - 1]
    # the parallel-order sums (rsx_topk_metrics_fast): deterministic, within the
    # stated bound of the user-order sums, the same rounded dict
    args = (torch.from_numpy(topk.astype(np.int64)).to(cuda), *stub.eval_csr(), cuts, gain)
    fast = ops.topk_metrics(*args, exact=False).cpu().numpy()
    assert np.array_equal(fast, ops.topk_metrics(*args, exact=False).cpu().numpy())
    assert np.array_equal(fast[4], sums[4])  # integer hit counts: exact in any order
    for row in range(4):
        for j in range(len(cuts)):
            assert abs(fast[row, j] - sums[row, j]) <= E.sum_order_bound(n, sums[row, j])
    metrics = ["recall", "recall2", "precision", "ndcg", "map"]
    got = E.device_metric_dict(args[0], *stub.eval_csr(), metrics, cuts, int(pos.sum()))
    for m, fn in zip(metrics, (E.recall, E.recall2, E.precision, E.ndcg, E.average_precision)):
        want = fn(hit, pos)
        for c in cuts:
            assert got[f"{m}@{c}"] == float(round(np.float64(want[c - 1]), 4)), (m, c)


@pytest.mark.parametrize("seed", [0, 1])
def test_device_edge_dropout_graph_equals_host_builder(cuda, seed):
    """LayerGCN's per-epoch masked adjacency built on the device (DeviceEdgeDropout)
    == the host builder (graph.layergcn_masked_adj, pinned against the reference's
    tensors by the e2e parity test) on the same kept edges: rowptr, col and the
    float32 values bit for bit.  Plus the draw: exactly keep_len distinct edges, for
    the multinomial and the uniform epochs; an edge with weight 0 never kept by the
    multinomial."""
    from rsx.layergcn import DeviceEdgeDropout

    rng = np.random.default_rng(seed)
    nu, ni = 700, 300
    pairs = np.unique(np.stack([rng.integers(0, nu, 9000), (rng.zipf(1.4, 9000) - 1) % ni], 1), axis=0)
    e_u, e_i = pairs[:, 0].astype(np.int64), pairs[:, 1].astype(np.int64)
    w = graph.layergcn_edge_values(e_u, e_i, nu, ni)
    w[5] = 0.0
    dd = DeviceEdgeDropout(e_u, e_i, nu, ni, w, cuda, chunk=32)
    E = e_u.size
    keep_len = int(E * 0.9)
    for pruning_random in (False, True):
        torch.manual_seed(seed)
        mask = dd.keep_mask(keep_len, pruning_random)
        m = mask.cpu().numpy()
        assert int(m.sum()) == keep_len
        if not pruning_random:
            assert not m[5]
        rp, col, val = dd.build(mask, keep_len)
        want = graph.layergcn_masked_adj(e_u[m], e_i[m], nu, ni)
        assert np.array_equal(rp.cpu().numpy(), want[0])
        assert np.array_equal(col.cpu().numpy(), want[1])
        assert np.array_equal(val.cpu().numpy().view(np.uint32), want[2].view(np.uint32))
        A = dd.epoch_graph(0.1, pruning_random)
        assert A.nnz == 2 * keep_len and A.n_rows == nu + ni
        x = torch.randn(nu + ni, 64, device=cuda)
        ref = torch.sparse_csr_tensor(A.rowptr, A.col.long(), A.val, (nu + ni, nu + ni)).to_dense() @ x
        assert torch.allclose(A.spmm(x), ref, rtol=1e-5, atol=1e-6)
        # the device-rebound schedule (template layout) == a fresh host schedule, bit for bit
        assert A.rowptr_host is None and A.n_long > 0
        B = ops.DeviceCSR.from_device(A.rowptr, A.col, A.val, nu + ni, 32)
        for d in (32, 64, 128):
            xd = torch.randn(nu + ni, d, device=cuda)
            assert torch.equal(A.spmm(xd), B.spmm(xd)), d


@pytest.mark.parametrize("drop", [0.1, 0.5, 0.97])
def test_schedule_rebind_on_random_subgraphs(cuda, drop):
    """rsx_csr_schedule_rebind: a CSR whose rows are random subsets of a template's
    (long rows that shrink below a chunk or to nothing included) multiplied on the
    rebound template layout equals the product on its own host schedule, bit for bit."""
    rng = np.random.default_rng(int(drop * 100))
    n = 1500
    deg = np.minimum(rng.zipf(1.3, n), 700)
    rows = np.repeat(np.arange(n), deg)
    cols = rng.integers(0, n, rows.size)
    t_rp = np.zeros(n + 1, np.int64)
    t_rp[1:] = np.cumsum(deg)
    T = ops.DeviceCSR(t_rp, cols.astype(np.int32), np.ones(rows.size, np.float32), n, cuda, 32)
    keep = rng.random(rows.size) >= drop
    keep[t_rp[np.argmax(deg)]:t_rp[np.argmax(deg) + 1]] = False  # the largest hub loses every edge
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(rows[keep], minlength=n))
    col = torch.from_numpy(cols[keep].astype(np.int32)).to(cuda)
    val = torch.from_numpy(rng.standard_normal(int(keep.sum())).astype(np.float32)).to(cuda)
    A = ops.DeviceCSR.rebind(T, torch.from_numpy(rp).to(cuda), col, val)
    B = ops.DeviceCSR(rp, col, val, n, cuda, 32)
    assert T.n_long > 0 and B.n_work <= A.n_work
    for d in (64, 256):
        x = torch.randn(n, d, device=cuda)
        assert torch.equal(A.spmm(x), B.spmm(x)), d


@pytest.mark.parametrize("K,d", [(2, 64), (3, 64), (3, 128), (2, 256), (3, 32), (4, 64), (4, 256)])
def test_batch_row_tags_equal_dense_step(cuda, K, d):
    """rsx_lgcn_step.row_tag (last forward layer on the batch rows, sparse G, G/R
    cleared on the batch rows) gives the dense path's parameters and losses on a
    power-law graph with hub rows; G and R are all-zero between tagged steps."""
    from rsx import synth
    from rsx.engine import LightGCNEngine

    df = synth.amazon_like(3000, 800, 30000, seed=3)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni = int(df.userID.max()) + 1, 800
    torch.manual_seed(5)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, d)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, d)).numpy()
    engs = []
    for tags in (True, False):
        e = LightGCNEngine(tu, ti, nu, ni, d, K, 1e-2, 1e-3, cuda, U0, I0, seed=0, batch=512)
        e.use_tags = tags
        e._fill_static()
        engs.append(e)
    assert engs[0].adj.n_long > 0  # hub rows split over several work items
    for s in range(0, 3 * 512, 512):
        for e in engs:
            e.step(epoch=0, start=s)
    torch.cuda.synchronize()
    a, b = engs
    assert torch.count_nonzero(a.g).item() == 0 and torch.count_nonzero(a.r).item() == 0
    # the one-launch BPR's occurrence counts are cleared by the Adam layer, its done counter re-armed
    n = nu + ni
    assert a.use_reg_cnt and torch.count_nonzero(a.reg_cnt[: 3 * n + 1]).item() == 0
    np.testing.assert_allclose(a.loss_acc.item(), b.loss_acc.item(), rtol=1e-9)
    # the moments carry the atomics-order rounding of g (~1e-7 here); Adam's step normalises
    # g by its RMS, which amplifies that rounding where g ~ 0 (up to ~lr per step): p 1e-5
    for name, tol in (("p", 1e-5), ("m", 1e-6), ("v", 1e-6)):
        np.testing.assert_allclose(getattr(a, name).cpu().numpy(), getattr(b, name).cpu().numpy(), rtol=0,
                                   atol=tol, err_msg=name)
    # the forward for evaluation (dense) is unaffected
    a.invalidate()
    b.invalidate()
    np.testing.assert_allclose(a.forward().cpu().numpy(), b.forward().cpu().numpy(), rtol=0, atol=1e-6)


@pytest.mark.parametrize("K", [1, 2, 3])
def test_layergcn_c_step_equals_python_sequence(cuda, K, monkeypatch):
    """rsx_layergcn_step (the LayerGCN batch as one C call) against the Python-issued
    kernel sequence it replaces: loss and parameters / moments after 3 batches (the
    BPR scatter adds repeated rows in either order: atol 1e-6)."""
    from rsx import synth
    from rsx.layergcn import LayerGCNEngine

    df = synth.amazon_like(1500, 500, 15000, seed=12)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni = int(df.userID.max()) + 1, 500
    torch.manual_seed(2)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, 64)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, 64)).numpy()
    engs = [LayerGCNEngine(tu, ti, nu, ni, 64, K, 1e-4, 1e-3, cuda, U0, I0) for _ in range(2)]
    assert engs[0].norm_adj.n_long > 0
    g = torch.Generator().manual_seed(4)
    for _ in range(3):
        t = torch.stack([torch.randint(0, nu, (512,), generator=g), torch.randint(0, ni, (512,), generator=g),
                         torch.randint(0, ni, (512,), generator=g)]).to(cuda)
        for e, flag in zip(engs, ("1", "0")):
            monkeypatch.setenv("RSX_LAYERGCN_CSTEP", flag)
            e.step(t)
    torch.cuda.synchronize()
    a, b = engs
    np.testing.assert_allclose(a.loss_acc.item(), b.loss_acc.item(), rtol=1e-9)
    # the moments carry the atomics-order rounding of g (~1e-7 here); Adam's step normalises
    # g by its RMS, which amplifies that rounding where g ~ 0 (up to ~lr per step): p 1e-5
    for name, tol in (("p", 1e-5), ("m", 1e-6), ("v", 1e-6)):
        np.testing.assert_allclose(getattr(a, name).cpu().numpy(), getattr(b, name).cpu().numpy(), rtol=0,
                                   atol=tol, err_msg=name)


@pytest.mark.parametrize("K,tags,fused_bpr", [(3, True, True), (3, True, False), (3, False, False),
                                               (4, True, True), (4, False, False), (5, True, False)])
def test_nan_loss_halts_the_fused_step(cuda, K, tags, fused_bpr):
    """A batch whose loss is NaN sets the step's halt flag to {1, its tag}; that step's
    Adam update and every later one are skipped, so p / m / v stay bit for bit those
    after the last finite batch (the reference stops before backward,
    src/common/trainer.py:192-203).  Every step path: the stored-layer step (K = 2, 3),
    the tag_rows + dense path (K >= 4, the reference's default depth), the untagged
    dense path, with the one-launch or the two-launch BPR."""
    from rsx import synth
    from rsx.engine import LightGCNEngine

    df = synth.amazon_like(2000, 600, 20000, seed=8)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni = int(df.userID.max()) + 1, 600
    torch.manual_seed(9)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, 64)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, 64)).numpy()
    eng = LightGCNEngine(tu, ti, nu, ni, 64, K, 1e-2, 1e-3, cuda, U0, I0, seed=0, batch=512)
    eng.use_tags, eng.use_reg_cnt = tags, fused_bpr
    eng._fill_static()
    g = torch.Generator().manual_seed(3)
    trip = lambda: torch.stack([torch.randint(0, nu, (512,), generator=g), torch.randint(0, ni, (512,), generator=g),  # noqa: E731
                                torch.randint(0, ni, (512,), generator=g)]).to(cuda)
    for _ in range(2):
        eng.step(triplets=trip())
    torch.cuda.synchronize()
    assert eng.halt.tolist() == [0, 0]
    eng.p[5, 3] = float("nan")  # user 5's row poisons any batch that holds user 5
    snap = [x.clone() for x in (eng.p, eng.m, eng.v)]
    bad = trip()
    bad[0, 7] = 5
    eng.step(triplets=bad)
    eng.step(triplets=trip())
    torch.cuda.synchronize()
    assert eng.halt.tolist() == [1, 3]
    assert np.isnan(eng.loss_out.item())
    for a, b in zip((eng.p, eng.m, eng.v), snap):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_tagged_step_vs_fixture(cuda, golden):
    """The engine's default step (batch-row tags, stored layers, one-launch BPR with the
    regulariser as counts) against the reference's first LightGCN step (fixture)."""
    from rsx.engine import LightGCNEngine

    z = golden("lightgcn_small")
    nu, ni = int(z["n_users"]), int(z["n_items"])
    U0, I0 = params(z, "init.", "LightGCN")
    eng = LightGCNEngine(z["train_u"], z["train_i"], nu, ni, 64, 3, 1e-2, 1e-3, cuda, U0, I0, batch=512)
    assert eng.use_tags and eng.use_reg_cnt
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).to(cuda)
    eng.step(triplets=trip)
    ref = float(z["step0_loss"])
    assert abs(eng.loss_out.item() - ref) <= 1e-5 * abs(ref)
    pu, pi = params(z, "step0_param.", "LightGCN")
    out = eng.p.cpu().numpy()
    np.testing.assert_allclose(out[:nu], pu, rtol=0, atol=2e-6)
    np.testing.assert_allclose(out[nu:], pi, rtol=0, atol=2e-6)


@pytest.mark.parametrize("d,world,n_max", [(64, 2, 300), (128, 4, 777), (128, 1, 64)])
def test_rowx_pack_combine_equals_the_torch_statement(cuda, d, world, n_max):
    """csrc/rowx.hip (data-parallel SMORE's batch-row gradient exchange) against its CPU
    statement (rsx.smore_dist.RowGradExchange._pack_torch / _combine_torch): the packs of
    `world` ranks, a hot repeated row, unequal batches (pad entries), garbage off the rows;
    the packed words, the union rows and the rebuilt tables bit for bit; a second call
    (the tag moves on, stale first-occurrence keys must not count)."""
    import ctypes as C

    from rsx.smore_dist import RowGradExchange

    class _C:  # a stand-in communicator: one process holds every rank's pack
        sim, rank = None, 0

        def __init__(self, w):
            self.world = w

    n_rows = 5000
    lib = L.lib()
    for call in range(2):
        g = torch.Generator().manual_seed(7 + call)
        ex_h = RowGradExchange(_C(world), n_rows, d, n_max, "cpu")
        ex_d = RowGradExchange(_C(world), n_rows, d, n_max, cuda) if call == 0 else ex_d
        tabs_h = [torch.full((n_rows, d), float("nan")) for _ in range(4)]
        tabs_d = [t.to(cuda) for t in tabs_h]
        for r in range(world):
            n = n_max - (r % 2) * 5
            rows = torch.randint(0, n_rows, (n,), generator=g)
            rows[: n // 4] = rows[1]
            full = [torch.randn(n_rows, d, generator=g) for _ in range(4)]  # one value per row (rows repeat)
            for th, td, f in zip(tabs_h, tabs_d, full):
                th[rows] = f[rows]
                td[rows.to(cuda)] = f[rows].to(cuda)
            ex_h._pack_torch(rows, tabs_h, ex_h.packed[r])
            tp = (C.c_void_p * 4)(*[t.data_ptr() for t in tabs_d])
            rd = rows.to(cuda)
            L.check(lib.rsx_rowx_pack(rd.data_ptr(), n, n_max, tp, 4, d, ex_d.lead.data_ptr(), ex_d.tag.data_ptr(),
                                      ex_d.packed[r].data_ptr(), ops._stream()), "rsx_rowx_pack")
            torch.cuda.synchronize()
            assert torch.equal(ex_d.packed[r].cpu().view(torch.int32), ex_h.packed[r].view(torch.int32)), r
        ex_h._combine_torch(tabs_h)
        tp = (C.c_void_p * 4)(*[t.data_ptr() for t in tabs_d])
        L.check(lib.rsx_rowx_combine(ex_d.packed.data_ptr(), world, n_max, tp, 4, d, ex_d.union.data_ptr(),
                                     ops._stream()), "rsx_rowx_combine")
        torch.cuda.synchronize()
        assert torch.equal(ex_d.union.cpu(), ex_h.union)
        u = ex_h.union.unique()
        for th, td in zip(tabs_h, tabs_d):
            assert torch.equal(td.cpu()[u].view(torch.int32), th[u].view(torch.int32))
