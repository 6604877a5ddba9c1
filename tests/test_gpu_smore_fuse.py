"""The fused SMORE kernels (csrc/smore_fuse.hip through rsx.smore_fuse) against the
reference's torch ops (src/models/smore.py:262-272 gates, :299-317 item views,
:320-341 preference block, :380-387 InfoNCE) evaluated in fp32 with autograd, on
the same inputs: outputs and every input / weight gradient within 1e-4 of the
tensor's scale (f32 sums in another order).  Dropout > 0 checks the kernel's mask
against a numpy restatement of its hash, then the same torch ops with that mask."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _close(got, want, name, tol=1e-4):
    g = got.detach().double().cpu().numpy()
    w = want.detach().double().cpu().numpy()
    scale = max(np.abs(w).max(), 1e-30)
    err = np.abs(g - w).max() if g.size else 0.0
    assert err <= tol * scale, f"{name}: max err {err:.3g} vs scale {scale:.3g}"


def _lin(d, gen, dev, bias=True):
    m = torch.nn.Linear(d, d, bias=bias)
    with torch.no_grad():
        m.weight.copy_(torch.randn(d, d, generator=gen) / d ** 0.5)
        if bias:
            m.bias.copy_(torch.randn(d, generator=gen) * 0.1)
    return m.to(dev)


def _drop_mask_np(seed, gate, n, d, p):
    """The kernel's dropout scale per element (mix32 of seed * phi + gate << 58 + row * d + f)."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    rows = np.arange(n, dtype=np.uint64)[:, None]
    feats = np.arange(d, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + (np.uint64(gate) << np.uint64(58))
             + rows * np.uint64(d) + feats) & M
        x ^= x >> np.uint64(33)
        x = (x * np.uint64(0xFF51AFD7ED558CCD)) & M
        x ^= x >> np.uint64(33)
        x = (x * np.uint64(0xC4CEB9FE1A85EC53)) & M
        x ^= x >> np.uint64(33)
    u = (x & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    thr = np.uint32(min(np.float32(p) * np.float32(4294967296.0), np.float32(4294967295.0)))
    scale = np.float32(1.0 / (1.0 - p))
    return np.where(u >= thr, scale, np.float32(0)).astype(np.float32)


@pytest.mark.parametrize("d,n,mul", [(64, 7050, False), (128, 1001, False), (64, 37, True), (128, 5, True)])
def test_gates_vs_torch(cuda, d, n, mul):
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(d + n)
    mk = lambda: torch.randn(n, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    cv, ct, cf, item = mk(), mk(), mk(), mk()
    gates = [torch.nn.Sequential(_lin(d, gen, cuda), torch.nn.Sigmoid()) for _ in range(3)]
    up = [torch.randn(n, d, generator=gen).to(cuda) for _ in range(3)]
    params = [cv, ct, cf, item] + [p for gm in gates for p in gm.parameters()]

    def ref():
        outs = []
        for c, gm in zip((cv, ct, cf), gates):
            outs.append(item * gm(c) if mul else item + 0.7 * gm(c))
        return outs

    want = ref()
    wg = torch.autograd.grad(sum((o * u).sum() for o, u in zip(want, up)), params)
    got = SF.gates(cv, ct, cf, item, *gates, 0.7, mul)
    gg = torch.autograd.grad(sum((o * u).sum() for o, u in zip(got, up)), params)
    for i, (a, b) in enumerate(zip(got, want)):
        _close(a, b, f"out{i}")
    for i, (a, b) in enumerate(zip(gg, wg)):
        _close(a, b, f"grad{i}")


@pytest.mark.parametrize("d,n", [(64, 7050), (128, 1001)])
def test_gates_saved_equals_recompute(cuda, d, n, monkeypatch):
    """rsx_smore_gates_saved (residual mode): the backward from the forward's sigmoid rows
    against the backward that recomputes them: every gradient agrees to float rounding."""
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(3 * d + n)
    mk = lambda: torch.randn(n, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    cv, ct, cf, item = mk(), mk(), mk(), mk()
    gates = [torch.nn.Sequential(_lin(d, gen, cuda), torch.nn.Sigmoid()) for _ in range(3)]
    up = [torch.randn(n, d, generator=gen).to(cuda) for _ in range(3)]
    params = [cv, ct, cf, item] + [p for gm in gates for p in gm.parameters()]
    res = {}
    for saved in (True, False):
        monkeypatch.setattr(SF, "_SAVED", saved)
        got = SF.gates(cv, ct, cf, item, *gates, 0.7, False)
        res[saved] = tuple(got) + tuple(torch.autograd.grad(sum((o * u).sum() for o, u in zip(got, up)), params))
    for i, (x, y) in enumerate(zip(res[True], res[False])):
        scale = float(y.abs().max()) + 1e-30
        assert float((x - y).abs().max()) <= 1e-6 * scale, i


class _PrefModel(torch.nn.Module):
    """The reference's preference-module submodules (smore.py:104-120)."""

    def __init__(self, d, gen, dev, p):
        super().__init__()
        self.query_v = torch.nn.Sequential(_lin(d, gen, dev), torch.nn.Tanh(), _lin(d, gen, dev, bias=False))
        self.query_t = torch.nn.Sequential(_lin(d, gen, dev), torch.nn.Tanh(), _lin(d, gen, dev, bias=False))
        self.gate_image_prefer = torch.nn.Sequential(_lin(d, gen, dev), torch.nn.Sigmoid())
        self.gate_text_prefer = torch.nn.Sequential(_lin(d, gen, dev), torch.nn.Sigmoid())
        self.gate_fusion_prefer = torch.nn.Sequential(_lin(d, gen, dev), torch.nn.Sigmoid())
        self.dropout = torch.nn.Dropout(p)

    def ref(self, C, IE, TE, FE, masks):
        sv = torch.softmax(self.query_v(FE), dim=-1)
        st = torch.softmax(self.query_t(FE), dim=-1)
        a1, a2 = sv * IE, st * TE
        ip, tp, fp = self.gate_image_prefer(C), self.gate_text_prefer(C), self.gate_fusion_prefer(C)
        if masks is not None:
            ip, tp, fp = ip * masks[0], tp * masks[1], fp * masks[2]
        side = torch.mean(torch.stack([ip * a1, tp * a2, fp * FE]), dim=0)
        return C + side, side


@pytest.mark.parametrize("d,n,p", [(64, 26495, 0.0), (128, 1000, 0.0), (64, 333, 0.1), (128, 45, 0.3)])
def test_preference_vs_torch(cuda, d, n, p):
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(d * 7 + n)
    mk = lambda: torch.randn(n, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    C_, IE, TE, FE = mk(), mk(), mk(), mk()
    m = _PrefModel(d, gen, cuda, p).train()
    seed = torch.tensor([12345], dtype=torch.int64, device=cuda)
    masks = None
    if p > 0:
        masks = [torch.from_numpy(_drop_mask_np(12345, k, n, d, p)).to(cuda) for k in range(3)]
        keep = float(np.mean([(mm > 0).float().mean().item() for mm in masks]))
        assert abs(keep - (1 - p)) < 0.02, keep
    up_a, up_s = torch.randn(n, d, generator=gen).to(cuda), torch.randn(n, d, generator=gen).to(cuda)
    params = [C_, IE, TE, FE] + list(m.parameters())
    wa, ws = m.ref(C_, IE, TE, FE, masks)
    wg = torch.autograd.grad((wa * up_a).sum() + (ws * up_s).sum(), params)
    ga, gs = SF.preference(m, C_, IE, TE, FE, seed)
    gg = torch.autograd.grad((ga * up_a).sum() + (gs * up_s).sum(), params)
    _close(ga, wa, "all")
    _close(gs, ws, "side")
    names = ["content", "image", "text", "fusion"] + [k for k, _ in m.named_parameters()]
    for name, a, b in zip(names, gg, wg):
        _close(a, b, name)
    # eval mode: no dropout whatever p
    m.eval()
    ea, _ = SF.preference(m, C_, IE, TE, FE, seed)
    _close(ea, m.ref(C_, IE, TE, FE, None)[0], "eval all")


# n = 20000 > the LDS copy's 16384 ids: pref_segsum's global-memory form
@pytest.mark.parametrize("d,N,n,p", [(64, 3000, 6144, 0.0), (128, 5000, 6144, 0.1), (128, 700, 999, 0.0),
                                     (64, 9000, 20000, 0.0)])
def test_preference_rows_vs_torch_and_deterministic(cuda, d, N, n, p):
    """The batch-row preference block (rsx_smore_pref_rows with per-occurrence row
    gradients + pref_segsum): repeated rows (a batch's popular items), gradients of the
    full tables vs torch autograd of the gathered rows (1e-4 of scale), and bit-identical
    gradients on a second run (no float atomics: a fixed summation order per row)."""
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(d + n)
    mk = lambda: torch.randn(N, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    C_, IE, TE, FE = mk(), mk(), mk(), mk()
    m = _PrefModel(d, gen, cuda, p).train()
    hot = torch.randint(0, 40, (n // 3,), generator=gen)  # heavy repeats
    rows = torch.cat([hot, torch.randint(0, N, (n - n // 3,), generator=gen)])[torch.randperm(n, generator=gen)]
    rows = rows.to(cuda)
    seed = torch.tensor([777], dtype=torch.int64, device=cuda)
    up = [torch.randn(n, d, generator=gen).to(cuda) for _ in range(3)]
    params = [C_, IE, TE, FE] + list(m.parameters())

    def run():
        a, s_, c = SF.preference_rows(m, C_, IE, TE, FE, rows, seed)
        return a, s_, c, torch.autograd.grad((a * up[0]).sum() + (s_ * up[1]).sum() + (c * up[2]).sum(), params)

    ga, gs, gc, gg = run()
    masks = None
    if p > 0:  # the kernel's dropout key is the table row
        full = [torch.from_numpy(_drop_mask_np(777, k, N, d, p)).to(cuda) for k in range(3)]
        masks = [x[rows] for x in full]
    wa, ws = m.ref(C_[rows], IE[rows], TE[rows], FE[rows], masks)
    wc = C_[rows]
    wg = torch.autograd.grad((wa * up[0]).sum() + (ws * up[1]).sum() + (wc * up[2]).sum(), params)
    _close(ga, wa, "all")
    _close(gs, ws, "side")
    names = ["content", "image", "text", "fusion"] + [k for k, _ in m.named_parameters()]
    for name, a, b in zip(names, gg, wg):
        _close(a, b, name)
    _, _, _, gg2 = run()
    for name, a, b in zip(names[:4], gg, gg2):
        assert torch.equal(a, b), name  # the table gradients: bit-stable run to run


@pytest.mark.parametrize("d,p", [(64, 0.0), (128, 0.1)])
def test_preference_rows_saved_equals_recompute(cuda, d, p, monkeypatch):
    """rsx_smore_pref_rows_saved: the backward from the forward's saved activations
    (7 products) against the backward that recomputes them (20 products): the same
    formulas on the same values, so every gradient agrees to float rounding."""
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(5 * d)
    N, n = 2000, 3000
    mk = lambda: torch.randn(N, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    C_, IE, TE, FE = mk(), mk(), mk(), mk()
    m = _PrefModel(d, gen, cuda, p).train()
    rows = torch.randint(0, N, (n,), generator=gen).to(cuda)
    seed = torch.tensor([99], dtype=torch.int64, device=cuda)
    up = [torch.randn(n, d, generator=gen).to(cuda) for _ in range(3)]
    params = [C_, IE, TE, FE] + list(m.parameters())
    out = {}
    for saved in (True, False):
        monkeypatch.setattr(SF, "_SAVED", saved)
        a, s_, c = SF.preference_rows(m, C_, IE, TE, FE, rows, seed)
        out[saved] = (a, s_, c) + tuple(torch.autograd.grad((a * up[0]).sum() + (s_ * up[1]).sum() +
                                                            (c * up[2]).sum(), params))
    names = ["all", "side", "content_rows", "content", "image", "text", "fusion"] + [k for k, _ in m.named_parameters()]
    for name, x, y in zip(names, out[True], out[False]):
        scale = float(y.abs().max()) + 1e-30
        assert float((x - y).abs().max()) <= 1e-6 * scale, name


@pytest.mark.parametrize("d", [64, 128])
def test_preference_rows_plan_equals_scan(cuda, d, monkeypatch):
    """The backward's per-row sums from the forward's occurrence plan (pref_segsum_plan)
    against the scan (pref_segsum_lds): the same occurrences in the same order, so the table
    gradients are bit-identical; rows past the plan's 128-entry lists take the scan."""
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(11 * d)
    N, n = 3000, 6144
    mk = lambda: torch.randn(N, d, generator=gen).to(cuda).requires_grad_()  # noqa: E731
    C_, IE, TE, FE = mk(), mk(), mk(), mk()
    m = _PrefModel(d, gen, cuda, 0.0).train()
    vhot = torch.randint(0, 4, (800,), generator=gen)  # ~200 occurrences each: the scan
    hot = torch.randint(4, 44, (n // 3,), generator=gen)  # ~50 each: long lists
    warm = torch.randint(44, 400, (n // 3,), generator=gen)  # ~6 each
    rows = torch.cat([vhot, hot, warm, torch.randint(0, N, (n - 2 * (n // 3) - 800,), generator=gen)])
    rows = rows[torch.randperm(n, generator=gen)].to(cuda)
    seed = torch.tensor([5], dtype=torch.int64, device=cuda)
    up = [torch.randn(n, d, generator=gen).to(cuda) for _ in range(3)]
    out = {}
    for plan in (True, False, True):
        monkeypatch.setattr(SF, "_PLAN", plan)
        a, s_, c = SF.preference_rows(m, C_, IE, TE, FE, rows, seed)
        out.setdefault(plan, []).append(torch.autograd.grad((a * up[0]).sum() + (s_ * up[1]).sum() + (c * up[2]).sum(),
                                                            [C_, IE, TE, FE]))
    for name, x, y, z in zip(["content", "image", "text", "fusion"], out[True][0], out[False][0], out[True][1]):
        assert torch.equal(x, y), name
        assert torch.equal(x, z), name  # a second call (the next plan tag) gives the same bits


def test_view_prop_vs_torch(cuda):
    from rsx import smore_fuse as SF
    from rsx.smore import _DevGraph

    rng = np.random.default_rng(3)
    nu, ni, d = 300, 200, 64
    g_r = rng.integers(0, ni, 3000), rng.integers(0, ni, 3000)
    gv = rng.random(3000).astype(np.float32)
    key = np.unique(g_r[0] * ni + g_r[1], return_index=True)[1]
    G = _DevGraph(g_r[0][key], g_r[1][key], gv[key], ni, ni, cuda, 32)
    r_r = rng.integers(0, nu, 4000), rng.integers(0, ni, 4000)
    key = np.unique(r_r[0] * ni + r_r[1], return_index=True)[1]
    rv = rng.random(key.size).astype(np.float32)
    R = _DevGraph(r_r[0][key], r_r[1][key], rv, nu, ni, cuda, 32)
    # dense references of the two operators from their CSR arrays
    def dense(A):
        rp = A.rowptr.cpu().numpy()
        M = torch.zeros(A.n_rows, A.n_cols, dtype=torch.float64)
        rows = np.repeat(np.arange(A.n_rows), np.diff(rp))
        M[torch.from_numpy(rows), A.col.cpu().long()] = A.val.cpu().double()
        return M.to(cuda)

    Gm, Rm = dense(G.A), dense(R.A)
    for L_ in (1, 2):
        x = torch.randn(ni, d, device=cuda, requires_grad=True)
        up = torch.randn(nu + ni, d, device=cuda)
        out = SF.view_prop(x, G, R, L_, nu)
        (gx,) = torch.autograd.grad((out * up).sum(), [x])
        xi = x.detach().double()
        for _ in range(L_):
            xi = Gm @ xi
        want = torch.cat([Rm @ xi, xi])
        _close(out, want, f"out L={L_}", 1e-5)
        gi = up[nu:].double() + Rm.t() @ up[:nu].double()
        for _ in range(L_):
            gi = Gm.t() @ gi
        _close(gx, gi, f"grad L={L_}", 1e-5)


@pytest.mark.parametrize("d,L_", [(64, 1), (128, 2), (64, 0)])
def test_view_prop3_equals_three_view_props(cuda, d, L_):
    """The three views batched into shared launches (rsx_spmm_batch; R used by all
    three products of one launch, each with its own partial-sum slab) equal three
    separate view_prop chains bit for bit, forward and backward, on graphs with hub
    rows (in-launch fixups)."""
    from rsx import smore_fuse as SF
    from rsx.smore import _DevGraph

    rng = np.random.default_rng(7 + d + L_)
    nu, ni = 900, 400

    def graph(nr, nc, nnz, zipf):
        r = rng.integers(0, nr, nnz)
        c = (rng.zipf(zipf, nnz) - 1) % nc
        key = np.unique(r * nc + c, return_index=True)[1]
        return _DevGraph(r[key], c[key], rng.random(key.size).astype(np.float32), nr, nc, cuda, 32)

    Gs = [graph(ni, ni, 6000, 1.3), graph(ni, ni, 5000, 1.6), graph(ni, ni, 9000, 1.2)]
    R = graph(nu, ni, 12000, 1.4)
    assert R.AT.n_long > 0 and any(G.AT.n_long > 0 for G in Gs)
    xs = [torch.randn(ni, d, device=cuda, requires_grad=True) for _ in range(3)]
    ups = [torch.randn(nu + ni, d, device=cuda) for _ in range(3)]
    outs = SF.view_prop3(xs, Gs, R, L_, nu)
    g3 = torch.autograd.grad(sum((o * u).sum() for o, u in zip(outs, ups)), xs)
    for x, G, o, u, g in zip(xs, Gs, outs, ups, g3):
        o1 = SF.view_prop(x, G, R, L_, nu)
        (g1,) = torch.autograd.grad((o1 * u).sum(), [x])
        assert torch.equal(o, o1) and torch.equal(g, g1)


@pytest.mark.parametrize("d", [64, 128])
def test_view_prop3_tagged_users(cuda, d):
    """view_prop3 with the batch-row tags (the R products on the tagged users only: the
    preference block reads no other user row) against the full form: the tagged users'
    and every item row of the forward bit for bit, and the input gradients bit for bit
    for an upstream gradient that is zero off the tagged users (the batch-row preference
    block's); kNN graphs in 64-wide work items."""
    from rsx import smore_fuse as SF
    from rsx.smore import _DevGraph, _RowTags

    rng = np.random.default_rng(d)
    nu, ni = 1200, 500

    def graph(nr, nc, nnz, zipf, chunk):
        r = rng.integers(0, nr, nnz)
        c = (rng.zipf(zipf, nnz) - 1) % nc
        key = np.unique(r * nc + c, return_index=True)[1]
        return _DevGraph(r[key], c[key], rng.random(key.size).astype(np.float32), nr, nc, cuda, chunk)

    Gs = [graph(ni, ni, 6000, 1.3, 64), graph(ni, ni, 5000, 1.6, 64), graph(ni, ni, 9000, 1.2, 64)]
    R = graph(nu, ni, 14000, 1.4, 32)
    tags = _RowTags(nu + ni, cuda)
    users = torch.from_numpy(rng.integers(0, nu, 300)).to(cuda)
    tags.mark(torch.cat([users, nu + torch.from_numpy(rng.integers(0, ni, 600)).to(cuda)]))
    xs = [torch.randn(ni, d, device=cuda, requires_grad=True) for _ in range(3)]
    outs = SF.view_prop3(xs, Gs, R, 1, nu, tags=tags)
    full = SF.view_prop3(xs, Gs, R, 1, nu)
    rows = torch.cat([torch.unique(users), torch.arange(nu, nu + ni, device=cuda)])
    for o, f in zip(outs, full):
        assert torch.equal(o[rows], f[rows])
    m = torch.zeros(nu + ni, 1, device=cuda)
    m[users] = 1.0
    m[nu:] = 1.0
    ups = [torch.randn(nu + ni, d, device=cuda) * m for _ in range(3)]
    gt = torch.autograd.grad(sum((o * w).sum() for o, w in zip(outs, ups)), xs)
    gf = torch.autograd.grad(sum((o * w).sum() for o, w in zip(full, ups)), xs)
    for a, b in zip(gt, gf):
        assert torch.equal(a, b)


class _Poison(torch.autograd.Function):
    """Identity forward; backward hands on the incoming gradient with every row off
    `rows` overwritten by NaN (what an unfilled table holds there)."""

    @staticmethod
    def forward(ctx, x, keep):
        ctx.save_for_backward(keep)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        (keep,) = ctx.saved_tensors
        return torch.where(keep, g, torch.full_like(g, float("nan"))), None


@pytest.mark.parametrize("d", [64, 128])
def test_view_prop3_sparse_gradients_read_only_the_batch_rows(cuda, d):
    """The views' backward with its own tags (gtags, rows: preference_rows(sparse_grads=
    True) leaves the table gradients unwritten off the batch rows): NaN in every other row
    of the upstream gradient changes nothing -- the input gradients equal, bit for bit, the
    dense backward's for the same gradient zero off the batch rows (users gathered through
    x_tag, items added through the item block's row tags); repeated batch rows."""
    from rsx import smore_fuse as SF
    from rsx.smore import _DevGraph, _RowTags

    rng = np.random.default_rng(11 + d)
    nu, ni = 1100, 450

    def graph(nr, nc, nnz, zipf, chunk):
        r = rng.integers(0, nr, nnz)
        c = (rng.zipf(zipf, nnz) - 1) % nc
        key = np.unique(r * nc + c, return_index=True)[1]
        return _DevGraph(r[key], c[key], rng.random(key.size).astype(np.float32), nr, nc, cuda, chunk)

    Gs = [graph(ni, ni, 6000, 1.3, 64), graph(ni, ni, 5000, 1.6, 64), graph(ni, ni, 9000, 1.2, 64)]
    R = graph(nu, ni, 14000, 1.4, 32)
    users = torch.from_numpy(rng.integers(0, nu, 256)).to(cuda)
    items = torch.from_numpy(rng.integers(0, ni, 512)).to(cuda)
    rows = torch.cat([users, nu + items])
    tags, gtags = _RowTags(nu + ni, cuda), _RowTags(nu + ni, cuda)
    tags.mark(rows)
    keep = torch.zeros(nu + ni, 1, dtype=torch.bool, device=cuda)
    keep[rows] = True
    xs = [torch.randn(ni, d, device=cuda, requires_grad=True) for _ in range(3)]
    ups = [torch.randn(nu + ni, d, device=cuda) * keep for _ in range(3)]
    for L_ in (1, 2):
        sp = SF.view_prop3(xs, Gs, R, L_, nu, tags=tags, gtags=gtags, rows=rows)
        sp = [_Poison.apply(o, keep) for o in sp]
        dn = SF.view_prop3(xs, Gs, R, L_, nu, tags=tags)
        gs_ = torch.autograd.grad(sum((o * w).sum() for o, w in zip(sp, ups)), xs)
        gd = torch.autograd.grad(sum((o * w).sum() for o, w in zip(dn, ups)), xs)
        for a, b in zip(gs_, gd):
            assert torch.isfinite(a).all() and torch.equal(a, b), L_


@pytest.mark.parametrize("kind", ["store", "add"])
def test_spmm_batch_many_fixups(cuda, kind):
    """rsx_spmm_batch with more hub-row fixups than ride along in one launch (> 1024 over
    the three products: the work blocks, then every product's fixups in a second
    launch), a graph repeated within the batch: each product equals its own rsx_spmm
    launch bit for bit."""
    from rsx import _lib as L
    from rsx import ops

    rng = np.random.default_rng(5)
    csrs = []
    for k in range(3):
        n = 1500
        deg = np.where(rng.random(n) < 0.4, rng.integers(33, 200, n), rng.integers(0, 32, n))
        rp = np.zeros(n + 1, np.int64)
        rp[1:] = np.cumsum(deg)
        col = rng.integers(0, n, int(rp[-1])).astype(np.int32)
        val = rng.standard_normal(int(rp[-1])).astype(np.float32)
        csrs.append(ops.DeviceCSR(rp, col, val, n, cuda, 32))
    csrs[2] = csrs[0]  # the same graph twice in one launch (separate slabs)
    assert sum(a.n_long for a in csrs) > 1024
    d = 64
    xs = [torch.randn(1500, d, device=cuda) for _ in range(3)]
    adds = [torch.randn(1500, d, device=cuda) for _ in range(3)]
    outs = [torch.empty(1500, d, device=cuda) for _ in range(3)]
    mk = (lambda y, r: ops.epi(L.RSX_EPI_STORE, y=y)) if kind == "store" else \
        (lambda y, r: ops.epi(L.RSX_EPI_ADD, y=y, r_add=r))
    ops.spmm_batch(csrs, xs, [mk(y, r) for y, r in zip(outs, adds)], d)
    for a, x, r, y in zip(csrs, xs, adds, outs):
        want = torch.empty_like(y)
        a.spmm_epi(x, mk(want, r), d)
        assert torch.equal(y, want)


def _infonce_ref(v1, v2, tau):
    """The reference's InfoNCE (smore.py:380-387)."""
    v1, v2 = F.normalize(v1, dim=1), F.normalize(v2, dim=1)
    pos = torch.exp((v1 * v2).sum(dim=-1) / tau)
    ttl = torch.exp(torch.matmul(v1, v2.transpose(0, 1)) / tau).sum(dim=1)
    return torch.mean(-torch.log(pos / ttl))


@pytest.mark.parametrize("d,B,nu,ni", [(64, 2048, 19445, 7050), (128, 2048, 3000, 2000), (64, 1000, 500, 300),
                                       (64, 17, 40, 30)])
def test_infonce2_vs_torch(cuda, d, B, nu, ni):
    from rsx import smore_fuse as SF

    gen = torch.Generator().manual_seed(B + d)
    side = torch.randn(nu + ni, d, generator=gen).to(cuda).requires_grad_()
    content = torch.randn(nu + ni, d, generator=gen).to(cuda).requires_grad_()
    users = torch.randint(0, nu, (B,), generator=gen).to(cuda)
    pos = torch.randint(0, min(ni, 50), (B,), generator=gen).to(cuda)  # heavy repeats: the atomics' case
    ci, cu = SF.infonce2(side, content, users, pos, nu, 0.2)
    gg = torch.autograd.grad(0.7 * ci + 1.3 * cu, [side, content])
    wi = _infonce_ref(side[nu:][pos], content[nu:][pos], 0.2)
    wu = _infonce_ref(side[:nu][users], content[:nu][users], 0.2)
    wg = torch.autograd.grad(0.7 * wi + 1.3 * wu, [side, content])
    _close(ci, wi, "cl_items", 2e-5)
    _close(cu, wu, "cl_users", 2e-5)
    _close(gg[0], wg[0], "d side")
    _close(gg[1], wg[1], "d content")


def test_adam_multi_vs_torch(cuda):
    """One launch over many tensors of odd sizes == torch.optim.Adam(foreach=False)."""
    from rsx.optim import RsxAdam

    shapes = [(300, 64), (64,), (1, 33, 2), (70, 4096), (5,), (7050, 384), (1,)] + [(3, 3)] * 30
    gen = torch.Generator(device="cpu").manual_seed(2)
    ps = [torch.randn(*s, generator=gen).to(cuda) for s in shapes]
    a = [p.clone().requires_grad_() for p in ps]
    b = [p.clone().requires_grad_() for p in ps]
    oa = torch.optim.Adam(a, lr=1e-2, foreach=False)
    ob = RsxAdam(b, lr=1e-2)
    for it in range(3):
        gs = [torch.randn(*s, generator=gen).to(cuda) for s in shapes]
        for k, (x, y, g) in enumerate(zip(a, b, gs)):
            if it == 1 and k % 5 == 0:  # a parameter without a gradient this step keeps its own step count
                x.grad = y.grad = None
                continue
            x.grad = g.clone()
            y.grad = g.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        np.testing.assert_allclose(y.detach().cpu().numpy(), x.detach().cpu().numpy(), rtol=0, atol=1e-6)


def test_mg_alpha_and_axpy_vs_torch(cuda):
    """rsx_mg_alpha (f64 sums of squares) against the trainer's torch restatement of the
    reference's alpha (f32 norms of the concatenations): equal to f32 rounding of the
    rms values; rsx_axpy_multi == p + g * float(alpha * mult) bit for bit."""
    from rsx import smore_fuse as SF
    from rsx.trainer import _mg_alpha

    shapes = [(7050, 4096), (64, 64), (64,), (1, 33, 2), (19445, 64)] + [(5, 7)] * 40
    gen = torch.Generator().manual_seed(9)
    ps = [torch.randn(*s, generator=gen).to(cuda) * 0.1 for s in shapes]
    gs = [torch.randn(*s, generator=gen).to(cuda) * 1e-3 for s in shapes]
    for lr, base in ((1e-3, 0.5), (1e-1, 0.5), (1e-3, 50.0)):
        a = SF.mg_alpha(ps, gs, base, lr, 1e-3, 20.0).item()
        b = _mg_alpha(ps, gs, base, lr, 1e-3, 20.0).item()
        assert abs(a - b) <= 1e-6 * abs(b), (a, b)
    alpha = SF.mg_alpha(ps, gs, 0.5, 1e-3, 1e-3, 20.0)
    want = [p + g * float(alpha.item() * -1e-3) for p, g in zip(ps, gs)]
    ys = [p.clone() for p in ps]
    SF.axpy_multi(ys, gs, alpha, -1e-3)
    for y, w in zip(ys, want):
        assert torch.equal(y, w)


@pytest.mark.gpu
def test_adam_multi_mg_equals_axpy_then_adam(cuda):
    """rsx_adam_multi_mg (the mirror gradient's restore folded into the Adam launch) ==
    rsx_axpy_multi then rsx_adam_multi_scaled, bit for bit: parameters and both
    moments, float4 and ragged tensors, host lr and device lr, with grad_scale; and a
    set halt flag leaves everything unchanged."""
    from rsx import smore_fuse as SF

    shapes = [(7050, 768), (128, 128), (128,), (1, 65, 2), (23033, 128), (5, 7), (3,)]
    gen = torch.Generator().manual_seed(11)
    mk = lambda s, sc: torch.randn(*s, generator=gen).to(cuda) * sc  # noqa: E731
    ps = [mk(s, 0.1) for s in shapes]
    gs = [mk(s, 1e-3) for s in shapes]
    xs = [mk(s, 1e-3) for s in shapes]
    ms = [mk(s, 1e-4) for s in shapes]
    vs = [mk(s, 1e-6).abs() for s in shapes]
    alpha = torch.tensor(3.7, dtype=torch.float64, device=cuda)
    for lr_dev in (None, torch.tensor([2e-3], dtype=torch.float64, device=cuda)):
        mult = 1.0 if lr_dev is not None else 1e-3
        ref = [[t.clone() for t in ts] for ts in (ps, ms, vs)]
        got = [[t.clone() for t in ts] for ts in (ps, ms, vs)]
        st_a = [torch.full((), 3, dtype=torch.int64, device=cuda) for _ in shapes]
        st_b = [t.clone() for t in st_a]
        SF.axpy_multi(ref[0], xs, alpha, mult, lr_dev)
        SF.adam_multi(ref[0], gs, ref[1], ref[2], st_a, 1e-3, grad_scale=-0.2, lr_dev=lr_dev)
        SF.adam_multi(got[0], gs, got[1], got[2], st_b, 1e-3, grad_scale=-0.2, lr_dev=lr_dev,
                      restore=(xs, alpha, mult))
        for name, a, b in zip(("p", "m", "v"), ref, got):
            for i, (x, y) in enumerate(zip(a, b)):
                assert torch.equal(x, y), (name, i, shapes[i], lr_dev is not None, (x - y).abs().max().item(),
                                           (x != y).sum().item())
    halt = torch.tensor([1, 4], dtype=torch.int32, device=cuda)
    got = [t.clone() for t in ps]
    st = [torch.full((), 3, dtype=torch.int64, device=cuda) for _ in shapes]
    SF.adam_multi(got, gs, [t.clone() for t in ms], [t.clone() for t in vs], st, 1e-3, halt=halt,
                  restore=(xs, alpha, 1e-3))
    for x, y in zip(got, ps):
        assert torch.equal(x, y)


@pytest.mark.parametrize("d", [64, 128])
def test_loss_rows_backward_one_launch_equals_the_parts(cuda, d):
    """rsx_smore_loss_rows_bwd (the compact-rows loss backward in one launch) against the
    parts it replaces: rsx_smore_infonce_bwd_scaled adding into zeros and g_bpr * g_total.
    The InfoNCE rows equal the added ones bit for bit (stores of the same values; +0.0
    folds a stored -0.0), the negatives' rows are zero in buffers that start as NaN, and
    the BPR rows are the same f32 products."""
    from rsx import _lib as L
    from rsx import ops

    B = 200
    g = torch.Generator(device=cuda).manual_seed(d)
    side = torch.randn(3 * B, d, generator=g, device=cuda)
    cont = torch.randn(3 * B, d, generator=g, device=cuda)
    gbpr = torch.randn(3 * B, d, generator=g, device=cuda)
    gt = torch.tensor([0.75], device=cuda)
    ar = torch.arange(B, device=cuda)
    lib, p = L.lib(), ops._p
    ws = torch.empty(int(lib.rsx_smore_infonce_ws_bytes(B, d)), dtype=torch.uint8, device=cuda)
    out = torch.empty(3, device=cuda)
    bl = torch.zeros(1, device=cuda)
    L.check(lib.rsx_smore_infonce_fwd_total(p(side), p(cont), p(ar), p(ar), B, B, d, 0.2, p(out), p(bl), 0.3,
                                            p(out[2:]), p(ws), ws.numel(), ops._stream()), "fwd_total")
    ref = torch.zeros(2, 3 * B, d, device=cuda)
    L.check(lib.rsx_smore_infonce_bwd_scaled(p(side), p(cont), p(ar), p(ar), B, B, d, 0.2, p(gt), 0, 0.3, p(ref[0]),
                                             p(ref[1]), p(ws), ws.numel(), ops._stream()), "bwd_scaled")
    got = torch.full((2, 3 * B, d), float("nan"), device=cuda)
    gall = torch.full((3 * B, d), float("nan"), device=cuda)
    L.check(lib.rsx_smore_loss_rows_bwd(p(side), p(cont), p(ar), B, d, 0.2, p(gt), 0.3, p(gbpr), p(gall), p(got[0]),
                                        p(got[1]), p(ws), ws.numel(), ops._stream()), "loss_rows_bwd")
    torch.cuda.synchronize()
    assert torch.equal(got + 0.0, ref + 0.0)
    assert torch.equal(gall, gbpr * gt)


def test_tag_rows_next_bumps_once_per_call(cuda):
    """rsx_tag_rows_next: one launch tags rows[j] with the next tag and leaves it in
    tag2[0] (the last of many blocks bumps it; the ticket word is re-armed), and an empty
    row list still bumps."""
    from rsx import _lib as L
    from rsx import ops

    n_rows, n = 9000, 5000  # 20 blocks
    gen = torch.Generator().manual_seed(3)
    row_tag = torch.zeros(n_rows, dtype=torch.int32, device=cuda)
    tag2 = torch.zeros(2, dtype=torch.int32, device=cuda)
    for call in (1, 2, 3):
        rows = torch.randint(0, n_rows, (n,), generator=gen).to(cuda)
        L.check(L.lib().rsx_tag_rows_next(ops._p(row_tag), ops._p(rows), n, ops._p(tag2), ops._stream()),
                "rsx_tag_rows_next")
        assert tag2.tolist() == [call, 0]
        assert torch.all(row_tag[rows] == call)
        assert int((row_tag == call).sum()) == int(torch.unique(rows).numel())
    L.check(L.lib().rsx_tag_rows_next(ops._p(row_tag), None, 0, ops._p(tag2), ops._stream()), "rsx_tag_rows_next")
    assert tag2.tolist() == [4, 0]
