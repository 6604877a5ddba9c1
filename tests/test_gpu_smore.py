"""SMORE on the GPU against the reference's own outputs (tests/golden/smore_small.npz):
identical initial weights (same module creation order under init_seed), graphs bit
for bit, forward within rtol 1e-5, first-batch loss / gradients / Adam step, and one
epoch through the Trainer with the model-level mirror gradient.  Dropout 0 (the
reference's dropout masks come from its own RNG and cannot be replayed on the GPU)."""
import os
import shutil

import numpy as np
import pytest
import torch

from helpers import coo_sorted, csr_to_sorted, metric_dict

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# (fixture, dataset name, .inter file, feature file names, config overrides)
FIXTURES = {
    "smore_small": ("baby", "gold_small.inter", ("image_feat_raw.npy", "text_feat_raw.npy"), {}),
    # C5-shaped: embedding_size 128, CLIP-like L2-normalised 768/768 features (clothing.yaml file names)
    "smore_d128_small": ("clothing", "gold_clothing.inter", ("image_feat.npy", "text_feat.npy"),
                         dict(embedding_size=128)),
}


def _setup(tmp_path, golden, fx="smore_small"):
    from rsx.config import Config
    from rsx.data import EvalDataLoader, RecDataset, TrainDataLoader

    dataset, inter, (vf, tf), extra = FIXTURES[fx]
    z = golden(fx)
    d = tmp_path / "data" / dataset
    d.mkdir(parents=True)
    shutil.copy(os.path.join(GOLD, inter), d / f"{dataset}.inter")
    np.save(d / vf, z["v_feat"])
    np.save(d / tf, z["t_feat"])
    c = Config("SMORE", dataset, dict(data_path=str(tmp_path / "data") + "/", train_batch_size=512,
                                      eval_batch_size=256, rsx_sampler="host", is_multimodal_model=True,
                                      dropout_rate=[0.0], mg_verbose=False, image_knn_k=[10], text_knn_k=[8],
                                      **extra))
    for k in c["hyper_parameters"]:
        if isinstance(c[k], list):
            c[k] = c[k][0]
    ds = RecDataset(c)
    tr, va, te = ds.split()
    for x in (ds, tr, va, te):
        str(x)
    train = TrainDataLoader(c, tr, batch_size=512, shuffle=True)
    valid = EvalDataLoader(c, va, additional_dataset=tr, batch_size=256)
    test = EvalDataLoader(c, te, additional_dataset=tr, batch_size=256)
    return z, c, train, valid, test


def _model(c, train):
    from rsx.smore import SMORE
    from rsx.utils import init_seed

    init_seed(c["seed"])
    train.pretrain_setup()
    return SMORE(c, train)


@pytest.mark.parametrize("fx", list(FIXTURES))
def test_smore_init_graphs_forward(tmp_path, golden, fx):
    z, c, train, valid, test = _setup(tmp_path, golden, fx)
    m = _model(c, train)
    for n, p in m.named_parameters():
        assert np.array_equal(p.detach().cpu().numpy(), z["init." + n]), n
    nu = m.n_users
    A = m.norm_adj_csr
    ref = coo_sorted(z["norm_adj_idx"].astype(np.int64), z["norm_adj_val"])
    for x, y in zip(ref, csr_to_sorted(A.rowptr.cpu().numpy(), A.col.cpu().numpy(), A.val.cpu().numpy())):
        assert np.array_equal(x, y)
    for name, g in (("image_original_adj", m.image_graph), ("text_original_adj", m.text_graph),
                    ("fusion_adj", m.fusion_graph), ("R", m.R)):
        ref = coo_sorted(z[name + "_idx"].astype(np.int64), z[name + "_val"])
        mine = csr_to_sorted(g.A.rowptr.cpu().numpy(), g.A.col.cpu().numpy(), g.A.val.cpu().numpy())
        assert np.array_equal(ref[0], mine[0]) and np.array_equal(ref[1], mine[1]), name
        if name == "R":
            assert np.array_equal(ref[2], mine[2])
        else:
            # kNN cosine similarities come from a CPU sgemm: a few ulp apart across host CPUs (768-long dots)
            np.testing.assert_allclose(mine[2], ref[2], rtol=3e-6, atol=0, err_msg=name)
    m.eval()
    with torch.no_grad():
        u, i = m.forward(None)
        np.testing.assert_allclose(u.cpu().numpy(), z["fwd_user"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(i.cpu().numpy(), z["fwd_item"], rtol=1e-5, atol=1e-6)
        cv, ct, cf = m._projected_spectrum()
        np.testing.assert_allclose(cv.cpu().numpy(), z["spec_conv_v"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(ct.cpu().numpy(), z["spec_conv_t"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(cf.cpu().numpy(), z["spec_conv_f"], rtol=1e-4, atol=1e-6)
        _, _, side, content = m.forward(None, train=True)
        np.testing.assert_allclose(side.cpu().numpy(), z["fwd_side"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(content.cpu().numpy(), z["fwd_content"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fx", list(FIXTURES))
def test_smore_first_step(tmp_path, golden, fx):
    z, c, train, valid, test = _setup(tmp_path, golden, fx)
    m = _model(c, train)
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=c["learning_rate"])
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).cuda()
    loss = m.calculate_loss(trip)
    loss.backward()
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    for n, p in m.named_parameters():
        key = "step0_grad." + n
        if key in z:
            g = p.grad.detach().cpu().numpy()
            scale = max(np.abs(z[key]).max(), 1e-12)
            np.testing.assert_allclose(g, z[key], rtol=1e-3, atol=1e-5 * scale, err_msg=n)
    mine = {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()}
    opt.step()
    lr = c["learning_rate"]
    for n, p in m.named_parameters():
        got, want = p.detach().cpu().numpy(), z["step0_param." + n]
        # Adam's first step is exactly -lr * g / (|g| + eps): the update differs from the
        # reference's by at most lr * |s(g_mine) - s(g_ref)| (plus rounding), which is large
        # only where |g| is within rounding noise of 0
        gr = z.get("step0_grad." + n, np.zeros_like(want))
        sgn = lambda g: g / (np.abs(g) + 1e-8)  # noqa: E731
        bound = lr * np.abs(sgn(mine[n]) - sgn(gr)) + 2e-6
        assert np.all(np.abs(got - want) <= bound), n


@pytest.mark.parametrize("fx,p_drop", [("smore_small", 0.0), ("smore_small", 0.1), ("smore_d128_small", 0.1)])
def test_smore_batch_rows_loss_equals_full_tables(tmp_path, golden, fx, p_drop):
    """The training loss with the preference block on the batch rows only
    (rsx_smore_batch_rows, the default) against the full-table form: the same loss and
    every parameter gradient, with the same dropout masks (keyed by the table row), on
    a batch with repeated users and items."""
    z, c, train, valid, test = _setup(tmp_path, golden, fx)
    c["dropout_rate"] = p_drop
    m = _model(c, train)
    m.train()
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)).cuda()
    trip[0, :40] = trip[0, 0]
    trip[1, 100:140] = trip[2, 7]
    out = []
    for rows in (True, False):
        m.batch_rows = rows
        m._drop_seed.fill_(12345)
        m.zero_grad(set_to_none=True)
        loss = m.calculate_loss(trip)
        loss.backward()
        out.append((loss.item(), {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()
                                  if p.grad is not None}))
    (la, ga), (lb, gb) = out
    assert abs(la - lb) <= 1e-6 * abs(lb)
    assert ga.keys() == gb.keys()
    for n in gb:
        scale = max(np.abs(gb[n]).max(), 1e-12)
        np.testing.assert_allclose(ga[n], gb[n], rtol=0, atol=2e-5 * scale, err_msg=n)


@pytest.mark.parametrize("K,d", [(1, 64), (2, 64), (3, 128), (4, 64), (4, 128)])
def test_prop_mean_rows_vs_dense(cuda, K, d):
    """The tagged mean propagation of the SMORE training loss (_PropMeanRows: stored
    layers, last layer + mean on the batch rows) equals the dense one (_PropMean) bit
    for bit on the batch rows; its Horner backward from a gradient that is zero off
    the batch rows equals the dense backward within f32 reassociation."""
    from rsx import graph, ops, synth
    from rsx.smore import _PropMean, _PropMeanRows, _RowTags

    df = synth.amazon_like(2500, 700, 25000, seed=11)
    tr = df[df.x_label == 0]
    nu, ni = int(df.userID.max()) + 1, 700
    rp, col, val = graph.smore_norm_adj(tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64), nu, ni)
    A = ops.DeviceCSR(rp, col, val, nu + ni, cuda, 32)
    assert A.n_long > 0
    gen = torch.Generator().manual_seed(K * 100 + d)
    x = torch.randn(nu + ni, d, generator=gen).to(cuda).requires_grad_()
    users = torch.randint(0, nu, (300,), generator=gen)
    items = torch.randint(0, ni, (600,), generator=gen)
    items[:50] = int(np.argmax(np.bincount(tr.itemID.values, minlength=ni)))  # a hub row, repeated
    rows = torch.cat([users, nu + items]).to(cuda)
    tags = _RowTags(nu + ni, cuda)
    tags.mark(torch.arange(nu + ni, device=cuda)[:7])  # stale tags of an earlier batch
    tags.mark(rows)
    out_t = _PropMeanRows.apply(x, A, K, tags, rows)
    out_d = _PropMean.apply(x, A, K)
    assert torch.equal(out_t[rows], out_d[rows])
    g = torch.zeros(nu + ni, d, device=cuda)
    g[rows] = torch.randn(rows.numel(), d, generator=gen).to(cuda)
    gt, = torch.autograd.grad(out_t, x, g)
    gd, = torch.autograd.grad(out_d, x, g)
    scale = gd.abs().max().item()
    np.testing.assert_allclose(gt.cpu().numpy(), gd.cpu().numpy(), rtol=0, atol=2e-6 * scale)


@pytest.mark.parametrize("fx", list(FIXTURES))
def test_smore_one_epoch_with_mirror_gradient(tmp_path, golden, fx):
    from rsx.trainer import Trainer

    z, c, train, valid, test = _setup(tmp_path, golden, fx)
    m = _model(c, train)
    t = Trainer(c, m)
    assert not t.fused and m.mg_enable
    m.pre_epoch_processing()
    loss, _ = t._train_epoch(train, 0)
    assert abs(loss - float(z["epoch_losses"][0])) <= 1e-4 * abs(float(z["epoch_losses"][0]))
    for n, p in m.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["epoch0_param." + n], rtol=0, atol=1e-4, err_msg=n)
    vres = t.evaluate(valid)
    tres = t.evaluate(test)
    for res, tag in ((vres, "epoch0_valid"), (tres, "epoch0_test")):
        ref = metric_dict(z, tag)
        for k in ref:
            assert abs(res[k] - ref[k]) <= 1e-4 + 1e-12, (tag, k, res[k], ref[k])


@pytest.mark.parametrize("graph", [True, False])
def test_smore_training_emits_no_accumulate_grad_stream_warning(tmp_path, golden, graph):
    """Two epochs of SMORE batches (the UI backbone on its side stream; eager, captured
    and replayed batches) raise no warning from torch's autograd engine: in particular
    not the AccumulateGrad stream-mismatch one (a leaf's gradient produced on another
    stream than its accumulator's, an extra cross-stream sync per backward)."""
    import warnings

    from rsx.trainer import Trainer

    z, c, train, valid, test = _setup(tmp_path, golden)
    c["rsx_graph_step"] = graph
    m = _model(c, train)
    t = Trainer(c, m)
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(True)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for ep in range(2):
            m.pre_epoch_processing()
            loss, _ = t._train_epoch(train, ep)
            assert not torch.is_tensor(loss)
        torch.cuda.synchronize()
    bad = [str(x.message)[:160] for x in w if "AccumulateGrad" in str(x.message) or "stream" in str(x.message)]
    assert not bad, bad
    if graph:
        assert t._graph is not None and t._graph.replays > 0


def test_smore_two_losses_before_one_backward(tmp_path, golden):
    """calculate_loss twice (two batches) and ONE backward of their sum = the two
    backwards one at a time: the batch-row propagation re-tags its forward's rows in its
    backward, so a later forward's tags cannot hide the earlier batch's rows."""
    z, c, train, valid, test = _setup(tmp_path, golden)
    m = _model(c, train)
    m.train()
    t = torch.from_numpy(z["epoch0_triplets"][:, :1024].astype(np.int64)).cuda()
    b1, b2 = t[:, :512].contiguous(), t[:, 512:].contiguous()
    (m.calculate_loss(b1) + m.calculate_loss(b2)).backward()
    joint = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    m.calculate_loss(b1).backward()
    m.calculate_loss(b2).backward()
    for n, p in m.named_parameters():
        scale = max(p.grad.abs().max().item(), 1e-12)
        assert (p.grad - joint[n]).abs().max().item() <= 1e-5 * scale, n


@pytest.mark.parametrize("graph", [True, False])
def test_smore_nan_loss_halts_the_step(tmp_path, golden, graph):
    """A NaN batch loss inside an epoch of graph-replayed (or eager) SMORE batches with
    the mirror gradient: the device NaN gate (rsx_nan_gate) stops every later Adam and
    mirror-gradient launch, so every parameter and Adam moment stays bit for bit what
    it was before the NaN batch, and the epoch reports that batch index (reference
    src/common/trainer.py:192-203: checked before backward, training stops)."""
    from rsx.trainer import Trainer

    z, c, train, valid, test = _setup(tmp_path, golden)
    c["rsx_graph_step"] = graph
    m = _model(c, train)
    t = Trainer(c, m)
    m.pre_epoch_processing()
    loss0, _ = t._train_epoch(train, 0)  # captures the graphs (both batch kinds)
    assert not torch.is_tensor(loss0)
    snap = {}
    bad = 3

    def poisoned():
        for i, b in enumerate(train):
            if i == bad:
                m.user_embedding.weight.data[b[0, 0]] = float("nan")
                snap["p"] = [p.detach().clone() for p in m.parameters()]
                snap["s"] = [(st["exp_avg"].clone(), st["exp_avg_sq"].clone())
                             for st in (t.optimizer.state[p] for p in m.parameters())]
            yield b

    m.pre_epoch_processing()
    loss1, _ = t._train_epoch(poisoned(), 1)
    assert torch.is_tensor(loss1) and torch.isnan(loss1)
    assert t._halt.tolist() == [1, bad + 1]
    if graph:
        assert t._graph is not None and t._graph.replays > 0
    eq = lambda a, b: torch.equal(a.view(torch.int32), b.view(torch.int32))  # noqa: E731  NaN-safe bitwise
    for p, q in zip(m.parameters(), snap["p"]):
        assert eq(p.detach(), q)
    for p, (em, ev) in zip(m.parameters(), snap["s"]):
        assert eq(t.optimizer.state[p]["exp_avg"], em) and eq(t.optimizer.state[p]["exp_avg_sq"], ev)


def test_smore_graph_step_equals_eager(tmp_path, golden):
    """Two epochs with the training batch replayed from captured HIP graphs
    (rsx_graph_step) == the same epochs run eagerly: the host step counter and the
    Adam step counts exactly; losses, parameters and Adam moments to the tolerance of
    the golden epoch test.  (Not bit for bit: the BPR kernel scatters its row
    gradients with float atomics, bpr.hip:14, so two eager runs already differ in
    the last bits, and Adam turns that into up to ~lr near g = 0.)  The epoch has 6
    full batches (plain and mirror-gradient kinds, each run eagerly once, then
    captured and replayed) and a partial one (eager)."""
    from rsx.trainer import Trainer

    runs = []
    for graph in (False, True):
        z, c, train, valid, test = _setup(tmp_path / str(graph), golden)
        c["rsx_graph_step"] = graph
        m = _model(c, train)
        t = Trainer(c, m)
        losses = []
        replays = 0
        for ep in range(2):
            m.pre_epoch_processing()
            loss, _ = t._train_epoch(train, ep)
            losses.append(loss)
            replays += t._graph.replays if t._graph is not None else 0
        st = [t.optimizer.state[p] for p in m.parameters()]
        runs.append(dict(losses=losses, step=m.global_step, replays=replays,
                         p={n: p.detach().cpu().numpy() for n, p in m.named_parameters()},
                         m=[s["exp_avg"].cpu().numpy() for s in st], v=[s["exp_avg_sq"].cpu().numpy() for s in st],
                         n=[int(s["step"]) for s in st]))
    eager, graph = runs
    assert eager["replays"] == 0 and graph["replays"] >= 4
    assert graph["step"] == eager["step"] and graph["n"] == eager["n"]
    np.testing.assert_allclose(graph["losses"], eager["losses"], rtol=1e-5)
    for k in eager["p"]:
        np.testing.assert_allclose(graph["p"][k], eager["p"][k], rtol=0, atol=1e-4, err_msg=k)
    for a, b in zip(graph["m"] + graph["v"], eager["m"] + eager["v"]):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-7)


@pytest.mark.parametrize("d,n,dv,dt", [(64, 1000, 512, 384), (128, 333, 768, 768), (64, 7, 48, 24)])
def test_spectral_fused_vs_torch_autograd(cuda, d, n, dv, dt):
    """rsx_smore_spectral_fwd/bwd against torch.nn.functional.linear + torch.fft (fp32, the
    reference's ops) with autograd: outputs rtol 1e-4, every gradient within 1e-4 of its scale."""
    from rsx.smore import spectrum_torch
    from rsx.smore_spectral import spectral

    g = torch.Generator(device="cpu").manual_seed(d + n)
    mk = lambda *s: torch.randn(*s, generator=g).to(cuda).requires_grad_()  # noqa: E731
    V, T = mk(n, dv), mk(n, dt)
    Wv, Wt = (mk(d, dv) / dv ** 0.5).detach().requires_grad_(), (mk(d, dt) / dt ** 0.5).detach().requires_grad_()
    bv, bt = mk(d), mk(d)
    wv, wt, wf = mk(1, d // 2 + 1, 2), mk(1, d // 2 + 1, 2), mk(1, d // 2 + 1, 2)
    leaves = [V, Wv, bv, T, Wt, bt, wv, wt, wf]
    up = [torch.randn(n, d, generator=g).to(cuda) for _ in range(3)]

    ref = spectrum_torch(torch.nn.functional.linear(V, Wv, bv), torch.nn.functional.linear(T, Wt, bt), wv, wt, wf)
    ref_g = torch.autograd.grad(sum((r * u).sum() for r, u in zip(ref, up)), leaves)
    got = spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf)[:3]
    got_g = torch.autograd.grad(sum((r * u).sum() for r, u in zip(got, up)), leaves)
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=1e-4,
                                   atol=1e-5 * b.abs().max().item())
    names = ["V", "Wv", "bv", "T", "Wt", "bt", "wv", "wt", "wf"]
    for name, a, b in zip(names, got_g, ref_g):
        scale = b.abs().max().item()
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-4 * scale, err_msg=name)


@pytest.mark.parametrize("d,n,dv,dt,mul", [(64, 1000, 512, 384, False), (128, 333, 768, 768, False),
                                           (64, 7, 48, 24, True), (64, 200, 4096, 384, False),
                                           (128, 23033, 768, 768, False), (128, 129, 1024, 96, True)])
def test_item_side_one_launch_equals_three_launch_chain(cuda, d, n, dv, dt, mul):
    """rsx_smore_item_fwd (projection -> spectral -> gates in one launch, the tile's last
    arriving block running the tail) against rsx_smore_spectral_fwd + rsx_smore_gates: every
    output bit for bit (the same arithmetic), K-split projections (4096-wide: 8 splits of a
    tile counted in), ragged last tiles, residual and mul inject; called three times so the
    arrival counters are re-armed; the backward's gradients equal the chain's, bit for bit."""
    from rsx import smore_fuse as SF
    from rsx.smore_spectral import item_side, spectral

    g = torch.Generator(device="cpu").manual_seed(3 * d + n)
    mk = lambda *s: torch.randn(*s, generator=g).to(cuda).requires_grad_()  # noqa: E731
    V, T = mk(n, dv), mk(n, dt)
    Wv, Wt = (mk(d, dv) / dv ** 0.5).detach().requires_grad_(), (mk(d, dt) / dt ** 0.5).detach().requires_grad_()
    bv, bt = mk(d), mk(d)
    wv, wt, wf = mk(1, d // 2 + 1, 2), mk(1, d // 2 + 1, 2), mk(1, d // 2 + 1, 2)
    item = mk(n, d)
    gates = [torch.nn.Sequential(torch.nn.Linear(d, d), torch.nn.Sigmoid()).to(cuda) for _ in range(3)]
    leaves = [V, Wv, bv, T, Wt, bt, wv, wt, wf, item] + [p for s in gates for p in s.parameters()]
    up = [torch.randn(n, d, generator=g).to(cuda) for _ in range(3)]

    cv, ct, cf, img, txt = spectral(V, Wv, bv, T, Wt, bt, wv, wt, wf)
    ref = SF.gates(cv, ct, cf, item, *gates, 0.7, mul)
    ref_g = torch.autograd.grad(sum((r * u).sum() for r, u in zip(ref, up)), leaves)
    for rep in range(3):
        got = item_side(V, Wv, bv, T, Wt, bt, wv, wt, wf, item, *gates, 0.7, mul)
        for name, a, b in zip(["img_i", "txt_i", "fus_i", "conv_v", "conv_t", "conv_f", "img", "txt"], got,
                              (*ref, cv, ct, cf, img, txt)):
            assert torch.equal(a, b), (rep, name, (a - b).abs().max().item())
    got_g = torch.autograd.grad(sum((r * u).sum() for r, u in zip(got[:3], up)), leaves)
    for i, (a, b) in enumerate(zip(got_g, ref_g)):
        assert torch.equal(a, b), (i, (a - b).abs().max().item())


@pytest.mark.parametrize("n,o,i", [(26495, 64, 64), (1000, 128, 64), (7, 32, 32), (513, 64, 128), (7050, 64, 4096),
                                   (7050, 64, 384), (0, 64, 64), (65, 32, 32), (300001, 64, 64)])
def test_linear_wgrad_vs_torch(cuda, n, o, i):
    """rsx_linear_wgrad = g^T x (fp32; tolerance relative to the magnitude of the sums)."""
    from rsx import ops

    gen = torch.Generator(device="cpu").manual_seed(n + o)
    g = torch.randn(n, o, generator=gen).to(cuda)
    x = torch.randn(n, i, generator=gen).to(cuda)
    got = ops.linear_wgrad(g, x)
    want = (g.double().t() @ x.double()).float()
    scale = (g.abs().double().t() @ x.abs().double()).float()
    assert torch.all((got - want).abs() <= 2e-6 * scale + 1e-6), (got - want).abs().max()
    assert torch.equal(got, ops.linear_wgrad(g, x))  # deterministic


@pytest.mark.parametrize("n,o,i", [(7050, 64, 4096), (7050, 64, 384), (23033, 128, 768), (1000, 128, 96),
                                   (37, 32, 64), (513, 32, 160), (0, 64, 64),
                                   (200, 64, 48), (200, 64, 24), (777, 128, 100), (3000, 64, 4)])
def test_linear_bwd_vs_torch(cuda, n, o, i):
    """rsx_linear_bwd (the projections' whole backward in one pass): dW = g^T x,
    dx = g W and db = colsum g against f64 products (tolerance relative to the
    magnitude of each sum); deterministic."""
    from rsx import ops

    gen = torch.Generator(device="cpu").manual_seed(n + 7 * o + i)
    g = torch.randn(n, o, generator=gen).to(cuda)
    x = torch.randn(n, i, generator=gen).to(cuda)
    W = torch.randn(o, i, generator=gen).to(cuda)
    dw, dx, db = ops.linear_bwd(g, x, W)
    gd, xd, Wd = g.double(), x.double(), W.double()
    for got, want, scale in ((dw, gd.t() @ xd, gd.abs().t() @ xd.abs()), (dx, gd @ Wd, gd.abs() @ Wd.abs()),
                             (db, gd.sum(0), gd.abs().sum(0))):
        assert got.shape == want.shape
        assert torch.all((got.double() - want).abs() <= 2e-6 * scale + 1e-6), (got.double() - want).abs().max()
    dw2, dx2, db2 = ops.linear_bwd(g, x, W)
    assert torch.equal(dw, dw2) and torch.equal(dx, dx2) and torch.equal(db, db2)
    _, _, none = ops.linear_bwd(g, x, W, bias=False)
    assert none is None


@pytest.mark.parametrize("n,o,i0,i1,bias", [(7050, 64, 4096, 384, (True, True)), (23033, 128, 768, 384, (True, True)),
                                             (513, 32, 192, 64, (True, False)), (200, 64, 128, 64, (False, True))])
def test_linear_bwd_pair_vs_torch(cuda, n, o, i0, i1, bias):
    """rsx_linear_bwd_pair (SMORE's image + text projection backward in one launch pair):
    each problem's dW, dx, db against f64 products (as test_linear_bwd_vs_torch), and
    deterministic; None (two single launches then) only when the tilings differ."""
    from rsx import ops

    gen = torch.Generator(device="cpu").manual_seed(n + o + i0 + i1)
    probs = []
    for i, b in ((i0, bias[0]), (i1, bias[1])):
        probs.append((torch.randn(n, o, generator=gen).to(cuda), torch.randn(n, i, generator=gen).to(cuda),
                      torch.randn(o, i, generator=gen).to(cuda), b))
    res = ops.linear_bwd_pair(*probs)
    if res is None:  # e.g. 48 and 24 columns tile differently: the caller's two-launch path
        pytest.skip("tilings differ")
    for (g, x, W, b), (dw, dx, db) in zip(probs, res):
        gd, xd, Wd = g.double(), x.double(), W.double()
        checks = [(dw, gd.t() @ xd, gd.abs().t() @ xd.abs()), (dx, gd @ Wd, gd.abs() @ Wd.abs())]
        if b:
            checks.append((db, gd.sum(0), gd.abs().sum(0)))
        else:
            assert db is None
        for got, want, scale in checks:
            assert got.shape == want.shape
            assert torch.all((got.double() - want).abs() <= 2e-6 * scale + 1e-6), (got.double() - want).abs().max()
    res2 = ops.linear_bwd_pair(*probs)
    for a, b in zip(res, res2):
        for x, y in zip(a, b):
            assert (x is None and y is None) or torch.equal(x, y)


def test_rsx_linear_matches_nn_linear(cuda):
    from rsx.nn import RsxLinear

    torch.manual_seed(3)
    a = torch.nn.Linear(64, 64).to(cuda)
    torch.manual_seed(3)
    b = RsxLinear(64, 64).to(cuda)
    assert torch.equal(a.weight, b.weight) and torch.equal(a.bias, b.bias)
    x = torch.randn(5000, 64, device=cuda, requires_grad=True)
    up = torch.randn(5000, 64, device=cuda)
    ga = torch.autograd.grad((a(x) * up).sum(), [x, a.weight, a.bias])
    gb = torch.autograd.grad((b(x) * up).sum(), [x, b.weight, b.bias])
    for p, q in zip(ga, gb):  # two fp32 summation orders over 5000 rows: relative to the magnitude
        np.testing.assert_allclose(q.cpu().numpy(), p.cpu().numpy(), rtol=1e-4, atol=1e-5 * p.abs().max().item())


def test_rsx_adam_matches_torch_single_tensor(cuda):
    """RsxAdam == torch.optim.Adam(foreach=False) (the reference's CPU path) over 4 steps."""
    from rsx.optim import RsxAdam

    shapes = [(300, 64), (64,), (1, 33, 2), (70, 4096)]
    gen = torch.Generator(device="cpu").manual_seed(1)
    ps = [torch.randn(*s, generator=gen).to(cuda) for s in shapes]
    a = [p.clone().requires_grad_() for p in ps]
    b = [p.clone().requires_grad_() for p in ps]
    oa = torch.optim.Adam(a, lr=1e-2, weight_decay=1e-4, foreach=False)
    ob = RsxAdam(b, lr=1e-2, weight_decay=1e-4)
    for _ in range(4):
        gs = [torch.randn(*s, generator=gen).to(cuda) for s in shapes]
        for x, y, gg in zip(a, b, gs):
            x.grad = gg.clone()
            y.grad = gg.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        np.testing.assert_allclose(y.detach().cpu().numpy(), x.detach().cpu().numpy(), rtol=0, atol=1e-6)


@pytest.mark.parametrize("src", ["golden_image", "golden_text", "random", "wide", "ragged"])
def test_knn_graph_device_vs_host(cuda, golden, src):
    """SMORE's kNN item graph built on the device (GEMM + topk + sym-norm) against the
    CPU restatement of the reference's build (knn_graph, pinned bit for bit to the
    reference's graphs by test_smore_init_graphs_forward): per row the same
    neighbours except where the host's cosine similarities of the swapped items tie
    with the k-th within 1e-5 (the GEMMs add in another order), and the normalised
    values of the common edges within rtol 2e-5."""
    from rsx.smore import knn_graph, knn_graph_device

    if src == "random":
        f = np.random.default_rng(3).standard_normal((1500, 768)).astype(np.float32)
        k = 20
    elif src == "wide":  # baby's raw image width, several 256-row panels and 128-row blocks
        f = np.random.default_rng(4).standard_normal((2000, 4096)).astype(np.float32)
        k = 20
    elif src == "ragged":  # features not a multiple of the 32-wide chunk, the largest k
        f = np.random.default_rng(5).standard_normal((777, 100)).astype(np.float32)
        k = 32
    else:
        z = golden("smore_small")
        f = z["v_feat" if src == "golden_image" else "t_feat"].astype(np.float32)
        k = 10 if src == "golden_image" else 8
    n = f.shape[0]
    hr, hc, hv = knn_graph(f, k)
    dr, dc, dv = knn_graph_device(torch.from_numpy(f).to(cuda), k)
    assert np.array_equal(hr, dr)
    fn = f.astype(np.float64) / np.linalg.norm(f.astype(np.float64), axis=1, keepdims=True)
    hc, dc, hv, dv = hc.reshape(n, k), dc.reshape(n, k), hv.reshape(n, k), dv.reshape(n, k)
    swapped = 0
    for r in range(n):
        a, b = set(hc[r].tolist()), set(dc[r].tolist())
        if a != b:
            sims = fn[r] @ fn.T
            kth = np.sort(sims)[-k]
            for c in a ^ b:
                assert abs(sims[c] - kth) <= 1e-5, (r, c, sims[c], kth)
            swapped += 1
            continue
        hm = dict(zip(hc[r].tolist(), hv[r].tolist()))
        for c, v in zip(dc[r].tolist(), dv[r].tolist()):
            assert abs(v - hm[c]) <= 2e-5 * abs(hm[c]) + 1e-7, (r, c, v, hm[c])
    assert swapped <= max(2, n // 100)
