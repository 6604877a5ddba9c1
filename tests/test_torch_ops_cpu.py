"""torch.ops.rsx.* (rsx/torch_ops.py) on the CPU: every op exists with its
schema, shape inference works under FakeTensorMode (torch.compile / meta tracing), and
CPU tensors run the C++ CPU kernels (csrc/cpu_ops.cpp) — checked here, op by op and with
their gradients, against the reference's own outputs in tests/golden (captured from the
reference by tools/capture_golden.py) and against the reference's torch ops on the same
inputs.  smore_spectral has no CPU kernel: CPU tensors raise."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import rsx  # noqa: F401  registers the ops
import rsx_oracle as O
from helpers import params, train_mask_pairs
from rsx import graph, torch_ops

SCHEMAS = {
    "spmm_csr": "rsx::spmm_csr(Tensor rowptr, Tensor col, Tensor val, Tensor x, SymInt n_cols) -> Tensor",
    "propagate_mean": "rsx::propagate_mean(Tensor rowptr, Tensor col, Tensor val, Tensor x, SymInt n_layers) -> Tensor",
    "fullsort_topk": ("rsx::fullsort_topk(Tensor user_emb, Tensor users, Tensor item_emb, Tensor mask_rowptr, "
                      "Tensor mask_col, SymInt k) -> (Tensor, Tensor)"),
}


def test_every_op_registered():
    for name in torch_ops.OPS:
        assert hasattr(torch.ops.rsx, name), name
    for name, schema in SCHEMAS.items():
        assert str(getattr(torch.ops.rsx, name).default._schema) == schema
    assert "Tensor(a0!) p" in str(torch.ops.rsx.adam_.default._schema)


def test_gpu_only_op_raises_on_cpu():
    z = torch.zeros
    with pytest.raises(NotImplementedError):
        torch.ops.rsx.smore_spectral(z(9, 32), z(64, 32), z(64), z(9, 16), z(64, 16), z(64), z(1, 33, 2), z(1, 33, 2),
                                     z(1, 33, 2), True)


def test_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        rp = torch.empty(11, dtype=torch.int64, device="cuda")
        col = torch.empty(40, dtype=torch.int32, device="cuda")
        val = torch.empty(40, device="cuda")
        x = torch.empty(7, 64, device="cuda")
        assert torch.ops.rsx.spmm_csr(rp, col, val, x, 7).shape == (10, 64)
        e = torch.empty(10, 64, device="cuda")
        assert torch.ops.rsx.propagate_mean(rp, col, val, e, 3).shape == (10, 64)
        v, i = torch.ops.rsx.fullsort_topk(torch.empty(5, 64, device="cuda"), torch.empty(3, dtype=torch.int64,
                                           device="cuda"), torch.empty(9, 64, device="cuda"), rp, col, 4)
        assert v.shape == (3, 4) and i.shape == (3, 4) and i.dtype == torch.int64
        cv, ct, cf = torch.ops.rsx.smore_spectral(torch.empty(9, 32, device="cuda"), torch.empty(64, 32, device="cuda"),
                                                  torch.empty(64, device="cuda"), torch.empty(9, 16, device="cuda"),
                                                  torch.empty(64, 16, device="cuda"), torch.empty(64, device="cuda"),
                                                  torch.empty(1, 33, 2, device="cuda"), torch.empty(1, 33, 2, device="cuda"),
                                                  torch.empty(1, 33, 2, device="cuda"), True)
        assert cv.shape == (9, 64)


# ---------------------------------------------------------------------------
# the CPU kernels against the golden fixtures and the reference's torch ops
# ---------------------------------------------------------------------------
def _close(got, want, name, tol=1e-5):
    g = got.detach().double()
    w = torch.as_tensor(want).detach().double()
    scale = max(w.abs().max().item(), 1e-30)
    err = (g - w).abs().max().item()
    assert err <= tol * scale, f"{name}: {err:.3g} vs scale {scale:.3g}"


def _csr(z):
    """The fixture's normalised adjacency (the reference's get_norm_adj_mat, lightgcn.py:65-103)
    as CSR tensors (rowptr int64, col int32, val f32) and as a dense torch matrix."""
    nu, ni = int(z["n_users"]), int(z["n_items"])
    n = nu + ni
    idx, val = z["adj_idx"], z["adj_val"]
    rp, col, v = graph.to_csr(idx[0].astype(np.int64), idx[1].astype(np.int64), val, n, n)
    dense = torch.sparse_coo_tensor(torch.from_numpy(idx.astype(np.int64)), torch.from_numpy(val), (n, n)).to_dense()
    return (torch.from_numpy(rp), torch.from_numpy(col.astype(np.int32)), torch.from_numpy(v.astype(np.float32))), \
        dense, nu, ni


def test_spmm_csr_and_grad(golden):
    (rp, col, val), Ad, nu, ni = _csr(golden("lightgcn_small"))
    n = nu + ni
    # a rectangular block (users x all) exercises the transposed-CSR backward
    urp = rp[: nu + 1].clone()
    ucol, uval = col[: int(urp[-1])].clone(), val[: int(urp[-1])].clone()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, 64, generator=g, requires_grad=True)
    y = torch.ops.rsx.spmm_csr(urp, ucol, uval, x, n)
    up = torch.randn(y.shape, generator=g)
    (gx,) = torch.autograd.grad((y * up).sum(), [x])
    xw = x.detach().clone().requires_grad_(True)
    yw = Ad[:nu] @ xw
    (gw,) = torch.autograd.grad((yw * up).sum(), [xw])
    _close(y, yw, "spmm")
    _close(gx, gw, "spmm grad")


def test_lightgcn_forward_loss_grads_adam_vs_fixture(golden):
    """The reference's first LightGCN batch through the ops: propagate_mean (K=3) = the
    fixture's forward tables, bpr_loss = its step-0 loss, autograd through both = its
    step-0 gradients, adam_ = its parameters after the first Adam step."""
    z = golden("lightgcn_small")
    (rp, col, val), _, nu, ni = _csr(z)
    U0, I0 = params(z, "init.", "LightGCN")
    p = torch.from_numpy(np.concatenate([U0, I0])).requires_grad_(True)
    f = torch.ops.rsx.propagate_mean(rp, col, val, p, 3)
    np.testing.assert_allclose(f[:nu].detach().numpy(), z["fwd_user"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(f[nu:].detach().numpy(), z["fwd_item"], rtol=1e-5, atol=1e-7)
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    loss = torch.ops.rsx.bpr_loss(f, p, trip, nu, 1e-2, 0, 0.0)
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    (gp,) = torch.autograd.grad(loss, [p])
    gu, gi = params(z, "step0_grad.", "LightGCN")
    _close(gp[:nu], gu, "user grad", 1e-4)
    _close(gp[nu:], gi, "item grad", 1e-4)
    w = p.detach().clone()
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    torch.ops.rsx.adam_(w, gp, m, v, torch.tensor(1), 1e-3, 0.9, 0.999, 1e-8, 0.0)
    pu, pi = params(z, "step0_param.", "LightGCN")
    np.testing.assert_allclose(w[:nu].numpy(), pu, rtol=0, atol=2e-6)
    np.testing.assert_allclose(w[nu:].numpy(), pi, rtol=0, atol=2e-6)


@pytest.mark.parametrize("K", [1, 3])
def test_propagate_mean_grad_vs_torch(golden, K):
    (rp, col, val), Ad, nu, ni = _csr(golden("lightgcn_small"))
    g = torch.Generator().manual_seed(K)
    x = torch.randn(nu + ni, 64, generator=g, requires_grad=True)
    y = torch.ops.rsx.propagate_mean(rp, col, val, x, K)
    up = torch.randn(y.shape, generator=g)
    (gx,) = torch.autograd.grad((y * up).sum(), [x])
    xw = x.detach().clone().requires_grad_(True)
    layers, cur = [xw], xw
    for _ in range(K):
        cur = Ad @ cur
        layers.append(cur)
    yw = torch.stack(layers, 1).mean(1)  # reference lightgcn.py:121-127
    (gw,) = torch.autograd.grad((yw * up).sum(), [xw])
    _close(y, yw, "propagate_mean")
    _close(gx, gw, "propagate_mean grad")


def test_layergcn_forward_loss_grads_vs_fixture(golden):
    """LayerGCN (K=2) on the fixture: propagate_layergcn = the fixture's forward tables;
    bpr_loss (variant 1: sum BPR + L2) through it (the fixture trains with dropout 0: the
    full normalised graph) = its step-0 loss and gradients; adam_ = its step-0 parameters."""
    z = golden("layergcn_small")
    (rp, col, val), _, nu, ni = _csr(z)
    U0, I0 = params(z, "init.", "LayerGCN")
    p = torch.from_numpy(np.concatenate([U0, I0])).requires_grad_(True)
    f = torch.ops.rsx.propagate_layergcn(rp, col, val, p, 2)
    np.testing.assert_allclose(f[:nu].detach().numpy(), z["fwd_user"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(f[nu:].detach().numpy(), z["fwd_item"], rtol=1e-5, atol=1e-7)
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    loss = torch.ops.rsx.bpr_loss(f, p, trip, nu, 1e-2, 1, 0.0)
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    (gp,) = torch.autograd.grad(loss, [p])
    gu, gi = params(z, "step0_grad.", "LayerGCN")
    _close(gp[:nu], gu, "user grad", 1e-4)
    _close(gp[nu:], gi, "item grad", 1e-4)
    w = p.detach().clone()
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    torch.ops.rsx.adam_(w, gp, m, v, torch.tensor(1), 1e-3, 0.9, 0.999, 1e-8, 0.0)
    pu, pi = params(z, "step0_param.", "LayerGCN")
    np.testing.assert_allclose(w[:nu].numpy(), pu, rtol=0, atol=2e-6)
    np.testing.assert_allclose(w[nu:].numpy(), pi, rtol=0, atol=2e-6)


@pytest.mark.parametrize("K", [1, 2, 4])
def test_propagate_layergcn_grad_vs_torch(golden, K):
    (rp, col, val), Ad, nu, ni = _csr(golden("lightgcn_small"))
    g = torch.Generator().manual_seed(10 + K)
    x = (torch.randn(nu + ni, 64, generator=g) * 0.1).requires_grad_(True)
    y = torch.ops.rsx.propagate_layergcn(rp, col, val, x, K)
    up = torch.randn(y.shape, generator=g)
    (gx,) = torch.autograd.grad((y * up).sum(), [x])
    xw = x.detach().clone().requires_grad_(True)
    cur, out = xw, 0
    for _ in range(K):  # reference layergcn.py:127-140
        cur = Ad @ cur
        w = F.cosine_similarity(cur, xw, dim=-1)
        cur = torch.einsum("a,ab->ab", w, cur)
        out = out + cur
    (gw,) = torch.autograd.grad((out * up).sum(), [xw])
    _close(y, out, "layergcn", 2e-5)
    _close(gx, gw, "layergcn grad", 1e-4)


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_bpr_loss_and_grad_vs_torch(golden, variant):
    z = golden("lightgcn_small")
    nu, ni = int(z["n_users"]), int(z["n_items"])
    g = torch.Generator().manual_seed(variant)
    fin = (torch.randn(nu + ni, 64, generator=g) * 0.1).requires_grad_(True)
    ego = (torch.randn(nu + ni, 64, generator=g) * 0.1).requires_grad_(True)
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    reg = 1e-2
    loss = torch.ops.rsx.bpr_loss(fin, ego if variant != 2 else None, trip, nu, reg, variant, 2048.0)
    leaves = [fin, ego] if variant != 2 else [fin]
    got_g = torch.autograd.grad(loss, leaves)
    fl, el = fin.detach().clone().requires_grad_(True), ego.detach().clone().requires_grad_(True)
    u, p_, n_ = trip[0], trip[1] + nu, trip[2] + nu
    ps, ns = (fl[u] * fl[p_]).sum(1), (fl[u] * fl[n_]).sum(1)
    if variant == 0:  # lightgcn.py:132-156
        ref = -torch.log(1e-10 + torch.sigmoid(ps - ns)).mean() + reg * sum(
            torch.norm(x, p=2) for x in (el[u], el[p_], el[n_])) / trip.shape[1]
    elif variant == 1:  # layergcn.py:142-177
        ref = torch.sum(-F.logsigmoid(ps - ns)) + reg * sum(torch.sum(x ** 2) * 0.5 for x in (el[u], el[p_], el[n_]))
    else:  # smore.py:366-378
        ref = -torch.mean(F.logsigmoid(ps - ns)) + reg * 0.5 * (
            (fl[u] ** 2).sum() + (fl[p_] ** 2).sum() + (fl[n_] ** 2).sum()) / 2048.0
    want_g = torch.autograd.grad(ref, [fl, el] if variant != 2 else [fl])
    _close(loss, ref, "loss")
    for a, b in zip(got_g, want_g):
        _close(a, b, "bpr grad", 1e-4)


@pytest.mark.parametrize("fx,model,tag", [("lightgcn_small", "LightGCN", "epoch2"),
                                          ("layergcn_small", "LayerGCN", "epoch1")])
def test_fullsort_topk_vs_fixture(golden, fx, model, tag):
    """The reference's top-50 of its trained model (scores on the full graph, training
    items masked to -1e10, trainer.py:509-528): indices exact wherever the fixture flags
    no tie in that row."""
    z = golden(fx)
    (rp, col, val), _, nu, ni = _csr(z)
    pu, pi = params(z, f"{tag}_param.", model)
    p = torch.from_numpy(np.concatenate([pu, pi]))
    with torch.no_grad():
        f = (torch.ops.rsx.propagate_mean(rp, col, val, p, 3) if model == "LightGCN"
             else torch.ops.rsx.propagate_layergcn(rp, col, val, p, 2))
    users = torch.from_numpy(z[f"{tag}_valid_users"].astype(np.int64))
    hrp, hcol = graph.history_csr(z["train_u"], z["train_i"], nu)
    _, idx = torch.ops.rsx.fullsort_topk(f[:nu].contiguous(), users, f[nu:].contiguous(), torch.from_numpy(hrp),
                                         torch.from_numpy(hcol), 50)
    ref = z[f"{tag}_valid_topk_idx"].astype(np.int64)
    ties = z[f"{tag}_valid_inner_tie"] | z[f"{tag}_valid_boundary_tie"]
    ok = np.all(idx.numpy() == ref, axis=1)
    assert np.all(ok | ties) and ok.mean() > 0.9


def test_fullsort_topk_canonical_order_and_mask(golden):
    """Exact (score desc, index asc) order with masked items at -1e10, against the
    oracle's canonical top-k of the fixture's own init scores."""
    z = golden("lightgcn_small")
    nu = int(z["n_users"])
    f = np.concatenate([z["fwd_user"], z["fwd_item"]])
    users = z["init_valid_users"].astype(np.int64)
    hrp, hcol = graph.history_csr(z["train_u"], z["train_i"], nu)
    val, idx = torch.ops.rsx.fullsort_topk(torch.from_numpy(f[:nu]), torch.from_numpy(users),
                                           torch.from_numpy(f[nu:]), torch.from_numpy(hrp), torch.from_numpy(hcol), 50)
    scores = z["init_valid_scores"].copy()
    r, c = train_mask_pairs(z, users)
    scores[r, c] = -1e10
    cv, ci = O.canonical_topk(scores, 50)
    ties = z["init_valid_inner_tie"] | z["init_valid_boundary_tie"]
    ok = np.all(idx.numpy() == ci, axis=1)
    assert np.all(ok | ties)
    np.testing.assert_allclose(val.numpy(), cv, rtol=1e-5, atol=1e-6)


def test_adam_op_vs_torch():
    g = torch.Generator().manual_seed(3)
    p = torch.randn(300, 64, generator=g)
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([ref], lr=1e-3, weight_decay=1e-4, foreach=False)
    w, m, v = p.clone(), torch.zeros(300, 64), torch.zeros(300, 64)
    step = torch.zeros((), dtype=torch.int64)
    for _ in range(3):
        grad = torch.randn(300, 64, generator=g)
        ref.grad = grad.clone()
        opt.step()
        step += 1
        torch.ops.rsx.adam_(w, grad, m, v, step, 1e-3, 0.9, 0.999, 1e-8, 1e-4)
    np.testing.assert_allclose(w.numpy(), ref.detach().numpy(), rtol=0, atol=1e-6)


def test_thread_count_does_not_change_results(golden, monkeypatch):
    """Every output row is written by one worker in a fixed order: the same bits at any
    RSX_CPU_THREADS (the count is read once per process, so a child process checks 1)."""
    import subprocess
    import sys

    (rp, col, val), _, nu, ni = _csr(golden("lightgcn_small"))
    x = torch.randn(nu + ni, 64, generator=torch.Generator().manual_seed(0))
    y = torch.ops.rsx.propagate_layergcn(rp, col, val, x, 2)
    code = ("import sys, numpy as np, torch; sys.path[:0] = sys.argv[1:3]; import rsx; "
            "a = np.load(sys.argv[3]); t = [torch.from_numpy(a[k]) for k in ('rp', 'col', 'val', 'x')]; "
            "np.save(sys.argv[4], torch.ops.rsx.propagate_layergcn(*t, 2).numpy())")
    import os
    import tempfile

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        np.savez(os.path.join(d, "in.npz"), rp=rp.numpy(), col=col.numpy(), val=val.numpy(), x=x.numpy())
        env = dict(os.environ, RSX_CPU_THREADS="1")
        subprocess.run([sys.executable, "-c", code, repo, os.path.join(repo, "recommendar-systems_amd"),
                        os.path.join(d, "in.npz"), os.path.join(d, "out.npy")], check=True, env=env)
        y1 = np.load(os.path.join(d, "out.npy"))
    assert np.array_equal(y.numpy(), y1)
