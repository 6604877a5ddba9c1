"""SMORE sharded over 2 and 4 CPU ranks (rsx.smore_dist, gloo) against the single-process
objective: the oracle's SMORE restatement (oracle/rsx_oracle.py:SMORECPU, pinned to the
reference's own forward / loss by tests/test_oracle_smore.py) on the golden fixture's
data and initial weights.  The HIP kernels cannot run here, so the sharded model's
compute backend is a torch restatement of the same ops; what is under test is the
partition (user / item row ranges, local operator row blocks), the differentiable
gathers and the replicated-gradient sum.  One batch: the loss equals the
single-process loss, every parameter's gradient (the sharded rows gathered) equals
the single-process gradient, and one Adam step gives the same parameters."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

import rsx_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class TorchSmoreBackend:
    """torch restatement of the ops rsx.smore_dist.HipSmoreBackend runs (reference
    src/models/smore.py:209-411)."""

    def operator(self, rowptr, col, val, n_cols):
        rows = np.repeat(np.arange(rowptr.size - 1), np.diff(rowptr))
        return torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])),
                                       torch.from_numpy(val.astype(np.float32)),
                                       (rowptr.size - 1, n_cols)).coalesce()

    def spmm(self, op, x):
        return torch.sparse.mm(op, x)

    def spectral(self, m, V, T):
        img, txt = F.linear(V, m.image_trs.weight, m.image_trs.bias), F.linear(T, m.text_trs.weight, m.text_trs.bias)
        fi, ft = torch.fft.rfft(img, dim=1, norm="ortho"), torch.fft.rfft(txt, dim=1, norm="ortho")

        def unit(w):
            wc = torch.view_as_complex(w)
            return wc / (torch.abs(wc) + 1e-8)

        n = img.shape[1]
        return (torch.fft.irfft(fi * unit(m.image_complex_weight), n=n, dim=1, norm="ortho"),
                torch.fft.irfft(ft * unit(m.text_complex_weight), n=n, dim=1, norm="ortho"),
                torch.fft.irfft(ft * fi * unit(m.fusion_complex_weight), n=n, dim=1, norm="ortho"))

    def gates(self, m, cv, ct, cf, item):
        return (item + m.inject_scale * m.gate_v(cv), item + m.inject_scale * m.gate_t(ct),
                item + m.inject_scale * m.gate_f(cf))

    def preference(self, m, C, IE, TE, FE):
        agg_img = torch.softmax(m.query_v(FE), dim=-1) * IE
        agg_txt = torch.softmax(m.query_t(FE), dim=-1) * TE
        ip, tp, fp = (m.dropout(m.gate_image_prefer(C)), m.dropout(m.gate_text_prefer(C)),
                      m.dropout(m.gate_fusion_prefer(C)))
        side = torch.mean(torch.stack([ip * agg_img, tp * agg_txt, fp * FE]), dim=0)
        return C + side, side

    def loss(self, m, all_e, side, content, inter):
        nu = m.n_users
        users, pos, neg = inter[0], inter[1], inter[2]
        ua, ia = all_e[:nu], all_e[nu:]
        u, p, n = ua[users], ia[pos], ia[neg]
        ps, ns = (u * p).sum(dim=1), (u * n).sum(dim=1)
        reg = (0.5 * (u ** 2).sum() + 0.5 * (p ** 2).sum() + 0.5 * (n ** 2).sum()) / m.batch_size
        mf = -torch.mean(F.logsigmoid(ps - ns))
        su, si, cu, ci = side[:nu], side[nu:], content[:nu], content[nu:]
        cl = O.SMORECPU.info_nce(si[pos], ci[pos], m.cl_temp) + O.SMORECPU.info_nce(su[users], cu[users], m.cl_temp)
        return mf + m.reg_weight * reg + 0.0 + m.cl_loss * cl

    def mean_layers(self, layers):
        return torch.stack(layers, dim=1).mean(dim=1)


def _csr(sp):
    sp = sp.coalesce()
    i = sp.indices().numpy()
    from rsx import graph

    return graph.to_csr(i[0], i[1], sp.values().numpy(), sp.shape[0], sp.shape[1])


def reference_setup():
    z = dict(np.load(os.path.join(GOLD, "smore_small.npz")))
    nu, ni = int(z["n_users"]), int(z["n_items"])
    init = {k[5:]: z[k] for k in z if k.startswith("init.")}
    torch.manual_seed(0)
    m = O.SMORECPU(z["train_u"], z["train_i"], nu, ni, z["v_feat"], z["t_feat"], d=64, image_k=10, text_k=8,
                   dropout=0.0, batch_size=2048, init=init)
    graphs = {"norm_adj": _csr(m.norm_adj), "R": _csr(m.R), "image": _csr(m.image_original_adj),
              "text": _csr(m.text_original_adj), "fusion": _csr(m.fusion_adj)}
    batch = torch.from_numpy(z["epoch0_triplets"][:, :300].astype(np.int64))
    return m, init, graphs, batch, nu, ni


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.smore_dist import ShardedSMORE

    _, init, graphs, batch, nu, ni = reference_setup()
    sm = ShardedSMORE(init, graphs, nu, ni, dict(reg_weight=1e-5, batch_size=2048, n_ui_layers=4, n_layers=1),
                      TorchSmoreBackend())
    loss = sm.calculate_loss(batch)
    loss.backward()
    sm.sync_grads()
    grads = {n: p.grad.clone().numpy() for n, p in sm.named_parameters()}
    opt = torch.optim.Adam(sm.parameters(), lr=1e-3)
    opt.step()
    params = {n: p.detach().clone().numpy() for n, p in sm.named_parameters()}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=loss.detach().numpy(), own=np.array([*sm.own_u, *sm.own_i]),
             **{"g." + k: v for k, v in grads.items()}, **{"p." + k: v for k, v in params.items()})
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _close(a, b, name, tol=2e-5):
    scale = max(np.abs(b).max(), 1e-12)
    err = np.abs(a - b).max()
    assert err <= tol * scale, f"{name}: {err:.3g} vs scale {scale:.3g}"


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_smore_step_matches_single_process(world):
    from rsx.smore_dist import SHARDED

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    m, _, _, batch, nu, ni = reference_setup()
    loss = m.calculate_loss(batch)
    loss.backward()
    ref_g = {n: p.grad.clone().numpy() for n, p in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    opt.step()
    ref_p = {n: p.detach().clone().numpy() for n, p in m.named_parameters()}
    # every rank's loss is 1/W of the single-process loss
    assert abs(sum(float(x["loss"]) for x in res) - loss.item()) <= 1e-5 * abs(loss.item())
    for name in ref_g:
        if name in SHARDED:
            g = np.concatenate([x["g." + name] for x in res])
            p = np.concatenate([x["p." + name] for x in res])
        else:
            g, p = res[0]["g." + name], res[0]["p." + name]
            for x in res[1:]:  # replicas stay identical
                assert np.array_equal(x["p." + name], p), name
        _close(g, ref_g[name], "grad " + name)
        np.testing.assert_allclose(p, ref_p[name], rtol=0, atol=2e-6, err_msg=name)


def _mg_worker(rank, world, port, out, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsx.smore_dist import ShardedSMORE

    _, init, graphs, batch, nu, ni = reference_setup()
    sm = ShardedSMORE(init, graphs, nu, ni, dict(reg_weight=1e-5, batch_size=2048, n_ui_layers=4, n_layers=1),
                      TorchSmoreBackend())
    opt = torch.optim.Adam(sm.parameters(), lr=1e-3)
    losses = [sm.train_batch(batch, opt, 1e-3, step + 1, mg_interval=1) for step in range(steps)]
    params = {n: p.detach().clone().numpy() for n, p in sm.named_parameters()}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=np.array(losses), **{"p." + k: v for k, v in params.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_smore_mirror_gradient_matches_single_process(world):
    """Two batches with the model-level mirror gradient firing on each (mg_interval 1):
    the sharded model's loss and every parameter (rows concatenated over the ranks)
    against the oracle's single-process Trainer batch (smore_train_batch)."""
    from rsx.smore_dist import SHARDED

    steps = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_mg_worker, args=(world, _free_port(), d, steps), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    m, _, _, batch, nu, ni = reference_setup()
    m.mg_interval = 1
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    ref_losses = [O.smore_train_batch(m, opt, batch, 1e-3) for _ in range(steps)]
    np.testing.assert_allclose(sum(x["loss"] for x in res), ref_losses, rtol=1e-5)
    for name, p in m.named_parameters():
        want = p.detach().numpy()
        got = np.concatenate([x["p." + name] for x in res]) if name in SHARDED else res[0]["p." + name]
        np.testing.assert_allclose(got, want, rtol=0, atol=2e-5, err_msg=name)
