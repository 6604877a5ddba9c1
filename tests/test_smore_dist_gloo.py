"""SMORE with users sharded over 2 and 4 CPU ranks and the item side replicated
(rsx.smore_dist, gloo) against the single-process objective: the oracle's SMORE
restatement (oracle/rsx_oracle.py:SMORECPU, pinned to the reference's own forward /
loss by tests/test_oracle_smore.py) on the golden fixture's data and initial weights.

Each rank trains on its own batch of its own users' interactions, so the objective is
the sum over ranks of the reference loss of each rank's batch (data-parallel batches).
The HIP kernels cannot run here, so the sharded model's compute backend is a torch
restatement of the same ops; what is under test is the partition (user row blocks of
the UI graph and of R, the replicated item side), the collective schedule (one
all-reduce of the item partial per UI layer, the views' item-row gradients summed in
one all-reduce, the preference weights' gradients summed) and that the replicas stay
identical.  One batch: losses, every gradient and one Adam step; and two batches with
the model-level mirror gradient (global alpha over the sharded parameter vector)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import init_pg, store_path
import torch.nn.functional as F

import rsx_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sp(rowptr, col, val, n_cols):
    rows = np.repeat(np.arange(rowptr.size - 1), np.diff(rowptr))
    return torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])),
                                   torch.from_numpy(val.astype(np.float32)), (rowptr.size - 1, n_cols)).coalesce()


class _Pair:
    def __init__(self, A):
        self.A, self.AT = A, A.t().coalesce()


class TorchSmoreBackend:
    """torch restatement of the ops rsx.smore_dist.HipSmoreBackend runs (reference
    src/models/smore.py:209-411), with the same collectives."""

    def operator(self, rowptr, col, val, n_cols, transpose=False):
        A = _sp(rowptr, col, val, n_cols)
        return _Pair(A) if transpose else A

    def ui_mean(self, core, x):
        nu, K = core.nu_own, core.K
        s, cur = x.clone(), x
        for _ in range(K):
            u = torch.sparse.mm(core.A_U, cur[nu:])
            i = torch.sparse.mm(core.A_I, cur[:nu]).contiguous()
            core.comm.allreduce_(i)
            cur = torch.cat([u, i])
            s = s + cur
        return s / (K + 1)

    def spectral(self, m):
        img = F.linear(m.image_embedding.weight, m.image_trs.weight, m.image_trs.bias)
        txt = F.linear(m.text_embedding.weight, m.text_trs.weight, m.text_trs.bias)
        fi, ft = torch.fft.rfft(img, dim=1, norm="ortho"), torch.fft.rfft(txt, dim=1, norm="ortho")

        def unit(w):
            wc = torch.view_as_complex(w)
            return wc / (torch.abs(wc) + 1e-8)

        n = img.shape[1]
        return (torch.fft.irfft(fi * unit(m.image_complex_weight), n=n, dim=1, norm="ortho"),
                torch.fft.irfft(ft * unit(m.text_complex_weight), n=n, dim=1, norm="ortho"),
                torch.fft.irfft(ft * fi * unit(m.fusion_complex_weight), n=n, dim=1, norm="ortho"))

    def item_side_sharded(self, core, m, item):
        """The item side on this rank's item rows (m's feature tables hold them), the inject
        terms gathered (rsx.smore_dist.gather_rows) and added to the replicated item table."""
        from rsx.smore_dist import ITEM_W, allreduce_grad, gather_rows

        w = dict(zip(ITEM_W, allreduce_grad(core.comm, *[m.get_parameter(n) for n in ITEM_W])))
        img = F.linear(m.image_embedding.weight, w["image_trs.weight"], w["image_trs.bias"])
        txt = F.linear(m.text_embedding.weight, w["text_trs.weight"], w["text_trs.bias"])
        fi, ft = torch.fft.rfft(img, dim=1, norm="ortho"), torch.fft.rfft(txt, dim=1, norm="ortho")

        def unit(x):
            wc = torch.view_as_complex(x)
            return wc / (torch.abs(wc) + 1e-8)

        n = img.shape[1]
        cv = torch.fft.irfft(fi * unit(w["image_complex_weight"]), n=n, dim=1, norm="ortho")
        ct = torch.fft.irfft(ft * unit(w["text_complex_weight"]), n=n, dim=1, norm="ortho")
        cf = torch.fft.irfft(ft * fi * unit(w["fusion_complex_weight"]), n=n, dim=1, norm="ortho")
        s = m.inject_scale
        D = gather_rows(core.comm, core.iq, core.n_items,
                        s * torch.sigmoid(F.linear(cv, w["gate_v.0.weight"], w["gate_v.0.bias"])),
                        s * torch.sigmoid(F.linear(ct, w["gate_t.0.weight"], w["gate_t.0.bias"])),
                        s * torch.sigmoid(F.linear(cf, w["gate_f.0.weight"], w["gate_f.0.bias"])))
        return (D + item.unsqueeze(0)).unbind(0)

    def gates(self, m, cv, ct, cf, item):
        return (item + m.inject_scale * m.gate_v(cv), item + m.inject_scale * m.gate_t(ct),
                item + m.inject_scale * m.gate_f(cf))

    def views(self, core, xs):
        from rsx.smore_dist import allreduce_grad

        outs = []
        for x, G in zip(xs, core.G):
            for _ in range(core.L):
                x = torch.sparse.mm(G.A, x)
            outs.append(x)
        outs = allreduce_grad(core.comm, *outs)
        return tuple(torch.cat([torch.sparse.mm(core.R.A, x), x]) for x in outs)

    @staticmethod
    def _pref(C, IE, TE, FE, w):
        (qv0, qv2, qt0, qt2, gi, gt, gf), (bqv0, _, bqt0, _, bgi, bgt, bgf) = w[:7], w[7:]
        agg_img = torch.softmax(F.linear(torch.tanh(F.linear(FE, qv0, bqv0)), qv2), dim=-1) * IE
        agg_txt = torch.softmax(F.linear(torch.tanh(F.linear(FE, qt0, bqt0)), qt2), dim=-1) * TE
        ip, tp, fp = (torch.sigmoid(F.linear(C, gi, bgi)), torch.sigmoid(F.linear(C, gt, bgt)),
                      torch.sigmoid(F.linear(C, gf, bgf)))
        side = torch.mean(torch.stack([ip * agg_img, tp * agg_txt, fp * FE]), dim=0)
        return C + side, side

    def pref_rows(self, m, content, views, rows, seed, weights):
        C = content[rows]
        a, s = self._pref(C, *(v[rows] for v in views), weights)
        return a, s, C

    def pref_full(self, m, content, views, seed):
        from rsx.smore_dist import PREF

        lin = [m.get_submodule(n) for n in PREF]
        return self._pref(content, *views, [x.weight for x in lin] + [x.bias for x in lin])

    def loss_rows(self, m, all_c, side_c, content_c, trip, ar, B):
        u, p, n = all_c[:B], all_c[B:2 * B], all_c[2 * B:]
        ps, ns = (u * p).sum(dim=1), (u * n).sum(dim=1)
        reg = (0.5 * (u ** 2).sum() + 0.5 * (p ** 2).sum() + 0.5 * (n ** 2).sum()) / m.batch_size
        mf = -torch.mean(F.logsigmoid(ps - ns))
        cl = (O.SMORECPU.info_nce(side_c[B:2 * B], content_c[B:2 * B], m.cl_temp)
              + O.SMORECPU.info_nce(side_c[:B], content_c[:B], m.cl_temp))
        return mf + m.reg_weight * reg + m.cl_loss * cl


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
    return m, init, graphs, z, nu, ni


def rank_batches(z, nu, world, per=120):
    """Each rank's batch: the first `per` fixture triplets whose user is in its block
    (global ids)."""
    from rsx.smore_dist import ranges

    t = z["epoch0_triplets"].astype(np.int64)
    out = []
    for a, b in ranges(nu, world):
        sel = np.nonzero((t[0] >= a) & (t[0] < b))[0][:per]
        out.append(torch.from_numpy(t[:, sel].copy()))
    return out


CFG = dict(reg_weight=1e-5, batch_size=2048, cl_loss=0.01, cl_temp=0.2, dropout_rate=0.0)


def _setup_rank(rank, world, store, item_shard=False):
    torch.set_num_threads(1)
    init_pg("gloo", rank, world, store)
    from rsx.smore_dist import Comm, SmoreShard, param_container

    _, init, graphs, z, nu, ni = reference_setup()
    core = SmoreShard(graphs, nu, ni, 4, 1, TorchSmoreBackend(), Comm(), item_shard=item_shard)
    assert core.item_shard == item_shard
    m = param_container(init, CFG, core.own_u, item_range=core.own_i if item_shard else None)
    inter = rank_batches(z, nu, world)[rank].clone()
    inter[0] -= core.own_u[0]  # local user rows
    return core, m, inter


def _sharded_names(item_shard):
    from rsx.smore_dist import ITEM_SHARDED, SHARDED

    return set(SHARDED) | (set(ITEM_SHARDED) if item_shard else set())


def _worker(rank, world, store, out, item_shard=False):
    core, m, inter = _setup_rank(rank, world, store, item_shard)
    loss = core.loss(m, inter, None)
    loss.backward()
    grads = {n: p.grad.clone().numpy() for n, p in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    opt.step()
    params = {n: p.detach().clone().numpy() for n, p in m.named_parameters()}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=loss.detach().numpy(), own=np.array(core.own_u),
             **{"g." + k: v for k, v in grads.items()}, **{"p." + k: v for k, v in params.items()})
    dist.destroy_process_group()



def _close(a, b, name, tol=2e-5):
    scale = max(np.abs(b).max(), 1e-12)
    err = np.abs(a - b).max()
    assert err <= tol * scale, f"{name}: {err:.3g} vs scale {scale:.3g}"


@pytest.mark.parametrize("world,item_shard", [(2, False), (4, False), (2, True), (4, True)])
def test_sharded_smore_step_matches_single_process(world, item_shard):
    """item_shard: the item side (projection, spectral fusion, the gates' inject term)
    computed on each rank's item rows, the raw feature tables row-sharded with it."""
    SHARDED = _sharded_names(item_shard)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, store_path(), d, item_shard), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    m, _, _, z, nu, ni = reference_setup()
    batches = rank_batches(z, nu, world)
    loss = sum(m.calculate_loss(b) for b in batches)
    loss.backward()
    ref_g = {n: p.grad.clone().numpy() for n, p in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    opt.step()
    ref_p = {n: p.detach().clone().numpy() for n, p in m.named_parameters()}
    assert abs(sum(float(x["loss"]) for x in res) - loss.item()) <= 1e-5 * abs(loss.item())
    for name in ref_g:
        if name in SHARDED:
            g = np.concatenate([x["g." + name] for x in res])
            p = np.concatenate([x["p." + name] for x in res])
        else:
            g, p = res[0]["g." + name], res[0]["p." + name]
            for x in res[1:]:  # replicas stay identical
                assert np.array_equal(x["g." + name], g), name
                assert np.array_equal(x["p." + name], p), name
        _close(g, ref_g[name], "grad " + name)
        # Adam's first update is -lr g/(|g|+eps): a gradient rounding difference delta (here
        # 2e-5 of the tensor's scale: f32 sums in another order) moves it by at most
        # lr |s(g + delta) - s(g)|, s(x) = x / (|x| + eps) -- large only where g ~ 0
        gr = ref_g[name]
        delta = 2e-5 * np.abs(gr).max() + 1e-30
        sfn = lambda x: x / (np.abs(x) + 1e-8)  # noqa: E731
        bound = 1e-3 * np.maximum(np.abs(sfn(gr + delta) - sfn(gr)), np.abs(sfn(gr - delta) - sfn(gr))) + 2e-7
        assert np.all(np.abs(p - ref_p[name]) <= bound), (name, np.abs(p - ref_p[name]).max())


def _shard_train_batch(core, m, inter, opt, lr, step_id, mg_interval, base=0.5, beta=0.2):
    """rsx.trainer.Trainer._train_batch + _mirror_gradient on the sharded model
    (reference src/common/trainer.py:186-201, 244-336): loss, backward, Adam, then the
    mirror gradient with alpha over the global parameter vector (SmoreShard.mg_alpha)."""
    opt.zero_grad(set_to_none=True)
    loss = core.loss(m, inter, None)
    value = float(loss.detach())
    loss.backward()
    opt.step()
    if step_id % mg_interval == 0:
        opt.zero_grad(set_to_none=True)
        core.loss(m, inter, None).backward()
        params = [p for p in m.parameters() if p.grad is not None]
        grads = [p.grad.detach().clone() for p in params]
        alpha = float(core.mg_alpha(m, params, grads, base, lr, 1e-3, 20.0))
        with torch.no_grad():
            for p, g in zip(params, grads):
                p.add_(-alpha * lr * g)
        opt.zero_grad(set_to_none=True)
        core.loss(m, inter, None).backward()
        with torch.no_grad():
            for p in m.parameters():
                if p.grad is not None:
                    p.grad.mul_(-beta)
            for p, g in zip(params, grads):
                p.add_(alpha * lr * g)
        opt.step()
        opt.zero_grad(set_to_none=True)
    return value


def _mg_worker(rank, world, store, out, steps, item_shard=False):
    core, m, inter = _setup_rank(rank, world, store, item_shard)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = [_shard_train_batch(core, m, inter, opt, 1e-3, s + 1, 1) for s in range(steps)]
    params = {n: p.detach().clone().numpy() for n, p in m.named_parameters()}
    np.savez(os.path.join(out, f"r{rank}.npz"), loss=np.array(losses), **{"p." + k: v for k, v in params.items()})
    dist.destroy_process_group()


class _SumOfBatches:
    """The single-process objective sum_g L(batch_g) as one 'model' for the oracle's
    Trainer batch (smore_train_batch): global_step advances once per call."""

    def __init__(self, m):
        self.m, self.global_step, self.mg_interval = m, 0, 1
        self.mg_alpha, self.mg_beta = m.mg_alpha, m.mg_beta

    def calculate_loss(self, batches):
        self.global_step += 1
        return sum(self.m.calculate_loss(b) for b in batches)

    def parameters(self):
        return self.m.parameters()


@pytest.mark.parametrize("world,item_shard", [(2, False), (4, False), (4, True)])
def test_sharded_smore_mirror_gradient_matches_single_process(world, item_shard):
    """Two batches with the model-level mirror gradient firing on each (mg_interval 1):
    the ranks' losses and every parameter (user rows concatenated over the ranks)
    against the oracle's single-process Trainer batch on the sum of the rank batches."""
    SHARDED = _sharded_names(item_shard)
    steps = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_mg_worker, args=(world, store_path(), d, steps, item_shard), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    m, _, _, z, nu, ni = reference_setup()
    batches = rank_batches(z, nu, world)
    s = _SumOfBatches(m)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    ref_losses = [O.smore_train_batch(s, opt, batches, 1e-3) for _ in range(steps)]
    np.testing.assert_allclose(sum(x["loss"] for x in res), ref_losses, rtol=1e-5)
    for name, p in m.named_parameters():
        want = p.detach().numpy()
        got = np.concatenate([x["p." + name] for x in res]) if name in SHARDED else res[0]["p." + name]
        np.testing.assert_allclose(got, want, rtol=0, atol=2e-5, err_msg=name)


def _rowx_worker(rank, world, store, out, n_rows, d, n_max):
    """RowGradExchange (data-parallel SMORE's one exchange) on `world` gloo ranks, its CPU
    statement of csrc/rowx.hip: rank r's four tables are defined on its own batch rows only
    (garbage elsewhere), its rows repeat, its batch may be shorter than n_max."""
    from rsx.smore_dist import Comm, RowGradExchange

    init_pg("gloo", rank, world, store)
    g = torch.Generator().manual_seed(100 + rank)
    n = n_max - (rank % 2)  # unequal batches: the pad entries
    rows = torch.randint(0, n_rows, (n,), generator=g)
    rows[: n // 3] = rows[0]  # a hot row, repeated
    tables = [torch.full((n_rows, d), float("nan")) for _ in range(4)]  # garbage off the batch rows
    for t in tables:
        t[rows] = torch.randn(rows.numel(), d, generator=g)
    mine = [t[rows].clone() for t in tables]
    wg = [torch.randn(d, d, generator=g), None, torch.randn(d, generator=g)]
    ex = RowGradExchange(Comm(None, "cpu"), n_rows, d, n_max, "cpu")
    got = ex.exchange(rows, tables, wg)
    np.savez(os.path.join(out, f"r{rank}.npz"), rows=rows.numpy(), mine=np.stack([m.numpy() for m in mine]),
             union=ex.union.numpy(), tabs=np.stack([t.numpy() for t in tables]), wg0=wg[0].numpy(),
             wg2=wg[2].numpy(), got0=got[0].numpy(), got2=got[2].numpy(), none1=np.array(got[1] is None))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_row_grad_exchange_sums_the_ranks_rows_in_rank_order(world):
    n_rows, d, n_max = 97, 8, 40
    with tempfile.TemporaryDirectory() as out:
        mp.spawn(_rowx_worker, args=(world, store_path(), out, n_rows, d, n_max), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
    want = np.zeros((4, n_rows, d), np.float32)
    for x in res:  # each rank's row value once, ranks in order (f32 adds)
        seen = set()
        for j, row in enumerate(x["rows"].tolist()):
            if row not in seen:
                seen.add(row)
                want[:, row] = want[:, row] + x["mine"][:, j]
    union = sorted(set(np.concatenate([x["rows"] for x in res]).tolist()))
    for x in res:
        assert set(x["union"].tolist()) == set(union)
        assert np.array_equal(x["tabs"][:, union], want[:, union])  # bit for bit, every rank
        assert np.array_equal(x["tabs"][:, union], res[0]["tabs"][:, union])
        np.testing.assert_allclose(x["got0"], sum(y["wg0"] for y in res), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(x["got2"], sum(y["wg2"] for y in res), rtol=1e-6, atol=1e-6)
        assert bool(x["none1"])
        assert np.array_equal(x["got0"], res[0]["got0"])
