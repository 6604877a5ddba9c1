"""Pin the CPU oracle (and the product's host-side graph builders) to the reference's
own outputs captured in tests/golden/ by tools/capture_golden.py."""
import numpy as np
import pytest
import torch

import rsx_oracle as O
from helpers import coo_from, coo_sorted, csr_to_sorted, eval_lists, metric_dict, params
from rsx import graph


def _nm(z):
    return int(z["n_users"]), int(z["n_items"])


@pytest.mark.parametrize("fx", ["lightgcn_small", "layergcn_small"])
def test_norm_adj_bit_exact(golden, fx):
    z = golden(fx)
    nu, ni = _nm(z)
    ref = coo_sorted(z["adj_idx"], z["adj_val"])
    a = O.lightgcn_norm_adj_dok(z["train_u"], z["train_i"], nu, ni).coalesce()
    mine = coo_sorted(a.indices().numpy(), a.values().numpy())
    for x, y in zip(ref, mine):
        assert np.array_equal(x, y)
    b = O.lightgcn_norm_adj_vec(z["train_u"], z["train_i"], nu, ni)
    vec = coo_sorted(b.indices().numpy(), b.values().numpy())
    for x, y in zip(ref, vec):
        assert np.array_equal(x, y)
    # product host builder (CSR) -- bit-identical values
    rp, col, val = graph.lightgcn_norm_adj(z["train_u"], z["train_i"], nu, ni)
    r, c, v = csr_to_sorted(rp, col, val)
    assert np.array_equal(r, ref[0]) and np.array_equal(c, ref[1]) and np.array_equal(v, ref[2])


def test_lightgcn_forward_loss_grads_adam(golden):
    z = golden("lightgcn_small")
    nu, ni = _nm(z)
    A = coo_from(z, "adj", nu + ni)
    U0, I0 = params(z, "init.", "LightGCN")
    f = O.lightgcn_forward(A, torch.from_numpy(np.concatenate([U0, I0])), 3)
    np.testing.assert_allclose(f[:nu].numpy(), z["fwd_user"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(f[nu:].numpy(), z["fwd_item"], rtol=1e-6, atol=1e-7)
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    cpu = O.LightGCNCPU(A, U0, I0, 3, 1e-2)
    cpu.opt.zero_grad()
    loss = O.lightgcn_loss(cpu.u, cpu.i, A, 3, trip, 1e-2)
    loss.backward()
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-6 * abs(float(z["step0_loss"]))
    gu, gi = params(z, "step0_grad.", "LightGCN")
    np.testing.assert_allclose(cpu.u.grad.numpy(), gu, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(cpu.i.grad.numpy(), gi, rtol=1e-5, atol=1e-9)
    cpu.opt.step()
    pu, pi = params(z, "step0_param.", "LightGCN")
    np.testing.assert_allclose(cpu.u.detach().numpy(), pu, rtol=0, atol=1e-6)
    np.testing.assert_allclose(cpu.i.detach().numpy(), pi, rtol=0, atol=1e-6)


@pytest.mark.parametrize("fx", ["lightgcn_small", "layergcn_small", "layergcn_drop_small"])
def test_metrics_restatement(golden, fx):
    z = golden(fx)
    last = max(int(k[5]) for k in z if k.startswith("epoch") and k.endswith("_valid_metric_keys"))
    for split in ("valid", "test"):
        tag = f"epoch{last}_{split}"
        topk = z[tag + "_topk_idx"].astype(np.int64)
        out = O.metrics_reference(topk, eval_lists(z, split))
        assert out == pytest.approx(metric_dict(z, tag), abs=0)


def test_layergcn_edge_values_and_forward(golden):
    z = golden("layergcn_small")
    nu, ni = _nm(z)
    ev = graph.layergcn_edge_values(z["edge_idx"][0], z["edge_idx"][1], nu, ni)
    assert np.array_equal(ev, z["edge_val"])
    ov = O.layergcn_normalize(torch.from_numpy(z["edge_idx"]), nu, ni).numpy()
    assert np.array_equal(ov, z["edge_val"])
    A = coo_from(z, "adj", nu + ni)
    U0, I0 = params(z, "init.", "LayerGCN")
    f = O.layergcn_forward(A, torch.from_numpy(np.concatenate([U0, I0])), 2)
    np.testing.assert_allclose(f[:nu].numpy(), z["fwd_user"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(f[nu:].numpy(), z["fwd_item"], rtol=1e-5, atol=1e-7)


def test_layergcn_step0(golden):
    z = golden("layergcn_small")
    nu, ni = _nm(z)
    # dropout 0: the training graph is the eval graph (layergcn.py:52-54)
    A = coo_from(z, "adj", nu + ni)
    U0, I0 = params(z, "init.", "LayerGCN")
    u = torch.nn.Parameter(torch.from_numpy(U0.copy()))
    i = torch.nn.Parameter(torch.from_numpy(I0.copy()))
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    loss = O.layergcn_loss(u, i, A, 2, trip, 1e-2)
    loss.backward()
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    gu, gi = params(z, "step0_grad.", "LayerGCN")
    np.testing.assert_allclose(u.grad.numpy(), gu, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(i.grad.numpy(), gi, rtol=1e-4, atol=1e-7)


def test_layergcn_dropout_graph_renormalisation(golden):
    """Kept edges -> f32 renormalised symmetric graph equals the reference's masked_adj."""
    z = golden("layergcn_drop_small")
    nu, ni = _nm(z)
    for ep in (0, 1):
        idx, val = z[f"e{ep}_masked_idx"].astype(np.int64), z[f"e{ep}_masked_val"]
        half = idx.shape[1] // 2
        ku, ki = idx[0][:half], idx[1][:half] - nu
        rp, col, v = graph.layergcn_masked_adj(ku, ki, nu, ni)
        mine = csr_to_sorted(rp, col, v)
        ref = coo_sorted(idx, val)
        for x, y in zip(ref, mine):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("fx", ["smore_small", "smore_d128_small"])
def test_smore_graphs(golden, fx):
    z = golden(fx)
    nu, ni = _nm(z)
    n = nu + ni
    norm, R = O.smore_norm_adj(z["train_u"], z["train_i"], nu, ni)
    ref = coo_sorted(z["norm_adj_idx"], z["norm_adj_val"])
    mine = coo_sorted(norm.coalesce().indices().numpy(), norm.coalesce().values().numpy())
    for x, y in zip(ref, mine):
        assert np.array_equal(x, y)
    rp, col, val = graph.smore_norm_adj(z["train_u"], z["train_i"], nu, ni)
    prod = csr_to_sorted(rp, col, val)
    for x, y in zip(ref, prod):
        assert np.array_equal(x, y)
    # kNN graphs from the (trainable, initial) raw features
    for name, feat, k in (("image_original_adj", "v_feat", 10), ("text_original_adj", "t_feat", 8)):
        # (768-dim CLIP-like rows: the cosine GEMM's sums can differ in the last bit from the
        # reference run's, so values are compared at rtol 1e-6 and indices exactly)
        g = O.knn_normalized_graph(torch.from_numpy(z[feat]), k).coalesce()
        ref = coo_sorted(z[name + "_idx"], z[name + "_val"])
        mine = coo_sorted(g.indices().numpy(), g.values().numpy())
        assert np.array_equal(ref[0], mine[0]) and np.array_equal(ref[1], mine[1])
        np.testing.assert_allclose(mine[2], ref[2], rtol=1e-6, atol=0)
    fu = O.max_pool_fusion(O.knn_normalized_graph(torch.from_numpy(z["v_feat"]), 10),
                           O.knn_normalized_graph(torch.from_numpy(z["t_feat"]), 8))
    ref = coo_sorted(z["fusion_adj_idx"], z["fusion_adj_val"])
    mine = coo_sorted(fu.indices().numpy(), fu.values().numpy())
    assert np.array_equal(ref[0], mine[0]) and np.array_equal(ref[1], mine[1])
    np.testing.assert_allclose(mine[2], ref[2], rtol=1e-6, atol=0)
    assert n == norm.shape[0]


def test_canonical_topk_matches_reference_modulo_ties(golden):
    z = golden("lightgcn_small")
    nu, ni = _nm(z)
    scores = z["init_valid_scores"].copy()
    users = z["init_valid_users"]
    from helpers import train_mask_pairs
    r, c = train_mask_pairs(z, users)
    scores[r, c] = -1e10
    _, idx = O.canonical_topk(scores, 50)
    ref = z["init_valid_topk_idx"].astype(np.int64)
    ties = z["init_valid_inner_tie"] | z["init_valid_boundary_tie"]
    same = np.all(idx == ref, axis=1)
    assert np.all(same | ties)


def test_reference_knn_cache_is_read(golden, tmp_path):
    """SMORE reads the kNN cache the reference writes (smore.py:46-47,56-62: torch.save of
    the sparse [n_items, n_items] graph) through the safe loader; the graph it returns is
    the reference's own, and the product's host build (knn_graph) equals it too."""
    from rsx.smore import knn_graph, load_reference_knn

    z = golden("smore_small")
    ni = int(z["n_items"])
    for name, feat, k in (("image_original_adj", "v_feat", 10), ("text_original_adj", "t_feat", 8)):
        # (768-dim CLIP-like rows: the cosine GEMM's sums can differ in the last bit from the
        # reference run's, so values are compared at rtol 1e-6 and indices exactly)
        ref = coo_sorted(z[name + "_idx"], z[name + "_val"])
        t = torch.sparse_coo_tensor(torch.from_numpy(z[name + "_idx"]), torch.from_numpy(z[name + "_val"]),
                                    (ni, ni))
        path = tmp_path / f"{name}_{k}_True.pt"
        torch.save(t, path)
        r, c, v = load_reference_knn(str(path), ni)
        for x, y in zip(ref, coo_sorted(np.stack([r, c]), v)):
            assert np.array_equal(x, y)
        dense = tmp_path / f"{name}_{k}_False.pt"  # is_sparse False: the dense matrix
        torch.save(t.to_dense(), dense)
        r, c, v = load_reference_knn(str(dense), ni)
        for x, y in zip(ref, coo_sorted(np.stack([r, c]), v)):
            assert np.array_equal(x, y)
        hr, hc, hv = knn_graph(z[feat], k)
        for x, y in zip(ref, coo_sorted(np.stack([hr, hc]), hv)):
            assert np.array_equal(x, y)
    # absent, wrong shape, or not a tensor file: rebuilt instead
    assert load_reference_knn(str(tmp_path / "missing.pt"), ni) is None
    torch.save(torch.zeros(3, 3), tmp_path / "small.pt")
    assert load_reference_knn(str(tmp_path / "small.pt"), ni) is None
    (tmp_path / "junk.pt").write_bytes(b"not a torch file")
    assert load_reference_knn(str(tmp_path / "junk.pt"), ni) is None


def test_layergcn_cpu_class_step0(golden):
    """oracle.LayerGCNCPU (the C1 cpu_baseline): its first Adam step equals the reference's."""
    z = golden("layergcn_small")
    nu, ni = _nm(z)
    U0, I0 = params(z, "init.", "LayerGCN")
    m = O.LayerGCNCPU(z["train_u"], z["train_i"], nu, ni, U0, I0, 2, 1e-2, dropout=0.0)
    m.pre_epoch()
    loss = m.step(torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64)))
    assert abs(loss - float(z["step0_loss"])) <= 1e-5 * abs(float(z["step0_loss"]))
    pu, pi = params(z, "step0_param.", "LayerGCN")
    np.testing.assert_allclose(m.u.detach().numpy(), pu, rtol=0, atol=2e-6)
    np.testing.assert_allclose(m.i.detach().numpy(), pi, rtol=0, atol=2e-6)
