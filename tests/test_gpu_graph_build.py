"""The device graph builders (csrc/graph.hip) against the host builders of rsx/graph.py,
which tests/test_oracle_golden.py pins bit for bit to the reference's own matrices
(LightGCN.get_norm_adj_mat f64 -> f32, SMORE.get_adj_mat f32, LayerGCN's f32 edge
dropout renormalisation): rowptr, columns and values identical, on the golden data and
on synthetic graphs with duplicate interactions and isolated users / items."""
import numpy as np
import pytest
import torch

from rsx import graph, ops, synth

pytestmark = pytest.mark.gpu


def _graphs(golden):
    z = golden("lightgcn_small")
    yield "golden", z["train_u"].astype(np.int64), z["train_i"].astype(np.int64), int(z["n_users"]), int(z["n_items"])
    df = synth.amazon_like(*synth.SHAPES["sports"], seed=1)
    tr = df[df.x_label == 0]
    yield "sports", tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64), \
        int(df.userID.max()) + 1, synth.SHAPES["sports"][1]
    rng = np.random.default_rng(7)
    u = rng.integers(0, 500, 6000)
    i = rng.integers(0, 300, 6000)
    u[:100], i[:100] = u[100:200], i[100:200]  # duplicate pairs
    yield "dups_isolated", u, i, 520, 330  # users 500..519 and items 300..329 have no edges
    # every degree 1..4000 on the user side (user k has k items) and item degrees up to
    # 4000: the per-degree factors across the whole range a C4-like hub graph reaches
    nu, ni = 4000, 4000
    u = np.repeat(np.arange(nu), np.arange(1, nu + 1))
    i = np.concatenate([np.arange(k) for k in range(1, nu + 1)])
    yield "all_degrees", u, i, nu, ni


def test_dinv_table_is_the_host_pow():
    """The per-degree factor table equals the host builders' own expressions elementwise."""
    deg = np.arange(100001)
    t0 = ops.dinv_table(100000, ops.ADJ_LIGHTGCN)
    assert np.array_equal(t0.view(np.uint64), np.power(deg.astype(np.float64) + 1e-7, -0.5).view(np.uint64))
    t1 = ops.dinv_table(100000, ops.ADJ_SMORE)
    with np.errstate(divide="ignore"):
        want = np.power(deg.astype(np.float32), np.float32(-0.5)).astype(np.float32)
    want[np.isinf(want)] = 0
    assert np.array_equal(t1.astype(np.float32).view(np.uint32), want.view(np.uint32)) and t1[0] == 0


@pytest.mark.parametrize("mode", [ops.ADJ_LIGHTGCN, ops.ADJ_SMORE])
def test_adj_build_equals_host(cuda, golden, mode):
    host = graph.lightgcn_norm_adj if mode == ops.ADJ_LIGHTGCN else graph.smore_norm_adj
    for name, u, i, nu, ni in _graphs(golden):
        rp, col, val = ops.adj_build(u, i, nu, ni, mode, cuda)
        hrp, hcol, hval = host(u, i, nu, ni)
        assert np.array_equal(rp.cpu().numpy(), hrp), name
        assert np.array_equal(col.cpu().numpy(), hcol), name
        got = val.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), hval.view(np.uint32)), (name, np.abs(got - hval).max())


def test_adj_build_empty(cuda):
    rp, col, val = ops.adj_build(np.zeros(0, np.int64), np.zeros(0, np.int64), 5, 3, ops.ADJ_LIGHTGCN, cuda)
    assert rp.cpu().tolist() == [0] * 9 and col.numel() == 0 and val.numel() == 0


@pytest.mark.parametrize("pruning_random", [False, True])
def test_edge_dropout_build_equals_host(cuda, golden, pruning_random):
    from rsx.layergcn import DeviceEdgeDropout

    for name, u, i, nu, ni in _graphs(golden):
        key = np.unique(u * (1 << 32) + i)
        eu, ei = key >> 32, key & 0xFFFFFFFF
        w = graph.layergcn_edge_values(eu, ei, nu, ni)
        dd = DeviceEdgeDropout(eu, ei, nu, ni, w, cuda)
        keep_len = int(eu.size * 0.9)
        torch.manual_seed(3)
        mask = dd.keep_mask(keep_len, pruning_random)
        rp, col, val = dd.build(mask, keep_len)
        kept = mask.cpu().numpy()
        hrp, hcol, hval = graph.layergcn_masked_adj(eu[kept], ei[kept], nu, ni)
        assert np.array_equal(rp.cpu().numpy(), hrp), name
        assert np.array_equal(col.cpu().numpy(), hcol), name
        assert np.array_equal(val.cpu().numpy().view(np.uint32), hval.view(np.uint32)), name
