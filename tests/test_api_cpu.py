"""Host side of the drop-in surface, on CPU: YAML config layering, dataset split,
the reference-identical (host) triplet stream, and the evaluator's metrics."""
import os
import shutil

import numpy as np
import pytest
import torch

from helpers import eval_lists, metric_dict
from rsx.config import Config
from rsx.data import EvalDataLoader, RecDataset, TrainDataLoader
from rsx.evaluator import TopKEvaluator
from rsx.utils import early_stopping, init_seed

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture()
def data_root(tmp_path):
    d = tmp_path / "data" / "baby"
    d.mkdir(parents=True)
    shutil.copy(os.path.join(GOLD, "gold_small.inter"), d / "baby.inter")
    return str(tmp_path / "data") + "/"


def test_config_layering():
    c = Config("LightGCN", "sports", {"gpu_id": 0})
    assert c["n_layers"] == [4] and c["reg_weight"] == [0.01] and isinstance(c["reg_weight"][0], float)
    assert c["hyper_parameters"] == ["seed", "n_layers", "reg_weight"]
    assert c["USER_ID_FIELD"] == "userID" and c["inter_file_name"] == "sports.inter"
    assert c["valid_metric_bigger"] is True and c["train_batch_size"] == 2048
    assert c["learning_rate_scheduler"] == [1.0, 50]
    s = Config("SMORE", "clothing", {"epochs": 3})
    assert s["learning_rate_scheduler"] == [0.96, 50] and s["epochs"] == 3 and s["mg_enable"] is True
    assert s["vision_feature_file"] == "image_feat.npy"
    b = Config("LayerGCN", "baby", None, mg=True)
    assert b["hyper_parameters"][-3:] == ["alpha1", "alpha2", "beta"] and b["vision_feature_file"] == "image_feat_raw.npy"
    assert b["reg_weight"] == [1e-2, 1e-3, 1e-4, 1e-5]


def test_early_stopping_semantics():
    assert early_stopping(0.5, 0.4, 3, 20) == (0.5, 0, False, True)
    assert early_stopping(0.3, 0.4, 20, 20) == (0.4, 21, True, False)
    assert early_stopping(0.3, 0.4, 2, 20, bigger=False) == (0.3, 0, False, True)


def _loaders(data_root, model="LightGCN"):
    cfg = Config(model, "baby", {"data_path": data_root, "use_gpu": False, "train_batch_size": 512,
                                  "eval_batch_size": 256, "rsx_sampler": "host", "is_multimodal_model": False})
    ds = RecDataset(cfg)
    tr, va, te = ds.split()
    for x in (ds, tr, va, te):
        str(x)
    train = TrainDataLoader(cfg, tr, batch_size=512, shuffle=True)
    valid = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=256)
    test = EvalDataLoader(cfg, te, additional_dataset=tr, batch_size=256)
    return cfg, ds, train, valid, test


def test_dataset_and_loaders_match_fixture(golden, data_root):
    z = golden("lightgcn_small")
    cfg, ds, train, valid, test = _loaders(data_root)
    assert ds.get_user_num() == int(z["n_users"]) and ds.get_item_num() == int(z["n_items"])
    coo = train.inter_matrix(form="coo")
    assert np.array_equal(coo.row, z["train_u"]) and np.array_equal(coo.col, z["train_i"])
    assert np.array_equal(valid.get_eval_users().numpy(), z["valid_eval_u"])
    assert np.array_equal(np.asarray(valid.get_eval_len_list()), z["valid_eval_len"])
    assert np.array_equal(np.concatenate(valid.get_eval_items()), z["valid_eval_items"])
    # eval batches: users + rebased mask, as the reference
    b = next(iter(valid))
    assert b[0].shape[0] == 256 and b[1][0].max().item() < 256


def test_host_sampler_reproduces_reference_triplets(golden, data_root):
    """Same seeds -> the reference's exact (user, pos, neg) stream (dataloader.py:226-275)."""
    z = golden("lightgcn_small")
    cfg, ds, train, valid, test = _loaders(data_root)
    init_seed(999)
    train.pretrain_setup()
    # the reference builds the model here: xavier_uniform_ draws from the torch CPU RNG only
    torch.nn.init.xavier_uniform_(torch.empty(int(z["n_users"]), 64))
    for epoch in range(3):
        got = torch.cat(list(train), dim=1).numpy()
        assert np.array_equal(got, z[f"epoch{epoch}_triplets"].astype(np.int64)), epoch


@pytest.mark.parametrize("fx", ["lightgcn_small", "layergcn_small", "layergcn_drop_small", "smore_small"])
def test_evaluator_matches_reference_metrics(golden, fx):
    z = golden(fx)
    cfg = Config("LightGCN", "baby", {"use_gpu": False})
    ev = TopKEvaluator(cfg)
    tags = [k[: -len("_metric_keys")] for k in z if k.endswith("_metric_keys")]
    assert tags
    for tag in tags:
        split = "test" if tag.endswith("test") else "valid"
        items = eval_lists(z, split)
        out = ev.evaluate_arrays(z[tag + "_topk_idx"].astype(np.int64), items, z[split + "_eval_len"])
        assert out == metric_dict(z, tag), tag


def test_device_metric_dict_falls_back_to_user_order_sums(monkeypatch):
    """device_metric_dict rounds the parallel-order sums and re-runs the user-ordered
    ones only when a mean lies within sum_order_bound of a 4-decimal rounding step."""
    import torch

    from rsx import evaluator as E
    from rsx import ops

    n = 1000
    calls = []

    def fake(topk, erp, ecol, cuts, gain, exact=True):
        calls.append(exact)
        s = np.zeros((5, len(cuts)))
        s[0, 0] = state["fast"] if not exact else state["exact"]
        return torch.from_numpy(s)

    monkeypatch.setattr(ops, "topk_metrics", fake)
    topk = torch.zeros(n, 5, dtype=torch.int64)
    # far from a rounding step: one pass
    state = {"fast": 0.123456 * n, "exact": 0.0}
    assert E.device_metric_dict(topk, None, None, ["recall"], [5], 10)["recall@5"] == 0.1235
    assert calls == [False]
    # mean 0.12345 (+1e-15): both sides of the step are within the bound -> user-order sums decide
    calls.clear()
    state = {"fast": 0.12345 * n + 1e-12, "exact": 0.12345 * n - 1e-12}
    got = E.device_metric_dict(topk, None, None, ["recall"], [5], 10)["recall@5"]
    assert calls == [False, True]
    assert got == float(round(np.float64(state["exact"] / n), 4))
    assert E.sum_order_bound(n, 1.0) < 1e-12


def test_latency_injection_needs_the_second_switch(monkeypatch):
    """RSX_COMM_SIM alone (left over in a shell) must not turn a real run into
    the benchmark's modelled job (stand-in peer triplets in every step)."""
    import warnings

    from rsx.dist import sim_comm_params

    monkeypatch.setenv("RSX_COMM_SIM", "4")
    monkeypatch.delenv("RSX_COMM_SIM_OPT_IN", raising=False)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert sim_comm_params() is None
    assert any("ignored" in str(x.message) for x in w)
    monkeypatch.setenv("RSX_COMM_SIM_OPT_IN", "1")
    assert sim_comm_params()["world"] == 4
