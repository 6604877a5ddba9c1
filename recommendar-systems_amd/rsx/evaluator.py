"""Top-K ranking metrics with the reference's definitions and rounding.

Same results as TopKEvaluator.evaluate + utils/metrics.py
(src/utils/topk_evaluator.py:58-102, src/utils/metrics.py:12-118): Recall,
Recall2, NDCG, Precision, MAP at every k of `topk`, each the mean over eval
users of the per-user cumulative value at rank k, rounded to 4 decimals.  The
reference builds the hit matrix with a Python `i in m` loop per (user, rank)
(its largest evaluation cost); here it is one vectorised membership
test on (row, item) keys, producing the identical boolean matrix, after which
the same float64 cumulative arithmetic runs.
"""
from __future__ import annotations

import numpy as np

_KNOWN = ("recall", "recall2", "precision", "ndcg", "map")


def hit_matrix(topk_idx: np.ndarray, eval_items: list) -> np.ndarray:
    n, k = topk_idx.shape
    lens = np.fromiter((len(x) for x in eval_items), dtype=np.int64, count=n)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    items = np.concatenate([np.asarray(x, dtype=np.int64) for x in eval_items]) if n else np.zeros(0, np.int64)
    span = int(max(int(topk_idx.max(initial=0)), int(items.max(initial=0)))) + 1
    truth = np.unique(rows * span + items)
    keys = np.arange(n, dtype=np.int64)[:, None] * span + topk_idx.astype(np.int64)
    return np.isin(keys, truth)


def _ranks(k):
    return np.arange(1, k + 1)


def recall(hit, pos_len):
    return (np.cumsum(hit, axis=1) / pos_len.reshape(-1, 1)).mean(axis=0)


def recall2(hit, pos_len):
    return np.cumsum(hit, axis=1).sum(axis=0) / pos_len.sum()


def precision(hit, pos_len):
    return (hit.cumsum(axis=1) / _ranks(hit.shape[1])).mean(axis=0)


def ndcg(hit, pos_len):
    k = hit.shape[1]
    rank = np.zeros_like(hit, dtype=np.float64)
    rank[:, :] = _ranks(k)
    gain = 1.0 / np.log2(rank + 1)
    ideal_full = np.cumsum(gain, axis=1)
    cap = np.minimum(pos_len, k)                       # IDCG over min(|pos|, k) relevant items
    col = np.minimum(np.arange(k)[None, :], (cap - 1)[:, None])
    idcg = np.take_along_axis(ideal_full, col, axis=1)
    dcg = np.cumsum(np.where(hit, gain, 0), axis=1)
    return (dcg / idcg).mean(axis=0)


def average_precision(hit, pos_len):
    k = hit.shape[1]
    prec = hit.cumsum(axis=1) / _ranks(k)
    acc = np.cumsum(prec * hit.astype(np.float64), axis=1)
    cap = np.minimum(pos_len, k)
    denom = np.minimum(_ranks(k)[None, :], cap[:, None])
    out = np.zeros_like(hit, dtype=np.float64)
    out[:, :] = acc / denom
    return out.mean(axis=0)


FUNCS = {"recall": recall, "recall2": recall2, "precision": precision, "ndcg": ndcg, "map": average_precision}


class TopKEvaluator:
    """Evaluator with the reference's config keys: metrics, topk."""

    def __init__(self, config):
        self.config = config
        metrics = config["metrics"]
        if isinstance(metrics, str):
            metrics = [metrics]
        if not isinstance(metrics, (list, tuple)):
            raise TypeError("metrics must be str or list")
        for m in metrics:
            if m.lower() not in _KNOWN:
                raise ValueError(f"There is no user grouped topk metric named {m}!")
        self.metrics = [m.lower() for m in metrics]
        topk = config["topk"]
        if isinstance(topk, int):
            topk = [topk]
        if not isinstance(topk, (list, tuple)):
            raise TypeError("The topk must be a integer, list")
        for k in topk:
            if k <= 0:
                raise ValueError(f"topk must be a positive integer or a list of positive integers, but get `{k}`")
        self.topk = list(topk)

    def evaluate_arrays(self, topk_idx: np.ndarray, eval_items: list, pos_len: np.ndarray) -> dict:
        assert len(pos_len) == len(topk_idx)
        hit = hit_matrix(topk_idx, eval_items)
        out = {}
        for m in self.metrics:
            v = FUNCS[m](hit, np.asarray(pos_len))
            for k in self.topk:
                out[f"{m}@{k}"] = round(v[k - 1], 4)
        return out

    def evaluate(self, batch_matrix_list, eval_data, is_test=False, idx=0):
        import torch

        topk = torch.cat(batch_matrix_list, dim=0)
        if topk.is_cuda and hasattr(eval_data, "eval_csr"):
            return self.evaluate_device(topk, eval_data)
        return self.evaluate_arrays(topk.cpu().numpy(), eval_data.get_eval_items(), eval_data.get_eval_len_list())

    def evaluate_sharded(self, pos, topk, eval_data) -> dict:
        """A user-sharded evaluation's dict (sharded_metric_dict: sums all-gathered)."""
        return sharded_metric_dict(pos, topk, eval_data, self.metrics, self.topk)

    def evaluate_device(self, topk, eval_data) -> dict:
        """The same dict from device-resident top-k lists (device_metric_dict)."""
        erp, ecol = eval_data.eval_csr()
        pos_total = int(np.asarray(eval_data.get_eval_len_list()).sum())
        return device_metric_dict(topk, erp, ecol, self.metrics, self.topk, pos_total)


_U = 2.0 ** -53


def sum_order_bound(n: int, total: float) -> float:
    """Bound on |parallel-order sum - user-order sum| of n values >= 0 summing to
    about `total` (rsx_topk_metrics_fast, include/rsx.h): (gamma_h + gamma_{n-1}) *
    sum, h the parallel tree's depth, gamma_j = j u / (1 - j u)."""
    nblk = min(1024, max(1, -(-n // 256)))
    h = -(-n // (256 * nblk)) + 16 + -(-nblk // 64)
    j = (n - 1) + h
    return j * _U / (1.0 - j * _U) * np.abs(total) * 1.0001


def device_metric_dict(topk, erp, ecol, metrics, topk_list, pos_total: int) -> dict:
    """The reference's metric dict from device-resident top-k lists: hits by binary
    search in each user's sorted held-out items, per-user float64 values and their
    column sums on the device (rsx_topk_metrics_fast: a fixed parallel order), then
    the reference's division and round(., 4) here.  Every mean whose rounding could
    differ between that order and numpy's user order (mean(axis=0)) -- one within
    sum_order_bound of a 4-decimal rounding step, for any realistic n a 1e-9-level
    event -- sends the dict through the user-ordered sums (rsx_topk_metrics), so the
    dict always equals the one from the sequential sums.  One [5, n_cut] float64
    copy to the host per pass."""
    import torch

    from . import ops

    k = topk.shape[1]
    cuts = sorted(set(int(c) for c in topk_list))
    if cuts[-1] > k:
        raise ValueError(f"topk {cuts[-1]} > ranked list length {k}")
    gain = _gain(k, topk.device)
    n = topk.shape[0]
    col = {c: j for j, c in enumerate(cuts)}
    rows = {"recall": 0, "precision": 1, "ndcg": 2, "map": 3, "recall2": 4}
    keys = [(m, kk) for m in metrics for kk in topk_list]
    ri = np.array([rows[m] for m, _ in keys], dtype=np.int64)
    ci = np.array([col[int(kk)] for _, kk in keys], dtype=np.int64)
    den = np.array([pos_total if m == "recall2" else n for m, _ in keys], dtype=np.float64)
    for exact in (False, True):
        sums = ops.topk_metrics(topk, erp, ecol, cuts, gain, exact=exact).cpu().numpy()
        s = sums[ri, ci]
        v = s / den
        # numpy's round on the float64s, as the reference's round(value[k - 1], 4)
        # (scale, round half to even): 0.05875 -> 0.0588, where float rounding gives 0.0587
        r = np.round(v, 4)
        if not exact:
            # the division rounds once more: relative u on either side
            b = sum_order_bound(n, s) / den + 4 * _U * np.abs(v)
            if not np.array_equal(np.round(v - b, 4), np.round(v + b, 4)):
                continue  # a mean within the order bound of a rounding step: user-order sums
        return {f"{m}@{kk}": float(x) for (m, kk), x in zip(keys, r)}
    raise AssertionError("unreachable")


_GAIN = {}


def _gain(k: int, device):
    """1/log2(r+1), r = 1..k, as metrics.py's ndcg computes it (cached per device)."""
    import torch

    key = (k, str(device))
    g = _GAIN.get(key)
    if g is None:
        ranks = np.arange(1, k + 1, dtype=np.float64)
        g = _GAIN[key] = torch.from_numpy(1.0 / np.log2(ranks + 1)).to(device)
    return g


def _collect(t):
    """all_gather of a small float64 tensor; returns the per-rank tensors on the host, in rank order."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):  # one rank (rsx_sharded without a group)
        return [t.cpu()]
    x = t if dist.get_backend() == "nccl" else t.cpu()
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, x)
    return [q.cpu() for q in parts]


def sharded_metric_dict(pos, topk, eval_data, metrics, topk_list) -> dict:
    """The metric dict of a user-sharded evaluation: this rank ranked the evaluation
    users at positions `pos` of eval_data's user list (top-k rows `topk`).  Each rank
    sums its users' per-user values in user order (rsx_topk_metrics), the [5, n_cut]
    sums are all-gathered and added in rank order, then divided by the global user
    count (and |held-out items| for recall2) and rounded as the reference does."""
    import torch

    from . import ops

    erp, ecol = eval_data.eval_csr()
    cache = getattr(eval_data, "_shard_csr", None)
    if cache is None or cache[0] is not pos and not torch.equal(cache[0], pos):
        lens = (erp[1:] - erp[:-1]).index_select(0, pos)
        rp = torch.zeros(pos.numel() + 1, dtype=torch.int64, device=erp.device)
        rp[1:] = torch.cumsum(lens, 0)
        starts = erp[:-1].index_select(0, pos)
        seg = torch.repeat_interleave(torch.arange(pos.numel(), device=erp.device), lens)
        idx = starts.index_select(0, seg) + (torch.arange(int(rp[-1].item()), device=erp.device) - rp[:-1].index_select(0, seg))
        cache = eval_data._shard_csr = (pos, rp, ecol.index_select(0, idx).contiguous())
    _, rp, col = cache
    k = topk.shape[1]
    cuts = sorted(set(int(c) for c in topk_list))
    sums = ops.topk_metrics(topk.contiguous(), rp, col, cuts, _gain(k, topk.device), exact=True)
    tot = None
    for part in _collect(sums):
        tot = part.clone() if tot is None else tot + part
    s = tot.numpy()
    n = int(eval_data.eval_u.numel())
    pos_total = int(np.asarray(eval_data.get_eval_len_list()).sum())
    rows = {"recall": 0, "precision": 1, "ndcg": 2, "map": 3, "recall2": 4}
    col_of = {c: j for j, c in enumerate(cuts)}
    out = {}
    for m in metrics:
        for kk in topk_list:
            den = pos_total if m == "recall2" else n
            out[f"{m}@{kk}"] = float(np.round(s[rows[m], col_of[int(kk)]] / den, 4))
    return out
