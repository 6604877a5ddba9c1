"""Kernel microbenchmarks on the sports-shaped graph (one process; interleaved reps).
Usage: python tools/gpu/micro.py [spmm|fullsort|all]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "recommendar-systems_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsx import graph, ops, synth  # noqa: E402


def t_ms(fn, reps=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main(what):
    dev = torch.device("cuda:0")
    nu, ni, ne = synth.SHAPES["sports"]
    df = synth.amazon_like(nu, ni, ne, seed=0)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    rp, col, val = graph.lightgcn_norm_adj(tu, ti, nu, ni)
    n = nu + ni
    out = {}
    if what in ("spmm", "all"):
        for chunk in (16, 32, 64):
            A = ops.DeviceCSR(rp, col, val, n, dev, chunk)
            x = torch.randn(n, 64, device=dev)
            y = torch.empty_like(x)
            out[f"spmm_store_chunk{chunk}_ms"] = t_ms(lambda: A.spmm(x, out=y))
            out[f"chunk{chunk}_nlong"] = A.n_long
    if what == "spmmx":
        # what bounds the SpMM: same schedule with (a) every gather on row 0 (all hits),
        # (b) neighbours = the next rows in order (streaming), (c) no nonzeros at all
        x = torch.randn(n, 64, device=dev)
        y = torch.empty_like(x)
        deg = np.diff(rp)
        variants = {
            "real": (rp, col),
            "same_row": (rp, np.zeros_like(col)),
            "sequential": (rp, ((np.repeat(np.arange(n), deg) + np.arange(col.size) % 8) % n).astype(np.int32)),
            "empty": (np.zeros_like(rp), col[:0]),
        }
        for name, (r, c) in variants.items():
            A = ops.DeviceCSR(r, c, val[: c.size].astype(np.float32), n, dev, 32)
            out[f"spmmx_{name}_us"] = round(t_ms(lambda: A.spmm(x, out=y), 100) * 1e3, 2)
        # the same real graph with d = 32 / 128 (bytes scale with d)
        for d in (32, 128):
            A = ops.DeviceCSR(rp, col, val, n, dev, 32)
            xd = torch.randn(n, d, device=dev)
            yd = torch.empty_like(xd)
            out[f"spmmx_real_d{d}_us"] = round(t_ms(lambda: A.spmm(xd, out=yd), 100) * 1e3, 2)
    if what == "floor":
        # what one SpMM layer costs beyond the work: launch, a plain 13.8 MB write, the
        # epilogues alone (rowwise), empty-graph and real launches per epilogue kind
        from rsx import _lib as L
        x = torch.randn(n, 64, device=dev)
        y = torch.empty_like(x)
        tabs = {k: torch.randn(n, 64, device=dev).abs() * 0.01 for k in ("p", "m", "v", "g", "r")}
        tiny = torch.empty(1, device=dev)
        out["launch_only_us"] = round(t_ms(lambda: tiny.zero_(), 200) * 1e3, 2)
        out["write_13.8MB_us"] = round(t_ms(lambda: y.zero_(), 200) * 1e3, 2)
        out["copy_13.8MB_us"] = round(t_ms(lambda: y.copy_(x), 200) * 1e3, 2)
        A = ops.DeviceCSR(rp, col, val, n, dev, 32)
        E = ops.DeviceCSR(np.zeros_like(rp), col[:0], val[:0], n, dev, 32)
        adam = ops.adam_struct(1e-3, 5)
        kinds = {
            "store": lambda: ops.epi(L.RSX_EPI_STORE, y=y),
            "add_sparse": lambda: ops.epi(L.RSX_EPI_ADD, y=y, s_in=tabs["g"]),
            "adam": lambda: ops.epi(L.RSX_EPI_ADAM, adam=adam, s_in=tabs["g"], r_add=tabs["r"], p=tabs["p"],
                                    m=tabs["m"], v=tabs["v"]),
        }
        for name, mk in kinds.items():
            e = mk()
            out[f"{name}_rowwise_us"] = round(t_ms(lambda: ops.rowwise(n, 64, e), 100) * 1e3, 2)
            out[f"{name}_empty_us"] = round(t_ms(lambda: E.spmm_epi(x, e, 64), 100) * 1e3, 2)
            out[f"{name}_real_us"] = round(t_ms(lambda: A.spmm_epi(x, e, 64), 100) * 1e3, 2)
    if what == "metrics":
        g = np.random.default_rng(1)
        nu_e, k = 35598, 50
        lens = g.integers(1, 6, nu_e)
        rp_e = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
        col_e = torch.from_numpy(np.sort(g.integers(0, ni, int(lens.sum()))).astype(np.int32)).to(dev)
        topk = torch.from_numpy(g.integers(0, ni, (nu_e, k))).to(dev)
        gain = torch.from_numpy(1.0 / np.log2(np.arange(1, k + 1, dtype=np.float64) + 1)).to(dev)
        out["metrics_ms"] = t_ms(lambda: ops.topk_metrics(topk, rp_e, col_e, [5, 10, 20, 50], gain), 20)
    if what in ("fullsort", "all"):
        f = torch.randn(n, 64, device=dev) * 0.1
        U, I = f[:nu], f[nu:]
        hr, hc = graph.history_csr(tu, ti, nu)
        hr, hc = torch.from_numpy(hr).to(dev), torch.from_numpy(hc).to(dev)
        users = torch.arange(int(os.environ.get("RSX_FS_NUSERS", nu)), device=dev)
        if os.environ.get("RSX_FS_MODE") == "4":  # per-segment s_memtime sums (fs_tiles<D, 4>)
            import ctypes as C  # noqa: F401
            from rsx import _lib as L
            v = torch.empty(users.numel(), 50, device=dev)
            idx = torch.zeros(users.numel(), 50, dtype=torch.int64, device=dev)
            lib = L.lib()
            ws = ops._ws(dev, lib.rsx_fullsort_ws_bytes(users.numel(), ni, 50))
            L.check(lib.rsx_fullsort_topk(ops._p(U), ops._p(users), users.numel(), ops._p(I), ni, 64, ops._p(hr),
                                          ops._p(hc), 50, ops._p(v), ops._p(idx), ops._p(ws), ws.numel(),
                                          ops._stream()), "fs")
            torch.cuda.synchronize()
            c = [int(x) for x in idx.view(-1)[:6].cpu()]
            tot = sum(c[:5])
            for name, x in zip(("mfma_issue", "insert", "filter_total", "compact", "mask_copy"), c[:5]):
                out["seg_" + name] = round(x / tot, 3)
            out["cycles_per_tile"] = round(tot / max(c[5], 1))
            print(out, flush=True)
            return
        out["fs_ms_all_users"] = t_ms(lambda: ops.fullsort_topk(U, users, I, hr, hc, 50), 10)
        out["fs_users"] = users.numel()
        out["fs_tflops"] = 2 * 64 * ni * users.numel() / (out["fs_ms_all_users"] * 1e-3) / 1e12
    print(out, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "all")
