"""LayerGCNEngine.step timing, the one-call C step vs the Python-issued sequence
(RSX_LAYERGCN_CSTEP), on the baby-shaped graph with fixed device triplets."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import synth  # noqa: E402
from rsx.layergcn import LayerGCNEngine  # noqa: E402


def main():
    df = synth.shaped("baby", seed=0)
    tr = df[df.x_label == 0]
    tu, ti = tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64)
    nu, ni = int(df.userID.max()) + 1, int(df.itemID.max()) + 1
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    U0 = rng.standard_normal((nu, 64)).astype(np.float32) * 0.1
    I0 = rng.standard_normal((ni, 64)).astype(np.float32) * 0.1
    eng = LayerGCNEngine(tu, ti, nu, ni, 64, 2, 1e-3, 1e-3, dev, U0, I0)
    sel = rng.integers(0, tu.size, size=2048)
    trip = torch.from_numpy(np.stack([tu[sel], ti[sel] + 0, rng.integers(0, ni, size=2048)])).to(dev)
    for mode in ("1", "0", "1", "0"):
        os.environ["RSX_LAYERGCN_CSTEP"] = mode
        for _ in range(20):
            eng.step(trip)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 300
        t0 = time.perf_counter()
        s.record()
        for _ in range(n):
            eng.step(trip)
        t1 = time.perf_counter()
        e.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"CSTEP={mode}: host issue {(t1 - t0) / n * 1e3:.4f} ms, wall {(t2 - t0) / n * 1e3:.4f} ms, "
              f"events {s.elapsed_time(e) / n:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
