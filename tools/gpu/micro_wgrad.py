"""Per-shape timing of the split-K weight gradient (rsx_linear_wgrad) against the
library GEMM g.t() @ x, for the SMORE shapes (C3 d=64, C5 d=128)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "recommendar-systems_amd"))
import torch  # noqa: E402

from rsx import ops  # noqa: E402


def t_us(fn, reps=20, rounds=5):
    """Device time per call: `reps` calls captured in a HIP graph (no host launch
    overhead), replayed `rounds` times."""
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(rounds):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (reps * rounds)


dev = torch.device("cuda:0")
for n, o, i in [(26495, 64, 64), (7050, 64, 64), (7050, 64, 4096), (7050, 64, 384), (62420, 128, 128),
                (23033, 128, 128), (23033, 128, 768)]:
    g = torch.randn(n, o, device=dev)
    x = torch.randn(n, i, device=dev)
    a = t_us(lambda: ops.linear_wgrad(g, x))
    b = t_us(lambda: g.t() @ x)
    fl = 2.0 * n * o * i
    by = 4.0 * n * (o + i)
    print(f"n={n:6d} {o:4d}x{i:<5d} rsx {a:7.1f} us ({fl / a / 1e6:6.1f} TF/s, {by / a / 1e3:6.0f} GB/s)  "
          f"torch {b:7.1f} us", flush=True)
