"""Projection GEMMs at the C5 shape: rsx_linear_bwd / smore_proj against torch.mm (the
library f32 GEMM), to size what a better kernel could give.  python tools/gpu/micro_gemm.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "recommendar-systems_amd"))
import torch  # noqa: E402

from rsx import ops  # noqa: E402


def t_ms(fn, reps=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    n, k, d = 23033, 768, 128
    x = torch.randn(n, k, device=dev)
    W = torch.randn(d, k, device=dev) / k ** 0.5
    g = torch.randn(n, d, device=dev)
    out = {}
    out["torch_fwd_xWt_ms"] = t_ms(lambda: torch.mm(x, W.t()))
    out["torch_dx_gW_ms"] = t_ms(lambda: torch.mm(g, W))
    out["torch_dW_gtx_ms"] = t_ms(lambda: torch.mm(g.t(), x))
    out["rsx_linear_bwd_ms"] = t_ms(lambda: ops.linear_bwd(g, x, W, bias=True))
    gf = 2 * n * k * d / 1e9
    for key in list(out):
        flops = gf * (2 if key.startswith("rsx_linear_bwd") else 1)
        out[key.replace("_ms", "_tflops")] = flops / out[key]  # GFLOP / ms = TFLOP/s
    print(json.dumps(out))


if __name__ == "__main__":
    main()
