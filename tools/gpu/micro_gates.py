"""gates forward/backward at the C5 clothing item shape (n = 23033, d = 128), timed alone
(tools/gpu/micro_gates.sh adds the SQ counters)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import _lib as L  # noqa: E402
from rsx import ops  # noqa: E402
from rsx.smore_fuse import _arr  # noqa: E402


def main():
    n, d = int(os.environ.get("G_N", 23033)), int(os.environ.get("G_D", 128))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, device=dev) * 0.1  # noqa: E731
    conv = [r(n, d) for _ in range(3)]
    item = r(n, d)
    W = [r(d, d) for _ in range(3)]
    b = [r(d) for _ in range(3)]
    gout = [r(n, d) for _ in range(3)]
    gi = torch.empty_like(item)
    gc = [torch.empty_like(item) for _ in range(3)]
    dz = [torch.empty_like(item) for _ in range(3)]
    outs = [torch.empty_like(item) for _ in range(3)]
    lib = L.lib()

    def fwd():
        L.check(lib.rsx_smore_gates(0, _arr(conv), item.data_ptr(), _arr(W), _arr(b), n, d, 0.7, 0, _arr(outs), None,
                                    None, None, None, ops._stream()), "gates fwd")

    def bwd():
        L.check(lib.rsx_smore_gates(1, _arr(conv), item.data_ptr(), _arr(W), _arr(b), n, d, 0.7, 0, None, _arr(gout),
                                    gi.data_ptr(), _arr(gc), _arr(dz), ops._stream()), "gates bwd")

    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"gates {name} n={n} d={d}: {s.elapsed_time(e) / 20 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
