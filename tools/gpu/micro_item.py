"""The SMORE item side forward timed alone: the one-launch rsx_smore_item_fwd against the
three-launch chain (rsx_smore_spectral_fwd = smore_proj + smore_spec_fwd, then
rsx_smore_gates forward) at the C5 clothing shape (23,033 items, 768/768 features, d = 128)
and the C3 baby shape (7,050 items, 4096/384, d = 64).  Prints one line per shape and
path, and whether the outputs agree bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import _lib as L  # noqa: E402
from rsx import ops  # noqa: E402
from rsx.smore_fuse import _arr  # noqa: E402


def run(n, dv, dt, d, iters=50):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, device=dev) * 0.1  # noqa: E731
    V, T = r(n, dv), r(n, dt)
    Wv, Wt, bv, bt = r(d, dv), r(d, dt), r(d), r(d)
    unit = r(3, d // 2 + 1, 2)
    item = r(n, d)
    gW, gb = [r(d, d) for _ in range(3)], [r(d) for _ in range(3)]
    lib = L.lib()
    p = ops._p
    bufs = {k: [torch.empty(n, d, device=dev) for _ in range(8)] for k in ("chain", "fused")}
    spec = torch.empty(int(lib.rsx_smore_spectral_spec_floats(n, d)), device=dev)
    ws = torch.empty(max(int(lib.rsx_smore_spectral_fwd_ws_bytes(n, d, dv, dt)), 4), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(int(lib.rsx_smore_item_tiles(n)), dtype=torch.int32, device=dev)

    def chain():
        img, txt, cv, ct, cf, o0, o1, o2 = bufs["chain"]
        L.check(lib.rsx_smore_spectral_fwd(p(V), dv, p(Wv), p(bv), p(T), dt, p(Wt), p(bt), p(unit[0]), p(unit[1]),
                                           p(unit[2]), n, d, p(img), p(txt), p(cv), p(ct), p(cf), p(spec), p(ws),
                                           ws.numel(), ops._stream()), "spectral_fwd")
        L.check(lib.rsx_smore_gates(0, _arr([cv, ct, cf]), p(item), _arr(gW), _arr(gb), n, d, 0.7, 0,
                                    _arr([o0, o1, o2]), None, None, None, None, ops._stream()), "gates")

    def fused():
        img, txt, cv, ct, cf, o0, o1, o2 = bufs["fused"]
        L.check(lib.rsx_smore_item_fwd(p(V), dv, p(Wv), p(bv), p(T), dt, p(Wt), p(bt), p(unit[0]), p(unit[1]),
                                       p(unit[2]), n, d, p(img), p(txt), p(cv), p(ct), p(cf), p(spec), p(ws),
                                       ws.numel(), p(cnt), p(item), _arr(gW), _arr(gb), 0.7, 0, _arr([o0, o1, o2]),
                                       ops._stream()), "item_fwd")

    img, txt, cv, ct, cf, o0, o1, o2 = bufs["chain"]
    gx = [torch.empty(n, d, device=dev) for _ in range(2)]
    part = torch.empty(int(lib.rsx_smore_spectral_bwd_partials(n, d)), device=dev)
    wsb = torch.empty(int(lib.rsx_smore_spectral_bwd_ws_bytes(n, d)), dtype=torch.uint8, device=dev)
    gconv = [r(n, d) for _ in range(3)]

    def spectral_fwd():
        L.check(lib.rsx_smore_spectral_fwd(p(V), dv, p(Wv), p(bv), p(T), dt, p(Wt), p(bt), p(unit[0]), p(unit[1]),
                                           p(unit[2]), n, d, p(img), p(txt), p(cv), p(ct), p(cf), p(spec), p(ws),
                                           ws.numel(), ops._stream()), "spectral_fwd")

    def gates():
        L.check(lib.rsx_smore_gates(0, _arr([cv, ct, cf]), p(item), _arr(gW), _arr(gb), n, d, 0.7, 0,
                                    _arr([o0, o1, o2]), None, None, None, None, ops._stream()), "gates")

    def spectral_bwd():
        L.check(lib.rsx_smore_spectral_bwd(p(spec), p(unit[0]), p(unit[1]), p(unit[2]), p(gconv[0]), p(gconv[1]),
                                           p(gconv[2]), n, d, p(gx[0]), p(gx[1]), p(part), p(wsb), wsb.numel(),
                                           ops._stream()), "spectral_bwd")

    res = {}
    for name, fn in (("chain", chain), ("fused", fused), ("chain", chain), ("fused", fused),
                     ("spectral_fwd", spectral_fwd), ("gates", gates), ("spectral_bwd", spectral_bwd)):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / iters * 1e3
    chain()
    fused()
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(bufs["chain"], bufs["fused"]))
    print(f"item side n={n} dv={dv} dt={dt} d={d}: chain {res['chain']:.1f} us (spectral_fwd "
          f"{res['spectral_fwd']:.1f} + gates {res['gates']:.1f}), one launch {res['fused']:.1f} us, "
          f"bit-identical {same}; spectral_bwd {res['spectral_bwd']:.1f} us", flush=True)


if __name__ == "__main__":
    run(23033, 768, 768, 128)
    run(7050, 4096, 384, 64)
