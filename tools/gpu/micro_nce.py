"""The InfoNCE pair's backward (rsx_smore_infonce_bwd_scaled: nce_bwd_t<128, NG>) at the C5
batch (B = 2048, d = 128) timed alone, and a digest of its gradients: run it once per
RSX_NCE_GROUPS value (the knob is read once per process) and compare the digests (the two
forms sum the same products in the same order, so the digests must match).
Usage: RSX_NCE_GROUPS=1|2 python tools/gpu/micro_nce.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import _lib as L  # noqa: E402
from rsx import ops  # noqa: E402


def main():
    B, d, nu, ni = 2048, 128, 39387, 23033
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    side = torch.randn(nu + ni, d, generator=g, device=dev)
    content = torch.randn(nu + ni, d, generator=g, device=dev)
    users = torch.randint(0, nu, (B,), generator=g, device=dev)
    pos = torch.randint(0, ni, (B,), generator=g, device=dev)
    lib = L.lib()
    p = ops._p
    ws = torch.empty(int(lib.rsx_smore_infonce_ws_bytes(B, d)), dtype=torch.uint8, device=dev)
    loss = torch.empty(2, device=dev)
    L.check(lib.rsx_smore_infonce_fwd(p(side), p(content), p(users), p(pos), nu, B, d, 0.2, p(loss), p(ws),
                                      ws.numel(), ops._stream()), "fwd")
    gl = torch.ones(2, device=dev)
    gs, gc = torch.zeros_like(side), torch.zeros_like(content)

    def bwd():
        gs.zero_()
        gc.zero_()
        L.check(lib.rsx_smore_infonce_bwd(p(side), p(content), p(users), p(pos), nu, B, d, 0.2, p(gl), p(gs), p(gc),
                                          p(ws), ws.numel(), ops._stream()), "bwd")

    bwd()
    torch.cuda.synchronize()
    # rows hit by several batch entries take float atomics: digest the rows hit once
    once = torch.zeros(nu + ni, dtype=torch.int32, device=dev)
    once.index_add_(0, users, torch.ones_like(users, dtype=torch.int32))
    once.index_add_(0, nu + pos, torch.ones_like(pos, dtype=torch.int32))
    keep = (once == 1).nonzero().squeeze(1)
    digest = hashlib.sha1(torch.cat([gs[keep], gc[keep]]).cpu().numpy().tobytes()).hexdigest()[:16]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fill = torch.cuda.Event(enable_timing=True)
    reps = 50
    s.record()
    for _ in range(reps):
        bwd()
    e.record()
    fill.record()
    for _ in range(reps):
        gs.zero_()
        gc.zero_()
    fe = torch.cuda.Event(enable_timing=True)
    fe.record()
    torch.cuda.synchronize()
    t = (s.elapsed_time(e) - fill.elapsed_time(fe)) / reps * 1e3
    print(f"infonce bwd B={B} d={d} groups={os.environ.get('RSX_NCE_GROUPS', '2')}: {t:.1f} us "
          f"(zero fills subtracted), digest {digest}", flush=True)


if __name__ == "__main__":
    main()
