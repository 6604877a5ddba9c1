"""Which rsx.smore_dist.Comm pattern under a latency-injected communicator breaks a HIP
graph capture (the C5 sim leg segfaulted in capture_end)?  One pattern per process:
python tools/gpu/diag_smore_sim.py PATTERN  (RSX_COMM_SIM=4 in the env)
  ar      allreduce_ on the capturing stream
  side    allreduce_start_ + wait on a side stream joined to the capture
  ag      allgather_ on the capturing stream
  grad    allreduce_grad's backward (autograd) inside the capture
  all     all of the above in one capture"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx.smore_dist import Comm, allreduce_grad  # noqa: E402


def main(pat):
    dev = torch.device("cuda:0")
    comm = Comm(None, dev)
    assert comm.sim is not None and comm.world == 4
    a = torch.ones(1 << 16, device=dev)
    b = torch.ones(4 * 1024, device=dev)
    w = torch.ones(256, device=dev, requires_grad=True)
    side = torch.cuda.Stream(device=dev)

    def body():
        if pat in ("ar", "all"):
            comm.allreduce_(a)
        if pat in ("side", "all"):
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                comm.allreduce_start_(a)
                a.add_(1.0)
                comm.wait()
            main.wait_stream(side)
        if pat in ("ag", "all"):
            comm.allgather_(b, 1024)
        if pat in ("grad", "all"):
            (y,) = allreduce_grad(comm, w)
            (y * 2).sum().backward()

    body()  # eager first
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"pattern {pat}: capture + replay ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
