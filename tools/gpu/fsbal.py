"""Full-sort timing vs the number of 32-user waves (sports item count, d = 64; env FS_NI,
FS_D for other shapes).

Random tables and a random train mask; prints ms per call and TF/s for each user
count, to show how the kernel's time follows waves per SIMD.
usage: python tools/gpu/fsbal.py [nb ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import ops  # noqa: E402


def main():
    ni, d, k = int(os.environ.get("FS_NI", 18357)), int(os.environ.get("FS_D", 64)), 50
    nbs = [int(x) for x in sys.argv[1:]] or [32768, 35598, 40960, 49152]
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda:0")
    gd = torch.Generator(device=dev).manual_seed(0)
    items = torch.randn(ni, d, generator=gd, device=dev) * 0.1
    for nb in nbs:
        users = torch.randn(nb, d, generator=gd, device=dev) * 0.1
        per = 8
        col = torch.randint(0, ni, (nb, per), generator=g).sort(1).values
        rp = torch.arange(0, nb * per + 1, per, dtype=torch.int64)
        rp_d, col_d = rp.to(dev), col.flatten().to(torch.int32).to(dev)
        fn = lambda: ops.fullsort_topk(users, None, items, rp_d, col_d, k)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        print(f"nb={nb} waves={(nb + 31) // 32} ms={ms:.3f} tflops={2 * nb * ni * d / ms / 1e9:.1f}", flush=True)


if __name__ == "__main__":
    main()
