"""Pass-2 candidate totals of the screened full-sort (RSX_FS_MODE=9 profiling build path):
queued (upper bound above tau) and kept (exact score above tau) per user, at the sports
shape with random tables (as tools/gpu/fsbal.py) and, with FS_BENCH=1, nothing else.
usage: RSX_FS_MODE=9 python tools/gpu/fs_count.py [nb ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommendar-systems_amd"))
from rsx import ops  # noqa: E402


def main():
    ni, d, k = int(os.environ.get("FS_NI", 18357)), int(os.environ.get("FS_D", 64)), 50
    nbs = [int(x) for x in sys.argv[1:]] or [35598]
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda:0")
    gd = torch.Generator(device=dev).manual_seed(0)
    items = torch.randn(ni, d, generator=gd, device=dev) * 0.1
    for nb in nbs:
        users = torch.randn(nb, d, generator=gd, device=dev) * 0.1
        per = 8
        col = torch.randint(0, ni, (nb, per), generator=g).sort(1).values
        rp = torch.arange(0, nb * per + 1, per, dtype=torch.int64).to(dev)
        cold = col.flatten().to(torch.int32).to(dev)
        _, idx = ops.fullsort_topk(users, None, items, rp, cold, k)
        torch.cuda.synchronize()
        # fullsort_topk allocated idx [nb, k]: the mode-9 kernel accumulated into its first two words
        q, kept = int(idx.view(-1)[0].item()), int(idx.view(-1)[1].item())
        print(f"nb={nb} queued/user={q / nb:.1f} kept/user={kept / nb:.1f}", flush=True)


if __name__ == "__main__":
    main()
