"""Summarise a rocprofv3 kernel trace: per-kernel durations and the idle gaps between
consecutive kernels over the last N steps (one step = the kernels between two
occurrences of the step's first kernel)."""
import csv
import sys
from collections import defaultdict

path, first = sys.argv[1], sys.argv[2]
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [k for k, r in enumerate(rows) if first in r["Kernel_Name"]]
if len(starts) < nsteps + 1:
    raise SystemExit(f"only {len(starts)} steps")
a, b = starts[-nsteps - 1], starts[-1]
seg = rows[a:b]
tot = (int(rows[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / nsteps / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / nsteps / 1e3
print(f"per step: {tot:.1f} us wall, {busy:.1f} us in kernels, {len(seg) / nsteps:.1f} kernels")
gap = defaultdict(float)
dur = defaultdict(float)
cnt = defaultdict(int)
for k, r in enumerate(seg):
    name = r["Kernel_Name"][:70]
    dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[name] += 1
    nxt = rows[a + k + 1]
    gap[name] += (int(nxt["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
for name in sorted(dur, key=lambda n: -dur[n]):
    print(f"{dur[name] / nsteps:8.2f} us  x{cnt[name] / nsteps:4.1f}  gap-after {gap[name] / nsteps:7.2f} us  {name}")
