"""Busy time vs wall span of the last `n` occurrences of an anchor kernel's period in a
rocprofv3 kernel_trace.csv (the per-step GPU timeline: kernel time, idle gaps, launches)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0, i1 = idx[-n - 1], idx[-1]
seg = rows[i0:i1]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3
print(f"{n} periods: span {span / n:.1f} us, busy {busy / n:.1f} us, idle {(span - busy) / n:.1f} us, "
      f"launches {len(seg) / n:.1f} per period")
by = defaultdict(lambda: [0.0, 0])
for r in seg:
    name = r["Kernel_Name"]
    k = name[:150] if "at::native" in name else name.split("(")[0][:70]
    by[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by[k][1] += 1
for k, (t, c) in sorted(by.items(), key=lambda x: -x[1][0])[: int(sys.argv[4]) if len(sys.argv) > 4 else 30]:
    print(f"{t / n:8.1f} us {c / n:6.2f}x  {k}")
