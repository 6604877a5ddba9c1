"""Summarise a rocprofv3 kernel_stats.csv: share, calls, average per kernel (top N)."""
import csv
import sys

f, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
r = list(csv.DictReader(open(f)))
tot = sum(float(x["TotalDurationNs"]) for x in r)
print(f"total {tot / 1e6:.1f} ms over {sum(int(x['Calls']) for x in r)} launches, {len(r)} kernels")
for x in r[:top]:
    print(f"{float(x['TotalDurationNs']) / tot * 100:5.1f}% {int(x['Calls']):7d} {float(x['AverageNs']) / 1e3:8.1f}us  {x['Name'][:120]}")
