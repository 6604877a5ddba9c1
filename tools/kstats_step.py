"""Per-step view of a rocprofv3 kernel_stats.csv: total ms / n_steps for each kernel (top N)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"all kernels: {tot / 1e6 / steps:.3f} ms/step, {calls / steps:.1f} launches/step")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e3 / steps:8.1f} us/step {int(r['Calls']) / steps:6.2f} calls "
          f"avg {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:100]}")
