"""Print one training step's kernel timeline from a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
anchor = sys.argv[2] if len(sys.argv) > 2 else 'bpr_fwd'
idx = [i for i, r in enumerate(rows) if anchor in r['Kernel_Name']]
k = int(sys.argv[3]) if len(sys.argv) > 3 else len(idx) // 2
back = int(sys.argv[4]) if len(sys.argv) > 4 else 8
i0, i1 = idx[k], idx[k + 1]
t0 = int(rows[i0]['Start_Timestamp'])
prev = None
tot = 0
for r in rows[i0 - back:i1 - back]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1000 if prev else 0
    tot += (e - s) / 1000
    print(f"{(s - t0) / 1000:8.1f} gap {gap:6.1f} dur {(e - s) / 1000:6.1f} {r['Kernel_Name'][:80]}")
    prev = e
print("busy", round(tot, 1), "span", (prev - int(rows[i0 - back]['Start_Timestamp'])) / 1000)
