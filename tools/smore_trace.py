"""Per-step kernel breakdown of a SMORE bench trace (tools/gpu/r06_smoretrace.sh output):
steps are delimited by the step's second adam_multi (the mirror-gradient step runs two);
prints, for step STEP (default: the last whole timed one), each kernel's total time in
the step, its count, and the step's GPU busy time vs wall time.

python tools/smore_trace.py gpurun_out/r06strace/c3_trace_min.csv [STEP]"""
import collections
import csv
import sys

rows = [(int(r["start"]), int(r["end"]), r["name"]) for r in csv.DictReader(open(sys.argv[1]))]
rows.sort()
adam = [i for i, r in enumerate(rows) if "adam_multi" in r[2]]
ends = adam[1::2]  # the second Adam of each step closes it
step = int(sys.argv[2]) if len(sys.argv) > 2 else len(ends) - 1
lo = ends[step - 1] + 1 if step > 0 else 0
hi = ends[step] + 1
seg = rows[lo:hi]
wall = (seg[-1][1] - seg[0][0]) / 1e3
busy = sum(e - s for s, e, _ in seg) / 1e3
agg = collections.defaultdict(lambda: [0.0, 0])
for s, e, n in seg:
    k = n.split("(")[0].replace("void ", "")
    agg[k][0] += (e - s) / 1e3
    agg[k][1] += 1
print(f"step {step} of {len(ends)}: {len(seg)} kernels, wall {wall:.1f} us, busy {busy:.1f} us")
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{t:9.1f} us {c:4d}x  {k[:100]}")
