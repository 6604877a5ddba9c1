"""One step's kernel time by kernel and by queue from a rocprofv3 kernel_trace.csv: the
window between the ends of two launches of a marker kernel `per` marker launches apart
(SMORE: adam_multi, two a step), with the latency-injected collectives (sim_collective)
listed one by one.  Usage:
python tools/step_breakdown.py KERNEL_TRACE.csv MARKER [per] [top]"""
import collections
import csv
import re
import sys


def short(n):
    m = re.search(r"rsx::(?:\(anonymous namespace\)::|sf::|knn::)?(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    mark = sys.argv[2]
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
    idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    a, b = idx[-1 - per], idx[-1]
    seg = rows[a + 1:b + 1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    print(f"step window {(t1 - t0) / 1e6:.3f} ms, {len(seg)} dispatches")
    agg = collections.defaultdict(lambda: [0, 0.0])
    q = collections.defaultdict(float)
    sims = []
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
        q[r.get("Queue_Id", "?")] += d
        if "sim_collective" in r["Kernel_Name"]:
            sims.append(round(d))
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{k[:48]:48s} {c:4d} {t:9.1f} us")
    print("busy per queue (ms):", {k: round(v / 1e3, 3) for k, v in q.items()})
    if sims:
        print(f"latency-injected collectives: {len(sims)}, {sum(sims) / 1e3:.2f} ms: {sims}")


if __name__ == "__main__":
    main()
