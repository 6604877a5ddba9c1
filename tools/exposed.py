"""Where a multi-stream step's time goes: over one step window of a rocprofv3 kernel_trace.csv
(between the ends of two marker launches `per` launches apart), each kernel's exclusive
time (no other kernel running: a kernel that is on the step's critical path shows here),
its shared time, and the idle time.  Usage:
python tools/exposed.py KERNEL_TRACE.csv MARKER [per] [top]"""
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
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    a, b = idx[-1 - per], idx[-1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    ev = []
    for r in rows:
        s, e = max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1)
        if e > s:
            k = short(r["Kernel_Name"])
            ev += [(s, 1, k), (e, -1, k)]
    ev.sort()
    active = collections.Counter()
    excl = collections.defaultdict(float)
    shared = collections.defaultdict(float)
    idle = 0.0
    prev = t0
    for t, d, k in ev:
        if t > prev:
            span = (t - prev) / 1e3
            n = sum(active.values())
            if n == 0:
                idle += span
            elif n == 1:
                excl[next(iter(+active))] += span
            else:
                for kk, c in active.items():
                    if c:
                        shared[kk] += span * c / n
            prev = t
        active[k] += d
    tot = (t1 - t0) / 1e3
    print(f"window {tot:.1f} us: exclusive {sum(excl.values()):.1f}, shared (split evenly) {sum(shared.values()):.1f}, "
          f"idle {idle:.1f}")
    keys = sorted(set(excl) | set(shared), key=lambda k: -(excl[k]))
    print(f"{'kernel':48s} {'exclusive':>10s} {'shared':>9s}")
    for k in keys[:top]:
        print(f"{k[:48]:48s} {excl[k]:10.1f} {shared[k]:9.1f}")


if __name__ == "__main__":
    main()
