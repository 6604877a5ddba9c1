"""One step's launch timeline from a rocprofv3 kernel_trace.csv: the dispatches between
two consecutive launches of a marker kernel (the step's first), with start offsets,
durations, queue, and the gaps on each queue.  Usage:
python tools/step_timeline.py KERNEL_TRACE.csv MARKER_SUBSTRING [step_index_from_end]"""
import csv
import re
import sys


def short(n):
    m = re.search(r"rsx::(?:\(anonymous namespace\)::|sf::)?(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:50]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    mark = sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    a, b = idx[-back - 1], idx[-back]
    t0 = int(rows[a]["Start_Timestamp"])
    t_end = int(rows[b]["Start_Timestamp"])
    print(f"step: {len(rows[a:b])} dispatches, {(t_end - t0) / 1e3:.1f} us marker to marker")
    busy = {}
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r["Queue_Id"]
        busy[q] = busy.get(q, 0) + (e - s)
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}us q{q:>2}  {short(r['Kernel_Name'])}")
    for q, v in busy.items():
        print(f"queue {q}: {v / 1e3:.1f} us busy")


if __name__ == "__main__":
    main()
