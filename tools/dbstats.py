"""Per-kernel statistics (calls, total, average) from a rocprofv3 rocpd database
(rocprofv3 without --output-format csv writes *_results.db), like kernel_stats.csv;
optionally only the dispatches after the first `skip` of a given kernel name.
Usage: python tools/dbstats.py RUN_results.db [top] [--csv OUT.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    return sorted(((n, k, t) for n, (k, t) in agg.items()), key=lambda x: -x[2]), rows


if __name__ == "__main__":
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    res, _ = stats(db)
    tot = sum(t for _, _, t in res)
    print(f"total {tot / 1e6:.2f} ms over {sum(k for _, k, _ in res)} launches, {len(res)} kernels")
    for n, k, t in res[:top]:
        print(f"{t / tot * 100:5.1f}% {k:7d} {t / k / 1e3:8.2f}us  {n[:110]}")
    if "--csv" in sys.argv:
        out = sys.argv[sys.argv.index("--csv") + 1]
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, k, t in res:
                w.writerow([n, k, t, t / k, t / tot * 100])
