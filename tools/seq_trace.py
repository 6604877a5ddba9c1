"""Print the kernel sequence of one training step from a rocprofv3 kernel_trace.csv:
the launches between the N-th and (N+1)-th launch of ANCHOR (default adam_multi), with
start offset, duration and grid size, so that the launches of one kernel template
(e.g. spmm_main<128, 0>) can be told apart by their place in the step.
usage: python tools/seq_trace.py TRACE.csv [ANCHOR] [N]"""
import csv
import sys


def main():
    f = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "adam_multi"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(idx) < n + 2:
        raise SystemExit(f"only {len(idx)} {anchor} launches")
    a, b = idx[n], idx[n + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    tot = 0
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        tot += e - s
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        q = r.get("Queue_Id") or r.get("Stream_Id") or ""
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}us q{q:>3} grid {g:>9}  {r['Kernel_Name'][:110]}")
    print(f"step span {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us, kernel sum {tot / 1e3:.1f} us")


if __name__ == "__main__":
    main()
