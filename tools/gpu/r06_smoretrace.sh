# round 6: a kernel trace of a few C3 / C5 steps (per-step kernel sequence, tools/smore_trace.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06strace}
mkdir -p "$OUT"
for W in ${WL:-c3 c5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$W" -o $W -- python bench.py --workload $W \
    --steps 4 --warmup 3 --no-cpu-baseline > "$OUT/$W.json" 2> "$OUT/$W.err" || { tail -20 "$OUT/$W.err"; exit 1; }
  f=$(find "$OUT/$W" -name '*kernel_trace.csv' | head -1)
  python - "$f" "$OUT/${W}_trace_min.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
with open(sys.argv[2], "w", newline="") as fo:
    w = csv.writer(fo)
    w.writerow(["start", "end", "name"])
    for r in rows:
        w.writerow([r["Start_Timestamp"], r["End_Timestamp"], r["Kernel_Name"][:120]])
PY
  find "$OUT/$W" -name '*kernel_trace.csv' -delete
done
echo done
