# round 6: kernel stats of the C3 line with the occurrence plan on and off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06planprof}
mkdir -p "$OUT"
for P in 1 0; do
  RSX_PREF_PLAN=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$P" -o c3 -- \
    python bench.py --workload c3 --steps 20 --warmup 4 --no-cpu-baseline > "$OUT/c3_p$P.json" 2> "$OUT/c3_p$P.err" \
    || { tail -20 "$OUT/c3_p$P.err"; exit 1; }
  find "$OUT/p$P" -name '*kernel_trace.csv' -delete
  python - "$OUT/p$P/c3_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("pref_", "tag_rows")):
        print(f'{float(r["AverageNs"])/1e3:8.2f} us x{r["Calls"]:>4}  {n[:80]}')
PY
done
echo done
