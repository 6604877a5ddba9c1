# round 6: pref_segsum_plan ablations (tools/build_variant.py libraries via RSX_LIB): kernel
# stats of a short C3 run per variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06segvar}
mkdir -p "$OUT"
for V in base ${VARS:-ub8 ub2 abl1 abl2}; do
  if [ "$V" = base ]; then unset RSX_LIB; else export RSX_LIB="$GRAFT_REPO_ROOT/recommendar-systems_amd/rsx/lib/variants/$V/librsx.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$V" -o c3 -- \
    python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/c3_$V.json" 2> "$OUT/c3_$V.err" \
    || { tail -20 "$OUT/c3_$V.err"; exit 1; }
  find "$OUT/$V" -name '*kernel_trace.csv' -delete
  python - "$OUT/$V/c3_kernel_stats.csv" "$V" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "segsum" in r["Name"]:
        print(sys.argv[2], f'{float(r["AverageNs"])/1e3:8.2f} us x{r["Calls"]:>4}  {r["Name"][:60]}')
PY
done
echo done
