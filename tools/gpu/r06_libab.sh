# round 6: alternating A/B of tools/build_variant.py libraries (RSX_LIB) on one workload:
# VARS="name ..." (base = the in-tree library), W, R rounds; medians of ms/step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06libab}
mkdir -p "$OUT"
W=${W:-c2}; R=${R:-3}
for r in $(seq 1 $R); do
  for V in base $VARS; do
    if [ "$V" = base ]; then unset RSX_LIB; else export RSX_LIB="$GRAFT_REPO_ROOT/recommendar-systems_amd/rsx/lib/variants/$V/librsx.so"; fi
    timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline \
      > "$OUT/${W}_${V}_$r.json" 2> "$OUT/${W}_${V}_$r.err" || { tail -20 "$OUT/${W}_${V}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${W}_${V}_$r.json')); print('$W $V run $r', round(d['ms_per_step'], 5), round(d['roofline']['avg_launch_ms']*1e3, 2))"
  done
done
python - "$OUT" "$W" base $VARS <<'PY'
import glob, json, statistics, sys
out, w = sys.argv[1], sys.argv[2]
for v in sys.argv[3:]:
    xs = [json.load(open(f))["ms_per_step"] for f in glob.glob(f"{out}/{w}_{v}_*.json")]
    print(w, v, "median", round(statistics.median(xs), 5), "min", round(min(xs), 5), "n", len(xs))
PY
echo done
