# round 6: alternating A/B of an environment knob on one workload: KNOB=name, W=workload,
# R=rounds; prints ms/step per run and the medians
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06ab}
mkdir -p "$OUT"
W=${W:-c5}; R=${R:-4}; KNOB=${KNOB:-RSX_LBWD_PAIR}
for r in $(seq 1 $R); do
  for v in 1 0; do
    env "$KNOB=$v" timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-60} --warmup 6 --no-cpu-baseline \
      > "$OUT/${W}_${v}_$r.json" 2> "$OUT/${W}_${v}_$r.err" || { tail -20 "$OUT/${W}_${v}_$r.err"; exit 1; }
    python -c "import json; print('$W $KNOB=$v run $r', round(json.load(open('$OUT/${W}_${v}_$r.json'))['ms_per_step'], 4))"
  done
done
python - "$OUT" "$W" <<'PY'
import glob, json, statistics, sys
for v in ("1", "0"):
    xs = [json.load(open(f))["ms_per_step"] for f in glob.glob(f"{sys.argv[1]}/{sys.argv[2]}_{v}_*.json")]
    print(sys.argv[2], "knob", v, "median", round(statistics.median(xs), 4), "min", round(min(xs), 4), "n", len(xs))
PY
echo done
