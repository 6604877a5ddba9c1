# round 6: C5 ms/step over settings of one environment knob (KNOB, VALS; "-" = unset), R rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06envsweep}
mkdir -p "$OUT"
W=${W:-c5}
for r in $(seq 1 ${R:-2}); do
  for v in $VALS; do
    if [ "$v" = "-" ]; then unset "$KNOB"; else export "$KNOB=$v"; fi
    timeout -k 10 300 python bench.py --workload $W --steps 60 --warmup 6 --no-cpu-baseline > "$OUT/${W}_${v}_$r.json" \
      2> "$OUT/${W}_${v}_$r.err" || { tail -20 "$OUT/${W}_${v}_$r.err"; exit 1; }
    python -c "import json; print('$W $KNOB=$v run $r', round(json.load(open('$OUT/${W}_${v}_$r.json'))['ms_per_step'], 4))"
  done
done
unset "$KNOB"
echo done
