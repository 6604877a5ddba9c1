# round 6: kernel stats of the C3 / C5 lines (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06sprof}
mkdir -p "$OUT"
for W in ${WL:-c3 c5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$W" -o $W -- python bench.py --workload $W \
    --steps 20 --warmup 4 --no-cpu-baseline > "$OUT/$W.json" 2> "$OUT/$W.err" || { tail -20 "$OUT/$W.err"; exit 1; }
  find "$OUT/$W" -name '*kernel_trace.csv' -delete
  python -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', d['ms_per_step'])"
done
echo done
