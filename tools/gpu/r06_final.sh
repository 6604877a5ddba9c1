# round 6 closing evidence at the final HEAD: the whole GPU suite (driver-style), smoke, the
# default bench line (+ its rocprofv3 kernel stats), the C1 / C3 / C5 lines with their CPU
# baselines, and the C1 CPU configuration on the box's host threads
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06final}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench_line.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_line.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['fullsort_items_per_s'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --no-cpu-baseline \
  > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_prof.err" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_trace.csv' -delete
for W in c3 c5 c1; do
  timeout -k 10 600 python bench.py --workload $W --steps 30 --warmup 6 > "$OUT/$W.json" 2> "$OUT/$W.err" || { tail -20 "$OUT/$W.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 600 python bench.py --workload c1 --cpu --steps 2 > "$OUT/c1_cpu.json" 2> "$OUT/c1_cpu.err" || { tail -20 "$OUT/c1_cpu.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/c1_cpu.json')); print('c1cpu', d['value'], d['cores'], d['cpu_baseline']['value'])"
echo done
