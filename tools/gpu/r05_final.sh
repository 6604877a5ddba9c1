# round-5 closing evidence: the GPU suite, smoke, the default bench line (with its CPU
# baseline) and its rocprofv3 kernel stats, the C5 / C3 legs and C5's kernel stats, then the
# C5 leg under latency injection (tools/gpu/r05_sims.sh PART=c5) and the DP legs (PART=dp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05final4}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_line.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench_line.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/bench_prof.err || exit 1
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 6 --cpu-budget 15 > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o c5 -- python bench.py --workload c5 --no-cpu-baseline --steps 20 --warmup 6 > $OUT/c5_under_rocprof.json 2> $OUT/c5_prof.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
OUT=$OUT PART=c5 bash tools/gpu/r05_sims.sh && OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
echo done
