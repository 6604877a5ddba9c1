# round-4 closing evidence at the final HEAD (after the projection / segsum / DP changes): the GPU suite, smoke,
# baseline) and its rocprofv3 kernel stats, the C5 / C3 legs and C5's kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04final2}
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

# the C2 ADAM layer's HBM bytes at this HEAD (FETCH_SIZE / WRITE_SIZE: separate passes)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_main<64, 3>" --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_main<64, 3>" --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || exit 1
echo done
