# round-3 evidence: the GPU suite, smoke, PMC FETCH/WRITE passes of the C2 SpMM launches
# (STORE and ADAM kinds), the default bench line under rocprofv3 --stats, the plain line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_main<64, [03]>" --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_main<64, [03]>" --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
