# PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes) for the C2 step's ADAM layer
# (spmm_main<64, 3>: the step's own launches and the bench's standalone ones), then
# the bench line with rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pa}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_main<64, 3>" --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_main<64, 3>" --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?
find $OUT -name '*kernel_trace.csv' -delete
echo "rc=$rc"
