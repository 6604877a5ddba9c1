# PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes) for the C5 step's three kNN
# item-view products (spmm_batch<128, 0>: the step's own launches and the bench's
# standalone roofline launches), so the view product's roofline fraction has a
# traffic ratio beside it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_knn}
mkdir -p $OUT
A="--workload c5 --steps 6 --warmup 3 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_batch<128, 0>" --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py $A > $OUT/fetch_line.json 2> $OUT/pmc_fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_batch<128, 0>" --output-format csv -d $OUT/pmc_write -o run -- python bench.py $A > $OUT/write_line.json 2> $OUT/pmc_write.err
rc=$?
echo "rc=$rc"
exit $rc
