# PMC passes for the bench's SpMM kernel (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass),
# then the kernel-trace summary and the full bench line (with the CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_main<64, 0>" --output-format csv -d gpurun_out/r11/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/r11/pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_main<64, 0>" --output-format csv -d gpurun_out/r11/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/r11/pmc_write.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r11/stats -o bench -- python bench.py --no-cpu-baseline > gpurun_out/r11/bench_prof.json 2> gpurun_out/r11/bench_prof.err && \
timeout -k 10 600 python bench.py > gpurun_out/r11/bench_full.json 2> gpurun_out/r11/bench_full.err
rc=$?
find gpurun_out/r11 -name '*kernel_trace.csv' -delete
echo "rc=$rc"
