# PMC passes for the bench's SpMM kernel (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err && \
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
echo "rc=$?"
ls gpurun_out/pmc_fetch gpurun_out/pmc_write
