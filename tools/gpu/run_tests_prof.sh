set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -15 gpurun_out/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo "rocprof rc=$?"
find gpurun_out/prof1 -name "*kernel_stats.csv" | head -3
