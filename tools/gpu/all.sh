set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fullsort']['kernel_ms_all_eval_users'])"
mkdir -p gpurun_out/pb && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb/prof -o b -- python bench.py --no-cpu-baseline > gpurun_out/pb/benchp.json 2> gpurun_out/pb/benchp.err || exit 1
find gpurun_out/pb/prof -name '*kernel_trace.csv' -delete
