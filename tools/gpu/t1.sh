set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
RSX_BATCH_TAGS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_dense.json 2> gpurun_out/bench_dense.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_dense.json')); print('dense', d['value'], d['ms_per_step'])"
