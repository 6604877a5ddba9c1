set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --steps 200 > gpurun_out/bench_sh1.json 2> gpurun_out/bench_sh1.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_sh1.json')); print(d['value'], d['ms_per_step'], d['gpu_ms_per_step_events'])"
