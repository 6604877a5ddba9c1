set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "metrics" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['ms_per_step'], d['fullsort']['s_per_eval'], d['fullsort_items_per_s'])"
