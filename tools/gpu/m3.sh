set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "metrics" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gpu/micro.py metrics || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['value'], d['ms_per_step'], d['fullsort_items_per_s'], d['fullsort'])"
