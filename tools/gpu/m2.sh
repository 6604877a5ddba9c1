set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do RSX_SPMM_XCD=$x timeout -k 10 200 python tools/gpu/micro.py floor || exit 1; echo "xcd $x"; done
for x in 0 1; do RSX_SPMM_XCD=$x timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_x$x.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/b_x$x.json')); print('xcd $x', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
