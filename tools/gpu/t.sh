set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "metrics" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['fullsort_items_per_s'], d['fullsort']['s_per_eval'])"
