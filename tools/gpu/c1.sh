set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_e2e.py tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "layergcn or edge_dropout" > gpurun_out/c1_tests.log 2>&1 || { tail -30 gpurun_out/c1_tests.log; exit 1; }
tail -2 gpurun_out/c1_tests.log
timeout -k 10 400 python bench.py --workload c1 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -20 gpurun_out/c1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c1.json')); print('c1', d['value'], d['ms_per_step'], d['steps'])"
