set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --workload c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -30 gpurun_out/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5.json')); print('c5', d['value'], d['ms_per_step'], d['model_build_s'], d['fullsort_items_per_s'], d['config'])"
