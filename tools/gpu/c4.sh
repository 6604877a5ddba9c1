set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 500 python bench.py --workload c4 --c4-chunks 1 --steps 10 --warmup 2 > gpurun_out/c4/c4_1of8.json 2> gpurun_out/c4/c4_1of8.err || { tail -20 gpurun_out/c4/c4_1of8.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4/c4_1of8.json')); print('1of8', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fullsort']['kernel_ms_all_eval_users'])"
timeout -k 10 650 python bench.py --workload c4 --steps 6 --warmup 2 > gpurun_out/c4/c4_full.json 2> gpurun_out/c4/c4_full.err || { tail -20 gpurun_out/c4/c4_full.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4/c4_full.json')); print('full', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fullsort']['kernel_ms_all_eval_users'])"
