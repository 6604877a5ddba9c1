# C4: one rank's 1/8 share (1.25M users x 1M items, d=256) through the sharded engine on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --workload c4 --c4-chunks 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c4one.json 2> gpurun_out/c4one.err
rc=$?; tail -3 gpurun_out/c4one.err; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/c4one.json')); print(round(d['value']), d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fullsort']['kernel_ms_all_eval_users'])"
