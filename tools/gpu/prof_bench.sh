set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pb
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pb/bench.json 2> gpurun_out/pb/bench.err || exit 1
cat gpurun_out/pb/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fullsort']['kernel_ms_all_eval_users'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb/prof -o b -- python bench.py --no-cpu-baseline > gpurun_out/pb/benchp.json 2> gpurun_out/pb/benchp.err || exit 1
f=$(find gpurun_out/pb/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -14
find gpurun_out/pb/prof -name '*kernel_trace.csv' -delete
