set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sm
for w in c1 c3 c5; do timeout -k 10 400 python bench.py --workload $w --steps 30 --warmup 5 > gpurun_out/sm/$w.json 2> gpurun_out/sm/$w.err || { tail -5 gpurun_out/sm/$w.err; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/sm/$w.json')); print('$w', d['value'], d['ms_per_step'], d['fullsort_items_per_s'], d['config'].get('graph_step'))"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sm/p3 -o c3 -- python3 bench.py --workload c3 --steps 20 --warmup 5 > gpurun_out/sm/c3p.json 2> gpurun_out/sm/c3p.err || exit 1
find gpurun_out/sm/p3 -name '*kernel_trace.csv' -delete
