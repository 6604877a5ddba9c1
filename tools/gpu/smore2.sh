set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pw
timeout -k 10 600 python -m pytest tests/test_gpu_smore.py -q -x -p no:cacheprovider > gpurun_out/smore_t.log 2>&1 || { tail -40 gpurun_out/smore_t.log; exit 1; }
tail -2 gpurun_out/smore_t.log
for w in c3 c5; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pw/$w -o $w -- python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/pw/$w.json 2> gpurun_out/pw/$w.err || exit 1
done
find gpurun_out/pw -name '*kernel_trace.csv' -delete
for w in c3 c5; do timeout -k 10 400 python bench.py --workload $w > gpurun_out/$w.json 2> gpurun_out/$w.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/$w.json')); print('$w', d['value'], d['ms_per_step'])"; done
