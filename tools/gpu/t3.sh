# sharded step with the one-launch BPR: dist tests, then the sharded bench at one rank
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
  RSX_BPR_FUSED=$f timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > gpurun_out/sh_$f.json 2> gpurun_out/sh_$f.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sh_$f.json')); print('fused=$f', round(d['value']), d['ms_per_step'])"
done
