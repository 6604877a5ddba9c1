# round 5, second GPU batch: the table-driven spectral kernels (forward, the two-pass
# backward) and the one-launch item side with its one-lane hand-off; the SMORE GPU tests,
# the item-side micro-benchmark, then the C5 and C3 step lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b2}
mkdir -p $OUT
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }  # a failed assertion: go on; a fault / abort / timeout: stop
timeout -k 10 500 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest_smore.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest_smore.log | tail -15; ok $rc || exit $rc
timeout -k 10 120 python tools/gpu/micro_item.py > $OUT/micro_item.txt 2>&1; rc3=$?; cat $OUT/micro_item.txt
[ $rc3 -eq 0 ] || exit $rc3
[ $rc -eq 0 ] || exit $rc
for w in c5 c3; do
  timeout -k 10 600 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err \
    || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', round(d['ms_per_step'], 4), 'ms/step')"
done
