# round 5, third GPU batch: the DP step with batched gradient bookkeeping and bucketed runs
# (tests, then the N = 1 / latency-injected W = 2 / 4 / 8 legs), the SMORE kernels' tests
# (sparse preference gradients, two-group InfoNCE backward), the InfoNCE backward's A/B
# (digests must match), and the C5 / C3 step lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b3}
mkdir -p $OUT
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }  # a failed assertion: go on; a fault / abort / timeout: stop
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_smore_fuse.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -15; ok $rc || exit $rc
for g in 1 2; do
  RSX_NCE_GROUPS=$g timeout -k 10 120 python tools/gpu/micro_nce.py >> $OUT/micro_nce.txt 2>&1 || exit 1
done
cat $OUT/micro_nce.txt
[ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
for w in c5 c3; do
  timeout -k 10 600 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err \
    || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', round(d['ms_per_step'], 4), 'ms/step')"
done
