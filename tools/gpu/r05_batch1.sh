# round 5, first GPU batch: the triplets-only DP step's tests, the one-launch SMORE item
# side against the three-launch chain, then the DP latency-injected legs (r05_sims.sh PART=dp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b1}
mkdir -p $OUT
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }  # a failed assertion: go on; a fault / abort / timeout: stop
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_dp.log 2>&1
rc=$?; tail -8 $OUT/pytest_dp.log; ok $rc || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_smore.py -m gpu -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "item_side or spectral" > $OUT/pytest_item.log 2>&1
rc2=$?; tail -12 $OUT/pytest_item.log; ok $rc2 || exit $rc2
timeout -k 10 120 python tools/gpu/micro_item.py > $OUT/micro_item.txt 2>&1; rc3=$?; cat $OUT/micro_item.txt
[ $rc3 -eq 0 ] || exit $rc3
[ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh
