# round 5, twenty-sixth GPU batch: the run places taken in the loss pass at W > 1 too
# (RSX_DP_PLACES_IN_LOSS=1): the DP tests with it on, then the latency-injected A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b26}
mkdir -p $OUT
RSX_DP_PLACES_IN_LOSS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -14; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=places bash tools/gpu/r05_sims.sh || exit 1
echo done
