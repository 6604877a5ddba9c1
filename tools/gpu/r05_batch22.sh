# round 5, twenty-second GPU batch: the DP tests with hot rows (long runs across chunks)
# and the run-state check, against the committed gradient pass + dp_bpr_round
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b22}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -14; [ $rc -eq 0 ] || exit $rc
echo done
