# round 5, twelfth GPU batch: the DP forward layers issued ahead of the comm branch (host
# order); DP tests, the DP legs, a one-rank DP kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b12}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace1 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace1.json 2> $OUT/trace1.err \
  || { tail -20 $OUT/trace1.err; exit 1; }
echo done
