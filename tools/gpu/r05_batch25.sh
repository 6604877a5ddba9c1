# round 5, twenty-fifth GPU batch: as the 24th, with the run places taken in the loss pass
# (dp_bpr_coef, no dp_scatter launch); DP tests, the A/B against the forked branch, a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b25}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -14; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=solo bash tools/gpu/r05_sims.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace1 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace1.json 2> $OUT/trace1.err \
  || { tail -20 $OUT/trace1.err; exit 1; }
echo done
