# round 5, twenty-first GPU batch: the DP gradient pass finishing crossing runs itself
# (per-row segment counters, the last segment's group rounds the sum; dp_bpr_round gone);
# DP tests (hot rows: long runs across chunks; the run state cleared after each step), the
# DP legs, one-rank and W = 8 kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b21}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace1 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace1.json 2> $OUT/trace1.err \
  || { tail -20 $OUT/trace1.err; exit 1; }
RSX_COMM_SIM=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace8 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace8.json 2> $OUT/trace8.err \
  || { tail -20 $OUT/trace8.err; exit 1; }
echo done
