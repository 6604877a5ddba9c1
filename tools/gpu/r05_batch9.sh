# round 5, ninth GPU batch: the DP loss passes with narrow lane groups on a small global
# batch (a triplet / 4 run places a group at W * B < 8192); DP tests (both forms), the DP
# legs, a one-rank DP kernel trace; one C5 step's kernel trace for its exclusive-time
# breakdown (tools/exposed.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b9}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace1 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace1.json 2> $OUT/trace1.err \
  || { tail -20 $OUT/trace1.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5 -o t -- \
  python3 bench.py --workload c5 --steps 12 --warmup 6 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err \
  || { tail -20 $OUT/c5.err; exit 1; }
python tools/exposed.py $OUT/c5/t_kernel_trace.csv adam_multi 2 40 > $OUT/c5_exposed.txt && head -30 $OUT/c5_exposed.txt
echo done
