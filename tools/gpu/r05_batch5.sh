# round 5, fifth GPU batch: the DP gradient pass finishing whole runs without atomics;
# DP tests, the DP legs, a kernel trace and one SQ counter pass of the DP loss kernels at
# a latency-injected W = 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b5}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
RSX_COMM_SIM=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace8 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace8.json 2> $OUT/trace8.err \
  || { tail -20 $OUT/trace8.err; exit 1; }
RSX_COMM_SIM=8 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "dp_" --output-format csv -d $OUT/pmc8 -o p -- \
  python3 bench.py --dp --steps 20 --warmup 5 --no-cpu-baseline > $OUT/pmc8.json 2> $OUT/pmc8.err \
  || { tail -20 $OUT/pmc8.err; exit 1; }
# the C5 embed-sharded leg under latency injection crashed (host segfault) at W = 4: one
# short run with the Python fault handler for its stack
RSX_COMM_SIM=4 PYTHONFAULTHANDLER=1 timeout -k 10 300 python -X faulthandler bench.py --workload c5 --steps 4 --warmup 2 \
  --no-cpu-baseline > $OUT/c5_sim_w4.json 2> $OUT/c5_sim_w4.err; echo "c5 sim w4 rc=$?"; tail -40 $OUT/c5_sim_w4.err
echo done
