# round 5, sixth GPU batch: the remaining capture patterns of the latency-injected Comm
# (autograd all-reduce), the C5 leg under latency injection with the UI backbone on the
# capturing stream, and the DP legs with the last forward layer dense over > 1 rank
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b6}
mkdir -p $OUT
RSX_COMM_SIM=4 timeout -k 10 120 python -X faulthandler tools/gpu/diag_smore_sim.py grad > $OUT/diag_grad.txt 2>&1
rc=$?; echo "diag grad rc=$rc"; tail -2 $OUT/diag_grad.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_dp.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest_dp.log | tail -5; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
OUT=$OUT PART=c5 bash tools/gpu/r05_sims.sh || exit 1
echo done
