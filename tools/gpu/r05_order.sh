# round 5: the sharded step's stream order (poisoned latency-injected collectives, comm
# priority on for eager issue, the capture stream at default priority; one-rank RCCL), then
# the multi-round capture experiment with the side stream at the greatest priority
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05order}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_dist.log 2>&1
rc=$?
tail -25 $OUT/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/gpu/exp/selfwait 0 0 100 16 2>&1 | tee -a $OUT/selfwait.txt || exit 1
timeout -k 10 60 tools/gpu/exp/selfwait 0 1 100 16 2>&1 | tee -a $OUT/selfwait.txt; rc=$?
echo "self_wait=0 priority=1 rounds=16 rc=$rc" | tee -a $OUT/selfwait.txt
