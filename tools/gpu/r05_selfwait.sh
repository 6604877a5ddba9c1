# round 5: isolate the graph-replay segfault: a captured fork/join with the side stream at
# default / greatest priority, without and with a self-wait (tools/gpu/exp/selfwait.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/r05sw}
mkdir -p $OUT
timeout -k 10 60 tools/gpu/exp/selfwait 0 0 200 2>&1 | tee -a $OUT/selfwait.txt || exit 1
timeout -k 10 60 tools/gpu/exp/selfwait 0 1 200 2>&1 | tee -a $OUT/selfwait.txt; rc=$?
echo "self_wait=0 priority=1 rc=$rc" | tee -a $OUT/selfwait.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/gpu/exp/selfwait 1 0 200 2>&1 | tee -a $OUT/selfwait.txt; rc=$?
echo "self_wait=1 priority=0 rc=$rc" | tee -a $OUT/selfwait.txt
