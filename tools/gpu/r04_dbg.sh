# round 4: bisect the one-rank RCCL sharded-step crash (test_native_sharded_step_equals_python_sequence[True])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r04dbg}
mkdir -p $OUT
T="${T:-tests/test_gpu_dist.py::test_native_sharded_step_equals_python_sequence}"
for cfg in ${CFGS:-"RSX_COMM_PRIORITY=0" "RSX_SHARDED_NBR=0" "RSX_SHARDED_HEAD=1" "RSX_SHARDED_GRAPH=0"}; do
  n=$(echo $cfg | tr '=' '_')
  timeout -k 10 200 env $cfg python -u -m pytest "$T" -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/$n.log 2>&1
  echo "$cfg rc=$?"
  grep -E "passed|failed|Fatal Python|File \"" $OUT/$n.log | head -12
done
