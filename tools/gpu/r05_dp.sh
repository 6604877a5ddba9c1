# round 5: the triplets-only data-parallel step (csrc/dp.hip) — its GPU tests, then the
# latency-injected W = 2/4/8 legs beside the N = 1 lines (tools/gpu/r05_sims.sh PART=dp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05dp}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_dp.log 2>&1
rc=$?
tail -12 $OUT/pytest_dp.log
[ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh
