# round 4: the data-parallel step with its Adam counter incremented by dp_pack (inc_step):
# the DP tests, then the one-rank measurement (r04_dpm.sh) into r04dpm2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04dpm2
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04dpm2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04dpm2/pytest.log; [ $rc -eq 0 ] || exit $rc
export OUT=gpurun_out/r04dpm2; bash tools/gpu/r04_dpm.sh
