set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest "$@" -q -p no:cacheprovider > gpurun_out/pytest_some.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_some.log
tail -40 gpurun_out/pytest_some.log
