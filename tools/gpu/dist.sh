# sharded LightGCN: GPU dist tests (2 ranks on one GPU over gloo + the 1-rank RCCL native step), then the
# one-rank sharded bench (RCCL communicator, sparse exchange schedule)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dist
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist.py ${EXTRA:-} > gpurun_out/dist/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/dist/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > gpurun_out/dist/c2_sharded.json 2> gpurun_out/dist/c2_sharded.err || { tail -20 gpurun_out/dist/c2_sharded.err; exit 1; }
cat gpurun_out/dist/c2_sharded.json
