# real-shape parity tests + the tests touched this round (round 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  ${RSX_TESTS:-tests/test_gpu_realshape.py tests/test_gpu_smore.py} tests/test_gpu_dist.py \
  "tests/test_gpu_kernels.py::test_topk_metrics_device_bitwise_vs_numpy" > gpurun_out/realshape.log 2>&1
rc=$?
tail -30 gpurun_out/realshape.log
exit $rc
