# fused SMORE kernels: parity tests, then the SMORE GPU tests and the C3/C5 legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sf
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_smore_fuse.py ${EXTRA:-} > gpurun_out/sf/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/sf/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in ${LEGS:-}; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/sf/$w.json 2> gpurun_out/sf/$w.err || { tail -20 gpurun_out/sf/$w.err; exit 1; }
  cat gpurun_out/sf/$w.json
done
