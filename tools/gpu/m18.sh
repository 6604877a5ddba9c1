# metrics_user with lockstep hit searches: metric parity tests, then the bench evaluation under rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_smore.py -k "metrics or topk or e2e or reference or epoch" -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/mu
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mu -o b -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/mu/b.json 2> gpurun_out/mu/b.err || exit 1
grep -h "metrics_user\|fs_select" gpurun_out/mu/*kernel_stats.csv | cut -d, -f1-4
find gpurun_out/mu -name '*kernel_trace.csv' -delete
