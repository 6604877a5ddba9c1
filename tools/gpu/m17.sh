# fs_select with the narrowed radix search: parity tests, then its kernel time under rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -k "fullsort or topk or lightgcn" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fs.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fs.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/fsel
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fsel -o fs -- python tools/gpu/micro.py fullsort > gpurun_out/fsel/out.txt 2>&1 || exit 1
grep -h "fs_select\|fs_tiles" gpurun_out/fsel/*kernel_stats.csv | cut -d, -f1-4
find gpurun_out/fsel -name '*kernel_trace.csv' -delete
