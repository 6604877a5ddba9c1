# fullsort: early-stopping running compactions (RSX_FS_SLACK; -1 = exact top k as before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -k "fullsort or topk or lightgcn or layergcn" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fs.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fs.log; [ $rc -eq 0 ] || exit $rc
for v in base slack-1 slack16 slack64 base slack-1; do
  if [ $v = base ]; then L=recommendar-systems_amd/rsx/lib/librsx.so; else L=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  RSX_LIB=$PWD/$L timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1
  echo " $v"
done
