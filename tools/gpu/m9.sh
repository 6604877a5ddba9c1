#!/bin/bash
# fullsort A/B: current tree vs the pre-change variant (fsold), after the fullsort parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fullsort" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fs.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fs.log; [ $rc -eq 0 ] || exit $rc
for v in base fsold rej rejng flng base fsold rej rejng flng; do
  if [ $v = base ]; then L=recommendar-systems_amd/rsx/lib/librsx.so; else L=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  for m in 0 1; do
    RSX_FS_MODE=$m RSX_LIB=$PWD/$L timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1
    echo " $v mode $m"
  done
done
