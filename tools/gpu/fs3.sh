# fs_screen A/B (HEAD-of-round baseline variant vs current, one/two phases, ABUF=2), the
# full-sort exactness tests in both phase modes, then a C5 kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fsv3
mkdir -p $O
(echo "base"; RSX_LIB=recommendar-systems_amd/rsx/lib/variants/base/librsx.so timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 && echo "cur"; timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 && echo "cur 1phase"; RSX_FS_2PHASE=0 timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 && echo "ab2"; RSX_LIB=recommendar-systems_amd/rsx/lib/variants/ab2/librsx.so timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768) > $O/t.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py tests/test_gpu_sharded_trainer.py -m gpu -x -q -k "fullsort or screen or topk or eval" --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
RSX_FS_2PHASE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -x -q -k "fullsort or screen or topk" --timeout 200 --timeout-method thread > $O/pytest1.txt 2>&1 || exit 1
LEGS=${LEGS-c5} OUT=gpurun_out/pl5 bash tools/gpu/prof_leg.sh > gpurun_out/pl5.txt 2>&1
