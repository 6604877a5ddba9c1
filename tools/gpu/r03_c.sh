set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -x -q -k "fullsort or screen or topk" --timeout 200 --timeout-method thread > gpurun_out/fsel_pytest.txt 2>&1 || { tail -20 gpurun_out/fsel_pytest.txt; exit 1; }
tail -n 1 gpurun_out/fsel_pytest.txt
NBS="35598" bash tools/gpu/fs_kstats.sh 2>&1 | grep -v "^W2026\|^E2026" | grep "fs_\|nb=" 
bash tools/gpu/smore_ab.sh
