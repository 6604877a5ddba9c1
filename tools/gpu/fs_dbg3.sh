set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "fullsort" 2>&1 | tail -2 || exit 1
RSX_FS_NUSERS=32768 RSX_FS_MODE=4 timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1
timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1
