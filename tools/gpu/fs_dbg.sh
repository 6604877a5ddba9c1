set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "fullsort" 2>&1 | tail -3 || exit 1
RSX_FS_MODE=1 timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "mode 1 (scores only)"
for c in 0 1 2 4 8; do RSX_FS_CHUNKS=$c timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "chunks $c"; done
