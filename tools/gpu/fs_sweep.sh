set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k fullsort -p no:cacheprovider 2>&1 | tail -2
for c in 1 2 3 4 6 8; do RSX_FS_CHUNKS=$c timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "chunks $c"; done
for m in 1 3; do RSX_FS_CHUNKS=4 RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "mode $m (chunks 4)"; done
