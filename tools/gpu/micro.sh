set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/gpu/micro.py spmm && \
for m in 1 2 3 0; do RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "mode $m"; done
