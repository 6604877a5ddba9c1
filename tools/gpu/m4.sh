set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in 4 1 2 3 0; do RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "mode $m"; done
