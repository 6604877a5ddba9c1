set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 32768 35598; do for m in 1 0; do RSX_FS_NUSERS=$n RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort || exit 1; echo "users $n mode $m"; done; done
