# fullsort per-segment memtime profile (RSX_FS_MODE=4) with the warm-up threshold
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
RSX_FS_MODE=4 timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null || exit 1
