# fullsort: waves per CU capped by reserved LDS (RSX_FS_LDS bytes/block) x item chunks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "0 2" "16384 2" "12288 2" "0 3" "16384 3" "0 4" "16384 4" "12288 4" "0 2"; do
  set -- $cfg
  for m in 0 1; do
    RSX_FS_LDS=$1 RSX_FS_CHUNKS=$2 RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1
    echo " lds $1 chunks $2 mode $m"
  done
done
