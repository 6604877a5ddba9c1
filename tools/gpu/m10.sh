#!/bin/bash
# fullsort: item chunks per 32-user wave (RSX_FS_CHUNKS) vs time, full and scores-only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in 1 2 3 4 5 6 8; do
  for m in 0 1; do
    RSX_FS_CHUNKS=$c RSX_FS_MODE=$m timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1
    echo " chunks $c mode $m"
  done
done
