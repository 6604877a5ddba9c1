# per-phase fs_screen times under the pass-2 ablations (RSX_FS_MODE 0 full, 6 no exact dots,
# 8 no candidates at all) at the sports shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fsm2}
mkdir -p $OUT
for m in 0 6 8; do
  RSX_FS_MODE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/m$m -o run -- python tools/gpu/fsbal.py ${NB:-35598} > $OUT/m$m.log 2>&1 || exit 1
  echo "== mode $m"; grep -v amdgpu $OUT/m$m.log | grep nb=
  python tools/kstats.py $(find $OUT/m$m -name '*kernel_stats.csv') 4
  find $OUT/m$m -name '*kernel_trace.csv' -delete
done
