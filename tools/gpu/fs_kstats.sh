# per-kernel times of one full-sort call shape (tools/gpu/fsbal.py) under rocprofv3: NBS="35598 32768"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fsk}
mkdir -p $OUT
for nb in ${NBS:-35598 32768}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/n$nb -o run -- python tools/gpu/fsbal.py $nb > $OUT/n$nb.log 2>&1 || exit 1
  echo "== nb $nb"; grep -v amdgpu $OUT/n$nb.log
  python tools/kstats.py $(find $OUT/n$nb -name '*kernel_stats.csv') 8
  find $OUT/n$nb -name '*kernel_trace.csv' -delete
done
