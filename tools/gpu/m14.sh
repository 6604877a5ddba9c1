# fullsort candidate-row capacity (RSX_FS_CAP) with the warm-up threshold in place
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base cap384 cap512 cap192 base cap384; do
  if [ $v = base ]; then L=recommendar-systems_amd/rsx/lib/librsx.so; else L=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  RSX_LIB=$PWD/$L timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1
  echo " $v"
done
