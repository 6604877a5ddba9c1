set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base cap512 cap128; do
  if [ $v = base ]; then L=recommendar-systems_amd/rsx/lib/librsx.so; else L=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  for c in 2 4; do RSX_FS_CHUNKS=$c RSX_LIB=$PWD/$L timeout -k 10 100 python tools/gpu/micro.py fullsort 2>/dev/null | tr -d '\n' || exit 1; echo " $v chunks $c"; done
done
