# full-sort timing of the librsx variants built by tools/build_variant.py (VARS), fs_tiles last
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/fsvar}
mkdir -p $OUT; rm -f $OUT/t.txt
for v in ${VARS-w2a1}; do
  echo "variant $v" >> $OUT/t.txt
  RSX_LIB=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so timeout -k 10 120 python tools/gpu/fsbal.py ${NBS:-32768 35598} >> $OUT/t.txt 2>&1 || exit 1
done
echo "fs_tiles" >> $OUT/t.txt
RSX_FS_SCREEN=0 timeout -k 10 120 python tools/gpu/fsbal.py ${NBS:-32768 35598} >> $OUT/t.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/t.txt
