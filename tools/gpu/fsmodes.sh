# full-sort timing per fs_screen ablation (RSX_FS_MODE 0 full, 5 pass 1 only, 6 no exact dots) and fs_tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/fsmodes}
mkdir -p $OUT
for m in 0 5 6; do
  echo "mode $m" >> $OUT/t.txt
  RSX_FS_MODE=$m timeout -k 10 120 python tools/gpu/fsbal.py ${NBS:-32768 35598} >> $OUT/t.txt 2>&1 || exit 1
done
echo "fs_tiles" >> $OUT/t.txt
RSX_FS_SCREEN=0 timeout -k 10 120 python tools/gpu/fsbal.py ${NBS:-32768 35598} >> $OUT/t.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/t.txt
