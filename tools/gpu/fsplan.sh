# full-sort timing over chunk plans (RSX_FS_CHUNKS) with and without the balanced split (RSX_FS_SEG)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/fsplan}
mkdir -p $OUT; rm -f $OUT/t.txt
for cfg in "2 1" "2 0" "3 0" "4 0" "4 1" "8 0"; do
  set -- $cfg
  echo "chunks=$1 seg=$2" >> $OUT/t.txt
  RSX_FS_CHUNKS=$1 RSX_FS_SEG=$2 timeout -k 10 120 python tools/gpu/fsbal.py ${NBS:-35598 19445} >> $OUT/t.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/t.txt
