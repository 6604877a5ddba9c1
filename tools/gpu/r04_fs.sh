# round 4: fs_screen pass 1 software-pipelined (variant p1pipe: -DRSX_FS_P1PIPE=1) vs the
# default build: exactness tests on the variant, then full-sort timings of both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04fs}
mkdir -p $OUT; rm -f $OUT/t.txt
V=recommendar-systems_amd/rsx/lib/variants/p1pipe/librsx.so
RSX_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -x -q -k "fullsort" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_variant.log 2>&1
rc=$?; tail -3 $OUT/pytest_variant.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  echo "default" >> $OUT/t.txt
  timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 >> $OUT/t.txt 2>&1 || exit 1
  echo "p1pipe" >> $OUT/t.txt
  RSX_LIB=$V timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 >> $OUT/t.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/t.txt
