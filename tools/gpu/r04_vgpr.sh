# round 4: MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form=1).  Three builds:
# base (no per-source flags), the product (the flag on linear.hip), vgpr_all (the flag on
# every source).  Exactness of vgpr_all on the SMORE / full-sort tests, then C5 / C3 and
# full-sort timings of each build, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04vgpr}
mkdir -p $OUT; rm -f $OUT/t.txt
VA=recommendar-systems_amd/rsx/lib/variants/vgpr_all/librsx.so
VB=recommendar-systems_amd/rsx/lib/variants/base/librsx.so
RSX_LIB=$VA timeout -k 10 500 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py tests/test_gpu_realshape.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_vgpr_all.log 2>&1
rc=$?; tail -2 $OUT/pytest_vgpr_all.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base prod vgpr_all; do
    unset RSX_LIB; [ $v = base ] && export RSX_LIB=$VB; [ $v = vgpr_all ] && export RSX_LIB=$VA
    for w in c5 c3; do
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || exit 1
      python -c "import json;d=json.load(open('$OUT/${w}_${v}_$rep.json'));print('$w $v $rep', round(d['ms_per_step'],4))" >> $OUT/t.txt
    done
    echo "fs $v" >> $OUT/t.txt
    timeout -k 10 120 python tools/gpu/fsbal.py 35598 32768 2>&1 | grep -v amdgpu.ids >> $OUT/t.txt || exit 1
  done
done
cat $OUT/t.txt
