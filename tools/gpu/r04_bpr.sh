# round 4: bpr_fused with its G' atomics issued after the block's done count (the release
# fence waits for the loss partials only): the kernel / step / DP tests, then C2 against
# the HEAD variant (three alternating pairs) and both builds' C2 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04bpr}
mkdir -p $OUT; rm -f $OUT/t.txt
VH=recommendar-systems_amd/rsx/lib/variants/head/librsx.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_realshape.py tests/test_gpu_dp.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in head new; do
    unset RSX_LIB; [ $v = head ] && export RSX_LIB=$VH
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $OUT/c2_${v}_$rep.json 2> $OUT/c2_${v}_$rep.err || exit 1
    python -c "import json;d=json.load(open('$OUT/c2_${v}_$rep.json'));print('c2 $v $rep', round(d['ms_per_step'],5))" >> $OUT/t.txt
  done
done
for v in head new; do
  unset RSX_LIB; [ $v = head ] && export RSX_LIB=$VH
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o c2 -- python bench.py --no-cpu-baseline > $OUT/c2prof_$v.json 2> $OUT/c2prof_$v.err || exit 1
done
find $OUT -name '*kernel_trace.csv' -delete
cat $OUT/t.txt
grep -h "bpr_fused" $OUT/stats_*/c2_kernel_stats.csv | cut -d, -f1-4
